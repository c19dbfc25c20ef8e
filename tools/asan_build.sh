#!/bin/bash
# Host-side AddressSanitizer builds of the runtime (tools/asan_suite.sh runs the CPU suite over them).
# Only HOST code is instrumented: every -fsanitize on a hipcc line sits right after -Xarch_host, and
# the host-only clang++ line carries -fno-gpu-sanitize; the device code of the kernels is unchanged.
# Outputs go to asan/ (git-ignored; gpurun-ignored, no GPU run uses them):
#   asan/liboxen_hash.so      the C ABI runtime + kernels, host part instrumented
#   asan/liboxen_hasher.so    the C++ mirror (liboxen::util::hasher, commit writer), instrumented
#   asan/oxh_hash_helper      the reader-pool helper (uninstrumented main; loads the library above)
# The shared objects link clang's libclang_rt.asan-x86_64.so, which every process also preloads
# (tools/asan_suite.sh): the runtime must come first in the load order.
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=asan
mkdir -p $OUT
HIPCC=/opt/rocm/bin/hipcc
CLANGXX=/opt/rocm/lib/llvm/bin/clang++
SAN="-Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer"
# the runtime as a DT_NEEDED of each library, so programs linked against them resolve its symbols
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
RTLINK="-Wl,$RT -Wl,-rpath,$(dirname "$RT")"
# the product library's own source list (oxen_amd/build.py SOURCES), so the two never drift apart
SRCS=$(python3 -c 'from oxen_amd import build; print(" ".join(build.SOURCES))')
$HIPCC --offload-arch=gfx950 -O3 -Xarch_host -g -std=c++17 -shared -fPIC -Wall $SAN -o $OUT/liboxen_hash.so \
  $SRCS $RTLINK
$CLANGXX -std=c++17 -O1 -g -fno-gpu-sanitize -fsanitize=address -fno-omit-frame-pointer -shared -fPIC -Wall \
  -o $OUT/liboxen_hasher.so oxen_amd/host/oxen_hasher.cpp oxen_amd/host/commit_writer.cpp \
  -L$OUT -l:liboxen_hash.so -Wl,-rpath,'$ORIGIN' $RTLINK
$CLANGXX -std=c++17 -O2 -Wall -o $OUT/oxh_hash_helper oxen_amd/csrc/hash_helper.cpp -L$OUT -l:liboxen_hash.so -Wl,-rpath,'$ORIGIN'
ls -l $OUT
