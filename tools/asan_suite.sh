#!/bin/bash
# Run the test suite over the host-ASan runtime built by tools/asan_build.sh: the tree is copied to a
# scratch directory, the instrumented libraries replace oxen_amd/'s, and every process preloads
# clang's ASan runtime (inherited by the reader-pool helpers and the native test programs).
#   bash tools/asan_suite.sh [pytest marker expression, default "not gpu"] [extra pytest args...]
# Writes gpurun_out/asan_pytest.log. GPU code is not instrumented (only -Xarch_host builds).
# CPU suite only: on the MI355X boxes the preloaded runtime intercepts hsa_amd_memory_pool_allocate
# and fails HIP's first device allocation ("AddressSanitizer: out-of-memory" inside
# torch.cuda.is_available(), r03c), so the GPU suite cannot run under it there.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$(pwd)
MARK=${1:-not gpu}
shift || true
export TMPDIR=${TMPDIR:-/tmp}
mkdir -p gpurun_out
[ -f asan/liboxen_hash.so ] || { echo "asan/ not built (tools/asan_build.sh)"; exit 2; }
W=$(mktemp -d "$TMPDIR/oxh_asan.XXXXXX")
tar --exclude=./gpurun_out --exclude=./.git -cf - . | tar -C "$W" -xf -
cp -p asan/liboxen_hash.so asan/liboxen_hasher.so asan/oxh_hash_helper "$W/oxen_amd/"
touch "$W/oxen_amd/liboxen_hasher.so"  # newer than liboxen_hash.so: no host rebuild over it
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
cd "$W"
# protect_shadow_gap=0: the HSA runtime maps memory inside ASan's default shadow gap
LD_PRELOAD="$RT" ASAN_OPTIONS=detect_leaks=0:protect_shadow_gap=0:detect_container_overflow=0:halt_on_error=1:abort_on_error=1 \
  timeout -k 10 1050 python -u -m pytest tests -x -v -m "$MARK" -p no:cacheprovider --timeout 300 --timeout-method thread "$@" \
  > "$ROOT/gpurun_out/asan_pytest.log" 2>&1
rc=$?
tail -5 "$ROOT/gpurun_out/asan_pytest.log"
grep -n "ERROR: AddressSanitizer" -A 30 "$ROOT/gpurun_out/asan_pytest.log" | head -80
cd "$ROOT" && rm -rf "$W"
exit $rc
