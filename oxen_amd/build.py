"""Build the in-tree HIP library (oxen_amd/liboxen_hash.so) for gfx950 with hipcc.

The .so is git-ignored but travels to the GPU box with the repo snapshot; no JIT cache is used.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "liboxen_hash.so")
# the C ABI runtime (capi_internal.hpp lists its pieces), the kernels, FastCDC, the reader pool, RCCL
SOURCES = [os.path.join(CSRC, f) for f in (
    "xxh3_kernels.hip", "capi_dispatch.hip", "capi_context.hip", "staging.hip", "large_items.hip", "xxh3_stream.hip",
    "engine.hip", "modified.hip", "publish.hip", "fastcdc.hip", "reader_pool.cpp", "comm.cpp", "fastcdc_host.cpp")]
DEPS = SOURCES + [os.path.join(CSRC, h) for h in ("capi_internal.hpp", "xxh3_device.hpp", "fastcdc_gear.h", "pool.hpp",
                                                 "scratch.hpp", "reader_pool.hpp")] + [os.path.join(ROOT, "include", "oxen_hash.h")]
HELPER_SRC = os.path.join(CSRC, "hash_helper.cpp")
HELPER = os.path.join(HERE, "oxh_hash_helper")  # the reader-pool helper process (oxh_pool_*)
ARCH = "gfx950"


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (expected /opt/rocm/bin/hipcc)")


def needs_build() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(d) > t for d in DEPS)


HOST_SRC = os.path.join(HERE, "host", "oxen_hasher.cpp")
HOST_HDR = os.path.join(HERE, "host", "oxen_hasher.hpp")
COMMIT_SRC = os.path.join(HERE, "host", "commit_writer.cpp")
COMMIT_HDR = os.path.join(HERE, "host", "commit_writer.hpp")
HOST_LIB = os.path.join(HERE, "liboxen_hasher.so")
NATIVE_TEST_SRC = os.path.join(ROOT, "tests", "native", "test_hasher.cpp")
NATIVE_TEST = os.path.join(ROOT, "tests", "native", "test_hasher")
COMMIT_CLI_SRC = os.path.join(ROOT, "tests", "native", "commit_tree_cli.cpp")
COMMIT_CLI = os.path.join(ROOT, "tests", "native", "commit_tree_cli")
FAKE_HELPER_SRC = os.path.join(ROOT, "tests", "native", "fake_pool_helper.cpp")
FAKE_HELPER = os.path.join(ROOT, "tests", "native", "fake_pool_helper")  # tests only: the pool without a GPU
C_CONSUMER_SRC = os.path.join(ROOT, "tests", "native", "abi_c_consumer.c")
C_CONSUMER = os.path.join(ROOT, "tests", "native", "abi_c_consumer")  # tests only: a plain C99 caller of the ABI
FAKE_RCCL_SRC = os.path.join(ROOT, "tests", "native", "fake_rccl.cpp")
# tests only: an "RCCL" for N processes on one GPU (OXH_RCCL_LIB), with and without ncclGather
FAKE_RCCL = os.path.join(ROOT, "tests", "native", "libfake_rccl.so")
FAKE_RCCL_NOGATHER = os.path.join(ROOT, "tests", "native", "libfake_rccl_nogather.so")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def _stale(target: str, deps: list[str]) -> bool:
    return not os.path.exists(target) or any(os.path.getmtime(d) > os.path.getmtime(target) for d in deps)


def build_host(force: bool = False, verbose: bool = False) -> str:
    """The C++ host mirror over the C ABI (oxen_amd/host, g++): liboxen `util::hasher` + MerkleHash
    and the commit writer's K2 driver, in liboxen_hasher.so; its native test programs
    (tests/native/test_hasher.cpp, commit_tree_cli.cpp). All link against liboxen_hash.so."""
    hdr = os.path.join(ROOT, "include", "oxen_hash.h")
    steps = [
        (HELPER, [HELPER_SRC, os.path.join(CSRC, "reader_pool.hpp"), hdr, LIB],
         ["g++", "-std=c++17", "-O2", "-Wall", "-o", HELPER + ".tmp", HELPER_SRC,
          f"-L{HERE}", "-l:liboxen_hash.so", "-Wl,-rpath,$ORIGIN"]),
        (HOST_LIB, [HOST_SRC, HOST_HDR, COMMIT_SRC, COMMIT_HDR, hdr, LIB],
         ["g++", "-std=c++17", "-O2", "-Wall", "-shared", "-fPIC", "-o", HOST_LIB + ".tmp", HOST_SRC, COMMIT_SRC,
          f"-L{HERE}", "-l:liboxen_hash.so", "-Wl,-rpath,$ORIGIN"]),
        (NATIVE_TEST, [NATIVE_TEST_SRC, HOST_HDR, HOST_LIB],
         ["g++", "-std=c++17", "-O2", "-Wall", "-o", NATIVE_TEST + ".tmp", NATIVE_TEST_SRC,
          f"-L{HERE}", "-l:liboxen_hasher.so", "-l:liboxen_hash.so", "-Wl,-rpath,$ORIGIN/../../oxen_amd"]),
        (FAKE_HELPER, [FAKE_HELPER_SRC, os.path.join(CSRC, "reader_pool.hpp")],
         ["g++", "-std=c++17", "-O2", "-Wall", "-o", FAKE_HELPER + ".tmp", FAKE_HELPER_SRC]),
        (C_CONSUMER, [C_CONSUMER_SRC, hdr, LIB],
         ["gcc", "-std=c99", "-O2", "-Wall", "-Wextra", "-pedantic", "-Werror", "-o", C_CONSUMER + ".tmp", C_CONSUMER_SRC,
          f"-L{HERE}", "-l:liboxen_hash.so", "-Wl,-rpath,$ORIGIN/../../oxen_amd"]),
        (COMMIT_CLI, [COMMIT_CLI_SRC, COMMIT_HDR, HOST_HDR, HOST_LIB],
         ["g++", "-std=c++17", "-O2", "-Wall", "-o", COMMIT_CLI + ".tmp", COMMIT_CLI_SRC,
          f"-L{HERE}", "-l:liboxen_hasher.so", "-l:liboxen_hash.so", "-Wl,-rpath,$ORIGIN/../../oxen_amd"]),
    ]
    for target, extra in ((FAKE_RCCL, []), (FAKE_RCCL_NOGATHER, ["-DFAKE_NO_GATHER"])):
        steps.append((target, [FAKE_RCCL_SRC],
                      ["g++", "-std=c++17", "-O2", "-Wall", "-shared", "-fPIC", "-fvisibility=hidden",
                       "-D__HIP_PLATFORM_AMD__", f"-I{ROCM}/include", "-o", target + ".tmp", FAKE_RCCL_SRC] + extra +
                      [f"-L{ROCM}/lib", "-lamdhip64", "-lrt", f"-Wl,-rpath,{ROCM}/lib"]))
    for target, deps, cmd in steps:
        if force or _stale(target, deps):
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            subprocess.run(cmd, check=True)
            os.replace(target + ".tmp", target)
    return HOST_LIB


def compile_lib(out: str, defines: tuple[str, ...] = (), verbose: bool = False) -> str:
    """hipcc every source to its own object in parallel (one hipcc per source), then link `out`."""
    from concurrent.futures import ThreadPoolExecutor

    objdir = os.path.join(HERE, "build", os.path.basename(out).replace(".so", ""))
    os.makedirs(objdir, exist_ok=True)
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall"] + [f"-D{d}" for d in defines]

    def one(src: str) -> str:
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        cmd = [hipcc()] + flags + ["-c", "-o", obj, src]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        return obj

    jobs = max(1, min(len(SOURCES), int(os.environ.get("MAX_JOBS", "0") or 0) or (os.cpu_count() or 4)))
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(one, SOURCES))
    tmp = out + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-Wl,--no-undefined", "-o", tmp] + objs
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)
    return out


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not needs_build():
        build_host(verbose=verbose)
        return LIB
    compile_lib(LIB, verbose=verbose)
    build_host(force=True, verbose=verbose)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
