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
SOURCES = [os.path.join(CSRC, "xxh3_kernels.hip"), os.path.join(CSRC, "oxen_hash_capi.hip"), os.path.join(CSRC, "fastcdc.hip")]
DEPS = SOURCES + [os.path.join(CSRC, "xxh3_device.hpp"), os.path.join(CSRC, "fastcdc_gear.h"), os.path.join(CSRC, "pool.hpp"), os.path.join(CSRC, "scratch.hpp"),
                  os.path.join(ROOT, "include", "oxen_hash.h")]
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


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not needs_build():
        return LIB
    tmp = LIB + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-shared", "-fPIC", "-Wall", "-Wl,--no-undefined",
           "-o", tmp] + SOURCES
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
