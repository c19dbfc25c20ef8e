"""Large files from disk (the reference's streaming branch, hasher.rs:150-174, files >= 1e9 B):
oxh_hash_files on N files of S GiB vs the CPU oracle two ways, one thread per file: mmap + one-shot
XXH3 (the fastest CPU form), and the reference's 4 KiB read() loop (oxo_hash_files_stream4k).

    python tools/big_file_probe.py [--files 2] [--gib 4] [--dir /tmp/oxh_big]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=2)
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--dir", default=os.path.join(os.environ.get("TMPDIR", "/tmp"), "oxh_big"))
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()

    from oracle import oracle
    from oxen_amd import _capi
    from oxen_amd.workloads import splitmix_bytes

    os.makedirs(a.dir, exist_ok=True)
    size = int(a.gib * 2**30)
    paths = []
    for f in range(a.files):
        p = os.path.join(a.dir, f"big{f}.bin")
        if not (os.path.exists(p) and os.path.getsize(p) == size):
            with open(p, "wb") as fh:
                piece = 256 << 20
                for off in range(0, size, piece):
                    fh.write(splitmix_bytes(700 + f, off, min(piece, size - off)).tobytes())
        paths.append(p)
    n = len(paths)
    arr = (ctypes.c_char_p * n)(*[os.fsencode(p) for p in paths])
    out = np.zeros((n, 2), dtype=np.uint64)
    sz = np.zeros(n, dtype=np.uint64)
    st = np.zeros(n, dtype=np.int32)
    L, O = _capi.lib(), oracle.lib()
    ctx = _capi.Context(0)
    res = {"files": n, "bytes_each": size}
    gpu, cpu, cpu4k = [], [], []
    ref = np.zeros((n, 2), dtype=np.uint64)
    ref4k = np.zeros((n, 2), dtype=np.uint64)
    for r in range(a.reps + 1):  # the first pass warms the page cache
        t0 = time.perf_counter()
        _capi.check(L.oxh_hash_files(ctx.handle, arr, n, out.ctypes.data_as(_capi._u64p), sz.ctypes.data_as(_capi._u64p),
                                     st.ctypes.data_as(_capi._i32p)), "hash")
        t1 = time.perf_counter()
        O.oxo_hash_files(arr, n, ref.ctypes.data_as(oracle._u64p), sz.ctypes.data_as(oracle._u64p),
                         st.ctypes.data_as(oracle._i32p), n)
        t2 = time.perf_counter()
        O.oxo_hash_files_stream4k(arr, n, ref4k.ctypes.data_as(oracle._u64p), sz.ctypes.data_as(oracle._u64p),
                                  st.ctypes.data_as(oracle._i32p), n)
        t3 = time.perf_counter()
        if r:
            gpu.append(t1 - t0)
            cpu.append(t2 - t1)
            cpu4k.append(t3 - t2)
    # cold page cache (posix_fadvise DONTNEED before each side)
    def drop():
        for p in paths:
            fd = os.open(p, os.O_RDONLY)
            os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
            os.close(fd)

    drop()
    t0 = time.perf_counter()
    _capi.check(L.oxh_hash_files(ctx.handle, arr, n, out.ctypes.data_as(_capi._u64p), sz.ctypes.data_as(_capi._u64p),
                                 st.ctypes.data_as(_capi._i32p)), "hash")
    res["gpu_cold_s"] = round(time.perf_counter() - t0, 3)
    cold_ok = bool(np.array_equal(out, ref))
    drop()
    t0 = time.perf_counter()
    O.oxo_hash_files(arr, n, ref.ctypes.data_as(oracle._u64p), sz.ctypes.data_as(oracle._u64p),
                     st.ctypes.data_as(oracle._i32p), n)
    res["cpu_mmap_cold_s"] = round(time.perf_counter() - t0, 3)
    res["gpu_s"] = round(float(np.median(gpu)), 3)
    res["gpu_GiBs"] = round(n * size / res["gpu_s"] / 2**30, 2)
    res["cpu_read_whole_one_thread_per_file_s"] = round(float(np.median(cpu)), 3)
    res["cpu_ref_4k_reads_one_thread_per_file_s"] = round(float(np.median(cpu4k)), 3)
    res["digests_bit_exact"] = bool(np.array_equal(out, ref) and np.array_equal(out, ref4k) and cold_ok)
    print(json.dumps(res), flush=True)
    if not res["digests_bit_exact"]:
        sys.exit(1)


if __name__ == "__main__":
    main()
