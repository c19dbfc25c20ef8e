"""Host buffers of 1-200 MiB through oxh_hash_buffers (staging.hip hash_host_items: the slot copy in 4 MiB
pieces over the pool, K1L for a batch's items of 1 MiB and more) against the C oracle over the same
buffers (16 threads). Medians of --reps calls; every digest checked. Prints one JSON line.

    python tools/buffers_probe.py [--reps 5]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from oracle import oracle
    from oxen_amd import _capi, hasher

    oracle.build()
    ctx = _capi.Context(0)
    rng = np.random.default_rng(81)
    res = {"reps": a.reps}
    ok = True
    for name, n, size in (("1x200MiB", 1, 200 << 20), ("16x16MiB", 16, 16 << 20), ("64x1MiB", 64, 1 << 20)):
        arena = rng.integers(0, 256, n * size, dtype=np.uint8)
        bufs = [arena[k * size:(k + 1) * size].tobytes() for k in range(n)]
        offs = np.arange(n, dtype=np.uint64) * np.uint64(size)
        lens = np.full(n, size, dtype=np.uint64)
        want = oracle.batch(arena, offs, lens, threads=16)
        want = [(int(h) << 64) | int(l) for l, h in want.tolist()]
        g, cpu = [], []
        for _ in range(a.reps + 1):
            t0 = time.perf_counter()
            got = hasher.hash_buffers_128bit(bufs, ctx)
            t1 = time.perf_counter()
            oracle.batch(arena, offs, lens, threads=16)
            t2 = time.perf_counter()
            ok &= got == want
            g.append(t1 - t0)
            cpu.append(t2 - t1)
        gs, cs = statistics.median(g[1:]), statistics.median(cpu[1:])
        res[name] = {"gpu_s": round(gs, 4), "gpu_GiBs": round(n * size / gs / 2**30, 1), "cpu16_s": round(cs, 4),
                     "cpu16_GiBs": round(n * size / cs / 2**30, 1)}
    res["bit_exact"] = bool(ok)
    ctx.close()
    print(json.dumps(res), flush=True)
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
