"""Host-buffer batches of many short items (oxh_hash_streams): the commit driver's bucket pass at the
C3 tree (200 000 paths of ~31 B) and its dir pass shape, timed in one process (median of --reps),
with OXH_TRACE's fill / drain / submit split on stderr. Digests checked against the C oracle.

    python tools/streams_probe.py [--n 200000] [--reps 9]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=200_000)
    ap.add_argument("--reps", type=int, default=9)
    a = ap.parse_args()

    import numpy as np

    from oracle import oracle
    from oxen_amd import _capi

    paths = [f"images/split_{i % 1000}/img_{i}.tiff".encode() for i in range(a.n)]
    lens = np.array([len(p) for p in paths], dtype=np.uint64)
    offs = np.zeros(a.n, dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1])
    arena = np.frombuffer(b"".join(paths), dtype=np.uint8)
    ctx = _capi.Context(0)
    L = _capi.lib()
    out = np.zeros((a.n, 2), dtype=np.uint64)

    def call():
        t0 = time.perf_counter()
        _capi.check(L.oxh_hash_streams(ctx.handle, arena.ctypes.data, offs.ctypes.data_as(_capi._u64p),
                                       lens.ctypes.data_as(_capi._u64p), a.n, out.ctypes.data_as(_capi._u64p)),
                    "oxh_hash_streams")
        return time.perf_counter() - t0

    call()
    ts = sorted(call() for _ in range(a.reps))
    oracle.build()
    want = [oracle.xxh3_128_int(p) for p in paths[:2000]]
    got = [(int(hi) << 64) | int(lo) for lo, hi in out[:2000]]
    res = {"items": a.n, "bytes": int(lens.sum()), "median_ms": round(1e3 * ts[len(ts) // 2], 3),
           "min_ms": round(1e3 * ts[0], 3), "bit_exact_first_2000": want == got}
    print(json.dumps(res), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
