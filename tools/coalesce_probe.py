"""Coalescer probe: the C3 image repo hashed in liboxen's 64-file batches (add.rs:41), from 1 caller
thread vs from 16 concurrent caller threads on one context, vs one whole-list call.

    python tools/coalesce_probe.py [--images 200000] [--batch 64] [--callers 16] [--flush-mib 16]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=200_000)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--callers", type=int, default=16)
    ap.add_argument("--dir", default="/tmp/oxh_c3")
    ap.add_argument("--flush-mib", default="16", help="OXH_FLUSH_MIB values to compare (comma list)")
    a = ap.parse_args()

    import numpy as np

    from oxen_amd import _capi
    from oxen_amd.workloads import write_image_repo_fast

    paths = write_image_repo_fast(a.dir, a.images)
    n = len(paths)
    enc = [os.fsencode(p) for p in paths]
    L = _capi.lib()
    batches = [(i, min(n, i + a.batch)) for i in range(0, n, a.batch)]
    outs = np.zeros((n, 2), dtype=np.uint64)
    arrs = [(ctypes.c_char_p * (e - s))(*enc[s:e]) for s, e in batches]

    ctx = None

    def run_batch(k):
        s, e = batches[k]
        o = outs[s:e]
        _capi.check(L.oxh_hash_files(ctx.handle, arrs[k], e - s, o.ctypes.data_as(_capi._u64p), None, None), "hash")

    def serial():
        for k in range(len(batches)):
            run_batch(k)

    def concurrent():
        nxt = [0]
        lock = threading.Lock()

        def worker():
            while True:
                with lock:
                    k = nxt[0]
                    nxt[0] += 1
                if k >= len(batches):
                    return
                run_batch(k)

        th = [threading.Thread(target=worker) for _ in range(a.callers)]
        for t in th:
            t.start()
        for t in th:
            t.join()

    whole_arr = (ctypes.c_char_p * n)(*enc)
    whole_out = np.zeros((n, 2), dtype=np.uint64)

    def whole():
        _capi.check(L.oxh_hash_files(ctx.handle, whole_arr, n, whole_out.ctypes.data_as(_capi._u64p), None, None), "hash")

    for fm in a.flush_mib.split(","):
        os.environ["OXH_FLUSH_MIB"] = fm
        ctx = _capi.Context(0)
        res = {"files": n, "batch": a.batch, "callers": a.callers, "flush_mib": int(fm)}
        for name, fn in (("whole_list", whole), ("serial_batches", serial), ("concurrent_batches", concurrent)):
            fn()  # warm
            ts = []
            for _ in range(3):
                t0 = time.perf_counter()
                fn()
                ts.append(time.perf_counter() - t0)
            res[f"{name}_s"] = round(min(ts), 3)
        res["same_digests"] = bool(np.array_equal(outs, whole_out))
        print(json.dumps(res), flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
