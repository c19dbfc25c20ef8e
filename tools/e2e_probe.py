"""Quick e2e probe: oxh_hash_files stage trace (OXH_TRACE=1) vs the C reference loop, alternating.

    python tools/e2e_probe.py [--images 200000] [--staging-mib 16] [--reps 3]
"""
from __future__ import annotations

import argparse
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=200_000)
    ap.add_argument("--dir", default="/tmp/oxh_c3")
    ap.add_argument("--staging-mib", default="16")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--reader-threads", default="16", help="OXH_NUM_THREADS values to compare")
    a = ap.parse_args()
    os.environ["OXH_TRACE"] = "1"
    os.environ.setdefault("OXH_NUM_THREADS", str(a.threads))
    import numpy as np

    from oracle import oracle
    from oxen_amd import _capi
    from oxen_amd.workloads import write_image_repo_fast

    paths = write_image_repo_fast(a.dir, a.images)
    n = len(paths)
    c_paths = (ctypes.c_char_p * n)(*[os.fsencode(p) for p in paths])
    L, O = _capi.lib(), oracle.lib()
    ctxs = {}
    for m in a.staging_mib.split(","):
        for t in a.reader_threads.split(","):
            os.environ["OXH_NUM_THREADS"] = t
            ctxs[f"{m}MiB/{t}thr"] = _capi.Context(0, staging_bytes=int(m) << 20)
    out = np.zeros((n, 2), dtype=np.uint64)
    sz = np.zeros(n, dtype=np.uint64)
    st = np.zeros(n, dtype=np.int32)
    for r in range(a.reps):
        for m, c in ctxs.items():
            t0 = time.perf_counter()
            L.oxh_hash_files(c.handle, c_paths, n, out.ctypes.data_as(_capi._u64p), sz.ctypes.data_as(_capi._u64p),
                             st.ctypes.data_as(_capi._i32p))
            print(f"gpu {m}: {time.perf_counter() - t0:.3f} s", file=sys.stderr, flush=True)
        t0 = time.perf_counter()
        O.oxo_hash_files(c_paths, n, out.ctypes.data_as(oracle._u64p), sz.ctypes.data_as(oracle._u64p),
                         st.ctypes.data_as(oracle._i32p), a.threads)
        print(f"cpu ref: {time.perf_counter() - t0:.3f} s", file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
