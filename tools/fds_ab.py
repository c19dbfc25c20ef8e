"""A/B of the streaming readers' private file-descriptor tables (pool.hpp make_fd_table_private) on
the warm C3 tree, in ONE process: context A is created with private tables (the default), context B
with OXH_SHARED_FDS=1 in the environment at its creation; calls alternate A, B, the CPU reference
loop (oracle/), 7 rounds; medians printed as one JSON line. Digests checked equal.

    python tools/fds_ab.py [--images 200000] [--rounds 7] [--pool-procs 2]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=200_000)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--dir", default=os.path.join(os.environ.get("TMPDIR", "/tmp"), "oxh_c3_fds"))
    ap.add_argument("--staging-mib", default="", help="extra private-fd contexts with these slot sizes")
    ap.add_argument("--pool-procs", type=int, default=0, help="also A/B reader-process pools of this many helpers")
    a = ap.parse_args()

    import numpy as np

    from oracle import oracle
    from oxen_amd import _capi
    from oxen_amd.workloads import write_image_repo_fast

    shutil.rmtree(a.dir, ignore_errors=True)
    paths = write_image_repo_fast(a.dir, a.images)
    n = len(paths)
    arr = (ctypes.c_char_p * n)(*[os.fsencode(p) for p in paths])
    ctx_a = _capi.Context(0)
    os.environ["OXH_SHARED_FDS"] = "1"
    ctx_b = _capi.Context(0)
    del os.environ["OXH_SHARED_FDS"]
    extra = {f"gpu_private_fds_staging{m}MiB": _capi.Context(0, staging_bytes=m << 20)
             for m in [int(x) for x in a.staging_mib.split(",") if x]}
    pools = {}
    if a.pool_procs:
        from oxen_amd.procpool import ShardedFileHasher

        pools["pool%d_private_fds" % a.pool_procs] = ShardedFileHasher(procs=a.pool_procs)
        os.environ["OXH_SHARED_FDS"] = "1"  # the helpers inherit it at spawn
        pools["pool%d_shared_fds" % a.pool_procs] = ShardedFileHasher(procs=a.pool_procs)
        del os.environ["OXH_SHARED_FDS"]
    oracle.build()
    L, O = _capi.lib(), oracle.lib()
    threads = min(16, os.cpu_count() or 1)

    def gpu(ctx):
        out = np.zeros((n, 2), dtype=np.uint64)
        st = np.zeros(n, dtype=np.int32)
        t0 = time.perf_counter()
        _capi.check(L.oxh_hash_files(ctx.handle, arr, n, out.ctypes.data_as(_capi._u64p), None,
                                     st.ctypes.data_as(_capi._i32p)), "oxh_hash_files")
        return time.perf_counter() - t0, out, st

    def cpu():
        out = np.zeros((n, 2), dtype=np.uint64)
        sizes = np.zeros(n, dtype=np.uint64)
        st = np.zeros(n, dtype=np.int32)
        t0 = time.perf_counter()
        O.oxo_hash_files(arr, n, out.ctypes.data_as(oracle._u64p), sizes.ctypes.data_as(oracle._u64p),
                         st.ctypes.data_as(oracle._i32p), threads)
        return time.perf_counter() - t0, out, st

    calls = {"gpu_private_fds": lambda: gpu(ctx_a), "gpu_shared_fds": lambda: gpu(ctx_b), "cpu_ref_loop": cpu}
    for k, c in extra.items():
        calls[k] = (lambda c=c: gpu(c))

    from oxen_amd.procpool import pack_paths

    blob, offs = pack_paths(paths)  # once, outside the timing (like the C-string table above)

    def pooled(pool):
        t0 = time.perf_counter()
        out, _, st = pool.hash_files_packed(blob, offs)
        return time.perf_counter() - t0, out, st

    for k, pl in pools.items():
        calls[k] = (lambda pl=pl: pooled(pl))
    for f in calls.values():
        f()  # warm
    ts = {k: [] for k in calls}
    ok = True
    ref = None
    for _ in range(a.rounds):
        for k, f in calls.items():
            dt, out, st = f()
            ts[k].append(round(dt, 4))
            ok = ok and bool((st == 0).all())
            ref = out if ref is None else ref
            ok = ok and bool(np.array_equal(out, ref))
    res = {"files": n, "rounds": a.rounds, "threads": threads, "bit_exact": ok}
    for k, v in ts.items():
        res[k + "_median_s"] = float(np.median(v))
        res[k + "_all"] = v
    print(json.dumps(res), flush=True)
    ctx_a.close()
    ctx_b.close()
    for c in extra.values():
        c.close()
    for pl in pools.values():
        pl.close()
    shutil.rmtree(a.dir, ignore_errors=True)


if __name__ == "__main__":
    main()
