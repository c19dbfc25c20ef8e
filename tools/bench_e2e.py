"""End-to-end `oxen add` hash stage from files on disk (config 3), recorded in DESIGN.md.

    python tools/bench_e2e.py [--images 200000] [--dir /tmp/oxh_c3]

Writes the C3 image repo (benchmark/generate_image_repo.py layout: 200 000 noise TIFFs of
49 292 B in 1 000 dirs + images.csv + README.md), then times, on the same files:
  gpu_e2e_meta  oxh_hash_files_meta: the same with the caller's stat sizes (no fstat per file)
  gpu_e2e    oxh_hash_files: parallel pread into pinned staging -> H2D on a side stream (3-slot
             ring, overlapped with K1 on the compute stream) -> D2H digests
  cpu_ref    the reference's per-file loop restated in C (oracle/): stat, read whole file, one-shot
             XXH3-128 (hasher.rs:126-148), one worker per host thread
  gpu_procsP oxen_amd.procpool.ShardedFileHasher: the list split over P worker processes, each with
             its own context and threads/P readers (the open/close floor is per process)
  cpu_procsP the restated reference loop in P processes of threads/P threads, for the same split
with the page cache warm, and cold (pages dropped with posix_fadvise DONTNEED). Also reports the
pinned H2D copy rate. Every GPU digest is checked against the CPU one.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def drop_cache(paths):
    os.sync()
    for p in paths:
        try:
            fd = os.open(p, os.O_RDONLY)
            os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
            os.close(fd)
        except OSError:
            pass


def sharded(a, paths, meta, nbytes, cpu_call, drop_cache):
    """The same files through P reader processes (GPU engines, then the CPU loop), warm alternating
    rounds + one cold run each; digests checked against the one-process CPU loop."""
    import numpy as np

    from cpu_procpool import CpuShardedLoop

    from oxen_amd.procpool import ShardedFileHasher, pack_paths

    res = {}
    _, want, _ = cpu_call()
    blob, offs = pack_paths(paths)  # packed once, outside the timing (as c_paths is)
    for P in [int(x) for x in a.procs.split(",") if x]:
        th = max(1, a.threads // P)
        devs = tuple(int(x) for x in a.devices.split(","))
        pools = {"gpu": ShardedFileHasher(procs=P, devices=devs, threads=th, staging_bytes=a.pool_staging_mib << 20),
                 "cpu": CpuShardedLoop(procs=P, threads=th)}
        try:
            ts = {"gpu": [], "cpu": []}
            ok = True
            for k in pools:
                pools[k].hash_files_packed(blob, offs, meta)  # warm-up
            for _ in range(5):
                for k in ("gpu", "cpu"):
                    t0 = time.perf_counter()
                    out, _, st = pools[k].hash_files_packed(blob, offs, meta)
                    ts[k].append(time.perf_counter() - t0)
                    ok = ok and bool((st == 0).all()) and np.array_equal(out, want)
            for k in ("gpu", "cpu"):
                med = float(np.median(ts[k]))
                res[f"{k}_procs{P}_warm_s"] = round(med, 3)
                res[f"{k}_procs{P}_warm_GiBs"] = round(nbytes / med / 2**30, 2)
                res[f"{k}_procs{P}_warm_s_all"] = [round(x, 3) for x in ts[k]]
                drop_cache(paths)
                t0 = time.perf_counter()
                out, _, st = pools[k].hash_files_packed(blob, offs, meta)
                res[f"{k}_procs{P}_cold_s"] = round(time.perf_counter() - t0, 3)
                ok = ok and bool((st == 0).all()) and np.array_equal(out, want)
            res[f"procs{P}_threads_each"] = th
            res[f"procs{P}_bit_exact"] = ok
        finally:
            for p in pools.values():
                p.close()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=200_000)
    ap.add_argument("--dir", default=os.path.join(os.environ.get("TMPDIR", "/tmp"), "oxh_c3"))
    ap.add_argument("--threads", type=int, default=min(16, os.cpu_count() or 1))
    ap.add_argument("--keep", action="store_true")
    ap.add_argument("--staging-mib", default="16,64,256", help="staging slot sizes to sweep (warm cache)")
    ap.add_argument("--procs", default="2,4", help="reader process counts for the sharded runs")
    ap.add_argument("--only-procs", action="store_true", help="skip the add / fsck / staging parts")
    ap.add_argument("--pool-staging-mib", type=int, default=0, help="staging slot size of the pool's helpers (0 = default)")
    ap.add_argument("--devices", default="0", help="GPUs of the pool's helpers (helper p on devices[p %% len]), e.g. 0,1,2,3,4,5,6,7")
    a = ap.parse_args()

    import numpy as np
    import torch

    from oracle import oracle
    from oxen_amd import _capi, hasher
    from oxen_amd.workloads import write_image_repo_fast

    shutil.rmtree(a.dir, ignore_errors=True)
    t0 = time.perf_counter()
    paths = write_image_repo_fast(a.dir, a.images)
    gen_s = time.perf_counter() - t0
    nbytes = sum(os.path.getsize(p) for p in paths)
    res = {"config": "C3: benchmark/generate_image_repo.py layout, %d TIFF 128x128x3 (49 292 B) in 1 000 dirs "
                     "+ images.csv + README.md" % a.images,
           "files": len(paths), "bytes": nbytes, "generate_s": round(gen_s, 1), "threads": a.threads}

    os.environ.setdefault("OXH_NUM_THREADS", str(a.threads))
    ctx = _capi.Context(0)
    # pinned H2D rate for context
    src = torch.empty(1 << 30, dtype=torch.uint8).pin_memory()
    dst = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
    dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    res["h2d_pinned_GBs"] = round(5 * (1 << 30) / (time.perf_counter() - t0) / 1e9, 1)
    del src, dst

    oracle.build()
    import ctypes

    n = len(paths)
    c_paths = (ctypes.c_char_p * n)(*[os.fsencode(p) for p in paths])  # built once, outside the timing
    L, O = _capi.lib(), oracle.lib()

    def gpu_call():
        out = np.zeros((n, 2), dtype=np.uint64)
        sizes = np.zeros(n, dtype=np.uint64)
        st = np.zeros(n, dtype=np.int32)
        t0 = time.perf_counter()
        _capi.check(L.oxh_hash_files(ctx.handle, c_paths, n, out.ctypes.data_as(_capi._u64p),
                                     sizes.ctypes.data_as(_capi._u64p), st.ctypes.data_as(_capi._i32p)),
                    "oxh_hash_files")
        return time.perf_counter() - t0, out, st

    # get_hash_given_metadata form: the sizes liboxen's walk already has (stat'ed outside the timing)
    meta = np.array([os.stat(p).st_size for p in paths], dtype=np.uint64)

    def gpu_meta_call():
        out = np.zeros((n, 2), dtype=np.uint64)
        sizes = np.zeros(n, dtype=np.uint64)
        st = np.zeros(n, dtype=np.int32)
        t0 = time.perf_counter()
        _capi.check(L.oxh_hash_files_meta(ctx.handle, c_paths, meta.ctypes.data_as(_capi._u64p), n,
                                          out.ctypes.data_as(_capi._u64p), sizes.ctypes.data_as(_capi._u64p),
                                          st.ctypes.data_as(_capi._i32p)), "oxh_hash_files_meta")
        return time.perf_counter() - t0, out, st

    def cpu_call():
        out = np.zeros((n, 2), dtype=np.uint64)
        sizes = np.zeros(n, dtype=np.uint64)
        st = np.zeros(n, dtype=np.int32)
        t0 = time.perf_counter()
        O.oxo_hash_files(c_paths, n, out.ctypes.data_as(oracle._u64p), sizes.ctypes.data_as(oracle._u64p),
                         st.ctypes.data_as(oracle._i32p), a.threads)
        return time.perf_counter() - t0, out, st

    if not a.only_procs:
        # fused add (hash + version-store publish from the same pinned bytes, one syncfs per slot before
        # the renames and one after) vs the reference loop restated (hash, then re-read + re-hash + write +
        # fsync + rename + parent fsync per new file), warm cache, fresh stores
        vroot = os.path.join(a.dir, ".oxen_gpu", "versions", "files")
        rroot = os.path.join(a.dir, ".oxen_ref", "versions", "files")
        oracle.hash_files(paths[: min(len(paths), 1000)], a.threads)
        t0 = time.perf_counter()
        gd, _, gst, gstored = hasher.add_files(paths, vroot, ctx)
        res["gpu_add_fused_s"] = round(time.perf_counter() - t0, 3)
        t0 = time.perf_counter()
        rout, _, rst, rstored = oracle.add_files(paths, rroot, a.threads)  # AtomicTempFile fsyncs per blob
        res["cpu_ref_add_s"] = round(time.perf_counter() - t0, 3)
        # the same loop without the per-blob fsyncs (the r01 restatement), for the A/B
        nroot = os.path.join(a.dir, ".oxen_nosync", "versions", "files")
        t0 = time.perf_counter()
        oracle.add_files(paths, nroot, a.threads, sync=False)
        res["cpu_ref_add_nosync_s"] = round(time.perf_counter() - t0, 3)
        shutil.rmtree(os.path.join(a.dir, ".oxen_nosync"), ignore_errors=True)
        res["gpu_add_fused_GiBs"] = round(nbytes / res["gpu_add_fused_s"] / 2**30, 2)
        res["cpu_ref_add_GiBs"] = round(nbytes / res["cpu_ref_add_s"] / 2**30, 2)
        res["add_blobs_written"] = [int(sum(gstored)), int(rstored.sum())]
        res["add_digests_bit_exact"] = [(int(hi) << 64) | int(lo) for lo, hi in rout] == gd
        # `oxen fsck` over the store the add just built (dry run: counts only), GPU vs the restated loop
        t0 = time.perf_counter()
        gf = hasher.clean_corrupted_versions(vroot, dry_run=True, ctx=ctx)
        res["gpu_fsck_s"] = round(time.perf_counter() - t0, 3)
        t0 = time.perf_counter()
        rf = oracle.clean_corrupted_versions(rroot, dry_run=True, threads=a.threads)
        res["cpu_ref_fsck_s"] = round(time.perf_counter() - t0, 3)
        res["fsck_counts"] = [{k: gf[k] for k in rf}, rf]
        shutil.rmtree(os.path.join(a.dir, ".oxen_gpu"), ignore_errors=True)
        shutil.rmtree(os.path.join(a.dir, ".oxen_ref"), ignore_errors=True)

        # staging-slot size sweep (warm cache): small slots stay in the host L3, so the pread copy and
        # the H2D DMA read do not both go through DRAM
        sweep = {}
        for mib in [int(x) for x in a.staging_mib.split(",") if x]:
            cs = _capi.Context(0, staging_bytes=mib << 20)
            ts = []
            for _ in range(3):
                out = np.zeros((n, 2), dtype=np.uint64)
                sz = np.zeros(n, dtype=np.uint64)
                stt = np.zeros(n, dtype=np.int32)
                t0 = time.perf_counter()
                _capi.check(L.oxh_hash_files(cs.handle, c_paths, n, out.ctypes.data_as(_capi._u64p),
                                             sz.ctypes.data_as(_capi._u64p), stt.ctypes.data_as(_capi._i32p)), "sweep")
                ts.append(time.perf_counter() - t0)
            cs.close()
            sweep[f"staging_{mib}MiB_GiBs"] = round(nbytes / min(ts) / 2**30, 2)
        res["gpu_e2e_warm_staging_sweep"] = sweep

    runs = {}
    # warm: GPU and CPU alternate, 5 rounds (host timings on a shared box vary by +-20 % run to run)
    oracle.hash_files(paths[: min(len(paths), 1000)], a.threads)
    wt = {"gpu_e2e": [], "gpu_e2e_meta": [], "cpu_ref": []}
    calls = {"gpu_e2e": gpu_call, "gpu_e2e_meta": gpu_meta_call, "cpu_ref": cpu_call}
    for _ in range(5):
        for who in ("gpu_e2e", "gpu_e2e_meta", "cpu_ref"):
            dt, out, st = calls[who]()
            assert (st == 0).all(), "file errors"
            runs[(who, "warm")] = out
            wt[who].append(dt)
    for who in wt:
        res[f"{who}_warm_s"] = round(float(np.median(wt[who])), 3)
        res[f"{who}_warm_GiBs"] = round(nbytes / float(np.median(wt[who])) / 2**30, 2)
        res[f"{who}_warm_s_all"] = [round(x, 3) for x in wt[who]]
    for who in ("gpu_e2e", "cpu_ref"):
        drop_cache(paths)
        dt, out, st = gpu_call() if who == "gpu_e2e" else cpu_call()
        assert (st == 0).all(), "file errors"
        runs[(who, "cold")] = out
        res[f"{who}_cold_s"] = round(dt, 3)
        res[f"{who}_cold_GiBs"] = round(nbytes / dt / 2**30, 2)
    res["digests_bit_exact"] = (all(np.array_equal(runs[("gpu_e2e", c)], runs[("cpu_ref", c)]) for c in ("warm", "cold"))
                                and np.array_equal(runs[("gpu_e2e_meta", "warm")], runs[("cpu_ref", "warm")]))
    res.update(sharded(a, paths, meta, nbytes, cpu_call, drop_cache))
    # the Python mirror (hasher.hash_files_128bit) on warm cache, for its wrapper overhead
    t0 = time.perf_counter()
    d, _, _ = hasher.hash_files_128bit(paths, ctx)
    res["python_mirror_warm_s"] = round(time.perf_counter() - t0, 3)
    print(json.dumps(res), flush=True)
    ctx.close()
    if not a.keep:
        shutil.rmtree(a.dir, ignore_errors=True)


if __name__ == "__main__":
    main()
