"""C5 end to end: FastCDC chunk tables + chunk digests of files ON DISK, results in host memory
(BASELINE configs[4], experiments/block-level-dedup fastcdchunker.rs:75-98: fs::read -> v2020 ->
xxh3_128 per chunk), through the C ABI's oxh_fastcdc_files. Prints one JSON object.

    python tools/bench_fastcdc_e2e.py --dir /tmp/c5 --files 16 --gib 8 --chunk 8192 --reps 3 [--cold] [--fixed]

--devices 0,1,...: one context per entry (oxh_*_files_multi: the files shared out by bytes, one PCIe
link per GPU on a multi-GPU node; a repeated device gives that device two pipelines).
--fixed: fixed-size chunks of --chunk bytes instead (fixedsize_multithreaded.rs:78-110, through
oxh_chunk_digests_files; the oracle's oxo_fixed_files beside it).

The files (splitmix64 bytes, seed 5000 + i) are written once (generated on the GPU, written through the
page cache) and reused. Warm = every file in the page cache; cold = posix_fadvise(DONTNEED) on every file
before the run. Beside the GPU call, the C oracle runs the same per-file loop on all host threads the
process may use (oracle/fastcdc_oracle.c oxo_fastcdc_files: read (or mmap) -> v2020 chunking ->
xxh3_128 per chunk, one file per thread), and every file's chunk count and record fingerprint
(XXH3-128 over its (offset, length, lo, hi) records) must be equal on both sides.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def usable_cpus() -> int:
    n = len(os.sched_getaffinity(0))
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max" and int(period) > 0:
            n = min(n, max(1, -(-int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def make_files(d: str, nfiles: int, size: int) -> list[str]:
    """splitmix64 files generated on the GPU 256 MiB at a time and written through the page cache."""
    import torch

    from oxen_amd.device import fill_splitmix

    os.makedirs(d, exist_ok=True)
    paths = [os.path.join(d, f"blob_{i:02d}.bin") for i in range(nfiles)]
    step = 256 << 20
    buf = torch.empty(step, dtype=torch.uint8, device="cuda")
    host = torch.empty(step, dtype=torch.uint8, pin_memory=True)
    for i, p in enumerate(paths):
        if os.path.exists(p) and os.path.getsize(p) == size:
            continue
        with open(p + ".tmp", "wb") as f:
            for o in range(0, size, step):
                n = min(step, size - o)
                fill_splitmix(buf, 5000 + i * 1_000_003 + o // step, (n + 7) // 8 * 8)
                host[:n].copy_(buf[:n])
                f.write(memoryview(host[:n].numpy()))
        os.replace(p + ".tmp", p)
    del buf
    return paths


def drop_cache(paths):
    for p in paths:
        fd = os.open(p, os.O_RDONLY)
        try:
            os.fsync(fd)
            os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
        finally:
            os.close(fd)


def warm_cache(paths, threads):
    """Read every file once (pages into the page cache) with a few threads."""
    from concurrent.futures import ThreadPoolExecutor

    def one(p):
        with open(p, "rb", buffering=0) as f:
            b = bytearray(64 << 20)
            while f.readinto(b):
                pass

    with ThreadPoolExecutor(min(threads, len(paths))) as ex:
        list(ex.map(one, paths))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default="/tmp/oxh_c5")
    ap.add_argument("--files", type=int, default=16)
    ap.add_argument("--gib", type=float, default=8.0)
    ap.add_argument("--chunk", type=int, default=8192)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cold", action="store_true", help="also time both sides from a cold page cache")
    ap.add_argument("--cpu", choices=["read", "mmap", "none"], default="mmap",
                    help="the CPU baseline's file access: read() whole files (fs::read) or mmap")
    ap.add_argument("--keep", action="store_true", help="keep the files")
    ap.add_argument("--fixed", action="store_true", help="fixed-size chunks of --chunk bytes instead of FastCDC")
    ap.add_argument("--devices", default="", help="comma-separated devices, one context each (the _multi entries)")
    args = ap.parse_args()

    from oracle import fastcdc as F
    from oracle import oracle
    from oxen_amd import _capi, dedup

    oracle.build()
    size = int(args.gib * (1 << 30))
    mn, av, mx = 4096, args.chunk, 2 * args.chunk
    threads = usable_cpus()
    t0 = time.perf_counter()
    paths = make_files(args.dir, args.files, size)
    gen_s = time.perf_counter() - t0
    total = size * len(paths)
    devices = [int(x) for x in args.devices.split(",") if x.strip()]
    ctxs = [_capi.Context(d) for d in devices] if len(devices) > 1 else None
    ctx = None if ctxs else _capi.Context(devices[0] if devices else 0)
    what = (f"fixed-size {args.chunk} B chunks" if args.fixed else f"FastCDC v2020 min {mn} avg {av} max {mx}")
    res = {"workload": f"{len(paths)} x {size} B files on disk (splitmix64), {what} "
                       f"+ XXH3-128 per chunk, chunk table + digests in host memory",
           "bytes": total, "gen_s": round(gen_s, 1), "host_threads": threads, "devices": devices or [0]}

    def gpu_once():
        t = time.perf_counter()
        if args.fixed:
            tab = dedup.chunk_digests_files(paths, args.chunk, ctx=ctx, ctxs=ctxs)
        else:
            tab = dedup.fastcdc_files(paths, mn, av, mx, ctx=ctx, ctxs=ctxs)
        return time.perf_counter() - t, tab

    def cpu_once():
        t = time.perf_counter()
        if args.fixed:
            c, fp, st = F.fixed_files(paths, args.chunk, threads=threads, mmap_files=args.cpu == "mmap")
        else:
            c, fp, st = F.files(paths, mn, av, mx, threads=threads, mmap_files=args.cpu == "mmap")
        return time.perf_counter() - t, (c, fp, st)

    warm_cache(paths, threads)
    gpu_once()  # first call: the pipeline's buffers are allocated
    gt, tab = [], None
    for _ in range(args.reps):
        dt, tab = gpu_once()
        gt.append(dt)
    assert (tab.status == 0).all(), tab.status
    res["gpu_warm_s"] = [round(x, 4) for x in gt]
    res["gpu_warm_median_s"] = round(float(np.median(gt)), 4)
    res["gpu_warm_gib_s"] = round(total / float(np.median(gt)) / 2**30, 2)
    res["chunks"] = int(tab.first[-1])
    # check: per file, the count and the record fingerprint against the C oracle's own loop
    if args.cpu != "none":
        ct, cres = [], None
        for _ in range(max(1, min(args.reps, 2))):
            dt, cres = cpu_once()
            ct.append(dt)
        c, fp, st = cres
        ok = bool((st == 0).all())
        for i in range(len(paths)):
            if args.fixed:
                dig = tab.file(i)
                sz = int(tab.sizes[i])
                off = np.arange(0, sz, args.chunk, dtype=np.uint64)
                ln = np.minimum(np.uint64(args.chunk), np.uint64(sz) - off)
            else:
                off, ln, dig = tab.file(i)
            ok = ok and int(c[i]) == len(off) and (int(fp[i, 0]), int(fp[i, 1])) == F.record_fingerprint(off, ln, dig)
        res["all_chunks_bit_exact"] = ok
        res["cpu_warm_s"] = [round(x, 3) for x in ct]
        res["cpu_warm_gib_s"] = round(total / min(ct) / 2**30, 2)
        res["cpu"] = {"threads": threads, "kind": "port", "access": args.cpu,
                      "what": "oracle/fastcdc_oracle.c " + ("oxo_fixed_files: per file read/mmap -> xxh3_128 per fixed chunk"
                                                            if args.fixed else
                                                            "oxo_fastcdc_files: per file read/mmap -> v2020 -> xxh3_128 per chunk")}
    if args.cold:
        gc = []
        for _ in range(max(1, min(args.reps, 2))):
            drop_cache(paths)
            dt, tab2 = gpu_once()
            gc.append(dt)
            assert int(tab2.first[-1]) == res["chunks"]
        res["gpu_cold_s"] = [round(x, 3) for x in gc]
        res["gpu_cold_gib_s"] = round(total / min(gc) / 2**30, 2)
        if args.cpu != "none":
            drop_cache(paths)
            dt, _ = cpu_once()
            res["cpu_cold_s"] = round(dt, 3)
            res["cpu_cold_gib_s"] = round(total / dt / 2**30, 2)
    try:
        res["cpu_model"] = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
    except (OSError, StopIteration):
        pass
    for c in ctxs or [ctx]:
        c.close()
    if not args.keep:
        for p in paths:
            os.unlink(p)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
