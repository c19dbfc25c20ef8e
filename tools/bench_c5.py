"""Config 5: large-file hashing (experiments/block-level-dedup), device-resident, 1 MI355X.

    python tools/bench_c5.py [--files 16] [--gib 8]

16 x 8 GiB blobs (128 GiB) resident in HBM. Times, with HIP events on the launch stream:
  chunk8k / chunk64k   fixed-size chunk digests (fixedsize.rs:52-102; TestOxen uses 64 KiB,
                       main.rs:129-133; the makefile default is 8 KiB) over all files
  whole_file           K1L whole-file digest of every file (hasher.rs:150-174 streams files
                       >= 1e9 B; same XXH3-128): block sums chip-wide + one serial chain per file,
                       the 16 files' chains on 16 streams so they run concurrently
Checks: every whole-file digest and a sample of chunk digests against the CPU oracle over bytes
regenerated on the host (splitmix64 stream), full-file oracle hashing on a subset of files.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=16)
    ap.add_argument("--gib", type=float, default=8.0)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--check-files", type=int, default=2, help="files whose whole digest is checked on the CPU")
    a = ap.parse_args()

    import numpy as np
    import torch

    from oracle import oracle
    from oxen_amd import _capi
    from oxen_amd.device import (chunk_digests_device, fill_splitmix, large_digest_device, large_digests_device,
                                 to_numpy_u64)
    from oxen_amd.workloads import splitmix_bytes

    flen = int(a.gib * (1 << 30))
    ctx = _capi.Context(0)
    bufs = []
    for f in range(a.files):
        b = torch.empty(flen, dtype=torch.uint8, device="cuda")
        fill_splitmix(b, 1000 + f)
        bufs.append(b)
    torch.cuda.synchronize()
    total = flen * a.files
    res = {"config": f"C5: {a.files} x {flen} B blobs device-resident (splitmix64, seeds 1000+f)",
           "bytes": total}

    def timed(fn, reps):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ts = []
        for _ in range(reps):
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 1e3)
        return float(np.median(ts))

    chunk_out = {}
    for chunk in (8192, 65536):
        outs = [torch.empty(((flen + chunk - 1) // chunk, 2), dtype=torch.int64, device="cuda") for _ in bufs]

        def run(chunk=chunk, outs=outs):
            for b, o in zip(bufs, outs):
                chunk_digests_device(b, chunk, out=o)

        t = timed(run, a.reps)
        res[f"chunk{chunk // 1024}k_s"] = round(t, 4)
        res[f"chunk{chunk // 1024}k_GiBs"] = round(total / t / 2**30, 1)
        res[f"chunk{chunk // 1024}k_TBs"] = round(total / t / 1e12, 3)
        chunk_out[chunk] = outs

    # K1 variant sweep on the chunk workloads (interleaved, median of reps)
    sweep = {}
    for chunk in (8192, 65536):
        outs = chunk_out[chunk]
        for v in (0, 4, 8, 64, 72):
            def runv(chunk=chunk, outs=outs, v=v):
                _capi.lib().oxh_set_kernel_variant(v)
                for b, o in zip(bufs[:4], outs[:4]):
                    chunk_digests_device(b, chunk, out=o)
            sweep[f"chunk{chunk // 1024}k_v{v}_TBs"] = round(4 * flen / timed(runv, a.reps) / 1e12, 3)
    _capi.lib().oxh_set_kernel_variant(0)
    res["variant_sweep"] = sweep

    # whole-file digests: one batched K1L call -- block sums per file, then all serial chains in one
    # launch (one wave per file, running concurrently)
    wall = torch.empty((len(bufs), 2), dtype=torch.int64, device="cuda")
    wouts = [wall[f] for f in range(len(bufs))]

    def whole():
        large_digests_device(bufs, out=wall)

    t = timed(whole, a.reps)
    res["whole_file_all_s"] = round(t, 4)
    res["whole_file_all_GiBs"] = round(total / t / 2**30, 1)
    # one file alone (the latency of a single chain)
    t1 = timed(lambda: large_digest_device(ctx, bufs[0], out=wouts[0]), a.reps)
    res["whole_file_one_s"] = round(t1, 4)

    # correctness
    ok = True
    for f in range(min(a.check_files, a.files)):
        data = np.empty(flen, dtype=np.uint8)
        step = 1 << 30
        for s0 in range(0, flen, step):
            n = min(step, flen - s0)
            data[s0:s0 + n] = splitmix_bytes(1000 + f, s0, n)
        want = oracle.batch(data, np.array([0], dtype=np.uint64), np.array([flen], dtype=np.uint64))
        got = to_numpy_u64(wouts[f]).reshape(1, 2)
        ok &= bool(np.array_equal(got, want))
        for chunk in (8192, 65536):
            idx = np.linspace(0, (flen + chunk - 1) // chunk - 1, 256).astype(np.uint64)
            g = to_numpy_u64(chunk_out[chunk][f]).reshape(-1, 2)
            lens = np.minimum(np.uint64(chunk), np.uint64(flen) - idx * np.uint64(chunk))
            want_c = oracle.batch(data, idx * np.uint64(chunk), lens, threads=8)
            ok &= bool(np.array_equal(g[idx.astype(np.int64)], want_c))
        del data
    # cross-check the remaining files' whole digests only against determinism (second run)
    first = [tuple(int(x) for x in to_numpy_u64(o)) for o in wouts]
    whole()
    torch.cuda.synchronize()
    ok &= first == [tuple(int(x) for x in to_numpy_u64(o)) for o in wouts]
    res["digests_bit_exact"] = bool(ok)
    res["checked_files_full_cpu"] = min(a.check_files, a.files)
    print(json.dumps(res), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
