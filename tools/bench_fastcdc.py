"""FastCDC v2020 chunking + chunk digests of device-resident blobs (BASELINE configs[4] shape:
16 x 8 GiB, experiments/block-level-dedup). Prints one JSON line.

    python tools/bench_fastcdc.py [--files 16] [--gib 8] [--chunk 65536] [--reps 3]

Timed: one oxh_fastcdc_device call (F1 scan, F2 speculative walks, F3 stitch, compaction, K1 over the
chunk table) with the inputs resident in HBM. The chunk table of the first file is checked against the
C oracle on a prefix (oracle/fastcdc_oracle.c), which is also timed as the single-core CPU baseline.
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


def check_all(arena, offs, size, c_off, c_len, dig, first, mn, av, mx, workers: int = 4) -> dict:
    """Every file's chunk table (offsets, lengths) and every chunk digest against the C oracle, files
    copied back one at a time per worker (host memory: workers x file size)."""
    import time as _t
    from concurrent.futures import ThreadPoolExecutor

    from oracle import fastcdc as F
    from oracle import oracle
    from oxen_amd.device import to_numpy_u64

    t0 = _t.perf_counter()
    got_off = to_numpy_u64(c_off)
    got_len = to_numpy_u64(c_len)
    got_dig = to_numpy_u64(dig).reshape(-1, 2)

    def one(i):
        lo, hi = int(first[i]), int(first[i + 1])
        o = int(offs[i])
        host = arena[o:o + size].cpu().numpy()
        want = F.chunks(host, mn, av, mx)  # the C oracle over the whole file (ctypes releases the GIL)
        ok = len(want) == hi - lo
        ok = ok and bool(np.array_equal(got_off[lo:hi] - np.uint64(o), want[:, 0]) and np.array_equal(got_len[lo:hi], want[:, 1]))
        if ok:
            ok = bool(np.array_equal(oracle.batch(host, want[:, 0], want[:, 1], threads=4), got_dig[lo:hi]))
        return ok, hi - lo

    with ThreadPoolExecutor(workers) as ex:
        rs = list(ex.map(one, range(len(offs))))
    return {"files_checked": len(rs), "chunks_checked": int(sum(r[1] for r in rs)),
            "all_files_bit_exact": all(r[0] for r in rs), "check_s": round(_t.perf_counter() - t0, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=16)
    ap.add_argument("--gib", type=float, default=8.0)
    ap.add_argument("--chunk", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--check-mib", type=int, default=256)
    ap.add_argument("--check-all", action="store_true",
                    help="also check EVERY file's whole chunk table and every chunk digest against the C oracle")
    ap.add_argument("--variant", type=int, default=0, help="force a K1 variant (0 = the library's choice)")
    args = ap.parse_args()

    import torch

    from oracle import fastcdc as F
    from oracle import oracle
    from oxen_amd.device import fastcdc_device, fastcdc_outputs, fill_splitmix, to_numpy_u64

    dev = torch.device("cuda:0")
    from oxen_amd import _capi
    _capi.lib().oxh_set_kernel_variant(args.variant)
    size = int(args.gib * 2**30)
    pitch = (size + 4095) // 4096 * 4096
    arena = torch.empty(pitch * args.files, dtype=torch.uint8, device=dev)
    fill_splitmix(arena, 77)
    offs = np.arange(args.files, dtype=np.uint64) * np.uint64(pitch)
    lens = np.full(args.files, size, dtype=np.uint64)
    mn, av, mx = 4096, args.chunk, 2 * args.chunk
    total = size * args.files

    # chunk tables allocated once, outside the timed region (a caller chunking repeatedly keeps them)
    outs = [fastcdc_outputs(arena, lens, mn) for _ in range(2)]
    c_off, c_len, dig, first = fastcdc_device(arena, offs, lens, mn, av, mx, out=outs[1])  # warm-up
    torch.cuda.synchronize()
    def fingerprint(c_off, c_len, dig, first):  # whole-output checksum: every rep must agree
        n_ = int(first[-1])
        return (n_, int(c_off[:n_].sum()), int(c_len[:n_].sum()), int(dig[:n_].view(torch.int64).sum()))

    fp0 = fingerprint(c_off, c_len, dig, first)
    times, same = [], True
    for r in range(args.reps):
        t0 = time.perf_counter()
        c_off, c_len, dig, first = fastcdc_device(arena, offs, lens, mn, av, mx, out=outs[r % 2])
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
        same = same and fingerprint(c_off, c_len, dig, first) == fp0
    t = float(np.median(times))
    nchunks = int(first[-1])

    # bit-exact check of a prefix of file 0 (chunks that end inside the prefix are final)
    m = min(size, args.check_mib << 20)
    host = arena[:m].cpu().numpy()
    t0 = time.perf_counter()
    want = F.chunks(host, mn, av, mx)
    cpu_s = time.perf_counter() - t0
    got_off = to_numpy_u64(c_off[: int(first[1])])
    got_len = to_numpy_u64(c_len[: int(first[1])])
    k = len(want) - 1  # the oracle's last chunk is cut by the prefix end
    exact = bool(np.array_equal(got_off[:k], want[:k, 0]) and np.array_equal(got_len[:k], want[:k, 1]))
    wd = oracle.batch(host, want[:k, 0], want[:k, 1], threads=16)
    exact = exact and bool(np.array_equal(to_numpy_u64(dig[:k]).reshape(-1, 2), wd))
    full = None
    if args.check_all:
        full = check_all(arena, offs, size, c_off, c_len, dig, first, mn, av, mx)
        exact = exact and full["all_files_bit_exact"]
    res = {"workload": f"{args.files} x {args.gib:g} GiB splitmix blobs, FastCDC v2020 min/avg/max {mn}/{av}/{mx} "
                       f"+ XXH3-128 per chunk, device-resident",
           "bytes": total, "chunks": nchunks, "mean_chunk": total / max(nchunks, 1),
           "s_median": round(t, 4), "s_all": [round(x, 4) for x in times],
           "GiB_s": round(total / t / 2**30, 1), "GB_s": round(total / t / 1e9, 1),
           "prefix_checked_bytes": m, "prefix_chunks_bit_exact": exact, "reps_identical": same,
           "cpu_oracle_1core_GiB_s": round(m / cpu_s / 2**30, 3)}
    if full:
        res["check_all"] = full
    print(json.dumps(res), flush=True)
    if not (exact and same):
        sys.exit(1)


if __name__ == "__main__":
    main()
