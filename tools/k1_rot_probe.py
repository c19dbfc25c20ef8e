"""A/B of K1's rotated start (variant bit 10, DESIGN §4 "K1 rotated start") against the shipped
shapes on C2 (100 000 x 64 KiB device-resident), after a clock-ramp pre-warm, interleaved, median of
rounds; and a parity sweep: ragged lengths (241 B .. 300 KiB, packed at byte offsets) hashed by every
variant must give variant 8's digests, and a sample the oracle's. Needs the probe build:

    python tools/build_probe_lib.py
    python tools/with_lib.py tools/probe/liboxen_hash.so tools/k1_rot_probe.py [--rounds 7]
Prints one JSON object.
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

VARIANTS = (8, 1032, 0, 1024)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    a = ap.parse_args()
    import torch

    from oracle import oracle
    from oxen_amd import _capi
    from oxen_amd.device import DeviceArena

    L = _capi.lib()
    res = {"variants": list(VARIANTS)}
    # parity: ragged packed items at byte offsets (every variant against variant 8, a sample against the oracle)
    rng = np.random.default_rng(11)
    lens = np.concatenate([rng.integers(241, 300_000, 3000), np.arange(241, 241 + 64), 1024 * np.arange(1, 80) + 1,
                           4096 * np.arange(1, 80), 4096 * np.arange(1, 80) - 1]).astype(np.uint64)
    offs = np.zeros(lens.size, dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1] + rng.integers(0, 7, lens.size - 1).astype(np.uint64))
    total = int(offs[-1] + lens[-1])
    host = rng.integers(0, 256, total, dtype=np.uint8)
    arena = torch.from_numpy(host).cuda()
    d_off = torch.from_numpy(offs.astype(np.int64)).cuda()
    d_len = torch.from_numpy(lens.astype(np.int64)).cuda()
    outs = {}
    for v in VARIANTS:
        L.oxh_set_kernel_variant(v)
        o = torch.zeros((lens.size, 2), dtype=torch.int64, device="cuda")
        _capi.check(L.oxh_xxh3_128_batch_device(arena.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), lens.size,
                                                o.data_ptr(), _capi.OXH_MODE_WAVE, None), "batch")
        torch.cuda.synchronize()
        outs[v] = o.cpu().numpy().view(np.uint64)
    L.oxh_set_kernel_variant(0)
    want = outs[8]
    sample = rng.choice(lens.size, 300, replace=False)
    ora = oracle.batch(host, offs[sample], lens[sample], threads=8)
    res["parity"] = {str(v): bool(np.array_equal(outs[v], want)) for v in VARIANTS}
    res["parity_oracle_sample"] = bool(np.array_equal(want[sample], ora))
    del arena
    # C2 timing
    n, item = 100_000, 65_536
    da = DeviceArena.splitmix([item] * n, seed=1)
    out = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.6:
        for _ in range(8):
            da.hash(out)
        torch.cuda.synchronize()
    times = {v: [] for v in VARIANTS}
    digests = {}
    for _ in range(a.rounds):
        for v in VARIANTS:
            L.oxh_set_kernel_variant(v)
            da.hash(out)
            ms = []
            for _ in range(10):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                da.hash(out)
                e1.record()
                torch.cuda.synchronize()
                ms.append(e0.elapsed_time(e1))
            times[v].append(statistics.median(ms))
            digests[v] = out.cpu()
    L.oxh_set_kernel_variant(0)
    res["c2_kernel_ms_median"] = {str(v): round(statistics.median(t), 4) for v, t in times.items()}
    res["c2_frac"] = {str(v): round(n * item / (statistics.median(t) / 1e3) / 8e12, 4) for v, t in times.items()}
    res["c2_digests_equal"] = all(torch.equal(digests[v], digests[8]) for v in VARIANTS)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
