"""K1 on small items: where the rate goes between 64 KiB items (C2, 6.9 TB/s) and FastCDC's ~8 KiB
chunks (5.7 TB/s). GPU box only.

    python tools/k1_small_probe.py [variant ...]

Cases (~6.4 GB device-resident each, K1 = oxh_xxh3_128_batch_device, HIP events, 20 reps):
  fixed_L         L-byte items at L pitch (L = 4, 8, 16, 64 KiB)
  fixed8k_shiftS  8 KiB items at 8 KiB pitch starting S bytes later (S = 1: every item takes the
                  byte-shift path; 4 / 16 / 64 / 128: dword-aligned loads that straddle lines)
  cdc_packed      lengths uniform in [4 KiB, 16 KiB) packed back to back (FastCDC-like)
  cdc_256         the same lengths at 256-B alignment
  cdc_packed_w64sort  cdc_packed, listed in length order within windows of 64 items (K1R lockstep)
  cdc64_packed / cdc64_256   lengths uniform in [4 KiB, 128 KiB) (FastCDC at 64 KiB), likewise
PROBE_BYTES sets the arena size (default 6.4 GB). PROBE_CASES=a,b limits the run to those cases. PROBE_WG=1,4 repeats every case with that many waves per
K1 workgroup (OXH_K1_WG_WAVES), alternating.
for each K1 variant given (default: 72 8).
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from oxen_amd import _capi
    from oxen_amd.device import fill_splitmix, xxh3_128_batch_device

    variants = [int(v) for v in sys.argv[1:]] or [72, 8]
    dev = torch.device("cuda:0")
    total = int(os.environ.get("PROBE_BYTES", 6_400_000_000))
    arena = torch.empty(total + (1 << 20), dtype=torch.uint8, device=dev)
    fill_splitmix(arena, 5)
    rng = np.random.default_rng(0)

    def case(offs, lens):
        o = torch.from_numpy(np.asarray(offs, dtype=np.uint64).view(np.int64)).to(dev)
        ln = torch.from_numpy(np.asarray(lens, dtype=np.uint64).view(np.int64)).to(dev)
        out = torch.empty((len(lens), 2), dtype=torch.int64, device=dev)
        for _ in range(3):
            xxh3_128_batch_device(arena, o, ln, out)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        e0.record()
        for _ in range(reps):
            xxh3_128_batch_device(arena, o, ln, out)
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / 1e3 / reps
        b = int(np.sum(lens))
        return {"ms": round(t * 1e3, 4), "TB_s": round(b / t / 1e12, 3), "items": len(lens)}

    layouts = {}
    for kib in (4, 8, 16, 64):
        L = kib * 1024
        n = total // L
        layouts[f"fixed_{kib}k"] = (np.arange(n) * L, np.full(n, L))
    n8 = total // 8192 - 1
    for sh in (1, 4, 16, 64, 128):
        layouts[f"fixed8k_shift{sh}"] = (np.arange(n8) * 8192 + sh, np.full(n8, 8192))
    lens = rng.integers(4096, 16384, 2 * total // (4096 + 16384))
    lens = lens[: np.searchsorted(np.cumsum((lens + 255) // 256 * 256), total)]
    layouts["cdc_packed"] = (np.concatenate([[0], np.cumsum(lens)[:-1]]), lens)
    layouts["cdc_256"] = (np.concatenate([[0], np.cumsum((lens + 255) // 256 * 256)[:-1]]), lens)
    # the same packed items, listed (not moved) in length order within each window of 64 consecutive
    # items: a K1R wave's four rows then carry items of similar length
    o_p, l_p = layouts["cdc_packed"]
    nwin = len(l_p) // 64 * 64
    order = np.argsort(l_p[:nwin].reshape(-1, 64), axis=1, kind="stable") + (np.arange(nwin // 64) * 64)[:, None]
    order = np.concatenate([order.ravel(), np.arange(nwin, len(l_p))])
    layouts["cdc_packed_w64sort"] = (o_p[order], l_p[order])
    lens = rng.integers(4096, 131072, 2 * total // (4096 + 131072))
    lens = lens[: np.searchsorted(np.cumsum((lens + 255) // 256 * 256), total)]
    layouts["cdc64_packed"] = (np.concatenate([[0], np.cumsum(lens)[:-1]]), lens)
    layouts["cdc64_256"] = (np.concatenate([[0], np.cumsum((lens + 255) // 256 * 256)[:-1]]), lens)
    only = os.environ.get("PROBE_CASES")
    if only:
        layouts = {k: v for k, v in layouts.items() if k in only.split(",")}
    res = {}
    wgs = os.environ.get("PROBE_WG", "")
    wgs = [int(x) for x in wgs.split(",")] if wgs else [None]
    for v in variants:
        _capi.lib().oxh_set_kernel_variant(v)
        for name, (o, ln) in layouts.items():
            for rep in range(2 if len(wgs) > 1 else 1):
                for w in wgs:
                    if w is not None:
                        os.environ["OXH_K1_WG_WAVES"] = str(w)
                    key = f"{name}_v{v}" + (f"_wg{w}_r{rep}" if w is not None else "")
                    res[key] = case(o, ln)
                    print(key, res[key], file=sys.stderr, flush=True)
    os.environ.pop("OXH_K1_WG_WAVES", None)
    _capi.lib().oxh_set_kernel_variant(0)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
