"""K1 throughput vs item alignment and raggedness (why K1 over FastCDC chunks runs below C2's rate).

    python tools/k1_align_probe.py

Cases (each ~6.5 GB device-resident, K1 = oxh_xxh3_128_batch_device, HIP-event timed):
  c2_aligned     100 000 x 64 KiB at 64 KiB pitch (the headline layout)
  c2_shift3      the same items starting 3 bytes later (every load misaligned)
  ragged_256     lengths uniform in [4 KiB, 128 KiB), packed at 256-B alignment
  ragged_packed  the same lengths packed back to back (arbitrary alignment, like FastCDC chunks)
  ragged_4       the same lengths packed at 4-B alignment (no item takes the byte-shift path)
  ragged_4p1     ragged_4 shifted by 1 B (every item takes the byte-shift path)
  ragged_packed_vN  ragged_packed with K1 variant N forced (oxh_set_kernel_variant)
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

    from oxen_amd.device import fill_splitmix, xxh3_128_batch_device

    dev = torch.device("cuda:0")
    rng = np.random.default_rng(0)
    total = 100_000 * 65536
    arena = torch.empty(total + (1 << 20), dtype=torch.uint8, device=dev)
    fill_splitmix(arena, 5)

    def case(offs, lens):
        o = torch.from_numpy(np.asarray(offs, dtype=np.uint64).view(np.int64)).to(dev)
        ln = torch.from_numpy(np.asarray(lens, dtype=np.uint64).view(np.int64)).to(dev)
        out = torch.empty((len(lens), 2), dtype=torch.int64, device=dev)
        for _ in range(3):
            xxh3_128_batch_device(arena, o, ln, out)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        reps = 20
        for _ in range(reps):
            xxh3_128_batch_device(arena, o, ln, out)
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / 1e3 / reps
        b = int(np.sum(lens))
        return {"ms": round(t * 1e3, 4), "TB_s": round(b / t / 1e12, 3), "items": len(lens), "bytes": b}

    res = {}
    n = 100_000
    res["c2_aligned"] = case(np.arange(n) * 65536, np.full(n, 65536))
    for sh in (1, 3, 4, 8, 12):
        res[f"c2_shift{sh}"] = case(np.arange(n) * 65536 + sh, np.full(n, 65536))
    lens = rng.integers(4096, 131072, 2 * total // (4096 + 131072))
    lens = lens[: np.searchsorted(np.cumsum((lens + 255) // 256 * 256), total)]
    offs256 = np.concatenate([[0], np.cumsum((lens + 255) // 256 * 256)[:-1]])
    res["ragged_256"] = case(offs256, lens)
    lens2 = lens[: np.searchsorted(np.cumsum(lens), total)]
    offs_packed = np.concatenate([[0], np.cumsum(lens2)[:-1]])
    res["ragged_packed"] = case(offs_packed, lens2)
    offs4 = np.concatenate([[0], np.cumsum((lens2 + 3) // 4 * 4)[:-1]])
    res["ragged_4"] = case(offs4, lens2)
    res["ragged_4p1"] = case(offs4 + 1, lens2)
    from oxen_amd import _capi
    layouts = {"c2_aligned": (np.arange(n) * 65536, np.full(n, 65536)), "ragged_256": (offs256, lens),
               "ragged_packed": (offs_packed, lens2), "ragged_4p1": (offs4 + 1, lens2)}
    for v in (64, 65, 66, 68, 72, 76, 8):
        _capi.lib().oxh_set_kernel_variant(v)
        for name, (o, ln) in layouts.items():
            res[f"{name}_v{v}"] = case(o, ln)
    _capi.lib().oxh_set_kernel_variant(0)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
