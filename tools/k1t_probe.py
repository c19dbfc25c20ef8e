"""K1T (XXH3-128 + fused text counts, repositories/metadata/text.rs:11-20) vs K1 per kernel variant.

    python tools/k1t_probe.py

Layouts (~6.5 GB device-resident, HIP-event timed, 20 launches): c2 = 100 000 x 64 KiB packed;
ragged = lengths uniform in [4 KiB, 128 KiB) packed back to back. Variant 8 / 72 / 4 (= the <0>
instantiation) forced with oxh_set_kernel_variant. Every K1T launch's digests must equal K1's and
its counts must match numpy on 256 sampled items.
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
    from oxen_amd.device import fill_splitmix, xxh3_128_batch_device, xxh3_128_text_batch_device

    dev = torch.device("cuda:0")
    rng = np.random.default_rng(3)
    total = 100_000 * 65536
    arena = torch.empty(total + (1 << 20), dtype=torch.uint8, device=dev)
    fill_splitmix(arena, 11)
    # make it text-like: map bytes to printable ASCII with ~1/64 newlines and some UTF-8 continuations
    a = arena[:total]
    a.remainder_(96).add_(32)
    a[a == 127] = 10
    a[a == 126] = 0x80 | 0x25
    lens_r = rng.integers(4096, 131072, 2 * total // (4096 + 131072))
    lens_r = lens_r[: np.searchsorted(np.cumsum(lens_r), total)]
    layouts = {"c2": (np.arange(100_000) * 65536, np.full(100_000, 65536)),
               "ragged": (np.concatenate([[0], np.cumsum(lens_r)[:-1]]), lens_r)}
    host = arena[:total].cpu().numpy()
    res = {}
    L = _capi.lib()
    for name, (offs, lens) in layouts.items():
        o = torch.from_numpy(np.asarray(offs, dtype=np.int64)).to(dev)
        ln = torch.from_numpy(np.asarray(lens, dtype=np.int64)).to(dev)
        n = len(lens)
        nbytes = int(np.sum(lens))
        ref = xxh3_128_batch_device(arena, o, ln)
        sample = rng.choice(n, 256, replace=False)
        want = np.array([[1 + np.count_nonzero(host[offs[i]:offs[i] + lens[i]] == 10),
                          lens[i] - np.count_nonzero((host[offs[i]:offs[i] + lens[i]] & 0xC0) == 0x80)] for i in sample])
        for v in (8, 72, 4):
            L.oxh_set_kernel_variant(v)
            out = torch.empty((n, 2), dtype=torch.int64, device=dev)
            cnt = torch.empty((n, 2), dtype=torch.int64, device=dev)
            for fn, key in ((lambda: xxh3_128_batch_device(arena, o, ln, out), "k1"),
                            (lambda: xxh3_128_text_batch_device(arena, o, ln, out, cnt), "k1t")):
                for _ in range(3):
                    fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                t = e0.elapsed_time(e1) / 1e3 / 20
                res[f"{name}_{key}_v{v}_TBs"] = round(nbytes / t / 1e12, 3)
                assert torch.equal(out, ref), (name, key, v)
            got = cnt.cpu().numpy()[sample]
            assert np.array_equal(got, want), (name, v)
        L.oxh_set_kernel_variant(0)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
