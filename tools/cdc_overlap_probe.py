"""Does FastCDC chunking (the scan F1 or the walk W, both VALU-bound) overlap with K1 over the chunks
(K1R: HBM/TA-bound, VALU issue ~55 %)? C5 shape (16 x 8 GiB device-resident), two ways:

  serial   one oxh_fastcdc_device call with digests (F1 -> F2/F3 -> emit -> K1 on one stream)
  overlap  files in G groups; group g is chunked (no digests) on stream A while K1 hashes group
           g-1's chunk table on stream B

Both must produce the same chunk digests (sum of all digest words and chunk count compared).
Prints one JSON line.

    python tools/cdc_overlap_probe.py [--files 16] [--gib 8] [--chunks 8192,65536] [--groups 2,4,8]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=16)
    ap.add_argument("--gib", type=float, default=8.0)
    ap.add_argument("--chunks", default="8192,65536")
    ap.add_argument("--groups", default="2,4,8")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cu-split", default="0", help="comma list of k: stream A gets CUs with i %% 8 < k, "
                    "stream B the rest (hipExtStreamCreateWithCUMask); 0 = unmasked torch streams")
    ap.add_argument("--k1-variant", type=int, default=0,
                    help="K1 shape for the overlap runs' separate K1 launches (oxh_set_kernel_variant; 0 = "
                    "OXH_MODE_WAVE_PACKED's default, 264 = K1R, the serial call's choice at small chunks)")
    args = ap.parse_args()

    import torch

    from oxen_amd import _capi
    from oxen_amd.device import fastcdc_device, fastcdc_outputs, fill_splitmix, xxh3_128_batch_device

    dev = torch.device("cuda:0")
    size = int(args.gib * 2**30)
    pitch = (size + 4095) // 4096 * 4096
    arena = torch.empty(pitch * args.files, dtype=torch.uint8, device=dev)
    fill_splitmix(arena, 77)
    offs = np.arange(args.files, dtype=np.uint64) * np.uint64(pitch)
    lens = np.full(args.files, size, dtype=np.uint64)
    total = size * args.files
    import ctypes

    hip = ctypes.CDLL("libamdhip64.so")

    def masked_stream(bits):
        words = (ctypes.c_uint32 * 8)()
        for i in bits:
            words[i // 32] |= 1 << (i % 32)
        h = ctypes.c_void_p()
        rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), 8, words)
        if rc != 0:
            raise RuntimeError(f"hipExtStreamCreateWithCUMask: {rc}")
        return h.value

    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    res = {"workload": f"{args.files} x {args.gib:g} GiB splitmix blobs, FastCDC v2020 + XXH3-128 per chunk",
           "bytes": total}

    def fp(dig, n):
        return (n, int(dig[:n].view(torch.int64).sum()) % 2**64)

    splits = [int(k) for k in args.cu_split.split(",")]
    for chunk in [int(c) for c in args.chunks.split(",")]:
        mn, av, mx = 4096, chunk, 2 * chunk
        mode = _capi.OXH_MODE_WAVE_PACKED
        out = fastcdc_outputs(arena, lens, mn)
        times = []
        for r in range(args.reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            _, _, dig, first = fastcdc_device(arena, offs, lens, mn, av, mx, out=out, stream=torch.cuda.current_stream())
            torch.cuda.synchronize()
            if r:
                times.append(time.perf_counter() - t0)
        want = fp(dig, int(first[-1]))
        res[f"c{chunk}_serial_s"] = round(float(np.median(times)), 4)
        del out, dig
        prev_variant = _capi.lib().oxh_set_kernel_variant(args.k1_variant)
        for split, G in [(k, int(g)) for k in splits for g in args.groups.split(",")]:
            if split:
                sa = masked_stream([i for i in range(n_cu) if i % 8 < split])
                sb = masked_stream([i for i in range(n_cu) if i % 8 >= split])
            else:
                sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
            groups = np.array_split(np.arange(args.files), G)
            outs = [fastcdc_outputs(arena, lens[g], mn) for g in groups]
            times, ok = [], True
            for r in range(args.reps + 1):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                tabs = []
                for gi, g in enumerate(groups):
                    c_off, c_len, _, first = fastcdc_device(arena, offs[g], lens[g], mn, av, mx, digests=False,
                                                            out=outs[gi], stream=sa)  # synchronises sa
                    tabs.append((c_off, c_len, int(first[-1])))
                    # K1 of this group on stream B runs under the next group's scan on stream A
                    xxh3_128_batch_device(arena, c_off, c_len, out=outs[gi][2], mode=mode, stream=sb)
                torch.cuda.synchronize()
                if r:
                    times.append(time.perf_counter() - t0)
                n_all = sum(t[2] for t in tabs)
                s_all = sum(int(outs[gi][2][: tabs[gi][2]].view(torch.int64).sum()) for gi in range(G))
                ok = ok and (n_all, s_all % 2**64) == want
            tag = f"c{chunk}_overlap_g{G}" + (f"_cu{split}of8" if split else "")
            res[tag + "_s"] = round(float(np.median(times)), 4)
            res[tag + "_same"] = ok
            del outs
        _capi.lib().oxh_set_kernel_variant(prev_variant)
        print(json.dumps(res), flush=True)
    res["GB"] = round(total / 1e9, 1)
    res["k1_variant"] = args.k1_variant
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
