"""A/B of K1L whole-file digests with the chains on CUs of their own (OXH_CHAIN_CUS) against the
shared form, on C5's 16 x 8 GiB device-resident blobs (or --files / --gib). Calls alternate in one
process; every digest of every call must equal the first call's, and one file is checked against
the C oracle over bytes regenerated on the host.

    python tools/chain_split_ab.py [--files 16] [--gib 8] [--rounds 3] [--cus 0,32]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=16)
    ap.add_argument("--gib", type=float, default=8.0)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--cus", default="0,32")
    ap.add_argument("--check", action="store_true", help="check file 0 against the C oracle (slow on one core)")
    a = ap.parse_args()

    import numpy as np
    import torch

    from oxen_amd.device import fill_splitmix, large_digests_device, to_numpy_u64

    flen = int(a.gib * (1 << 30))
    bufs = []
    for f in range(a.files):
        b = torch.empty(flen, dtype=torch.uint8, device="cuda")
        fill_splitmix(b, 1000 + f)
        bufs.append(b)
    torch.cuda.synchronize()
    out = torch.empty((a.files, 2), dtype=torch.int64, device="cuda")
    forms = [int(x) for x in a.cus.split(",")]
    times = {c: [] for c in forms}
    ref = None
    for r in range(a.rounds + 1):
        for c in forms:
            os.environ["OXH_CHAIN_CUS"] = str(c)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            large_digests_device(bufs, out=out)
            e1.record()
            torch.cuda.synchronize()
            got = to_numpy_u64(out).reshape(-1, 2).copy()
            if ref is None:
                ref = got
            assert np.array_equal(got, ref), f"digests differ with OXH_CHAIN_CUS={c}"
            if r > 0:  # round 0 warms both forms
                times[c].append(e0.elapsed_time(e1) / 1e3)
            print(json.dumps({"round": r, "chain_cus": c, "s": round(e0.elapsed_time(e1) / 1e3, 4)}), flush=True)
    res = {"files": a.files, "bytes_per_file": flen,
           "median_s": {str(c): round(float(np.median(v)), 4) for c, v in times.items()},
           "all_s": {str(c): [round(x, 4) for x in v] for c, v in times.items()}}
    if a.check:
        from oracle import oracle
        from oxen_amd.workloads import splitmix_bytes

        want = oracle.xxh3_128(splitmix_bytes(1000, 0, flen).tobytes())
        res["file0_oracle_exact"] = (int(ref[0, 0]), int(ref[0, 1])) == want
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
