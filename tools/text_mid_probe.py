"""Mid-size text files through K1T (oxh_hash_files_text: digests + MetadataText counts in the same read):
N files of S MiB of UTF-8 text from the page cache, median of --reps calls, every digest against the C
oracle and every count against numpy. Run it with OXH_SLOT_CHAINS=0 / 1 to compare one K1T wave per item
with K1L + text_count_kernel for items of 1 MiB and more (staging.hip submit_slot). Prints one JSON line.

    python tools/text_mid_probe.py [--files 16] [--mib 100] [--reps 3]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=16)
    ap.add_argument("--mib", type=int, default=100)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--dir", default=os.path.join(os.environ.get("TMPDIR", "/tmp"), "oxh_text_mid"))
    a = ap.parse_args()
    from oracle import oracle
    from oxen_amd import _capi, hasher

    os.makedirs(a.dir, exist_ok=True)
    line = "row,é,中,\U0001f600 some text\n".encode()
    size = a.mib << 20
    paths, want, counts = [], [], []
    for f in range(a.files):
        p = os.path.join(a.dir, f"t{f}.txt")
        data = (line * (size // len(line) + 1))[: size - f]
        if not (os.path.exists(p) and os.path.getsize(p) == len(data)):
            with open(p, "wb") as fh:
                fh.write(data)
        arr = np.frombuffer(data, dtype=np.uint8)
        paths.append(p)
        want.append(oracle.xxh3_128_int(data))
        counts.append({"text": {"num_lines": 1 + data.count(b"\n"), "num_chars": len(data) - int(((arr & 0xC0) == 0x80).sum())}})
    ctx = _capi.Context(0)
    ts, ok = [], True
    for _ in range(a.reps + 1):
        t0 = time.perf_counter()
        d, _, st, meta = hasher.hash_files_text_128bit(paths, ctx=ctx)
        ts.append(time.perf_counter() - t0)
        ok &= d == want and meta == counts and not any(st)
    ctx.close()
    g = statistics.median(ts[1:])
    print(json.dumps({"files": a.files, "bytes_each": size, "slot_chains": os.environ.get("OXH_SLOT_CHAINS", "1"),
                      "gpu_s": round(g, 4), "gpu_GiBs": round(a.files * size / g / 2**30, 1), "bit_exact": bool(ok)}), flush=True)
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
