"""Config 1 (BASELINE configs[0]): `oxen add .` on the 1 000-file text repo of
benchmark/generate_text_repo.py (texts/file_{i}.txt = f"File content {i}" + README.md).

    python tools/bench_c1.py [--threads 16] [--reps 5]

The reference times this on its CPU path; no `oxen` binary exists in this image, so the CPU number is
the add loop restated in C (oracle/: stat, read, one-shot XXH3-128, then store_version_from_reader's
re-read + verify hash + write + rename per new file), next to:
  gpu_add_fused   oxh_add_files (read once into pinned staging, K1s, publish from the same bytes)
  gpu_text_nodes  the hashing half of add.rs:833-842 for text files: content hash + (num_lines,
                  num_chars) in one K1T pass, then metadata and combined hashes in batched passes
Every digest is checked against the oracle. At ~16 KB of payload this config is syscall- and
launch-latency-bound, not bandwidth-bound; it is reported, not optimised for.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default=os.path.join(os.environ.get("TMPDIR", "/tmp"), "oxh_c1"))
    ap.add_argument("--threads", type=int, default=min(16, os.cpu_count() or 1))
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()

    import numpy as np

    from oracle import oracle
    from oxen_amd import _capi, hasher
    from oxen_amd.workloads import write_text_repo

    shutil.rmtree(a.dir, ignore_errors=True)
    paths = write_text_repo(a.dir, 1000)
    nbytes = sum(os.path.getsize(p) for p in paths)
    oracle.build()
    ctx = _capi.Context(0)
    res = {"config": "C1: generate_text_repo.py, 1 000 text files + README.md", "files": len(paths), "bytes": nbytes,
           "threads": a.threads}

    def timed(fn):
        best, out = None, None
        for r in range(a.reps):
            for d in (".oxen_gpu", ".oxen_ref"):
                shutil.rmtree(os.path.join(a.dir, d), ignore_errors=True)
            t0 = time.perf_counter()
            out = fn()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        return best, out

    vroot = os.path.join(a.dir, ".oxen_gpu", "versions", "files")
    rroot = os.path.join(a.dir, ".oxen_ref", "versions", "files")
    hasher.add_files(paths, vroot, ctx)  # warm-up (first launch, page cache)
    res["cpu_ref_add_s"], (rout, _, rst, rstored) = timed(lambda: oracle.add_files(paths, rroot, a.threads))
    res["gpu_add_fused_s"], (gd, _, gst, gstored) = timed(lambda: hasher.add_files(paths, vroot, ctx))
    res["gpu_text_nodes_s"], nodes = timed(lambda: hasher.text_file_nodes(paths, ctx))
    want = [(int(hi) << 64) | int(lo) for lo, hi in rout]
    res["digests_bit_exact"] = want == gd == [n["hash"] for n in nodes]
    res["blobs_written"] = [int(sum(gstored)), int(rstored.sum())]
    res["example_node"] = {k: (format(v, "x") if isinstance(v, int) and k != "num_bytes" else v)
                           for k, v in nodes[0].items()}
    for k in ("cpu_ref_add_s", "gpu_add_fused_s", "gpu_text_nodes_s"):
        res[k] = round(res[k] * 1e3, 2)
    res["unit"] = "ms (best of %d)" % a.reps
    res = {k.replace("_s", "_ms") if k.endswith("_s") else k: v for k, v in res.items()}
    print(json.dumps(res), flush=True)
    ctx.close()
    shutil.rmtree(a.dir, ignore_errors=True)
    if not res["digests_bit_exact"]:
        sys.exit(1)


if __name__ == "__main__":
    main()
