"""A/B of the fused durable add's publish modes (oxh_add_files, VersionPublisher) on the C3 tree, in
ONE process, calls alternating, each into a fresh version store:
  inline      OXH_PUBLISH_INLINE=1: syncfs / renames / syncfs inside the slot's drain (r02 form)
  async       the committer thread (default)
  async_fsync the committer thread with per-blob fsync / rename / parent fsync (OXH_PUBLISH_SYNC=fsync)
  inline_fsync the same steps inside the slot's drain
  cpu_ref     the reference add restated (oracle/: hash, re-read, verify, write, fsync blob + parent)
Medians printed as one JSON line; digests and stored counts checked equal across modes. Each call
starts after a sync and a pause: back-to-back 10 GB durable writes slow the GPU boxes' disks down
call after call (5.9 s for the first C3 add, 20-70 s for later ones in one r03 run), so use a
smaller tree (--images 20000) for A/Bs.

    python tools/add_ab.py [--images 200000] [--rounds 2] [--modes inline,async,async_fsync,cpu_ref]
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

ENV = {"inline": {"OXH_PUBLISH_INLINE": "1"}, "async": {},
       "async_fsync": {"OXH_PUBLISH_SYNC": "fsync"}, "inline_fsync": {"OXH_PUBLISH_INLINE": "1", "OXH_PUBLISH_SYNC": "fsync"}}
KNOBS = ("OXH_PUBLISH_INLINE", "OXH_PUBLISH_SYNC")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=200_000)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--modes", default="inline,async,async_fsync,cpu_ref")
    ap.add_argument("--settle", type=float, default=3.0, help="seconds to wait (after a sync) before each call")
    ap.add_argument("--dir", default=os.path.join(os.environ.get("TMPDIR", "/tmp"), "oxh_c3_add"))
    a = ap.parse_args()

    import numpy as np

    from oracle import oracle
    from oxen_amd import _capi, hasher
    from oxen_amd.workloads import write_image_repo_fast

    shutil.rmtree(a.dir, ignore_errors=True)
    paths = write_image_repo_fast(a.dir, a.images)
    nbytes = sum(os.path.getsize(p) for p in paths)
    threads = min(16, os.cpu_count() or 1)
    ctx = _capi.Context(0)
    oracle.build()
    modes = [m for m in a.modes.split(",") if m]
    ts = {m: [] for m in modes}
    ref = None
    ok = True
    for r in range(a.rounds):
        for m in modes[r % len(modes):] + modes[:r % len(modes)]:  # rotated: no mode always goes first
            root = os.path.join(a.dir, f".oxen_{m}_{r}", "versions", "files")
            os.sync()  # each call starts with the disk's queue drained (the previous store's removal too)
            time.sleep(a.settle)
            if m == "cpu_ref":
                t0 = time.perf_counter()
                rout, _, rst, rstored = oracle.add_files(paths, root, threads)
                dt = time.perf_counter() - t0
                digests = [(int(hi) << 64) | int(lo) for lo, hi in rout]
                stored = int(rstored.sum())
                good = bool((rst == 0).all())
            else:
                saved = {k: os.environ.get(k) for k in KNOBS}
                for k in saved:
                    os.environ.pop(k, None)
                os.environ.update(ENV[m])
                try:
                    t0 = time.perf_counter()
                    digests, _, st, gstored = hasher.add_files(paths, root, ctx)
                    dt = time.perf_counter() - t0
                finally:
                    for k, v in saved.items():
                        if v is None:
                            os.environ.pop(k, None)
                        else:
                            os.environ[k] = v
                stored = int(sum(gstored))
                good = bool((np.asarray(st) == 0).all())
            ts[m].append(round(dt, 3))
            key = (list(digests), stored)
            ref = key if ref is None else ref
            ok = ok and good and key == ref
            shutil.rmtree(os.path.dirname(os.path.dirname(root)), ignore_errors=True)
            print(f"round {r} {m}: {dt:.3f} s", file=sys.stderr, flush=True)
    res = {"files": len(paths), "bytes": nbytes, "rounds": a.rounds, "threads": threads, "consistent": ok,
           "stored": ref[1] if ref else 0}
    for m, v in ts.items():
        res[m + "_median_s"] = float(np.median(v))
        res[m + "_all"] = v
    print(json.dumps(res), flush=True)
    ctx.close()
    shutil.rmtree(a.dir, ignore_errors=True)


if __name__ == "__main__":
    main()
