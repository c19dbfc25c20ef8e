"""C3 (200 002 files on disk -> digests, warm page cache) under alternating runtime settings on one box,
each setting in a fresh process (the knobs are read once per process): one dataset, generated once.

    python tools/c3_ab.py --reps 3 --env "OXH_TIMER_SLACK_NS=0 OXH_SPIN_US=0" --env ""

Prints one JSON line: per setting the median of its processes' medians (5 calls each).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CHILD = r"""
import ctypes, json, os, sys, time
import numpy as np
sys.path.insert(0, %r)
from oxen_amd import _capi
paths = open(%r).read().split("\n")
n = len(paths)
c_paths = (ctypes.c_char_p * n)(*[os.fsencode(p) for p in paths])
ctx = _capi.Context(0)
L = _capi.lib()
ts = []
for _ in range(6):
    out = np.zeros((n, 2), dtype=np.uint64); sizes = np.zeros(n, dtype=np.uint64); st = np.zeros(n, dtype=np.int32)
    t0 = time.perf_counter()
    _capi.check(L.oxh_hash_files(ctx.handle, c_paths, n, out.ctypes.data_as(_capi._u64p), sizes.ctypes.data_as(_capi._u64p),
                                 st.ctypes.data_as(_capi._i32p)), "oxh_hash_files")
    ts.append(time.perf_counter() - t0)
    assert (st == 0).all()
print(json.dumps({"s": sorted(ts[1:])[len(ts[1:]) // 2], "all": [round(t, 4) for t in ts], "fp": int(out[:, 0].sum() & 0xffffffff)}))
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default=os.path.join(os.environ.get("TMPDIR", "/tmp"), "oxh_c3ab"))
    ap.add_argument("--images", type=int, default=200_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--env", action="append", default=[])
    a = ap.parse_args()
    from oxen_amd.workloads import write_image_repo_fast

    lst = os.path.join(a.dir, "paths.txt")
    if not os.path.exists(lst):
        paths = write_image_repo_fast(a.dir, a.images)
        with open(lst, "w") as f:
            f.write("\n".join(paths))
    os.sync()
    time.sleep(2)
    res = {v: [] for v in a.env}
    fps = set()
    for _ in range(a.reps):
        for v in a.env:
            env = dict(os.environ)
            for kv in v.split():
                k, _, x = kv.partition("=")
                env[k] = x
            r = subprocess.run([sys.executable, "-c", CHILD % (ROOT, lst)], env=env, capture_output=True, text=True,
                               timeout=300)
            if r.returncode != 0:
                print(r.stderr[-2000:], file=sys.stderr)
                sys.exit(1)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            res[v].append(d["s"])
            fps.add(d["fp"])
    out = {"config": "C3 warm, oxh_hash_files over %d files, one process per run" % (a.images + 2),
           "settings": {v or "(default)": {"median_s": round(statistics.median(x), 4), "runs": [round(t, 4) for t in x]}
                        for v, x in res.items()},
           "digests_agree": len(fps) == 1}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
