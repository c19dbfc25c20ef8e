"""Reproduce the intermittent stall seen in test_commit_driver: repeat its three hash passes in one
process under the slot watchdog (OXH_WAIT_LIMIT_S) and report the first failure."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

import _commit  # noqa: E402
from oxen_amd import hasher, merkle  # noqa: E402

ctx = hasher.default_context()
cases = [(s, v) for s in (False, True) for v in (10_000, 7)]
data = {c: _commit.staged_commit(n_files=500, n_dirs=9, second=c[0]) for c in cases}
t0 = time.time()
ref = None
for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 300):
    for c in cases:
        e, x = data[c]
        vn, dh = merkle.commit_tree(_commit.to_staged(e), _commit.to_staged(x), c[1], _commit.salt, ctx=ctx)
    if it % 50 == 0:
        print(f"iter {it} ok {time.time() - t0:.1f}s", flush=True)
print("done", flush=True)
