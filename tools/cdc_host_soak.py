"""Soak of the host chunking entries against the C oracle: FastCDC (oxh_fastcdc_files / _host) and
fixed-size chunks (oxh_chunk_digests_files / _host) over random file sets (empty, tiny, around min /
avg / max, a few MiB to 200 MiB, constant runs), random chunk parameters and piece sizes
(OXH_CDC_PIECE_MIB changes the context's pipeline between iterations), the four entries in turn, a third
of the iterations on a fresh context, a third on one long-lived context, a third over two contexts
(the _multi entries); every boundary and digest checked. Prints one JSON object.

    python tools/cdc_host_soak.py --seconds 120 [--dir /tmp/oxh_soak]
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

FIXED = [64, 1000, 4096, 5000, 65536, 1 << 20, (3 << 20) + 7]
PARAMS = [(4096, 8192, 16384), (4096, 65536, 131072), (4096, 4096, 8192), (64, 256, 1024), (300, 257, 1500),
          (8192, 16384, 65536)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=120)
    ap.add_argument("--dir", default="/tmp/oxh_soak")
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()

    from oracle import fastcdc as F
    from oracle import oracle
    from oxen_amd import _capi, dedup

    oracle.build()
    rng = np.random.default_rng(a.seed)
    os.makedirs(a.dir, exist_ok=True)
    t_end = time.time() + a.seconds
    it = files_checked = chunks_checked = bytes_checked = 0
    failures = []
    last = time.time()
    shared = _capi.Context(0)
    shared2 = _capi.Context(0)  # with `shared`: the _multi entries over two contexts
    while time.time() < t_end:
        entry = ("files", "host", "fixed_files", "fixed_host")[it % 4]
        fixed = int(rng.choice(FIXED))
        mn, av, mx = PARAMS[int(rng.integers(len(PARAMS)))]
        piece = int(rng.choice([32, 48, 64, 256, 1024]))
        if piece * (1 << 20) < 2 * max(16 << 20, 4 * mx + 256):
            piece = 64
        os.environ["OXH_CDC_PIECE_MIB"] = str(piece)
        n = int(rng.integers(1, 12))
        datas = []
        for _ in range(n):
            kind = int(rng.integers(6))
            if kind == 0:
                size = int(rng.integers(0, 3))
            elif kind == 1:
                size = int(rng.integers(max(0, mn - 2), mn + 3))
            elif kind == 2:
                size = int(rng.integers(1, 4 * mx))
            elif kind == 3:
                size = int(rng.integers(1 << 20, 8 << 20))
            else:
                size = int(rng.integers(8 << 20, 200 << 20))
            d = rng.integers(0, 256, size, dtype=np.uint8)
            if size and rng.random() < 0.2:  # a constant run somewhere
                lo = int(rng.integers(0, size))
                d[lo:lo + int(rng.integers(1, 3 * mx))] = int(rng.integers(256))
            datas.append(d)
        own = (it // 4) % 3 == 0
        multi = (it // 4) % 3 == 2  # one context per share (oxh_*_multi), both long-lived
        ctx = _capi.Context(0) if own else shared
        kw = {"ctxs": [shared, shared2]} if multi else {"ctx": ctx}
        try:
            if entry in ("files", "fixed_files"):
                paths = []
                for i, d in enumerate(datas):
                    p = os.path.join(a.dir, f"f{i}")
                    d.tofile(p)
                    paths.append(p)
                if entry == "files":
                    tab = dedup.fastcdc_files(paths, mn, av, mx, **kw)
                else:
                    tab = dedup.chunk_digests_files(paths, fixed, **kw)
                if not (tab.status == 0).all():
                    failures.append({"it": it, "what": "status", "status": tab.status.tolist()})
            elif entry == "host":
                tab = dedup.fastcdc_host(datas, mn, av, mx, **kw)
            else:
                tab = dedup.chunk_digests_host(datas, fixed, **kw)
        finally:
            if own:
                ctx.close()
        for i, d in enumerate(datas):
            if entry.startswith("fixed"):
                dig = tab.file(i)
                off = np.arange(0, d.size, fixed, dtype=np.uint64)
                ln = np.minimum(np.uint64(fixed), np.uint64(d.size) - off)
                want = np.stack([off, ln], axis=1) if d.size else np.zeros((0, 2), dtype=np.uint64)
            else:
                off, ln, dig = tab.file(i)
                want = F.chunks(d, mn, av, mx)
            ok = len(off) == len(want) and np.array_equal(off, want[:, 0]) and np.array_equal(ln, want[:, 1])
            if ok and len(want):
                ok = np.array_equal(dig, oracle.batch(d, want[:, 0], want[:, 1], threads=8))
            if not ok:
                failures.append({"it": it, "file": i, "size": int(d.size), "piece_mib": piece, "entry": entry, "multi": multi,
                                 "params": [fixed] if entry.startswith("fixed") else [mn, av, mx]})
            files_checked += 1
            chunks_checked += len(want)
            bytes_checked += int(d.size)
        it += 1
        if time.time() - last >= 20:  # progress (a silent GPU command is taken for a hung one)
            print(f"[soak] {it} iterations, {files_checked} files, {chunks_checked} chunks, {len(failures)} failures",
                  file=sys.stderr, flush=True)
            last = time.time()
    shared.close()
    shared2.close()
    shutil.rmtree(a.dir, ignore_errors=True)
    print(json.dumps({"iterations": it, "files_checked": files_checked, "chunks_checked": chunks_checked,
                      "bytes_checked": bytes_checked, "failures": failures[:20], "n_failures": len(failures)}),
          flush=True)
    sys.exit(1 if failures else 0)


if __name__ == "__main__":
    main()
