"""Soak the streaming engine: several threads issue mixed requests against shared contexts for a fixed
time, and every answer is checked against digests the C oracle computed up front. GPU box only.

    python tools/engine_soak.py [--seconds 240] [--threads 8] [--files 3000]

Corpus: files of 0 B .. 300 KB (binary and text), a few above a 1 MiB staging slot (large-file
path), duplicates, a missing path. Contexts: one with 1 MiB staging slots (every call cycles slots,
seals early and takes the large-file path), one default. Requests, picked at random per iteration:
  files      oxh_hash_files over a random subset (random order, duplicates)
  text       oxh_hash_files_text: digests + (num_lines, num_chars)
  add        oxh_add_files into a per-thread version store; every reported blob re-read and hashed
  buffers    oxh_hash_buffers over random host slices
  stream     the streaming Xxh3 over a file in random-sized updates
  meta       oxh_hash_files_meta with the true sizes
  streams    oxh_hash_streams over random byte strings (K2's path: arena spans and per-item copies)
  modified   oxh_files_modified: equal sizes, drifted mtimes, node hashes right or off by one
  utf8       oxh_hash_files_text_utf8 (digests, counts and the is_utf8 sniff)
  pool       the reader-process pool (oxh_pool, 2 helpers) over a random subset
  cdc        oxh_fastcdc_files (8 KiB FastCDC) on the same contexts, every table against the oracle
  fixed      oxh_chunk_digests_files (4 KiB / 64 KiB / 1 MiB chunks), against the oracle
--regrow: a thread keeps creating a context with 1 MiB staging slots, hashing 1, 2, then 4 of the
corpus's large files side by side (each step regrows the context's large-file piece buffers:
stream-ordered, no device-wide sync) and destroying it again -- while the other threads (and any
device-resident callers in other processes) run.
--mutate: a mutator thread atomically replaces files of a hot tenth of the corpus (sizes across the
1 MiB slot too) while the requests run; a digest must then be one of the file's versions (no torn
read: the engine's re-read on a size change, read to EOF) with that version's counts and is_utf8.
--split: about 0.5 % of the corpus 8-24 MiB (read in 4 MiB parts by several readers, engine.hip
run_part), a third context with 32 MiB slots (split files compete for slots), and the mutator's sizes
include 10 MiB.
Prints one JSON line: per-kind counts, items checked, failures (the first few described). Exit 1 on any
mismatch.
"""
from __future__ import annotations

import argparse
import json
import os
import random
import shutil
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=240)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--files", type=int, default=3000)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--mutate", action="store_true",
                    help="a thread keeps replacing 10 %% of the files (new content, temp + rename): every digest must be "
                         "one of that file's versions, with that version's text counts and is_utf8")
    ap.add_argument("--regrow", action="store_true",
                    help="a thread keeps creating contexts whose large-file piece buffers regrow (1, 2, 4 files side by side)")
    ap.add_argument("--split", action="store_true",
                    help="files of 8-24 MiB (split reads), a 32 MiB-slot context, 10 MiB mutations")
    a = ap.parse_args()

    import numpy as np

    from oracle import oracle
    from oxen_amd import _capi, hasher

    rng = random.Random(a.seed)
    base = tempfile.mkdtemp(prefix="oxh_soak_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        corpus = os.path.join(base, "corpus")
        os.makedirs(corpus)
        paths, want, text, hist = [], {}, {}, {}

        def counts_of(data):
            arr = np.frombuffer(data, dtype=np.uint8)
            return 1 + data.count(b"\n"), len(data) - int(((arr & 0xC0) == 0x80).sum())
        words = [b"alpha", b"beta", b"\xc3\xa9t\xc3\xa9", b"\n", b"line\n", b"\xe2\x9c\x93", b" "]
        for i in range(a.files):
            p = os.path.join(corpus, f"d{i % 37}", f"f{i}.{'txt' if i % 3 == 0 else 'bin'}")
            os.makedirs(os.path.dirname(p), exist_ok=True)
            r = rng.random()
            n = 0 if r < 0.02 else rng.randint(1, 240) if r < 0.2 else rng.randint(241, 300_000) if r < 0.99 \
                else rng.randint(1_200_000, 3_000_000)
            if a.split and rng.random() < 0.005:
                n = rng.randint(8 << 20, 24 << 20)
            if i % 3 == 0:
                data = b"".join(rng.choice(words) for _ in range(n // 4 + 1))[:n]
            else:
                data = rng.randbytes(n)
            with open(p, "wb") as f:
                f.write(data)
            paths.append(p)
            want[p] = oracle.xxh3_128_int(data)
            text[p] = counts_of(data)
            hist[p] = {want[p]: (text[p], oracle.is_utf8_prefix(data[:4096]))}
        missing = os.path.join(corpus, "does-not-exist")
        hot = set(paths[::10]) if a.mutate else set()
        stable = [p for p in paths if p not in hot]

        def version(p, d):  # (counts, is_utf8) of the version of p with digest d, or None
            with lock:
                return hist[p].get(d)

        ctxs = [_capi.Context(0, staging_bytes=1 << 20), _capi.Context(0)]
        if a.split:
            ctxs.append(_capi.Context(0, staging_bytes=32 << 20))
        lock = threading.Lock()
        counts = {k: 0 for k in ("files", "text", "add", "buffers", "stream", "meta", "streams", "modified", "utf8", "pool",
                                 "cdc", "fixed")}
        from oracle import fastcdc as F
        from oxen_amd import dedup
        from oxen_amd.procpool import ShardedFileHasher

        pool = ShardedFileHasher(procs=2, devices=(0,), threads=4)
        pool_lock = threading.Lock()  # oxh_pool serves one call at a time anyway

        def utf8_ok(p):
            with open(p, "rb") as f:
                return oracle.is_utf8_prefix(f.read(4096))
        checked = [0]
        fails = []
        deadline = time.time() + a.seconds

        def fail(msg):
            with lock:
                if len(fails) < 20:
                    fails.append(msg)

        def worker(t):
            try:
                work(t)
            except Exception as e:  # a raised OxenError is a failure too
                fail(f"thread {t}: {e!r}")

        def work(t):
            r = random.Random(a.seed * 1000 + t)
            store = os.path.join(base, f"store{t}")
            while time.time() < deadline and not fails:
                kind = r.choice(list(counts))
                ctx = r.choice(ctxs)
                sub = [r.choice(paths) for _ in range(r.choice((1, 7, 64, 64, 400)))]
                n_ok = 0
                if kind in ("files", "meta"):
                    with_missing = r.random() < 0.2
                    q = sub + ([missing] if with_missing else [])
                    if kind == "files":
                        dg, _, st = hasher.hash_files_128bit(q, ctx)
                    else:
                        sizes = [os.path.getsize(p) for p in sub] + ([0] if with_missing else [])
                        dg, _, st = hasher.hash_files_given_metadata_128bit(q, sizes, ctx)
                    for p, d, s in zip(q, dg, st):
                        if p == missing:
                            if s == 0:
                                fail(f"{kind}: missing path reported OK")
                        elif s != 0 or version(p, d) is None:
                            fail(f"{kind}: {p} status {s} digest {d} is no version of the file")
                        else:
                            n_ok += 1
                elif kind == "text":
                    dg, _, st, meta = hasher.hash_files_text_128bit(sub, ctx)
                    for p, d, s, m in zip(sub, dg, st, meta):
                        v = version(p, d) if s == 0 else None
                        if v is None or (m["text"]["num_lines"], m["text"]["num_chars"]) != v[0]:
                            fail(f"text: {p} status {s} digest {d} meta {m} version {v}")
                        else:
                            n_ok += 1
                elif kind == "add":
                    dg, _, st, stored = hasher.add_files(sub, store, ctx)
                    for p, d, s in zip(sub, dg, st):
                        if s != 0 or version(p, d) is None:
                            fail(f"add: {p} status {s} digest {d} is no version of the file")
                            continue
                        with open(hasher.version_path(store, d), "rb") as f:
                            blob = f.read()
                        if oracle.xxh3_128_int(blob) != d:
                            fail(f"add: blob of {p} does not hash to its name")
                        else:
                            n_ok += 1
                elif kind == "buffers":
                    bufs = []
                    for p in sub[:64]:
                        with open(p, "rb") as f:
                            data = f.read()
                        lo = r.randint(0, len(data))
                        bufs.append(data[lo:])
                    got = hasher.hash_buffers_128bit(bufs, ctx)
                    for b, d in zip(bufs, got):
                        if d != oracle.xxh3_128_int(b):
                            fail(f"buffers: slice of {len(b)} B")
                        else:
                            n_ok += 1
                elif kind == "streams":
                    ss = [r.randbytes(r.choice((0, 5, 32, 200, 3210, 70_000))) for _ in range(r.choice((1, 50, 500)))]
                    got = hasher.hash_streams_128bit(ss, ctx)
                    for b, d in zip(ss, got):
                        if d != oracle.xxh3_128_int(b):
                            fail(f"streams: {len(b)} B")
                        else:
                            n_ok += 1
                elif kind == "modified":
                    sub = [r.choice(stable) for _ in sub]
                    flip = [r.random() < 0.3 for _ in sub]
                    sizes = [os.path.getsize(p) for p in sub]
                    nodes = [(want[p] ^ 1) if f else want[p] for p, f in zip(sub, flip)]
                    mod, st, _ = hasher.files_modified(sub, sizes, sizes, [False] * len(sub), nodes, ctx)
                    for p, f, m, s_ in zip(sub, flip, mod, st):
                        if s_ != 0 or m != f:
                            fail(f"modified: {p} status {s_} modified {m} want {f}")
                        else:
                            n_ok += 1
                elif kind == "utf8":
                    dg, _, st, meta, u8 = hasher.hash_files_text_utf8_128bit(sub, ctx)
                    for p, d, s_, m, u in zip(sub, dg, st, meta, u8):
                        v = version(p, d) if s_ == 0 else None
                        if v is None or (m["text"]["num_lines"], m["text"]["num_chars"]) != v[0] or bool(u) != v[1]:
                            fail(f"utf8: {p} status {s_} digest {d} meta {m} utf8 {u}")
                        else:
                            n_ok += 1
                elif kind == "pool":
                    with pool_lock:
                        out, _, st = pool.hash_files(sub)
                    for p, o, s_ in zip(sub, out, st):
                        if s_ != 0 or version(p, int(o[1]) << 64 | int(o[0])) is None:
                            fail(f"pool: {p} status {s_}")
                        else:
                            n_ok += 1
                elif kind in ("cdc", "fixed"):  # the host chunk entries on the same contexts (stable files)
                    sub = [r.choice(stable) for _ in sub[:64]]
                    datas = []
                    for p in sub:
                        with open(p, "rb") as f:
                            datas.append(np.frombuffer(f.read(), dtype=np.uint8))
                    if kind == "cdc":
                        tab = dedup.fastcdc_files(sub, 4096, 8192, 16384, ctx=ctx)
                    else:
                        chunk = r.choice((4096, 65536, 1 << 20))
                        tab = dedup.chunk_digests_files(sub, chunk, ctx=ctx)
                    for i, (p, d) in enumerate(zip(sub, datas)):
                        if int(tab.status[i]) != 0:
                            fail(f"{kind}: {p} status {int(tab.status[i])}")
                            continue
                        if kind == "cdc":
                            off, ln, dig = tab.file(i)
                            w = F.chunks(d, 4096, 8192, 16384)
                            ok = np.array_equal(off, w[:, 0]) and np.array_equal(ln, w[:, 1]) and \
                                (len(w) == 0 or np.array_equal(dig, oracle.batch(d, w[:, 0], w[:, 1])))
                        else:
                            ok = np.array_equal(tab.file(i), oracle.chunk_digests(d, chunk))
                        if not ok:
                            fail(f"{kind}: {p} table differs from the oracle")
                        else:
                            n_ok += 1
                else:  # stream
                    p = r.choice(paths)
                    with open(p, "rb") as f:
                        data = f.read()
                    x = hasher.Xxh3(ctx)
                    try:
                        i = 0
                        while i < len(data):
                            k = r.choice((1, 63, 1000, 70_000, 1 << 20))
                            x.update(data[i:i + k])
                            i += k
                        if x.digest128() != oracle.xxh3_128_int(data):
                            fail(f"stream: {p}")
                        else:
                            n_ok += 1
                    finally:
                        x.close()
                with lock:
                    counts[kind] += 1
                    checked[0] += n_ok

        mutations = [0]
        regrows = [0]

        def regrower():
            r = random.Random(a.seed + 7)
            big = [p for p in stable if os.path.getsize(p) > (1 << 20)]
            while time.time() < deadline and not fails and big:
                c = _capi.Context(0, staging_bytes=1 << 20)
                try:
                    for k in (1, 2, 4):
                        q = [r.choice(big) for _ in range(k)]
                        dg, _, st = hasher.hash_files_128bit(q, c)
                        for p, d, s_ in zip(q, dg, st):
                            if s_ != 0 or d != want[p]:
                                fail(f"regrow: {p} status {s_} digest {d}")
                        with lock:
                            checked[0] += len(q)
                finally:
                    c.close()
                regrows[0] += 1

        def mutator():
            r = random.Random(a.seed + 99)
            hot_list = sorted(hot)
            while time.time() < deadline and not fails:
                p = r.choice(hot_list)
                n = r.choice((0, 100, 5000, 60_000, 300_000, 1_500_000) + ((10 << 20,) if a.split else ()))
                data = r.randbytes(n) if r.random() < 0.5 else b"".join(r.choice(words) for _ in range(n // 4 + 1))[:n]
                d = oracle.xxh3_128_int(data)
                with lock:
                    hist[p][d] = (counts_of(data), oracle.is_utf8_prefix(data[:4096]))
                tmp = p + ".mut"
                with open(tmp, "wb") as f:
                    f.write(data)
                os.replace(tmp, p)
                mutations[0] += 1

        ths = [threading.Thread(target=worker, args=(t,)) for t in range(a.threads)]
        if a.mutate:
            ths.append(threading.Thread(target=mutator))
        if a.regrow:
            ths.append(threading.Thread(target=regrower))
        t0 = time.time()
        for th in ths:
            th.start()
        while any(th.is_alive() for th in ths):  # a progress line every 20 s (long runs must not look hung)
            for th in ths:
                th.join(timeout=20.0 / len(ths))
            with lock:
                print(json.dumps({"t": round(time.time() - t0), "requests": dict(counts), "items_checked": checked[0],
                                  "failures": len(fails)}), file=sys.stderr, flush=True)
        for c in ctxs:
            c.close()
        pool.close()
        res = {"seconds": round(time.time() - t0, 1), "threads": a.threads, "files": a.files, "mutations": mutations[0],
               "regrow_contexts": regrows[0], "big_piece_mib": os.environ.get("OXH_BIG_PIECE_MIB", "1024 (default)"),
               "requests": counts, "items_checked": checked[0], "failures": len(fails), "first_failures": fails[:5]}
        print(json.dumps(res), flush=True)
        sys.exit(1 if fails else 0)
    finally:
        shutil.rmtree(base, ignore_errors=True)


if __name__ == "__main__":
    main()
