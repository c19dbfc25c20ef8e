"""Soak the device-resident entry points from several threads at once, each on its own HIP stream;
every answer is checked against the C oracle over the same bytes copied to the host. GPU box only.

    python tools/device_soak.py [--seconds 240] [--threads 6]

Per iteration a thread picks one of:
  batch      oxh_xxh3_128_batch_device over ragged items at random offsets (every OXH_MODE_*)
  text       oxh_xxh3_128_text_batch_device: digests + (num_lines, num_chars)
  chunks     oxh_chunk_digests_device, fixed-size chunks of a random size
  large      oxh_xxh3_128_large_batch_device over 1-3 buffers of 2-40 MiB (block sums + chains, the
             scratch lease and its aux stream shared per device by two callers at a time)
  fastcdc    oxh_fastcdc_device over 1-3 files (1-24 MB, avg 4-64 KiB): chunk table and digests
  stream     the streaming Xxh3 over host bytes in random pieces (its device pieces use the lease too)
Prints a progress line every 20 s on stderr and one JSON line at the end; exit 1 on any mismatch.
"""
from __future__ import annotations

import argparse
import json
import os
import random
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=240)
    ap.add_argument("--threads", type=int, default=6)
    ap.add_argument("--seed", type=int, default=11)
    a = ap.parse_args()

    import numpy as np
    import torch

    from oracle import fastcdc as F
    from oracle import oracle
    from oxen_amd import hasher
    from oxen_amd.device import (chunk_digests_device, fastcdc_device, fill_splitmix, large_digests_device,
                                 to_numpy_u64, xxh3_128_batch_device, xxh3_128_text_batch_device)

    oracle.build()
    dev = torch.device("cuda:0")
    pool_bytes = 96 << 20
    base = torch.empty(pool_bytes, dtype=torch.uint8, device=dev)
    fill_splitmix(base, a.seed)
    # a text-like region: bytes from a small alphabet with newlines and UTF-8 sequences
    words = np.frombuffer(b"ab\nc \xc3\xa9\xe2\x9c\x93xyz\n", dtype=np.uint8)
    text_host = words[np.random.default_rng(a.seed).integers(0, len(words), 8 << 20)]
    base[: 8 << 20].copy_(torch.from_numpy(text_host))
    torch.cuda.synchronize()
    host = base.cpu().numpy()  # the same bytes on the host, for the oracle

    lock = threading.Lock()
    kinds = ("batch", "text", "chunks", "large", "fastcdc", "stream")
    counts = {k: 0 for k in kinds}
    checked = [0]
    fails = []
    deadline = time.time() + a.seconds

    def fail(msg):
        with lock:
            if len(fails) < 20:
                fails.append(msg)

    def digest_list(t):
        return [(int(lo), int(hi)) for lo, hi in to_numpy_u64(t).reshape(-1, 2)]

    def oracle_batch(offs, lens):
        return [(int(lo), int(hi)) for lo, hi in oracle.batch(host, np.asarray(offs, dtype=np.uint64),
                                                                np.asarray(lens, dtype=np.uint64), 4)]

    def work(t):
        r = random.Random(a.seed * 100 + t)
        st = torch.cuda.Stream(device=dev)
        with torch.cuda.stream(st):
            while time.time() < deadline and not fails:
                kind = r.choice(kinds)
                ok = 0
                if kind in ("batch", "text"):
                    n = r.choice((1, 10, 300, 3000))
                    lens = [r.choice((0, 17, 240, 241, 1024, 1025, 8192 + r.randint(0, 99), r.randint(0, 300_000)))
                            for _ in range(n)]
                    region = (8 << 20) if kind == "text" else pool_bytes
                    offs = [r.randint(0, region - max(1, ln)) for ln in lens]
                    o = torch.tensor(offs, dtype=torch.int64, device=dev)
                    ln = torch.tensor(lens, dtype=torch.int64, device=dev)
                    if kind == "batch":
                        got = digest_list(xxh3_128_batch_device(base, o, ln, mode=r.choice((0, 1, 2, 3, 4)), stream=st))
                    else:
                        out, cnt = xxh3_128_text_batch_device(base, o, ln, stream=st)
                        got = digest_list(out)
                        cnts = to_numpy_u64(cnt).reshape(-1, 2)
                        for k, (off, L) in enumerate(zip(offs, lens)):
                            b = host[off:off + L]
                            want_c = (1 + int((b == 10).sum()), L - int(((b & 0xC0) == 0x80).sum()))
                            if (int(cnts[k][0]), int(cnts[k][1])) != want_c:
                                fail(f"text counts: item {k} len {L}")
                    want = oracle_batch(offs, lens)
                    for k, (g, w) in enumerate(zip(got, want)):
                        if g != w:
                            fail(f"{kind}: item {k} len {lens[k]} off {offs[k]}")
                        else:
                            ok += 1
                elif kind == "chunks":
                    chunk = r.choice((1024, 4096, 8192, 65536, 1 << 20))
                    nbytes = r.randint(1, 24 << 20)
                    off = r.randint(0, pool_bytes - nbytes)
                    got = digest_list(chunk_digests_device(base[off:], chunk, nbytes=nbytes, stream=st))
                    starts = list(range(0, nbytes, chunk))
                    want = oracle_batch([off + s_ for s_ in starts], [min(chunk, nbytes - s_) for s_ in starts])
                    if got != want:
                        fail(f"chunks: {chunk} B chunks of {nbytes} B")
                    else:
                        ok += len(want)
                elif kind == "large":
                    m = r.randint(1, 3)
                    spans = []
                    for _ in range(m):
                        L = r.randint(2 << 20, 40 << 20)
                        o0 = r.randint(0, pool_bytes - L)
                        spans.append((o0, L))
                    got = digest_list(large_digests_device([base[o0:o0 + L] for o0, L in spans], stream=st))
                    want = oracle_batch([o0 for o0, _ in spans], [L for _, L in spans])
                    if got != want:
                        fail(f"large: {spans}")
                    else:
                        ok += m
                elif kind == "fastcdc":
                    avg = r.choice((4096, 8192, 16384, 65536))
                    mn, mx = 4096 if avg >= 8192 else 1024, 2 * avg
                    m = r.randint(1, 3)
                    lens = [r.randint(1 << 20, 24 << 20) for _ in range(m)]
                    offs = [r.randint(0, pool_bytes - L) for L in lens]
                    c_off, c_len, dig, first = fastcdc_device(base, offs, lens, mn, avg, mx, stream=st)
                    go, gl, gd = to_numpy_u64(c_off), to_numpy_u64(c_len), digest_list(dig)
                    for f_ in range(m):
                        lo, hi = int(first[f_]), int(first[f_ + 1])
                        want_t = F.chunks(host[offs[f_]:offs[f_] + lens[f_]], mn, avg, mx)
                        got_t = np.stack([go[lo:hi] - np.uint64(offs[f_]), gl[lo:hi]], axis=1)
                        if len(want_t) != hi - lo or not np.array_equal(got_t, want_t):
                            fail(f"fastcdc: file {f_} ({lens[f_]} B, avg {avg}) chunk table")
                            continue
                        want_d = oracle_batch(list(go[lo:hi]), list(gl[lo:hi]))
                        if gd[lo:hi] != want_d:
                            fail(f"fastcdc: file {f_} digests")
                        else:
                            ok += hi - lo
                else:  # stream
                    L = r.randint(0, 40 << 20)
                    o0 = r.randint(0, pool_bytes - L)
                    data = host[o0:o0 + L]
                    x = hasher.Xxh3()
                    try:
                        i = 0
                        while i < L:
                            k = r.choice((1, 4096, 1 << 20, 17 << 20))
                            x.update(data[i:i + k])
                            i += k
                        if x.digest128() != oracle.xxh3_128_int(data.tobytes()):
                            fail(f"stream: {L} B")
                        else:
                            ok += 1
                    finally:
                        x.close()
                with lock:
                    counts[kind] += 1
                    checked[0] += ok

    def worker(t):
        try:
            work(t)
        except Exception as e:
            fail(f"thread {t}: {e!r}")

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(a.threads)]
    t0 = time.time()
    for th in ths:
        th.start()
    while any(th.is_alive() for th in ths):
        for th in ths:
            th.join(timeout=20.0 / len(ths))
        with lock:
            print(json.dumps({"t": round(time.time() - t0), "requests": dict(counts), "items_checked": checked[0],
                              "failures": len(fails)}), file=sys.stderr, flush=True)
    res = {"seconds": round(time.time() - t0, 1), "threads": a.threads, "requests": counts,
           "items_checked": checked[0], "failures": len(fails), "first_failures": fails[:5]}
    print(json.dumps(res), flush=True)
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
