"""Generate the committed golden vectors (run in the build container; needs python `xxhash`).

The generator is libxxhash 0.8.2 via python-xxhash 3.8.1 -- an implementation of the same frozen
XXH3-128 that liboxen gets from xxhash-rust 0.8.15 (Cargo.lock:10355-10358). Inputs are either
deterministic (splitmix64 stream, oxen_amd/workloads.py) or data files the reference's own tests
hold (/root/reference/data/test, copied under tests/golden/data_test/ when <= 64 KiB). Outputs:

  lengths.json     every length 0..2048 and XXH3 boundary sizes up to 1 MiB+1
  kat.json         the reference's own known-answer digest (schemas.rs:131) + sanity vectors
  data_test.json   XXH3-128 of every file under reference data/test (48 files)
  text_repo.json   config 1: the 1 000-file text repo of benchmark/generate_text_repo.py + README
  streams.json     K2 parent-node streams (vnode / dir / commit / combined / metadata JSON)

Usage: python tests/golden/make_golden.py [--reference /root/reference]
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import xxhash  # noqa: E402

from oxen_amd.workloads import splitmix_bytes, text_repo_files  # noqa: E402

LEN_SEED = 0x0DE5EED
BOUNDARY = [3, 4, 8, 9, 16, 17, 32, 33, 64, 65, 96, 97, 128, 129, 159, 160, 191, 192, 223, 224, 239,
            240, 241, 255, 256, 257, 511, 512, 1023, 1024, 1025, 2047, 2048, 2049, 3071, 3072, 3073,
            4095, 4096, 4097, 4159, 4160, 5119, 5120, 5121, 8191, 8192, 8193, 16383, 16384, 16385,
            49_292, 65_535, 65_536, 65_537, 131_071, 131_072, 262_143, 262_144, 262_145,
            1_048_575, 1_048_576, 1_048_577]


def digest(data: bytes) -> dict:
    v = xxhash.xxh3_128_intdigest(data)
    return {"hex": format(v, "x"), "lo": v & (2**64 - 1), "hi": v >> 64}


def length_start(L: int) -> int:
    return (L * 97) % 4093


def text_metadata(data: bytes) -> dict:
    """repositories/metadata/text.rs:11-20 + util/fs.rs:217-263: lines = 1 + count(b'\\n'),
    chars = bytes that are not UTF-8 continuation bytes (bytecount::num_chars)."""
    return {"text": {"num_lines": 1 + data.count(b"\n"), "num_chars": sum(1 for b in data if (b & 0xC0) != 0x80)}}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    args = ap.parse_args()
    meta = {"generator": f"python-xxhash {xxhash.VERSION} / libxxhash {xxhash.XXHASH_VERSION}",
            "algorithm": "XXH3-128, seed 0, default secret (== xxhash-rust 0.8.15 xxh3_128)"}

    # 1. lengths
    lengths = sorted(set(list(range(0, 2049)) + BOUNDARY))
    vecs = []
    for L in lengths:
        s = length_start(L)
        d = digest(splitmix_bytes(LEN_SEED, s, L).tobytes())
        vecs.append({"len": L, "start": s, **d})
    json.dump({**meta, "seed": LEN_SEED, "input": "splitmix_bytes(seed, start, len)", "vectors": vecs},
              open(os.path.join(HERE, "lengths.json"), "w"))

    # 2. known answers
    kat = [
        {"source": "crates/liboxen/src/repositories/data_frames/schemas.rs:131 (reference test)",
         "input": "filestrlabelstrmin_xf64min_yf64widthi64heighti64",
         "expected": "b821946753334c083124fd563377d795"},
    ]
    for s in ["", "hello", "File content 0"]:
        kat.append({"source": "SURVEY.md §8c sanity vector", "input": s, "expected": digest(s.encode())["hex"]})
    kat.append({"source": "SURVEY.md F3 (31-char unpadded hex)", "input_repeat": ["x", 65536],
                "expected": digest(b"x" * 65536)["hex"]})
    for k in kat:
        if "input" in k:
            assert digest(k["input"].encode())["hex"] == k["expected"], k
    json.dump({**meta, "vectors": kat}, open(os.path.join(HERE, "kat.json"), "w"), indent=1)

    # 3. data/test fixture files
    dt_src = os.path.join(args.reference, "data", "test")
    dt_dst = os.path.join(HERE, "data_test")
    files = []
    if os.path.isdir(dt_src):
        os.makedirs(dt_dst, exist_ok=True)
        for dp, _, fns in os.walk(dt_src):
            for fn in sorted(fns):
                p = os.path.join(dp, fn)
                if not os.path.isfile(p):
                    continue
                rel = os.path.relpath(p, dt_src)
                data = open(p, "rb").read()
                # data fixtures only: the text of a reference source file or script is never copied
                # (its digest stays; tests read the original from /root/reference when present)
                copied = len(data) <= 65536 and not fn.endswith((".py", ".sh", ".rs", ".js", ".ts"))
                if copied:
                    q = os.path.join(dt_dst, rel)
                    os.makedirs(os.path.dirname(q), exist_ok=True)
                    shutil.copyfile(p, q)
                files.append({"path": rel, "size": len(data), "copied": copied, **digest(data)})
        files.sort(key=lambda r: r["path"])
        json.dump({**meta, "source": "reference data/test (fixtures the reference's own tests hold)", "files": files},
                  open(os.path.join(HERE, "data_test.json"), "w"), indent=1)

    # 4. config 1 text repo (+ text metadata / combined hashes, hasher.rs:67-100)
    recs = []
    for rel, data in text_repo_files(1000, "text_files").items():
        md = text_metadata(data)
        mjson = json.dumps(md, separators=(",", ":"))
        mh = xxhash.xxh3_128_intdigest(mjson.encode())
        ch = xxhash.xxh3_128_intdigest(xxhash.xxh3_128_intdigest(data).to_bytes(16, "little") + mh.to_bytes(16, "little"))
        recs.append({"path": rel, "size": len(data), **digest(data), "metadata_json": mjson,
                     "metadata_hash": format(mh, "x"), "combined_hash": format(ch, "x")})
    json.dump({**meta, "source": "benchmark/generate_text_repo.py:5-33 (num_files=1000, output_dir=text_files)",
               "files": recs}, open(os.path.join(HERE, "text_repo.json"), "w"))

    # 5. K2 parent-node streams
    from oxen_amd import merkle

    child = [int(r["hex"], 16) for r in recs[:200]]
    combined = [int(r["combined_hash"], 16) for r in recs[:200]]
    streams = {
        "vnode_small": merkle.vnode_stream("texts", combined[:3]),
        "vnode_200": merkle.vnode_stream("texts", combined),
        "vnode_salted": merkle.vnode_stream("texts", combined[:5], bytes(range(16))),
        "vnode_root_empty": merkle.vnode_stream("", []),
        "dir_texts": merkle.dir_stream("texts", [(child[0], [(f"file_{i}.txt", combined[i]) for i in range(50)])]),
        "dir_root": merkle.dir_stream("", [(child[1], [("texts", child[2]), ("README.md", combined[3])])]),
        "commit": merkle.commit_stream(["abc", "def"], "add files", "ox", "ox@oxen.ai", 1_700_000_000),
        "combined_0": child[0].to_bytes(16, "little") + int(recs[0]["metadata_hash"], 16).to_bytes(16, "little"),
        "metadata_null": b"null",
        "metadata_text": recs[0]["metadata_json"].encode(),
    }
    out = [{"name": k, "bytes_hex": v.hex(), **digest(v)} for k, v in streams.items()]
    json.dump({**meta, "source": "commit_writer.rs:686-720, 757-766, 995-1147; hasher.rs:67-100",
               "streams": out}, open(os.path.join(HERE, "streams.json"), "w"), indent=1)
    print(f"wrote {len(vecs)} length vectors, {len(kat)} KATs, {len(files)} data/test files, "
          f"{len(recs)} text-repo files, {len(out)} streams")


if __name__ == "__main__":
    main()
