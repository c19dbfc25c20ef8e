"""Pin the CPU oracle (oracle/xxh3_oracle.c) before trusting it as the checker.

Anchors: the reference's own known-answer digest (schemas.rs:131), the reference's data/test
fixture files, and libxxhash-generated golden vectors (tests/golden/make_golden.py).
"""
import os

import numpy as np
import pytest

from oxen_amd.workloads import splitmix_bytes

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_reference_known_answer(oracle_lib, golden):
    for v in golden("kat.json")["vectors"]:
        data = v["input"].encode() if "input" in v else v["input_repeat"][0].encode() * v["input_repeat"][1]
        assert oracle_lib.format_hex(*oracle_lib.xxh3_128(data)) == v["expected"], v["source"]


def test_every_length_golden(oracle_lib, golden):
    g = golden("lengths.json")
    seed = g["seed"]
    vecs = g["vectors"]
    span = max(v["start"] + v["len"] for v in vecs)
    arena = splitmix_bytes(seed, 0, span)
    offs = np.array([v["start"] for v in vecs], dtype=np.uint64)
    lens = np.array([v["len"] for v in vecs], dtype=np.uint64)
    got = oracle_lib.batch(arena, offs, lens, threads=4)
    want = np.array([[v["lo"], v["hi"]] for v in vecs], dtype=np.uint64)
    bad = [vecs[i]["len"] for i in np.nonzero((got != want).any(axis=1))[0]]
    assert not bad, f"oracle mismatch at lengths {bad[:10]}"


def test_data_test_fixture_files(oracle_lib, golden):
    g = golden("data_test.json")
    paths, want = [], []
    for r in g["files"]:
        if r["copied"]:
            paths.append(os.path.join(GOLDEN, "data_test", r["path"]))
            want.append(r["hex"])
    out, sizes, status = oracle_lib.hash_files(paths, threads=4)
    assert (status == 0).all()
    got = [oracle_lib.format_hex(int(lo), int(hi)) for lo, hi in out]
    assert got == want


@pytest.mark.skipif(not os.path.isdir("/root/reference/data/test"), reason="reference tree not present")
def test_data_test_all_reference_files(oracle_lib, golden):
    g = golden("data_test.json")
    paths = [os.path.join("/root/reference/data/test", r["path"]) for r in g["files"]]
    out, sizes, status = oracle_lib.hash_files(paths, threads=4)
    assert (status == 0).all()
    assert [oracle_lib.format_hex(int(lo), int(hi)) for lo, hi in out] == [r["hex"] for r in g["files"]]
    assert [int(s) for s in sizes] == [r["size"] for r in g["files"]]


def test_text_repo_config1(oracle_lib, golden):
    from oxen_amd.workloads import text_repo_files

    files = text_repo_files(1000, "text_files")
    recs = golden("text_repo.json")["files"]
    assert len(recs) == 1001
    for r in recs:
        data = files[r["path"]]
        c = oracle_lib.xxh3_128_int(data)
        assert format(c, "x") == r["hex"]
        m = oracle_lib.xxh3_128_int(r["metadata_json"].encode())
        assert format(m, "x") == r["metadata_hash"]
        assert format(oracle_lib.combined_hash(c, m), "x") == r["combined_hash"]


def test_parent_streams(oracle_lib, golden):
    for s in golden("streams.json")["streams"]:
        assert format(oracle_lib.xxh3_128_int(bytes.fromhex(s["bytes_hex"])), "x") == s["hex"], s["name"]


def test_unpadded_hex_and_missing_file(oracle_lib, tmp_path):
    # 65 536 x 'x' hashes to a value with a leading zero nibble -> 31 chars
    h = oracle_lib.format_hex(*oracle_lib.xxh3_128(b"x" * 65536))
    assert len(h) == 31
    out, sizes, status = oracle_lib.hash_files([str(tmp_path / "nope.txt")])
    assert status[0] != 0


def test_clean_corrupted_versions_oracle(oracle_lib, tmp_path):
    """The fsck restatement (storage/local.rs:417-610) counts like the reference on a damaged store."""
    from _store import make_version_store

    root = str(tmp_path / "files")
    dry, real, again = make_version_store(root, lambda b: oracle_lib.format_hex(*oracle_lib.xxh3_128(b)))
    assert oracle_lib.clean_corrupted_versions(root, dry_run=True, threads=4) == dry
    assert oracle_lib.clean_corrupted_versions(root, dry_run=False, threads=4) == real
    assert oracle_lib.clean_corrupted_versions(root, dry_run=False, threads=4) == again


def test_large_file_branches_agree(oracle_lib, tmp_path):
    """Files >= 1e9 B (hasher.rs:150-174): the mmap one-shot form and the 4 KiB read-loop form the
    CPU baseline times (oxo_hash_files_stream4k) give the same digest (XXH3 streaming == one-shot).
    A sparse file with a few written regions keeps this cheap."""
    import ctypes

    from oracle import oracle

    p = tmp_path / "big.bin"
    size = 1_000_000_007
    with open(p, "wb") as fh:
        fh.truncate(size)
        for off in (0, 123_456_789, size - 5000):
            fh.seek(off)
            fh.write(splitmix_bytes(off, 0, 4096).tobytes())
    arr = (ctypes.c_char_p * 1)(os.fsencode(str(p)))
    outs = []
    for fn in (oracle.lib().oxo_hash_files, oracle.lib().oxo_hash_files_stream4k):
        out = np.zeros((1, 2), dtype=np.uint64)
        sz = np.zeros(1, dtype=np.uint64)
        st = np.zeros(1, dtype=np.int32)
        fn(arr, 1, out.ctypes.data_as(oracle._u64p), sz.ctypes.data_as(oracle._u64p), st.ctypes.data_as(oracle._i32p), 1)
        assert int(st[0]) == 0 and int(sz[0]) == size
        outs.append((int(out[0, 0]), int(out[0, 1])))
    assert outs[0] == outs[1]
