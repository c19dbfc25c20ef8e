"""Host-side logic that needs no GPU: synthetic generators, layouts, merkle streams and formatting."""
import io
import os

import numpy as np
import pytest

from oxen_amd import merkle, workloads


def _splitmix_py(seed, i):
    m = (1 << 64) - 1
    z = (seed + (i + 1) * 0x9E3779B97F4A7C15) & m
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
    return z ^ (z >> 31)


def test_splitmix_bytes_matches_scalar_definition():
    words = [_splitmix_py(7, i) for i in range(10)]
    ref = b"".join(w.to_bytes(8, "little") for w in words)
    assert workloads.splitmix_bytes(7, 0, 80).tobytes() == ref
    assert workloads.splitmix_bytes(7, 3, 50).tobytes() == ref[3:53]
    assert workloads.splitmix_bytes(7, 0, 0).size == 0


def test_packed_layout_alignment():
    offs, total = workloads.packed_layout([1, 300, 0, 256, 5], align=256)
    assert list(offs) == [0, 256, 768, 768, 1024]
    assert total == 1029
    assert all(int(o) % 256 == 0 for o in offs)


def test_text_repo_matches_generator():
    files = workloads.text_repo_files(1000)
    assert files[os.path.join("texts", "file_0.txt")] == b"File content 0"
    assert files[os.path.join("texts", "file_999.txt")] == b"File content 999"
    assert files["README.md"].startswith(b"# Sample Repo\n\nGenerated 1000 text files")
    assert len(files) == 1001


def test_image_repo_tiffs_are_valid(tmp_path):
    from PIL import Image

    b = workloads.image_bytes_fast(3)
    assert len(b) == 49_292  # 128x128x3 TIFF written by PIL
    im = Image.open(io.BytesIO(b))
    assert im.size == (128, 128) and im.mode == "RGB"
    assert np.array_equal(np.asarray(im).reshape(-1), workloads.splitmix_bytes(0, 3 * 49152, 49152))
    paths = workloads.write_image_repo_fast(str(tmp_path), 25, num_dirs=10)
    assert len(paths) == 27
    assert os.path.exists(tmp_path / "images" / "split_4" / "noise_image_14.tiff")
    assert open(paths[14], "rb").read() == workloads.image_bytes_fast(14)


def test_merkle_hash_formatting():
    h = merkle.MerkleHash.from_str("2da4b9c5a75caad3688558138047f8a")
    assert str(h) == "2da4b9c5a75caad3688558138047f8a"  # unpadded (31 chars)
    assert h.node_db_prefix() == "2da/4b9c5a75caad3688558138047f8a"
    assert h.version_dir() == "2d/a4b9c5a75caad3688558138047f8a"
    assert h.to_le_bytes() == h.value.to_bytes(16, "little")
    assert merkle.MerkleHash(0).__str__() == "0"
    rng = np.random.default_rng(1)
    for _ in range(200):  # merkle_hash.rs:155-190 round trip
        v = int.from_bytes(rng.bytes(16), "little")
        assert merkle.MerkleHash.from_str(str(merkle.MerkleHash(v))).value == v


def test_num_vnodes_f32_semantics():
    assert merkle.num_vnodes(0, 10_000) == 0
    assert merkle.num_vnodes(1, 10_000) == 1
    assert merkle.num_vnodes(10_000, 10_000) == 1
    assert merkle.num_vnodes(10_001, 10_000) == 2
    assert merkle.num_vnodes(1000, 6) == 167


def test_parent_streams_bytes(golden):
    streams = {s["name"]: bytes.fromhex(s["bytes_hex"]) for s in golden("streams.json")["streams"]}
    assert merkle.vnode_stream("", []) == b"vnode"
    v = merkle.vnode_stream("texts", [1, 2])
    assert v == b"vnodetexts" + (1).to_bytes(16, "little") + (2).to_bytes(16, "little")
    assert streams["vnode_root_empty"] == b"vnode"
    d = merkle.dir_stream("a", [(5, [("x", 7)])])
    assert d == b"dira" + (5).to_bytes(16, "little") + b"x" + (7).to_bytes(16, "little")
    c = merkle.commit_stream(["abc", "def"], "m", "a", "e", 1)
    assert c == b'commit["abc", "def"]mae' + (1).to_bytes(8, "little")
    assert streams["commit"] == merkle.commit_stream(["abc", "def"], "add files", "ox", "ox@oxen.ai", 1_700_000_000)


def test_metadata_json_matches_serde(golden):
    from oxen_amd.hasher import metadata_json

    r0 = golden("text_repo.json")["files"][0]
    assert metadata_json({"text": {"num_lines": 1, "num_chars": 14}}) == r0["metadata_json"]
    assert metadata_json(None) == "null"
    from oxen_amd.hasher import text_metadata_json

    for lines, chars in ((1, 14), (0, 0), (123456, 7890123)):
        md = {"text": {"num_lines": lines, "num_chars": chars}}
        assert text_metadata_json(md) == metadata_json(md)


# serde_json's f64 text (ryu's format64), hand-derived -- parity unpinned: no reference fixture holds
# float-bearing metadata. d = shortest digits, value = d x 10^k, kk = len(d) + k:
#   12.5    d=125 k=-1 kk=2   -> point after 2 digits          "12.5"
#   12.0    d=12  k=0  kk=2   -> digits + k zeros + ".0"        "12.0"
#   1e-5    d=1   k=-5 kk=-4  -> -5 < kk <= 0: "0." 4 zeros d   "0.00001"
#   1e-6    d=1   k=-6 kk=-5  -> one digit: "1e" (kk-1)         "1e-6"
#   1e16    d=1   k=16 kk=17  -> kk > 16, one digit             "1e16"
#   1e15    d=1   k=15 kk=16  -> digits + 15 zeros + ".0"       "1000000000000000.0"
#   1.5e16  d=15  k=15 kk=17  -> d0 "." rest "e" (kk-1)         "1.5e16"
#   NaN, inf                  -> serde_json's serialize_f64     "null"
SERDE_F64 = [(12.5, "12.5"), (12.0, "12.0"), (1e-5, "0.00001"), (1e-6, "1e-6"), (1e16, "1e16"),
             (1e15, "1000000000000000.0"), (1.5e16, "1.5e16"), (1.25e-7, "1.25e-7"), (0.1, "0.1"), (0.0, "0.0"),
             (-0.0, "-0.0"), (-3.75, "-3.75"), (5e-324, "5e-324"), (1.7976931348623157e308, "1.7976931348623157e308"),
             (9007199254740992.0, "9007199254740992.0"), (float("nan"), "null"), (float("inf"), "null"),
             (float("-inf"), "null"),
             # serde_json's own `test_write_f64` cases (tests/test.rs of the crate, not vendored here)
             (3.0, "3.0"), (3.1, "3.1"), (-1.5, "-1.5"), (0.5, "0.5"),
             (-1.7976931348623157e308, "-1.7976931348623157e308"), (2.220446049250313e-16, "2.220446049250313e-16")]


@pytest.mark.parametrize("x,want", SERDE_F64, ids=[w if w != "null" else repr(x) for x, w in SERDE_F64])
def test_serde_f64(x, want):
    from oxen_amd.hasher import serde_f64

    assert serde_f64(x) == want


def test_metadata_json_audio_video_floats():
    """MetadataAudio / MetadataVideo (model/metadata/metadata_audio.rs:5-15, metadata_video.rs:5-15) as
    serde_json writes them through GenericMetadata (untagged): field order, f64 num_seconds in ryu form
    (an int given for it still prints as a float), usize fields as integers, NaN as null."""
    from oxen_amd.hasher import metadata_json

    for secs, txt in [(12.5, "12.5"), (12.0, "12.0"), (12, "12.0"), (1e-5, "0.00001"), (1e16, "1e16"),
                      (float("nan"), "null")]:
        assert metadata_json({"audio": {"num_seconds": secs, "num_channels": 2, "sample_rate": 44100}}) == \
            '{"audio":{"num_seconds":%s,"num_channels":2,"sample_rate":44100}}' % txt
        assert metadata_json({"video": {"num_seconds": secs, "width": 1920, "height": 1080}}) == \
            '{"video":{"num_seconds":%s,"width":1920,"height":1080}}' % txt
    # integers stay integers outside the f64 fields; strings escape like serde_json
    assert metadata_json({"text": {"num_lines": 3, "num_chars": 9}}) == '{"text":{"num_lines":3,"num_chars":9}}'
    assert metadata_json({"x": "a\"b\\c\n\x01\u00e9/"}) == '{"x":"a\\"b\\\\c\\n\\u0001\u00e9/"}'
    assert metadata_json({"x": [True, None, 1.0]}) == '{"x":[true,null,1.0]}'


def test_metadata_hash_audio_on_oracle(oracle_lib):
    """get_metadata_hash / get_combined_hash (hasher.rs:67-100) of a non-text GenericMetadata, on the
    oracle: XXH3-128 of the serde_json text above, then of content || metadata (LE u128s)."""
    from oxen_amd.hasher import metadata_json

    js = metadata_json({"audio": {"num_seconds": 12.5, "num_channels": 2, "sample_rate": 44100}})
    assert js == '{"audio":{"num_seconds":12.5,"num_channels":2,"sample_rate":44100}}'
    m = oracle_lib.xxh3_128_int(js.encode())
    c = oracle_lib.xxh3_128_int(b"audio bytes")
    comb = oracle_lib.combined_hash(c, m)
    assert comb == oracle_lib.xxh3_128_int(c.to_bytes(16, "little") + m.to_bytes(16, "little"))


@pytest.mark.parametrize("second", [False, True])
@pytest.mark.parametrize("vnode_size", [10_000, 7])
def test_commit_driver_host_logic(monkeypatch, oracle_lib, second, vnode_size):
    """K2 commit driver (split_into_vnodes + compute_dir_node) against the scalar restatement, with the
    batched GPU hash swapped for the oracle so the host-side tree logic is checked on CPU."""
    import _commit

    from oracle import commit_oracle
    from oxen_amd import hasher, merkle

    def cpu_streams(streams, ctx=None):
        return [oracle_lib.xxh3_128_int(s) for s in streams]

    monkeypatch.setattr(hasher, "hash_streams_128bit", cpu_streams)
    entries, existing = _commit.staged_commit(n_files=120, n_dirs=5, second=second)
    vn, dh = merkle.commit_tree(_commit.to_staged(entries), _commit.to_staged(existing), vnode_size, _commit.salt)
    rvn, rdh = commit_oracle.commit_tree(entries, existing, vnode_size, _commit.salt)
    assert set(vn) == set(rvn)
    for d in rvn:
        assert [v.id.value for v in vn[d][0]] == [i for i, _ in rvn[d]], d
        assert [[c.path for c in v.entries] for v in vn[d][0]] == [[n[0] for n in ns] for _, ns in rvn[d]], d
    assert {d: h.value for d, h in dh.items()} == rdh
    if vnode_size == 7:
        assert max(len(v[0]) for v in vn.values()) > 1


def test_thread_pool_stress(tmp_path):
    """The runtime's thread pool survives 100 000 back-to-back parallel_for calls of ragged sizes
    (regression: the caller kept the completion mutex while waiting for the pool to go idle, so the
    worker finishing the last task could block on it forever)."""
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "pool_stress")
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-I", os.path.join(root, "oxen_amd", "csrc"),
                    os.path.join(root, "tests", "native", "pool_stress.cpp"), "-o", exe], check=True)
    r = subprocess.run([exe, "100000"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "done" in r.stdout


def test_utf8_oracles_agree():
    """is_utf8 (util/fs.rs:652-668): Python's strict decoder and the from_utf8 walk restated agree."""
    import random

    from oracle import oracle

    rng = random.Random(4)
    pieces = [b"a", b"\xc3\xa9", b"\xe2\x82\xac", b"\xf0\x9f\x98\x80", b"\xed\x9f\xbf", b"\xf4\x8f\xbf\xbf",
              b"\xc0", b"\xc1\x80", b"\xe0\x80\x80", b"\xed\xa0\x80", b"\xf4\x90\x80\x80", b"\xf5", b"\xff", b"\x80",
              b"\xe2\x82", b"\xf0\x9f", b"\x0a"]
    for _ in range(3000):
        s = b"".join(rng.choice(pieces) for _ in range(rng.randint(0, 40)))
        if rng.random() < 0.3:
            s = s[: rng.randint(0, len(s))]
        if rng.random() < 0.2:
            s = b"x" * (4096 - rng.randint(0, 3)) + s
        assert oracle.is_utf8_prefix(s) == oracle.is_utf8_prefix_dfa(s), s[-8:]
    assert oracle.is_utf8_prefix(b"") and oracle.is_utf8_prefix(b"\xe2\x82")
    assert not oracle.is_utf8_prefix(b"\xe2\x28")
    assert oracle.is_utf8_prefix(b"a" * 4096 + b"\xff")  # only the first 4 KiB count


def test_bench_reference_add_c1(oracle_lib):
    """bench.py's same-run CPU timing of the reference's own case (configs[0]: `oxen add .` on the
    1 001-file text repo, the add loop restated in oracle/): every blob stored, the known answer of
    texts/file_0.txt matched."""
    import bench

    r = bench.cpu_oxen_add_c1(threads=2, reps=1)
    assert r["ok"] and r["files"] == 1001 and r["ms"] > 0


def test_rust_debug_forms():
    """Rust's `{:?}` of a Path (OsStr on Unix: Utf8Chunks Debug) and of a str, as hasher.rs's and
    util::fs::metadata's error texts carry them (error.rs:1176-1182): a Path escapes the single quote and
    writes bytes outside UTF-8 as \\xNN; both escape non-printable and grapheme-extended chars as \\u{..}."""
    from oxen_amd import hasher

    assert hasher.rust_path_debug("/tmp/a") == '"/tmp/a"'
    assert hasher.rust_path_debug(b"it's\xff\xfe") == '"it\\\'s\\xFF\\xFE"'
    assert hasher.rust_path_debug("a​b c x́é漢\U0001f402") == '"a\\u{200b}b\\u{a0}c x\\u{301}é漢\U0001f402"'
    assert hasher.rust_path_debug('q"\\\n\r\t\0\x01\x7f') == '"q\\"\\\\\\n\\r\\t\\0\\u{1}\\u{7f}"'
    assert hasher.rust_str_debug("it's") == '"it\'s"'
    assert hasher.rust_io_error_debug(20) == 'Os { code: 20, kind: NotADirectory, message: "Not a directory" }'
