"""Verify-before-publish version-store writes (oxen_amd/version_store.py), restating the reference's
own tests: util/fs/atomic_file.rs (temp name pattern :879-909, streams :911-935, verified stream /
write commits on match and aborts on mismatch leaving nothing behind :801-835, :1101-1230, read
failure cleans up :937-985) and storage/version_store.rs verify_suite (:596-650). Known answers:
xxh3_128 of the reference's 50 000-u32 payload (the C oracle and libxxhash agree on it)."""
import io
import os
import struct

import pytest

PAYLOAD = b"".join(struct.pack("<I", i) for i in range(50_000))  # (0..50_000u32).flat_map(to_le_bytes)
PAYLOAD_HASH = 0x290EE6C54069340C8A3C8891CE6B2D9
BOGUS = 0xDEADBEEF_DEADBEEF_DEADBEEF_DEADBEEF
DATA = b"the quick brown fox jumps over the lazy dog"
WRONG_HASH = "deadbeefdeadbeefdeadbeefdeadbeef"
DATA_HASH = "e9a1932627d7f46d15c21eead63fa21f"


class FailingReader:
    """Yields `good` bytes, then raises (atomic_file.rs:937-985)."""

    def __init__(self, good: bytes):
        self.good, self.done = good, False

    def read(self, n):
        if not self.done:
            self.done = True
            return self.good
        raise OSError("simulated read failure")


def test_known_answers_pinned_by_oracle():
    from oracle import oracle

    oracle.build()
    assert oracle.xxh3_128_int(PAYLOAD) == PAYLOAD_HASH
    assert format(oracle.xxh3_128_int(DATA), "x") == DATA_HASH


def test_temp_file_name_pattern(tmp_path):
    from oxen_amd.version_store import ATOMIC_TEMP_INFIX, _TempFile

    tmp = _TempFile(str(tmp_path / "HEAD"))
    name = os.path.basename(tmp.path)
    assert name.startswith("HEAD") and ATOMIC_TEMP_INFIX in name and os.path.dirname(tmp.path) == str(tmp_path)
    tmp.discard()
    assert not os.path.exists(tmp.path)


def test_unverified_stream_and_write_leave_only_the_target(tmp_path):
    """No expected hash: nothing is hashed (no GPU needed), the temp protocol alone."""
    from oxen_amd.version_store import AtomicFile

    AtomicFile(tmp_path / "blob.bin").stream(io.BytesIO(PAYLOAD))
    assert (tmp_path / "blob.bin").read_bytes() == PAYLOAD and os.listdir(tmp_path) == ["blob.bin"]
    AtomicFile(tmp_path / "sub" / "x").write(b"abc")  # parent created
    assert (tmp_path / "sub" / "x").read_bytes() == b"abc" and os.listdir(tmp_path / "sub") == ["x"]
    with pytest.raises(OSError):
        AtomicFile(tmp_path / "c.bin").stream(FailingReader(b"x" * 100))
    assert sorted(os.listdir(tmp_path)) == ["blob.bin", "sub"]


@pytest.mark.gpu
def test_verified_stream_commits_on_match(cuda, tmp_path):
    from oxen_amd.version_store import AtomicFile

    AtomicFile(tmp_path / "blob.bin").with_hash(PAYLOAD_HASH).stream(io.BytesIO(PAYLOAD))
    assert (tmp_path / "blob.bin").read_bytes() == PAYLOAD and os.listdir(tmp_path) == ["blob.bin"]


@pytest.mark.gpu
@pytest.mark.parametrize("how", ["stream", "write"])
def test_verified_aborts_on_mismatch(cuda, tmp_path, how):
    from oxen_amd.version_store import AtomicFile, HashMismatchError

    target = str(tmp_path / "blob.bin")
    f = AtomicFile(target).with_hash(BOGUS)
    with pytest.raises(HashMismatchError) as ei:
        f.stream(io.BytesIO(PAYLOAD)) if how == "stream" else f.write(PAYLOAD)
    e = ei.value
    assert e.path == target and e.expected == BOGUS and e.actual == PAYLOAD_HASH
    assert "mismatch" in str(e).lower()
    assert os.listdir(tmp_path) == []


@pytest.mark.gpu
def test_verified_stream_cleans_up_on_read_failure(cuda, tmp_path):
    from oxen_amd.version_store import AtomicFile

    with pytest.raises(OSError):
        AtomicFile(tmp_path / "blob.bin").with_hash(PAYLOAD_HASH).stream(FailingReader(PAYLOAD[:4096]))
    assert os.listdir(tmp_path) == []


@pytest.mark.gpu
def test_version_store_rejects_mismatched_content(cuda, tmp_path):
    """verify_suite::assert_rejects_mismatched_content for the local store's two content-addressed
    writes, then the accepted path, the existing-blob skip and the batched receive."""
    from oxen_amd import hasher
    from oxen_amd.version_store import HashMismatchError, LocalVersionStore

    store = LocalVersionStore(tmp_path / "versions")
    assert hasher.hash_buffer(DATA) != WRONG_HASH
    with pytest.raises(HashMismatchError):
        store.store_version(WRONG_HASH, DATA)
    assert not store.version_exists(WRONG_HASH)
    with pytest.raises(HashMismatchError):
        store.store_version_from_reader(WRONG_HASH, io.BytesIO(DATA), len(DATA))
    assert not store.version_exists(WRONG_HASH)

    store.store_version_from_reader(DATA_HASH, io.BytesIO(DATA), len(DATA))
    assert store.version_path(DATA_HASH) == str(tmp_path / "versions" / "e9" / "a1932627d7f46d15c21eead63fa21f" / "data")
    assert open(store.version_path(DATA_HASH), "rb").read() == DATA
    store.store_version(DATA_HASH, b"ignored: the blob exists")  # local.rs:127-129
    assert open(store.version_path(DATA_HASH), "rb").read() == DATA

    big = os.urandom((3 << 20) + 17)
    hs = [hasher.hash_buffer(PAYLOAD), WRONG_HASH, DATA_HASH, hasher.hash_buffer(b""), hasher.hash_buffer(big),
          hasher.hash_buffer(PAYLOAD), "not-hex"]
    ds = [PAYLOAD, DATA, DATA, b"", big, PAYLOAD, b"x"]
    errs = store.store_versions(hs, ds)
    assert [type(e).__name__ if e else None for e in errs] == [None, "HashMismatchError", None, None, None, None, "OxenError"]
    assert open(store.version_path(hs[0]), "rb").read() == PAYLOAD
    assert open(store.version_path(hs[4]), "rb").read() == big
    assert os.path.getsize(store.version_path(hs[3])) == 0 and not store.version_exists(WRONG_HASH)
    for h in hs[:6]:
        if store.version_exists(h):
            assert os.listdir(store.version_dir(h)) == ["data"]


@pytest.mark.gpu
def test_stream_from_paths_concatenates_and_verifies(cuda, oracle_lib, tmp_path):
    """atomic_file.rs:598-632 / :634-650: the in-order concatenation of chunk files is published
    under the expected digest (hashed on the GPU), nothing else is left beside the target; a wrong
    digest publishes nothing."""
    from oracle import oracle
    from oxen_amd.version_store import AtomicFile, HashMismatchError

    chunks = tmp_path / "chunks"
    chunks.mkdir()
    parts = [b"hello ", b"brave ", b"world"]
    paths = []
    for i, part in enumerate(parts):
        (chunks / str(i)).write_bytes(part)
        paths.append(str(chunks / str(i)))
    full = b"".join(parts)
    target = tmp_path / "blob.bin"
    AtomicFile(target).with_hash(oracle.xxh3_128_int(full)).stream_from_paths(paths)
    assert target.read_bytes() == full
    assert sorted(os.listdir(tmp_path)) == ["blob.bin", "chunks"]

    (tmp_path / "chunk0").write_bytes(b"payload")
    target2 = tmp_path / "blob2.bin"
    with pytest.raises(HashMismatchError):
        AtomicFile(target2).with_hash(BOGUS).stream_from_paths([str(tmp_path / "chunk0")])
    assert not target2.exists() and not any(".oxentmp." in n for n in os.listdir(tmp_path))


@pytest.mark.gpu
def test_combine_version_chunks(cuda, tmp_path):
    """local.rs:862-891: chunks stored at their byte offsets are reassembled in offset order (the
    offsets sort numerically, not as names), verified against the blob's hash and the chunks
    directory removed; here also with chunks larger than one streaming piece, and a mismatch that
    publishes nothing and keeps the chunks."""
    from oxen_amd import hasher
    from oxen_amd.version_store import HashMismatchError, LocalVersionStore, STREAMING_BUF_SIZE

    store = LocalVersionStore(tmp_path / "versions")
    data = b"chunk-zero-byteschunk-one-bytes"
    h = hasher.hash_buffer(data)
    store.store_version_chunk(h, 0, data[:16])
    store.store_version_chunk(h, 16, data[16:])
    assert os.path.isdir(store.version_chunks_dir(h))
    store.combine_version_chunks(h)
    assert store.get_version(h) == data and not os.path.exists(store.version_chunks_dir(h))

    big = os.urandom(2 * STREAMING_BUF_SIZE + 12345)
    hb = hasher.hash_buffer(big)
    cuts = [0, 7, 100_000, STREAMING_BUF_SIZE + 3, len(big)]  # offsets 7 and 100000 sort after 0, before 10 MiB
    for a, b in zip(cuts, cuts[1:]):
        store.store_version_chunk(hb, a, big[a:b])
    assert store.list_version_chunks(hb) == cuts[:-1]
    store.combine_version_chunks(hb)
    assert store.get_version(hb) == big

    store.store_version_chunk(WRONG_HASH, 0, DATA)
    with pytest.raises(HashMismatchError):
        store.combine_version_chunks(WRONG_HASH)
    assert not store.version_exists(WRONG_HASH) and store.list_version_chunks(WRONG_HASH) == [0]


def test_list_version_chunks_parses_like_rust(tmp_path):
    """chunk directory names are parsed as `name.parse::<u64>()` (local.rs:367-382): an
    optional '+' and ASCII digits below 2**64; entries that are not directories themselves (a file, a
    symlink to a directory: DirEntry::file_type does not follow it) are skipped. Python's int() would
    also have taken '-1', ' 7', '1_0' and non-ASCII digits. No hashing: runs anywhere."""
    from oxen_amd.version_store import LocalVersionStore, parse_u64

    store = LocalVersionStore(tmp_path / "versions")
    d = store.version_chunks_dir(WRONG_HASH)
    os.makedirs(d)
    for name in ["-1", "+5", "1_0", " 7", "7 ", "٣", "18446744073709551616", "18446744073709551615", "007", "x",
                 "+", "", "12"]:
        if name:
            os.makedirs(os.path.join(d, name))
    with open(os.path.join(d, "42"), "w") as f:
        f.write("a file, not a chunk directory")
    os.symlink(os.path.join(d, "12"), os.path.join(d, "99"))
    assert store.list_version_chunks(WRONG_HASH) == [5, 7, 12, 18446744073709551615]
    assert [parse_u64(s) for s in ["0", "+0", "-0", "00", "+-1", "1e3"]] == [0, 0, None, 0, None, None]
