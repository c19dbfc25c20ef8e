"""The fixed-size dedup chunkers (experiments/block-level-dedup/src/chunker/fixedsize.rs and
fixedsize_multithreaded.rs) over the GPU chunk-digest kernel, against a restatement of those files'
pack loops over the oracle: the same chunk files, the same metadata.bin bytes, unpack round trips."""
import ctypes
import os
import struct

import numpy as np
import pytest


def test_bincode_layouts_round_trip():
    from oxen_amd import dedup

    entries = [{"path": ".", "is_dir": True, "chunks": None, "size": None},
               {"path": "d/ü.bin", "is_dir": False, "chunks": ["123", "45"], "size": 9},
               {"path": "e", "is_dir": False, "chunks": [], "size": 0}]
    b = dedup.encode_archive_metadata(4096, entries)
    assert b[:16] == struct.pack("<QQ", 4096, 3)
    assert dedup.decode_archive_metadata(b) == (4096, entries)
    f = dedup.encode_fixed_metadata("x.bin", 70_000, 65_536, ["1", "2"])
    assert dedup.decode_fixed_metadata(f) == ("x.bin", 70_000, 65_536, ["1", "2"])
    with pytest.raises(Exception):
        dedup.decode_fixed_metadata(f[:-1])


def test_chunker_arguments():
    from oxen_amd import dedup

    with pytest.raises(ValueError, match="Chunk size cannot be zero"):
        dedup.FixedSizeChunker(0)
    with pytest.raises(ValueError, match="Concurrency must be greater than zero"):
        dedup.FixedSizeMultiChunker(4096, 0)
    assert dedup.get_chunker("fixed-size", 4096).name() == "fixed-size-chunker"
    assert dedup.get_chunker("fixed-size-multithreaded", 4096).name() == "fixed-size-64k-multithreaded"
    assert dedup.get_chunker("fastcdc", 8192).name() == "fastcdc-chunker"
    with pytest.raises(Exception, match="not found"):
        dedup.get_chunker("nope", 4096)


def _ref_chunks(oracle_lib, data: bytes, chunk: int, out_dir: str, bufreader: bool = False) -> list[str]:
    """fixedsize.rs:69-94 (bufreader: its BufReader read loop, oracle/fixedsize.reads) or
    fixedsize_multithreaded.rs:78-110 (every chunk) restated: name = u128 decimal, write if absent."""
    from oracle import fixedsize

    names = []
    for lo, n in (fixedsize.reads if bufreader else fixedsize.extents)(len(data), chunk):
        piece = data[lo:lo + n]
        name = str(oracle_lib.xxh3_128_int(piece))
        names.append(name)
        p = os.path.join(out_dir, name)
        if not os.path.exists(p):
            open(p, "wb").write(piece)
    return names


def _tree(root, rng):
    os.makedirs(os.path.join(root, "sub", "deeper"))
    os.makedirs(os.path.join(root, "empty_dir"))
    files = {"a.bin": 70_001, "sub/b.bin": 8192 * 3, "sub/deeper/c.txt": 5, "sub/empty.bin": 0, "dup.bin": 70_001}
    data = {}
    for rel, n in files.items():
        data[rel] = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    data["dup.bin"] = data["a.bin"]  # identical content: chunk files shared
    for rel, b in data.items():
        open(os.path.join(root, rel), "wb").write(b)
    return data


def test_bufreader_prefix_matches_the_read_loop():
    """dedup.bufreader_prefix (the product's closed form) against oracle/fixedsize.reads stepping
    BufReader read by read: the reference chunks exactly the fixed-size chunks of that prefix."""
    from oracle import fixedsize

    from oxen_amd import dedup

    sizes = [0, 1, 4095, 4096, 5000, 8191, 8192, 8193, 10_000, 16_384, 70_001, 1 << 20]
    chunks = [1, 3, 1000, 3000, 4096, 5000, 8191, 8192, 8193, 10_000, 65_536]
    for size in sizes:
        for chunk in chunks:
            got = fixedsize.reads(size, chunk)
            pre = dedup.bufreader_prefix(size, chunk)
            assert got == fixedsize.extents(pre, chunk), (size, chunk)
    # chunks beyond one read(2): the first read comes back at MAX_RW_COUNT and the loop stops
    for size, chunk in [(5 << 30, 3 << 30), (1 << 30, 3 << 30), (3 << 30, 0x7FFFF000), (3 << 30, 0x7FFFF001)]:
        assert fixedsize.reads(size, chunk) == fixedsize.extents(dedup.bufreader_prefix(size, chunk), chunk)
    assert dedup.bufreader_prefix(70_001, 5000) == 8192  # 5000 + a short 3192, then the loop ends


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", [4096, 5000, 8192, 65_536])
def test_fixed_size_chunker_tree(cuda, oracle_lib, tmp_path, chunk):
    from oxen_amd import dedup

    rng = np.random.default_rng(chunk)
    src = str(tmp_path / "src")
    _tree(src, rng)
    out, ref = str(tmp_path / "out"), str(tmp_path / "ref")
    dedup.FixedSizeChunker(chunk).pack(src, out)
    # the reference's walk restated: root entry, then read_dir order, dirs before their contents
    os.makedirs(ref)
    entries = [{"path": ".", "is_dir": True, "chunks": None, "size": None}]

    def walk(cur):
        with os.scandir(cur) as it:
            for e in it:
                rel = os.path.relpath(e.path, src)
                if e.is_dir():
                    entries.append({"path": rel, "is_dir": True, "chunks": None, "size": None})
                    walk(e.path)
                elif e.is_file():
                    b = open(e.path, "rb").read()
                    entries.append({"path": rel, "is_dir": False, "chunks": _ref_chunks(oracle_lib, b, chunk, ref, True),
                                    "size": len(b)})

    walk(src)
    assert open(os.path.join(out, "metadata.bin"), "rb").read() == dedup.encode_archive_metadata(chunk, entries)
    got = sorted(f for f in os.listdir(out) if f != "metadata.bin")
    assert got == sorted(os.listdir(ref))
    for f in got:
        assert open(os.path.join(out, f), "rb").read() == open(os.path.join(ref, f), "rb").read()
    back = str(tmp_path / "back")
    dedup.FixedSizeChunker(chunk).unpack(out, back)
    for dp, _, fns in os.walk(src):
        for fn in fns:
            rel = os.path.relpath(os.path.join(dp, fn), src)
            b = open(os.path.join(src, rel), "rb").read()
            # what the reference packed: all of the file, or the prefix its read loop reached
            assert open(os.path.join(back, rel), "rb").read() == b[:dedup.bufreader_prefix(len(b), chunk)]
    assert os.path.isdir(os.path.join(back, "empty_dir"))
    assert dedup.FixedSizeChunker(chunk).get_chunk_hashes(out) == [c for e in entries if not e["is_dir"] for c in e["chunks"]]


@pytest.mark.gpu
@pytest.mark.parametrize("size", [0, 1, 65_536, 65_536 * 5, 65_536 * 5 + 17, (3 << 20) + 1])
def test_fixed_size_multi_chunker_file(cuda, oracle_lib, tmp_path, size):
    from oxen_amd import dedup

    data = np.random.default_rng(size).integers(0, 256, size, dtype=np.uint8).tobytes()
    p = tmp_path / "input.parquet"
    p.write_bytes(data)
    out, ref = str(tmp_path / "out"), str(tmp_path / "ref")
    os.makedirs(ref)
    dedup.FixedSizeMultiChunker(65_536, 16).pack(str(p), out)
    names = _ref_chunks(oracle_lib, data, 65_536, ref)
    assert open(os.path.join(out, "metadata.bin"), "rb").read() == dedup.encode_fixed_metadata("input.parquet", size, 65_536, names)
    for n in names:
        assert open(os.path.join(out, n), "rb").read() == open(os.path.join(ref, n), "rb").read()
    back = str(tmp_path / "back.bin")
    dedup.FixedSizeMultiChunker(65_536, 16).unpack(out, back)
    assert open(back, "rb").read() == data
    if names:
        os.remove(os.path.join(out, names[-1]))
        with pytest.raises(FileNotFoundError, match="Chunk file not found during unpack"):
            dedup.FixedSizeMultiChunker(65_536, 16).unpack(out, back)
    with pytest.raises(FileNotFoundError, match="Failed to read input file metadata"):
        dedup.FixedSizeMultiChunker(65_536, 16).pack(str(tmp_path / "missing"), out)


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", [64, 4096, 5000, 65_536, (1 << 20) + 3, 40 << 20])
def test_chunk_digests_files_segments(cuda, oracle_lib, tmp_path, monkeypatch, chunk):
    """oxh_chunk_digests_files / _host over files that span several 64 MiB device pieces (segments of
    whole chunks, none carried), ragged tails, an empty file, a missing one and a directory, against
    the oracle's xxh3_128 of every chunk."""
    from oracle import fixedsize

    from oxen_amd import dedup

    monkeypatch.setenv("OXH_CDC_PIECE_MIB", "64")
    rng = np.random.default_rng(chunk)
    sizes = [150_000_017, 0, 3, chunk, chunk * 7 + 1, 70_000_000, 5_000_001]
    paths, blobs = [], []
    for i, n in enumerate(sizes):
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        p = tmp_path / f"f{i}.bin"
        p.write_bytes(b)
        paths.append(str(p))
        blobs.append(b)
    paths.insert(2, str(tmp_path / "missing"))
    blobs.insert(2, None)
    paths.insert(4, str(tmp_path))
    blobs.insert(4, None)
    t = dedup.chunk_digests_files(paths, chunk)
    h = dedup.chunk_digests_host([b for b in blobs if b is not None], chunk)
    k = 0
    for i, b in enumerate(blobs):
        got = t.file(i)
        if b is None:
            assert len(got) == 0 and int(t.status[i]) != 0
            assert int(t.os_error[i]) in (2, 21)  # ENOENT, EISDIR
            continue
        assert int(t.status[i]) == 0 and int(t.sizes[i]) == len(b)
        want = oracle_lib.chunk_digests(np.frombuffer(b, dtype=np.uint8), chunk, threads=8)
        assert len(want) == len(fixedsize.extents(len(b), chunk))
        assert np.array_equal(got, want), i
        assert np.array_equal(h.file(k), want), i
        k += 1


@pytest.mark.gpu
def test_chunk_digests_host_one_byte_chunks(cuda, oracle_lib):
    """chunk_size 1 over 9 M bytes: more chunks than one round's budget (4 M), so rounds end on the
    budget rather than the piece; every digest is the xxh3_128 of its byte."""
    from oxen_amd import dedup

    data = np.random.default_rng(1).integers(0, 256, 9_000_001, dtype=np.uint8)
    t = dedup.chunk_digests_host([data, b"", b"xy"], 1)
    table = np.array([oracle_lib.xxh3_128(bytes([v])) for v in range(256)], dtype=np.uint64).reshape(-1, 2)
    assert list(t.first) == [0, data.size, data.size, data.size + 2]
    assert np.array_equal(t.file(0), table[data])
    assert np.array_equal(t.file(2), table[np.frombuffer(b"xy", dtype=np.uint8)])


def test_chunk_digests_arguments():
    """Argument errors before any device work (no GPU needed)."""
    from oxen_amd import _capi, dedup

    with pytest.raises(_capi.OxenError, match="Chunk size cannot be zero"):
        dedup.chunk_digests_host([b"abc"], 0)
    L = _capi.lib()
    first = np.zeros(2, dtype=np.uint64)
    rc = L.oxh_chunk_digests_host(None, None, None, 0, 0, None, 0, first.ctypes.data_as(_capi._u64p))
    assert rc == _capi.OXH_ERR_INVALID and b"zero" in L.oxh_last_error()


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", [4096, 65_536, 100_003])
def test_chunker_test_command_round_trip(cuda, oracle_lib, tmp_path, chunk):
    """main.rs:156-241 (`Test`) with the multithreaded fixed-size chunker: pack, unpack, and the
    whole-file hash_file_128bit of both agree; the digest is the oracle's xxh3_128 of the file."""
    from oxen_amd import dedup

    data = np.random.default_rng(chunk).integers(0, 256, 3_000_017, dtype=np.uint8).tobytes()
    src = tmp_path / "input.bin"
    src.write_bytes(data)
    r = dedup.run_chunker_test("fixed-size-multithreaded", chunk, str(src), str(tmp_path))
    assert r["original_file_hash"] == str(oracle_lib.xxh3_128_int(data))
    assert dedup.hash_file_128bit(os.path.join(r["test_dir"], "unpacked_output")) == int(r["original_file_hash"])
    with pytest.raises(OSError):
        dedup.hash_file_128bit(str(tmp_path / "missing"))


@pytest.mark.gpu
def test_chunker_test_command_fixed_size_reads(cuda, tmp_path):
    """The `fixed-size` (tree) chunker's unpack writes a DIRECTORY at unpacked_output, so the Test
    command fails hashing it, as the reference does (File::open of a directory succeeds, its first
    read fails with EISDIR): "Failed to hash unpacked file"."""
    from oxen_amd import _capi, dedup

    src = tmp_path / "input.bin"
    src.write_bytes(np.random.default_rng(5).integers(0, 256, 70_001, dtype=np.uint8).tobytes())
    with pytest.raises(_capi.OxenError, match="Failed to hash unpacked file"):
        dedup.run_chunker_test("fixed-size", 5000, str(src), str(tmp_path))
    # fastcdc's unpack is the reference's stub: nothing at unpacked_output, the hash fails (ENOENT)
    with pytest.raises(_capi.OxenError, match="Failed to hash unpacked file"):
        dedup.run_chunker_test("fastcdc", 8192, str(src), str(tmp_path))


@pytest.mark.gpu
def test_chunk_digests_capacity_errors(cuda, tmp_path):
    """A digest table too small fails the call with OXH_ERR_INVALID and the count it needs (the caller
    retries with it, as dedup.chunk_digests_files does for a file that grew); no entry past capacity is
    written."""
    from oxen_amd import _capi
    from oxen_amd.hasher import _PathTable, default_context

    data = np.random.default_rng(3).integers(0, 256, 10 * 4096 + 5, dtype=np.uint8).tobytes()
    p = tmp_path / "f.bin"
    p.write_bytes(data)
    L = _capi.lib()
    ctx = default_context()
    table = _PathTable([str(p)])
    dig = np.full((8, 2), 7, dtype=np.uint64)
    first = np.zeros(2, dtype=np.uint64)
    rc = L.oxh_chunk_digests_files(ctx.handle, table.arg, 1, 4096, dig.ctypes.data_as(_capi._u64p), 5,
                                   first.ctypes.data_as(_capi._u64p), None, None, None)
    assert rc == _capi.OXH_ERR_INVALID and b"need 11 entries" in L.oxh_last_error()
    assert (dig[5:] == 7).all()  # nothing past the capacity
    bufs = (ctypes.c_char_p * 1)(data)
    lens = np.array([len(data)], dtype=np.uint64)
    rc = L.oxh_chunk_digests_host(ctx.handle, bufs, lens.ctypes.data_as(_capi._u64p), 1, 4096,
                                  dig.ctypes.data_as(_capi._u64p), 3, first.ctypes.data_as(_capi._u64p))
    assert rc == _capi.OXH_ERR_INVALID and b"need 11 entries" in L.oxh_last_error()


def test_host_entry_routing_rule():
    """INTEGRATION.md §2's rule as code (dedup.host_entry_pays_off; C++ liboxen::dedup::host_entry_pays_off
    in test_hasher.cpp): on the measured 16-core box with one GPU the fixed-size host entry loses to the
    CPU loop (67.7 vs 50.8 GiB/s) and FastCDC's wins (46.9-50.0 vs 34.9-40.3); more links or fewer cores
    move the crossover."""
    from oxen_amd import dedup

    assert not dedup.host_entry_pays_off(16, 1, fastcdc=False)
    assert dedup.host_entry_pays_off(16, 1, fastcdc=True)
    assert dedup.host_entry_pays_off(8, 1, fastcdc=False)       # 33.6 < 49 GiB/s
    assert not dedup.host_entry_pays_off(128, 8, fastcdc=False)  # 537.6 > 392
    assert dedup.host_entry_pays_off(128, 8, fastcdc=True)       # 307.2 < 392
    assert not dedup.host_entry_pays_off(64, 0, fastcdc=True)    # no GPU, no link
