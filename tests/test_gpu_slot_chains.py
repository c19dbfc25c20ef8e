"""Large items of a staged batch take K1L (staging.hip `submit_slot`): items of 1 MiB and more, the 32
largest of a batch, get their block sums chip-wide and a serial chain instead of one K1 wave, which
reads ~10 GB/s (a slot holding one 200 MiB file waited ~20 ms on its wave). The K1 wave launch sees
those items as empty and the chains overwrite their digests.

Every digest here is checked against the oracle (the published XXH3-128, oracle/xxh3_oracle.c):
lengths around the 1 MiB threshold and the 1 KiB block edges, more large items in one slot than one
chain launch takes, items just below a slot, unaligned items in a stream arena, and every staged
entry (the file engine, the small-request path, host buffers, streams, the fused add); in K1T
batches the large items' text counts come from text_count_kernel, checked against a direct count.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

MIB = 1 << 20
EDGES = [MIB - 1, MIB, MIB + 1, MIB + 1023, MIB + 1024, MIB + 1025, 3 * MIB + 17, 5, 0]


def _blobs(sizes, seed):
    rng = np.random.default_rng(seed)
    return [rng.integers(0, 256, s, dtype=np.uint8).tobytes() for s in sizes]


def _write(tmp_path, blobs, prefix="f"):
    paths = []
    for i, b in enumerate(blobs):
        p = tmp_path / f"{prefix}{i}"
        p.write_bytes(b)
        paths.append(str(p))
    return paths


def test_threshold_lengths_every_entry(ctx, oracle_lib, tmp_path):
    from oxen_amd import hasher

    blobs = _blobs(EDGES, 71)
    want = [oracle_lib.xxh3_128_int(b) for b in blobs]
    paths = _write(tmp_path, blobs)
    d, sizes, st = hasher.hash_files_128bit(paths, ctx=ctx)  # one engine request
    assert d == want and sizes == EDGES and not any(st)
    for p, w in zip(paths, want):  # one file per call: the small-request path
        assert hasher.hash_files_with_errors_128bit([p], ctx=ctx)[0] == [w]
    assert hasher.hash_buffers_128bit(blobs, ctx) == want
    assert hasher.hash_streams_128bit(blobs, ctx) == want  # back to back: unaligned large items
    assert hasher.hash_streams_128bit(blobs[::-1], ctx) == want[::-1]
    digests, _, st, stored = hasher.add_files(paths, str(tmp_path / "versions"), ctx=ctx)
    assert digests == want and not any(st)
    for b, dg in zip(blobs, digests):
        with open(hasher.version_path(str(tmp_path / "versions"), dg), "rb") as f:
            assert f.read() == b


def test_more_large_items_than_one_chain_launch(cuda, oracle_lib, tmp_path):
    """A 96 MiB slot holding ~60 items of 1-1.5 MiB among small ones: the 32 largest on K1L, the rest
    on waves, across several slots."""
    from oxen_amd import _capi, hasher

    rng = np.random.default_rng(72)
    sizes = []
    for _ in range(150):
        sizes.append(int(rng.integers(MIB, MIB + MIB // 2)) if rng.random() < 0.6 else int(rng.integers(0, 70_000)))
    blobs = _blobs(sizes, 73)
    want = [oracle_lib.xxh3_128_int(b) for b in blobs]
    paths = _write(tmp_path, blobs)
    with _capi.Context(0, staging_bytes=96 * MIB) as c:
        d, got_sizes, st = hasher.hash_files_128bit(paths, ctx=c)
        assert d == want and got_sizes == sizes and not any(st)
        assert hasher.hash_buffers_128bit(blobs, c) == want


def test_items_just_below_a_slot(cuda, oracle_lib, tmp_path):
    """Files of a slot's size less one byte (the engine reserves L + 1) and less 257, with small files
    around them, on a 24 MiB staging context: one large item per slot."""
    from oxen_amd import _capi, hasher

    stage = 24 * MIB
    sizes = [stage - 1, 3, stage - 257, 4096, MIB + 7, stage - 1 - 4096]
    blobs = _blobs(sizes, 74)
    want = [oracle_lib.xxh3_128_int(b) for b in blobs]
    paths = _write(tmp_path, blobs)
    with _capi.Context(0, staging_bytes=stage) as c:
        d, got_sizes, st = hasher.hash_files_128bit(paths, ctx=c)
        assert d == want and got_sizes == sizes and not any(st)
        assert hasher.hash_buffers_128bit(blobs, c) == want


def _counts(b):
    """MetadataText of bytes (repositories/metadata/text.rs:12-20): 1 + newlines, and the bytes that
    are not UTF-8 continuation bytes (bytecount::num_chars)."""
    a = np.frombuffer(b, dtype=np.uint8)
    return {"text": {"num_lines": 1 + b.count(b"\n"), "num_chars": len(b) - int(((a & 0xC0) == 0x80).sum())}}


def test_text_request_with_large_files(ctx, oracle_lib, tmp_path):
    """K1T batches too: large items take K1L for the digest and text_count_kernel for the counts, the
    rest K1T's wave. Text of 1 MiB +- a byte, ragged tails, multi-byte characters across 16-B loads,
    random bytes, a 20 MiB text file read in parts; digests against the oracle, counts against a direct
    count of the bytes, is_utf8 against the oracle's sniff."""
    from oxen_amd import hasher

    line = "row,é,中,\U0001f600\n".encode()
    rnd = _blobs([2 * MIB + 3, MIB + 9], 75)
    blobs = [(line * (MIB // len(line) + 2))[:n] for n in (MIB - 1, MIB, MIB + 1, 3 * MIB + 13)]
    blobs += [rnd[0], b"a\nb", rnd[1], (line * (20 * MIB // len(line) + 1))[: 20 * MIB + 5], b""]
    paths = _write(tmp_path, blobs)
    d, _, st, meta = hasher.hash_files_text_128bit(paths, ctx=ctx)
    assert not any(st) and d == [oracle_lib.xxh3_128_int(b) for b in blobs]
    assert meta == [_counts(b) for b in blobs]
    d, _, st, meta, u8 = hasher.hash_files_text_utf8_128bit(paths, ctx=ctx)
    assert not any(st) and d == [oracle_lib.xxh3_128_int(b) for b in blobs]
    assert meta == [_counts(b) for b in blobs]
    assert u8 == [oracle_lib.is_utf8_prefix(b[:4096]) for b in blobs]
    for p, b in zip(paths, blobs):  # one file per call: the small-request path (up to 2 MiB)
        _, _, st, m = hasher.hash_files_text_128bit([p], ctx=ctx)
        assert st == [0] and m == [_counts(b)]


# Files of 8 MiB and more in a slot are read in 4 MiB parts by several readers (engine.hip run_part);
# the parts cover [0, L + 1) so a size that changed since the stat (or the caller's metadata) still
# sends the file to the engine's re-read.
SPLIT = [8 * MIB - 1, 8 * MIB, 8 * MIB + 1, 12 * MIB - 1, 12 * MIB, 12 * MIB + 1, 40 * MIB + 5, 77, 0]


def test_split_reads(ctx, oracle_lib, tmp_path):
    from oxen_amd import hasher

    blobs = _blobs(SPLIT, 76)
    want = [oracle_lib.xxh3_128_int(b) for b in blobs]
    paths = _write(tmp_path, blobs)
    d, sizes, st = hasher.hash_files_128bit(paths, ctx=ctx)
    assert d == want and sizes == SPLIT and not any(st)
    d, _, st, meta = hasher.hash_files_text_128bit(paths, ctx=ctx)  # K1T over split reads
    assert d == want and not any(st)
    digests, _, st, _ = hasher.add_files(paths, str(tmp_path / "versions"), ctx=ctx)
    assert digests == want and not any(st)
    for b, dg in zip(blobs, digests):
        with open(hasher.version_path(str(tmp_path / "versions"), dg), "rb") as f:
            assert f.read() == b


def test_split_reads_with_wrong_caller_sizes(ctx, oracle_lib, tmp_path):
    """Caller sizes (get_hash_given_metadata) that miss the file by a byte, a block or a part, both
    ways, on files read in parts: each is re-read whole and hashed as it is."""
    from oxen_amd import hasher

    sizes = [8 * MIB, 12 * MIB + 1, 20 * MIB + 3, 9 * MIB, 16 * MIB]
    blobs = _blobs(sizes, 77)
    want = [oracle_lib.xxh3_128_int(b) for b in blobs]
    paths = _write(tmp_path, blobs)
    for delta in (-1, 1, -1024, 4 * MIB, -4 * MIB - 1, 0):
        meta = [max(0, s + delta) for s in sizes]
        d, got, st, _ = hasher.hash_files_with_errors_128bit(paths, meta, ctx=ctx)
        assert d == want and got == sizes and not any(st), delta


def test_split_reads_small_slots(cuda, oracle_lib, tmp_path):
    """A 24 MiB staging context: one or two split files per slot, so readers wait for slots whose
    files still have parts queued (they read those parts meanwhile), across many slot turns."""
    from oxen_amd import _capi, hasher

    rng = np.random.default_rng(78)
    sizes = [int(rng.integers(8 * MIB, 23 * MIB)) if k % 3 else int(rng.integers(0, 300_000)) for k in range(36)]
    blobs = _blobs(sizes, 79)
    want = [oracle_lib.xxh3_128_int(b) for b in blobs]
    paths = _write(tmp_path, blobs)
    with _capi.Context(0, staging_bytes=24 * MIB) as c:
        for _ in range(2):
            d, got, st = hasher.hash_files_128bit(paths, ctx=c)
            assert d == want and got == sizes and not any(st)


def test_split_reads_under_replacement(ctx, oracle_lib, tmp_path):
    """A 20 MiB file replaced (new content, temp + rename) and briefly removed while it is hashed again
    and again: every answer is one whole version of the file (the parts read the inode the first reader
    opened) or, when the path did not exist at the open, OXH_ERR_OPEN with ENOENT."""
    import errno
    import os
    import threading

    from oxen_amd import _capi, hasher

    p = tmp_path / "hot.bin"
    versions = _blobs([20 * MIB + 11, 20 * MIB - 5, 12 * MIB, 9 * MIB + 1], 80)
    digests = {oracle_lib.xxh3_128_int(v) for v in versions}
    p.write_bytes(versions[0])
    stop = threading.Event()

    def mutate():
        k = 0
        while not stop.is_set():
            k += 1
            tmp = tmp_path / "hot.tmp"
            tmp.write_bytes(versions[k % len(versions)])
            if k % 5 == 0:
                os.remove(p)
            os.replace(tmp, p)

    th = threading.Thread(target=mutate)
    th.start()
    seen = set()
    try:
        for _ in range(60):
            d, _, st, oserr = hasher.hash_files_with_errors_128bit([str(p)] * 9, ctx=ctx)  # 9: the engine
            for dg, s, e in zip(d, st, oserr):
                assert (s == 0 and dg in digests) or (s == _capi.OXH_ERR_OPEN and e == errno.ENOENT), (s, e)
                seen.add(dg)
    finally:
        stop.set()
        th.join()
    assert len(seen - {None}) >= 2  # the test did race the replacements
