"""The fused add's version-store publish and the file engine's failure isolation, through the C ABI.

Covers the round-1 advisor findings: oversize files streamed into a `data.oxentmp.<random>` temp
(never whole in host memory), per-file allocation failures as per-item statuses (the live run keeps
going), a failed publish shared by every duplicate of that content, read-to-EOF semantics for files
whose stat size is wrong, and a context at the staging-size limit.
"""
import os

import pytest

pytestmark = pytest.mark.gpu

BIG_SIZES = [(9 << 20) + 17, (6 << 20) + 3]  # > the 4 MiB staging slots below


def _small(k):
    from oxen_amd.workloads import splitmix_bytes

    return splitmix_bytes(500 + k, 0, 70_000 + k).tobytes()


def _big(k):
    from oxen_amd.workloads import splitmix_bytes

    return splitmix_bytes(700 + k, 0, BIG_SIZES[k]).tobytes()


def _write(tmp_path, name, data):
    p = tmp_path / name
    p.write_bytes(data)
    return str(p)


def _tree(root):
    return sorted(os.path.relpath(os.path.join(dp, f), root) for dp, _, fs in os.walk(root) for f in fs)


PUBLISH_MODES = {"committer": {}, "inline": {"OXH_PUBLISH_INLINE": "1"}, "fsync_each": {"OXH_PUBLISH_SYNC": "fsync"},
                 "inline_fsync_each": {"OXH_PUBLISH_INLINE": "1", "OXH_PUBLISH_SYNC": "fsync"}}


@pytest.mark.parametrize("mode", sorted(PUBLISH_MODES))
def test_add_files_streams_oversize_blobs_and_shares_publish_failures(cuda, oracle_lib, tmp_path, monkeypatch, mode):
    """Every publish form (committer thread or inline drain; two syncfs barriers or the reference's
    per-blob fsync / rename / parent fsync) gives the same store and the same per-item outcomes."""
    for k, v in PUBLISH_MODES[mode].items():
        monkeypatch.setenv(k, v)
    from oracle import oracle
    from oxen_amd import _capi, hasher

    smalls = {k: _small(k) for k in (0, 2, 3, 4, 6, 7)}
    bigs = [_big(0), _big(1)]
    paths, blobs = [], []
    for k, b in smalls.items():
        paths.append(_write(tmp_path, f"s{k}", b)), blobs.append(b)
    for k, b in enumerate(bigs):
        paths.append(_write(tmp_path, f"b{k}", b)), blobs.append(b)
    paths.append(_write(tmp_path, "b0-copy", bigs[0])), blobs.append(bigs[0])      # duplicate big content
    paths.append(_write(tmp_path, "s7-copy", smalls[7])), blobs.append(smalls[7])  # duplicate small content
    paths.append(str(tmp_path / "missing"))
    want = [oracle.xxh3_128_int(b) for b in blobs]
    hexes = [format(w, "x") for w in want]
    blocked = hexes[paths.index(str(tmp_path / "s7"))][:2]
    assert sum(h[:2] == blocked for h in hexes) == 2  # only s7 and its copy live under that prefix
    root = tmp_path / "store" / "versions" / "files"
    root.mkdir(parents=True)
    (root / blocked).write_bytes(b"not a directory")  # s7's publish cannot create its blob dir

    with _capi.Context(0, staging_bytes=4 << 20) as c:
        d, sz, st, stored = hasher.add_files(paths, str(root), c)
        for i, p in enumerate(paths[:-1]):
            if hexes[i][:2] == blocked:  # the publish failed: both items fail, digest None
                assert st[i] == _capi.OXH_ERR_IO and d[i] is None and not stored[i], p
                continue
            assert st[i] == 0 and d[i] == want[i] and sz[i] == len(blobs[i]), p
            with open(hasher.version_path(str(root), want[i]), "rb") as f:
                assert f.read() == blobs[i], p
        assert st[-1] != 0 and d[-1] is None
        # every distinct published content stored exactly once (the big duplicate included)
        ok_hex = {hexes[i] for i in range(len(paths) - 1) if hexes[i][:2] != blocked}
        assert sum(stored) == len(ok_hex)
        assert stored[paths.index(str(tmp_path / "b0"))] != stored[paths.index(str(tmp_path / "b0-copy"))]
        assert not any(".oxentmp." in f for f in _tree(root)), _tree(root)
        # a second add publishes nothing new; the blocked content still fails
        d2, _, st2, stored2 = hasher.add_files(paths[:-1], str(root), c)
        assert not any(stored2) and [s != 0 for s in st2] == [h[:2] == blocked for h in hexes]
        assert not any(".oxentmp." in f for f in _tree(root))


def test_big_file_allocation_failure_is_per_file(cuda, oracle_lib, tmp_path, monkeypatch):
    """A device allocation the large-file path cannot get (here: 512 GiB pieces) fails that file with
    OXH_ERR_NOMEM; the other files of the same call, and later calls, are unaffected."""
    from oracle import oracle
    from oxen_amd import _capi, hasher

    small, big = _small(0), _big(1)
    paths = [_write(tmp_path, "s", small), _write(tmp_path, "b", big)]
    root = str(tmp_path / "store")
    with _capi.Context(0, staging_bytes=4 << 20) as c:
        monkeypatch.setenv("OXH_BIG_PIECE_MIB", str(1 << 19))
        d, sz, st = hasher.hash_files_128bit(paths, c)
        assert st == [0, _capi.OXH_ERR_NOMEM] and d == [oracle.xxh3_128_int(small), None]
        # os_error is the errno of a failed open or read only: 0 for an allocation failure (include/oxen_hash.h)
        d, sz, st, oserr = hasher.hash_files_with_errors_128bit(paths, None, c)
        assert st == [0, _capi.OXH_ERR_NOMEM] and oserr == [0, 0]
        d, sz, st, stored = hasher.add_files(paths, root, c)
        assert st == [0, _capi.OXH_ERR_NOMEM] and stored == [True, False]
        assert not any(".oxentmp." in f for f in _tree(root))
        monkeypatch.delenv("OXH_BIG_PIECE_MIB")
        d, sz, st, stored = hasher.add_files(paths, root, c)
        assert st == [0, 0] and stored == [False, True]
        assert d == [oracle.xxh3_128_int(small), oracle.xxh3_128_int(big)]
        with open(hasher.version_path(root, d[1]), "rb") as f:
            assert f.read() == big


def test_big_files_fall_back_to_fewer_side_by_side(cuda, oracle_lib, tmp_path, monkeypatch):
    """large files share one piece pipeline, 2 device piece buffers each. When the buffers
    for all of them do not fit (here 4 files x 2 x 40 GiB pieces, more than the device holds), the
    engine takes fewer side by side, down to one, instead of failing every file with OXH_ERR_NOMEM."""
    from oracle import oracle
    from oxen_amd import _capi, hasher

    from oxen_amd.workloads import splitmix_bytes

    bigs = [splitmix_bytes(800 + k, 0, (5 << 20) + 1000 * k + 7).tobytes() for k in range(4)]
    paths = [_write(tmp_path, f"b{k}", b) for k, b in enumerate(bigs)]
    monkeypatch.setenv("OXH_BIG_FILES", "4")
    monkeypatch.setenv("OXH_BIG_PIECE_MIB", str(40 << 10))
    with _capi.Context(0, staging_bytes=4 << 20) as c:
        d, sz, st = hasher.hash_files_128bit(paths, c)
    assert st == [0] * 4 and d == [oracle.xxh3_128_int(b) for b in bigs]


def test_files_are_read_to_eof_whatever_the_stat_size(cuda, oracle_lib, tmp_path):
    """read_to_end semantics (hasher.rs:126-148): /proc/version stats as 0 bytes but reads as text;
    the fstat path and the caller-metadata path both hash what the read returns."""
    from oracle import oracle
    from oxen_amd import _capi, hasher

    if not os.path.exists("/proc/version") or os.stat("/proc/version").st_size != 0:
        pytest.skip("needs a procfs file whose stat size is 0")
    data = open("/proc/version", "rb").read()
    assert data
    other = _write(tmp_path, "f", _small(2))
    paths = ["/proc/version", other]
    want = [oracle.xxh3_128_int(data), oracle.xxh3_128_int(_small(2))]
    with _capi.Context(0, staging_bytes=1 << 20) as c:
        d, sz, st = hasher.hash_files_128bit(paths, c)
        assert st == [0, 0] and d == want and sz[0] == len(data)
        d, sz, st = hasher.hash_files_given_metadata_128bit(paths, [0, os.path.getsize(other)], c)
        assert st == [0, 0] and d == want


def test_context_at_the_staging_limit(cuda, oracle_lib, tmp_path):
    """The largest accepted staging size (3 x (2 GiB - 256) pinned + device) hashes files correctly."""
    from oracle import oracle
    from oxen_amd import _capi, hasher

    blobs = [_small(k) for k in range(4)] + [b"", _big(0)]
    paths = [_write(tmp_path, f"f{k}", b) for k, b in enumerate(blobs)]
    with _capi.Context(0, staging_bytes=_capi.OXH_MAX_STAGING_BYTES) as c:
        d, sz, st = hasher.hash_files_128bit(paths * 3, c)
    assert st == [0] * len(paths) * 3
    assert d == [oracle.xxh3_128_int(b) for b in blobs] * 3


@pytest.mark.parametrize("piece_mib", [None, "2"], ids=["one-piece", "2MiB-pieces"])
def test_host_buffers_larger_than_staging(cuda, oracle_lib, monkeypatch, piece_mib):
    """oxh_hash_buffers / oxh_hash_streams with items above the 1 MiB staging slot: they go straight
    from the caller's memory through the bounce buffers and the device pieces (no whole-item copy on
    the host or the device), between ordinary staged items."""
    from oracle import oracle
    from oxen_amd import _capi, hasher
    from oxen_amd.workloads import splitmix_bytes

    if piece_mib:
        monkeypatch.setenv("OXH_BIG_PIECE_MIB", piece_mib)
    sizes = [100, (5 << 20) + 3, 70_000, 1 << 20, (1 << 20) + 1, 0, (2 << 20) + 1025, 241]
    bufs = [splitmix_bytes(900 + k, 0, s).tobytes() for k, s in enumerate(sizes)]
    want = [oracle.xxh3_128_int(b) for b in bufs]
    with _capi.Context(0, staging_bytes=1 << 20) as c:
        assert hasher.hash_buffers_128bit(bufs, c) == want
        assert hasher.hash_streams_128bit(bufs, c) == want


def test_concurrent_adds_into_one_store(cuda, oracle_lib, tmp_path):
    """Several threads add overlapping file lists into one version store through one context (their
    requests join the engine's live run; each call's publisher commits on its own thread): every
    blob ends up whole under its digest, no temp is left, and each call reports every file."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import oracle
    from oxen_amd import _capi, hasher

    blobs = [_small(k) for k in range(40)] + [_big(0)]
    paths = [_write(tmp_path, f"f{k}", b) for k, b in enumerate(blobs)]
    want = [oracle.xxh3_128_int(b) for b in blobs]
    root = str(tmp_path / "store" / "versions" / "files")
    lists = [list(range(k, len(paths), 3)) + list(range(0, len(paths), 5)) for k in range(3)] + [list(range(len(paths)))]
    with _capi.Context(0, staging_bytes=2 << 20) as c:
        def add(idx):
            d, _, st, stored = hasher.add_files([paths[i] for i in idx], root, c)
            return idx, d, st, stored

        with ThreadPoolExecutor(4) as ex:
            results = list(ex.map(add, lists * 2))
    for idx, d, st, stored in results:
        assert st == [0] * len(idx) and d == [want[i] for i in idx]
    assert sum(s for _, _, _, stored in results for s in stored) >= len(set(want))
    for w, b in zip(want, blobs):
        with open(hasher.version_path(root, w), "rb") as f:
            assert f.read() == b
    assert not any(".oxentmp." in f for f in _tree(root)), _tree(root)


@pytest.mark.parametrize("layout", ["forward", "gaps", "repeats", "backward", "sparse"])
def test_hash_streams_arena_layouts(cuda, oracle_lib, layout):
    """oxh_hash_streams over the arena layouts a caller can pass: items running forward (copied as
    spans), with small gaps, the same stream referenced several times, offsets running backward and
    a sparse arena (both copied item by item); empty items, items above the 1 MiB staging slot and
    more items than one slot's descriptor table, against the oracle."""
    import numpy as np

    from oracle import oracle
    from oxen_amd import _capi
    from oxen_amd.workloads import splitmix_bytes

    rng = np.random.default_rng(11)
    sizes = [int(x) for x in rng.integers(0, 300, 3000)] + [0, (1 << 20) + 77, 5000, 241, 240, 0]
    sizes += [int(x) for x in rng.integers(1, 64, 2000)]
    blobs = [splitmix_bytes(1300 + k, 0, s).tobytes() for k, s in enumerate(sizes)]
    if layout == "repeats":
        blobs = [blobs[k // 3] for k in range(len(blobs))]
    parts, offs, pos = [], [], 0
    for k, b in enumerate(blobs):
        gap = {"gaps": k % 5, "sparse": 20_000}.get(layout, 0)
        if layout == "repeats" and k % 3:
            offs.append(offs[-1])  # the same bytes again
            continue
        parts.append(b"\xee" * gap)
        pos += gap
        offs.append(pos)
        parts.append(b)
        pos += len(b)
    arena = np.frombuffer(b"".join(parts) + b"\0", dtype=np.uint8)
    order = list(range(len(blobs)))
    if layout == "backward":
        order = order[::-1]
    lens = np.array([len(blobs[k]) for k in order], dtype=np.uint64)
    o = np.array([offs[k] for k in order], dtype=np.uint64)
    out = np.zeros((len(order), 2), dtype=np.uint64)
    with _capi.Context(0, staging_bytes=1 << 20) as c:  # 1024 items per slot: several batches
        _capi.check(_capi.lib().oxh_hash_streams(c.handle, arena.ctypes.data, o.ctypes.data_as(_capi._u64p),
                                                 lens.ctypes.data_as(_capi._u64p), len(order),
                                                 out.ctypes.data_as(_capi._u64p)), "oxh_hash_streams")
    got = [(int(hi) << 64) | int(lo) for lo, hi in out]
    assert got == [oracle.xxh3_128_int(blobs[k]) for k in order]
