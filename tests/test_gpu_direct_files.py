"""Small file requests on an idle context run on the caller's thread (engine.hip `direct_files`): the
per-file callers of hasher.rs (hash_file_contents from restore / checkout / the metadata CLI,
hasher.rs:102-124) pay one read, one H2D, one launch and one D2H instead of an engine run's hand-offs.

The answers must be the engine's, item for item: digests, sizes, statuses, errnos, text counts and
is_utf8, for good files, empty ones, directories, FIFOs, missing paths, files used as directories,
unreadable modes, files whose size differs from the caller's metadata (handed back to the engine),
and requests the direct path declines (more than 8 files, more than 2 MiB, a file above a staging
slot). Each case runs with OXH_DIRECT_FILES=0 (the engine) and =1, the context's counters show which
form ran, and every good digest is checked against the oracle. A concurrent test mixes single-file
calls with large engine requests on one context.
"""
import os
import threading
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _ex(ctx, paths, meta=None, text=True, utf8=True):
    """oxh_hash_files_ex with every output: (out, sizes, status, os_error, counts, is_utf8) as lists."""
    from oxen_amd import _capi, hasher

    n = len(paths)
    table = hasher._PathTable(paths)
    m = None if meta is None else np.ascontiguousarray(meta, dtype=np.uint64)
    out = np.full((n, 2), 7, dtype=np.uint64)
    sizes = np.zeros(n, dtype=np.uint64)
    st = np.full(n, -99, dtype=np.int32)
    oserr = np.full(n, -99, dtype=np.int32)
    counts = np.full((n, 2), 7, dtype=np.uint64) if text else None
    u8 = np.full(n, 7, dtype=np.int32) if utf8 else None
    _capi.check(_capi.lib().oxh_hash_files_ex(
        ctx.handle, table.arg, None if m is None else m.ctypes.data_as(_capi._u64p), n,
        out.ctypes.data_as(_capi._u64p), sizes.ctypes.data_as(_capi._u64p), st.ctypes.data_as(_capi._i32p),
        oserr.ctypes.data_as(_capi._i32p), None if counts is None else counts.ctypes.data_as(_capi._u64p),
        None if u8 is None else u8.ctypes.data_as(_capi._i32p)), "oxh_hash_files_ex")
    return (out.tolist(), sizes.tolist(), st.tolist(), oserr.tolist(),
            None if counts is None else counts.tolist(), None if u8 is None else u8.tolist())


def _both(monkeypatch, ctx, fn):
    """fn() through the engine and through the direct path: (engine result, direct result, direct calls)."""
    monkeypatch.setenv("OXH_DIRECT_FILES", "0")
    before = ctx.counters()["direct_requests"]
    eng = fn()
    assert ctx.counters()["direct_requests"] == before
    monkeypatch.setenv("OXH_DIRECT_FILES", "1")
    # the engine closes its run a few us after its last request returns; a request arriving before
    # that joins the live run instead (also correct, but not the form under test)
    time.sleep(0.05)
    d = fn()
    return eng, d, ctx.counters()["direct_requests"] - before


@pytest.fixture
def tree(tmp_path):
    rng = np.random.default_rng(61)
    files = {
        "empty": b"",
        "one": b"a",
        "hello": b"hello",
        "k4": rng.integers(0, 256, 4096, dtype=np.uint8).tobytes(),
        "text": ("line é中\U0001f600 x\n" * 12000).encode(),
        "latin1": b"caf\xe9\n" * 100,
        "m1": rng.integers(0, 256, 1 << 20, dtype=np.uint8).tobytes(),
        "big": rng.integers(0, 256, 3 << 20, dtype=np.uint8).tobytes(),  # above the direct path's 2 MiB
    }
    for k, v in files.items():
        (tmp_path / k).write_bytes(v)
    (tmp_path / "adir").mkdir()
    os.mkfifo(tmp_path / "fifo")
    locked = tmp_path / "locked"
    locked.write_bytes(b"secret")
    locked.chmod(0)
    bad = {"adir": None, "fifo": None, "missing": None, "notdir": None, "locked": None}
    paths = {k: str(tmp_path / k) for k in list(files) + list(bad)}
    paths["notdir"] = str(tmp_path / "hello" / "x")
    yield paths, files
    locked.chmod(0o600)


def _check_oracle(oracle_lib, names, res, files):
    out, sizes, st = res[0], res[1], res[2]
    for k, name in enumerate(names):
        if name in files:
            assert st[k] == 0, name
            lo, hi = oracle_lib.xxh3_128(files[name])
            assert out[k] == [lo, hi], name
            assert sizes[k] == len(files[name]), name


def test_single_files_match_the_engine(monkeypatch, ctx, oracle_lib, tree):
    paths, files = tree
    for name, p in paths.items():
        for text, utf8 in ((False, False), (True, False), (True, True)):
            eng, d, ndirect = _both(monkeypatch, ctx, lambda: _ex(ctx, [p], text=text, utf8=utf8))
            assert d == eng, (name, text, utf8)
            assert ndirect == (0 if name == "big" else 1), name
            _check_oracle(oracle_lib, [name], d, files)


def test_small_requests_match_the_engine(monkeypatch, ctx, oracle_lib, tree):
    paths, files = tree
    small = ["empty", "one", "hello", "k4", "text", "latin1", "m1", "adir"]
    cases = [
        (small, True),                                                  # 8 files, ~1.4 MiB: direct
        (["missing", "fifo", "notdir", "locked", "hello"], True),       # failures around one good file
        (["missing", "adir"], True),                                    # nothing to hash
        (small + ["fifo"], False),                                      # 9 files: the engine
        (["hello", "big"], False),                                      # 3 MiB: the engine
        (["m1", "m1", "k4"], False),                                    # > 2 MiB staged: the engine
    ]
    for names, direct in cases:
        ps = [paths[n] for n in names]
        eng, d, ndirect = _both(monkeypatch, ctx, lambda: _ex(ctx, ps))
        assert d == eng, names
        assert ndirect == int(direct), names
        _check_oracle(oracle_lib, names, d, files)


def test_caller_sizes(monkeypatch, ctx, oracle_lib, tree):
    """get_hash_given_metadata's sizes: right ones stay direct; a size that no longer matches the file
    (grown or shrunk since the caller's stat) hands the request to the engine, which re-reads it."""
    paths, files = tree
    names = ["hello", "k4", "text", "empty"]
    ps = [paths[n] for n in names]
    right = [len(files[n]) for n in names]
    grown = [4, 4096, right[2], 0]     # hello holds more than the caller saw
    shrunk = [6, 4096, right[2], 0]    # ... less
    for meta, direct in ((right, True), (grown, False), (shrunk, False), ([5, 4000, right[2], 0], False),
                         ([5, 4096, right[2], 9], False)):
        eng, d, ndirect = _both(monkeypatch, ctx, lambda: _ex(ctx, ps, meta=meta))
        assert d == eng, meta
        assert ndirect == int(direct), meta
        _check_oracle(oracle_lib, names, d, files)
    # a caller size at or above a staging slot is not used for the read: fstat's size decides
    eng, d, ndirect = _both(monkeypatch, ctx, lambda: _ex(ctx, [paths["hello"]], meta=[1 << 62]))
    assert d == eng and ndirect == 1
    _check_oracle(oracle_lib, ["hello"], d, files)


def test_fused_add_small(monkeypatch, ctx, oracle_lib, tree, tmp_path_factory):
    from oxen_amd import hasher

    paths, files = tree
    names = ["hello", "k4", "missing", "text", "hello", "empty"]
    ps = [paths[n] for n in names]
    roots = [str(tmp_path_factory.mktemp("versions_engine")), str(tmp_path_factory.mktemp("versions_direct"))]
    it = iter(roots)
    eng, d, ndirect = _both(monkeypatch, ctx, lambda: hasher.add_files(ps, next(it), ctx=ctx))
    assert d == eng and ndirect == 1
    digests, sizes, st, stored = d
    assert stored[0] and stored[1] and stored[3] and not stored[2]
    for root in roots:
        for name, dg, s in zip(names, digests, st):
            if name in files:
                assert s == 0 and dg == oracle_lib.xxh3_128_int(files[name])
                with open(hasher.version_path(root, dg), "rb") as f:
                    assert f.read() == files[name]


def test_direct_beside_engine_runs(monkeypatch, ctx, oracle_lib, tmp_path):
    """Single-file calls from 8 threads while another thread runs 2 000-file requests on the same
    context: every answer against the oracle, and both forms seen."""
    from oxen_amd import hasher

    monkeypatch.setenv("OXH_DIRECT_FILES", "1")
    rng = np.random.default_rng(62)
    blobs = [rng.integers(0, 256, int(rng.integers(0, 20_000)), dtype=np.uint8).tobytes() for _ in range(2000)]
    paths = []
    for i, b in enumerate(blobs):
        p = tmp_path / f"f{i}"
        p.write_bytes(b)
        paths.append(str(p))
    want = [oracle_lib.xxh3_128_int(b) for b in blobs]
    c0 = ctx.counters()
    errors = []

    batches_done = threading.Event()

    def singles(t):
        # during the batch requests (joining their runs, or direct between them), then after them
        # (direct once the last run has closed)
        try:
            r = np.random.default_rng(100 + t)
            calls = 0
            while calls < 150 or not batches_done.is_set():
                calls += 1
                k = int(r.integers(0, len(paths)))
                d, sizes, st, _ = hasher.hash_files_with_errors_128bit([paths[k]], ctx=ctx)
                if st != [0] or d != [want[k]] or sizes != [len(blobs[k])]:
                    errors.append((t, k, d, st))
            time.sleep(0.05)
            for k in range(t, len(paths), 200):
                d, sizes, st, _ = hasher.hash_files_with_errors_128bit([paths[k]], ctx=ctx)
                if st != [0] or d != [want[k]] or sizes != [len(blobs[k])]:
                    errors.append((t, k, d, st))
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append((t, repr(e)))

    def batches():
        try:
            for _ in range(3):
                d, _, st = hasher.hash_files_128bit(paths, ctx=ctx)
                if d != want or any(st):
                    errors.append(("batch", sum(a != b for a, b in zip(d, want))))
        except Exception as e:  # noqa: BLE001
            errors.append(("batch", repr(e)))
        finally:
            batches_done.set()

    threads = [threading.Thread(target=singles, args=(t,)) for t in range(8)] + [threading.Thread(target=batches)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=120)
    assert not any(th.is_alive() for th in threads), "a file call did not return"
    assert not errors, errors[:5]
    c1 = ctx.counters()
    assert c1["direct_requests"] > c0["direct_requests"] and c1["engine_runs"] > c0["engine_runs"]
