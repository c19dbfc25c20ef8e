"""The C ABI's reader-process pool (oxh_pool_*, oxen_amd/csrc/reader_pool.cpp + oxh_hash_helper) and its
Python mirror oxen_amd.procpool.ShardedFileHasher: the file list split over helper processes, each
with its own context (device p % ndevices), paths and outputs in one shared region."""
import os
import signal

import numpy as np
import pytest


def _tree(tmp_path, n=300):
    rng = np.random.default_rng(5)
    paths = []
    for i in range(n):
        d = tmp_path / f"split_{i % 7}"
        d.mkdir(exist_ok=True)
        p = d / f"f{i}.bin"
        p.write_bytes(rng.integers(0, 256, int(rng.integers(0, 70_000)), dtype=np.uint8).tobytes())
        paths.append(str(p))
    paths.append(str(tmp_path / "missing.bin"))
    return paths


def test_pack_paths_roundtrip():
    from oxen_amd.procpool import pack_paths

    ps = ["/a/b", "x", "/dir with space/ü.txt", ""]
    blob, offs = pack_paths(ps)
    b = blob.tobytes()
    assert [b[o:b.index(b"\0", o)].decode() for o in offs.tolist()] == ps


def test_pool_helper_is_built(built_lib):
    from oxen_amd import build

    assert os.access(build.HELPER, os.X_OK)


def test_pool_fails_loudly_without_a_gpu(built_lib):
    """On a host without a gfx950 device every helper reports OXH_ERR_NODEVICE and creation fails with
    it (no CPU fallback); the helpers are reaped."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    from oxen_amd import _capi
    from oxen_amd.procpool import ShardedFileHasher

    with pytest.raises(_capi.OxenError) as e:
        ShardedFileHasher(procs=2)
    assert e.value.code == _capi.OXH_ERR_NODEVICE, str(e.value)


@pytest.fixture
def fake_helper(built_lib, monkeypatch):
    """The pool's mechanics on any host: OXH_HELPER points at tests/native/fake_pool_helper (the same
    wire protocol, no GPU; its "digest" is (size, the file's index in the call))."""
    from oxen_amd import build

    build.build_host()
    monkeypatch.setenv("OXH_HELPER", build.FAKE_HELPER)
    return build.FAKE_HELPER


def _fake_want(paths, meta):
    sizes = [os.path.getsize(p) if os.path.isfile(p) else None for p in paths]
    out = np.array([[s or 0, (i + (1 << 40 if meta else 0)) if s is not None else 0] for i, s in enumerate(sizes)],
                   dtype=np.uint64).reshape(-1, 2)
    return out, np.array([s or 0 for s in sizes], dtype=np.uint64), np.array([0 if s is not None else 7 for s in sizes], dtype=np.int32)


@pytest.mark.parametrize("procs,devices", [(1, (0,)), (3, (0, 1)), (4, (2, 3, 5))])
def test_pool_mechanics_with_a_fake_helper(fake_helper, tmp_path, procs, devices):
    """Every item lands in its own slot whatever the split; meta sizes reach the helpers; the shared
    region grows between calls (helpers re-map it); empty calls and fewer files than helpers."""
    from oxen_amd.procpool import ShardedFileHasher

    paths = _tree(tmp_path, 300)
    meta = [os.path.getsize(p) if os.path.exists(p) else 0 for p in paths]
    with ShardedFileHasher(procs=procs, devices=devices, threads=2) as pool:
        assert len(set(pool.pids())) == procs
        for m in (None, meta):
            got = pool.hash_files(paths, m)
            for g, w in zip(got, _fake_want(paths, m is not None)):
                assert np.array_equal(g, w)
        big = paths * 40  # ~12 000 paths: a larger region
        got = pool.hash_files(big)
        for g, w in zip(got, _fake_want(big, False)):
            assert np.array_equal(g, w)
        assert pool.hash_files(paths[:1])[0][0, 0] == os.path.getsize(paths[0])
        assert pool.hash_files([])[0].shape == (0, 2)


def test_pool_fake_helper_concurrency_and_death(fake_helper, tmp_path):
    """Concurrent callers serialise and each gets its own answers; a killed helper fails the call
    and every later one; a helper that fails at start-up fails creation with its status."""
    import signal
    from concurrent.futures import ThreadPoolExecutor

    from oxen_amd import _capi
    from oxen_amd.procpool import ShardedFileHasher

    paths = _tree(tmp_path, 200)
    with ShardedFileHasher(procs=3, threads=2) as pool:
        lists = [paths[k::4] for k in range(4)]

        def call(ps):
            got = pool.hash_files(ps)
            return all(np.array_equal(g, w) for g, w in zip(got, _fake_want(ps, False)))

        with ThreadPoolExecutor(4) as ex:
            assert all(ex.map(call, lists * 5))
        os.kill(pool.pids()[2], signal.SIGKILL)
        with pytest.raises(_capi.OxenError):
            pool.hash_files(paths)
        with pytest.raises(_capi.OxenError, match="unusable"):
            pool.hash_files(paths)
    os.environ["OXH_FAKE_FAIL_DEVICE"] = "1"
    try:
        with pytest.raises(_capi.OxenError) as e:
            ShardedFileHasher(procs=2, devices=(0, 1))
        assert e.value.code == _capi.OXH_ERR_NODEVICE and "no device" in str(e.value)
    finally:
        del os.environ["OXH_FAKE_FAIL_DEVICE"]


def test_pool_created_on_a_thread_that_exits(fake_helper, tmp_path):
    """a pool created on a short-lived thread (a tokio spawn_blocking worker, a Python
    worker thread) keeps its helpers after that thread exits: the helpers watch their socket and
    their parent PROCESS, not the creating thread (PR_SET_PDEATHSIG would have killed them)."""
    import threading
    import time

    from oxen_amd.procpool import ShardedFileHasher

    paths = _tree(tmp_path, 50)
    box = {}
    t = threading.Thread(target=lambda: box.setdefault("pool", ShardedFileHasher(procs=2, threads=1)))
    t.start()
    t.join()
    pool = box["pool"]
    try:
        time.sleep(1.5)  # a helper killed by its creator thread's exit would be gone by now
        for pid in pool.pids():
            os.kill(pid, 0)  # still alive
        got = pool.hash_files(paths)
        for g, w in zip(got, _fake_want(paths, False)):
            assert np.array_equal(g, w)
    finally:
        pool.close()


def test_pool_reports_open_and_read_errors(fake_helper, tmp_path):
    """oxh_pool_hash_files_ex carries each failure's errno across the process boundary: a missing path
    is an open failure (OXH_ERR_OPEN, ENOENT), a directory a read failure (OXH_ERR_IO, EISDIR)."""
    import errno

    from oxen_amd import _capi
    from oxen_amd.procpool import ShardedFileHasher

    f = tmp_path / "ok.bin"
    f.write_bytes(b"x" * 10)
    (tmp_path / "adir").mkdir()
    paths = [str(f), str(tmp_path / "nope"), str(tmp_path / "adir")]
    with ShardedFileHasher(procs=2, threads=1) as pool:
        out, sizes, status, oserr = pool.hash_files(paths, with_errors=True)
    assert status.tolist() == [0, _capi.OXH_ERR_OPEN, _capi.OXH_ERR_IO]
    assert oserr.tolist() == [0, errno.ENOENT, errno.EISDIR]


def test_pool_call_deadline(fake_helper, tmp_path, monkeypatch):
    """a helper that stops answering no longer hangs the caller forever when a deadline is
    set (OXH_POOL_CALL_LIMIT_S): the call fails with OXH_ERR_HIP and the pool is marked unusable."""
    import time

    from oxen_amd import _capi
    from oxen_amd.procpool import ShardedFileHasher

    paths = _tree(tmp_path, 20)
    monkeypatch.setenv("OXH_FAKE_STALL_S", "30")
    monkeypatch.setenv("OXH_POOL_CALL_LIMIT_S", "2")
    with ShardedFileHasher(procs=1, threads=1) as pool:
        t0 = time.monotonic()
        with pytest.raises(_capi.OxenError) as e:
            pool.hash_files(paths)
        assert e.value.code == _capi.OXH_ERR_HIP
        assert time.monotonic() - t0 < 15
        with pytest.raises(_capi.OxenError, match="unusable"):
            pool.hash_files(paths)


def test_pool_rejects_bad_arguments(built_lib, monkeypatch):
    from oxen_amd import _capi
    from oxen_amd.procpool import ShardedFileHasher

    with pytest.raises(_capi.OxenError):
        ShardedFileHasher(procs=0)
    monkeypatch.setenv("OXH_HELPER", "/nonexistent/oxh_hash_helper")
    with pytest.raises(_capi.OxenError) as e:
        ShardedFileHasher(procs=1)
    assert "helper not found" in str(e.value)


@pytest.mark.gpu
@pytest.mark.parametrize("procs,devices", [(2, (0,)), (3, (0, 0))])
def test_sharded_gpu_engines_match_oracle(cuda, tmp_path, oracle_lib, procs, devices):
    from oxen_amd.procpool import ShardedFileHasher

    paths = _tree(tmp_path, 2000)
    want_out, want_sizes, _ = oracle_lib.hash_files(paths, threads=4)
    meta = [os.path.getsize(p) if os.path.exists(p) else 0 for p in paths]
    with ShardedFileHasher(procs=procs, devices=devices, threads=4, staging_bytes=8 << 20) as pool:
        pids = pool.pids()
        assert len(set(pids)) == procs and os.getpid() not in pids
        for m in (None, meta):
            out, sizes, st = pool.hash_files(paths, m)
            assert (st[:-1] == 0).all() and st[-1] != 0
            assert np.array_equal(out[:-1], want_out[:-1]) and (out[-1] == 0).all()
            assert np.array_equal(sizes[:-1], want_sizes[:-1])
        out, _, st = pool.hash_files(paths[:1])  # fewer files than helpers
        assert np.array_equal(out, want_out[:1]) and st[0] == 0
        out, _, _ = pool.hash_files(paths * 3)  # the shared region grows (helpers re-map it)
        assert np.array_equal(out[:-1][: len(paths) - 1], want_out[:-1])
        assert np.array_equal(out[2 * len(paths):2 * len(paths) + len(paths) - 1], want_out[:-1])
        assert pool.hash_files([])[0].shape == (0, 2)


@pytest.mark.gpu
def test_pool_concurrent_callers(cuda, tmp_path, oracle_lib):
    """Several threads share one pool (liboxen's tokio tasks holding one process-wide pool): calls
    serialise inside the library and each gets its own list's digests."""
    from concurrent.futures import ThreadPoolExecutor

    from oxen_amd.procpool import ShardedFileHasher

    paths = _tree(tmp_path, 600)[:-1]
    want, _, _ = oracle_lib.hash_files(paths, threads=4)
    lists = [list(range(k, len(paths), 5)) for k in range(5)]
    with ShardedFileHasher(procs=2, threads=4, staging_bytes=8 << 20) as pool:
        def call(idx):
            out, _, st = pool.hash_files([paths[i] for i in idx])
            return (st == 0).all() and np.array_equal(out, want[idx])

        with ThreadPoolExecutor(5) as ex:
            assert all(ex.map(call, lists * 3))


@pytest.mark.gpu
def test_pool_helper_death_breaks_the_pool(cuda, tmp_path):
    """A helper that dies fails the call and every later one (no stale replies, no partial outputs)."""
    from oxen_amd import _capi
    from oxen_amd.procpool import ShardedFileHasher

    paths = _tree(tmp_path, 50)
    pool = ShardedFileHasher(procs=2, threads=2, staging_bytes=8 << 20)
    try:
        pool.hash_files(paths)
        os.kill(pool.pids()[1], signal.SIGKILL)
        with pytest.raises(_capi.OxenError):
            pool.hash_files(paths)
        with pytest.raises(_capi.OxenError) as e:
            pool.hash_files(paths)
        assert "unusable" in str(e.value)
    finally:
        pool.close()
