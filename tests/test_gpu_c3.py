"""BASELINE configs[2] (C3) in its real form: the image repo of benchmark/generate_image_repo.py
written to disk (images/split_{i % dirs}/noise_image_{i}.tiff + images.csv + README.md, TIFF
128x128x3 = 49 292 B) and run through the file engine -- oxh_hash_files, oxh_hash_files_meta,
the fused oxh_add_files and the reader-process pool -- against the oracle."""
import os
import shutil

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _u128(out):
    return [(int(h) << 64) | int(l) for l, h in out]


def test_c3_reduced_image_repo(ctx, oracle_lib, tmp_path):
    """5 000 TIFFs in 50 dirs: every digest of every engine entry point bit-exact vs the oracle; the
    fused add publishes every blob at its version path with the file's bytes."""
    from oxen_amd import hasher
    from oxen_amd.procpool import ShardedFileHasher
    from oxen_amd.workloads import write_image_repo_fast

    paths = write_image_repo_fast(str(tmp_path / "repo"), 5000, num_dirs=50)
    assert len(paths) == 5002 and os.path.getsize(paths[0]) == 49_292
    want_out, want_sizes, want_st = oracle_lib.hash_files(paths, threads=8)
    assert (want_st == 0).all()
    want = _u128(want_out)
    assert len(set(want)) == len(want)

    d, sizes, st = hasher.hash_files_128bit(paths, ctx)
    assert st == [0] * len(paths) and d == want and sizes == [int(s) for s in want_sizes]
    d, sizes, st = hasher.hash_files_given_metadata_128bit(paths, [int(s) for s in want_sizes], ctx)
    assert st == [0] * len(paths) and d == want

    root = str(tmp_path / "versions")
    d, sizes, st, stored = hasher.add_files(paths, root, ctx)
    assert st == [0] * len(paths) and d == want and all(stored)
    for i in range(0, len(paths), 499):
        with open(hasher.version_path(root, want[i]), "rb") as f, open(paths[i], "rb") as g:
            assert f.read() == g.read()
    # again: every blob already in the store, nothing rewritten
    d, _, st, stored = hasher.add_files(paths, root, ctx)
    assert d == want and not any(stored)

    with ShardedFileHasher(procs=2, threads=4) as pool:
        out, _, st = pool.hash_files(paths, [int(s) for s in want_sizes])
        assert (st == 0).all() and np.array_equal(out, want_out)


def test_c3_full_image_repo(cuda, oracle_lib, tmp_path):
    """The full 200 002-file C3 tree (9.87 GB) through the engine, one process and the 2-process
    pool: every status OK, both agree, no two images collide, and a 1 000-file sample plus
    images.csv / README.md equal the oracle."""
    from oxen_amd import _capi
    from oxen_amd.procpool import ShardedFileHasher, pack_paths
    from oxen_amd.workloads import write_image_repo_fast

    root = str(tmp_path / "c3")
    try:
        paths = write_image_repo_fast(root, 200_000)
        assert len(paths) == 200_002
        blob, offs = pack_paths(paths)
        with _capi.Context(0) as c:
            import ctypes

            n = len(paths)
            arr = (ctypes.c_char_p * n)(*[os.fsencode(p) for p in paths])
            out = np.zeros((n, 2), dtype=np.uint64)
            sizes = np.zeros(n, dtype=np.uint64)
            st = np.zeros(n, dtype=np.int32)
            _capi.check(_capi.lib().oxh_hash_files(c.handle, arr, n, out.ctypes.data_as(_capi._u64p),
                                                   sizes.ctypes.data_as(_capi._u64p), st.ctypes.data_as(_capi._i32p)),
                        "oxh_hash_files")
        assert (st == 0).all()
        assert (sizes[:-2] == 49_292).all() and int(sizes.sum()) > 9_800_000_000
        with ShardedFileHasher(procs=2) as pool:
            pout, psizes, pst = pool.hash_files_packed(blob, offs, sizes)
        assert (pst == 0).all() and np.array_equal(pout, out) and np.array_equal(psizes, sizes)
        assert len({(int(a), int(b)) for a, b in out}) == n  # no collisions
        idx = list(np.random.default_rng(3).choice(n - 2, 1000, replace=False)) + [n - 2, n - 1]
        wout, _, wst = oracle_lib.hash_files([paths[i] for i in idx], threads=8)
        assert (wst == 0).all() and np.array_equal(wout, out[idx])
    finally:
        shutil.rmtree(root, ignore_errors=True)
