"""oxen_amd.procpool.ShardedFileHasher: the file list split over worker processes (packed paths in
shared memory, per-worker char* tables, outputs written in place). The pool mechanics are checked on
CPU with the oracle's restated reference loop in the workers; the GPU test runs the real engines."""
import os

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


def test_pool_mechanics_with_the_cpu_loop(tmp_path, oracle_lib):
    from oxen_amd.procpool import ShardedFileHasher

    paths = _tree(tmp_path)
    want_out, want_sizes, want_st = oracle_lib.hash_files(paths, threads=2)
    meta = [os.path.getsize(p) if os.path.exists(p) else 0 for p in paths]
    with ShardedFileHasher(procs=3, threads=2, mode="cpu") as pool:
        for m in (None, meta):
            out, sizes, st = pool.hash_files(paths, m)
            assert np.array_equal(out[:-1], want_out[:-1]) and st[-1] != 0 and (st[:-1] == 0).all()
            assert np.array_equal(sizes[:-1], want_sizes[:-1])
        out, sizes, st = pool.hash_files(paths[:2])  # fewer files than workers
        assert np.array_equal(out, want_out[:2])


@pytest.mark.gpu
def test_sharded_gpu_engines_match_oracle(cuda, tmp_path, oracle_lib):
    from oxen_amd.procpool import ShardedFileHasher

    paths = _tree(tmp_path, 2000)
    want_out, _, _ = oracle_lib.hash_files(paths, threads=4)
    meta = [os.path.getsize(p) if os.path.exists(p) else 0 for p in paths]
    with ShardedFileHasher(procs=2, threads=4, staging_bytes=8 << 20) as pool:
        for m in (None, meta):
            out, sizes, st = pool.hash_files(paths, m)
            assert (st[:-1] == 0).all() and st[-1] != 0
            assert np.array_equal(out[:-1], want_out[:-1]) and (out[-1] == 0).all()
