"""The C++ K2 commit driver (oxen_amd/host/commit_writer.cpp: split_into_vnodes + compute_dir_node of
commit_writer.rs over oxh_hash_streams) against the scalar restatement oracle/commit_oracle.py, driven
through tests/native/commit_tree_cli. Parity scope as for the Python driver: XXH3-128 is pinned;
HashMap order and the UUID salt are inputs."""
import os
import subprocess

import pytest

import _commit


@pytest.fixture(scope="module")
def cli(built_lib):
    from oxen_amd import build

    build.build_host()
    return build.COMMIT_CLI


def _run(cli, entries, existing, vnode_size, reps=1):
    r = subprocess.run([cli, "--reps", str(reps)], input=_commit.to_cli_input(entries, existing, vnode_size),
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    return _commit.parse_cli_output(r.stdout)


def test_commit_driver_exports(cli):
    from oxen_amd import build

    out = subprocess.run(["nm", "-DC", "--defined-only", build.HOST_LIB], capture_output=True, text=True, check=True).stdout
    for name in ["liboxen::commit_writer::split_into_vnodes", "liboxen::commit_writer::compute_dir_hashes",
                 "liboxen::commit_writer::commit_tree", "liboxen::commit_writer::num_vnodes"]:
        assert name in out, name
    assert os.access(cli, os.X_OK)


def test_commit_driver_refuses_without_a_gpu(cli):
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    entries, existing = _commit.staged_commit(n_files=20, n_dirs=3)
    r = subprocess.run([cli], input=_commit.to_cli_input(entries, existing), capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "oxh_ctx_create" in r.stderr  # no CPU fallback


def _check(got, entries, existing, vnode_size):
    from oracle import commit_oracle

    vn, dh, removed, _ = got
    rvn, rdh = commit_oracle.commit_tree(entries, existing, vnode_size, _commit.salt)
    assert set(vn) == {d for d in rvn if rvn[d]}
    for d in rvn:
        assert vn.get(d, []) == [(i, [n[0] for n in ns]) for i, ns in rvn[d]], d
    assert dh == rdh
    return vn, removed


@pytest.mark.gpu
@pytest.mark.parametrize("second", [False, True])
@pytest.mark.parametrize("vnode_size", [10_000, 7, 1])
def test_native_commit_driver(cuda, cli, second, vnode_size):
    entries, existing = _commit.staged_commit(n_files=500, n_dirs=9, second=second)
    vn, removed = _check(_run(cli, entries, existing, vnode_size), entries, existing, vnode_size)
    if second:  # the removed file of the follow-up commit is reported, and is in no vnode
        (d0, gone), = removed.items()
        assert all(gone[0] not in paths for _, paths in vn[d0])
    if vnode_size < 10_000:
        assert max(len(v) for v in vn.values()) > 1


@pytest.mark.gpu
def test_native_commit_driver_image_repo_shape(cuda, cli):
    """C3's tree: 200 000 files in 1 000 dirs."""
    entries, _ = _commit.staged_commit(n_files=200_000, n_dirs=1000)
    _check(_run(cli, entries, {}, 10_000), entries, {}, 10_000)


def _odd_paths_commit():
    """Paths the way a caller may hand them over: leading "./", doubled and trailing slashes, "."
    components, a child staged under a dir whose name prefixes a sibling's ("img" vs "img2"), the same
    path staged twice (the later one wins), and a removal that is re-added."""
    rand = iter(range(1, 10_000))
    h = lambda: (next(rand) * 0x9E3779B97F4A7C15) & ((1 << 128) - 1)
    entries = {
        "": [("README.md", h(), False, "added", "README.md"), ("./data", h(), True, "added", "data")],
        "data": [("data/img/", h(), True, "added", "data/img"), ("data//img2", h(), True, "added", "data/img2"),
                 ("data/./a.csv", h(), False, "added", "data/a.csv"), ("b.csv", h(), False, "added", "b.csv")],
        "data/img": [("data/img/x.png", h(), False, "added", "data/img/x.png"),
                     ("data/img/x.png", h(), False, "modified", "data/img/x.png"),
                     ("data/img/y.png", h(), False, "removed", "data/img/y.png"),
                     ("data/img/y.png", h(), False, "added", "data/img/y.png"),
                     ("z.png", h(), False, "added", "z.png")],
        "data/img2": [("data/img2/q.png", h(), False, "added", "data/img2/q.png")],
    }
    existing = {"data/img": [("data/img/old.png", h(), False, "unmodified", "data/img/old.png"),
                             ("data/img/gone.png", h(), False, "unmodified", "data/img/gone.png")]}
    entries["data/img"].append(("data/img/gone.png", h(), False, "removed", "data/img/gone.png"))
    return entries, existing


@pytest.mark.gpu
@pytest.mark.parametrize("vnode_size", [10_000, 2])
def test_native_commit_driver_odd_paths(cuda, cli, vnode_size):
    entries, existing = _odd_paths_commit()
    vn, removed = _check(_run(cli, entries, existing, vnode_size), entries, existing, vnode_size)
    assert "data/img" in removed


def test_odd_paths_python_driver_matches_oracle(monkeypatch, oracle_lib):
    """The same odd-path commit through the Python driver (hash calls answered by the oracle on the
    CPU): the reference point the native driver is held to above."""
    from oracle import commit_oracle
    from oxen_amd import hasher, merkle

    monkeypatch.setattr(hasher, "hash_streams_128bit", lambda s, ctx=None: [oracle_lib.xxh3_128_int(x) for x in s])
    entries, existing = _odd_paths_commit()
    for vnode_size in (10_000, 2):
        vn, dh = merkle.commit_tree(_commit.to_staged(entries), _commit.to_staged(existing), vnode_size, _commit.salt)
        rvn, rdh = commit_oracle.commit_tree(entries, existing, vnode_size, _commit.salt)
        for d in rvn:
            assert [v.id.value for v in vn[d][0]] == [i for i, _ in rvn[d]], d
        assert {d: x.value for d, x in dh.items()} == rdh
