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
