"""The reference's commit-writer tree-shape tests (repositories/commits/commit_writer.rs:1234-1319
test_first_commit, :1560-1636 test_commit_configurable_vnode_size, :1639-1703
test_commit_20_files_6_vnode_size) restated over the GPU commit driver (oxen_amd.merkle.commit_tree:
bucket hashes, vnode ids and dir hashes computed by K1/K1s). The repo is the reference's
add_n_files_m_dirs (test.rs:203-250): README.md, files.csv and files/dir_{i % m}/file{i}.txt with
"File {i}". Node hashes are the files' content digests (the shape and which vnodes change depend
only on the paths' bucket hashes and the entries' statuses)."""
import pytest

pytestmark = pytest.mark.gpu


def _staged(n_files, n_dirs, ctx, extra=()):
    from oxen_amd import hasher
    from oxen_amd.merkle import StagedNode

    files = [(f"files/dir_{i % n_dirs}/file{i}.txt", f"File {i}".encode()) for i in range(n_files)]
    csv = b"file,label\n" + b"".join(f"file{i}.txt,{'cat' if i % 2 == 0 else 'dog'}\n".encode() for i in range(n_files))
    top = [("README.md", f"Repo with {n_files} files".encode()), ("files.csv", csv)]
    digests = hasher.hash_buffers_128bit([b for _, b in top + files + list(extra)], ctx)
    h = dict(zip([p for p, _ in top + files + list(extra)], digests))
    dirs = sorted({f"files/dir_{i % n_dirs}" for i in range(n_files)})
    entries = {"": [StagedNode(p, h[p], False, "added", p) for p, _ in top] + [StagedNode("files", 1, True, "added", "files")],
               "files": [StagedNode(d, 2 + k, True, "added", d) for k, d in enumerate(dirs)]}
    for p, _ in files:
        entries.setdefault(p.rsplit("/", 1)[0], []).append(StagedNode(p, h[p], False, "added", p))
    return entries, h


def _as_existing(entries):
    from dataclasses import replace

    return {k: [replace(c, status="unmodified") for c in v] for k, v in entries.items()}


def test_first_commit_vnodes(ctx):
    """commit_writer.rs:1234-1319: 10 files in 2 dirs -> 4 vnodes; the root's one vnode holds
    README.md, files.csv and files."""
    from oxen_amd import merkle

    entries, _ = _staged(10, 2, ctx)
    vn, dh = merkle.commit_tree(entries, None, 10_000, ctx=ctx)
    assert sum(len(v[0]) for v in vn.values()) == 4
    root = vn[""][0]
    assert len(root) == 1 and sorted(c.path for c in root[0].entries) == ["README.md", "files", "files.csv"]
    assert sorted(c.path for c in vn["files/dir_0"][0][0].entries) == [f"files/dir_0/file{i}.txt" for i in (0, 2, 4, 6, 8)]
    assert set(dh) == {"", "files", "files/dir_0", "files/dir_1"} and len(set(dh.values())) == 4


def test_commit_configurable_vnode_size(ctx):
    """commit_writer.rs:1560-1636: vnode size 5, 23 files in 2 dirs -> the root 1 vnode, each dir
    ceil(12 / 5) = ceil(11 / 5) = 3; then 10 new files (5 per dir) in a second commit, each found in
    its dir's vnodes."""
    from oxen_amd import merkle
    from oxen_amd.merkle import StagedNode

    entries, _ = _staged(23, 2, ctx)
    vn, _ = merkle.commit_tree(entries, None, 5, ctx=ctx)
    assert len(vn[""][0]) == 1 and len(vn["files/dir_0"][0]) == 3 and len(vn["files/dir_1"][0]) == 3
    existing = _as_existing(entries)
    new = {}
    for i in range(10):
        d = f"files/dir_{i % 2}"
        p = f"{d}/new_file_{i}.txt"
        new.setdefault(d, []).append(StagedNode(p, 1000 + i, False, "added", p))
    vn2, _ = merkle.commit_tree(new, existing, 5, uuid_salt=lambda d, j: bytes(16), ctx=ctx)
    for d in ("files/dir_0", "files/dir_1"):
        paths = {c.path for v in vn2[d][0] for c in v.entries}
        assert {f"{d}/new_file_{i}.txt" for i in range(10) if f"dir_{i % 2}" in d} <= paths
        assert len(paths) == (12 if d.endswith("0") else 11) + 5
        assert len(vn2[d][0]) == 4  # ceil(17 / 5) = ceil(16 / 5) = 4


def test_commit_20_files_6_vnode_size(ctx):
    """commit_writer.rs:1639-1703: vnode size 6, 20 files in 1 dir -> 4 vnodes; one new file -> still
    4 vnodes, and exactly 3 of them keep their id (the new path's bucket is the only vnode that
    changes: bucket = xxh3_128(path) % num_vnodes on the GPU)."""
    from oxen_amd import merkle
    from oxen_amd.merkle import StagedNode

    entries, _ = _staged(20, 1, ctx)
    vn, _ = merkle.commit_tree(entries, None, 6, ctx=ctx)
    assert len(vn[""][0]) == 1 and len(vn["files/dir_0"][0]) == 4
    first = {v.id.value for v in vn["files/dir_0"][0]}
    new = {"files/dir_0": [StagedNode("files/dir_0/new_file.txt", 77, False, "added", "files/dir_0/new_file.txt")]}
    vn2, _ = merkle.commit_tree(new, _as_existing(entries), 6, ctx=ctx)
    second = {v.id.value for v in vn2["files/dir_0"][0]}
    assert len(second) == 4 and len(first & second) == 3
