"""Synthetic staged commits for the K2 commit-driver tests (shape of benchmark/generate_image_repo.py:
images/split_{i % n_dirs}/img_{i}.tiff + a couple of top-level files)."""
import numpy as np


def staged_commit(n_files=300, n_dirs=7, seed=3, second=False):
    """Returns (entries, existing) as {dir: [(path, hash, is_dir, status, name)]}.

    First commit: everything "added", no existing tree. second=True: a follow-up commit against the
    first one's tree -- some files modified, some removed, one added, one staged with a leaf-only
    path (exercises the defensive prefixing), the rest unmodified children of HEAD."""
    rng = np.random.default_rng(seed)
    rand = lambda: int(rng.integers(0, 2**63)) << 65 | int(rng.integers(0, 2**63))
    dirs = [f"images/split_{d}" for d in range(n_dirs)]
    files = {d: [] for d in dirs}
    for i in range(n_files):
        d = dirs[i % n_dirs]
        p = f"{d}/img_{i}.tiff"
        files[d].append((p, rand(), False, "added", p))
    top = [("README.md", rand(), False, "added", "README.md"), ("images.csv", rand(), False, "added", "images.csv")]
    dir_nodes = [(d, rand(), True, "added", d) for d in dirs]
    entries = {"": top + [("images", rand(), True, "added", "images")], "images": dir_nodes}
    entries.update(files)
    if not second:
        return entries, {}
    existing = {k: [(p, h, isd, "unmodified", nm) for (p, h, isd, _, nm) in v] for k, v in entries.items()}
    new = {}
    d0, d1 = dirs[0], dirs[1 % n_dirs]
    f0 = existing[d0]
    new[d0] = [(f0[0][0], rand(), False, "modified", f0[0][0]), (f0[1][0], f0[1][1], False, "removed", f0[1][0]),
               (f"{d0}/new.tiff", rand(), False, "added", f"{d0}/new.tiff")]
    new[d1] = [("leaf_only.tiff", rand(), False, "added", "leaf_only.tiff")]
    new["images"] = [(d0, rand(), True, "modified", d0), (d1, rand(), True, "modified", d1)]
    new[""] = [("images", rand(), True, "modified", "images")]
    return new, existing


def salt(directory, j):
    """Deterministic stand-in for Uuid::new_v4() (an input of the hash, F8)."""
    return (directory + "#" + str(j)).encode().ljust(16, b"\0")[:16]


def to_staged(entries):
    from oxen_amd.merkle import StagedNode

    return {k: [StagedNode(path=p, hash=h, is_dir=isd, status=st, name=nm) for (p, h, isd, st, nm) in v]
            for k, v in entries.items()}


def to_cli_input(entries, existing, vnode_size=10_000) -> str:
    """The staged commit as tests/native/commit_tree_cli reads it (entries in dict order)."""
    lines = [f"vnode_size\t{vnode_size}"]

    def nodes(v):
        for (p, h, isd, st, nm) in v:
            lines.append(f"node\t{p}\t{h:x}\t{int(isd)}\t{st}\t{nm if nm is not None else chr(1)}")

    for d, v in entries.items():
        lines.append(f"entries\t{d}")
        nodes(v)
    for d, v in (existing or {}).items():
        lines.append(f"existing\t{d}")
        nodes(v)
    return "\n".join(lines) + "\n"


def parse_cli_output(text: str):
    """({dir: [(vnode_id, [entry paths])]}, {dir: hash}, {dir: [removed paths]}, best seconds)."""
    vn, dh, removed, t = {}, {}, {}, None
    for line in text.splitlines():
        f = line.split("\t")
        if f[0] == "vnode":
            vn.setdefault(f[1], []).append((int(f[3], 16), f[5:5 + int(f[4])]))
        elif f[0] == "removed":
            removed.setdefault(f[1], []).append(f[2])
        elif f[0] == "dir":
            dh[f[1]] = int(f[2], 16)
        elif f[0] == "time":
            t = float(f[1])
    return vn, dh, removed, t
