"""Merkle digest type and parent-node byte streams (K2) for the commit path.

* `MerkleHash` mirrors model/merkle_tree/merkle_hash.rs: a u128, `Display` = unpadded lowercase hex
  (:73-77), `FromStr` radix-16 (:54-61), `to_le_bytes` (:25-27), `node_db_prefix` 3/29 split
  (:125-131); `version_dir` is the version-store 2/.. split (storage/local.rs:66-75).
* The stream builders serialise exactly the bytes commit_writer.rs feeds to `Xxh3::update`
  (vnode ids :686-720, dir hashes :995-1147, commit id :757-766), so that one batched GPU pass
  (`hash_streams_128bit`) produces every parent digest of a commit. Which children, in which order,
  and whether a vnode gets a UUID salt is the caller's decision (the reference iterates a
  HashMap and salts with a random UUID, so parent digests are not reproducible run to run; parity is
  "same bytes in -> same digest as the CPU XXH3-128").
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field, replace
from typing import Callable, Iterable, Optional, Sequence

import numpy as np

from . import hasher


@dataclass(frozen=True, order=True)
class MerkleHash:
    value: int

    def __post_init__(self):
        if not (0 <= self.value < 1 << 128):
            raise ValueError("MerkleHash is a u128")

    @classmethod
    def from_str(cls, s: str) -> "MerkleHash":
        return cls(int(s, 16))

    def __str__(self) -> str:
        return format(self.value, "x")

    def to_u128(self) -> int:
        return self.value

    def to_le_bytes(self) -> bytes:
        return self.value.to_bytes(16, "little")

    def to_short_str(self) -> str:
        return str(self)[:10]

    def node_db_prefix(self) -> str:
        s = str(self)
        return f"{s[:3]}/{s[3:]}"

    def version_dir(self) -> str:
        s = str(self)
        return f"{s[:2]}/{s[2:]}"


def num_vnodes(total_children: int, vnode_size: int) -> int:
    """commit_writer.rs:660: `(total_children as f32 / vnode_size as f32).ceil() as u128`."""
    return int(math.ceil(float(np.float32(total_children) / np.float32(vnode_size))))


def vnode_buckets(paths: Sequence[str], n_vnodes: int) -> list[int]:
    """commit_writer.rs:673-681 / commit_merkle_tree.rs:813-814: xxh3_128(path bytes) % num_vnodes,
    for all paths in one batched GPU pass."""
    if n_vnodes <= 0:
        raise ValueError("num_vnodes must be positive")
    digests = hasher.hash_streams_128bit([p.encode("utf-8") for p in paths])
    return [d % n_vnodes for d in digests]


def vnode_stream(directory: str, child_hashes: Iterable[int], uuid_salt: Optional[bytes] = None) -> bytes:
    """commit_writer.rs:697-718: "vnode" || dir || for each child (sorted by path):
    combined_hash (files) or hash (dirs) as u128 LE || [uuid bytes if the dir existed and changed]."""
    parts = [b"vnode", directory.encode("utf-8")]
    parts += [int(h).to_bytes(16, "little") for h in child_hashes]
    if uuid_salt is not None:
        if len(uuid_salt) != 16:
            raise ValueError("uuid salt is 16 bytes")
        parts.append(bytes(uuid_salt))
    return b"".join(parts)


def dir_stream(path: str, vnodes: Iterable[tuple[int, Iterable[tuple[str, int]]]]) -> bytes:
    """commit_writer.rs:1003-1147: "dir" || path || for each (child dir, vnode) in caller order:
    vnode.id LE || for each entry: name || (dir.hash | file.combined_hash) LE."""
    parts = [b"dir", path.encode("utf-8")]
    for vnode_id, entries in vnodes:
        parts.append(int(vnode_id).to_bytes(16, "little"))
        for name, h in entries:
            parts.append(name.encode("utf-8"))
            parts.append(int(h).to_bytes(16, "little"))
    return b"".join(parts)


def commit_stream(parent_ids: Sequence[str], message: str, author: str, email: str, unix_timestamp: int) -> bytes:
    """commit_writer.rs:757-766: "commit" || format!("{:?}", parent_ids) || message || author ||
    email || unix_timestamp (i64) LE."""
    debug = "[" + ", ".join('"' + p.replace("\\", "\\\\").replace('"', '\\"') + '"' for p in parent_ids) + "]"
    return (b"commit" + debug.encode() + message.encode() + author.encode() + email.encode()
            + int(unix_timestamp).to_bytes(8, "little", signed=True))


def hash_parents(streams: Sequence[bytes]) -> list[MerkleHash]:
    """K2: every parent digest of a commit in one batched GPU pass."""
    return [MerkleHash(d) for d in hasher.hash_streams_128bit(list(streams))]


# ------------------------------------------------------------------------------ K2 commit driver
# One commit's parent digests in three batched GPU passes (bucket hashes, vnode ids, dir hashes),
# restating commit_writer.rs:544-755 (split_into_vnodes) and :995-1165 (compute_dir_node). The two
# levels do not chain: a vnode hashes its entries' staged hashes, and a dir hashes its descendants'
# vnode ids plus the staged dir hashes (dir_node.hash(), not the recomputed ones -- the reference's
# bottom-up update is a TODO at :722), so every dir of the commit is independent of every other.

STATUSES = ("added", "modified", "removed", "unmodified")


@dataclass(frozen=True)
class StagedNode:
    """A StagedMerkleTreeNode as the commit writer sees it (model/merkle_tree/node/staged...):
    `path` is maybe_path() (repo-relative), `hash` is what both parent streams take from it --
    file_node.combined_hash() for files, node.hash for dirs -- and `name` is the node name the dir
    stream uses (file_node.name() / dir_node.name(); staged nodes carry the full relative path)."""

    path: str
    hash: int
    is_dir: bool = False
    status: str = "added"
    name: Optional[str] = None

    def node_name(self) -> str:
        return self.path if self.name is None else self.name


@dataclass
class EntryVNode:
    """commit_writer.rs EntryVNode: a vnode id and its entries sorted by path."""

    id: MerkleHash
    entries: list = field(default_factory=list)


def path_components(p: str) -> tuple:
    """std::path::Path::components for a relative unix path (empty and "." parts dropped), the key
    Path's Ord and starts_with compare by."""
    return tuple(c for c in p.split("/") if c not in ("", "."))


def _path_starts_with(p: tuple, base: tuple) -> bool:
    return p[: len(base)] == base


def _uuid4_bytes(directory: str, vnode_index: int) -> bytes:
    """uuid::Uuid::new_v4().as_bytes(): 16 random bytes with the version/variant bits set."""
    b = bytearray(os.urandom(16))
    b[6] = (b[6] & 0x0F) | 0x40
    b[8] = (b[8] & 0x3F) | 0x80
    return bytes(b)


def split_into_vnodes(entries: dict, existing: Optional[dict] = None, vnode_size: int = 10_000,
                      uuid_salt: Callable[[str, int], bytes] = _uuid4_bytes, ctx=None) -> dict:
    """commit_writer.rs:544-755. entries: {directory: [StagedNode]} (the staged changes),
    existing: {directory: [StagedNode]} (children of that dir in HEAD's tree, status "unmodified").
    Returns {directory: ([EntryVNode], [removed StagedNode])}. All bucket hashes of all dirs are one
    GPU batch, and so are all vnode ids. uuid_salt(dir, vnode_index) gives the 16 salt bytes the
    reference takes from Uuid::new_v4() for a changed vnode of a dir that existed (:713-716)."""
    existing = existing or {}
    per_dir = []
    for directory, new_children in entries.items():
        dkey = path_components(directory)
        children = {}
        for c in existing.get(directory, ()):
            children[path_components(c.path)] = c
        removed = {}
        for c in new_children:
            ckey = path_components(c.path)
            if not ckey:  # child_path != "" (:589)
                continue
            if dkey and not _path_starts_with(ckey, dkey):  # defensive prefixing (:591-612)
                full = "/".join(dkey + ckey)
                c = replace(c, path=full, name=full)
                ckey = path_components(full)
            if c.status == "removed":
                children.pop(ckey, None)
                removed[ckey] = c
            else:
                children[ckey] = c
        per_dir.append((directory, children, list(removed.values())))

    # bucket = xxh3_128(path) % num_vnodes (:665-681), every child of every dir in one pass
    all_children = [(i, k, c) for i, (_, ch, _) in enumerate(per_dir) for k, c in ch.items()]
    digests = hasher.hash_streams_128bit([c.path.encode("utf-8") for _, _, c in all_children], ctx)
    vnodes_of = [[EntryVNode(MerkleHash(0)) for _ in range(num_vnodes(len(ch), vnode_size))] if ch else []
                 for _, ch, _ in per_dir]
    for (i, k, c), d in zip(all_children, digests):
        vnodes_of[i][d % len(vnodes_of[i])].entries.append((k, c))

    # vnode id = xxh3("vnode" || dir || child hashes LE [|| uuid]) (:683-720), all vnodes in one pass
    streams, where = [], []
    for i, (directory, _, _) in enumerate(per_dir):
        for j, vn in enumerate(vnodes_of[i]):
            vn.entries.sort(key=lambda kc: kc[0])
            vn.entries = [c for _, c in vn.entries]
            changed = any(c.status != "unmodified" for c in vn.entries)
            salt = uuid_salt(directory, j) if (directory in existing and changed) else None
            streams.append(vnode_stream(directory, (c.hash for c in vn.entries), salt))
            where.append((i, j))
    for (i, j), d in zip(where, hasher.hash_streams_128bit(streams, ctx)):
        vnodes_of[i][j].id = MerkleHash(d)
    return {directory: (vnodes_of[i], removed) for i, (directory, _, removed) in enumerate(per_dir)}


def _vnode_segment(vn: EntryVNode) -> bytes:
    """What compute_dir_node feeds for one vnode (:1042-1071): id LE, then name || hash LE per entry."""
    parts = [vn.id.value.to_bytes(16, "little")]
    for c in vn.entries:
        parts.append(c.node_name().encode("utf-8"))
        parts.append(int(c.hash).to_bytes(16, "little"))
    return b"".join(parts)


def compute_dir_hashes(vnodes: dict, dirs: Optional[Iterable[str]] = None, ctx=None) -> dict:
    """compute_dir_node's hash (commit_writer.rs:995-1165) for `dirs` (default: "" and every key of
    `vnodes`), all in one GPU batch. A dir's stream covers every key of `vnodes` that starts_with it,
    component-wise, in the mapping's iteration order (get_children :979-993 -- a HashMap in the
    reference, so the order is the caller's)."""
    keys = list(vnodes.keys())
    if dirs is None:
        dirs = [""] + [k for k in keys if path_components(k)]
    dirs = list(dirs)
    segs = {k: b"".join(_vnode_segment(vn) for vn in vnodes[k][0]) for k in keys}
    # descendants by ancestor prefix: O(keys x depth) instead of O(dirs x keys)
    under = {}
    for k in keys:
        comps = path_components(k)
        for d in range(len(comps) + 1):
            under.setdefault(comps[:d], []).append(k)
    streams = []
    for d in dirs:
        body = b"".join(segs[k] for k in under.get(path_components(d), ()))
        streams.append(b"dir" + d.encode("utf-8") + body)
    return {d: MerkleHash(h) for d, h in zip(dirs, hasher.hash_streams_128bit(streams, ctx))}


def commit_tree(entries: dict, existing: Optional[dict] = None, vnode_size: int = 10_000,
                uuid_salt: Callable[[str, int], bytes] = _uuid4_bytes, ctx=None):
    """Every parent digest of one commit: (vnodes per dir, dir hashes incl. the root "")."""
    vn = split_into_vnodes(entries, existing, vnode_size, uuid_salt, ctx)
    return vn, compute_dir_hashes(vn, None, ctx)
