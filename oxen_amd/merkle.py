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
from dataclasses import dataclass
from typing import Iterable, Optional, Sequence

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
