"""TEST INFRASTRUCTURE ONLY -- scalar restatement of the commit writer's parent-node hashing.

Follows liboxen `repositories/commits/commit_writer.rs` statement by statement, feeding the bytes
the reference passes to `Xxh3::update` into one growing buffer and hashing it one-shot with the C
oracle (streaming == one-shot for XXH3, tests/test_oracle.py):
  * split_into_vnodes  :544-755  (child set :561-638, num_vnodes :657-660, bucket :669-681,
                                  sort :684-694, vnode id :696-720)
  * compute_dir_node   :995-1165 (get_children :979-993, hash stream :1001-1004, :1037-1071)
The staged nodes are plain tuples here (path, hash, is_dir, status, name) so this module shares no
code with oxen_amd.merkle. Only tests/ import it.

Parity scope: the reference pins none of these digests (its tests compare tree contents, not
values); what is pinned is XXH3-128 itself. HashMap order and the UUID salt are inputs (F8).
"""
from __future__ import annotations

import math
import struct

from . import oracle


def _xxh3(b: bytes) -> int:
    return oracle.xxh3_128_int(b)


def _components(p: str):
    return [c for c in p.split("/") if c not in ("", ".")]


def _f32(x: float) -> float:
    return struct.unpack("f", struct.pack("f", x))[0]


def split_into_vnodes(entries, existing, vnode_size, salt):
    """entries/existing: {dir: [(path, hash, is_dir, status, name)]}; salt(dir, j) -> 16 bytes.
    Returns {dir: [(vnode_id, [node, ...]), ...]}."""
    results = {}
    for directory, new_children in entries.items():
        children = {}
        for node in existing.get(directory, []):
            children[tuple(_components(node[0]))] = node
        for node in new_children:
            path, h, is_dir, status, name = node
            if not _components(path):
                continue
            d = _components(directory)
            if d and _components(path)[: len(d)] != d:
                full = "/".join(d + _components(path))
                node = (full, h, is_dir, status, full)
            key = tuple(_components(node[0]))
            if status == "removed":
                children.pop(key, None)
            else:
                children[key] = node
        total = len(children)
        n_vnodes = int(math.ceil(_f32(_f32(float(total)) / _f32(float(vnode_size))))) if total else 0
        buckets = [[] for _ in range(n_vnodes)]
        for key, node in children.items():
            buckets[_xxh3(node[0].encode()) % n_vnodes].append((key, node))
        vnodes = []
        for j, bucket in enumerate(buckets):
            bucket.sort(key=lambda kn: kn[0])
            stream = bytearray(b"vnode")
            stream += directory.encode()
            has_new = False
            for _, node in bucket:
                stream += int(node[1]).to_bytes(16, "little")
                if node[3] != "unmodified":
                    has_new = True
            if directory in existing and has_new:
                stream += salt(directory, j)
            vnodes.append((_xxh3(bytes(stream)), [node for _, node in bucket]))
        results[directory] = vnodes
    return results


def compute_dir_hash(vnodes, path):
    stream = bytearray(b"dir")
    stream += path.encode()
    base = _components(path)
    for child in vnodes:  # get_children: every key that starts_with(path), in map order
        if _components(child)[: len(base)] != base:
            continue
        for vnode_id, nodes in vnodes[child]:
            stream += int(vnode_id).to_bytes(16, "little")
            for node in nodes:
                stream += (node[4] if node[4] is not None else node[0]).encode()
                stream += int(node[1]).to_bytes(16, "little")
    return _xxh3(bytes(stream))


def commit_tree(entries, existing, vnode_size, salt):
    vn = split_into_vnodes(entries, existing, vnode_size, salt)
    dirs = [""] + [k for k in vn if _components(k)]
    return vn, {d: compute_dir_hash(vn, d) for d in dirs}
