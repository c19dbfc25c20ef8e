"""The restore / merge "may this working file be overwritten?" checks, batched over the C ABI
(core/v_latest/index/restore.rs:231-297 `should_restore_partial_node`, :300-405 `should_restore_file`;
called per file by merge.rs:742-829, 1304-1398 and checkout).

Per file the reference decides, in order:
  * the working file does not exist                               -> true (nothing to lose)
  * util::fs::metadata(working_path)?                             (an error is the call's error)
  * with a base node: mtime_matches && size == base's size        -> true
    without one:      mtime_matches && size == the target's size  -> true
  * otherwise it hashes the file (u128_hash_file_contents, :261/:290/:334/:377):
      partial node: hash == target.hash -> true; hash != base.hash -> false (no base: != target -> false)
      file node:    combined = get_combined_hash(maybe_get_metadata_hash(metadata), hash), compared
                    with target.combined_hash / base.combined_hash the same way
  * true.

Here every file that reaches the hash is read once, all in one GPU pass (oxh_hash_files_ex; text files
through K1T, whose line / char counts give MetadataText on the same read); mtime_matches is the repo's
tolerance rule (local_repository.rs:556) and stays with the caller, as in hasher.files_modified.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional, Sequence

from . import _capi
from .hasher import (TEXT, OxenError, file_error, hash_files_text_128bit,
                     hash_files_with_errors_128bit, hash_streams_128bit, metadata_json, rust_io_error_debug,
                     rust_path_debug)


@dataclass
class NodeHashes:
    """What the checks read from a node: PartialNode {hash, size} (restore.rs:231) or FileNode
    {hash, combined_hash, num_bytes} (:300)."""
    hash: int
    num_bytes: int
    combined_hash: Optional[int] = None


def should_restore(paths: Sequence[str], targets: Sequence[NodeHashes], bases: Sequence[Optional[NodeHashes]],
                   mtime_matched: Sequence[bool], combined: bool = False, file_metadata: Optional[Sequence] = None,
                   ctx: Optional[_capi.Context] = None) -> list[bool]:
    """should_restore_partial_node (combined=False) or should_restore_file (combined=True) for every
    working path. file_metadata[i] (combined only) is the working file's side of the combined hash:
    None (no metadata for its type), hasher.TEXT (MetadataText counted on the hashing read), an int
    (the caller's maybe_get_metadata_hash) or the GenericMetadata itself. The reference extracts it from
    the repo-relative `path` (restore.rs:336-339), so the caller supplies it here. Errors raise as the
    reference's `?` does, the first failing file in order."""
    n = len(paths)
    if not (len(targets) == len(bases) == len(mtime_matched) == n):
        raise _capi.OxenError("should_restore: argument lengths differ", _capi.OXH_ERR_INVALID)
    if file_metadata is not None and len(file_metadata) != n:
        raise _capi.OxenError("should_restore: argument lengths differ", _capi.OXH_ERR_INVALID)
    out: list[Optional[bool]] = [None] * n
    need: list[int] = []
    stat_error: Optional[tuple[int, OxenError]] = None  # the first file whose metadata(..)? fails
    for i, p in enumerate(paths):
        if not os.path.exists(p):  # working_path.exists() (follows symlinks)
            out[i] = True
            continue
        try:
            size = os.stat(p).st_size  # util::fs::metadata(&working_path)? (only a race after exists())
        except OSError as e:
            # raised after the hashes of the files before it: an earlier file's hash error comes first
            stat_error = (i, OxenError(f"Could not get file metadata: {rust_path_debug(p)} error "
                                       f"{rust_io_error_debug(e.errno or 0)}", _capi.OXH_ERR_IO))
            break
        ref = bases[i] if bases[i] is not None else targets[i]
        if mtime_matched[i] and size == ref.num_bytes:
            out[i] = True
            continue
        need.append(i)
    if not need:
        if stat_error is not None:
            raise stat_error[1]
        return [bool(x) for x in out]
    meta = [None] * n if file_metadata is None else list(file_metadata)
    text = [i for i in need if combined and isinstance(meta[i], str) and meta[i] == TEXT]
    text_set = set(text)
    plain = [i for i in need if i not in text_set]
    content: dict[int, int] = {}
    meta_hash: dict[int, Optional[int]] = {}
    if plain:
        digests, _, status, oserr = hash_files_with_errors_128bit([paths[i] for i in plain], ctx=ctx)
        for j, i in enumerate(plain):
            content[i] = (digests[j], status[j], oserr[j])
    if text:
        d, _, st, m = hash_files_text_128bit([paths[i] for i in text], ctx)
        for j, i in enumerate(text):
            content[i] = (d[j], st[j], 0)
            meta_hash[i] = None
        ok = [j for j, i in enumerate(text) if st[j] == 0]
        for j, h in zip(ok, hash_streams_128bit([metadata_json(m[j]).encode("utf-8") for j in ok], ctx)):
            meta_hash[text[j]] = h
    if combined:
        objs = [i for i in plain if meta[i] is not None and not isinstance(meta[i], (int, str))]
        for i, h in zip(objs, hash_streams_128bit([metadata_json(meta[i]).encode("utf-8") for i in objs], ctx)):
            meta_hash[i] = h
        for i in plain:
            if i not in meta_hash:
                meta_hash[i] = int(meta[i]) if isinstance(meta[i], int) and not isinstance(meta[i], bool) else None
    for i in need:  # in path order: the first failing file is the error
        h, st, oe = content[i]
        if st != 0:
            if i in text_set:  # the K1T pass reports no errno: take the file's error from the plain path
                _, _, st2, oe2 = hash_files_with_errors_128bit([paths[i]], ctx=ctx)
                st, oe = (st2[0], oe2[0]) if st2[0] != 0 else (st, 0)
            raise file_error(paths[i], st, oe)
    if stat_error is not None:  # every file before it hashed cleanly
        raise stat_error[1]
    if combined:  # get_combined_hash (hasher.rs:67-80) of every file with a metadata hash, one batch
        for i in need:
            t, b = targets[i], bases[i]
            if t.combined_hash is None or (b is not None and b.combined_hash is None):
                raise _capi.OxenError("should_restore: combined=True needs combined hashes", _capi.OXH_ERR_INVALID)
        withm = [i for i in need if meta_hash.get(i) is not None]
        streams = [int(content[i][0]).to_bytes(16, "little") + int(meta_hash[i]).to_bytes(16, "little") for i in withm]
        for i, c in zip(withm, hash_streams_128bit(streams, ctx)):
            content[i] = (c,) + content[i][1:]
    for i in need:
        h = content[i][0]
        t, b = targets[i], bases[i]
        if combined:
            want, base_h = t.combined_hash, (b.combined_hash if b is not None else None)
        else:
            want, base_h = t.hash, (b.hash if b is not None else None)
        if b is not None:
            out[i] = True if h == want else h == base_h
        else:
            out[i] = h == want
    return [bool(x) for x in out]
