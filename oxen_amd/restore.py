"""The restore / merge "may this working file be overwritten?" checks, batched over the C ABI
(core/v_latest/index/restore.rs:231-297 `should_restore_partial_node`, :300-405 `should_restore_file`;
called per file by merge.rs:742-829, 1304-1398 and checkout), and checkout's own three-way
classification of the target tree's files (core/v_latest/branches.rs:653-757, `classify_checkout`).

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
                     rust_path_debug, text_metadata_json)


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
        for j, h in zip(ok, hash_streams_128bit([text_metadata_json(m[j]).encode("utf-8") for j in ok], ctx)):
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


# Outcomes of checkout's File arm (core/v_latest/branches.rs:653-757, r_restore_missing_or_modified_files)
SKIP = "skip"                  # the working file already is the target's version: nothing to do
RESTORE = "restore"            # goes to results.files_to_restore
CONFLICT = "conflict"          # goes to results.cannot_overwrite_entries (OnConflict::Abort)
KEEP_DELETED = "keep_deleted"  # an uncommitted deletion of a file both trees hold unchanged: preserved


def classify_checkout(paths: Sequence[str], targets: Sequence[NodeHashes], froms: Sequence[Optional[NodeHashes]],
                      target_mtime_matched: Sequence[bool], from_mtime_matched: Sequence[bool],
                      overwrite: bool = False, ctx: Optional[_capi.Context] = None) -> list[str]:
    """The File arm of checkout's target-tree walk (branches.rs:653-757) for every file, in the walk's
    order. targets[i]: the target FileNode's content hash and num_bytes (node.hash is the content hash,
    merkle_tree_node.rs:147-159); froms[i]: the from tree's PartialNode at the same path (hash, size), or
    None for a path new in the target. The two mtime verdicts are the repo's tolerance rule applied by
    the caller (repo.mtime_matches of the disk mtime against the target's / the PartialNode's), as for
    should_restore. overwrite = OnConflict::Overwrite (`oxen merge --abort`). Per file the reference:
      * not on disk: from has the target's hash -> KEEP_DELETED; a from node otherwise -> CONFLICT
        (abort) or RESTORE (overwrite); no from node -> RESTORE (new in the target);
      * util::fs::metadata(..)? ; target mtime + size match -> SKIP; from mtime + size match -> RESTORE;
      * get_hash_given_metadata(..)? : == target -> SKIP; == from -> RESTORE; else CONFLICT / RESTORE.
    Every file that reaches the hash is read once, all in one GPU pass; errors raise as the reference's
    `?` does -- the first failing file in order, its metadata before its read."""
    n = len(paths)
    if not (len(targets) == len(froms) == len(target_mtime_matched) == len(from_mtime_matched) == n):
        raise _capi.OxenError("classify_checkout: argument lengths differ", _capi.OXH_ERR_INVALID)
    out: list[Optional[str]] = [None] * n
    need: list[int] = []
    sizes: dict[int, int] = {}
    stat_error: Optional[OxenError] = None
    for i, p in enumerate(paths):
        t, f = targets[i], froms[i]
        if not os.path.exists(p):  # full_path.exists()
            if f is not None and f.hash == t.hash:
                out[i] = KEEP_DELETED
            elif f is not None and not overwrite:
                out[i] = CONFLICT
            else:
                out[i] = RESTORE
            continue
        try:
            size = os.stat(p).st_size  # util::fs::metadata(&full_path)? (only a race after exists())
        except OSError as e:
            stat_error = OxenError(f"Could not get file metadata: {rust_path_debug(p)} error "
                                   f"{rust_io_error_debug(e.errno or 0)}", _capi.OXH_ERR_IO)
            break
        if target_mtime_matched[i] and size == t.num_bytes:
            out[i] = SKIP
        elif f is not None and from_mtime_matched[i] and size == f.num_bytes:
            out[i] = RESTORE
        else:
            need.append(i)
            sizes[i] = size
    if need:
        digests, _, status, oserr = hash_files_with_errors_128bit([paths[i] for i in need],
                                                                  meta_sizes=[sizes[i] for i in need], ctx=ctx)
        for j, i in enumerate(need):  # in walk order: the first failing file is the error
            if status[j] != 0:
                raise file_error(paths[i], status[j], oserr[j], sizes[i])
        for j, i in enumerate(need):
            h, t, f = digests[j], targets[i], froms[i]
            if h == t.hash:
                out[i] = SKIP
            elif f is not None and h == f.hash:
                out[i] = RESTORE
            else:
                out[i] = RESTORE if overwrite else CONFLICT
    if stat_error is not None:  # every file before it classified without an error
        raise stat_error
    return [str(x) for x in out]
