"""Host-side mirror of liboxen `util::hasher` (crates/liboxen/src/util/hasher.rs) over the GPU C ABI.

Same function names, argument meaning and error behaviour as the Rust module; every digest is
computed by the HIP kernels in oxen_amd/csrc through include/oxen_hash.h -- there is no CPU
hashing fallback (a missing library or device raises `OxenError`). On top of the per-item
functions, `hash_buffers_128bit` / `hash_files_128bit` expose the batched form the add loop would
call once per batch of files (core/v_latest/add.rs:422-444).

u128 digests are Python ints: ``(hi << 64) | lo``, exactly the Rust `u128` / `MerkleHash` value.
"""
from __future__ import annotations

import ctypes
import json
import os
import threading
import time
from typing import Iterable, Optional, Sequence

import numpy as np

from . import _capi
from ._capi import OxenError

_ctx: Optional[_capi.Context] = None
_ctx_lock = threading.Lock()


def default_context() -> _capi.Context:
    """Process-wide context on device $OXH_DEVICE (default 0), created on first use."""
    global _ctx
    with _ctx_lock:
        if _ctx is None:
            _ctx = _capi.Context(int(os.environ.get("OXH_DEVICE", "0")))
        return _ctx


class _PathTable:
    """A `const char* const*` table over NUL-terminated paths packed in one buffer (the pointer table
    built with numpy: ~20x cheaper than a ctypes array of 200 000 c_char_p objects)."""

    def __init__(self, paths: Sequence):
        if all(isinstance(p, str) for p in paths):  # one encode of the joined list, NULs found by numpy
            joined = os.fsencode("\0".join(paths) + "\0")
        else:
            joined = b"\0".join(p if isinstance(p, bytes) else os.fsencode(str(p)) for p in paths) + b"\0"
        self.blob = np.frombuffer(joined, dtype=np.uint8)
        ends = np.flatnonzero(self.blob == 0).astype(np.uint64) if len(paths) else np.zeros(0, dtype=np.uint64)
        if len(ends) != len(paths):
            raise OxenError("a path contains a NUL byte", _capi.OXH_ERR_INVALID)
        offs = np.zeros(len(paths), dtype=np.uint64)
        if len(paths) > 1:
            offs[1:] = ends[:-1] + np.uint64(1)
        self.ptrs = offs + np.uint64(self.blob.ctypes.data)

    @property
    def arg(self):
        return self.ptrs.ctypes.data_as(ctypes.POINTER(ctypes.c_char_p))


def _to_u128(lo: int, hi: int) -> int:
    return (int(hi) << 64) | int(lo)


def _u128_list(out: np.ndarray, status=None) -> list:
    """(n, 2) uint64 (lo, hi) rows -> Python ints (None where status != 0), via tolist() (C loops)
    instead of iterating numpy scalars, which costs ~1 us per row."""
    lo, hi = out[:, 0].tolist(), out[:, 1].tolist()
    if status is None:
        return [(h << 64) | l for l, h in zip(lo, hi)]
    st = status.tolist() if hasattr(status, "tolist") else list(status)
    return [((h << 64) | l) if s == 0 else None for l, h, s in zip(lo, hi, st)]


def format_hex(value: int) -> str:
    """`format!("{:x}", u128)` -- lowercase, not zero-padded (merkle_hash.rs:73-77)."""
    return format(value, "x")


# ---------------------------------------------------------------------------- batch entry points
def hash_buffers_128bit(buffers: Sequence[bytes], ctx: Optional[_capi.Context] = None) -> list[int]:
    """`hash_buffer_128bit` over many host buffers in one batched GPU pass."""
    ctx = ctx or default_context()
    n = len(buffers)
    if n == 0:
        return []
    keep = [bytes(b) for b in buffers]
    ptrs = (ctypes.c_char_p * n)(*keep)
    lens = np.array([len(b) for b in keep], dtype=np.uint64)
    out = np.zeros((n, 2), dtype=np.uint64)
    _capi.check(_capi.lib().oxh_hash_buffers(ctx.handle, ptrs, lens.ctypes.data_as(_capi._u64p), n,
                                             out.ctypes.data_as(_capi._u64p)), "oxh_hash_buffers")
    return _u128_list(out)


def hash_streams_128bit(streams: Sequence[bytes], ctx: Optional[_capi.Context] = None) -> list[int]:
    """K2: XXH3-128 of caller-serialised parent-node byte streams (one lane per short stream)."""
    ctx = ctx or default_context()
    n = len(streams)
    if n == 0:
        return []
    lens = np.fromiter(map(len, streams), dtype=np.uint64, count=len(streams))
    offs = np.zeros(n, dtype=np.uint64)
    if n > 1:
        offs[1:] = np.cumsum(lens[:-1])
    arena = np.frombuffer(b"".join(streams) or b"\0", dtype=np.uint8)
    out = np.zeros((n, 2), dtype=np.uint64)
    _capi.check(_capi.lib().oxh_hash_streams(ctx.handle, arena.ctypes.data, offs.ctypes.data_as(_capi._u64p),
                                             lens.ctypes.data_as(_capi._u64p), n,
                                             out.ctypes.data_as(_capi._u64p)), "oxh_hash_streams")
    return _u128_list(out)


def hash_files_128bit(paths: Sequence[str], ctx: Optional[_capi.Context] = None):
    """`get_hash_given_metadata` over many files: returns (digests, sizes, status).

    digests[i] is None where status[i] != 0 (the add loop logs and skips such files,
    add.rs:533-544); sizes are the stat sizes used for the read.
    """
    ctx = ctx or default_context()
    n = len(paths)
    if n == 0:
        return [], [], []
    table = _PathTable(paths)
    arr = table.arg
    out = np.zeros((n, 2), dtype=np.uint64)
    sizes = np.zeros(n, dtype=np.uint64)
    status = np.zeros(n, dtype=np.int32)
    _capi.check(_capi.lib().oxh_hash_files(ctx.handle, arr, n, out.ctypes.data_as(_capi._u64p),
                                           sizes.ctypes.data_as(_capi._u64p),
                                           status.ctypes.data_as(_capi._i32p)), "oxh_hash_files")
    digests = _u128_list(out, status)
    return digests, sizes.tolist(), status.tolist()



def hash_files_with_errors_128bit(paths: Sequence[str], meta_sizes: Optional[Sequence[int]] = None,
                                  ctx: Optional[_capi.Context] = None):
    """hash_files_128bit (meta_sizes None) or hash_files_given_metadata_128bit through oxh_hash_files_ex:
    returns (digests, sizes, status, os_error), os_error[i] being the errno of item i's failed open
    (status OXH_ERR_OPEN) or read (OXH_ERR_IO), from which `file_error` builds hasher.rs's message."""
    ctx = ctx or default_context()
    n = len(paths)
    if n == 0:
        return [], [], [], []
    if meta_sizes is not None and len(meta_sizes) != n:
        raise _capi.OxenError("paths and meta_sizes differ in length", _capi.OXH_ERR_INVALID)
    table = _PathTable(paths)
    meta = None if meta_sizes is None else np.ascontiguousarray(meta_sizes, dtype=np.uint64)
    out = np.zeros((n, 2), dtype=np.uint64)
    sizes = np.zeros(n, dtype=np.uint64)
    status = np.zeros(n, dtype=np.int32)
    oserr = np.zeros(n, dtype=np.int32)
    _capi.check(_capi.lib().oxh_hash_files_ex(ctx.handle, table.arg, None if meta is None else meta.ctypes.data_as(_capi._u64p),
                                              n, out.ctypes.data_as(_capi._u64p), sizes.ctypes.data_as(_capi._u64p),
                                              status.ctypes.data_as(_capi._i32p), oserr.ctypes.data_as(_capi._i32p),
                                              None, None), "oxh_hash_files_ex")
    return _u128_list(out, status), sizes.tolist(), status.tolist(), oserr.tolist()


# std::io::ErrorKind of an OS error (Rust std, sys/pal/unix decode_error_kind): the `kind` field of
# the io::Error Debug text that hasher.rs puts in its open-failure message
_IO_ERROR_KINDS = {
    "E2BIG": "ArgumentListTooLong", "EADDRINUSE": "AddrInUse", "EADDRNOTAVAIL": "AddrNotAvailable",
    "EBUSY": "ResourceBusy", "ECONNABORTED": "ConnectionAborted", "ECONNREFUSED": "ConnectionRefused",
    "ECONNRESET": "ConnectionReset", "EDEADLK": "Deadlock", "EDQUOT": "FilesystemQuotaExceeded",
    "EEXIST": "AlreadyExists", "EFBIG": "FileTooLarge", "EHOSTUNREACH": "HostUnreachable", "EINTR": "Interrupted",
    "EINVAL": "InvalidInput", "EISDIR": "IsADirectory", "ELOOP": "FilesystemLoop", "ENOENT": "NotFound",
    "ENOMEM": "OutOfMemory", "ENOSPC": "StorageFull", "ENOSYS": "Unsupported", "EMLINK": "TooManyLinks",
    "ENAMETOOLONG": "InvalidFilename", "ENETDOWN": "NetworkDown", "ENETUNREACH": "NetworkUnreachable",
    "ENOTCONN": "NotConnected", "ENOTDIR": "NotADirectory", "ENOTEMPTY": "DirectoryNotEmpty", "EPIPE": "BrokenPipe",
    "EROFS": "ReadOnlyFilesystem", "ESPIPE": "NotSeekable", "ESTALE": "StaleNetworkFileHandle", "ETIMEDOUT": "TimedOut",
    "ETXTBSY": "ExecutableFileBusy", "EXDEV": "CrossesDevices", "EINPROGRESS": "InProgress",
    "EACCES": "PermissionDenied", "EPERM": "PermissionDenied", "EAGAIN": "WouldBlock", "EWOULDBLOCK": "WouldBlock",
}


# Other_Grapheme_Extend code points outside categories Mn / Me (DerivedCoreProperties: Grapheme_Extend =
# Mn + Me + Other_Grapheme_Extend); the Cf ones among them are escaped as non-printable anyway
_OTHER_GRAPHEME_EXTEND = frozenset([0x09BE, 0x09D7, 0x0B3E, 0x0B57, 0x0BBE, 0x0BD7, 0x0CC2, 0x0CD5, 0x0CD6, 0x0D3E,
                                    0x0D57, 0x0DCF, 0x0DDF, 0x1B35, 0x200C, 0x302E, 0x302F, 0xFF9E, 0xFF9F, 0x1133E,
                                    0x11357, 0x114B0, 0x114BD, 0x115AF, 0x11930, 0x1D165, 0x1D16E, 0x1D16F, 0x1D170,
                                    0x1D171, 0x1D172])


def _rust_escape_char(ch: str, escape_single_quote: bool) -> str:
    """char::escape_debug_ext (Rust core): the named escapes, then \\u{..} for grapheme-extended and
    non-printable chars. core::unicode::printable marks as non-printable every code point of general
    category Cc, Cf, Cs, Co, Cn, Zl, Zp or Zs except the space (its generator, printable.py); the
    categories come from Python's unicodedata, whose Unicode version may trail Rust's for recently
    assigned code points ("Error texts")."""
    import unicodedata

    esc = {"\0": "\\0", "\t": "\\t", "\r": "\\r", "\n": "\\n", "\\": "\\\\", '"': '\\"'}
    if ch in esc:
        return esc[ch]
    if ch == "'" and escape_single_quote:
        return "\\'"
    o = ord(ch)
    cat = unicodedata.category(ch)
    if cat in ("Mn", "Me") or o in _OTHER_GRAPHEME_EXTEND:
        return "\\u{%x}" % o
    if cat in ("Cc", "Cf", "Cs", "Co", "Cn", "Zl", "Zp", "Zs") and ch != " ":
        return "\\u{%x}" % o
    return ch


def rust_str_debug(text: str) -> str:
    """`{:?}` of a Rust str (e.g. io::Error's message): double quotes; the escapes of char::escape_debug
    except that a single quote stays as it is."""
    return '"' + "".join(_rust_escape_char(ch, False) for ch in text) + '"'


def rust_path_debug(path) -> str:
    """`{:?}` of a Rust Path on Unix (OsStr -> the byte string's Utf8Chunks Debug, core/src/str/lossy.rs):
    the valid UTF-8 runs escaped by char::escape_debug (a single quote too), every byte of an invalid
    sequence as \\xNN (upper-case hex)."""
    raw = os.fsencode(path)
    out = ['"']
    for ch in raw.decode("utf-8", errors="surrogateescape"):
        o = ord(ch)
        if 0xDC80 <= o <= 0xDCFF:  # a byte that is not part of valid UTF-8
            out.append("\\x%02X" % (o - 0xDC00))
        else:
            out.append(_rust_escape_char(ch, True))
    out.append('"')
    return "".join(out)


def rust_io_error_debug(errno_value: int) -> str:
    """`{:?}` of std::io::Error::from_raw_os_error(errno_value): `Os { code, kind, message }`."""
    import errno as _errno

    name = _errno.errorcode.get(int(errno_value), "")
    kind = _IO_ERROR_KINDS.get(name, "Uncategorized")
    return f"Os {{ code: {int(errno_value)}, kind: {kind}, message: {rust_str_debug(os.strerror(int(errno_value)))} }}"


LARGE_FILE_BYTES = 1_000_000_000  # hasher.rs:56-65, 106: one-shot below, 4 KiB streamed at or above


def file_error(path, status: int, os_error: int, size_hint: Optional[int] = None) -> OxenError:
    """The OxenError hasher.rs returns for a file that could not be hashed: File::open failed
    (status OXH_ERR_OPEN; hasher.rs:141-145, or :151-154 for the streamed branch a size >= 1e9 picks),
    or the read did (OXH_ERR_IO; :135-139 / :161-165)."""
    if status == _capi.OXH_ERR_OPEN:
        p = rust_path_debug(path)
        err = rust_io_error_debug(os_error)
        if size_hint is not None and size_hint >= LARGE_FILE_BYTES:
            return OxenError(f"Could not open file {p} due to {err}", _capi.OXH_ERR_OPEN)
        return OxenError(f"util::hasher::hash_file_contents Could not open file {p} {err}", _capi.OXH_ERR_OPEN)
    if status == _capi.OXH_ERR_NOMEM:
        return OxenError("Could not allocate the buffers to hash a large file", _capi.OXH_ERR_NOMEM)
    return OxenError("Could not read file for hashing", _capi.OXH_ERR_IO)


def hash_files_given_metadata_128bit(paths: Sequence[str], meta_sizes: Sequence[int],
                                     ctx: Optional[_capi.Context] = None):
    """`get_hash_given_metadata(path, &metadata)` over many files (hasher.rs:56-65) with the sizes
    the caller's directory walk already has: no fstat per file; a file whose size changed since is
    re-read. Returns (digests, sizes, status) like hash_files_128bit."""
    ctx = ctx or default_context()
    n = len(paths)
    if n == 0:
        return [], [], []
    if len(meta_sizes) != n:
        raise _capi.OxenError("paths and meta_sizes differ in length", _capi.OXH_ERR_INVALID)
    table = _PathTable(paths)
    arr = table.arg
    meta = np.ascontiguousarray(meta_sizes, dtype=np.uint64)
    out = np.zeros((n, 2), dtype=np.uint64)
    sizes = np.zeros(n, dtype=np.uint64)
    status = np.zeros(n, dtype=np.int32)
    _capi.check(_capi.lib().oxh_hash_files_meta(ctx.handle, arr, meta.ctypes.data_as(_capi._u64p), n,
                                                out.ctypes.data_as(_capi._u64p), sizes.ctypes.data_as(_capi._u64p),
                                                status.ctypes.data_as(_capi._i32p)), "oxh_hash_files_meta")
    return _u128_list(out, status), sizes.tolist(), status.tolist()


def _split_u128(values) -> np.ndarray:
    return np.array([(int(h) & 0xFFFFFFFFFFFFFFFF, int(h) >> 64) for h in values], dtype=np.uint64).reshape(-1, 2)


TEXT = "text"  # files_modified's file_metadata marker for data type Text (MetadataText counted on the read)


def files_modified(paths: Sequence[str], sizes: Sequence[int], node_bytes: Sequence[int],
                   mtime_matched: Sequence[bool], node_hashes: Sequence[int],
                   ctx: Optional[_capi.Context] = None, node_metadata_hashes: Optional[Sequence[Optional[int]]] = None,
                   file_metadata: Optional[Sequence] = None, os_errors: Optional[list] = None):
    """`classify_modified_from_node_with_metadata` (util/fs.rs:1580-1619) over many working-tree files
    (oxh_files_modified): the modified check `oxen status` runs per tracked file
    (core/v_latest/status.rs:710,734). sizes = the walk's metadata.len(), node_bytes / node_hashes =
    the committed FileNode's num_bytes / hash (u128), mtime_matched = the caller's mtime verdict,
    node_metadata_hashes[i] = node.metadata_hash() (None or u128; omitted: all None).
    file_metadata[i] is the working file's side of fs.rs:1600-1607 (omitted: all None):
      None            no metadata for its data type (maybe_get_metadata_hash -> None)
      hasher.TEXT     data type Text: MetadataText is counted on the hashing read itself (K1T)
      int             the metadata hash the caller already extracted
      dict / object   the GenericMetadata itself (its serde_json is hashed on the device)
      Exception       the caller's extraction failed (status[i] = OXH_ERR_META, as the reference's `?`)
    Returns (modified, status, n_hashed): only files with an equal size and a drifted mtime whose
    metadata hash does not already differ are read, all in one GPU pass; status[i] != 0 is that
    file's error (the reference returns it); a list passed as `os_errors` receives the errno of each
    such failure (hasher.file_error builds the reference's message from it)."""
    ctx = ctx or default_context()
    n = len(paths)
    if not (len(sizes) == len(node_bytes) == len(mtime_matched) == len(node_hashes) == n):
        raise _capi.OxenError("files_modified: argument lengths differ", _capi.OXH_ERR_INVALID)
    if (node_metadata_hashes is not None and len(node_metadata_hashes) != n) or (file_metadata is not None and len(file_metadata) != n):
        raise _capi.OxenError("files_modified: argument lengths differ", _capi.OXH_ERR_INVALID)
    if n == 0:
        return [], [], 0
    table = _PathTable(paths)
    arr = table.arg
    sz = np.ascontiguousarray(sizes, dtype=np.uint64)
    nb = np.ascontiguousarray(node_bytes, dtype=np.uint64)
    mm = np.ascontiguousarray([1 if m else 0 for m in mtime_matched], dtype=np.uint8)
    nh = _split_u128(node_hashes)
    nmp = nmh = fk = fh = None
    if node_metadata_hashes is not None:
        nmp = np.array([0 if h is None else 1 for h in node_metadata_hashes], dtype=np.uint8)
        nmh = _split_u128([0 if h is None else h for h in node_metadata_hashes])
    if file_metadata is not None:
        fk = np.zeros(n, dtype=np.uint8)
        fhv = [0] * n
        objs = []
        for i, f in enumerate(file_metadata):
            if f is None:
                continue
            if isinstance(f, BaseException):
                fk[i] = _capi.OXH_META_ERROR
            elif isinstance(f, str):
                if f != TEXT:
                    raise _capi.OxenError(f"files_modified: file_metadata[{i}] is a string other than hasher.TEXT",
                                          _capi.OXH_ERR_INVALID)
                fk[i] = _capi.OXH_META_TEXT
            elif isinstance(f, (int, np.integer)) and not isinstance(f, bool):
                fk[i], fhv[i] = _capi.OXH_META_GIVEN, int(f)
            else:
                fk[i] = _capi.OXH_META_GIVEN
                objs.append(i)
        if objs:  # get_metadata_hash of every GenericMetadata object, one batched GPU pass
            for i, h in zip(objs, hash_streams_128bit([metadata_json(file_metadata[i]).encode("utf-8") for i in objs], ctx)):
                fhv[i] = h
        fh = _split_u128(fhv)
    modified = np.zeros(n, dtype=np.uint8)
    status = np.zeros(n, dtype=np.int32)
    oserr = np.zeros(n, dtype=np.int32)
    hashed = (ctypes.c_uint64 * 1)()
    ptr = lambda a: None if a is None else a.ctypes.data  # noqa: E731
    _capi.check(_capi.lib().oxh_files_modified_ex(ctx.handle, arr, sz.ctypes.data_as(_capi._u64p),
                                                  nb.ctypes.data_as(_capi._u64p), mm.ctypes.data,
                                                  nh.ctypes.data_as(_capi._u64p), ptr(nmp), ptr(nmh), ptr(fk), ptr(fh),
                                                  n, modified.ctypes.data, status.ctypes.data_as(_capi._i32p),
                                                  oserr.ctypes.data_as(_capi._i32p), hashed), "oxh_files_modified_ex")
    if os_errors is not None:
        os_errors[:] = oserr.tolist()
    return [bool(m) for m in modified], [int(s) for s in status], int(hashed[0])


def classify_modified_from_node_with_metadata(path, node_num_bytes: int, node_hash: int,
                                              metadata: os.stat_result, mtime_matched: bool,
                                              node_metadata_hash: Optional[int] = None, file_metadata=None) -> bool:
    """util/fs.rs:1580-1619 for one file (the batched form is files_modified); an extraction or read
    error raises OxenError like the reference's `?`."""
    oserr: list = []
    modified, status, _ = files_modified([path], [metadata.st_size], [node_num_bytes], [mtime_matched], [node_hash],
                                         node_metadata_hashes=[node_metadata_hash], file_metadata=[file_metadata],
                                         os_errors=oserr)
    if status[0] == _capi.OXH_ERR_META:
        err = file_metadata
        raise OxenError(str(err) if str(err) else "could not compute file metadata", _capi.OXH_ERR_META)
    if status[0] != 0:  # get_hash_given_metadata(path, metadata)? (fs.rs:1616-1618)
        raise file_error(path, status[0], oserr[0], int(metadata.st_size))
    return modified[0]


def add_files(paths: Sequence[str], versions_root: str, ctx: Optional[_capi.Context] = None):
    """Fused hash + version-store publish (oxh_add_files): returns (digests, sizes, status, stored).
    stored[i] is True when the blob {versions_root}/{hex[:2]}/{hex[2:]}/data was written now."""
    ctx = ctx or default_context()
    n = len(paths)
    if n == 0:
        return [], [], [], []
    table = _PathTable(paths)
    arr = table.arg
    out = np.zeros((n, 2), dtype=np.uint64)
    sizes = np.zeros(n, dtype=np.uint64)
    status = np.zeros(n, dtype=np.int32)
    stored = np.zeros(n, dtype=np.int32)
    _capi.check(_capi.lib().oxh_add_files(ctx.handle, arr, n, os.fsencode(str(versions_root)),
                                          out.ctypes.data_as(_capi._u64p), sizes.ctypes.data_as(_capi._u64p),
                                          status.ctypes.data_as(_capi._i32p), stored.ctypes.data_as(_capi._i32p)),
                "oxh_add_files")
    digests = _u128_list(out, status)
    return digests, sizes.tolist(), status.tolist(), [bool(s) for s in stored]


def clean_corrupted_versions(versions_root: str, dry_run: bool = False, ctx: Optional[_capi.Context] = None) -> dict:
    """`oxen fsck`: LocalVersionStore::clean_corrupted_versions (storage/local.rs:417-610) as one batched
    GPU re-hash of every {versions_root}/{prefix}/{suffix}/data. Returns CleanCorruptedVersionsResult's
    fields: scanned, corrupted, cleaned, errors, elapsed (seconds)."""
    ctx = ctx or default_context()
    res = np.zeros(4, dtype=np.uint64)
    t0 = time.perf_counter()
    _capi.check(_capi.lib().oxh_clean_corrupted_versions(ctx.handle, os.fsencode(str(versions_root)), int(bool(dry_run)),
                                                         res.ctypes.data_as(_capi._u64p)),
                "oxh_clean_corrupted_versions")
    return {"scanned": int(res[0]), "corrupted": int(res[1]), "cleaned": int(res[2]), "errors": int(res[3]),
            "elapsed": time.perf_counter() - t0}


def version_path(versions_root: str, digest: int) -> str:
    """LocalVersionStore::version_path (storage/local.rs:66-75): {root}/{hex[..2]}/{hex[2..]}/data."""
    h = format_hex(digest)
    return os.path.join(versions_root, h[:2], h[2:], "data")


def hash_files_text_128bit(paths: Sequence[str], ctx: Optional[_capi.Context] = None):
    """K1T: digests plus the text metadata liboxen computes in a second pass
    (repositories/metadata/text.rs:11-20): returns (digests, sizes, status, metadata) where
    metadata[i] = {"text": {"num_lines": L, "num_chars": C}} (MetadataText's serde shape), or None
    where status[i] != 0."""
    ctx = ctx or default_context()
    n = len(paths)
    if n == 0:
        return [], [], [], []
    table = _PathTable(paths)
    arr = table.arg
    out = np.zeros((n, 2), dtype=np.uint64)
    sizes = np.zeros(n, dtype=np.uint64)
    status = np.zeros(n, dtype=np.int32)
    counts = np.zeros((n, 2), dtype=np.uint64)
    _capi.check(_capi.lib().oxh_hash_files_text(ctx.handle, arr, n, out.ctypes.data_as(_capi._u64p),
                                                sizes.ctypes.data_as(_capi._u64p),
                                                status.ctypes.data_as(_capi._i32p),
                                                counts.ctypes.data_as(_capi._u64p)), "oxh_hash_files_text")
    digests = _u128_list(out, status)
    meta = [({"text": {"num_lines": int(c[0]), "num_chars": int(c[1])}} if st == 0 else None)
            for c, st in zip(counts, status)]
    return digests, [int(s) for s in sizes], [int(s) for s in status], meta


def hash_files_text_utf8_128bit(paths: Sequence[str], ctx: Optional[_capi.Context] = None):
    """hash_files_text_128bit plus util::fs::is_utf8 (util/fs.rs:652-668) of every file, all from one
    read of each file: returns (digests, sizes, status, metadata, is_utf8)."""
    ctx = ctx or default_context()
    n = len(paths)
    if n == 0:
        return [], [], [], [], []
    table = _PathTable(paths)
    arr = table.arg
    out = np.zeros((n, 2), dtype=np.uint64)
    sizes = np.zeros(n, dtype=np.uint64)
    status = np.zeros(n, dtype=np.int32)
    counts = np.zeros((n, 2), dtype=np.uint64)
    utf8 = np.zeros(n, dtype=np.int32)
    _capi.check(_capi.lib().oxh_hash_files_text_utf8(ctx.handle, arr, n, out.ctypes.data_as(_capi._u64p),
                                                     sizes.ctypes.data_as(_capi._u64p),
                                                     status.ctypes.data_as(_capi._i32p),
                                                     counts.ctypes.data_as(_capi._u64p),
                                                     utf8.ctypes.data_as(_capi._i32p)), "oxh_hash_files_text_utf8")
    digests = _u128_list(out, status)
    meta = [({"text": {"num_lines": int(c[0]), "num_chars": int(c[1])}} if st == 0 else None)
            for c, st in zip(counts, status)]
    return digests, [int(s) for s in sizes], [int(s) for s in status], meta, [bool(u) for u in utf8]


def is_utf8(path) -> bool:
    """util/fs.rs:652-668 (one file; the batched form is hash_files_text_utf8_128bit)."""
    return hash_files_text_utf8_128bit([path])[4][0]


def text_file_nodes(paths: Sequence[str], ctx: Optional[_capi.Context] = None):
    """The hashing half of add.rs:833-842 for text files, batched: content hash and text counts in one
    GPU pass (K1T), then metadata_hash = XXH3(serde_json(metadata)) and combined_hash =
    XXH3(content LE || metadata LE) in batched passes. Returns a list of dicts (None for unreadable
    files) with keys hash, num_bytes, metadata, metadata_hash, combined_hash."""
    ctx = ctx or default_context()
    digests, sizes, status, meta = hash_files_text_128bit(paths, ctx)
    ok = [i for i, st in enumerate(status) if st == 0]
    mh = hash_streams_128bit([text_metadata_json(meta[i]).encode("utf-8") for i in ok], ctx)
    comb = hash_streams_128bit([digests[i].to_bytes(16, "little") + m.to_bytes(16, "little") for i, m in zip(ok, mh)], ctx)
    res: list = [None] * len(paths)
    for j, i in enumerate(ok):
        res[i] = {"hash": digests[i], "num_bytes": sizes[i], "metadata": meta[i], "metadata_hash": mh[j],
                  "combined_hash": comb[j]}
    return res


# ---------------------------------------------------------------------------- hasher.rs mirror
def hash_buffer_128bit(buffer: bytes) -> int:
    """hasher.rs:28-30."""
    return hash_buffers_128bit([buffer])[0]


def hash_buffer(buffer: bytes) -> str:
    """hasher.rs:11-14: unpadded lowercase hex of the XXH3-128."""
    return format_hex(hash_buffer_128bit(buffer))


def hash_str(buffer: str) -> str:
    """hasher.rs:16-19."""
    return hash_buffer(buffer.encode("utf-8"))


def _hash_one_file(path, size_hint: Optional[int] = None) -> int:
    digests, _, status, oserr = hash_files_with_errors_128bit([path])
    if status[0] != 0:
        raise file_error(path, status[0], oserr[0], size_hint)
    return digests[0]


def get_hash_given_metadata(path, metadata: os.stat_result) -> int:
    """hasher.rs:56-65. Both size branches (one-shot < 1e9 B, streamed otherwise) give the same
    XXH3-128; here both go through the batched file path (K1 or, for files larger than a staging
    slot, K1L). The size only picks which of hasher.rs's two open-failure messages an error gets."""
    return _hash_one_file(path, int(metadata.st_size))


def u128_hash_file_contents(path) -> int:
    """hasher.rs:102-112 (stats the file itself; a missing file is an error)."""
    try:
        size = os.stat(path).st_size
    except OSError as e:  # util::fs::metadata -> OxenError::file_metadata_error (util/fs.rs:593-601, error.rs:1176-1182)
        raise OxenError(f"Could not get file metadata: {rust_path_debug(path)} error {rust_io_error_debug(e.errno or 0)}",
                        _capi.OXH_ERR_IO) from None
    return _hash_one_file(path, size)


def hash_file_contents(path) -> str:
    """hasher.rs:114-124."""
    return format_hex(u128_hash_file_contents(path))


def hash_file_contents_with_retry(path, total_retries: int = 5, sleep=time.sleep) -> str:
    """hasher.rs:32-54: exponential backoff (2, 4, 8 ... s), give up after `total_retries` retries."""
    timeout, retries = 1, 0
    while True:
        try:
            return hash_file_contents(path)
        except OxenError:
            retries += 1
            timeout *= 2
            sleep(timeout)
            if retries > total_retries:
                raise


def serde_f64(x: float) -> str:
    """serde_json's text for an f64 field: non-finite values are `null` (serde_json's
    serialize_f64), finite ones ryu's shortest round-trip form (ryu::Buffer::format_finite, the crate's
    pretty.rs `format64`). With d the shortest digit string (length L, no trailing zeros) and the value
    d x 10^k, kk = L + k (10^(kk-1) <= |x| < 10^kk):
      0 <= k and kk <= 16    digits, k zeros, ".0"            12.0 -> "12.0", 1e15 -> "1000000000000000.0"
      0 < kk <= 16           the point after kk digits         12.5 -> "12.5"
      -5 < kk <= 0           "0.", -kk zeros, digits           1e-5 -> "0.00001", 0.1 -> "0.1"
      L == 1                 d "e" (kk - 1)                    1e16 -> "1e16", 1e-6 -> "1e-6"
      otherwise              d0 "." rest "e" (kk - 1)          1.5e16 -> "1.5e16", 1.25e-7 -> "1.25e-7"
    (no "+" and no zero padding in the exponent; zero is "0.0" / "-0.0"). The digit string is
    Python's repr's -- both pick the shortest string that round-trips, nearest the value."""
    import math
    from decimal import Decimal

    x = float(x)
    if not math.isfinite(x):
        return "null"
    if x == 0.0:
        return "-0.0" if math.copysign(1.0, x) < 0 else "0.0"
    sign = "-" if x < 0 else ""
    _, digits, k = Decimal(repr(abs(x))).as_tuple()
    d = "".join(map(str, digits))
    stripped = d.rstrip("0")
    k += len(d) - len(stripped)
    d = stripped
    n = len(d)
    kk = n + k
    if 0 <= k and kk <= 16:
        return f"{sign}{d}{'0' * k}.0"
    if 0 < kk <= 16:
        return f"{sign}{d[:kk]}.{d[kk:]}"
    if -5 < kk <= 0:
        return f"{sign}0.{'0' * -kk}{d}"
    if n == 1:
        return f"{sign}{d}e{kk - 1}"
    return f"{sign}{d[0]}.{d[1:]}e{kk - 1}"


# GenericMetadata variants with f64 fields (model/metadata/metadata_audio.rs:11, metadata_video.rs:11):
# serde writes them as floats even when the value is integral (12 -> "12.0")
_F64_FIELDS = {"audio": ("num_seconds",), "video": ("num_seconds",)}


def _serde_json(v) -> str:
    """serde_json::to_string's compact form: struct fields in order, strings escaped as serde_json
    does (", \\, \\b \\f \\n \\r \\t, other controls \\u00xx lowercase; non-ASCII as UTF-8)."""
    if v is None:
        return "null"
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, int):
        return str(v)
    if isinstance(v, float):
        return serde_f64(v)
    if isinstance(v, str):
        return json.dumps(v, ensure_ascii=False)
    if isinstance(v, dict):
        return "{" + ",".join(f"{json.dumps(str(k), ensure_ascii=False)}:{_serde_json(x)}" for k, x in v.items()) + "}"
    if isinstance(v, (list, tuple)):
        return "[" + ",".join(_serde_json(x) for x in v) + "]"
    raise TypeError(f"cannot serialise {type(v).__name__} as serde_json")


def _no_floats(v) -> bool:
    """True when nothing in v is a float: json.dumps then writes exactly serde_json's text."""
    stack = [v]
    while stack:
        x = stack.pop()
        t = type(x)
        if t is dict:
            stack.extend(x.values())
        elif t is list or t is tuple:
            stack.extend(x)
        elif isinstance(x, float):
            return False
    return True


def text_metadata_json(m) -> str:
    """metadata_json of a MetadataText (model/metadata/metadata_text.rs: {"text": {num_lines, num_chars}},
    both usize) as serde_json writes it -- the per-file string of a text add, built directly."""
    t = m["text"]
    return f'{{"text":{{"num_lines":{int(t["num_lines"])},"num_chars":{int(t["num_chars"])}}}}}'


def metadata_json(oxen_metadata) -> str:
    """serde_json::to_string of the (untagged) GenericMetadata (model/metadata/generic_metadata.rs:8-17),
    or "null" for None (hasher.rs:95-100).

    Dicts are serialised compactly in insertion order (= Rust struct field order); non-ASCII is
    written as UTF-8 like serde_json; floats as serde_json's f64 (serde_f64: ryu, NaN / inf -> null),
    and the f64 fields of MetadataAudio / MetadataVideo (num_seconds) as floats even when given an int.
    An object with to_json() serialises itself."""
    if hasattr(oxen_metadata, "to_json"):
        return oxen_metadata.to_json()
    if type(oxen_metadata) is dict and len(oxen_metadata) == 1:
        (kind, body), = oxen_metadata.items()
        if kind in _F64_FIELDS and isinstance(body, dict):
            body = {k: (float(x) if k in _F64_FIELDS[kind] and isinstance(x, int) and not isinstance(x, bool) else x)
                    for k, x in body.items()}
            oxen_metadata = {kind: body}
    if _no_floats(oxen_metadata):  # the common case (text, image, tabular metadata): the C encoder
        return json.dumps(oxen_metadata, separators=(",", ":"), ensure_ascii=False)
    return _serde_json(oxen_metadata)


def get_metadata_hash(oxen_metadata) -> int:
    """hasher.rs:95-100: XXH3-128 of serde_json(Option<GenericMetadata>) ("null" when None)."""
    return hash_streams_128bit([metadata_json(oxen_metadata).encode("utf-8")])[0]


def maybe_get_metadata_hash(oxen_metadata) -> Optional[int]:
    """hasher.rs:82-93."""
    if oxen_metadata is None:
        return None
    return get_metadata_hash(oxen_metadata)


def get_combined_hash(oxen_metadata_hash: Optional[int], content_hash: int) -> int:
    """hasher.rs:67-80: XXH3-128(content.to_le_bytes() || metadata.to_le_bytes()), or the content
    hash unchanged when there is no metadata hash."""
    if oxen_metadata_hash is None:
        return content_hash
    stream = int(content_hash).to_bytes(16, "little") + int(oxen_metadata_hash).to_bytes(16, "little")
    return hash_streams_128bit([stream])[0]


class Xxh3:
    """xxhash-rust `Xxh3` (new / update / digest128) on the GPU through oxh_xxh3_stream_*: bytes are
    staged in pinned memory and hashed on the device in 16 MiB pieces as they arrive, so a stream of
    any length holds bounded memory. `digest128()` does not consume the state."""

    def __init__(self, ctx: Optional[_capi.Context] = None):
        self._ctx = ctx or default_context()  # keeps the context alive as long as the stream
        h = _capi._vp()
        _capi.check(_capi.lib().oxh_xxh3_stream_create(self._ctx.handle, ctypes.byref(h)), "oxh_xxh3_stream_create")
        self._h = h

    def update(self, data) -> None:
        mv = memoryview(data).cast("B")
        if not mv.nbytes:
            return
        arr = np.frombuffer(mv, dtype=np.uint8)  # no copy, read-only buffers included
        _capi.check(_capi.lib().oxh_xxh3_stream_update(self._h, arr.ctypes.data, mv.nbytes), "oxh_xxh3_stream_update")

    def digest128(self) -> int:
        out = (ctypes.c_uint64 * 2)()
        _capi.check(_capi.lib().oxh_xxh3_stream_digest(self._h, out), "oxh_xxh3_stream_digest")
        return _to_u128(out[0], out[1])

    def reset(self) -> None:
        _capi.check(_capi.lib().oxh_xxh3_stream_reset(self._h), "oxh_xxh3_stream_reset")

    def close(self) -> None:
        if getattr(self, "_h", None):
            _capi.lib().oxh_xxh3_stream_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class HashingReader:
    """hasher.rs:183-209: wraps a reader, feeds every byte read into an `Xxh3` (GPU stream)."""

    def __init__(self, inner, ctx: Optional[_capi.Context] = None):
        self.inner = inner
        self.hasher = Xxh3(ctx)

    def read(self, n: int = -1) -> bytes:
        b = self.inner.read(n)
        if b:
            self.hasher.update(b)
        return b

    def digest128(self) -> int:
        return self.hasher.digest128()


class HashingWriter:
    """hasher.rs:214-244: wraps a writer, feeds every byte successfully written into an `Xxh3`
    (only the bytes the inner writer accepted, as in the reference's short-write test)."""

    def __init__(self, inner, ctx: Optional[_capi.Context] = None):
        self.inner = inner
        self.hasher = Xxh3(ctx)

    def write(self, b: bytes) -> int:
        n = self.inner.write(b)
        if n is None:
            n = memoryview(b).nbytes
        if n > 0:  # n counts bytes: slice the byte view, not the elements of e.g. array('H')
            self.hasher.update(memoryview(b).cast("B")[:n])
        return n

    def flush(self) -> None:
        self.inner.flush()

    def digest128(self) -> int:
        return self.hasher.digest128()
