"""Verify-before-publish writes of liboxen's version store, with the content hash on the GPU.

Mirrors `util::fs::atomic_file` (crates/liboxen/src/util/fs/atomic_file.rs) -- `AtomicFile::with_hash`
+ `stream` / `stream_async` / `write` -- and the content-addressed writes of `LocalVersionStore`
(storage/local.rs:104-139): bytes go to an `AtomicTempFile` sibling `<target>.oxentmp.<random>`
(:54-159) while a GPU `Xxh3` stream hashes them; a digest other than the expected one unlinks the
temp and raises `HashMismatchError` (:396-431, error.rs:463-471), otherwise the temp's data is
fsynced, renamed over the target and the parent directory fsynced (:116-159). There is no CPU
hashing here: every digest comes from the HIP kernels through the C ABI.

`LocalVersionStore.store_versions` is the batched receive (pull / clone downloads,
api/client/versions.rs): every buffer hashed in ONE GPU pass, then each verified blob published.
"""
from __future__ import annotations

import os
import secrets
import string
from typing import Optional, Sequence

from . import _capi, hasher
from ._capi import OxenError

STREAMING_BUF_SIZE = 10 * 1024 * 1024  # constants.rs:196
ATOMIC_TEMP_INFIX = ".oxentmp."        # atomic_file.rs:25
VERSION_FILE_NAME = "data"
VERSION_CHUNKS_DIR = "chunks"          # constants.rs:120
VERSION_CHUNK_FILE_NAME = "chunk"      # constants.rs:118


class HashMismatchError(OxenError):
    """OxenError::HashMismatch { path, expected, actual } (error.rs:463-471)."""

    def __init__(self, path: str, expected: int, actual: int):
        self.path, self.expected, self.actual = path, expected, actual
        super().__init__(f'Hash mismatch writing "{path}": expected {expected:x}, got {actual:x}', _capi.OXH_ERR_IO)


class _TempFile:
    """AtomicTempFile (atomic_file.rs:54-159): unlinked unless committed."""

    _ALNUM = string.ascii_letters + string.digits

    def __init__(self, target: str):
        name = os.path.basename(target)
        if not name:
            raise OxenError(f"Could not create file {target!r}: target path has no filename component", _capi.OXH_ERR_IO)
        parent = os.path.dirname(target)
        if parent:
            os.makedirs(parent, exist_ok=True)
        self.target = target
        for _ in range(64):
            rnd = "".join(secrets.choice(self._ALNUM) for _ in range(6))
            self.path = os.path.join(parent, name + ATOMIC_TEMP_INFIX + rnd)
            try:
                self.fd = os.open(self.path, os.O_CREAT | os.O_EXCL | os.O_WRONLY | os.O_CLOEXEC, 0o600)
                break
            except FileExistsError:
                continue
        else:
            raise OxenError(f"Could not create file {self.path!r}", _capi.OXH_ERR_IO)
        self.committed = False

    def write_all(self, data) -> None:
        mv = memoryview(data).cast("B")
        while mv.nbytes:
            n = os.write(self.fd, mv)
            mv = mv[n:]

    def commit(self) -> None:
        os.fsync(self.fd)
        os.close(self.fd)
        self.fd = -1
        os.rename(self.path, self.target)
        self.committed = True
        try:  # best-effort parent fsync
            dfd = os.open(os.path.dirname(self.target) or ".", os.O_RDONLY | os.O_DIRECTORY)
            try:
                os.fsync(dfd)
            finally:
                os.close(dfd)
        except OSError:
            pass

    def discard(self) -> None:
        if self.fd >= 0:
            os.close(self.fd)
            self.fd = -1
        if not self.committed:
            try:
                os.unlink(self.path)
            except FileNotFoundError:
                pass


class AtomicFile:
    """AtomicFile::new(target)[.with_hash(expected)] (atomic_file.rs:161-463)."""

    def __init__(self, target, ctx: Optional[_capi.Context] = None):
        self.target = str(target)
        self.expected: Optional[int] = None
        self.ctx = ctx

    def with_hash(self, expected: int) -> "AtomicFile":
        self.expected = int(expected)
        return self

    def stream(self, reader) -> None:
        """stream / stream_async: `reader.read(n)` (b"" at EOF) in STREAMING_BUF_SIZE pieces."""
        tmp = _TempFile(self.target)
        h = hasher.Xxh3(self.ctx) if self.expected is not None else None
        try:
            while True:
                chunk = reader.read(STREAMING_BUF_SIZE)
                if not chunk:
                    break
                if h is not None:
                    h.update(chunk)
                tmp.write_all(chunk)
            if h is not None:
                actual = h.digest128()
                if actual != self.expected:
                    raise HashMismatchError(self.target, self.expected, actual)
            tmp.commit()
        finally:
            if h is not None:
                h.close()  # the device stream is released now, not at garbage collection
            tmp.discard()

    def stream_from_paths(self, paths: Sequence) -> None:
        """stream_from_paths (atomic_file.rs:320-351): the in-order concatenation of the files at
        `paths`, one source open at a time, hashed on the GPU as it goes to the temp and published on
        a match -- the reassembly of a chunked upload (LocalVersionStore.combine_version_chunks)."""
        tmp = _TempFile(self.target)
        h = hasher.Xxh3(self.ctx) if self.expected is not None else None
        try:
            for path in paths:
                with open(path, "rb") as src:
                    while True:
                        chunk = src.read(STREAMING_BUF_SIZE)
                        if not chunk:
                            break
                        if h is not None:
                            h.update(chunk)
                        tmp.write_all(chunk)
            if h is not None:
                actual = h.digest128()
                if actual != self.expected:
                    raise HashMismatchError(self.target, self.expected, actual)
            tmp.commit()
        except OSError as e:
            raise OxenError(str(e), _capi.OXH_ERR_IO) from e
        finally:
            if h is not None:
                h.close()
            tmp.discard()

    def write(self, data: bytes) -> None:
        tmp = _TempFile(self.target)
        try:
            tmp.write_all(data)
            if self.expected is not None:
                actual = hasher.hash_buffers_128bit([bytes(data)], self.ctx)[0]
                if actual != self.expected:
                    raise HashMismatchError(self.target, self.expected, actual)
            tmp.commit()
        finally:
            tmp.discard()


def _parse_hash(h: str) -> int:
    """MerkleHash::from_str (merkle_hash.rs:54-61): u128 radix 16."""
    try:
        v = int(h, 16)
    except ValueError:
        raise OxenError(f"invalid digit found in string: {h!r}", _capi.OXH_ERR_INVALID) from None
    if v >> 128:
        raise OxenError("number too large to fit in target type", _capi.OXH_ERR_INVALID)
    return v


def parse_u64(name: str):
    """`name.parse::<u64>()` (Rust core's from_str_radix): an optional '+' then ASCII digits only, below
    2**64; anything else (a '-', whitespace, '_', non-ASCII digits, which Python's int() would accept)
    is None."""
    digits = name[1:] if name.startswith("+") else name
    if not digits or not digits.isascii() or not digits.isdigit():
        return None
    v = int(digits)
    return v if v < (1 << 64) else None


class LocalVersionStore:
    """storage/local.rs: version paths and the verified content-addressed writes."""

    def __init__(self, root_path, ctx: Optional[_capi.Context] = None):
        self.root_path = str(root_path)
        self.ctx = ctx

    def version_dir(self, hash: str) -> str:  # :66-70
        return os.path.join(self.root_path, hash[:2], hash[2:])

    def version_path(self, hash: str) -> str:  # :72-75
        return os.path.join(self.version_dir(hash), VERSION_FILE_NAME)

    def version_exists(self, hash: str) -> bool:  # :259-261
        return os.path.exists(self.version_path(hash))

    def store_version(self, hash: str, data: bytes) -> None:  # :123-139
        if self.version_exists(hash):
            return
        AtomicFile(self.version_path(hash), self.ctx).with_hash(_parse_hash(hash)).write(data)

    def store_version_from_reader(self, hash: str, reader, size: int) -> None:  # :104-121
        del size  # `_size` in the reference too
        if self.version_exists(hash):
            return
        AtomicFile(self.version_path(hash), self.ctx).with_hash(_parse_hash(hash)).stream(reader)

    # chunked uploads (local.rs:78-92, 315-330, 367-413): chunks land under
    # {version_dir}/chunks/{offset}/chunk, unverified; the reassembled blob is verified once
    def version_chunks_dir(self, hash: str) -> str:
        return os.path.join(self.version_dir(hash), VERSION_CHUNKS_DIR)

    def version_chunk_file(self, hash: str, offset: int) -> str:
        return os.path.join(self.version_chunks_dir(hash), str(int(offset)), VERSION_CHUNK_FILE_NAME)

    def store_version_chunk(self, hash: str, offset: int, data: bytes) -> None:  # :315-330
        path = self.version_chunk_file(hash, offset)
        if os.path.exists(path):
            return
        AtomicFile(path, self.ctx).write(data)

    def list_version_chunks(self, hash: str) -> list:  # :367-382
        out = []
        with os.scandir(self.version_chunks_dir(hash)) as it:
            for e in it:
                # DirEntry::file_type() does not follow symlinks; the name must parse as Rust's u64
                if e.is_dir(follow_symlinks=False):
                    v = parse_u64(e.name)
                    if v is not None:
                        out.append(v)
        return sorted(out)

    def combine_version_chunks(self, hash: str) -> None:  # :384-413
        """The chunks in offset order, concatenated, hashed on the GPU and published only if the
        digest is `hash` (HashMismatchError otherwise, and the chunks stay); then the chunks
        directory is removed."""
        import shutil

        expected = _parse_hash(hash)
        paths = [self.version_chunk_file(hash, o) for o in self.list_version_chunks(hash)]
        AtomicFile(self.version_path(hash), self.ctx).with_hash(expected).stream_from_paths(paths)
        shutil.rmtree(self.version_chunks_dir(hash), ignore_errors=False)

    def get_version(self, hash: str) -> bytes:
        with open(self.version_path(hash), "rb") as f:
            return f.read()

    def store_versions(self, hashes: Sequence[str], datas: Sequence[bytes]) -> list:
        """Many received blobs: one batched GPU hash of every buffer, then each verified blob is
        published as store_version would. Returns, per item, None or the OxenError it raised."""
        if len(hashes) != len(datas):
            raise OxenError("hashes and datas differ in length", _capi.OXH_ERR_INVALID)
        got = hasher.hash_buffers_128bit(list(datas), self.ctx)
        errs: list = [None] * len(hashes)
        for i, (h, d) in enumerate(zip(hashes, datas)):
            try:
                if self.version_exists(h):
                    continue
                expected = _parse_hash(h)
                if got[i] != expected:
                    raise HashMismatchError(self.version_path(h), expected, got[i])
                AtomicFile(self.version_path(h), self.ctx).write(d)  # verified above
            except OxenError as e:
                errs[i] = e
        return errs
