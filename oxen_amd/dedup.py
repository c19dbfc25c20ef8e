"""Block-level dedup chunkers on the GPU.

Fixed-size chunkers (experiments/block-level-dedup/src/chunker/fixedsize.rs, `FixedSizeChunker`, and
fixedsize_multithreaded.rs, `FixedSizeMultiChunker`): a file is cut into chunk_size pieces (the last
one shorter), each piece is named by the decimal xxh3_128 of its bytes and written to output_dir
unless a chunk of that name exists; metadata.bin lists the names (bincode). Here the file is read in
segments of whole chunks, each segment goes to the device once and `oxh_chunk_digests_device` hashes
all its chunks in one launch; the chunk files are written by `concurrency` host threads.

FastCDC (fastcdchunker.rs, `FastCDChunker`): the file is
chunked with FastCDC v2020 (min 4096, avg = chunk_size, max = 2 * chunk_size, :55-57, :83-88) and
every chunk is written to `output_dir/<decimal xxh3_128 of the chunk>` (:96-107); the chunk names go
to `metadata.bin` as bincode 1.x of `ChunkMetadata {original_file_name: String, original_file_size:
u64, chunks: Vec<String>}` (:11-16, :110-121). Boundaries and digests both come from the GPU
(`oxh_fastcdc_device`: FastCDC candidate scan + speculative walks + K1 over the chunk table).
"""
from __future__ import annotations

import ctypes
import os
import struct
from typing import Optional

import numpy as np
import torch

from . import _capi
from .device import fastcdc_device, to_numpy_u64

METADATA_FILE_NAME = "metadata.bin"  # fastcdchunker.rs:18
MIN_CHUNK_SIZE = 4096                # fastcdchunker.rs:55


def chunk_name(lo: int, hi: int) -> str:
    """u128::to_string() of the chunk digest (fastcdchunker.rs:98)."""
    return str((int(hi) << 64) | int(lo))


def _bincode_string(s: str) -> bytes:
    b = s.encode("utf-8")
    return struct.pack("<Q", len(b)) + b


def encode_metadata(original_file_name: str, original_file_size: int, chunks: list[str]) -> bytes:
    """bincode 1.x default (fixint, little-endian, u64 lengths) of ChunkMetadata."""
    out = [_bincode_string(original_file_name), struct.pack("<Q", original_file_size), struct.pack("<Q", len(chunks))]
    out += [_bincode_string(c) for c in chunks]
    return b"".join(out)


class _Bincode:
    """A reader over bincode 1.x default encoding (fixint, little-endian, u64 lengths)."""

    def __init__(self, buf: bytes):
        self.buf, self.pos = buf, 0

    def take(self, n: int) -> bytes:
        if self.pos + n > len(self.buf):
            raise _capi.OxenError("Bincode error: unexpected end of metadata", _capi.OXH_ERR_IO)
        v = self.buf[self.pos:self.pos + n]
        self.pos += n
        return v

    def u64(self) -> int:
        return struct.unpack("<Q", self.take(8))[0]

    def u8(self) -> int:
        return self.take(1)[0]

    def string(self) -> str:
        return self.take(self.u64()).decode("utf-8")

    def strings(self) -> list[str]:
        return [self.string() for _ in range(self.u64())]


def decode_metadata(buf: bytes) -> tuple[str, int, list[str]]:
    r = _Bincode(buf)
    name = r.string()
    size = r.u64()
    return name, size, r.strings()


def _strings(items: list[str]) -> bytes:
    return struct.pack("<Q", len(items)) + b"".join(_bincode_string(c) for c in items)


def encode_fixed_metadata(original_file_name: str, original_file_size: int, chunk_size: int, chunks: list[str]) -> bytes:
    """fixedsize_multithreaded.rs:14-20 ChunkMetadata {original_file_name, original_file_size: u64,
    chunk_size: usize, chunks: Vec<String>} in bincode 1.x."""
    return (_bincode_string(original_file_name) + struct.pack("<QQ", original_file_size, chunk_size) + _strings(chunks))


def decode_fixed_metadata(buf: bytes) -> tuple[str, int, int, list[str]]:
    r = _Bincode(buf)
    name = r.string()
    size, chunk = r.u64(), r.u64()
    return name, size, chunk, r.strings()


def encode_archive_metadata(chunk_size: int, entries: list[dict]) -> bytes:
    """fixedsize.rs:22-35 ArchiveMetadata {chunk_size: usize, entries: Vec<ArchiveEntry {path: PathBuf,
    is_dir: bool, chunks: Option<Vec<String>>, size: Option<u64>}>} in bincode 1.x (Option = u8 tag)."""
    out = [struct.pack("<QQ", chunk_size, len(entries))]
    for e in entries:
        out.append(_bincode_string(e["path"]))
        out.append(b"\x01" if e["is_dir"] else b"\x00")
        out.append(b"\x00" if e["chunks"] is None else b"\x01" + _strings(e["chunks"]))
        out.append(b"\x00" if e["size"] is None else b"\x01" + struct.pack("<Q", e["size"]))
    return b"".join(out)


def decode_archive_metadata(buf: bytes) -> tuple[int, list[dict]]:
    r = _Bincode(buf)
    chunk = r.u64()
    entries = []
    for _ in range(r.u64()):
        path = r.string()
        is_dir = r.u8() != 0
        chunks = r.strings() if r.u8() else None
        size = r.u64() if r.u8() else None
        entries.append({"path": path, "is_dir": is_dir, "chunks": chunks, "size": size})
    return chunk, entries


class FastCdcTable:
    """A chunk table in host memory: chunk k = bytes [offsets[k], offsets[k] + lens[k]) of its file,
    digests[k] = (lo, hi) of its XXH3-128 (None when not asked for); file i's chunks are rows
    first[i] .. first[i+1]-1. sizes / status / os_error per file (oxh_fastcdc_files)."""

    def __init__(self, offsets, lens, digests, first, sizes=None, status=None, os_error=None):
        self.offsets, self.lens, self.digests, self.first = offsets, lens, digests, first
        self.sizes, self.status, self.os_error = sizes, status, os_error

    def file(self, i: int):
        a, b = int(self.first[i]), int(self.first[i + 1])
        return self.offsets[a:b], self.lens[a:b], (self.digests[a:b] if self.digests is not None else None)


def _need_from_error(e: _capi.OxenError) -> Optional[int]:
    import re

    m = re.search(r"need (\d+) entries", str(e))
    return int(m.group(1)) if m and e.code == _capi.OXH_ERR_INVALID else None


def _ctx_array(ctxs):
    arr = (ctypes.c_void_p * len(ctxs))(*[c.handle.value if isinstance(c.handle, ctypes.c_void_p) else c.handle
                                          for c in ctxs])
    return arr


def fastcdc_files(paths, min_size: int, avg_size: int, max_size: int, level: int = 1, digests: bool = True,
                  ctx: Optional[_capi.Context] = None, ctxs=None) -> FastCdcTable:
    """oxh_fastcdc_files: FastCDC v2020 boundaries and XXH3-128 chunk digests of files on disk, read by
    the library (fastcdchunker.rs:75-98: fs::read, v2020 chunking, xxh3_128 per chunk), results in
    host memory. A file that cannot be opened / read has no chunks and its status / errno set.
    ctxs (several contexts, e.g. one per device): oxh_fastcdc_files_multi, the files shared out."""
    from .hasher import _PathTable, default_context

    ctx = ctx or (None if ctxs else default_context())
    n = len(paths)
    sizes_hint = np.zeros(n, dtype=np.uint64)
    for i, p in enumerate(paths):
        try:
            sizes_hint[i] = os.stat(p).st_size
        except OSError:
            pass
    L = _capi.lib()
    cap = max(1, int(L.oxh_fastcdc_max_chunks(sizes_hint.ctypes.data_as(_capi._u64p), n, max(1, int(min_size)))))
    table = _PathTable(paths) if n else None
    for _ in range(3):  # a file that grew since the stat above needs a larger table: retry with the count
        off = np.zeros(cap, dtype=np.uint64)
        ln = np.zeros(cap, dtype=np.uint64)
        dig = np.zeros((cap, 2), dtype=np.uint64) if digests else None
        first = np.zeros(n + 1, dtype=np.uint64)
        sizes = np.zeros(n, dtype=np.uint64)
        status = np.zeros(n, dtype=np.int32)
        oserr = np.zeros(n, dtype=np.int32)
        tail = (int(min_size), int(avg_size), int(max_size), int(level), off.ctypes.data_as(_capi._u64p),
                ln.ctypes.data_as(_capi._u64p), dig.ctypes.data_as(_capi._u64p) if dig is not None else None, cap,
                first.ctypes.data_as(_capi._u64p), sizes.ctypes.data_as(_capi._u64p), status.ctypes.data_as(_capi._i32p),
                oserr.ctypes.data_as(_capi._i32p))
        if ctxs:
            rc = L.oxh_fastcdc_files_multi(_ctx_array(ctxs), len(ctxs), table.arg if table else None, n, *tail)
        else:
            rc = L.oxh_fastcdc_files(ctx.handle, table.arg if table else None, n, *tail)
        try:
            _capi.check(rc, "oxh_fastcdc_files")
        except _capi.OxenError as e:
            need = _need_from_error(e)
            if need is None:
                raise
            cap = need
            continue
        total = int(first[n])
        return FastCdcTable(off[:total], ln[:total], dig[:total] if dig is not None else None, first, sizes, status, oserr)
    raise _capi.OxenError("oxh_fastcdc_files: the files keep growing", _capi.OXH_ERR_INVALID)


def fastcdc_host(buffers, min_size: int, avg_size: int, max_size: int, level: int = 1, digests: bool = True,
                 ctx: Optional[_capi.Context] = None, ctxs=None) -> FastCdcTable:
    """oxh_fastcdc_host: the same over host buffers (bytes / numpy uint8 arrays); ctxs: over several
    contexts (oxh_fastcdc_host_multi)."""
    from .hasher import default_context

    ctx = ctx or (None if ctxs else default_context())
    arrs = [np.frombuffer(b, dtype=np.uint8) if isinstance(b, (bytes, bytearray, memoryview)) else np.ascontiguousarray(b, dtype=np.uint8)
            for b in buffers]
    n = len(arrs)
    lens_in = np.array([a.size for a in arrs], dtype=np.uint64)
    ptrs = (ctypes.c_char_p * max(n, 1))(*[ctypes.cast(a.ctypes.data, ctypes.c_char_p) if a.size else None for a in arrs])
    L = _capi.lib()
    cap = max(1, int(L.oxh_fastcdc_max_chunks(lens_in.ctypes.data_as(_capi._u64p), n, max(1, int(min_size)))))
    off = np.zeros(cap, dtype=np.uint64)
    ln = np.zeros(cap, dtype=np.uint64)
    dig = np.zeros((cap, 2), dtype=np.uint64) if digests else None
    first = np.zeros(n + 1, dtype=np.uint64)
    tail = (lens_in.ctypes.data_as(_capi._u64p), n, int(min_size), int(avg_size), int(max_size), int(level),
            off.ctypes.data_as(_capi._u64p), ln.ctypes.data_as(_capi._u64p),
            dig.ctypes.data_as(_capi._u64p) if dig is not None else None, cap, first.ctypes.data_as(_capi._u64p))
    if ctxs:
        _capi.check(L.oxh_fastcdc_host_multi(_ctx_array(ctxs), len(ctxs), ptrs, *tail), "oxh_fastcdc_host_multi")
    else:
        _capi.check(L.oxh_fastcdc_host(ctx.handle, ptrs, *tail), "oxh_fastcdc_host")
    total = int(first[n])
    return FastCdcTable(off[:total], ln[:total], dig[:total] if dig is not None else None, first)


class FixedChunkTable:
    """Fixed-size chunk digests in host memory (oxh_chunk_digests_files / _host): digests[k] = (lo, hi)
    of chunk k; file i's chunks are rows first[i] .. first[i+1]-1, chunk j of a file being its bytes
    [j*chunk, min((j+1)*chunk, size)). sizes / status / os_error per file (files only)."""

    def __init__(self, digests, first, sizes=None, status=None, os_error=None):
        self.digests, self.first, self.sizes, self.status, self.os_error = digests, first, sizes, status, os_error

    def file(self, i: int):
        return self.digests[int(self.first[i]):int(self.first[i + 1])]


def _fixed_count(sizes, chunk: int) -> int:
    return int(sum((int(x) + chunk - 1) // chunk for x in sizes))


# Measured rates behind INTEGRATION.md §2 "When NOT to call the host chunk entries" (DESIGN §5,
# profiles/r05/r05j_fixed_e2e_*, r05as_h2d_probe.json): host-resident bytes cross one PCIe link per GPU
# first (~49 GiB/s each, the host entries at 92-93 % of the link), the reference's CPU loops hash at
# these rates per core (16 threads: fixed-size 67.7 GiB/s, FastCDC 34.9-40.3 GiB/s).
LINK_GIBS = 49.0
CPU_GIBS_PER_CORE = {"fixed": 4.2, "fastcdc": 2.4}


def host_entry_pays_off(host_cores: int, links: int, fastcdc: bool) -> bool:
    """Whether chunk_digests_files / fastcdc_files (and _multi) beat the reference's own CPU loop for
    host-resident files on this node: links x LINK_GIBS against host_cores x the per-core rate. A
    routing rule for the caller (bytes already in HBM take the device entries regardless); the library
    itself has no CPU hashing path."""
    cpu = host_cores * CPU_GIBS_PER_CORE["fastcdc" if fastcdc else "fixed"]
    return links * LINK_GIBS > cpu


def chunk_digests_files(paths, chunk_size: int, ctx: Optional[_capi.Context] = None, ctxs=None) -> FixedChunkTable:
    """oxh_chunk_digests_files: XXH3-128 of every fixed-size chunk of files on disk, read by the library
    (fixedsize_multithreaded.rs:78-110), digests in host memory; per-file errors as fastcdc_files.
    ctxs: oxh_chunk_digests_files_multi over several contexts."""
    from .hasher import _PathTable, default_context

    if chunk_size <= 0:
        raise _capi.OxenError("Chunk size cannot be zero", _capi.OXH_ERR_INVALID)
    ctx = ctx or (None if ctxs else default_context())
    n = len(paths)
    hint = []
    for p in paths:
        try:
            hint.append(os.stat(p).st_size)
        except OSError:
            hint.append(0)
    cap = max(1, _fixed_count(hint, chunk_size))
    table = _PathTable(paths) if n else None
    L = _capi.lib()
    for _ in range(3):  # a file that grew since the stat above: retry with the count the call reports
        dig = np.zeros((cap, 2), dtype=np.uint64)
        first = np.zeros(n + 1, dtype=np.uint64)
        sizes = np.zeros(n, dtype=np.uint64)
        status = np.zeros(n, dtype=np.int32)
        oserr = np.zeros(n, dtype=np.int32)
        tail = (int(chunk_size), dig.ctypes.data_as(_capi._u64p), cap, first.ctypes.data_as(_capi._u64p),
                sizes.ctypes.data_as(_capi._u64p), status.ctypes.data_as(_capi._i32p), oserr.ctypes.data_as(_capi._i32p))
        if ctxs:
            rc = L.oxh_chunk_digests_files_multi(_ctx_array(ctxs), len(ctxs), table.arg if table else None, n, *tail)
        else:
            rc = L.oxh_chunk_digests_files(ctx.handle, table.arg if table else None, n, *tail)
        try:
            _capi.check(rc, "oxh_chunk_digests_files")
        except _capi.OxenError as e:
            need = _need_from_error(e)
            if need is None:
                raise
            cap = need
            continue
        return FixedChunkTable(dig[:int(first[n])], first, sizes, status, oserr)
    raise _capi.OxenError("oxh_chunk_digests_files: the files keep growing", _capi.OXH_ERR_INVALID)


def chunk_digests_host(buffers, chunk_size: int, ctx: Optional[_capi.Context] = None, ctxs=None) -> FixedChunkTable:
    """oxh_chunk_digests_host: the same over host buffers (bytes / numpy uint8 arrays); ctxs: over
    several contexts (oxh_chunk_digests_host_multi)."""
    from .hasher import default_context

    if chunk_size <= 0:
        raise _capi.OxenError("Chunk size cannot be zero", _capi.OXH_ERR_INVALID)
    ctx = ctx or (None if ctxs else default_context())
    arrs = [np.frombuffer(b, dtype=np.uint8) if isinstance(b, (bytes, bytearray, memoryview)) else np.ascontiguousarray(b, dtype=np.uint8)
            for b in buffers]
    n = len(arrs)
    lens_in = np.array([a.size for a in arrs], dtype=np.uint64)
    ptrs = (ctypes.c_char_p * max(n, 1))(*[ctypes.cast(a.ctypes.data, ctypes.c_char_p) if a.size else None for a in arrs])
    cap = max(1, _fixed_count(lens_in, chunk_size))
    dig = np.zeros((cap, 2), dtype=np.uint64)
    first = np.zeros(n + 1, dtype=np.uint64)
    tail = (lens_in.ctypes.data_as(_capi._u64p), n, int(chunk_size), dig.ctypes.data_as(_capi._u64p), cap,
            first.ctypes.data_as(_capi._u64p))
    if ctxs:
        _capi.check(_capi.lib().oxh_chunk_digests_host_multi(_ctx_array(ctxs), len(ctxs), ptrs, *tail),
                    "oxh_chunk_digests_host_multi")
    else:
        _capi.check(_capi.lib().oxh_chunk_digests_host(ctx.handle, ptrs, *tail), "oxh_chunk_digests_host")
    return FixedChunkTable(dig[:int(first[n])], first)


# fixedsize.rs:67-91 reads through `BufReader::new(File)` (8 KiB buffer) and stops at the first read
# shorter than chunk_size. BufReader::read serves a request from what is buffered (refilling with one
# 8 KiB read when empty) unless the buffer is empty and the request is >= 8 KiB, which goes to the
# file directly; Linux returns at most MAX_RW_COUNT (0x7ffff000) bytes from one read(2).
BUFREADER_CAPACITY = 8192
MAX_RW_COUNT = 0x7FFFF000


def bufreader_prefix(size: int, chunk: int) -> int:
    """Bytes of a `size`-byte regular file that fixedsize.rs's loop chunks (its chunks are then the
    fixed-size chunks of that prefix): the whole file unless chunk < 8 KiB does not divide 8 KiB (the
    read after the last whole chunk of the first buffer comes back short: the file stops at 8 KiB) or
    chunk > MAX_RW_COUNT (the first read comes back short)."""
    if chunk < BUFREADER_CAPACITY:
        return min(size, BUFREADER_CAPACITY) if BUFREADER_CAPACITY % chunk else size
    return min(size, MAX_RW_COUNT) if chunk > MAX_RW_COUNT else size


class FastCDChunker:
    """fastcdchunker.rs:30-66 + the Chunker trait (chunker.rs): name / pack / unpack / get_chunk_hashes."""

    def __init__(self, chunk_size: int, concurrency: int = 1, device: Optional[str] = None):
        if chunk_size == 0:
            raise ValueError("Chunk size cannot be zero")
        if concurrency == 0:
            raise ValueError("Concurrency must be greater than zero")
        self.min_chunk_size = MIN_CHUNK_SIZE
        self.avg_chunk_size = int(chunk_size)
        self.max_chunk_size = int(chunk_size) * 2
        self.device = device or "cuda"

    def name(self) -> str:
        return "fastcdc-chunker"

    def chunk_buffer(self, data: torch.Tensor):
        """(offsets, lengths, digests) of one device-resident buffer, as numpy uint64 arrays."""
        c_off, c_len, dig, _ = fastcdc_device(data, [0], [data.numel()], self.min_chunk_size, self.avg_chunk_size,
                                              self.max_chunk_size)
        return to_numpy_u64(c_off), to_numpy_u64(c_len), to_numpy_u64(dig).reshape(-1, 2)

    def pack(self, input_file: str, output_dir: str, ctx: Optional[_capi.Context] = None) -> str:
        """fastcdchunker.rs:72-122. The library reads the file (oxh_fastcdc_files: its bytes stream to
        the device once; boundaries and chunk digests come back to host memory); the chunk files are
        then written from a read-only map of the input, as the reference writes its slices."""
        import errno as _errno
        import mmap

        os.makedirs(output_dir, exist_ok=True)
        tab = fastcdc_files([input_file], self.min_chunk_size, self.avg_chunk_size, self.max_chunk_size, ctx=ctx)
        if int(tab.status[0]) != _capi.OXH_OK:  # fs::read(input_file)? (:75): the io::Error
            e = int(tab.os_error[0]) or _errno.EIO
            raise OSError(e, os.strerror(e), input_file)
        size = os.stat(input_file).st_size  # input_file.metadata()?.len() (:77-78)
        names = []
        with open(input_file, "rb") as fh:
            content = mmap.mmap(fh.fileno(), 0, access=mmap.ACCESS_READ) if size else b""
            try:
                for o, l, (lo, hi) in zip(tab.offsets, tab.lens, tab.digests):
                    name = chunk_name(lo, hi)
                    names.append(name)
                    with open(os.path.join(output_dir, name), "wb") as out:
                        out.write(content[int(o):int(o) + int(l)])
            finally:
                if size:
                    content.close()
        base = os.path.basename(os.path.normpath(input_file)) or "unknown_file"
        with open(os.path.join(output_dir, METADATA_FILE_NAME), "wb") as meta:
            meta.write(encode_metadata(base, size, names))
        return output_dir

    def unpack(self, input_dir: str, output_path: str) -> str:
        """fastcdchunker.rs:123-126: the reference's unpack is a stub -- it prints and returns
        output_path without writing anything (so its `Test` command fails to hash the unpacked file).
        Kept as such; `restore` is the working inverse."""
        print(f"To Implement: Unpacking files from {input_dir!r}")
        return output_path

    def restore(self, input_dir: str, output_path: str) -> str:
        """Not in the reference: concatenate the chunks listed in metadata.bin into output_path."""
        _, _, chunks = decode_metadata(open(os.path.join(input_dir, METADATA_FILE_NAME), "rb").read())
        with open(output_path, "wb") as out:
            for c in chunks:
                with open(os.path.join(input_dir, c), "rb") as fh:
                    out.write(fh.read())
        return output_path

    def get_chunk_hashes(self, input_dir: str) -> list[str]:
        return decode_metadata(open(os.path.join(input_dir, METADATA_FILE_NAME), "rb").read())[2]


class _FixedSizeBase:
    """Shared by both fixed-size chunkers: a file -> its chunk names, chunks written as they are named."""

    def __init__(self, chunk_size: int, concurrency: int = 1, device: Optional[str] = None):
        if chunk_size == 0:
            raise ValueError("Chunk size cannot be zero")
        if concurrency == 0:
            raise ValueError("Concurrency must be greater than zero")
        self.chunk_size = int(chunk_size)
        self.concurrency = int(concurrency)
        self.device = device or "cuda"

    def _prefix(self, size: int) -> int:
        """Bytes of the file the reference chunks (all of them; FixedSizeChunker overrides)."""
        return size

    def chunk_file(self, path: str, output_dir: str) -> list[str]:
        """Decimal xxh3_128 names of the file's chunks; a chunk file is written unless one of that
        name exists (fixedsize.rs:78-89, fixedsize_multithreaded.rs:95-105). The library reads the file
        and returns the digests (oxh_chunk_digests_files); the chunk files are written from a read-only
        map of it by `concurrency` threads."""
        import errno as _errno
        import mmap
        from concurrent.futures import ThreadPoolExecutor

        size = os.stat(path).st_size
        pre = self._prefix(size)
        if pre == size:
            tab = chunk_digests_files([path], self.chunk_size)
            if int(tab.status[0]) != _capi.OXH_OK:  # File::open / read: the io::Error
                e = int(tab.os_error[0]) or _errno.EIO
                raise OSError(e, os.strerror(e), path)
            size = int(tab.sizes[0])
            dig = tab.digests
        else:  # the reference's loop stops early: chunk the prefix it reads
            with open(path, "rb") as fh:
                head = fh.read(pre)
            dig = chunk_digests_host([head], self.chunk_size).digests
        names = [chunk_name(lo, hi) for lo, hi in dig.tolist()]
        if not names:
            return names
        with open(path, "rb") as fh:
            content = mmap.mmap(fh.fileno(), 0, access=mmap.ACCESS_READ)
            try:
                def write(k):
                    p = os.path.join(output_dir, names[k])
                    if not os.path.exists(p):
                        lo = k * self.chunk_size
                        with open(p, "wb") as out:
                            out.write(content[lo:min(pre, lo + self.chunk_size)])

                with ThreadPoolExecutor(self.concurrency) as ex:
                    list(ex.map(write, range(len(names))))
            finally:
                content.close()
        return names


class FixedSizeChunker(_FixedSizeBase):
    """fixedsize.rs:37-296 + the Chunker trait: packs a file or a whole directory tree (entries in
    read_dir order, a directory's entry before its contents) into chunk files + ArchiveMetadata."""

    def __init__(self, chunk_size: int, device: Optional[str] = None):
        super().__init__(chunk_size, 1, device)

    def name(self) -> str:
        return "fixed-size-chunker"

    def _prefix(self, size: int) -> int:
        return bufreader_prefix(size, self.chunk_size)

    def _file_entry(self, path: str, base: str, output_dir: str) -> dict:
        chunks = self.chunk_file(path, output_dir)
        return {"path": os.path.relpath(path, base), "is_dir": False, "chunks": chunks, "size": os.stat(path).st_size}

    def _walk(self, cur: str, base: str, output_dir: str, entries: list) -> None:
        with os.scandir(cur) as it:  # read_dir order (fixedsize.rs:116)
            for e in it:
                if e.is_dir():  # metadata() follows symlinks, as here
                    entries.append({"path": os.path.relpath(e.path, base), "is_dir": True, "chunks": None, "size": None})
                    self._walk(e.path, base, output_dir, entries)
                elif e.is_file():
                    entries.append(self._file_entry(e.path, base, output_dir))

    def pack(self, input_path: str, output_dir: str) -> str:
        os.makedirs(output_dir, exist_ok=True)
        entries: list = []
        if os.path.isfile(input_path):
            base = os.path.dirname(os.path.abspath(input_path))
            entries.append(self._file_entry(os.path.abspath(input_path), base, output_dir))
        elif os.path.isdir(input_path):
            entries.append({"path": ".", "is_dir": True, "chunks": None, "size": None})
            self._walk(input_path, input_path, output_dir, entries)
        else:
            raise _capi.OxenError("Input path must be a file or a directory", _capi.OXH_ERR_INVALID)
        with open(os.path.join(output_dir, METADATA_FILE_NAME), "wb") as f:
            f.write(encode_archive_metadata(self.chunk_size, entries))
        return output_dir

    def unpack(self, chunk_dir: str, output_dir: str) -> str:
        _, entries = decode_archive_metadata(open(os.path.join(chunk_dir, METADATA_FILE_NAME), "rb").read())
        os.makedirs(output_dir, exist_ok=True)
        for e in entries:
            out = os.path.join(output_dir, e["path"])
            if e["is_dir"]:
                os.makedirs(out, exist_ok=True)
                continue
            os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
            with open(out, "wb") as fh:
                for c in e["chunks"] or []:
                    p = os.path.join(chunk_dir, c)
                    if not os.path.exists(p):
                        raise FileNotFoundError(f"Chunk file not found during unpack: {p}")
                    with open(p, "rb") as ch:
                        fh.write(ch.read())
        return output_dir

    def get_chunk_hashes(self, input_dir: str) -> list[str]:
        _, entries = decode_archive_metadata(open(os.path.join(input_dir, METADATA_FILE_NAME), "rb").read())
        return [c for e in entries if not e["is_dir"] for c in (e["chunks"] or [])]


class FixedSizeMultiChunker(_FixedSizeBase):
    """fixedsize_multithreaded.rs:24-245 (the reference's rayon pool of `concurrency`): one file ->
    chunk files + ChunkMetadata {original_file_name, original_file_size, chunk_size, chunks}."""

    def name(self) -> str:
        return "fixed-size-64k-multithreaded"

    def pack(self, input_file: str, output_dir: str) -> str:
        os.makedirs(output_dir, exist_ok=True)
        try:
            size = os.stat(input_file).st_size
        except OSError as e:
            raise FileNotFoundError(f"Failed to read input file metadata '{input_file}': {e}") from e
        names = self.chunk_file(input_file, output_dir) if size else []
        base = os.path.basename(os.path.normpath(input_file)) or "unknown_file"
        with open(os.path.join(output_dir, METADATA_FILE_NAME), "wb") as f:
            f.write(encode_fixed_metadata(base, size, self.chunk_size, names))
        return output_dir

    def unpack(self, chunk_dir: str, output_path: str) -> str:
        _, _, _, chunks = decode_fixed_metadata(open(os.path.join(chunk_dir, METADATA_FILE_NAME), "rb").read())
        with open(output_path, "wb") as out:
            for c in chunks:
                p = os.path.join(chunk_dir, c)
                if not os.path.exists(p):
                    raise FileNotFoundError(f"Chunk file not found during unpack: {p}")
                with open(p, "rb") as fh:
                    out.write(fh.read())
        return output_path

    def get_chunk_hashes(self, input_dir: str) -> list[str]:
        return decode_fixed_metadata(open(os.path.join(input_dir, METADATA_FILE_NAME), "rb").read())[3]


def get_chunker(algorithm: str, chunk_size: int):
    """chunker.rs:60-124 get_chunker: "fixed-size", "fixed-size-multithreaded" (16 threads) and
    "fastcdc" (the "copier" baseline copies files and hashes nothing: not on this path)."""
    if algorithm == "fixed-size":
        return FixedSizeChunker(chunk_size)
    if algorithm == "fixed-size-multithreaded":
        return FixedSizeMultiChunker(chunk_size, 16)
    if algorithm == "fastcdc":
        return FastCDChunker(chunk_size, 16)
    raise _capi.OxenError(f"Chunker '{algorithm}' not found", _capi.OXH_ERR_INVALID)


def fastcdc_gear() -> list[int]:
    """The GEAR table compiled into the library (host call, no GPU needed)."""
    out = np.zeros(256, dtype=np.uint64)
    _capi.check(_capi.lib().oxh_fastcdc_gear(out.ctypes.data_as(_capi._u64p)), "oxh_fastcdc_gear")
    return [int(v) for v in out]


def fastcdc_masks(avg_size: int, level: int = 1) -> tuple[int, int]:
    s = np.zeros(1, dtype=np.uint64)
    l = np.zeros(1, dtype=np.uint64)
    _capi.check(_capi.lib().oxh_fastcdc_masks(int(avg_size), int(level), s.ctypes.data_as(_capi._u64p),
                                              l.ctypes.data_as(_capi._u64p)), "oxh_fastcdc_masks")
    return int(s[0]), int(l[0])


def hash_file_128bit(path) -> int:
    """xhash.rs:6-20: File::open, 8 KiB BufReader reads into Xxh3, digest128 -- the XXH3-128 of the
    whole file, here read and hashed by the library (oxh_hash_files_ex). The io::Error of the open /
    read comes back as OSError."""
    import errno as _errno

    from .hasher import hash_files_with_errors_128bit

    digests, _, status, oserr = hash_files_with_errors_128bit([os.fspath(path)])
    if status[0] != _capi.OXH_OK:
        e = int(oserr[0]) or _errno.EIO
        raise OSError(e, os.strerror(e), os.fspath(path))
    return int(digests[0])


class VerificationFailed(Exception):
    """FrameworkError::VerificationFailed (main.rs:232-234)."""


def run_chunker_test(algorithm: str, chunk_size: int, input_file: str, base_dir: Optional[str] = None) -> dict:
    """main.rs:156-241, `Commands::Test`: pack input_file into base_dir/chunker_test_<ns>, unpack it to
    <that dir>/unpacked_output, time both, then compare hash_file_128bit of the original and of the
    unpacked file (VerificationFailed when they differ; a failed hash is "Failed to hash ... file")."""
    import time

    chunker = get_chunker(algorithm, chunk_size)
    base = base_dir if base_dir is not None else os.getcwd()
    test_dir = os.path.join(base, f"chunker_test_{time.time_ns()}")
    os.makedirs(test_dir, exist_ok=True)
    t0 = time.perf_counter()
    chunker.pack(input_file, test_dir)
    pack_s = time.perf_counter() - t0
    unpacked = os.path.join(test_dir, "unpacked_output")
    t0 = time.perf_counter()
    chunker.unpack(test_dir, unpacked)
    unpack_s = time.perf_counter() - t0
    try:
        original = hash_file_128bit(input_file)
    except OSError as e:
        raise _capi.OxenError(f"Failed to hash original file: {e}", _capi.OXH_ERR_IO) from e
    try:
        restored = hash_file_128bit(unpacked)
    except OSError as e:
        raise _capi.OxenError(f"Failed to hash unpacked file: {e}", _capi.OXH_ERR_IO) from e
    if original != restored:
        raise VerificationFailed("Verification FAILED: Unpacked file does NOT match original.")
    return {"test_dir": test_dir, "pack_s": pack_s, "unpack_s": unpack_s, "original_file_hash": str(original)}
