"""TEST INFRASTRUCTURE ONLY -- ctypes wrapper around the CPU oracle (oracle/xxh3_oracle.c).

The oracle is a scalar C restatement of XXH3-128 (seed 0, default secret), the content hash of
liboxen `util/hasher.rs:28-30`. It is pinned by tests/test_oracle.py against the reference's own
known-answer digest (`repositories/data_frames/schemas.rs:131`) and against the golden vectors in
tests/golden/ (libxxhash 0.8.2). Only tests/, `__graft_entry__.smoke()` and bench.py's
`cpu_baseline` leg may import this module; the product path (oxen_amd) never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "liboxh_oracle.so")
_lib = None

_u64p = ctypes.POINTER(ctypes.c_uint64)
_i32p = ctypes.POINTER(ctypes.c_int32)


def build(force: bool = False) -> str:
    """Compile the oracle with gcc (oracle/Makefile)."""
    srcs = [os.path.join(_HERE, s) for s in ("xxh3_oracle.c", "fastcdc_oracle.c", "Makefile")]
    if force or not os.path.exists(LIB_PATH) or any(os.path.getmtime(LIB_PATH) < os.path.getmtime(s) for s in srcs):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.oxo_xxh3_128.argtypes = [ctypes.c_void_p, ctypes.c_uint64, _u64p]
        L.oxo_xxh3_128.restype = None
        L.oxo_combined_hash.argtypes = [_u64p, _u64p, _u64p]
        L.oxo_combined_hash.restype = None
        L.oxo_xxh3_128_batch.argtypes = [ctypes.c_void_p, _u64p, _u64p, ctypes.c_uint64, _u64p, ctypes.c_int]
        L.oxo_xxh3_128_batch.restype = None
        L.oxo_hash_files.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.c_uint64, _u64p, _u64p, _i32p, ctypes.c_int]
        L.oxo_hash_files.restype = None
        L.oxo_hash_files_stream4k.argtypes = L.oxo_hash_files.argtypes
        L.oxo_hash_files_stream4k.restype = None
        L.oxo_add_files.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.c_uint64, ctypes.c_char_p, _u64p, _u64p,
                                    _i32p, _i32p, ctypes.c_int]
        L.oxo_add_files.restype = None
        L.oxo_set_add_sync.argtypes = [ctypes.c_int]
        L.oxo_set_add_sync.restype = None
        L.oxo_chunk_digests.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, _u64p, ctypes.c_int]
        L.oxo_chunk_digests.restype = None
        L.oxo_format_hex.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_char_p]
        L.oxo_format_hex.restype = ctypes.c_int
        _lib = L
    return _lib


def _ptr(a: np.ndarray, t=_u64p):
    return a.ctypes.data_as(t)


def xxh3_128(data: bytes) -> tuple[int, int]:
    """(low64, high64) of XXH3-128(data)."""
    out = np.zeros(2, dtype=np.uint64)
    buf = ctypes.create_string_buffer(bytes(data), len(data)) if len(data) else None
    lib().oxo_xxh3_128(ctypes.cast(buf, ctypes.c_void_p) if buf is not None else None, len(data), _ptr(out))
    return int(out[0]), int(out[1])


def xxh3_128_int(data: bytes) -> int:
    lo, hi = xxh3_128(data)
    return (hi << 64) | lo


def combined_hash(content: int, metadata: int) -> int:
    c = np.array([content & (2**64 - 1), content >> 64], dtype=np.uint64)
    m = np.array([metadata & (2**64 - 1), metadata >> 64], dtype=np.uint64)
    out = np.zeros(2, dtype=np.uint64)
    lib().oxo_combined_hash(_ptr(c), _ptr(m), _ptr(out))
    return (int(out[1]) << 64) | int(out[0])


def batch(arena: np.ndarray, offsets: np.ndarray, lens: np.ndarray, threads: int = 1) -> np.ndarray:
    """Digests of arena[offsets[i] : offsets[i]+lens[i]] -> uint64 array (n, 2) = (lo, hi)."""
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint64)
    n = len(lens)
    out = np.zeros((n, 2), dtype=np.uint64)
    lib().oxo_xxh3_128_batch(arena.ctypes.data, _ptr(offsets), _ptr(lens), n, _ptr(out), int(threads))
    return out


def hash_files(paths: list[str], threads: int = 1):
    n = len(paths)
    arr = (ctypes.c_char_p * max(n, 1))(*[os.fsencode(p) for p in paths])
    out = np.zeros((n, 2), dtype=np.uint64)
    sizes = np.zeros(n, dtype=np.uint64)
    status = np.zeros(n, dtype=np.int32)
    lib().oxo_hash_files(arr, n, _ptr(out), _ptr(sizes), _ptr(status, _i32p), int(threads))
    return out, sizes, status


def add_files(paths: list[str], versions_root: str, threads: int = 1, sync: bool = True):
    """Reference add loop restated (hash, then store_version_from_reader with verify-before-publish,
    AtomicTempFile's fsync of each blob and its parent; sync=False skips the fsyncs for timing A/Bs)."""
    n = len(paths)
    lib().oxo_set_add_sync(1 if sync else 0)
    arr = (ctypes.c_char_p * max(n, 1))(*[os.fsencode(p) for p in paths])
    out = np.zeros((n, 2), dtype=np.uint64)
    sizes = np.zeros(n, dtype=np.uint64)
    status = np.zeros(n, dtype=np.int32)
    stored = np.zeros(n, dtype=np.int32)
    lib().oxo_add_files(arr, n, os.fsencode(versions_root), _ptr(out), _ptr(sizes), _ptr(status, _i32p),
                        _ptr(stored, _i32p), int(threads))
    return out, sizes, status, stored


def chunk_digests(data: np.ndarray, chunk: int, threads: int = 1) -> np.ndarray:
    data = np.ascontiguousarray(data, dtype=np.uint8)
    n = (len(data) + chunk - 1) // chunk if chunk else 0
    out = np.zeros((n, 2), dtype=np.uint64)
    lib().oxo_chunk_digests(data.ctypes.data, len(data), chunk, _ptr(out), int(threads))
    return out


def format_hex(lo: int, hi: int) -> str:
    buf = ctypes.create_string_buffer(40)
    lib().oxo_format_hex(lo, hi, buf)
    return buf.value.decode()


def clean_corrupted_versions(versions_root: str, dry_run: bool = False, threads: int = 1) -> dict:
    """storage/local.rs:417-610 restated: walk {root}/{prefix}/{suffix}/data, hash every blob with the
    C oracle (fs::read + hash_buffer), compare with prefix+suffix, remove_dir_all mismatches and
    unreadable blobs unless dry_run. Same counting rules as the reference (see include/oxen_hash.h)."""
    import shutil

    errors = 0
    prefixes = []
    for e in os.scandir(versions_root):
        if e.is_dir(follow_symlinks=False):
            prefixes.append(e)
        else:
            errors += 1
    dirs, expected = [], []
    for pre in prefixes:
        try:
            entries = list(os.scandir(pre.path))
        except OSError:
            errors += 1
            continue
        for e in entries:
            if not e.is_dir(follow_symlinks=False):
                continue
            dirs.append(e.path)
            expected.append(pre.name + e.name)
    out, _, status = hash_files([os.path.join(d, "data") for d in dirs], threads=threads)
    scanned = corrupted = cleaned = 0
    for d, exp, (lo, hi), st in zip(dirs, expected, out, status):
        if st != 0:
            errors += 1
            if not dry_run:
                try:
                    shutil.rmtree(d)
                    cleaned += 1
                except OSError:
                    pass
            continue
        scanned += 1
        if format((int(hi) << 64) | int(lo), "x") == exp:
            continue
        corrupted += 1
        if not dry_run:
            try:
                shutil.rmtree(d)
                cleaned += 1
            except OSError:
                errors += 1
    return {"scanned": scanned, "corrupted": corrupted, "cleaned": cleaned, "errors": errors}


def is_utf8_prefix(data: bytes) -> bool:
    """util/fs.rs:652-668 (is_utf8) on bytes already read: the first min(len, 4096) bytes decode as
    UTF-8, or the first error is a sequence cut off by the end ("unexpected end of data" = Rust's
    Utf8Error::error_len() == None). Python's strict UTF-8 decoder (no surrogates, no overlongs,
    <= U+10FFFF) applies the same validity rules as core::str::from_utf8."""
    b = bytes(data[:4096])
    if not b:
        return True
    try:
        b.decode("utf-8")
        return True
    except UnicodeDecodeError as e:
        return e.reason == "unexpected end of data"


def is_utf8_prefix_dfa(data: bytes) -> bool:
    """The same predicate as core::str::run_utf8_validation walks it (second-byte ranges per lead),
    restated independently of Python's decoder; tests cross-check the two."""
    b = bytes(data[:4096])
    i, n = 0, len(b)
    second = {0xE0: (0xA0, 0xBF), 0xED: (0x80, 0x9F), 0xF0: (0x90, 0xBF), 0xF4: (0x80, 0x8F)}
    while i < n:
        c = b[i]
        if c < 0x80:
            i += 1
            continue
        width = 2 if 0xC2 <= c <= 0xDF else 3 if 0xE0 <= c <= 0xEF else 4 if 0xF0 <= c <= 0xF4 else 0
        if width == 0:
            return False
        lo, hi = second.get(c, (0x80, 0xBF))
        for k in range(1, width):
            if i + k >= n:
                return True  # cut off by the end of the prefix
            x = b[i + k]
            if not ((lo <= x <= hi) if k == 1 else (0x80 <= x <= 0xBF)):
                return False
        i += width
    return True
