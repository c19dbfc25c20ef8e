"""TEST INFRASTRUCTURE ONLY -- FastCDC v2020 oracle (block-level dedup).

Reference call site: experiments/block-level-dedup/src/chunker/fastcdchunker.rs:83-98
(`v2020::FastCDC::new(&content, 4096, chunk_size, 2 * chunk_size)`, then xxh3_128 of every chunk,
named by its DECIMAL u128 string). The algorithm is in the un-vendored crate `fastcdc` 3.2.1.

* `gear_table()` derives the 256-entry GEAR table from the crate's documented generation rule
  (each entry = the first 8 bytes, big-endian, of MD5 over 64 copies of the byte value) with
  Python's hashlib -- independently of the product's compiled-in table.
* `chunks_py()` is a per-byte restatement (hash = (hash << 1) + GEAR[b]; test the mask at every
  byte of the normalised ranges), written differently from the C oracle's two-bytes-per-step loop,
  so the two cross-check each other on small inputs.
* `chunks()` drives the C oracle (oracle/fastcdc_oracle.c) for larger inputs.
Parity against a reference run is PARTLY PINNED: no FastCDC fixtures exist in the reference and the
crate (fastcdc 3.2.1) is neither vendored nor buildable here, but two of the crate's own published
tests are restated in tests/test_fastcdc.py -- `test_all_zeros` (10 chunks of 1 024 B, each cut with
hash 14169102344523991076 = -GEAR[0] mod 2^64: pins GEAR[0], hence the MD5 rule, and the min/max
walk) and `test_masks` (the MASKS entries level 1 picks). Only tests/ may import this module.
"""
from __future__ import annotations

import ctypes
import hashlib
import math
import os

import numpy as np

from . import oracle as _oracle

MASKS = [0, 0, 0, 0, 0,
         0x0000000001804110, 0x0000000001803110, 0x0000000018035100, 0x0000001800035300,
         0x0000019000353000, 0x0000590003530000, 0x0000d90003530000, 0x0000d90103530000,
         0x0000d90303530000, 0x0000d90313530000, 0x0000d90f03530000, 0x0000d90303537000,
         0x0000d90703537000, 0x0000d90707537000, 0x0000d91707537000, 0x0000d91747537000,
         0x0000d91767537000, 0x0000d93767537000, 0x0000d93777537000, 0x0000d93777577000,
         0x0000db3777577000]
M64 = (1 << 64) - 1


def gear_table() -> list[int]:
    return [int.from_bytes(hashlib.md5(bytes([i]) * 64).digest()[:8], "big") for i in range(256)]


def masks(avg: int, level: int = 1) -> tuple[int, int]:
    bits = int(round(math.log2(avg)))
    return MASKS[bits + level], MASKS[bits - level]


def chunks_py(data: bytes, min_size: int, avg: int, max_size: int, level: int = 1) -> list[tuple[int, int]]:
    """Per-byte restatement (small inputs only): [(offset, length)]."""
    gear = gear_table()
    mask_s, mask_l = masks(avg, level)
    out, pos, n = [], 0, len(data)
    while pos < n:
        rem = n - pos
        if rem <= min_size:
            out.append((pos, rem))
            break
        center = avg
        if rem > max_size:
            rem = max_size
        elif rem < center:
            center = rem
        start = (min_size // 2) * 2
        cut, h = rem, 0
        # the two-byte loop tests positions [start, 2*floor(center/2)) with mask_s and
        # [2*floor(center/2), 2*floor(rem/2)) with mask_l, one rolling hash throughout
        for q in range(start, (rem // 2) * 2):
            h = ((h << 1) + gear[data[pos + q]]) & M64
            mask = mask_s if q < (center // 2) * 2 else mask_l
            if h & mask == 0:
                cut = q
                break
        out.append((pos, cut))
        pos += cut
    return out


_bound = False


def _lib():
    global _bound
    L = _oracle.lib()
    if not _bound:
        u64p = ctypes.POINTER(ctypes.c_uint64)
        L.oxo_fastcdc.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                  ctypes.c_uint32, u64p, u64p, u64p, ctypes.c_uint64]
        L.oxo_fastcdc.restype = ctypes.c_uint64
        _bound = True
    return L


_GEAR = None


def chunks(data, min_size: int, avg: int, max_size: int, level: int = 1) -> np.ndarray:
    """C oracle: uint64 array (n, 2) of (offset, length)."""
    global _GEAR
    if _GEAR is None:
        _GEAR = np.array(gear_table(), dtype=np.uint64)
    buf = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else np.ascontiguousarray(data, dtype=np.uint8)
    cap = len(buf) // max(1, min_size) + 2
    offs = np.zeros(cap, dtype=np.uint64)
    lens = np.zeros(cap, dtype=np.uint64)
    u64p = ctypes.POINTER(ctypes.c_uint64)
    n = _lib().oxo_fastcdc(buf.ctypes.data if len(buf) else None, len(buf), min_size, avg, max_size, level,
                           _GEAR.ctypes.data_as(u64p), offs.ctypes.data_as(u64p), lens.ctypes.data_as(u64p), cap)
    assert n <= cap
    return np.stack([offs[:n], lens[:n]], axis=1)


def files(paths, min_size: int, avg: int, max_size: int, level: int = 1, threads: int = 1, mmap_files: bool = False):
    """C oracle over files (oxo_fastcdc_files): the reference's per-file read -> v2020 chunking ->
    xxh3_128 per chunk, `threads` files at a time. Returns (counts (n,), fingerprints (n, 2), status (n,)),
    a file's fingerprint being XXH3-128 of its (offset, length, lo, hi) u64 records (record_fingerprint)."""
    global _GEAR
    if _GEAR is None:
        _GEAR = np.array(gear_table(), dtype=np.uint64)
    L = _lib()
    u64p = ctypes.POINTER(ctypes.c_uint64)
    L.oxo_fastcdc_files.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                    ctypes.c_uint32, ctypes.c_uint32, u64p, ctypes.c_int, ctypes.c_int, u64p, u64p,
                                    ctypes.POINTER(ctypes.c_int32)]
    L.oxo_fastcdc_files.restype = None
    n = len(paths)
    arr = (ctypes.c_char_p * max(n, 1))(*[os.fsencode(p) for p in paths])
    counts = np.zeros(n, dtype=np.uint64)
    fp = np.zeros((n, 2), dtype=np.uint64)
    status = np.zeros(n, dtype=np.int32)
    L.oxo_fastcdc_files(arr, n, min_size, avg, max_size, level, _GEAR.ctypes.data_as(u64p), 1 if mmap_files else 0,
                        int(threads), counts.ctypes.data_as(u64p), fp.ctypes.data_as(u64p),
                        status.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
    return counts, fp, status


def fixed_files(paths, chunk: int, threads: int = 1, mmap_files: bool = False):
    """C oracle over files (oxo_fixed_files): fixedsize_multithreaded.rs:78-110 per file -- chunk i =
    [i*chunk, min((i+1)*chunk, size)), xxh3_128 of each -- `threads` files at a time; returns as files()."""
    L = _lib()
    u64p = ctypes.POINTER(ctypes.c_uint64)
    L.oxo_fixed_files.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int,
                                  ctypes.c_int, u64p, u64p, ctypes.POINTER(ctypes.c_int32)]
    L.oxo_fixed_files.restype = None
    n = len(paths)
    arr = (ctypes.c_char_p * max(n, 1))(*[os.fsencode(p) for p in paths])
    counts = np.zeros(n, dtype=np.uint64)
    fp = np.zeros((n, 2), dtype=np.uint64)
    status = np.zeros(n, dtype=np.int32)
    L.oxo_fixed_files(arr, n, int(chunk), 1 if mmap_files else 0, int(threads), counts.ctypes.data_as(u64p),
                      fp.ctypes.data_as(u64p), status.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
    return counts, fp, status


def record_fingerprint(offsets, lens, digests) -> tuple[int, int]:
    """XXH3-128 (lo, hi) of a chunk table's (offset, length, lo, hi) u64 LE records -- what
    oxo_fastcdc_files reports per file -- for comparing a GPU table against the C oracle at full size."""
    from . import oracle as _o

    rec = np.empty((len(offsets), 4), dtype=np.uint64)
    rec[:, 0], rec[:, 1] = offsets, lens
    rec[:, 2:] = np.asarray(digests, dtype=np.uint64).reshape(-1, 2)
    return _o.xxh3_128(rec.tobytes())
