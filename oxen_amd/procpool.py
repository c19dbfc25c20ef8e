"""Process-sharded file hashing over the C ABI's reader-process pool (`oxh_pool_*`,
include/oxen_hash.h; implementation oxen_amd/csrc/reader_pool.cpp + the helper process
oxen_amd/oxh_hash_helper).

Why processes: on the MI355X boxes the warm-cache floor of the `oxen add` read is open + close
themselves, and that floor belongs to the process -- 200 000 open + close pairs take 0.28 s in one
process whatever its thread count, 0.16 s in two and 0.13 s in four or more (tools/open_probe.cpp
with PROCS=P, profiles/r02e_open_procs.json). One context's engine is one process, so it sits on the
one-process floor; the pool runs P helper processes, each with its own context, and gives each a
contiguous share of the list. Helper p uses devices[p % len(devices)]: on a node with several GPUs
every GPU gets its own share over its own PCIe link.

This module is a thin ctypes mirror; a Rust liboxen binds the same functions.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence

import numpy as np

from . import _capi


def pack_paths(paths: Sequence) -> tuple[np.ndarray, np.ndarray]:
    """NUL-terminated paths back to back (uint8) and the offset of each."""
    enc = [os.fsencode(str(p)) for p in paths]
    lens = np.fromiter((len(e) + 1 for e in enc), dtype=np.uint64, count=len(enc))
    offs = np.zeros(len(enc), dtype=np.uint64)
    if len(enc) > 1:
        offs[1:] = np.cumsum(lens[:-1])
    blob = np.frombuffer(b"\0".join(enc) + b"\0", dtype=np.uint8)
    return blob, offs


class ShardedFileHasher:
    """`get_hash_given_metadata` / `u128_hash_file_contents` over many files with the reads spread
    over `procs` helper processes (oxh_pool), each with its own GPU context on
    devices[p % len(devices)] and `threads` reader threads (None: the CPU quota split over procs)."""

    def __init__(self, procs: int = 2, devices: Sequence[int] = (0,), threads: Optional[int] = None,
                 staging_bytes: int = 0):
        if procs < 1:
            raise _capi.OxenError("procs must be >= 1", _capi.OXH_ERR_INVALID)
        devs = (ctypes.c_int * max(1, len(devices)))(*[int(d) for d in devices])
        h = _capi._vp()
        _capi.check(_capi.lib().oxh_pool_create(devs, len(devices), int(procs), int(threads or 0), int(staging_bytes),
                                                ctypes.byref(h)), "oxh_pool_create")
        self._h = h
        self.procs = procs
        self.devices = tuple(int(d) for d in devices)

    def pids(self) -> list[int]:
        n = _capi._int(0)
        pids = (ctypes.c_int * self.procs)()
        _capi.check(_capi.lib().oxh_pool_size(self._h, ctypes.byref(n), pids), "oxh_pool_size")
        return list(pids[: n.value])

    def hash_files_packed(self, blob: np.ndarray, offsets: np.ndarray, meta_sizes: Optional[np.ndarray] = None,
                          with_errors: bool = False):
        """Paths packed by `pack_paths`. Returns (out (n, 2) uint64 lo/hi, sizes, status), plus os_error
        (the errno of each failed open / read, oxh_pool_hash_files_ex) when with_errors."""
        n = len(offsets)
        out = np.zeros((n, 2), dtype=np.uint64)
        sizes = np.zeros(n, dtype=np.uint64)
        status = np.zeros(n, dtype=np.int32)
        oserr = np.zeros(n, dtype=np.int32)
        if n == 0:
            return (out, sizes, status, oserr) if with_errors else (out, sizes, status)
        if self._h is None:
            raise _capi.OxenError("pool is closed", _capi.OXH_ERR_INVALID)
        blob = np.ascontiguousarray(blob, dtype=np.uint8)
        ptrs = (np.asarray(offsets, dtype=np.uint64) + np.uint64(blob.ctypes.data)).astype(np.uint64)  # char* table
        meta = None if meta_sizes is None else np.ascontiguousarray(meta_sizes, dtype=np.uint64)
        if meta is not None and len(meta) != n:
            raise _capi.OxenError("paths and meta_sizes differ in length", _capi.OXH_ERR_INVALID)
        _capi.check(_capi.lib().oxh_pool_hash_files_ex(self._h, ptrs.ctypes.data_as(ctypes.POINTER(ctypes.c_char_p)),
                                                       None if meta is None else meta.ctypes.data, n,
                                                       out.ctypes.data_as(_capi._u64p), sizes.ctypes.data_as(_capi._u64p),
                                                       status.ctypes.data_as(_capi._i32p),
                                                       oserr.ctypes.data_as(_capi._i32p)), "oxh_pool_hash_files_ex")
        return (out, sizes, status, oserr) if with_errors else (out, sizes, status)

    def hash_files(self, paths: Sequence, meta_sizes: Optional[Sequence[int]] = None, with_errors: bool = False):
        blob, offs = pack_paths(paths)
        meta = None if meta_sizes is None else np.ascontiguousarray(meta_sizes, dtype=np.uint64)
        return self.hash_files_packed(blob, offs, meta, with_errors)

    def close(self) -> None:
        if getattr(self, "_h", None):
            _capi.lib().oxh_pool_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
