"""Process-sharded file hashing: the engine's per-file syscalls split over reader PROCESSES.

Why: on the MI355X boxes the warm-cache floor of the `oxen add` read is open + close themselves,
and that floor belongs to the process -- 200 000 open + close pairs take 0.28 s in one process
whatever its thread count (no scaling past 4 threads), 0.16 s in two and 0.13 s in four or more;
a whole read (open + fstat + pread + close) 0.27-0.29 s in one process, 0.155-0.175 s in 2-8
(tools/open_probe.cpp with PROCS=P, profiles/r02e_open_procs.json). One context's engine is one
process, so it sits on the one-process floor; this pool runs P engines (one `oxh_ctx` each, all on
the same GPU) in P spawned worker processes and gives each a contiguous share of the list.
Measured on C3 warm (tools/bench_e2e.py, profiles/r02e_e2e_c3_procs.json): one engine 0.30-0.32 s,
2 processes x 8 readers 0.21 s, 4 x 4 0.22 s -- the GPU side is then at its PCIe floor (9.87 GB of
pinned H2D at 55 GB/s = 0.18 s), so 2 is the default.

The list crosses the process boundary once, as NUL-terminated paths packed in one shared-memory
arena plus an offsets table (`pack_paths`); each worker points its own char* table into its mapping
of that arena (no per-path marshalling) and writes digests, sizes and statuses straight into shared
output arrays. Workers are started with the `spawn` method (fresh interpreters: nothing is forked
from a process that holds the GPU) and live until `close()`.
"""
from __future__ import annotations

import ctypes
import multiprocessing as mp
import os
from multiprocessing import shared_memory
from typing import Optional, Sequence

import numpy as np

from . import _capi

_FIELDS = ("blob", "offs", "meta", "out", "sizes", "status")


def pack_paths(paths: Sequence) -> tuple[np.ndarray, np.ndarray]:
    """NUL-terminated paths back to back (uint8) and the offset of each."""
    enc = [os.fsencode(str(p)) for p in paths]
    lens = np.fromiter((len(e) + 1 for e in enc), dtype=np.uint64, count=len(enc))
    offs = np.zeros(len(enc), dtype=np.uint64)
    if len(enc) > 1:
        offs[1:] = np.cumsum(lens[:-1])
    blob = np.frombuffer(b"\0".join(enc) + b"\0", dtype=np.uint8)
    return blob, offs


def _attach(name: str) -> shared_memory.SharedMemory:
    # spawned workers share the parent's resource tracker: their (re-)registration of the name is the
    # parent's own entry, which the parent's unlink in close() removes
    return shared_memory.SharedMemory(name=name)


def _worker(conn, device: int, staging_bytes: int, mode: str, threads: int) -> None:
    if threads:
        os.environ["OXH_NUM_THREADS"] = str(threads)
    if mode == "gpu":
        from . import _capi as capi

        ctx = capi.Context(device, staging_bytes=staging_bytes) if staging_bytes else capi.Context(device)
        L = capi.lib()
    else:  # the CPU reference loop restated (oracle/), for the same-shape comparison in tools/
        from oracle import oracle

        oracle.build()
        O = oracle.lib()
    attached: dict = {}
    conn.send(("ready", os.getpid()))
    while True:
        msg = conn.recv()
        if msg is None:
            break
        names, lo, hi, has_meta = msg
        try:
            shms = {}
            for f, nm in zip(_FIELDS, names):
                if nm not in attached:
                    attached[nm] = _attach(nm)
                shms[f] = attached[nm]
            k = hi - lo
            base = np.frombuffer(shms["blob"].buf, dtype=np.uint8)
            offs = np.frombuffer(shms["offs"].buf, dtype=np.uint64)[lo:hi]
            ptrs = (offs + np.uint64(base.ctypes.data)).astype(np.uint64)  # char* table into this mapping
            out = np.frombuffer(shms["out"].buf, dtype=np.uint64)
            sizes = np.frombuffer(shms["sizes"].buf, dtype=np.uint64)
            status = np.frombuffer(shms["status"].buf, dtype=np.int32)
            pp = ptrs.ctypes.data_as(ctypes.POINTER(ctypes.c_char_p))
            o_p = ctypes.cast(out.ctypes.data + 16 * lo, _capi._u64p)
            s_p = ctypes.cast(sizes.ctypes.data + 8 * lo, _capi._u64p)
            t_p = ctypes.cast(status.ctypes.data + 4 * lo, _capi._i32p)
            if mode == "gpu":
                if has_meta:
                    meta = np.frombuffer(shms["meta"].buf, dtype=np.uint64)
                    m_p = ctypes.cast(meta.ctypes.data + 8 * lo, _capi._u64p)
                    rc = L.oxh_hash_files_meta(ctx.handle, pp, m_p, k, o_p, s_p, t_p)
                else:
                    rc = L.oxh_hash_files(ctx.handle, pp, k, o_p, s_p, t_p)
                err = "" if rc == 0 else capi.lib().oxh_last_error().decode(errors="replace")
            else:
                O.oxo_hash_files(pp, k, o_p, s_p, t_p, threads or 1)
                rc, err = 0, ""
            del base, offs, out, sizes, status
            if has_meta and mode == "gpu":
                del meta
            conn.send(("done", rc, err))
        except Exception as e:  # reported to the caller, which raises
            conn.send(("done", -1, repr(e)))
    for s in attached.values():
        try:
            s.close()
        except BufferError:  # a view from a failed call still holds it; the process is exiting
            pass
    if mode == "gpu":
        ctx.close()


class ShardedFileHasher:
    """`get_hash_given_metadata` / `u128_hash_file_contents` over many files with the reads spread
    over `procs` worker processes, each with its own GPU context (device `device`) and `threads`
    reader threads. `mode="cpu"` runs the oracle's restated reference loop in the workers instead
    (tools/ only: a comparison at the same process count)."""

    def __init__(self, procs: int = 2, device: int = 0, threads: Optional[int] = None, staging_bytes: int = 0,
                 mode: str = "gpu"):
        if procs < 1:
            raise _capi.OxenError("procs must be >= 1", _capi.OXH_ERR_INVALID)
        self.procs = procs
        threads = threads if threads is not None else max(1, (os.cpu_count() or 1) // procs)
        ctx = mp.get_context("spawn")
        self._conns, self._procs = [], []
        for _ in range(procs):
            parent, child = ctx.Pipe()
            p = ctx.Process(target=_worker, args=(child, device, staging_bytes, mode, threads), daemon=True)
            p.start()
            self._conns.append(parent)
            self._procs.append(p)
        for c in self._conns:
            msg = c.recv()
            if msg[0] != "ready":
                raise _capi.OxenError(f"worker failed to start: {msg}", _capi.OXH_ERR_HIP)
        self._shm: dict = {}

    def _seg(self, field: str, nbytes: int) -> shared_memory.SharedMemory:
        s = self._shm.get(field)
        if s is None or s.size < nbytes:
            if s is not None:
                s.close()
                s.unlink()
            s = shared_memory.SharedMemory(create=True, size=max(nbytes, 16))
            self._shm[field] = s
        return s

    def hash_files_packed(self, blob: np.ndarray, offsets: np.ndarray, meta_sizes: Optional[np.ndarray] = None):
        """Paths packed by `pack_paths`. Returns (out (n, 2) uint64 lo/hi, sizes, status) copies."""
        n = len(offsets)
        out = np.zeros((n, 2), dtype=np.uint64)
        if n == 0:
            return out, np.zeros(0, dtype=np.uint64), np.zeros(0, dtype=np.int32)
        segs = {"blob": self._seg("blob", blob.nbytes), "offs": self._seg("offs", 8 * n),
                "meta": self._seg("meta", 8 * n if meta_sizes is not None else 16),
                "out": self._seg("out", 16 * n), "sizes": self._seg("sizes", 8 * n), "status": self._seg("status", 4 * n)}
        np.frombuffer(segs["blob"].buf, dtype=np.uint8, count=blob.nbytes)[:] = blob
        np.frombuffer(segs["offs"].buf, dtype=np.uint64, count=n)[:] = offsets
        if meta_sizes is not None:
            np.frombuffer(segs["meta"].buf, dtype=np.uint64, count=n)[:] = meta_sizes
        names = tuple(segs[f].name for f in _FIELDS)
        # contiguous shares, balanced by bytes when the sizes are known
        if meta_sizes is not None:
            cum = np.cumsum(np.asarray(meta_sizes, dtype=np.float64) + 4096.0)
            cuts = [0] + [int(np.searchsorted(cum, cum[-1] * p / self.procs)) for p in range(1, self.procs)] + [n]
        else:
            cuts = [n * p // self.procs for p in range(self.procs + 1)]
        busy = []
        for p, c in enumerate(self._conns):
            lo, hi = cuts[p], cuts[p + 1]
            if hi > lo:
                c.send((names, lo, hi, meta_sizes is not None))
                busy.append(c)
        errs = [m for m in (c.recv() for c in busy) if m[1] != 0]
        if errs:
            raise _capi.OxenError(f"sharded hash failed: {errs[0][2]}", _capi.OXH_ERR_HIP)
        out[:] = np.frombuffer(segs["out"].buf, dtype=np.uint64, count=2 * n).reshape(n, 2)
        sizes = np.frombuffer(segs["sizes"].buf, dtype=np.uint64, count=n).copy()
        status = np.frombuffer(segs["status"].buf, dtype=np.int32, count=n).copy()
        return out, sizes, status

    def hash_files(self, paths: Sequence, meta_sizes: Optional[Sequence[int]] = None):
        blob, offs = pack_paths(paths)
        meta = None if meta_sizes is None else np.ascontiguousarray(meta_sizes, dtype=np.uint64)
        return self.hash_files_packed(blob, offs, meta)

    def close(self) -> None:
        for c in self._conns:
            try:
                c.send(None)
            except Exception:
                pass
        for p in self._procs:
            p.join(timeout=30)
            if p.is_alive():
                p.terminate()
        self._conns, self._procs = [], []
        for s in self._shm.values():
            s.close()
            s.unlink()
        self._shm = {}

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
