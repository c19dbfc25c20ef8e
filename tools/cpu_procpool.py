"""The CPU reference loop restated (oracle/, test infrastructure) split over P worker processes, for
tools/bench_e2e.py's same-shape comparison with oxen_amd.procpool.ShardedFileHasher (the product's
oxh_pool). Not part of the shipped package: only measurement scripts import it.

Paths cross the process boundary once, packed in shared memory (oxen_amd.procpool.pack_paths); each
worker points a char* table into its mapping and writes digests, sizes and statuses in place.
Workers are `spawn`ed and live until close()."""
from __future__ import annotations

import ctypes
import multiprocessing as mp
import os
import sys
from multiprocessing import shared_memory

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

_FIELDS = ("blob", "offs", "out", "sizes", "status")


def _worker(conn, threads: int) -> None:
    from oracle import oracle

    oracle.build()
    O = oracle.lib()
    attached: dict = {}
    conn.send(("ready", os.getpid()))
    while True:
        msg = conn.recv()
        if msg is None:
            break
        seq, names, lo, hi = msg
        try:
            for nm in list(attached):  # segments the parent replaced since the last call
                if nm not in names:
                    try:
                        attached.pop(nm).close()
                    except BufferError:
                        pass
            shms = {}
            for f, nm in zip(_FIELDS, names):
                if nm not in attached:
                    attached[nm] = shared_memory.SharedMemory(name=nm)
                shms[f] = attached[nm]
            k = hi - lo
            base = np.frombuffer(shms["blob"].buf, dtype=np.uint8)
            offs = np.frombuffer(shms["offs"].buf, dtype=np.uint64)[lo:hi]
            ptrs = (offs + np.uint64(base.ctypes.data)).astype(np.uint64)
            out = np.frombuffer(shms["out"].buf, dtype=np.uint64)
            sizes = np.frombuffer(shms["sizes"].buf, dtype=np.uint64)
            status = np.frombuffer(shms["status"].buf, dtype=np.int32)
            O.oxo_hash_files(ptrs.ctypes.data_as(ctypes.POINTER(ctypes.c_char_p)), k,
                             ctypes.cast(out.ctypes.data + 16 * lo, oracle._u64p),
                             ctypes.cast(sizes.ctypes.data + 8 * lo, oracle._u64p),
                             ctypes.cast(status.ctypes.data + 4 * lo, oracle._i32p), threads)
            del base, offs, out, sizes, status
            conn.send((seq, 0, ""))
        except Exception as e:
            conn.send((seq, -1, repr(e)))
    for s in attached.values():
        try:
            s.close()
        except BufferError:
            pass


class CpuShardedLoop:
    def __init__(self, procs: int = 2, threads: int = 1):
        ctx = mp.get_context("spawn")
        self._conns, self._procs, self._shm, self._seq = [], [], {}, 0
        for _ in range(procs):
            parent, child = ctx.Pipe()
            p = ctx.Process(target=_worker, args=(child, max(1, threads)), daemon=True)
            p.start()
            self._conns.append(parent)
            self._procs.append(p)
        for c in self._conns:
            assert c.recv()[0] == "ready"

    def _seg(self, field, nbytes):
        s = self._shm.get(field)
        if s is None or s.size < nbytes:
            if s is not None:
                s.close()
                s.unlink()
            s = shared_memory.SharedMemory(create=True, size=max(nbytes, 16))
            self._shm[field] = s
        return s

    def hash_files_packed(self, blob, offsets, meta_sizes=None):
        n = len(offsets)
        segs = {"blob": self._seg("blob", blob.nbytes), "offs": self._seg("offs", 8 * n),
                "out": self._seg("out", 16 * n), "sizes": self._seg("sizes", 8 * n), "status": self._seg("status", 4 * n)}
        np.frombuffer(segs["blob"].buf, dtype=np.uint8, count=blob.nbytes)[:] = blob
        np.frombuffer(segs["offs"].buf, dtype=np.uint64, count=n)[:] = offsets
        names = tuple(segs[f].name for f in _FIELDS)
        if meta_sizes is not None:
            cum = np.cumsum(np.asarray(meta_sizes, dtype=np.float64) + 4096.0)
            P = len(self._conns)
            cuts = [0] + [int(np.searchsorted(cum, cum[-1] * p / P)) for p in range(1, P)] + [n]
        else:
            cuts = [n * p // len(self._conns) for p in range(len(self._conns) + 1)]
        self._seq += 1
        busy = []
        for p, c in enumerate(self._conns):
            if cuts[p + 1] > cuts[p]:
                c.send((self._seq, names, cuts[p], cuts[p + 1]))
                busy.append(c)
        for c in busy:
            seq, rc, err = c.recv()
            assert seq == self._seq and rc == 0, err
        out = np.frombuffer(segs["out"].buf, dtype=np.uint64, count=2 * n).reshape(n, 2).copy()
        sizes = np.frombuffer(segs["sizes"].buf, dtype=np.uint64, count=n).copy()
        status = np.frombuffer(segs["status"].buf, dtype=np.int32, count=n).copy()
        return out, sizes, status

    def close(self):
        for c in self._conns:
            try:
                c.send(None)
            except Exception:
                pass
        for p in self._procs:
            p.join(timeout=30)
            if p.is_alive():
                p.terminate()
        for s in self._shm.values():
            s.close()
            s.unlink()
        self._conns, self._procs, self._shm = [], [], {}
