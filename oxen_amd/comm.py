"""Python mirror of the C ABI's digest gather (include/oxen_hash.h, oxh_comm_*; csrc/comm.cpp).

Files shard across the GPUs of a node (shard.shard_bounds); each rank hashes its share with K1 and
the one exchange is the digest table, gathered over xGMI by RCCL through the library -- the same
calls a Rust liboxen binds. torch is used only for device memory and streams.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import numpy as np

from . import _capi


class DigestComm:
    """An oxh_comm: one rank's RCCL communicator for the digest gather."""

    @staticmethod
    def unique_id() -> bytes:
        """oxh_comm_unique_id: created by one rank, handed to every rank out of band."""
        buf = ctypes.create_string_buffer(_capi.OXH_COMM_ID_BYTES)
        _capi.check(_capi.lib().oxh_comm_unique_id(buf), "oxh_comm_unique_id")
        return buf.raw

    def __init__(self, uid: bytes, rank: int, nranks: int, device: int):
        if len(uid) != _capi.OXH_COMM_ID_BYTES:
            raise _capi.OxenError(f"a comm id is {_capi.OXH_COMM_ID_BYTES} bytes", _capi.OXH_ERR_INVALID)
        h = ctypes.c_void_p()
        _capi.check(_capi.lib().oxh_comm_create(uid, int(rank), int(nranks), int(device), ctypes.byref(h)),
                    "oxh_comm_create")
        self.handle = h
        self.rank, self.nranks, self.device = int(rank), int(nranks), int(device)

    def info(self) -> tuple[int, int, int]:
        r, n, d = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _capi.check(_capi.lib().oxh_comm_info(self.handle, ctypes.byref(r), ctypes.byref(n), ctypes.byref(d)),
                    "oxh_comm_info")
        return r.value, n.value, d.value

    def gather(self, local, counts: Sequence[int], full=None, root: int = -1, stream=None) -> None:
        """oxh_gather_digests: `local` a (counts[rank], 2) int64 CUDA tensor, `full` (sum(counts), 2) on
        the receiving rank(s); enqueued on `stream` (a torch.cuda.Stream, default the current one)."""
        import torch

        if len(counts) != self.nranks:
            raise _capi.OxenError("counts needs one entry per rank", _capi.OXH_ERR_INVALID)
        if local.shape != (int(counts[self.rank]), 2) or local.dtype != torch.int64:
            raise _capi.OxenError("local table must be (counts[rank], 2) int64", _capi.OXH_ERR_INVALID)
        if full is not None and (full.shape != (int(sum(counts)), 2) or full.dtype != torch.int64):
            raise _capi.OxenError("full table must be (sum(counts), 2) int64", _capi.OXH_ERR_INVALID)
        if full is None and (root < 0 or root == self.rank) and sum(counts):
            raise _capi.OxenError("the receiving rank needs a full table", _capi.OXH_ERR_INVALID)
        st = stream if stream is not None else torch.cuda.current_stream(local.device)
        c = np.ascontiguousarray(counts, dtype=np.uint64)
        _capi.check(_capi.lib().oxh_gather_digests(self.handle, ctypes.c_void_p(local.data_ptr()),
                                                   c.ctypes.data_as(_capi._u64p),
                                                   ctypes.c_void_p(full.data_ptr() if full is not None else 0),
                                                   int(root), ctypes.c_void_p(st.cuda_stream)),
                    "oxh_gather_digests")

    def close(self) -> None:
        if self.handle:
            _capi.check(_capi.lib().oxh_comm_destroy(self.handle), "oxh_comm_destroy")
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def comm_check(device: int) -> Optional[_capi.OxenError]:
    """oxh_comm_check: None when RCCL loads and `device` is visible, else the error oxh_comm_create
    would fail with (nothing is joined)."""
    rc = _capi.lib().oxh_comm_check(int(device))
    if rc == _capi.OXH_OK:
        return None
    return _capi.OxenError(f"oxh_comm_check: {_capi.lib().oxh_last_error().decode(errors='replace')}", rc)


def comm_from_process_group(rank: int, nranks: int, device: int, group=None) -> DigestComm:
    """A DigestComm for the ranks of a torch.distributed group: every rank checks its device and RCCL
    (oxh_comm_check) and the group agrees on the outcome first; then rank 0 creates the id, the group
    broadcasts it (the "out of band" step of the ABI), and every rank creates its communicator. A
    failure on any rank -- a bad device, no RCCL, rank 0 unable to make the id -- is raised on every
    rank together, rather than the others waiting in the broadcast or in RCCL's bootstrap (inside
    oxh_comm_create) for a rank that never comes."""
    import torch.distributed as dist

    errs: list[Optional[object]] = [None] * nranks
    err = comm_check(device)
    dist.all_gather_object(errs, None if err is None else (str(err), err.code), group=group)
    bad = [(q, e) for q, e in enumerate(errs) if e is not None]
    if bad:
        q, (msg, code) = bad[0]
        raise _capi.OxenError(f"rank {q} cannot join the digest gather: {msg}", int(code))
    obj: list[Optional[object]] = [None]
    if rank == 0:
        try:
            obj[0] = DigestComm.unique_id()
        except _capi.OxenError as e:
            obj[0] = ("error", str(e), e.code)
    dist.broadcast_object_list(obj, src=0, group=group)
    if isinstance(obj[0], tuple):
        raise _capi.OxenError(f"rank 0 could not create the comm id: {obj[0][1]}", int(obj[0][2]))
    return DigestComm(obj[0], rank, nranks, device)
