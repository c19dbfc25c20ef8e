"""Multi-GPU sharding of the hashing stage: one process per GPU, files split into contiguous
byte-balanced ranges (no data-path collective), and ONE collective at the end -- an all-gather of
the 16-B-per-file digest table: on GPUs the C ABI's oxh_gather_digests (RCCL over xGMI, comm.py),
in CPU tests torch.distributed over gloo.
"""
from __future__ import annotations

from typing import Sequence

import numpy as np
import torch
import torch.distributed as dist


def shard_bounds(lens: Sequence[int], world: int) -> list[tuple[int, int]]:
    """Contiguous item ranges [lo, hi) per rank, balanced by bytes (every item goes to exactly one rank)."""
    lens = np.asarray(lens, dtype=np.float64)
    n = len(lens)
    if world <= 1 or n == 0:
        return [(0, n)] + [(n, n)] * max(0, world - 1)
    cum = np.concatenate([[0.0], np.cumsum(lens + 1.0)])  # +1: empty files still cost a slot
    total = cum[-1]
    cuts = [0]
    for r in range(1, world):
        cuts.append(int(np.searchsorted(cum, total * r / world, side="left")))
    cuts.append(n)
    cuts = np.maximum.accumulate(np.clip(cuts, 0, n))
    return [(int(cuts[r]), int(cuts[r + 1])) for r in range(world)]


def gather_digest_table(local: torch.Tensor, counts: Sequence[int], group=None) -> torch.Tensor:
    """All-gather per-rank (n_r, 2) int64 digest tables into the full (sum n_r, 2) table on every
    rank. Tables are padded to max(n_r) so a single all_gather_into_tensor moves them."""
    world = dist.get_world_size(group)
    m = max(counts) if counts else 0
    if local.shape[0] < m:
        pad = torch.zeros((m - local.shape[0], 2), dtype=local.dtype, device=local.device)
        local = torch.cat([local, pad], 0)
    full = torch.empty((world * m, 2), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(full, local.contiguous(), group=group)
    parts = [full[r * m:r * m + counts[r]] for r in range(world)]
    return torch.cat(parts, 0) if parts else full[:0]


class PipelinedGather:
    """Double-buffered digest tables whose all-gather overlaps the next batch's hashing (bench.py's
    N > 1 step): fill(b) hands out local table b; gather(b) starts its all-gather asynchronously; a
    table is handed out again only after the gather that read it has completed. Every rank must hold
    the same count n.

    With `comm` (a comm.DigestComm) the gather is the C ABI's oxh_gather_digests (RCCL all-gather over
    xGMI, what a Rust host links) on a side stream of its own, ordered against the hashing stream with
    HIP events; without one it is torch.distributed's all_gather_into_tensor (the gloo rehearsal and
    CPU tests)."""

    def __init__(self, n: int, world: int, device, group=None, buffers: int = 2, comm=None):
        self.local = [torch.empty((n, 2), dtype=torch.int64, device=device) for _ in range(buffers)]
        self.full = [torch.empty((n * world, 2), dtype=torch.int64, device=device) for _ in range(buffers)]
        self.pending = [None] * buffers
        self.group = group
        self.comm = comm
        self.counts = [n] * world
        self.side = torch.cuda.Stream(device) if comm is not None else None
        self.k = 0

    def next_local(self) -> tuple[int, torch.Tensor]:
        """The next local table to fill, once no gather still reads it."""
        b = self.k % len(self.local)
        self.k += 1
        if self.pending[b] is not None:
            if self.comm is not None:  # the hashing stream waits for that gather's event
                torch.cuda.current_stream(self.local[b].device).wait_event(self.pending[b])
            else:
                self.pending[b].wait()
            self.pending[b] = None
        return b, self.local[b]

    def gather(self, b: int) -> torch.Tensor:
        """Start the all-gather of local table b; returns the full table it will fill."""
        if self.comm is not None:
            cur = torch.cuda.current_stream(self.local[b].device)
            self.side.wait_stream(cur)  # the hash that filled table b comes first
            self.comm.gather(self.local[b], self.counts, self.full[b], root=-1, stream=self.side)
            ev = torch.cuda.Event()
            ev.record(self.side)
            self.pending[b] = ev
        else:
            self.pending[b] = dist.all_gather_into_tensor(self.full[b], self.local[b], group=self.group, async_op=True)
        return self.full[b]

    def drain(self) -> None:
        for i, w in enumerate(self.pending):
            if w is not None:
                if self.comm is not None:
                    torch.cuda.current_stream(self.local[i].device).wait_event(w)
                else:
                    w.wait()
                self.pending[i] = None
