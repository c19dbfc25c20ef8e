"""N > 1 path on CPU: byte-balanced sharding and the single all-gather of the digest table (gloo)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oxen_amd.shard import gather_digest_table, shard_bounds


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_bounds_cover_and_balance():
    rng = np.random.default_rng(0)
    for world in (1, 2, 3, 8):
        for n in (0, 1, 7, 1000):
            lens = rng.integers(0, 300_000, n)
            b = shard_bounds(lens, world)
            assert len(b) == world
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))
            if n >= 100 * world:
                per = [lens[lo:hi].sum() for lo, hi in b]
                assert max(per) <= lens.sum() / world + lens.max() + world


def _worker(rank, world, port, lens, seed, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle
        from oxen_amd.workloads import packed_layout, splitmix_bytes

        offs, total = packed_layout(lens)
        arena = splitmix_bytes(seed, 0, total)
        lo, hi = shard_bounds(lens, world)[rank]
        # this rank's shard (the oracle stands in for the device here -- test infrastructure)
        local = oracle.batch(arena, offs[lo:hi], lens[lo:hi]).view(np.int64)
        counts = [h - l for l, h in shard_bounds(lens, world)]
        full = gather_digest_table(torch.from_numpy(local.copy()).reshape(-1, 2), counts)
        if rank == 0:
            want = oracle.batch(arena, offs, lens).view(np.int64)
            q.put(bool(np.array_equal(full.numpy(), want)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_digest_table_gloo(world, oracle_lib):
    rng = np.random.default_rng(world)
    lens = rng.integers(0, 20_000, 101).astype(np.uint64)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, lens, 5, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert q.get(timeout=10) is True


def _pipe_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oxen_amd.shard import PipelinedGather

        n, steps = 37, 7

        def table(r, k):  # what rank r hashes at step k
            return torch.arange(2 * n, dtype=torch.int64).reshape(n, 2) * 1000 + r * 100 + k

        want = [torch.cat([table(r, k) for r in range(world)]) for k in range(steps)]
        pipe = PipelinedGather(n, world, "cpu")
        ok, fulls = True, {}
        for k in range(steps):
            b, local = pipe.next_local()  # waits for the gather that last read this table
            if k >= 2:
                ok &= bool(torch.equal(pipe.full[b], want[k - 2]))  # step k-2's result, intact
            local.copy_(table(rank, k))
            fulls[k] = pipe.gather(b)
        pipe.drain()
        ok &= bool(torch.equal(fulls[steps - 1], want[steps - 1]) and torch.equal(fulls[steps - 2], want[steps - 2]))
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


def test_pipelined_gather_gloo():
    """bench.py's N > 1 step (shard.PipelinedGather): double-buffered tables, each step's all-gather
    in flight while the next table is filled, every step's gathered table correct (world size 2)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipe_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = dict(q.get(timeout=10) for _ in range(world))
    assert res == {0: True, 1: True}


def _comm_id_worker(rank, world, port, q, bad_rank):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oxen_amd import _capi, comm

        def no_rccl():
            raise _capi.OxenError("RCCL unavailable (test)", _capi.OXH_ERR_HIP)

        def never(*a, **k):  # no rank may go on to create a communicator
            raise AssertionError("DigestComm created after a failed id")

        comm.DigestComm.unique_id = staticmethod(no_rccl)
        comm.DigestComm.__init__ = never
        # every rank's own check passes, or (bad_rank) one rank's device/RCCL check fails
        comm.comm_check = lambda device: (_capi.OxenError("device index out of range (test)", _capi.OXH_ERR_INVALID)
                                          if rank == bad_rank else None)
        try:
            comm.comm_from_process_group(rank, world, 0)
            q.put((rank, "no error"))
        except _capi.OxenError as e:
            want = "rank 0 could not create the comm id" if bad_rank < 0 else f"rank {bad_rank} cannot join"
            q.put((rank, e.code, want in str(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("bad_rank", [-1, 2])
def test_comm_id_failure_raises_on_every_rank(bad_rank):
    """comm_from_process_group: when rank 0 cannot create the RCCL id (bad_rank -1), or when one
    rank's own oxh_comm_check fails (a bad device index or no RCCL on rank 2: ADVICE r05), every rank
    raises the same error before any rank enters oxh_comm_create (none waits in the broadcast or in
    RCCL's bootstrap), so bench.py's collective fallback to torch's all-gather is reached by all."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_comm_id_worker, args=(r, world, port, q, bad_rank)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    from oxen_amd import _capi

    got = sorted(q.get(timeout=10) for _ in range(world))
    code = _capi.OXH_ERR_HIP if bad_rank < 0 else _capi.OXH_ERR_INVALID
    assert got == [(r, code, True) for r in range(world)]
