"""bench.py's multi-GPU launch (one process per GPU: `--gpus N` starts the N ranks itself when no
launcher set WORLD_SIZE) and the RCCL leg of the N > 1 step (shard.PipelinedGather on "nccl")."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env=None, timeout=300):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, BENCH] + args, env=e, capture_output=True, text=True, timeout=timeout)


def test_bench_rejects_bad_gpu_counts():
    r = _run(["--gpus", "0"])
    assert r.returncode == 2
    r = _run(["--gpus", "2"], env={"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE=3 but --gpus 2" in r.stderr


def test_bench_launches_ranks_and_propagates_failure():
    """Without a GPU (or with fewer GPUs than ranks) every spawned rank refuses to put two RCCL ranks
    on one device; the launcher exits non-zero instead of reporting a one-GPU number."""
    import torch

    if torch.cuda.device_count() >= 2:
        pytest.skip("enough GPUs for a real 2-rank run")
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0", "--no-cpu-baseline", "--workload", "t"])
    assert r.returncode == 2, r.stderr[-2000:]
    assert r.stderr.count("RCCL needs one GPU per rank") == 2
    assert not r.stdout.strip()


@pytest.mark.gpu
def test_bench_two_ranks_gloo_one_gpu(cuda):
    """`bench.py --gpus 2` spawns two ranks itself (gloo rehearsal on the one GPU of the test box):
    the JSON line reports n_gpus 2 and rank 0 checked both ranks' digests against the oracle."""
    r = _run(["--gpus", "2", "--backend", "gloo", "--workload", "t", "--steps", "3", "--warmup", "1",
              "--no-cpu-baseline"])
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(line) == 1, r.stdout
    d = json.loads(line[0])
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["config"]["items_per_gpu"] == 2048


@pytest.mark.gpu
@pytest.mark.parametrize("ranks", [2, 4, 8])
def test_bench_ranks_abi_gather_fake_rccl(cuda, ranks):
    """The whole N > 1 bench step as the driver's 8-GPU run takes it -- ranks started by bench.py itself,
    comm_from_process_group (oxh_comm_check agreed, the id broadcast), shard.PipelinedGather with
    oxh_gather_digests per step on a side stream, the max over ranks, rank 0's checks of every rank's
    shard against the oracle -- with every rank on the one GPU of the test box and RCCL replaced by the
    test double (tests/native/libfake_rccl.so via OXH_RCCL_LIB; the id travels over gloo)."""
    from oxen_amd import build

    r = _run(["--gpus", str(ranks), "--backend", "gloo", "--gather", "abi", "--workload", "t", "--steps", "3",
              "--warmup", "1", "--no-cpu-baseline", "--prewarm-s", "0"],
             env={"OXH_RCCL_LIB": build.FAKE_RCCL, "OXH_FAKE_RCCL_SLOT_BYTES": str(8 << 20)})
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(line) == 1, r.stdout
    d = json.loads(line[0])
    assert d["n_gpus"] == ranks and d["steps"] == 3
    assert "oxh_gather_digests" in d["config"]["parallelism"], d["config"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
def test_pipelined_gather_rccl_in_process(cuda, oracle_lib):
    """The RCCL leg of C4 in the GPU suite, through the C ABI (oxh_comm_* / oxh_gather_digests, what
    bench.py's N > 1 step and a Rust host call): a communicator of one rank, bench.py's pipelined step
    (K1 into one of two digest tables while the previous table's all-gather runs on a side stream) for
    several steps; every gathered table equals the local K1 digests, which equal the oracle on a sample.
    Then the rooted gather (root 0) and the argument checks."""
    import torch

    from oxen_amd import _capi
    from oxen_amd.comm import DigestComm
    from oxen_amd.device import DeviceArena, to_numpy_u64
    from oxen_amd.shard import PipelinedGather

    from oxen_amd.comm import comm_check

    assert comm_check(cuda.index or 0) is None  # RCCL loads, the device is visible
    bad = comm_check(99)
    assert bad is not None and bad.code == _capi.OXH_ERR_INVALID and "out of range" in str(bad)
    with DigestComm(DigestComm.unique_id(), 0, 1, cuda.index or 0) as comm:
        assert comm.info() == (0, 1, cuda.index or 0)
        rng = np.random.default_rng(11)
        lens = rng.integers(0, 300_000, 3000).astype(np.uint64)
        da = DeviceArena.splitmix(lens, seed=19, device=cuda)
        ref = torch.empty((len(lens), 2), dtype=torch.int64, device=cuda)
        da.hash(ref)
        pipe = PipelinedGather(len(lens), 1, cuda, comm=comm)
        fulls = []
        for _ in range(6):
            b, local = pipe.next_local()
            local.zero_()
            da.hash(local)
            fulls.append(pipe.gather(b))
        pipe.drain()
        torch.cuda.synchronize()
        want = to_numpy_u64(ref).reshape(-1, 2)
        for f in fulls[-2:]:  # the two tables still holding their last step's gather
            assert np.array_equal(to_numpy_u64(f).reshape(-1, 2), want)
        host = da.arena.cpu().numpy()
        idx = rng.choice(len(lens), 200, replace=False)
        got = oracle_lib.batch(host, da.offsets_host[idx], da.lens_host[idx])
        assert np.array_equal(got, want[idx])
        # rooted (ncclGather) and empty tables
        full = torch.zeros_like(ref)
        comm.gather(ref, [len(lens)], full, root=0)
        torch.cuda.synchronize()
        assert torch.equal(full, ref)
        comm.gather(ref[:0], [0], torch.empty((0, 2), dtype=torch.int64, device=cuda), root=-1)
        # the ragged-share form (grouped ncclBroadcast for every rank, send/recv + the root's own copy)
        import os

        os.environ["OXH_GATHER_P2P"] = "1"
        try:
            for root in (-1, 0):
                full = torch.zeros_like(ref)
                comm.gather(ref, [len(lens)], full, root=root)
                torch.cuda.synchronize()
                assert torch.equal(full, ref), root
        finally:
            del os.environ["OXH_GATHER_P2P"]
        with pytest.raises(_capi.OxenError) as e:
            comm.gather(ref, [len(lens)], full, root=1)
        assert e.value.code == _capi.OXH_ERR_INVALID
