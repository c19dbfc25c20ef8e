"""The C ABI's digest gather with more than one rank (VERDICT r05 "next" #1).

oxh_gather_digests (csrc/comm.cpp) stands in for the fan-out of
/root/reference/crates/liboxen/src/core/v_latest/add.rs:421-424 when the shards sit on several GPUs.
At one rank every one of its forms -- all-gather, rooted gather, grouped broadcast, grouped send/recv
-- is a copy, and the real RCCL refuses two ranks on one GPU (profiles/r05/r05i_comm_two_ranks_one_gpu.txt),
so on the one-GPU test box the per-rank offsets, the ragged branch and the rooted receive into each
rank's slot had never moved a byte between ranks. Here N = 2, 3 and 8 ranks run as N processes on
device 0 with RCCL replaced by tests/native/fake_rccl.cpp (loaded through OXH_RCCL_LIB; it copies
through host shared memory and checks that the ranks' calls match, stricter than RCCL about the call
pattern). The library under test is the shipped liboxen_hash.so, unchanged; only the RCCL it dlopens
differs. The parent does not touch the GPU before it spawns the ranks beyond the suite's own fixture.

Every scenario checks, on every receiving rank, that the gathered table equals the concatenation of
every rank's own K1 table in rank order, that a non-receiving rank's table is untouched, and that a
sample of up to 200 rows per rank equals the CPU oracle over those items' bytes.
"""
import json
import os
import subprocess
import sys
import time

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "_gather_rank.py")
SENTINEL = 0x5A5A5A5A


def scenarios(world: int) -> list[dict]:
    eq = [300] * world
    ragged = [200 + 37 * q for q in range(world)]
    ragged[1] = 0  # a rank with no files
    ragged0 = list(ragged)
    ragged0[0], ragged0[1] = 0, 123  # the root itself holds nothing
    last0 = [150 + 11 * q for q in range(world)]
    last0[-1] = 0
    return [
        {"counts": eq, "root": -1},                                  # ncclAllGather
        {"counts": eq, "root": 0, "sentinel": True},                 # ncclGather to the first rank
        {"counts": eq, "root": world - 1, "sentinel": True},         # ... and to the last
        {"counts": ragged, "root": -1},                              # grouped ncclBroadcast, a zero-count rank
        {"counts": ragged, "root": world - 1, "sentinel": True},     # grouped send/recv to the last rank
        {"counts": ragged0, "root": 0},                              # the root owns zero items (local NULL)
        {"counts": eq, "root": -1, "p2p": True},                     # OXH_GATHER_P2P=1: the ragged forms
        {"counts": eq, "root": 0, "p2p": True, "sentinel": True},    # with equal shares
        {"counts": last0, "root": -1, "p2p": True},
        {"counts": [0] * world, "root": -1, "none_full": True},      # nothing anywhere: a no-op
        {"counts": eq, "root": -1},                                  # the communicator still works after all that
    ]


def _cleanup_region(tmp):
    uid = os.path.join(tmp, "uid.bin")
    if os.path.exists(uid):
        name = open(uid, "rb").read().rstrip(b"\0").decode(errors="replace").lstrip("/")
        path = os.path.join("/dev/shm", name)
        if name.startswith("oxh_fake_rccl.") and os.path.exists(path):
            os.unlink(path)


@pytest.mark.gpu
@pytest.mark.parametrize("world,variant", [(2, "gather"), (3, "gather"), (3, "nogather"), (8, "gather")])
def test_abi_gather_multi_rank(cuda, oracle_lib, tmp_path, world, variant):
    from oxen_amd import build

    fake = build.FAKE_RCCL if variant == "gather" else build.FAKE_RCCL_NOGATHER
    assert os.path.exists(fake), "build the test double first (python -m oxen_amd.build)"
    plan = scenarios(world)
    tmp = str(tmp_path)
    with open(os.path.join(tmp, "plan.json"), "w") as f:
        json.dump({"scenarios": plan}, f)
    env = dict(os.environ)
    env.update({"OXH_RCCL_LIB": fake, "OXH_FAKE_RCCL_SLOT_BYTES": str(8 << 20), "OXH_FAKE_RCCL_TIMEOUT_S": "60"})
    env.pop("OXH_GATHER_P2P", None)
    procs, logs = [], []
    try:
        for r in range(world):
            log = open(os.path.join(tmp, f"rank{r}.log"), "w")
            logs.append(log)
            procs.append(subprocess.Popen([sys.executable, "-u", WORKER, str(r), str(world), tmp], env=env,
                                          stdout=log, stderr=subprocess.STDOUT))
        codes = []
        deadline = time.monotonic() + 150  # one deadline for the whole job, not one per rank
        for p in procs:
            try:
                codes.append(p.wait(timeout=max(1.0, deadline - time.monotonic())))
            except subprocess.TimeoutExpired:
                codes.append("timeout")
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        for log in logs:
            log.close()
        _cleanup_region(tmp)
    if any(c != 0 for c in codes):
        tails = {r: open(os.path.join(tmp, f"rank{r}.log")).read()[-1500:] for r in range(world)}
        pytest.fail(f"ranks exited {codes}:\n" + "\n".join(f"--- rank {r}\n{t}" for r, t in tails.items()))

    for si, sc in enumerate(plan):
        counts, root = sc["counts"], sc["root"]
        base = np.concatenate([[0], np.cumsum(counts)]).astype(int)
        ranks = [np.load(os.path.join(tmp, f"s{si}_r{r}.npz")) for r in range(world)]
        for r in range(world):
            assert ranks[r]["local"].shape == (counts[r], 2), (si, r)
        want = np.concatenate([ranks[r]["local"] for r in range(world)]).view(np.uint64)
        for r in range(world):
            receives = root < 0 or root == r
            if receives and "full" in ranks[r]:
                assert np.array_equal(ranks[r]["full"].view(np.uint64), want), (si, sc, r)
            elif receives:
                assert sum(counts) == 0 and sc.get("none_full"), (si, r)
            elif sc.get("sentinel"):
                assert (ranks[r]["full"] == SENTINEL).all(), (si, sc, r)
        # up to 200 oracle rows per rank, read from a receiving rank's table
        recv = 0 if root < 0 else root
        rows, got_bytes, got_lens = [], [], []
        for r in range(world):
            if counts[r]:
                rows.append(base[r] + ranks[r]["s_idx"])
                got_bytes.append(ranks[r]["s_bytes"])
                got_lens.append(ranks[r]["s_lens"])
        if not rows:
            continue
        rows = np.concatenate(rows)
        lens = np.concatenate(got_lens).astype(np.uint64)
        arena = np.concatenate(got_bytes).astype(np.uint8)
        offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
        oracle = oracle_lib.batch(arena, offs, lens)
        table = ranks[recv]["full"].view(np.uint64)
        assert np.array_equal(table[rows], oracle), (si, sc)
        assert len(rows) == sum(min(c, 200) for c in counts)


def test_fake_rccl_builds_and_exports(built_lib):
    """The test double is built with the host tools and exports what comm.cpp resolves; the
    no-gather variant lacks only ncclGather (comm.cpp's "RCCL without ncclGather" branch)."""
    import ctypes

    from oxen_amd import build

    build.build_host()
    syms = ["ncclGetUniqueId", "ncclCommInitRank", "ncclCommDestroy", "ncclAllGather", "ncclBroadcast", "ncclSend",
            "ncclRecv", "ncclGroupStart", "ncclGroupEnd", "ncclGetErrorString"]
    for path, has_gather in ((build.FAKE_RCCL, True), (build.FAKE_RCCL_NOGATHER, False)):
        L = ctypes.CDLL(path)
        for s in syms:
            assert hasattr(L, s), (path, s)
        assert hasattr(L, "ncclGather") == has_gather
