"""One rank of tests/test_gpu_gather_ranks.py: the C ABI's digest gather (oxh_comm_* /
oxh_gather_digests, csrc/comm.cpp) with N ranks as N processes on the one GPU of the test box, RCCL
replaced by the test double tests/native/fake_rccl.cpp (OXH_RCCL_LIB, set by the parent).

    python tests/_gather_rank.py RANK WORLD DIR

DIR/plan.json lists the scenarios (counts per rank, root, OXH_GATHER_P2P, whether a non-receiving
rank passes a sentinel-filled table). For each, this rank hashes its own share with K1
(DeviceArena.splitmix, seeded by scenario and rank), gathers, and saves DIR/s{i}_r{rank}.npz: its
local table, the gathered table it holds (if any), and up to 200 of its items' bytes for
the parent's oracle sample. Rank 0 makes the communicator id (oxh_comm_unique_id) and hands it over in DIR/uid.bin.
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SENTINEL = 0x5A5A5A5A


def main(rank: int, world: int, tmp: str) -> int:
    with open(os.path.join(tmp, "plan.json")) as f:
        plan = json.load(f)
    import torch

    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    from oxen_amd.comm import DigestComm, comm_check
    from oxen_amd.device import DeviceArena

    err = comm_check(0)
    if err is not None:
        raise err
    uid_path = os.path.join(tmp, "uid.bin")
    if rank == 0:
        uid = DigestComm.unique_id()
        with open(uid_path + ".tmp", "wb") as f:
            f.write(uid)
        os.replace(uid_path + ".tmp", uid_path)
    else:
        deadline = time.time() + 90
        while not os.path.exists(uid_path):
            if time.time() > deadline:
                raise TimeoutError("rank 0 never published the comm id")
            time.sleep(0.05)
        with open(uid_path, "rb") as f:
            uid = f.read()
    with DigestComm(uid, rank, world, 0) as comm:
        assert comm.info() == (rank, world, 0)
        for si, sc in enumerate(plan["scenarios"]):
            counts, root = sc["counts"], sc["root"]
            if sc.get("p2p"):
                os.environ["OXH_GATHER_P2P"] = "1"
            else:
                os.environ.pop("OXH_GATHER_P2P", None)
            n = counts[rank]
            rng = np.random.default_rng(1000 * si + rank)
            save = {}
            if n:
                lens = rng.integers(0, 6000, n).astype(np.uint64)
                lens[rng.integers(0, n)] = 70_000  # one item on K1's long path
                da = DeviceArena.splitmix(lens, seed=7919 * si + 31 * rank + 1, device=dev)
                local = da.hash()
                host = da.arena.cpu().numpy()
                idx = np.sort(rng.choice(n, min(n, 200), replace=False))
                save["s_idx"] = idx.astype(np.int64)
                save["s_lens"] = da.lens_host[idx].astype(np.uint64)
                save["s_bytes"] = np.concatenate([host[int(o):int(o) + int(ln)] for o, ln in
                                                  zip(da.offsets_host[idx], da.lens_host[idx])] + [np.zeros(0, np.uint8)])
            else:
                local = torch.empty((0, 2), dtype=torch.int64, device=dev)
            total = sum(counts)
            receives = root < 0 or root == rank
            full = None
            if receives and not (total == 0 and sc.get("none_full")):
                full = torch.full((total, 2), -1, dtype=torch.int64, device=dev)
            elif not receives and sc.get("sentinel"):
                full = torch.full((total, 2), SENTINEL, dtype=torch.int64, device=dev)
            comm.gather(local, counts, full, root=root)
            torch.cuda.synchronize()
            save["local"] = local.cpu().numpy()
            if full is not None:
                save["full"] = full.cpu().numpy()
            np.savez(os.path.join(tmp, f"s{si}_r{rank}.npz"), **save)
    os.environ.pop("OXH_GATHER_P2P", None)
    print(f"rank {rank}: {len(plan['scenarios'])} scenarios done", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main(int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]))
