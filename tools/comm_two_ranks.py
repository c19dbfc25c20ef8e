"""Two ranks of the ABI's digest gather (oxh_comm_* / oxh_gather_digests) in two processes. On a
multi-GPU box each rank takes its own device; on a one-GPU box both ranks share device 0, which RCCL
may refuse (the result says so). Checks the all-gather (equal shares), the rooted gather, and the
ragged-share form (counts differ per rank) against the tables each rank filled. Prints one JSON object.

    python tools/comm_two_ranks.py [--same-device]
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def table(rank: int, n: int):
    import torch

    t = torch.arange(2 * n, dtype=torch.int64).reshape(n, 2) * 1000 + rank * 7 + 1
    return t


def rank_main(rank: int, world: int, device: int, q_in, q_out):
    try:
        import torch

        torch.cuda.set_device(device)
        from oxen_amd.comm import DigestComm

        if rank == 0:
            uid = DigestComm.unique_id()
            for _ in range(world - 1):
                q_in.put(uid)
        else:
            uid = q_in.get(timeout=60)
        dev = torch.device(f"cuda:{device}")
        res = {}
        with DigestComm(uid, rank, world, device) as comm:
            # equal shares: all-gather and rooted gather
            n = 1000
            counts = [n] * world
            local = table(rank, n).to(dev)
            want = torch.cat([table(r, n) for r in range(world)]).to(dev)
            full = torch.zeros_like(want)
            comm.gather(local, counts, full, root=-1)
            torch.cuda.synchronize()
            res["allgather"] = bool(torch.equal(full, want))
            full = torch.zeros_like(want)
            comm.gather(local, counts, full if rank == 0 else None, root=0)
            torch.cuda.synchronize()
            res["gather_root0"] = bool(torch.equal(full, want)) if rank == 0 else True
            # ragged shares (the byte-balanced ranges of shard_bounds differ in item count)
            counts = [1000 + 37 * r for r in range(world)]
            local = table(rank, counts[rank]).to(dev)
            want = torch.cat([table(r, counts[r]) for r in range(world)]).to(dev)
            full = torch.zeros_like(want)
            comm.gather(local, counts, full, root=-1)
            torch.cuda.synchronize()
            res["ragged_all"] = bool(torch.equal(full, want))
            full = torch.zeros_like(want)
            comm.gather(local, counts, full if rank == world - 1 else None, root=world - 1)
            torch.cuda.synchronize()
            res["ragged_root_last"] = bool(torch.equal(full, want)) if rank == world - 1 else True
        q_out.put((rank, res, None))
    except Exception as e:  # noqa: BLE001
        q_out.put((rank, None, f"{e!r}\n{traceback.format_exc()[-1500:]}"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--same-device", action="store_true", help="every rank on device 0")
    a = ap.parse_args()
    import torch

    ndev = torch.cuda.device_count()
    ctx = mp.get_context("spawn")
    q_in, q_out = ctx.Queue(), ctx.Queue()
    procs = []
    for r in range(a.world):
        d = 0 if (a.same_device or ndev < a.world) else r
        procs.append(ctx.Process(target=rank_main, args=(r, a.world, d, q_in, q_out)))
    for p in procs:
        p.start()
    out = {}
    for _ in procs:
        try:
            r, res, err = q_out.get(timeout=180)
        except Exception:  # noqa: BLE001
            break
        out[r] = res if err is None else {"error": err}
    for p in procs:
        p.join(30)
        if p.is_alive():
            p.kill()
    ok = len(out) == a.world and all(v and "error" not in v and all(v.values()) for v in out.values())
    print(json.dumps({"world": a.world, "devices_visible": ndev, "same_device": a.same_device or ndev < a.world,
                      "ranks": {str(k): v for k, v in sorted(out.items())}, "all_ok": ok}), flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
