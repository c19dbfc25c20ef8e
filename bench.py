"""Benchmark: device-resident XXH3-128 content hashing (the `oxen add` hash stage) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|c4]

One step = one batched K1 launch hashing every buffer of the rank's shard, already resident in HBM
(plus, for N > 1, the single all-gather of the 16-B digest table over RCCL). Workload (weak
scaling, per GPU): BASELINE.json configs[1] -- 100 000 x 64 KiB splitmix64 blobs (6.1 GiB).
N > 1: one process per GPU. Under torch.distributed.run (WORLD_SIZE set) this process is one rank
and WORLD_SIZE must equal --gpus; without a launcher, `--gpus N` starts the N ranks itself before
anything touches the GPU and exits with the worst rank's status.
Prints ONE JSON line on rank 0 (the driver's contract), including:
  roofline      achieved HBM read GB/s of the K1 kernel (algorithmic bytes = buffer lengths) vs the
                8 TB/s MI355X peak; `traffic` = PMC-measured HBM bytes per launch when a matching
                profiles/*traffic*.json exists (rocprofv3 FETCH_SIZE, gfx950 x2 correction).
  cpu_baseline  the C oracle (oracle/, a restatement of the reference's XXH3-128) timed on the
                host cores over a bounded sample of the same workload; the GPU digests of that
                sample are checked bit-exact against it.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GiB/s hashed device-resident on `oxen add` (N files); digests bit-exact"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
WORKLOADS = {
    # name: (items per GPU, bytes per item, BASELINE config)
    "c2": (100_000, 65_536, "100 000 x 64 KiB random blobs, device-resident, 1 MI355X (BASELINE configs[1])"),
    "c4": (125_000, 262_144, "1 000 000 x 256 KiB blobs / 8 GPUs = 125 000 x 256 KiB per GPU (BASELINE configs[3])"),
    # launcher / multi-rank mechanics in tests only; never a bench line
    "t": (2_048, 65_536, "test size: 2 048 x 64 KiB (rank-launch mechanics)"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def usable_cpus() -> int:
    """CPUs this process may use: the affinity mask capped by the cgroup-v2 quota (cpu.max), as the
    library's engine counts them; os.cpu_count() sees the whole machine on the GPU box."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max" and int(period) > 0:
            n = min(n, max(1, -(-int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` without a launcher: start N rank processes of this script (one per GPU,
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their environment, as torch.distributed.run sets
    them) before this process touches the GPU, wait for all, and return the worst exit code. The
    first rank to fail takes the others down (a dead rank would leave the rest in a barrier)."""
    import subprocess

    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GROUP_RANK="0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    worst = 0
    live = set(range(n))
    while live:
        for r in sorted(live):
            rc = procs[r].poll()
            if rc is None:
                continue
            live.discard(r)
            if rc != 0:
                log(f"[bench] rank {r} exited with {rc}; stopping the other ranks")
                worst = worst or rc
                for q in live:
                    procs[q].terminate()
        time.sleep(0.05)
    for p in procs:
        p.wait()
        if p.returncode != 0 and worst == 0:
            worst = p.returncode
    return worst if worst >= 0 else 128 - worst


def cpu_baseline(da, gpu_digests: np.ndarray, seed: int, budget_s: float = 10.0) -> dict:
    """Oracle (C, multi-threaded) on a bounded sample of the workload; checks the GPU digests of it."""
    import torch

    from oracle import oracle
    from oxen_amd.workloads import splitmix_bytes

    oracle.build()
    threads = usable_cpus()
    item_len = int(da.lens_host[0])
    nsample = min(da.n, max(threads, (1 << 30) // max(item_len, 1)))  # 1 GiB: beyond the host L3
    idx = np.linspace(0, da.n - 1, nsample).astype(np.int64)
    host = np.empty(nsample * item_len, dtype=np.uint8)
    # the sampled items are copied back from HBM (regenerating 1 GiB on the host is slower)
    idx_t = torch.from_numpy(idx).to(da.arena.device)
    rows = da.arena[: da.n * item_len].view(da.n, item_len) if int(da.offsets_host[1] - da.offsets_host[0]) == item_len else None
    if rows is not None:
        host[:] = rows.index_select(0, idx_t).cpu().numpy().reshape(-1)
    else:
        for j, i in enumerate(idx):
            host[j * item_len:(j + 1) * item_len] = splitmix_bytes(seed, int(da.offsets_host[i]), item_len)
    # spot-check that what came back is the splitmix stream the host can regenerate
    assert np.array_equal(host[:item_len], splitmix_bytes(seed, int(da.offsets_host[idx[0]]), item_len))
    offs = np.arange(nsample, dtype=np.uint64) * np.uint64(item_len)
    lens = np.full(nsample, item_len, dtype=np.uint64)
    want = oracle.batch(host, offs, lens, threads)  # warm + reference digests
    exact = bool(np.array_equal(want, gpu_digests[idx]))
    t0 = time.perf_counter()
    passes = 0
    while True:
        oracle.batch(host, offs, lens, threads)
        passes += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    gib = passes * nsample * item_len / 2**30
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": round(gib / dt, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": f"{nsample} of {da.n} items x {item_len} B ({nsample * item_len / 2**20:.0f} MiB), "
                      f"{passes} passes in {dt:.1f} s, oracle/xxh3_oracle.c (SSE2 stripes, as xxhash-rust on x86-64), {threads} threads, {cpu_model}",
            "digests_bit_exact_on_sample": exact,
            "oxen_add_c1": cpu_oxen_add_c1(threads)}


def cpu_oxen_add_c1(threads: int, reps: int = 3) -> dict:
    """The reference's own CPU-runnable case (BASELINE configs[0]: `oxen init; oxen add .` on the
    1 000-file text repo of benchmark/generate_text_repo.py), timed in the same run: no `oxen` binary
    exists here, so it is the add loop restated in C (oracle/: stat, read, XXH3-128, then
    store_version_from_reader's re-read, verify hash, write, fsync of blob and parent, rename)."""
    import shutil
    import tempfile

    from oracle import oracle
    from oxen_amd.workloads import write_text_repo

    d = tempfile.mkdtemp(prefix="oxh_c1_")
    try:
        paths = write_text_repo(d, 1000)
        nbytes = sum(os.path.getsize(p) for p in paths)
        root = os.path.join(d, ".oxen", "versions", "files")
        best, ok = None, True
        for _ in range(reps):
            shutil.rmtree(os.path.join(d, ".oxen"), ignore_errors=True)
            t0 = time.perf_counter()
            out, _, status, stored = oracle.add_files(paths, root, threads)
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
            ok = ok and bool((status == 0).all()) and int(stored.sum()) == len(paths)
        # the known answer of texts/file_0.txt ("File content 0")
        ok = ok and format((int(out[0][1]) << 64) | int(out[0][0]), "x") == "393ba5849f5590fc5985c4bbcec0003f"
        return {"ms": round(best * 1e3, 2), "files": len(paths), "bytes": nbytes, "cores": threads, "kind": "port",
                "what": "oxen add . restated (hash + verify-before-publish + durable blob write), best of %d" % reps,
                "ok": ok}
    finally:
        shutil.rmtree(d, ignore_errors=True)


def load_traffic(workload: str):
    """PMC-derived HBM bytes per K1 launch for this workload, if profiled (tools/pmc_traffic.py)."""
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*traffic*.json"))):
        try:
            d = json.load(open(p))
        except (OSError, ValueError):
            continue
        if d.get("workload") == workload and d.get("hbm_bytes_per_launch"):
            best = d
    return best


def load_profile(workload: str):
    """The newest rocprofv3 kernel-trace summary of the K1 kernel for this workload
    (profiles/*_profile_<workload>.json, written by tools/prof_summary.py from the stats CSV)."""
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_profile_{workload}.json"))):
        try:
            d = json.load(open(p))
        except (OSError, ValueError):
            continue
        if d.get("avg_ms"):
            best = dict(d, source=os.path.relpath(p, ROOT))
    return best


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--prewarm-s", type=float, default=0.5,
                    help="seconds of untimed hashing before the warmup steps (clock ramp); 0 = off")
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--backend", default="nccl", help="nccl (= RCCL on ROCm); gloo only to rehearse N>1 on one GPU")
    ap.add_argument("--gather", choices=["abi", "torch", "host"], default=None,
                    help="N > 1: the digest gather through the C ABI (oxh_gather_digests; the default on nccl), "
                         "torch.distributed's all-gather (the fallback when the ABI gather cannot come up), or "
                         "host tables over the process group (the default on gloo). abi on gloo: the ABI gather "
                         "with the id broadcast over gloo -- with OXH_RCCL_LIB=tests/native/libfake_rccl.so it "
                         "rehearses the whole N > 1 step with every rank on one GPU (tests/test_bench_launch.py)")
    ap.add_argument("--dist", action="store_true",
                    help="take the N>1 path (process group, pipelined RCCL gather) even at WORLD_SIZE=1: "
                         "rehearses the multi-GPU step on a one-GPU box under torch.distributed.run")
    args = ap.parse_args()
    if args.gather is None:
        args.gather = "abi" if args.backend == "nccl" else "host"
    if args.gpus < 1:
        log("[bench] --gpus must be >= 1")
        sys.exit(2)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))  # this process never touches the GPU
    if env_world is not None and int(env_world) != args.gpus:
        log(f"[bench] WORLD_SIZE={env_world} but --gpus {args.gpus}: launch one rank per GPU, N = --gpus")
        sys.exit(2)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = max(1, torch.cuda.device_count())
    if world > ndev and args.backend == "nccl":
        log(f"[bench] {world} ranks but {ndev} visible GPU(s): RCCL needs one GPU per rank "
            "(--backend gloo rehearses N > 1 on fewer GPUs)")
        sys.exit(2)
    dev = torch.device(f"cuda:{local_rank % ndev}")
    torch.cuda.set_device(dev)
    multi = world > 1 or args.dist  # the distributed step (barriers, gather, max over ranks)
    if multi:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.backend)

    from oxen_amd import _capi
    from oxen_amd import build as hb
    from oxen_amd.device import DeviceArena, to_numpy_u64
    from oxen_amd.shard import PipelinedGather, gather_digest_table

    if rank == 0:
        hb.build()
    if multi:
        dist.barrier()
    _capi.lib().oxh_set_kernel_variant(args.variant)

    n_items, item_len, desc = WORKLOADS[args.workload]
    # weak scaling: every rank owns its own n_items (global item ids rank*n_items ...); the seed is
    # offset per rank so shards differ
    seed = args.seed + rank
    lens = np.full(n_items, item_len, dtype=np.uint64)
    da = DeviceArena.splitmix(lens, seed=seed, device=dev)
    out = torch.empty((n_items, 2), dtype=torch.int64, device=dev)
    counts = [n_items] * world
    torch.cuda.synchronize()

    # N > 1 over RCCL: each step's digest gather runs on the collective's stream while the next step
    # hashes into the other of two digest tables (shard.PipelinedGather: the gather of step k overlaps
    # the hash of k+1; a table is rewritten only after the gather that read it has finished)
    # The gather is the C ABI's oxh_gather_digests (comm.py / csrc/comm.cpp: RCCL all-gather over xGMI),
    # the call a Rust host links; rank 0's communicator id travels over the process group.
    comm = None
    gather_via = "none"
    if multi and args.backend != "nccl" and args.gather == "abi":
        # the ABI gather over a gloo group (the id travels over gloo): no fallback, a failure is the run's
        from oxen_amd.comm import comm_from_process_group

        comm = comm_from_process_group(rank, world, dev.index)
        gather_via = "oxh_gather_digests (process group: %s)" % args.backend
    elif multi and args.backend == "nccl":
        from oxen_amd.comm import comm_from_process_group

        err = None
        try:
            if args.gather == "torch":
                raise RuntimeError("--gather torch")
            comm = comm_from_process_group(rank, world, dev.index)
        except Exception as e:  # noqa: BLE001 -- decided below, by every rank together
            err = e
        # every rank takes the same path: the ABI gather only if it came up on all of them
        ok = torch.tensor([0 if err is None else 1], dtype=torch.int32, device=dev)
        dist.all_reduce(ok)
        if int(ok.item()):
            if err is not None:
                log(f"[bench] rank {rank}: oxh_comm_create failed ({err})")
            if comm is not None:
                comm.close()
                comm = None
            why = "--gather torch" if args.gather == "torch" else "the ABI gather failed to come up"
            if args.gather != "torch":
                log("[bench] the ABI gather is unavailable on some rank: torch's all-gather over the process group instead")
            gather_via = f"torch.distributed all_gather_into_tensor (RCCL; {why})"
        else:
            gather_via = "oxh_gather_digests"
    pipe = PipelinedGather(n_items, world, dev, comm=comm) if (comm is not None or gather_via.startswith("torch")) else None

    def step():
        if pipe is not None:
            b, local = pipe.next_local()
            da.hash(local)
            return pipe.gather(b), local
        da.hash(out)
        if multi:
            return gather_digest_table(out.cpu(), counts), out  # gloo rehearsal: host tables
        return out, out

    def drain():  # the current stream waits for every outstanding gather
        if pipe is not None:
            pipe.drain()

    # Clock ramp: the first bench process on a fresh box ran K1 2-4 % slow when only the W warmup steps
    # (a few ms of work) came before the timed region (profiles/r05/r05v_*, r05u_*). Hash the same
    # tables for prewarm_s seconds first (untimed; its launch count goes into the JSON line so the
    # profile summary can find the timed launches), then the W warmup steps and the K timed steps.
    t_pre = time.perf_counter()
    prewarm_launches = 0
    while time.perf_counter() - t_pre < args.prewarm_s:
        for _ in range(8):
            da.hash(out)
        prewarm_launches += 8
        torch.cuda.synchronize()
    prewarm_s = time.perf_counter() - t_pre
    for _ in range(args.warmup):
        step()
    drain()
    torch.cuda.synchronize()
    if multi:
        dist.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(args.steps):
        table, last = step()
    drain()
    ev1.record()
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    if multi:
        dist.barrier()
    torch.cuda.synchronize()
    gpu_s = ev0.elapsed_time(ev1) / 1e3
    # per-launch kernel time, from HIP events on the launch stream (no collective in this window):
    # (a) each launch alone between its own two events, the GPU idle before it -- what a profiler's
    # per-dispatch duration measures, and the figure the roofline uses; (b) back to back, where one
    # launch's last waves overlap the next one's first (a throughput figure, reported beside it)
    kreps = max(5, args.steps)
    iso = []
    for _ in range(kreps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        da.hash(out)
        e1.record()
        torch.cuda.synchronize()
        iso.append(e0.elapsed_time(e1) / 1e3)
    kernel_s = float(np.median(iso))
    kev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    kev[0].record()
    for _ in range(kreps):
        da.hash(out)
    kev[1].record()
    torch.cuda.synchronize()
    kernel_b2b_s = kev[0].elapsed_time(kev[1]) / 1e3 / kreps

    elapsed = max(wall, gpu_s)
    log(f"[bench] rank {rank}: wall {wall * 1e3:.3f} ms, events {gpu_s * 1e3:.3f} ms, enqueue {t_enq * 1e3:.3f} ms, "
        f"kernel {kernel_s * 1e3:.4f} ms alone (median of {kreps}), {kernel_b2b_s * 1e3:.4f} ms back to back; "
        f"x {args.steps} = {kernel_b2b_s * args.steps * 1e3:.3f} ms")
    t = torch.tensor([elapsed, kernel_s], dtype=torch.float64, device=dev)
    if multi:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, kernel_max = float(t[0]), float(t[1])

    bytes_per_rank = int(lens.sum())
    total_bytes = bytes_per_rank * world * args.steps
    value = total_bytes / elapsed / 2**30

    result = None
    if rank == 0:
        digests = to_numpy_u64(last).reshape(-1, 2)
        if multi:
            assert table.shape[0] == n_items * world
            assert np.array_equal(to_numpy_u64(table[:n_items]).reshape(-1, 2), digests)
            # every rank's shard digests arrived: rank r's first item is regenerated and checked
            from oracle import oracle
            from oxen_amd.workloads import splitmix_bytes

            full = to_numpy_u64(table).reshape(-1, 2)
            for r in range(world):
                want = oracle.xxh3_128(splitmix_bytes(args.seed + r, int(da.offsets_host[0]), item_len).tobytes())
                assert (int(full[r * n_items, 0]), int(full[r * n_items, 1])) == want, r
        achieved = bytes_per_rank / kernel_s / 1e9
        tr = load_traffic(args.workload)
        roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 4),
                    "traffic": (tr["hbm_bytes_per_launch"] if tr else None),
                    "kernel": "xxh3_wave_kernel (K1)", "kernel_ms": round(kernel_s * 1e3, 4),
                    "kernel_ms_how": f"HIP events around each launch alone on the launch stream, median of {kreps}",
                    "kernel_ms_back_to_back": round(kernel_b2b_s * 1e3, 4),
                    "algorithmic_bytes_per_launch": bytes_per_rank}
        if tr:
            roofline["traffic_source"] = tr.get("source")
        prof = load_profile(args.workload)
        if prof:  # the rocprofv3 kernel-trace average of this same command, committed under profiles/
            roofline["profile"] = {"avg_ms": prof["avg_ms"], "calls": prof["calls"], "command": prof["command"],
                                   "source": prof["source"],
                                   "frac": round(bytes_per_rank / (prof["avg_ms"] / 1e3) / 1e9 / HBM_PEAK_GBS, 4)}
            if prof.get("timed_region"):  # the profiled launches of the timed steps alone
                tr = prof["timed_region"]
                roofline["profile"]["timed_region"] = {"avg_ms": tr["avg_ms"], "launches": tr["launches"],
                                                       "frac": round(bytes_per_rank / (tr["avg_ms"] / 1e3) / 1e9 / HBM_PEAK_GBS, 4)}
        cpu = None
        if not args.no_cpu_baseline and world == 1:  # the CPU baseline is a rank-0, N = 1 figure
            cpu = cpu_baseline(da, digests, seed, args.cpu_budget)
        result = {
            "metric": METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (splitmix64 byte stream, seed %d+rank), device-resident in HBM" % args.seed,
            "config": {"workload": desc, "items_per_gpu": n_items, "item_bytes": item_len,
                       "bytes_per_gpu": bytes_per_rank, "parallelism": (f"files sharded x{world}, one RCCL all-gather of the digests per step "
                                               f"({gather_via if gather_via != 'none' else 'torch gloo rehearsal'})")
                       if multi else "single GPU",
                       "kernel_variant": args.variant or "auto (8: 2-round ring, items > 16 KiB)"},
            "roofline": roofline,
            "prewarm": {"seconds": round(prewarm_s, 3), "launches": prewarm_launches,
                        "what": "untimed K1 launches over the same tables before the warmup steps (clock ramp)"},
            "cpu_baseline": cpu,
        }
        print(json.dumps(result), flush=True)
    if multi:
        dist.barrier()
        if comm is not None:
            comm.close()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
