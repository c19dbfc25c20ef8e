"""K2 commit driver timing at config 3's tree shape (200 000 files in 1 000 dirs), GPU box only.

Times the C++ K2 driver (oxen_amd/host/commit_writer.cpp via tests/native/commit_tree_cli, best of 5
calls in one process) and merkle.commit_tree (the Python driver; both issue three batched GPU passes)
against the Python driver with its hash calls answered by the C oracle on the host threads, and the
scalar restatement of commit_writer.rs (oracle/commit_oracle.py); checks every vnode id and dir hash
equal. Prints one JSON line.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]


def main():
    import numpy as np

    import _commit
    from oracle import commit_oracle, oracle
    from oxen_amd import hasher, merkle

    threads = int(os.environ.get("OXH_NUM_THREADS", "16"))
    entries, _ = _commit.staged_commit(n_files=200_000, n_dirs=1000)
    staged = _commit.to_staged(entries)
    ctx = hasher.default_context()
    merkle.commit_tree(staged, None, 10_000, _commit.salt, ctx=ctx)  # warm-up
    stages = {}
    real = hasher.hash_streams_128bit

    def timed(streams, ctx=None):
        t0 = time.perf_counter()
        r = real(streams, ctx)
        stages.setdefault("hash_calls_s", []).append(round(time.perf_counter() - t0, 4))
        stages.setdefault("stream_bytes", []).append(sum(len(s) for s in streams))
        return r

    hasher.hash_streams_128bit = timed
    t0 = time.perf_counter()
    vn, dh = merkle.commit_tree(staged, None, 10_000, _commit.salt, ctx=ctx)
    gpu_s = time.perf_counter() - t0
    hasher.hash_streams_128bit = real

    def cpu_streams(streams, ctx=None):
        lens = np.array([len(s) for s in streams], dtype=np.uint64)
        offs = np.zeros(len(streams), dtype=np.uint64)
        offs[1:] = np.cumsum(lens[:-1])
        out = oracle.batch(np.frombuffer(b"".join(streams), dtype=np.uint8), offs, lens, threads)
        return [(int(hi) << 64) | int(lo) for lo, hi in out]

    hasher.hash_streams_128bit = cpu_streams
    t0 = time.perf_counter()
    cvn, cdh = merkle.commit_tree(staged, None, 10_000, _commit.salt)
    cpu_driver_s = time.perf_counter() - t0
    hasher.hash_streams_128bit = real
    t0 = time.perf_counter()
    rvn, rdh = commit_oracle.commit_tree(entries, {}, 10_000, _commit.salt)
    scalar_s = time.perf_counter() - t0
    import subprocess

    from oxen_amd import build

    build.build_host()
    r = subprocess.run([build.COMMIT_CLI, "--reps", "5"], input=_commit.to_cli_input(entries, {}, 10_000),
                       capture_output=True, text=True, check=True)
    nvn, ndh, _, native_s = _commit.parse_cli_output(r.stdout)
    exact = ({d: h.value for d, h in dh.items()} == rdh == {d: h.value for d, h in cdh.items()} == ndh
             and all([v.id.value for v in vn[d][0]] == [i for i, _ in rvn[d]] for d in rvn)
             and all([i for i, _ in nvn[d]] == [i for i, _ in rvn[d]] for d in rvn))
    print(json.dumps({
        "config": "K2 commit at C3 shape: 200 000 files, 1 000 dirs, vnode_size 10 000",
        "native_cpp_commit_tree_s": round(native_s, 4),
        "gpu_commit_tree_s": round(gpu_s, 3), **stages,
        "host_driver_with_cpu_hash_s": round(cpu_driver_s, 3), "cpu_threads": threads,
        "scalar_restatement_s": round(scalar_s, 3),
        "vnodes": sum(len(v[0]) for v in vn.values()), "dirs": len(dh), "bit_exact": exact,
    }))


if __name__ == "__main__":
    main()
