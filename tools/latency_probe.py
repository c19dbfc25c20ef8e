"""Per-call latency of the file and buffer entries at the sizes a liboxen caller hands them one at a
time (DESIGN §5 "Per-call latency"): hash_file_contents of one file (hasher.rs:114-124, called per
file by restore / checkout / the metadata CLI), one add.rs batch of 64 files (FILE_BATCH_SIZE,
add.rs:41), one host buffer, one device-resident item; the C oracle beside each (read + one-shot XXH3
on one thread, or 16 threads for the batch). Medians over many sequential calls. Prints one JSON line.

    python tools/latency_probe.py [--calls 300]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def med_us(fn, calls: int) -> float:
    fn()
    ts = []
    for _ in range(calls):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(statistics.median(ts) * 1e6, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=300)
    a = ap.parse_args()

    import torch

    from oracle import oracle
    from oxen_amd import _capi, hasher
    from oxen_amd.device import DeviceArena

    oracle.build()
    ctx = _capi.Context(0)
    L = _capi.lib()
    d = tempfile.mkdtemp(prefix="oxh_lat_")
    rng = np.random.default_rng(5)
    res = {"calls": a.calls}
    try:
        files = {}
        for name, size in (("4k", 4096), ("64k", 65536), ("1m", 1 << 20)):
            p = os.path.join(d, name)
            with open(p, "wb") as f:
                f.write(rng.integers(0, 256, size, dtype=np.uint8).tobytes())
            files[name] = p
        batch = []
        for i in range(64):
            p = os.path.join(d, f"b{i}")
            with open(p, "wb") as f:
                f.write(rng.integers(0, 256, int(rng.integers(100, 50_000)), dtype=np.uint8).tobytes())
            batch.append(p)

        def abi_call(paths):
            n = len(paths)
            arr = (ctypes.c_char_p * n)(*[os.fsencode(p) for p in paths])
            out = np.zeros(2 * n, dtype=np.uint64)
            sizes = np.zeros(n, dtype=np.uint64)
            st = np.zeros(n, dtype=np.int32)
            return lambda: _capi.check(L.oxh_hash_files(ctx.handle, arr, n, out.ctypes.data_as(_capi._u64p),
                                                        sizes.ctypes.data_as(_capi._u64p),
                                                        st.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))),
                                       "oxh_hash_files")

        for name, p in files.items():
            res[f"file_{name}_abi_us"] = med_us(abi_call([p]), a.calls)
            res[f"file_{name}_hash_file_contents_us"] = med_us(lambda p=p: hasher.u128_hash_file_contents(p), a.calls)
            res[f"file_{name}_cpu_1thread_us"] = med_us(lambda p=p: oracle.hash_files([p], threads=1), a.calls)
        res["batch64_abi_us"] = med_us(abi_call(batch), a.calls)
        res["batch64_cpu_16threads_us"] = med_us(lambda: oracle.hash_files(batch, threads=16), a.calls)
        res["batch64_cpu_1thread_us"] = med_us(lambda: oracle.hash_files(batch, threads=1), a.calls)
        buf = rng.integers(0, 256, 4096, dtype=np.uint8).tobytes()
        res["buffer_4k_us"] = med_us(lambda: hasher.hash_buffers_128bit([buf], ctx), a.calls)
        streams = [bytes(rng.integers(0, 256, int(rng.integers(5, 200)), dtype=np.uint8)) for _ in range(50)]
        res["streams_50_short_us"] = med_us(lambda: hasher.hash_streams_128bit(streams, ctx), a.calls)
        buf1m = open(files["1m"], "rb").read()
        res["buffer_1m_us"] = med_us(lambda: hasher.hash_buffers_128bit([buf1m], ctx), a.calls)
        res["read_1m_us"] = med_us(lambda: open(files["1m"], "rb").read(), a.calls)
        out = torch.empty((1, 2), dtype=torch.int64, device="cuda")
        for name, size in (("4k", 4096), ("1m", 1 << 20)):
            da = DeviceArena.splitmix([size], seed=3, device="cuda")

            def dev():
                da.hash(out)
                torch.cuda.synchronize()

            res[f"device_item_{name}_launch_sync_us"] = med_us(dev, a.calls)
        # digests agree
        got = hasher.u128_hash_file_contents(files["4k"])
        o, _, _ = oracle.hash_files([files["4k"]], threads=1)
        res["bit_exact"] = got == ((int(o[0, 1]) << 64) | int(o[0, 0]))
    finally:
        ctx.close()
        for f in os.listdir(d):
            os.remove(os.path.join(d, f))
        os.rmdir(d)
    print(json.dumps(res), flush=True)
    if not res.get("bit_exact"):
        sys.exit(1)


if __name__ == "__main__":
    main()
