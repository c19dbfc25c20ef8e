"""Measure attainable HBM read bandwidth on this GPU (diagnostic for the K1 roofline).

    python tools/readbw.py [--gib 6.1]

Prints one JSON line: best flat dwordx4 read stream, the K1 access pattern with the hash replaced
by an xor, and the real K1 kernel on the same bytes (C2 shape), all timed with HIP events on the
launch stream, interleaved in one process (median of rounds).
"""
from __future__ import annotations

import ctypes
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SO = os.path.join(ROOT, "tools", "libreadbw.so")


def build():
    src = os.path.join(ROOT, "tools", "readbw.hip")
    if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(src):
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", "-o", SO, src],
                       check=True)
    L = ctypes.CDLL(SO)
    L.readbw_flat.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    L.readbw_items.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    return L


def main():
    import torch

    from oxen_amd.device import DeviceArena

    L = build()
    n, item = 100_000, 65_536
    da = DeviceArena.splitmix([item] * n, seed=1)
    nbytes = n * item
    sink = torch.zeros(1024, dtype=torch.int32, device="cuda")
    out = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    st = torch.cuda.current_stream().cuda_stream

    def timed(fn, reps=10):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / 1e3 / reps

    variants = {}
    for blocks in (2048, 4096, 8192, 16384):
        for unroll in (1, 4, 8, 108):
            variants[f"flat_b{blocks}_u{unroll}"] = (lambda b=blocks, u=unroll:
                                                      L.readbw_flat(da.arena.data_ptr(), nbytes, sink.data_ptr(), b, u, st))
    # memory-pattern-only kernels over a larger arena so item pitches can be skewed
    big = torch.empty(n * (item + 4096), dtype=torch.uint8, device="cuda")
    big.fill_(7)
    for kind, kname in ((0, "rows"), (1, "flat1k"), (2, "rows_nt"), (3, "flat1k_nt")):
        for pitch in (item, item + 256, item + 4096):
            variants[f"items_{kname}_pitch{pitch}"] = (lambda k=kind, p=pitch:
                                                       L.readbw_items(big.data_ptr(), n, item, p, k, sink.data_ptr(), st))
    from oxen_amd import _capi

    def k1(v):
        def f():
            _capi.lib().oxh_set_kernel_variant(v)
            da.hash(out)
        return f

    ref = None
    for v in (0, 8, 72):  # the shipped K1 shapes (the probe build has the others: tools/build_probe_lib.py)
        variants[f"k1_xxh3_v{v}"] = k1(v)
        k1(v)()
        torch.cuda.synchronize()
        d = out.cpu()
        if ref is None:
            ref = d
        assert torch.equal(ref, d), f"variant {v} digests differ from variant 0"
    # K1T (hash + fused text counts) on the same arena: the price of the fusion
    from oxen_amd.device import xxh3_128_text_batch_device

    cnt = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    variants["k1t_text_fused"] = lambda: (_capi.lib().oxh_set_kernel_variant(0),
                                         xxh3_128_text_batch_device(da.arena, da.offsets, da.lens, out, cnt))
    # K1 (default variant) on skewed pitches and on a 4x larger batch (tail effect)
    _capi.lib().oxh_set_kernel_variant(0)
    for pad in (256, 4096):
        dap = DeviceArena.splitmix([item] * n, seed=1, pad=pad)
        variants[f"k1_xxh3_v0_pitch{item + pad}"] = (lambda d=dap: (_capi.lib().oxh_set_kernel_variant(0), d.hash(out)))
    big4 = DeviceArena.splitmix([item] * (4 * n), seed=1)
    out4 = torch.empty((4 * n, 2), dtype=torch.int64, device="cuda")
    variants["k1_xxh3_v0_x4items_per_byte"] = lambda: (_capi.lib().oxh_set_kernel_variant(0), big4.hash(out4))
    # clock ramp first (as bench.py's pre-warm): 0.5 s of K1 before any timed round
    import time as _time

    t_pre = _time.perf_counter()
    while _time.perf_counter() - t_pre < 0.5:
        for _ in range(8):
            da.hash(out)
        torch.cuda.synchronize()
    res = {k: [] for k in variants}
    for _ in range(5):
        for k, fn in variants.items():
            res[k].append((4 if "x4items" in k else 1) * nbytes / timed(fn) / 1e9)
    med = {k: round(statistics.median(v), 1) for k, v in res.items()}
    best_flat = max((v, k) for k, v in med.items() if k.startswith("flat"))
    print(json.dumps({"unit": "GB/s", "bytes": nbytes, "median_of_5": med,
                      "attainable_read_GBs": best_flat[0], "attainable_variant": best_flat[1]}))


if __name__ == "__main__":
    main()
