"""C5 as the dedup experiment runs it: FastCDC chunk digests AND the whole-file digests of the same
16 x 8 GiB device-resident blobs, one after the other vs concurrently (two host threads, two
streams: the 16 serial K1L chains occupy 16 CUs, chunking takes the rest of the chip).

    python tools/dedup_probe.py [--files 16] [--gib 8] [--chunk 65536]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=16)
    ap.add_argument("--gib", type=float, default=8.0)
    ap.add_argument("--chunk", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()

    import torch

    from oxen_amd.device import fastcdc_device, fastcdc_outputs, fill_splitmix, large_digests_device

    dev = torch.device("cuda:0")
    size = int(a.gib * 2**30)
    pitch = (size + 4095) // 4096 * 4096
    arena = torch.empty(pitch * a.files, dtype=torch.uint8, device=dev)
    fill_splitmix(arena, 77)
    offs = np.arange(a.files, dtype=np.uint64) * np.uint64(pitch)
    lens = np.full(a.files, size, dtype=np.uint64)
    bufs = [arena[int(o):int(o) + size] for o in offs]
    mn, av, mx = 4096, a.chunk, 2 * a.chunk
    outs = fastcdc_outputs(arena, lens, mn)
    wall = torch.empty((a.files, 2), dtype=torch.int64, device=dev)
    s_cdc, s_whole = torch.cuda.Stream(), torch.cuda.Stream()

    def chunking():
        with torch.cuda.stream(s_cdc):
            fastcdc_device(arena, offs, lens, mn, av, mx, out=outs, stream=s_cdc)
        s_cdc.synchronize()

    def whole():
        with torch.cuda.stream(s_whole):
            large_digests_device(bufs, out=wall, stream=s_whole)
        s_whole.synchronize()

    chunking(), whole()  # warm-up
    ref = wall.clone()
    seq, conc, t_cdc, t_whole = [], [], [], []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        chunking()
        t1 = time.perf_counter()
        whole()
        t2 = time.perf_counter()
        seq.append(t2 - t0)
        t_cdc.append(t1 - t0)
        t_whole.append(t2 - t1)
        t0 = time.perf_counter()
        th = [threading.Thread(target=chunking), threading.Thread(target=whole)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        conc.append(time.perf_counter() - t0)
    same = bool(torch.equal(wall, ref))
    print(json.dumps({"files": a.files, "gib_each": a.gib, "chunk": a.chunk,
                      "chunking_s": round(float(np.median(t_cdc)), 4), "whole_file_s": round(float(np.median(t_whole)), 4),
                      "sequential_s": round(float(np.median(seq)), 4), "concurrent_s": round(float(np.median(conc)), 4),
                      "whole_digests_identical": same}), flush=True)
    if not same:
        sys.exit(1)


if __name__ == "__main__":
    main()
