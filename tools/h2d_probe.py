"""Pinned host -> device copy rate on this box: one 64 MiB window per copy, spread over 1, 2 or 4
streams, from 8 pinned windows (the host chunk pipeline's ring shape) and from one 1 GiB buffer.
Prints one JSON object (GB/s per shape, best of 5 passes over 4 GiB)."""
import json
import time

import torch


def rate(nstreams: int, win: int, nwin: int, total: int) -> float:
    host = [torch.empty(win, dtype=torch.uint8).pin_memory() for _ in range(nwin)]
    dev = torch.empty(total, dtype=torch.uint8, device="cuda")
    streams = [torch.cuda.Stream() for _ in range(nstreams)]
    best = 0.0
    for _ in range(5):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for k in range(total // win):
            with torch.cuda.stream(streams[k % nstreams]):
                dev[k * win:(k + 1) * win].copy_(host[k % nwin], non_blocking=True)
        torch.cuda.synchronize()
        best = max(best, total / (time.perf_counter() - t) / 1e9)
    return round(best, 2)


def main():
    torch.ones(1, device="cuda")
    total = 4 << 30
    res = {}
    for win_mib in (64, 256, 1024):
        for ns in (1, 2, 4):
            res[f"{win_mib}MiB_x{ns}streams"] = rate(ns, win_mib << 20, max(1, min(8, 512 // win_mib)), total)
            print(json.dumps(res), flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
