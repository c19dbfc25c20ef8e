"""Probe K1T counts on simple patterns (debug aid)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
from oxen_amd.device import xxh3_128_text_batch_device
for fill, name in ((0x00, "zero"), (0x0A, "nl"), (0x80, "cont")):
    for L in (241, 255, 256, 300, 1024, 1025, 4096, 4097):
        a = torch.full((L + 64,), fill, dtype=torch.uint8, device="cuda")
        offs = torch.tensor([0], dtype=torch.int64, device="cuda")
        lens = torch.tensor([L], dtype=torch.int64, device="cuda")
        out, cnt = xxh3_128_text_batch_device(a, offs, lens)
        c = cnt.cpu().numpy()[0]
        want = {"zero": (1, L), "nl": (L + 1, L), "cont": (1, 0)}[name]
        print(name, L, tuple(int(x) for x in c), "want", want, "OK" if tuple(int(x) for x in c) == want else "BAD")
