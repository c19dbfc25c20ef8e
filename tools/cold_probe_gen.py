"""Writes C3-shaped files for tools/cold_probe (200 000 x 49 292 B in 1 000 dirs; content irrelevant to
the I/O being measured) and prints their paths. python tools/cold_probe_gen.py DIR [N]"""
import os
import sys

import numpy as np

root, n = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 200_000
block = np.random.default_rng(0).integers(0, 256, 49_292 + 4096, dtype=np.uint8).tobytes()
for i in range(n):
    d = os.path.join(root, f"split_{i % 1000}")
    if i < 1000:
        os.makedirs(d, exist_ok=True)
    p = os.path.join(d, f"img_{i}.tiff")
    with open(p, "wb") as f:
        f.write(block[i % 4096:i % 4096 + 49_292])
    print(p)
