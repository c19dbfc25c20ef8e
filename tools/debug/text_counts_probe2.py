import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
from oxen_amd.device import xxh3_128_text_batch_device
L = 256
for name, pos in (("first16", range(0, 16)), ("b64", range(64, 80)), ("b192", range(192, 208)), ("last16", range(240, 256)), ("b200", [200])):
    h = np.full(L + 64, ord("a"), dtype=np.uint8)
    for p in pos: h[p] = 10
    a = torch.from_numpy(h).cuda()
    out, cnt = xxh3_128_text_batch_device(a, torch.tensor([0], device="cuda"), torch.tensor([L], device="cuda"))
    print(name, int(cnt[0, 0]) - 1, "newlines counted; true", len(list(pos)))
