import sys, os, ctypes
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oxen_amd import _capi
_capi.LIB_PATH = os.path.join(ROOT, "tools/debug/build/liboxen_hash_dbg.so")
import numpy as np, torch
L = 256
h = np.full(L + 64, 10, dtype=np.uint8)
a = torch.from_numpy(h).cuda()
out = torch.zeros((1, 2), dtype=torch.int64, device="cuda")
cnt = torch.zeros(400, dtype=torch.int64, device="cuda")
offs = torch.tensor([0], device="cuda"); lens = torch.tensor([L], device="cuda")
_capi.check(_capi.lib().oxh_xxh3_128_text_batch_device(a.data_ptr(), offs.data_ptr(), lens.data_ptr(), 1, out.data_ptr(), cnt.data_ptr(), 0), "x")
torch.cuda.synchronize()
c = cnt.cpu().numpy()
print("total", c[0] - 1)
for lane in range(64):
    print(lane, "ring", c[2 + 3 * lane], "after", c[3 + 3 * lane], "skip", c[4 + 3 * lane])
