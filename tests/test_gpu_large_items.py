"""K1 on device-resident items above 1 GiB and above 2 GiB: each wave's buffer descriptor covers a
1 GiB window and is re-based as the wave walks its item (xxh3_kernels.hip, the `rr >> 18` window
step), so these are the lengths that exercise it. Misaligned starts (byte-packed arena) included."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GIB = 1 << 30


@pytest.mark.parametrize("lens", [
    [4097, GIB + 4097, 3],           # 1 GiB + 4 097 B starting at byte 4 097 (not dword-aligned)
    [13, 2 * GIB + 12_345, 1000],    # above 2 GiB (two re-bases), start at byte 13
], ids=["1GiB+4097_misaligned", "2GiB+12345_misaligned"])
def test_k1_items_over_a_descriptor_window(cuda, oracle_lib, lens):
    import torch

    from oxen_amd import _capi
    from oxen_amd.device import DeviceArena, to_numpy_u64

    da = DeviceArena.splitmix(lens, seed=77, device=cuda, align=1)
    assert int(da.offsets_host[1]) == lens[0]  # byte-packed: the big item starts unaligned
    host = da.arena.cpu().numpy()
    want = oracle_lib.batch(host, da.offsets_host, da.lens_host, 4)
    for mode in (_capi.OXH_MODE_AUTO, _capi.OXH_MODE_WAVE, _capi.OXH_MODE_WAVE_PACKED):
        got = to_numpy_u64(da.hash(mode=mode)).reshape(-1, 2)
        torch.cuda.synchronize()
        assert np.array_equal(got, want), mode
    del da
    torch.cuda.empty_cache()
