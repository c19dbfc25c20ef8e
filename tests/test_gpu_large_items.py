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
    [7, 4 * GIB + 777, 5],           # above 2^32 bytes (four re-bases; any 32-bit offset wraps here)
], ids=["1GiB+4097_misaligned", "2GiB+12345_misaligned", "4GiB+777_misaligned"])
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


def test_k1l_default_pieces_device(cuda, oracle_lib, monkeypatch):
    """K1L as it ships -- OXH_BIG_PIECE_MIB unset (1 GiB pieces) -- over buffers
    larger than one piece: 2 GiB + 4 097 B at a misaligned start (two full pieces and a last piece of
    4 097 B), 1 GiB - 1 B (one piece) and 4 GiB + 333 B (above 2^32), through
    oxh_xxh3_128_large_batch_device."""
    import torch

    from oxen_amd.device import fill_splitmix, large_digests_device

    monkeypatch.delenv("OXH_BIG_PIECE_MIB", raising=False)
    sizes = [2 * GIB + 4097, GIB - 1, 4 * GIB + 333]  # the last one above 2^32 bytes, five pieces
    starts = [5, 0, 3]
    bufs, views = [], []
    for i, (n, s) in enumerate(zip(sizes, starts)):
        b = torch.empty(n + 64, dtype=torch.uint8, device=cuda)
        fill_splitmix(b, 900 + i)
        bufs.append(b)
        views.append(b[s:s + n])
    got = large_digests_device(views, sizes).cpu().numpy().view(np.uint64).reshape(-1, 2)
    torch.cuda.synchronize()
    for i, (b, n, s) in enumerate(zip(bufs, sizes, starts)):
        host = b.cpu().numpy()
        want = oracle_lib.batch(host, np.array([s], dtype=np.uint64), np.array([n], dtype=np.uint64), 8)
        assert np.array_equal(got[i], want[0]), (i, n)
        del host
    del bufs, views
    torch.cuda.empty_cache()


def test_k1l_default_pieces_file(cuda, oracle_lib, tmp_path, monkeypatch):
    """The C5 whole-file digest path as it ships (hasher.rs:150-174's branch): one 2.5 GiB file --
    sparse, with written regions at the start, across both 1 GiB piece boundaries and at the end --
    through oxh_hash_files (three 1 GiB-piece rounds of the large-file pipeline) and oxh_add_files
    (the same pieces also streamed to the blob's temp, renamed once the digest is known), checked
    against the oracle's read of the file and of the published blob."""
    import os

    from oxen_amd import hasher
    from oxen_amd.workloads import splitmix_bytes

    monkeypatch.delenv("OXH_BIG_PIECE_MIB", raising=False)
    size = 5 * GIB // 2 + 333
    p = tmp_path / "big.parquet"
    with open(p, "wb") as fh:
        fh.truncate(size)
        for off in (0, GIB - 2000, GIB + 77, 2 * GIB - 4096, size - 5000):
            fh.seek(off)
            fh.write(splitmix_bytes(off, 0, 4096).tobytes()[: size - off])
    out, sizes, status = oracle_lib.hash_files([str(p)], threads=8)
    want_int = (int(out[0, 1]) << 64) | int(out[0, 0])
    assert int(status[0]) == 0 and int(sizes[0]) == size
    d, sz, st = hasher.hash_files_128bit([str(p)])
    assert st == [0] and sz == [size] and d == [want_int]
    root = tmp_path / "versions"
    root.mkdir()
    d2, sz2, st2, stored = hasher.add_files([str(p)], str(root))
    assert st2 == [0] and d2 == [want_int] and stored == [True]
    blob = hasher.version_path(str(root), want_int)
    out_b, sizes_b, status_b = oracle_lib.hash_files([blob], threads=8)
    assert int(status_b[0]) == 0 and int(sizes_b[0]) == size
    assert (int(out_b[0, 1]) << 64) | int(out_b[0, 0]) == want_int
    os.remove(blob)


def test_large_item_buffer_allocations_stay_rare(cuda, oracle_lib, tmp_path, monkeypatch):
    """the large-file piece buffers (files above a staging slot) are sized for the most
    files the engine batches (OXH_BIG_FILES) on first use, so a context allocates them once -- each
    allocation is a hipFree / hipMalloc that synchronises the whole device -- not once per new batch
    size. Rising batches of 1, 2, 3, 4 and 6 large files, the device entry beside them: one allocation;
    raising OXH_BIG_FILES to 8 takes exactly one more. Every digest equals the oracle's."""
    from oxen_amd import _capi, hasher

    monkeypatch.setenv("OXH_BIG_PIECE_MIB", "4")
    monkeypatch.delenv("OXH_BIG_FILES", raising=False)
    rng = np.random.default_rng(45)
    paths, want = [], []
    for i in range(8):
        d = rng.integers(0, 256, (3 << 20) + 5000 + 777 * i, dtype=np.uint8)  # 3 MiB + : above a 1 MiB slot
        p = tmp_path / f"big{i}"
        p.write_bytes(d.tobytes())
        paths.append(str(p))
        w = oracle_lib.batch(d, np.zeros(1, np.uint64), np.array([len(d)], np.uint64))[0]
        want.append((int(w[1]) << 64) | int(w[0]))
    with _capi.Context(0, staging_bytes=1 << 20) as ctx:
        assert ctx.counters()["big_allocs"] == 0
        for n in (1, 2, 3, 4, 6):
            got, sizes, status = hasher.hash_files_128bit(paths[:n], ctx=ctx)
            assert status == [0] * n and got == want[:n], n
        c = ctx.counters()
        assert c["big_allocs"] == 1, c
        monkeypatch.setenv("OXH_BIG_FILES", "8")
        got, _, status = hasher.hash_files_128bit(paths, ctx=ctx)
        assert status == [0] * 8 and got == want
        c2 = ctx.counters()
        assert c2["big_allocs"] <= 2 and c2["big_bytes"] >= c["big_bytes"], (c, c2)
        got, _, _ = hasher.hash_files_128bit(paths[:3], ctx=ctx)
        assert got == want[:3] and ctx.counters()["big_allocs"] == c2["big_allocs"]


def test_file_paths_above_4_gib(cuda, oracle_lib, tmp_path, monkeypatch):
    """A file above 2^32 bytes through the file entries as they ship: oxh_hash_files (the large-file
    pipeline, five 1 GiB pieces) and oxh_chunk_digests_files (the host chunk pipeline, 1 MiB chunks, the
    piece boundaries and the 2^32 offset inside the file) -- sparse, with written regions at the start,
    around 2^32 and at the end; whole-file digest and every chunk digest against the oracle."""
    import os

    from oxen_amd import dedup, hasher
    from oxen_amd.workloads import splitmix_bytes

    monkeypatch.delenv("OXH_BIG_PIECE_MIB", raising=False)
    monkeypatch.delenv("OXH_CDC_PIECE_MIB", raising=False)
    size = 4 * GIB + 4097
    p = tmp_path / "huge.bin"
    with open(p, "wb") as fh:
        fh.truncate(size)
        for off in (0, 4 * GIB - 2000, 4 * GIB + 77, size - 3000):
            fh.seek(off)
            fh.write(splitmix_bytes(off, 1, 4096).tobytes()[: size - off])
    out, sizes, status = oracle_lib.hash_files([str(p)], threads=8)
    want = (int(out[0, 1]) << 64) | int(out[0, 0])
    assert int(status[0]) == 0 and int(sizes[0]) == size
    d, sz, st = hasher.hash_files_128bit([str(p)])
    assert st == [0] and sz == [size] and d == [want]
    chunk = 1 << 20
    tab = dedup.chunk_digests_files([str(p)], chunk)
    assert list(tab.status) == [0] and int(tab.first[1]) == (size + chunk - 1) // chunk
    data = np.memmap(str(p), dtype=np.uint8, mode="r")
    offs = np.arange(0, size, chunk, dtype=np.uint64)
    lens = np.minimum(np.uint64(chunk), np.uint64(size) - offs)
    assert np.array_equal(tab.file(0), oracle_lib.batch(data, offs, lens, 8))
    del data
    os.remove(p)
