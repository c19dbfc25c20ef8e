"""Parity of the HIP path (through the C ABI) with the golden vectors and the CPU oracle.

Bit-exact digests are the bar for every case: this is integer/byte work.
"""
import ctypes
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _u64(t):
    from oxen_amd.device import to_numpy_u64

    return to_numpy_u64(t).reshape(-1, 2)


def _golden_arena(golden, cuda):
    import torch

    from oxen_amd.device import fill_splitmix

    g = golden("lengths.json")
    vecs = g["vectors"]
    span = max(v["start"] + v["len"] for v in vecs)
    arena = torch.empty((span + 7) // 8 * 8, dtype=torch.uint8, device=cuda)
    fill_splitmix(arena, g["seed"])
    offs = np.array([v["start"] for v in vecs], dtype=np.uint64)
    lens = np.array([v["len"] for v in vecs], dtype=np.uint64)
    want = np.array([[v["lo"], v["hi"]] for v in vecs], dtype=np.uint64)
    return arena, offs, lens, want, vecs


def _mismatch(got, want, lens):
    bad = np.nonzero((got != want).any(axis=1))[0]
    return [int(lens[i]) for i in bad[:20]]


# The K1 variants the shipped library instantiates (xxh3_kernels.hip Cfg): the shapes the dispatch picks
# (8 long items, 72 short, 104 block-wise packed, 264 K1R: a row per item) and the 4-round ring 0, which
# also runs for any other forced variant. The experiments are in the probe build (tools/build_probe_lib.py).
VARIANTS = [0, 8, 72, 104, 264]


@pytest.mark.parametrize("mode", [0, 1, 2, 3])
@pytest.mark.parametrize("variant", VARIANTS)
def test_every_length_unaligned(cuda, golden, mode, variant):
    """Every length 0..2048 + boundaries up to 1 MiB+1, at the golden (mostly unaligned) offsets."""
    import torch

    from oxen_amd import _capi
    from oxen_amd.device import xxh3_128_batch_device

    arena, offs, lens, want, _ = _golden_arena(golden, cuda)
    prev = _capi.lib().oxh_set_kernel_variant(variant)
    try:
        out = xxh3_128_batch_device(arena, torch.from_numpy(offs.view(np.int64)).to(cuda),
                                    torch.from_numpy(lens.view(np.int64)).to(cuda), mode=mode)
        got = _u64(out)
    finally:
        _capi.lib().oxh_set_kernel_variant(prev)
    assert not _mismatch(got, want, lens)


@pytest.mark.parametrize("wg_waves", ["1", "2"])
@pytest.mark.parametrize("variant", VARIANTS)
def test_every_length_workgroup_width(cuda, golden, variant, wg_waves, monkeypatch):
    """K1 launched with 1 or 2 items (waves) per workgroup instead of 4 (OXH_K1_WG_WAVES): the item
    index comes from blockDim, so every item is still hashed exactly once; the ragged golden batch."""
    import torch

    from oxen_amd import _capi
    from oxen_amd.device import xxh3_128_batch_device

    monkeypatch.setenv("OXH_K1_WG_WAVES", wg_waves)
    arena, offs, lens, want, _ = _golden_arena(golden, cuda)
    prev = _capi.lib().oxh_set_kernel_variant(variant)
    try:
        out = xxh3_128_batch_device(arena, torch.from_numpy(offs.view(np.int64)).to(cuda),
                                    torch.from_numpy(lens.view(np.int64)).to(cuda), mode=1)
        got = _u64(out)
    finally:
        _capi.lib().oxh_set_kernel_variant(prev)
    assert not _mismatch(got, want, lens)


@pytest.mark.parametrize("variant", VARIANTS)
def test_every_length_aligned(cuda, golden, variant):
    """Same vectors re-packed at 256-B aligned offsets (the coalesced dwordx4 path)."""
    from oxen_amd import _capi
    from oxen_amd.device import DeviceArena
    from oxen_amd.workloads import splitmix_bytes

    g = golden("lengths.json")
    vecs = g["vectors"]
    lens = np.array([v["len"] for v in vecs], dtype=np.uint64)
    da = DeviceArena.splitmix(lens, seed=0)
    host = np.zeros(da.arena.numel(), dtype=np.uint8)
    for v, o in zip(vecs, da.offsets_host):
        host[int(o):int(o) + v["len"]] = splitmix_bytes(g["seed"], v["start"], v["len"])
    import torch

    da.arena.copy_(torch.from_numpy(host))
    prev = _capi.lib().oxh_set_kernel_variant(variant)
    try:
        got = _u64(da.hash())
    finally:
        _capi.lib().oxh_set_kernel_variant(prev)
    want = np.array([[v["lo"], v["hi"]] for v in vecs], dtype=np.uint64)
    assert not _mismatch(got, want, lens)


def test_fill_splitmix_matches_host(cuda):
    import torch

    from oxen_amd.device import fill_splitmix
    from oxen_amd.workloads import splitmix_bytes

    for n in [8, 13, 4096, 1 << 20, (1 << 20) + 5]:
        t = torch.empty((n + 7) // 8 * 8, dtype=torch.uint8, device=cuda)
        fill_splitmix(t, 1234, n)
        assert np.array_equal(t[:n].cpu().numpy(), splitmix_bytes(1234, 0, n))


def test_random_mixed_batch_vs_oracle(cuda, oracle_lib):
    """A ragged batch (14 B .. 300 KiB, log-uniform) against the oracle."""
    from oxen_amd.device import DeviceArena

    rng = np.random.default_rng(5)
    lens = np.exp(rng.uniform(np.log(1), np.log(300_000), 3000)).astype(np.uint64)
    lens[:5] = [0, 1, 240, 241, 1024]
    da = DeviceArena.splitmix(lens, seed=99)
    got = _u64(da.hash())
    want = oracle_lib.batch(da.arena.cpu().numpy(), da.offsets_host, da.lens_host, threads=8)
    assert not _mismatch(got, want, lens)


def test_c3_shape_49292(cuda, oracle_lib):
    """Config 3 item size (128x128x3 TIFF = 49 292 B; last stripe overlaps, len % 64 != 0)."""
    from oxen_amd.device import DeviceArena

    lens = np.full(20_000, 49_292, dtype=np.uint64)
    da = DeviceArena.splitmix(lens, seed=3)
    got = _u64(da.hash())
    want = oracle_lib.batch(da.arena.cpu().numpy(), da.offsets_host, da.lens_host, threads=8)
    assert not _mismatch(got, want, lens)


def test_c4_shape_262144(cuda, oracle_lib):
    """Config 4 item size (256 KiB), 4 096 items fully checked."""
    from oxen_amd.device import DeviceArena

    lens = np.full(4096, 262_144, dtype=np.uint64)
    da = DeviceArena.splitmix(lens, seed=4)
    got = _u64(da.hash())
    want = oracle_lib.batch(da.arena.cpu().numpy(), da.offsets_host, da.lens_host, threads=8)
    assert not _mismatch(got, want, lens)


def test_c2_full_size_sampled(cuda, oracle_lib):
    """Config 2 at full size: 100 000 x 64 KiB (6.1 GiB) in HBM. Size-independent checks:
    512 sampled items regenerated on the host and hashed by the oracle; a second pass is identical;
    no two digests collide."""
    import torch

    from oxen_amd.device import DeviceArena
    from oxen_amd.workloads import C2_LEN, C2_N, splitmix_bytes

    lens = np.full(C2_N, C2_LEN, dtype=np.uint64)
    da = DeviceArena.splitmix(lens, seed=2024)
    a = _u64(da.hash())
    b = _u64(da.hash())
    assert np.array_equal(a, b)
    assert len({(int(x), int(y)) for x, y in a}) == C2_N
    idx = np.sort(np.random.default_rng(1).choice(C2_N, 512, replace=False))
    idx[0], idx[-1] = 0, C2_N - 1
    for i in idx:
        data = splitmix_bytes(2024, int(da.offsets_host[i]), C2_LEN).tobytes()
        lo, hi = oracle_lib.xxh3_128(data)
        assert (int(a[i, 0]), int(a[i, 1])) == (lo, hi), i
    del da
    torch.cuda.empty_cache()


@pytest.mark.parametrize("variant", [0, 264, 392])
def test_chunk_digests(cuda, oracle_lib, variant):
    """Fixed-size chunk digests (no descriptor table), with the default K1, with K1R forced, and with a
    variant number that no kernel has (392: the default kernel runs, with its own launch geometry)."""
    import torch

    from oxen_amd import _capi
    from oxen_amd.device import chunk_digests_device, fill_splitmix

    n = (5 << 20) + 123
    buf = torch.empty((n + 7) // 8 * 8, dtype=torch.uint8, device=cuda)
    fill_splitmix(buf, 77)
    host = buf[:n].cpu().numpy()
    prev = _capi.lib().oxh_set_kernel_variant(variant)
    try:
        for chunk in [8192, 65536, 1000, 200, 1 << 20]:
            got = _u64(chunk_digests_device(buf, chunk, nbytes=n))
            want = oracle_lib.chunk_digests(host, chunk, threads=8)
            assert np.array_equal(got, want), chunk
    finally:
        _capi.lib().oxh_set_kernel_variant(prev)


@pytest.mark.parametrize("piece_mib", [None, "1", "3"], ids=["one-piece", "1MiB-pieces", "3MiB-pieces"])
@pytest.mark.parametrize("n", [1 << 20, (1 << 20) + 1, (4 << 20) + 7, 64 << 20, (64 << 20) + 4097])
def test_large_single_buffer_k1l(cuda, ctx, oracle_lib, n, piece_mib, monkeypatch):
    """K1L, whole and in pieces (rounds of block sums + resumed chains, OXH_BIG_PIECE_MIB)."""
    import torch

    if piece_mib:
        monkeypatch.setenv("OXH_BIG_PIECE_MIB", piece_mib)

    from oxen_amd.device import fill_splitmix, large_digest_device

    buf = torch.empty((n + 7) // 8 * 8 + 16, dtype=torch.uint8, device=cuda)
    fill_splitmix(buf, n)
    for start in (0, 3):  # aligned and misaligned starts
        view = buf[start:start + n]
        got = _u64(large_digest_device(ctx, view, n))
        torch.cuda.synchronize()
        want = oracle_lib.xxh3_128(view.cpu().numpy().tobytes())
        assert (int(got[0, 0]), int(got[0, 1])) == want, (n, start)


@pytest.mark.parametrize("piece_mib", [None, "1"], ids=["one-piece", "1MiB-pieces"])
def test_large_batch_k1l(cuda, oracle_lib, piece_mib, monkeypatch):
    """Several large buffers in one call (concurrent chains), mixed with small and misaligned ones;
    with 1 MiB pieces the buffers need different numbers of rounds."""
    import torch

    if piece_mib:
        monkeypatch.setenv("OXH_BIG_PIECE_MIB", piece_mib)

    from oxen_amd.device import fill_splitmix, large_digests_device

    sizes = [(3 << 20) + 5, 1000, (1 << 20) + 64, 0, (9 << 20) + 1, 300, (2 << 20) - 1]
    bufs = []
    for i, n in enumerate(sizes):
        b = torch.empty(n + 16, dtype=torch.uint8, device=cuda)
        fill_splitmix(b, 77 + i)
        bufs.append(b[i % 3:i % 3 + n])  # misaligned starts for some
    got = _u64(large_digests_device(bufs, sizes))
    torch.cuda.synchronize()
    for i, (b, n) in enumerate(zip(bufs, sizes)):
        assert (int(got[i, 0]), int(got[i, 1])) == oracle_lib.xxh3_128(b.cpu().numpy().tobytes()), i


def test_combined_hash_device(cuda, golden):
    import torch

    from oxen_amd.device import combined_hash_device

    recs = golden("text_repo.json")["files"]
    content = np.array([[r["lo"], r["hi"]] for r in recs], dtype=np.uint64)
    meta = np.array([[int(r["metadata_hash"], 16) & (2**64 - 1), int(r["metadata_hash"], 16) >> 64] for r in recs],
                    dtype=np.uint64)
    out = combined_hash_device(torch.from_numpy(content.view(np.int64)).to(cuda),
                               torch.from_numpy(meta.view(np.int64)).to(cuda))
    got = [format((int(hi) << 64) | int(lo), "x") for lo, hi in _u64(out)]
    assert got == [r["combined_hash"] for r in recs]


def test_hash_files_data_test_fixtures(ctx, golden, tmp_path):
    """get_hash_given_metadata over the reference's data/test fixture files, plus error isolation."""
    from oxen_amd import hasher

    recs = [r for r in golden("data_test.json")["files"] if r["copied"]]
    paths = [os.path.join(GOLDEN, "data_test", r["path"]) for r in recs]
    paths.insert(3, str(tmp_path / "missing.bin"))
    digests, sizes, status = hasher.hash_files_128bit(paths, ctx)
    assert status[3] != 0 and digests[3] is None
    del digests[3], sizes[3], status[3]
    assert all(s == 0 for s in status)
    assert [format(d, "x") for d in digests] == [r["hex"] for r in recs]
    assert sizes == [r["size"] for r in recs]


def test_hash_files_text_repo_config1(ctx, golden, tmp_path):
    """Config 1: the 1 000-file text repo + README written to disk and hashed as files."""
    from oxen_amd import hasher
    from oxen_amd.workloads import write_text_repo

    paths = write_text_repo(str(tmp_path))
    digests, sizes, status = hasher.hash_files_128bit(paths, ctx)
    want = {r["path"]: r["hex"] for r in golden("text_repo.json")["files"]}
    got = {os.path.relpath(p, str(tmp_path)): format(d, "x") for p, d in zip(paths, digests)}
    assert got == want


def test_hash_files_small_staging_and_oversize(cuda, oracle_lib, tmp_path):
    """Staging of 1 MiB: many batches through the 3-slot pipeline and oversize files (K1L)."""
    from oxen_amd import _capi, hasher
    from oxen_amd.workloads import splitmix_bytes

    rng = np.random.default_rng(11)
    sizes = list(rng.integers(0, 200_000, 300)) + [(1 << 20) + 1, 3 << 20, 0, 5]
    paths = []
    for i, s in enumerate(sizes):
        p = tmp_path / f"f{i}.bin"
        p.write_bytes(splitmix_bytes(i, 0, int(s)).tobytes())
        paths.append(str(p))
    with _capi.Context(0, staging_bytes=1 << 20) as c:
        digests, got_sizes, status = hasher.hash_files_128bit(paths, c)
    assert all(s == 0 for s in status)
    out, _, st = oracle_lib.hash_files(paths, threads=8)
    assert [(int(hi) << 64) | int(lo) for lo, hi in out] == digests
    assert got_sizes == [int(s) for s in sizes]


def test_hash_buffers_and_streams(ctx, oracle_lib, golden):
    from oxen_amd import hasher

    rng = np.random.default_rng(3)
    bufs = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in rng.integers(0, 5000, 500)]
    assert hasher.hash_buffers_128bit(bufs, ctx) == [oracle_lib.xxh3_128_int(b) for b in bufs]
    streams = golden("streams.json")["streams"]
    got = hasher.hash_streams_128bit([bytes.fromhex(s["bytes_hex"]) for s in streams], ctx)
    assert [format(d, "x") for d in got] == [s["hex"] for s in streams]


def test_hasher_mirror_api(ctx, golden, tmp_path, oracle_lib):
    """liboxen util::hasher names and semantics (hasher.rs:11-244) on the GPU path."""
    import io

    from oxen_amd import hasher
    from oxen_amd._capi import OxenError

    assert hasher.hash_str("filestrlabelstrmin_xf64min_yf64widthi64heighti64") == "b821946753334c083124fd563377d795"
    assert hasher.hash_buffer(b"") == "99aa06d3014798d86001c324468d497f"
    assert hasher.hash_buffer(b"x" * 65536) == "2da4b9c5a75caad3688558138047f8a"
    r0 = golden("text_repo.json")["files"][0]
    md = {"text": {"num_lines": 1, "num_chars": 14}}
    assert format(hasher.get_metadata_hash(md), "x") == r0["metadata_hash"]
    assert hasher.maybe_get_metadata_hash(None) is None
    c = int(r0["hex"], 16)
    assert format(hasher.get_combined_hash(hasher.get_metadata_hash(md), c), "x") == r0["combined_hash"]
    assert hasher.get_combined_hash(None, c) == c
    # a non-text GenericMetadata (MetadataAudio, an f64 field) through the GPU path, against the oracle
    # over serde_json's text (tests/test_host.py pins the text)
    O = oracle_lib
    audio = {"audio": {"num_seconds": 1e-5, "num_channels": 2, "sample_rate": 44100}}
    js = b'{"audio":{"num_seconds":0.00001,"num_channels":2,"sample_rate":44100}}'
    assert hasher.get_metadata_hash(audio) == O.xxh3_128_int(js)
    assert hasher.get_combined_hash(hasher.get_metadata_hash(audio), c) == O.combined_hash(c, O.xxh3_128_int(js))
    p = tmp_path / "a.txt"
    p.write_bytes(b"File content 0")
    assert hasher.hash_file_contents(str(p)) == r0["hex"]
    assert hasher.u128_hash_file_contents(str(p)) == c
    assert hasher.get_hash_given_metadata(str(p), os.stat(p)) == c
    with pytest.raises(OxenError):
        hasher.hash_file_contents(str(tmp_path / "missing"))
    rd = hasher.HashingReader(io.BytesIO(b"File content 0"))
    while rd.read(3):
        pass
    assert rd.digest128() == c
    sink = io.BytesIO()
    w = hasher.HashingWriter(sink)
    w.write(b"File ")
    w.write(b"content 0")
    assert w.digest128() == c and sink.getvalue() == b"File content 0"


def test_merkle_parents_k2(ctx):
    from oracle import oracle
    from oxen_amd import merkle

    paths = [f"texts/file_{i}.txt" for i in range(1000)]
    nv = merkle.num_vnodes(len(paths), 100)
    assert nv == 10
    got = merkle.vnode_buckets(paths, nv)
    assert got == [oracle.xxh3_128_int(p.encode()) % nv for p in paths]
    streams = [merkle.vnode_stream("texts", range(i)) for i in range(0, 300, 7)]
    assert [h.value for h in merkle.hash_parents(streams)] == [oracle.xxh3_128_int(s) for s in streams]


def test_empty_batch(cuda):
    import torch

    from oxen_amd.device import xxh3_128_batch_device

    z = torch.zeros(0, dtype=torch.int64, device=cuda)
    out = xxh3_128_batch_device(torch.zeros(8, dtype=torch.uint8, device=cuda), z, z)
    assert out.shape == (0, 2)


def _text_counts(b: bytes):
    return 1 + b.count(b"\n"), sum(1 for x in b if (x & 0xC0) != 0x80)


@pytest.mark.parametrize("variant", [0, 8])
def test_text_counts_fused_every_length(cuda, oracle_lib, variant):
    """K1T: digests identical to K1 and text counts exact for every length class, aligned and not.
    Only K1T<72> ships; a forced K1 variant (8) must not change which K1T runs."""
    import torch

    from oxen_amd import _capi
    from oxen_amd.device import xxh3_128_text_batch_device

    _capi.lib().oxh_set_kernel_variant(variant)
    try:
        _check_text_counts(cuda, oracle_lib, torch, xxh3_128_text_batch_device)
    finally:
        _capi.lib().oxh_set_kernel_variant(0)


def _check_text_counts(cuda, oracle_lib, torch, xxh3_128_text_batch_device):
    rng = np.random.default_rng(9)
    alphabet = np.frombuffer("ab\nc é漢\n🐂 z\n".encode(), dtype=np.uint8)
    lens = list(range(0, 300)) + [1023, 1024, 1025, 4095, 4096, 4097, 8191, 8192, 49_292, 65_536, 100_003]
    span = sum(lens) + 64 * len(lens)
    host = alphabet[rng.integers(0, len(alphabet), span)]
    offs = np.cumsum([0] + [L + int(rng.integers(0, 17)) for L in lens[:-1]]).astype(np.uint64)
    arena = torch.from_numpy(host).to(cuda)
    out, counts = xxh3_128_text_batch_device(arena, torch.from_numpy(offs.view(np.int64)).to(cuda),
                                             torch.from_numpy(np.array(lens, dtype=np.uint64).view(np.int64)).to(cuda))
    got = _u64(out)
    cnt = counts.cpu().numpy()
    for i, L in enumerate(lens):
        b = host[int(offs[i]):int(offs[i]) + L].tobytes()
        assert (int(got[i, 0]), int(got[i, 1])) == oracle_lib.xxh3_128(b), L
        assert tuple(int(x) for x in cnt[i]) == _text_counts(b), L


def test_text_file_nodes_config1(ctx, golden, tmp_path):
    """Config 1 end to end: content hash, text metadata, metadata hash and combined hash of every
    file of the 1 000-file text repo (add.rs:833-842) match the goldens."""
    from oxen_amd import hasher
    from oxen_amd.workloads import write_text_repo

    paths = write_text_repo(str(tmp_path))
    nodes = hasher.text_file_nodes(paths, ctx)
    want = {r["path"]: r for r in golden("text_repo.json")["files"]}
    for p, nd in zip(paths, nodes):
        r = want[os.path.relpath(p, str(tmp_path))]
        assert format(nd["hash"], "x") == r["hex"]
        assert hasher.metadata_json(nd["metadata"]) == r["metadata_json"]
        assert format(nd["metadata_hash"], "x") == r["metadata_hash"]
        assert format(nd["combined_hash"], "x") == r["combined_hash"]


def test_text_files_oversize_and_errors(cuda, tmp_path):
    from oxen_amd import _capi, hasher

    rng = np.random.default_rng(4)
    texts = [("x\n" * 700_000 + "é").encode(), b"", b"\n", "🐂".encode() * 1000]
    paths = []
    for i, t in enumerate(texts):
        p = tmp_path / f"t{i}.txt"
        p.write_bytes(t)
        paths.append(str(p))
    paths.append(str(tmp_path / "missing.txt"))
    with _capi.Context(0, staging_bytes=1 << 20) as c:  # the 1.4 MB file is oversize
        d, sizes, st, meta = hasher.hash_files_text_128bit(paths, c)
    assert st[-1] != 0 and meta[-1] is None
    for t, m in zip(texts, meta):
        assert (m["text"]["num_lines"], m["text"]["num_chars"]) == _text_counts(t)


def test_add_files_fused_version_store(ctx, oracle_lib, golden, tmp_path):
    """oxh_add_files: one read, K1 hash, blob published from the same pinned bytes; the store it
    builds is identical to the reference loop's (oracle restatement of add + store_version_from_reader)."""
    from oxen_amd import hasher

    recs = [r for r in golden("data_test.json")["files"] if r["copied"]]
    paths = [os.path.join(GOLDEN, "data_test", r["path"]) for r in recs]
    paths.append(paths[0])  # the same content twice: second add finds the blob
    paths.append(str(tmp_path / "missing.bin"))
    root = str(tmp_path / ".oxen" / "versions" / "files")  # parents created on first publish
    d, sizes, st, stored = hasher.add_files(paths, root, ctx)
    assert st[-1] != 0 and stored[-1] is False
    for p, r, dg in zip(paths, recs, d):
        assert format(dg, "x") == r["hex"]
        blob = hasher.version_path(root, dg)
        assert open(blob, "rb").read() == open(p, "rb").read()
    # identical content is stored once
    n_unique = len({r["hex"] for r in recs})
    assert sum(stored) == n_unique
    # a second add stores nothing new
    d2, _, st2, stored2 = hasher.add_files(paths[:-1], root, ctx)
    assert not any(stored2) and d2 == d[:-1]
    # the reference loop builds the same store
    ref_root = str(tmp_path / "ref" / "versions" / "files")
    out, _, rst, rstored = oracle_lib.add_files(paths[:-1], ref_root, threads=4)
    assert (rst == 0).all()
    walk = lambda r: sorted(os.path.relpath(os.path.join(dp, f), r) for dp, _, fs in os.walk(r) for f in fs)
    assert walk(root) == walk(ref_root)


def test_clean_corrupted_versions(ctx, oracle_lib, tmp_path):
    """`oxen fsck` as one batched GPU re-hash: same counts and the same surviving store as the oracle."""
    from _store import make_version_store

    from oxen_amd import hasher

    hexer = lambda b: oracle_lib.format_hex(*oracle_lib.xxh3_128(b))
    gpu_root, ref_root = str(tmp_path / "gpu"), str(tmp_path / "ref")
    dry, real, again = make_version_store(gpu_root, hexer)
    make_version_store(ref_root, hexer)
    strip = lambda r: {k: r[k] for k in ("scanned", "corrupted", "cleaned", "errors")}
    assert strip(hasher.clean_corrupted_versions(gpu_root, dry_run=True, ctx=ctx)) == dry
    assert strip(hasher.clean_corrupted_versions(gpu_root, dry_run=False, ctx=ctx)) == real
    assert oracle_lib.clean_corrupted_versions(ref_root, dry_run=False, threads=4) == real
    walk = lambda r: sorted(os.path.relpath(os.path.join(dp, f), r) for dp, _, fs in os.walk(r) for f in fs)
    assert walk(gpu_root) == walk(ref_root)
    assert strip(hasher.clean_corrupted_versions(gpu_root, dry_run=False, ctx=ctx)) == again


@pytest.mark.parametrize("second", [False, True])
@pytest.mark.parametrize("vnode_size", [10_000, 7])
def test_commit_driver(ctx, second, vnode_size):
    """K2 end to end: every vnode id and dir hash of a commit from three batched GPU passes equals the
    scalar restatement of commit_writer.rs (oracle/commit_oracle.py)."""
    import _commit

    from oracle import commit_oracle
    from oxen_amd import merkle

    entries, existing = _commit.staged_commit(n_files=500, n_dirs=9, second=second)
    vn, dh = merkle.commit_tree(_commit.to_staged(entries), _commit.to_staged(existing), vnode_size, _commit.salt,
                                ctx=ctx)
    rvn, rdh = commit_oracle.commit_tree(entries, existing, vnode_size, _commit.salt)
    for d in rvn:
        assert [v.id.value for v in vn[d][0]] == [i for i, _ in rvn[d]], d
    assert {d: h.value for d, h in dh.items()} == rdh


def test_commit_driver_image_repo_shape(ctx):
    """C3's tree (200 000 files in 1 000 dirs): root and images/ dir streams are ~10 MB each and go
    through the wave kernel; the split dirs' vnode streams through the lane kernel."""
    import _commit

    from oracle import commit_oracle
    from oxen_amd import merkle

    entries, _ = _commit.staged_commit(n_files=200_000, n_dirs=1000)
    vn, dh = merkle.commit_tree(_commit.to_staged(entries), None, 10_000, _commit.salt, ctx=ctx)
    rvn, rdh = commit_oracle.commit_tree(entries, {}, 10_000, _commit.salt)
    assert {d: [v.id.value for v in vn[d][0]] for d in vn} == {d: [i for i, _ in rvn[d]] for d in rvn}
    assert {d: h.value for d, h in dh.items()} == rdh


def _utf8_cases():
    import random

    rng = random.Random(9)
    pieces = [b"a", b"\xc3\xa9", b"\xe2\x82\xac", b"\xf0\x9f\x98\x80", b"\xed\x9f\xbf", b"\xf4\x8f\xbf\xbf", b"\xc0",
              b"\xc1\x80", b"\xe0\x80\x80", b"\xed\xa0\x80", b"\xf4\x90\x80\x80", b"\xf5", b"\xff", b"\x80", b"\x0a"]
    cases = [b"", b"hello", b"\xe2\x82", b"\xe2\x28", b"a" * 4096 + b"\xff", b"a" * 4095 + b"\xe2\x82\xac",
             b"a" * 4094 + b"\xe2\x82\xac", b"a" * 4093 + b"\xf0\x9f\x98\x80", b"a" * 4095 + b"\xe0\x80",
             "héllo wörld €".encode() * 500]
    for _ in range(600):
        s = b"".join(rng.choice(pieces) for _ in range(rng.randint(0, 60)))
        if rng.random() < 0.3:
            s = s[: rng.randint(0, len(s))]
        if rng.random() < 0.3:
            s = b"t" * rng.randint(4000, 4100) + s
        cases.append(s)
    return cases


def test_utf8_sniff_device(cuda, oracle_lib):
    """util::fs::is_utf8 (util/fs.rs:652-668) on the device, vs the oracle, at misaligned offsets."""
    import torch

    from oxen_amd import _capi

    cases = _utf8_cases()
    offs, pos = [], 0
    for c in cases:
        offs.append(pos)
        pos += len(c) + 5
    arena = np.zeros(max(pos, 1), dtype=np.uint8)
    for o, c in zip(offs, cases):
        arena[o:o + len(c)] = np.frombuffer(c, dtype=np.uint8)
    d_arena = torch.from_numpy(arena).to(cuda)
    d_offs = torch.tensor(offs, dtype=torch.int64, device=cuda)
    d_lens = torch.tensor([len(c) for c in cases], dtype=torch.int64, device=cuda)
    flags = torch.empty(len(cases), dtype=torch.int32, device=cuda)
    _capi.check(_capi.lib().oxh_utf8_prefix_device(d_arena.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), len(cases),
                                                   flags.data_ptr(), 0), "oxh_utf8_prefix_device")
    torch.cuda.synchronize()
    got = flags.cpu().numpy().tolist()
    want = [int(oracle_lib.is_utf8_prefix(c)) for c in cases]
    assert got == want


def test_hash_files_text_utf8(ctx, oracle_lib, tmp_path):
    """One read per file: digest, text counts and is_utf8, including oversize files (> staging) and
    unreadable paths."""
    from oxen_amd import _capi, hasher

    cases = _utf8_cases()[:200] + [b"\xff" + b"a" * (3 << 20), "ü".encode() * (2 << 20)]
    paths = []
    for i, c in enumerate(cases):
        p = tmp_path / f"f{i}.txt"
        p.write_bytes(c)
        paths.append(str(p))
    paths.append(str(tmp_path / "missing.txt"))
    with _capi.Context(0, staging_bytes=1 << 20) as c:
        d, sizes, st, meta, utf8 = hasher.hash_files_text_utf8_128bit(paths, c)
    assert st[-1] != 0 and utf8[-1] is False and d[-1] is None
    out, _, _ = oracle_lib.hash_files(paths[:-1], threads=8)
    assert [(int(hi) << 64) | int(lo) for lo, hi in out] == d[:-1]
    assert utf8[:-1] == [oracle_lib.is_utf8_prefix(c) for c in cases]
    for c, m in zip(cases, meta):
        assert m["text"]["num_lines"] == 1 + c.count(b"\n")
        assert m["text"]["num_chars"] == len(c) - sum(1 for x in c if (x & 0xC0) == 0x80)


def test_concurrent_callers_coalesce(oracle_lib, tmp_path, cuda):
    """liboxen calls the hasher from many tokio tasks at once, 64 files per batch (add.rs:41,
    422-425): concurrent oxh_hash_files / oxh_add_files / oxh_hash_files_text_utf8 calls on one
    context coalesce into shared pipeline runs, and every caller gets exactly its own results."""
    import threading

    from oxen_amd import _capi, hasher
    from oxen_amd.workloads import splitmix_bytes

    rng = np.random.default_rng(21)
    paths = []
    for i in range(16 * 64):
        p = tmp_path / f"f{i}.bin"
        p.write_bytes(splitmix_bytes(500 + i, 0, int(rng.integers(0, 70_000))).tobytes())
        paths.append(str(p))
    want_out, _, _ = oracle_lib.hash_files(paths, threads=8)
    want = [(int(hi) << 64) | int(lo) for lo, hi in want_out]
    results, errors = {}, []
    with _capi.Context(0, staging_bytes=4 << 20) as c:
        def worker(t):
            try:
                batch = paths[t * 64:(t + 1) * 64] + ([str(tmp_path / "missing")] if t % 3 == 0 else [])
                if t % 4 == 1:
                    d, _, st, _ = hasher.add_files(batch, str(tmp_path / "store" / f"t{t}"), c)
                elif t % 4 == 2:
                    d, _, st, _, _ = hasher.hash_files_text_utf8_128bit(batch, c)
                else:
                    d, _, st = hasher.hash_files_128bit(batch, c)
                results[t] = (d, st)
            except Exception as e:  # pragma: no cover - reported below
                errors.append(repr(e))

        for _round in range(3):
            th = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
            for x in th:
                x.start()
            for x in th:
                x.join()
            assert not errors, errors
            for t in range(16):
                d, st = results[t]
                assert d[:64] == want[t * 64:(t + 1) * 64], t
                if t % 3 == 0:
                    assert st[64] != 0 and d[64] in (None, 0)


@pytest.mark.gpu
def test_concurrent_mixed_requests_join_live_run(oracle_lib, tmp_path, cuda):
    """Requests of every kind join one live engine run: text/UTF-8 requests arriving while plain hash
    requests stream (the slots switch to K1T + is_utf8 mid-run), files larger than the staging slot
    (oversize path inside the live run), missing files, and empty requests -- each caller gets
    exactly the reference's digests, text counts and is_utf8 for its own files."""
    import threading

    from oracle import oracle
    from oxen_amd import _capi, hasher
    from oxen_amd.workloads import splitmix_bytes

    rng = np.random.default_rng(33)
    paths, blobs = [], []
    for i in range(12 * 48):
        kind = i % 3
        if kind == 0:
            b = splitmix_bytes(900 + i, 0, int(rng.integers(0, 40_000))).tobytes()
        elif kind == 1:
            b = ("line %d é ü\n" % i * int(rng.integers(1, 3000))).encode()
        else:
            # a 2-byte sequence cut off by the end (still UTF-8 for is_utf8), or broken mid-file
            b = ("x" * int(rng.integers(0, 5000))).encode() + (b"\xc3x" if i % 2 else b"\xc3")
        if i == 60:
            b = splitmix_bytes(77, 0, (3 << 20) + 12345).tobytes()  # > the 2 MiB staging slot
        p = tmp_path / f"m{i}.dat"
        p.write_bytes(b)
        paths.append(str(p))
        blobs.append(b)
    want = [oracle.xxh3_128_int(b) for b in blobs]
    want_counts = [(1 + b.count(b"\n"), len(b) - sum(1 for x in b if (x & 0xC0) == 0x80)) for b in blobs]
    want_utf8 = [oracle.is_utf8_prefix(b[:4096]) for b in blobs]
    results, errors = {}, []
    with _capi.Context(0, staging_bytes=2 << 20) as c:
        def worker(t):
            try:
                batch = paths[t * 48:(t + 1) * 48]
                if t % 5 == 4:
                    batch = batch + [str(tmp_path / "nope")]
                if t == 7:
                    results[("empty", t)] = hasher.hash_files_128bit([], c)
                if t % 2 == 1:
                    d, sz, st, meta, u8 = hasher.hash_files_text_utf8_128bit(batch, c)
                    results[t] = (d, st, meta, u8)
                else:
                    d, sz, st = hasher.hash_files_128bit(batch, c)
                    results[t] = (d, st, None, None)
            except Exception as e:  # pragma: no cover - reported below
                errors.append(repr(e))

        for _round in range(2):
            results.clear()
            th = [threading.Thread(target=worker, args=(t,)) for t in range(12)]
            for x in th:
                x.start()
            for x in th:
                x.join()
            assert not errors, errors
            for t in range(12):
                d, st, meta, u8 = results[t]
                lo = t * 48
                assert d[:48] == want[lo:lo + 48], t
                assert all(s == 0 for s in st[:48]), t
                if meta is not None:
                    got = [(m["text"]["num_lines"], m["text"]["num_chars"]) for m in meta[:48]]
                    assert got == want_counts[lo:lo + 48], t
                    assert u8[:48] == want_utf8[lo:lo + 48], t
                if t % 5 == 4:
                    assert st[48] != 0 and d[48] is None


@pytest.mark.parametrize("piece_mib", [None, "32"], ids=["one-piece", "32MiB-pieces"])
def test_big_file_streamed_pieces(oracle_lib, tmp_path, cuda, monkeypatch, piece_mib):
    """Files above a staging slot stream through the large-file path in 64 MiB pieces (parallel
    preads into two pinned bounce buffers, H2D, K1L on the device): several pieces, a ragged last
    piece, an exact multiple, digests + text counts + is_utf8 against the oracle / numpy, and the
    sink (fused add) variant that keeps the whole file on the host."""
    from oracle import oracle
    from oxen_amd import _capi, hasher
    from oxen_amd.workloads import splitmix_bytes

    if piece_mib:  # device pieces of 32 MiB: resumed chains, a last piece of 32 MiB + 10 B
        monkeypatch.setenv("OXH_BIG_PIECE_MIB", piece_mib)
    sizes = [(150 << 20) + 17, 64 << 20, (5 << 20) + 3, (64 << 20) + 10]
    blobs = [splitmix_bytes(300 + k, 0, s).tobytes() for k, s in enumerate(sizes)]
    paths = []
    for k, b in enumerate(blobs):
        p = tmp_path / f"big{k}.bin"
        p.write_bytes(b)
        paths.append(str(p))
    want = [oracle.xxh3_128_int(b) for b in blobs]
    arrs = [np.frombuffer(b, dtype=np.uint8) for b in blobs]
    want_counts = [(1 + int(np.count_nonzero(a == 10)), len(a) - int(np.count_nonzero((a & 0xC0) == 0x80))) for a in arrs]
    want_utf8 = [oracle.is_utf8_prefix(b[:4096]) for b in blobs]
    with _capi.Context(0, staging_bytes=4 << 20) as c:
        d, sz, st = hasher.hash_files_128bit(paths, c)
        assert st == [0] * len(sizes) and sz == sizes and d == want
        d, sz, st, meta, u8 = hasher.hash_files_text_utf8_128bit(paths, c)
        assert d == want and u8 == want_utf8
        assert [(m["text"]["num_lines"], m["text"]["num_chars"]) for m in meta] == want_counts
        d, sz, st, stored = hasher.add_files(paths, str(tmp_path / "store"), c)
        assert d == want and all(s == 0 for s in st) and all(stored)


@pytest.mark.parametrize("at_once", ["1", "3", "32"])
def test_big_files_side_by_side(oracle_lib, tmp_path, cuda, monkeypatch, at_once):
    """Several files above a staging slot share one piece pipeline (OXH_BIG_FILES at a time): piece r of
    every file goes to the device, then one chain launch continues every file's chain. Files of
    different piece counts (1 .. 5 pieces, last pieces of 1 025 B .. P + 1 024 B), mixed with small
    files, in one call and through the fused add; digests, text counts and is_utf8 vs the oracle."""
    from oxen_amd import _capi, hasher
    from oxen_amd.workloads import splitmix_bytes

    monkeypatch.setenv("OXH_BIG_PIECE_MIB", "8")
    monkeypatch.setenv("OXH_BIG_FILES", at_once)
    P = 8 << 20
    big = [5 << 20, 2 * P + 1025, P + 1024, P + 1025, 4 * P + 12_345, 3 * P, (5 << 20) + 1, 2 * P - 7]
    rng = np.random.default_rng(int(at_once))
    sizes = []
    for b in big:
        sizes += [int(x) for x in rng.integers(0, 100_000, 7)] + [b]
    blobs = [splitmix_bytes(700 + k, 0, s).tobytes() for k, s in enumerate(sizes)]
    blobs[1] = ("héllo\nwörld\n" * 1000).encode()  # a text-ish one
    paths = []
    for k, b in enumerate(blobs):
        p = tmp_path / f"f{k}.bin"
        p.write_bytes(b)
        paths.append(str(p))
    want = [oracle_lib.xxh3_128_int(b) for b in blobs]
    arrs = [np.frombuffer(b, dtype=np.uint8) for b in blobs]
    want_counts = [(1 + int(np.count_nonzero(a == 10)), len(a) - int(np.count_nonzero((a & 0xC0) == 0x80))) for a in arrs]
    want_utf8 = [oracle_lib.is_utf8_prefix(b[:4096]) for b in blobs]
    with _capi.Context(0, staging_bytes=4 << 20) as c:
        d, sz, st = hasher.hash_files_128bit(paths, c)
        assert st == [0] * len(paths) and sz == [len(b) for b in blobs] and d == want
        d, sz, st, meta, u8 = hasher.hash_files_text_utf8_128bit(paths, c)
        assert d == want and u8 == want_utf8
        assert [(m["text"]["num_lines"], m["text"]["num_chars"]) for m in meta] == want_counts
        root = str(tmp_path / "store")
        d, sz, st, stored = hasher.add_files(paths, root, c)
        assert d == want and all(s == 0 for s in st) and all(stored)
        for k in range(7, len(paths), 8):  # every big blob published with the file's bytes
            assert open(hasher.version_path(root, want[k]), "rb").read() == blobs[k]


def test_hash_files_given_metadata(oracle_lib, tmp_path, cuda):
    """oxh_hash_files_meta (get_hash_given_metadata with the walk's sizes, hasher.rs:56-65): no
    fstat per file; sizes that are stale (file grew, shrank, emptied; a walk size above a staging
    slot for a file now below one, and a wrong size above a slot for a file still above one), a
    directory, a missing path and an oversize file are all handled so that every digest covers the
    file's current content."""
    from oxen_amd import _capi, hasher
    from oxen_amd.workloads import splitmix_bytes

    rng = np.random.default_rng(41)
    blobs = [splitmix_bytes(900 + k, 0, int(s)).tobytes() for k, s in enumerate(rng.integers(0, 300_000, 400))]
    blobs += [splitmix_bytes(6, 0, 1000).tobytes(), splitmix_bytes(7, 0, (3 << 19) + 3).tobytes()]
    blobs += [b"", b"x", splitmix_bytes(5, 0, (3 << 20) + 9).tobytes()]  # the last one is oversize
    paths = []
    for k, b in enumerate(blobs):
        p = tmp_path / f"m{k}.bin"
        p.write_bytes(b)
        paths.append(str(p))
    meta = [len(b) for b in blobs]
    meta[3] += 1          # file shrank since the walk
    meta[4] = max(0, meta[4] - 7)  # file grew
    meta[5] = 0           # grew from empty
    meta[-3] = 10         # now empty
    meta[-5] = 2 << 20    # the walk saw a file larger than a staging slot; it is 1000 B now
    meta[-4] = 3 << 20    # larger than a slot either way, but not the size the walk saw
    os.mkdir(tmp_path / "adir")
    paths += [str(tmp_path / "adir"), str(tmp_path / "missing")]
    meta += [4096, 5]
    want_out, want_sizes, want_st = oracle_lib.hash_files(paths, threads=8)
    with _capi.Context(0, staging_bytes=1 << 20) as c:
        d, sz, st = hasher.hash_files_given_metadata_128bit(paths, meta, c)
    assert st[:-2] == [0] * len(blobs) and st[-2] != 0 and st[-1] != 0
    assert sz[:-2] == [len(b) for b in blobs]
    assert d[:-2] == [(int(hi) << 64) | int(lo) for lo, hi in want_out[:-2]]
    assert d[-2] is None and d[-1] is None


def test_files_modified_status_check(oracle_lib, tmp_path, cuda):
    """oxh_files_modified = classify_modified_from_node_with_metadata (util/fs.rs:1580-1619) per
    tracked file, against that function restated here over oracle digests: size differs -> modified
    (not read); mtime matched -> clean (not read); else content hash vs node hash. Covers edited files
    of the same size, untouched files with a drifted mtime, empty files, a file larger than a staging
    slot, a file removed after the walk and a directory (read errors: status != 0)."""
    from oxen_amd import _capi, hasher
    from oxen_amd.workloads import splitmix_bytes

    rng = np.random.default_rng(7)
    blobs = [splitmix_bytes(300 + k, 0, int(s)).tobytes() for k, s in enumerate(rng.integers(0, 200_000, 300))]
    blobs += [b"", splitmix_bytes(9, 0, (3 << 20) + 5).tobytes()]  # empty; larger than the 1 MiB staging slot
    paths = []
    for k, b in enumerate(blobs):
        p = tmp_path / f"f{k}.bin"
        p.write_bytes(b)
        paths.append(str(p))
    node_hashes = [oracle_lib.xxh3_128_int(b) for b in blobs]  # the committed FileNode hashes
    node_bytes = [len(b) for b in blobs]
    mtime_matched = [bool(x) for x in rng.integers(0, 2, len(blobs))]
    mtime_matched[-1] = mtime_matched[-2] = False
    # edit the working tree: same-size rewrites, grown files, shrunk files
    for k in range(0, len(blobs), 3):
        b = bytearray(blobs[k])
        if b:
            b[int(rng.integers(0, len(b)))] ^= 0x5A
        open(paths[k], "wb").write(bytes(b))
    for k in range(1, len(blobs) - 2, 17):
        open(paths[k], "ab").write(b"+")
    mtime_matched[-1] = False
    big = bytearray(blobs[-1])
    big[-1] ^= 1
    open(paths[-1], "wb").write(bytes(big))
    sizes = [os.stat(p).st_size for p in paths]
    # a file removed after the walk and a directory, both with a size equal to the node's
    os.mkdir(tmp_path / "adir")
    paths += [str(tmp_path / "gone.bin"), str(tmp_path / "adir")]
    sizes += [11, 4096]
    node_bytes += [11, 4096]
    node_hashes += [1, 2]
    mtime_matched += [False, False]

    def want_of(i):
        if sizes[i] != node_bytes[i]:
            return True, 0, False
        if mtime_matched[i]:
            return False, 0, False
        try:
            data = open(paths[i], "rb").read()
        except OSError:
            return False, 1, True
        return oracle_lib.xxh3_128_int(data) != node_hashes[i], 0, True

    want = [want_of(i) for i in range(len(paths))]
    with _capi.Context(0, staging_bytes=1 << 20) as c:
        modified, status, n_hashed = hasher.files_modified(paths, sizes, node_bytes, mtime_matched, node_hashes, c)
        assert hasher.files_modified([], [], [], [], [], c) == ([], [], 0)
    assert modified == [w[0] for w in want]
    assert [s != 0 for s in status] == [w[1] != 0 for w in want]
    assert n_hashed == sum(w[2] for w in want)
    assert any(m for m, w in zip(modified, want) if w[2]) and any(not m for m, w in zip(modified, want) if w[2])
    assert modified[-3] is True  # the oversize file with one changed byte


def _text_meta_hash(oracle_lib, data: bytes) -> int:
    """maybe_get_metadata_hash(MetadataText) restated: count_lines (util/fs.rs:217-263, with_chars,
    no trailing-line removal) -> serde_json -> XXH3-128 (hasher.rs:95-100), on the oracle."""
    lines = 1 + data.count(b"\n")
    chars = sum(1 for b in data if (b & 0xC0) != 0x80)
    return oracle_lib.xxh3_128_int(('{"text":{"num_lines":%d,"num_chars":%d}}' % (lines, chars)).encode())


def test_files_modified_metadata_hash_step(oracle_lib, tmp_path, cuda):
    """The metadata-hash step of classify_modified_from_node_with_metadata (util/fs.rs:1599-1614):
    with the size equal and the mtime drifted, node.metadata_hash() and the working file's
    maybe_get_metadata_hash are compared BEFORE the content hash -- both Some and different gives
    modified even when the content is unchanged; an extraction error is returned. Every combination
    of node side (None / the right hash / a stale hash) and file side (None, caller-given equal or
    different, Text counted on the read, extraction error) against fs.rs restated over the oracle."""
    from oxen_amd import _capi, hasher

    rng = np.random.default_rng(23)
    texts = [b"", b"one line", b"a\nb\nc\n", "naïve café ✓\n".encode() * 40, b"x" * 70_000 + b"\n"]
    blobs = texts + [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in (1, 777, 65_536)]
    paths = []
    for k, b in enumerate(blobs):
        p = tmp_path / f"m{k}.dat"
        p.write_bytes(b)
        paths.append(str(p))
    rows = []  # (path index, node meta, file meta, content edited)
    for k, b in enumerate(blobs):
        right = _text_meta_hash(oracle_lib, b)
        for node_meta in (None, right, right ^ (1 << 100)):
            for file_meta in (None, right, right ^ 5, hasher.TEXT, RuntimeError("bad metadata")):
                rows.append((k, node_meta, file_meta))
    # same-size content edits of two files (the node hashes stay the committed ones)
    committed = [oracle_lib.xxh3_128_int(b) for b in blobs]
    for k in (3, 6):
        b = bytearray(blobs[k])
        b[len(b) // 2] ^= 0x01
        open(paths[k], "wb").write(bytes(b))
    now = [open(p, "rb").read() for p in paths]

    def want_of(k, node_meta, file_meta):
        if isinstance(file_meta, Exception):
            return False, _capi.OXH_ERR_META
        if file_meta is hasher.TEXT:
            file_meta = _text_meta_hash(oracle_lib, now[k])
        if node_meta is not None and file_meta is not None and node_meta != file_meta:
            return True, 0
        return oracle_lib.xxh3_128_int(now[k]) != committed[k], 0

    idx = [r[0] for r in rows]
    want = [want_of(*r) for r in rows]
    with _capi.Context(0, staging_bytes=1 << 20) as c:
        modified, status, n_hashed = hasher.files_modified(
            [paths[k] for k in idx], [len(now[k]) for k in idx], [len(blobs[k]) for k in idx], [False] * len(rows),
            [committed[k] for k in idx], c, node_metadata_hashes=[r[1] for r in rows], file_metadata=[r[2] for r in rows])
        assert modified == [w[0] for w in want]
        assert status == [w[1] for w in want]
        # read: everything but extraction errors and caller-given metadata that already differs
        assert n_hashed == sum(1 for r in rows if not isinstance(r[2], Exception)
                               and not (isinstance(r[2], int) and r[1] is not None and r[1] != r[2]))
        # unchanged content, stale node metadata hash -> modified (the case the content check alone misses)
        k = 0
        st = os.stat(paths[k])
        assert hasher.classify_modified_from_node_with_metadata(paths[k], len(blobs[k]), committed[k], st, False,
                                                                node_metadata_hash=123, file_metadata=hasher.TEXT)
        assert not hasher.classify_modified_from_node_with_metadata(paths[k], len(blobs[k]), committed[k], st, False,
                                                                    node_metadata_hash=None, file_metadata=hasher.TEXT)
        with pytest.raises(_capi.OxenError) as e:
            hasher.classify_modified_from_node_with_metadata(paths[k], len(blobs[k]), committed[k], st, False,
                                                             file_metadata=ValueError("no extractor"))
        assert e.value.code == _capi.OXH_ERR_META and "no extractor" in str(e.value)
        # a GenericMetadata object on the file side is hashed as serde_json, like get_metadata_hash
        meta = {"text": {"num_lines": 1, "num_chars": 0}}
        assert not hasher.classify_modified_from_node_with_metadata(paths[0], 0, committed[0], os.stat(paths[0]), False,
                                                                    node_metadata_hash=_text_meta_hash(oracle_lib, b""),
                                                                    file_metadata=meta)


@pytest.mark.parametrize("variant", [0, 264, 1])
def test_k1r_lockstep_rows(cuda, oracle_lib, variant):
    """K1R runs a wave's four items in lockstep to the longest: MiB items next to tiny ones, short-path
    items (<= 240 B) in the same wave, every byte shift, a batch size that leaves the last wave with 1-3
    rows, and items in reverse order and overlapping (the descriptor spans [lowest start, highest end))."""
    import torch

    from oxen_amd import _capi
    from oxen_amd.device import fill_splitmix, xxh3_128_batch_device

    rng = np.random.default_rng(264)
    lens = rng.integers(241, 12_000, 4001).astype(np.uint64)
    lens[5::16] = rng.integers(1 << 20, 3 << 20, len(lens[5::16]))
    lens[7::9] = rng.integers(0, 241, len(lens[7::9]))
    lens[::37] = 1024 * rng.integers(1, 9, len(lens[::37])) + rng.integers(0, 2, len(lens[::37]))  # block edges
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64) + 1
    offs[1000:1400] = offs[1000:1400][::-1].copy()  # reverse order inside some waves
    offs[2000:2100] = offs[2000]  # overlapping items
    total = int((offs + lens).max()) + 64
    arena = torch.empty(total, dtype=torch.uint8, device=cuda)
    fill_splitmix(arena, 99)
    prev = _capi.lib().oxh_set_kernel_variant(variant)
    try:
        got = _u64(xxh3_128_batch_device(arena, torch.from_numpy(offs.view(np.int64)).to(cuda),
                                         torch.from_numpy(lens.view(np.int64)).to(cuda), mode=_capi.OXH_MODE_WAVE_PACKED))
    finally:
        _capi.lib().oxh_set_kernel_variant(prev)
    want = oracle_lib.batch(arena.cpu().numpy(), offs, lens, threads=8)
    bad = np.nonzero((got != want).any(axis=1))[0]
    assert not len(bad), [(int(i), int(lens[i]), int(offs[i]) % 4) for i in bad[:10]]


@pytest.mark.parametrize("variant", [264])
def test_k1r_items_far_apart(cuda, oracle_lib, variant):
    """K1R with a wave's items more than 4 GiB apart (one descriptor cannot span them): each row's item
    is hashed alone, still bit-exact."""
    import torch

    from oxen_amd import _capi
    from oxen_amd.device import fill_splitmix, xxh3_128_batch_device

    size = (4 << 30) + (64 << 20)
    arena = torch.empty(size, dtype=torch.uint8, device=cuda)
    fill_splitmix(arena, 5)
    offs = np.array([3, (4 << 30) + 17, 1 << 20, (4 << 30) + (1 << 20) + 2, 77, 5000], dtype=np.uint64)
    lens = np.array([70_001, 5_000, 200, 1 << 20, 1025, 90], dtype=np.uint64)
    prev = _capi.lib().oxh_set_kernel_variant(variant)
    try:
        got = _u64(xxh3_128_batch_device(arena, torch.from_numpy(offs.view(np.int64)).to(cuda),
                                         torch.from_numpy(lens.view(np.int64)).to(cuda), mode=_capi.OXH_MODE_WAVE_PACKED))
    finally:
        _capi.lib().oxh_set_kernel_variant(prev)
    for i, (o, L) in enumerate(zip(offs, lens)):
        b = arena[int(o):int(o) + int(L)].cpu().numpy().tobytes()
        assert (int(got[i, 0]), int(got[i, 1])) == oracle_lib.xxh3_128(b), i
    del arena
    torch.cuda.empty_cache()


@pytest.mark.parametrize("mode", ["short", "packed", "auto"])
def test_k1_many_ragged_items(cuda, oracle_lib, mode):
    """Many ragged, byte-packed items (FastCDC-chunk-like, with short-path items mixed in): the
    short-item, packed (block-wise) and default K1 dispatch against the oracle."""
    import torch

    from oxen_amd import _capi
    from oxen_amd.device import fill_splitmix, xxh3_128_batch_device

    rng = np.random.default_rng(17)
    lens = rng.integers(0, 20_000, 40_000).astype(np.uint64)
    lens[::97] = rng.integers(0, 241, len(lens[::97]))  # short-path items mixed in
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64) + 3
    total = int(offs[-1] + lens[-1]) + 64
    arena = torch.empty(total, dtype=torch.uint8, device=cuda)
    fill_splitmix(arena, 1234)
    o = torch.from_numpy(offs.view(np.int64)).to(cuda)
    ln = torch.from_numpy(lens.view(np.int64)).to(cuda)
    m = {"short": _capi.OXH_MODE_WAVE_SHORT, "packed": _capi.OXH_MODE_WAVE_PACKED}.get(mode, _capi.OXH_MODE_AUTO)
    got = _u64(xxh3_128_batch_device(arena, o, ln, mode=m))
    want = oracle_lib.batch(arena.cpu().numpy(), offs, lens, threads=8)
    assert np.array_equal(got, want)


def test_hash_files_path_edge_cases(oracle_lib, tmp_path, cuda):
    """The same path many times in one call, non-ASCII and space-containing names, a symlink to a
    file, a symlink to a directory, a FIFO-free special case (a directory) and empty files, through
    the engine with tiny staging (many slots): digests/status as the reference loop sees them."""
    from oxen_amd import _capi, hasher
    from oxen_amd.workloads import splitmix_bytes

    d = tmp_path / "dir with space"
    d.mkdir()
    files = []
    for k, name in enumerate(["a.bin", "ünïcödé ✓.txt", "x y z", "empty"]):
        p = d / name
        p.write_bytes(b"" if name == "empty" else splitmix_bytes(60 + k, 0, 70_000 + k).tobytes())
        files.append(str(p))
    link = d / "link"
    link.symlink_to(files[0])
    dlink = d / "dlink"
    dlink.symlink_to(d)
    paths = files * 50 + [str(link), str(dlink), str(d)]
    want_out, want_sizes, want_st = oracle_lib.hash_files(paths, threads=8)
    with _capi.Context(0, staging_bytes=1 << 20) as c:
        dg, sz, st = hasher.hash_files_128bit(paths, c)
    assert [s != 0 for s in st] == [int(s) != 0 for s in want_st]
    assert st[-2] != 0 and st[-1] != 0 and st[-3] == 0  # dirs fail, the file symlink is followed
    for i, (lo, hi) in enumerate(want_out):
        if st[i] == 0:
            assert dg[i] == (int(hi) << 64) | int(lo), i
            assert sz[i] == int(want_sizes[i]), i


def test_engine_back_to_back_small_requests(oracle_lib, tmp_path, cuda):
    """Regression: back-to-back calls on one context with tiny staging make the engine flush small
    slots early, so the 3-slot ring can go all the way round while a reader sleeps; a reader waiting
    for a sealed slot must notice the slot was reopened (it used to wait on the slot index alone and
    hang). 300 calls x 203 paths, every result checked."""
    from oxen_amd import _capi, hasher
    from oxen_amd.workloads import splitmix_bytes

    files = []
    for k in range(4):
        p = tmp_path / f"f{k}"
        p.write_bytes(b"" if k == 3 else splitmix_bytes(60 + k, 0, 70_000 + k).tobytes())
        files.append(str(p))
    paths = files * 50 + [str(tmp_path), files[0], str(tmp_path / "missing")]
    want_out, _, want_st = oracle_lib.hash_files(paths, threads=8)
    want = [((int(hi) << 64) | int(lo)) if s == 0 else None for (lo, hi), s in zip(want_out, want_st)]
    with _capi.Context(0, staging_bytes=1 << 20) as c:
        for _ in range(300):
            d, _, st = hasher.hash_files_128bit(paths, c)
            assert d == want


def test_staging_slot_boundaries(oracle_lib, tmp_path, cuda):
    """Items at the staging slot's edges on every host entry: exactly a slot (staged), a slot + 1 (the
    oversize path), a slot - 1, and runs whose 256-B placement overflows the slot by one alignment step
    (the batch must close there) -- oxh_hash_buffers, oxh_hash_streams (span and per-item forms) and
    oxh_hash_files, all against the oracle."""
    from oxen_amd import _capi, hasher
    from oxen_amd.workloads import splitmix_bytes

    S = 1 << 20
    sizes = [S, S + 1, S - 1, 0, 241, S - 300, 300, 1, S // 2 + 1, S // 2, 240, S - 256, 256, 255, S]
    bufs = [splitmix_bytes(900 + i, 0, s).tobytes() for i, s in enumerate(sizes)]
    want = [oracle_lib.xxh3_128_int(b) for b in bufs]
    paths = []
    for i, b in enumerate(bufs):
        p = tmp_path / f"edge{i}"
        p.write_bytes(b)
        paths.append(str(p))
    arena = b"".join(bufs)
    offs = np.cumsum([0] + sizes[:-1]).astype(np.uint64)
    with _capi.Context(0, staging_bytes=S) as c:
        assert hasher.hash_buffers_128bit(bufs, c) == want
        assert hasher.hash_streams_128bit(bufs, c) == want  # forward arena: the span form
        # a scattered arena (items out of order) takes the per-item form
        order = list(range(len(bufs)))[::-1]
        scattered = b"".join(bufs[i] for i in order)
        s_offs = np.zeros(len(bufs), dtype=np.uint64)
        pos = 0
        for i in order:
            s_offs[i] = pos
            pos += sizes[i]
        out = np.zeros((len(bufs), 2), dtype=np.uint64)
        lens = np.array(sizes, dtype=np.uint64)
        src = np.frombuffer(scattered, dtype=np.uint8)
        _capi.check(_capi.lib().oxh_hash_streams(c.handle, ctypes.c_void_p(src.ctypes.data),
                                                 s_offs.ctypes.data_as(_capi._u64p), lens.ctypes.data_as(_capi._u64p),
                                                 len(bufs), out.ctypes.data_as(_capi._u64p)), "oxh_hash_streams")
        assert [(int(hi) << 64) | int(lo) for lo, hi in out] == want
        d, got_sizes, st = hasher.hash_files_128bit(paths, c)
        assert st == [0] * len(paths) and d == want and got_sizes == sizes
    assert len(arena) == int(offs[-1]) + sizes[-1]
