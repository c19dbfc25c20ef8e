"""FastCDC v2020 chunk boundaries + chunk digests (block-level dedup).

Oracle: oracle/fastcdc_oracle.c (two-bytes-per-step loop, as the crate writes it) cross-checked
against oracle/fastcdc.py's per-byte restatement; GEAR derived from the crate's documented MD5 rule.
The crate is not vendored and no reference fixture exists; two of the crate's own published tests
(fastcdc 3.2.1 `test_all_zeros`, `test_masks`) are restated below and pin GEAR[0] (hence the MD5
rule), the mask selection and the min/max walk. Beyond them the bar is: GPU chunk table and digests
bit-identical to the oracle on the same bytes, for every parameter class and the edge cases (empty,
< min, odd tails, dense/pathological candidates).
"""
import ctypes
import os

import numpy as np
import pytest

from oracle import fastcdc as F

CONFIGS = [
    (4096, 8192, 16384),      # makefile:2 chunk size 8 KiB (min 4096 fixed, fastcdchunker.rs:55)
    (4096, 65536, 131072),    # main.rs:129-133 chunk size 64 KiB
    (4096, 4096, 8192),       # avg == min: the truncated window overlaps the mask_l range
    (64, 256, 1024),          # the smallest parameters the crate accepts (dense candidates)
    (300, 257, 1500),         # min > avg, odd sizes
    (1048576, 4194304, 16777216),  # largest: chunks span many 256 KiB sections
]


# ------------------------------------------------------------------------------ CPU (oracle, host)
def test_gear_rule_matches_compiled_table(built_lib):
    from oxen_amd import dedup

    assert dedup.fastcdc_gear() == F.gear_table()


def test_crate_all_zeros_known_answer():
    """The crate's own known answer (fastcdc 3.2.1, src/v2020/mod.rs `test_all_zeros`, a published test
    of the dependency that is not vendored here): 10 240 zero bytes at (64, 256, 1024) give 10 chunks of
    1 024 B at multiples of 1 024, each returned with hash 14169102344523991076. For zeros the rolled
    hash after 64+ steps is -GEAR[0] mod 2^64, so this pins GEAR[0] -- and with it the MD5 rule the
    whole table is derived by -- and the min/max walk."""
    chunks = F.chunks(np.zeros(10240, dtype=np.uint8), 64, 256, 1024)
    assert chunks.tolist() == [[1024 * i, 1024] for i in range(10)]
    gear = F.gear_table()
    h = 0
    for _ in range(1024 - 64):  # cut_gear rolls positions [min, max) of each chunk from hash 0
        h = ((h << 1) + gear[0]) & F.M64
    assert h == 14169102344523991076
    assert F.chunks_py(bytes(10240), 64, 256, 1024) == [(1024 * i, 1024) for i in range(10)]


def test_crate_mask_selection():
    """fastcdc 3.2.1 `test_masks` (src/v2020/mod.rs): which MASKS entries level 1 picks for three
    average sizes (mask_s = MASKS[bits + 1], mask_l = MASKS[bits - 1], bits = log2(avg) rounded)."""
    assert F.masks(256, 1) == (F.MASKS[9], F.MASKS[7])
    assert F.masks(16384, 1) == (F.MASKS[15], F.MASKS[13])
    assert F.masks(4194304, 1) == (F.MASKS[23], F.MASKS[21])


@pytest.mark.parametrize("level", [0, 1, 2, 3])
def test_masks_match_oracle(built_lib, oracle_lib, level):
    import ctypes

    from oxen_amd import dedup

    L = oracle_lib.lib()
    for avg in [256, 300, 362, 363, 512, 4096, 8192, 65536, 100_000, 1 << 20, 4194304]:
        want = (ctypes.c_uint64 * 2)()
        L.oxo_fastcdc_masks.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64)]
        assert L.oxo_fastcdc_masks(avg, level, want) == 0
        assert dedup.fastcdc_masks(avg, level) == (want[0], want[1]) == F.masks(avg, level)
        # every mask bit is below bit 48: the GPU's 48-byte window argument depends on it
        assert want[0] >> 48 == 0 and want[1] >> 48 == 0


def test_mask_popcounts():
    for bits in range(5, 26):
        assert bin(F.MASKS[bits]).count("1") == bits


def test_two_restatements_agree(oracle_lib):
    rng = np.random.default_rng(11)
    for trial in range(12):
        n = int(rng.integers(0, 50_000))
        data = rng.integers(0, 256 if trial % 2 else 4, n, dtype=np.uint8).tobytes()
        for mn, av, mx in CONFIGS[:5]:
            assert F.chunks_py(data, mn, av, mx) == [tuple(map(int, r)) for r in F.chunks(data, mn, av, mx)]


def test_oracle_chunk_invariants(oracle_lib):
    rng = np.random.default_rng(5)
    data = rng.integers(0, 256, 3_000_000, dtype=np.uint8)
    for mn, av, mx in CONFIGS:
        ch = F.chunks(data, mn, av, mx)
        assert int(ch[:, 1].sum()) == len(data)
        assert np.array_equal(ch[1:, 0], np.cumsum(ch[:-1, 1]))
        assert (ch[:-1, 1] >= mn).all() and (ch[:, 1] <= mx).all()


def test_metadata_roundtrip():
    from oxen_amd import dedup

    blob = dedup.encode_metadata("data.parquet", 123456789, ["1", "340282366920938463463374607431768211455"])
    assert dedup.decode_metadata(blob) == ("data.parquet", 123456789, ["1", "340282366920938463463374607431768211455"])
    # bincode 1.x fixint layout: u64 length + utf-8 bytes
    assert blob[:8] == (12).to_bytes(8, "little") and blob[8:20] == b"data.parquet"


def test_chunker_argument_errors(built_lib):
    from oxen_amd import dedup

    with pytest.raises(ValueError, match="Chunk size cannot be zero"):
        dedup.FastCDChunker(0, 1)
    with pytest.raises(ValueError, match="Concurrency must be greater than zero"):
        dedup.FastCDChunker(8192, 0)


# ------------------------------------------------------------------------------ GPU parity
@pytest.fixture(params=["auto", "scan"] + (["fold"] if os.environ.get("OXH_TEST_FOLD") else []))
def cdc_path(request, monkeypatch):
    """Every chunking path: "auto" takes the walk (W + X) wherever it applies (avg <= 16 KiB, masks at
    bit 16 or above: the 8 KiB and 4 KiB configs), F1 + F2 elsewhere; "scan" forces F1 + F2
    (OXH_CDC_WALK=0) everywhere; with OXH_TEST_FOLD=1 (against the probe build,
    tools/build_probe_lib.py + tools/with_lib.py) also "fold": the walk with K1's block sums folded in
    (W2 + K1F, OXH_CDC_FOLD=1; measured and not kept, DESIGN §4 "W2")."""
    monkeypatch.delenv("OXH_CDC_WALK", raising=False)
    monkeypatch.delenv("OXH_CDC_FOLD", raising=False)
    if request.param == "scan":
        monkeypatch.setenv("OXH_CDC_WALK", "0")
    elif request.param == "fold":
        monkeypatch.setenv("OXH_CDC_FOLD", "1")
    return request.param


def _pack(files, align_pad=3):
    """Pack byte arrays back to back with a small odd gap (misaligned starts)."""
    offs, pos = [], 0
    for f in files:
        offs.append(pos)
        pos += len(f) + align_pad
    arena = np.zeros(max(pos, 1), dtype=np.uint8)
    for o, f in zip(offs, files):
        arena[o:o + len(f)] = f
    return arena, np.array(offs, dtype=np.uint64), np.array([len(f) for f in files], dtype=np.uint64)


def _check(cuda, oracle_lib, files, mn, av, mx, level=1):
    import torch

    from oxen_amd.device import fastcdc_device, to_numpy_u64

    arena, offs, lens = _pack(files)
    d_arena = torch.from_numpy(arena).to(cuda)
    c_off, c_len, dig, first = fastcdc_device(d_arena, offs, lens, mn, av, mx, level)
    got_off, got_len = to_numpy_u64(c_off), to_numpy_u64(c_len)
    got_dig = to_numpy_u64(dig).reshape(-1, 2) if dig.numel() else np.zeros((0, 2), np.uint64)
    assert first[0] == 0 and len(first) == len(files) + 1
    for i, f in enumerate(files):
        want = F.chunks(f, mn, av, mx, level)
        a, b = int(first[i]), int(first[i + 1])
        assert b - a == len(want), (i, len(f), b - a, len(want))
        assert np.array_equal(got_off[a:b] - offs[i], want[:, 0]), (i, len(f))
        assert np.array_equal(got_len[a:b], want[:, 1]), (i, len(f))
    if len(got_off):
        want_dig = oracle_lib.batch(arena, got_off, got_len, threads=8)
        assert np.array_equal(got_dig, want_dig)
    return int(first[-1])


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", CONFIGS, ids=lambda c: "-".join(map(str, c)))
def test_fastcdc_random_ragged(cuda, oracle_lib, cfg, cdc_path):
    rng = np.random.default_rng(sum(cfg))
    sizes = [0, 1, 63, 64, 65, cfg[0] - 1, cfg[0], cfg[0] + 1, cfg[1] + 7, cfg[2] - 1, cfg[2], cfg[2] + 1,
             262_143, 262_144, 262_145, 1_000_003, 3 * 262_144 + 17]
    if cfg[0] >= 1 << 20:
        sizes += [40_000_001]
    files = [rng.integers(0, 256, s, dtype=np.uint8) for s in sizes]
    assert _check(cuda, oracle_lib, files, *cfg) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", CONFIGS[:4], ids=lambda c: "-".join(map(str, c)))
def test_fastcdc_low_entropy(cuda, oracle_lib, cfg, cdc_path):
    """Text-like and small-alphabet data: candidates cluster, speculative walks converge late."""
    rng = np.random.default_rng(99)
    text = np.frombuffer(b"".join(b"File content %d\n" % i for i in range(200_000)), dtype=np.uint8)
    files = [text[:3_000_000].copy(), rng.integers(0, 2, 2_000_000, dtype=np.uint8),
             np.tile(rng.integers(0, 256, 4096, dtype=np.uint8), 300)]
    _check(cuda, oracle_lib, files, *cfg)


@pytest.mark.gpu
@pytest.mark.parametrize("byte", [0, 9, 57, 91])
def test_fastcdc_constant_data(cuda, oracle_lib, byte, cdc_path):
    """Constant bytes: the full-window hash is constant. For avg 256 bytes 9/91 make EVERY position a
    mask_l candidate and 57 every position a mask_s candidate: the per-section lists overflow and the
    walk scans bytes (the dense fallback); byte 0 gives no candidates (every chunk is max-sized)."""
    files = [np.full(s, byte, dtype=np.uint8) for s in (100, 5000, 1_500_001)]
    _check(cuda, oracle_lib, files, 64, 256, 1024)
    _check(cuda, oracle_lib, files, 4096, 8192, 16384)


@pytest.mark.gpu
def test_fastcdc_crate_all_zeros_on_device(cuda, cdc_path):
    """The crate's `test_all_zeros` case through the device path: 10 chunks of 1 024 B."""
    import torch

    from oxen_amd.device import fastcdc_device, to_numpy_u64

    arena = torch.zeros(10240, dtype=torch.uint8, device=cuda)
    c_off, c_len, _, first = fastcdc_device(arena, [0], [10240], 64, 256, 1024, digests=False)
    assert int(first[1]) == 10
    assert to_numpy_u64(c_off).tolist() == [1024 * i for i in range(10)]
    assert to_numpy_u64(c_len).tolist() == [1024] * 10


@pytest.mark.gpu
def test_fastcdc_levels(cuda, oracle_lib):
    rng = np.random.default_rng(3)
    files = [rng.integers(0, 256, s, dtype=np.uint8) for s in (10_000, 700_001)]
    for level in (0, 2, 3):
        _check(cuda, oracle_lib, files, 4096, 16384, 65536, level)


@pytest.mark.gpu
def test_fastcdc_invalid_params(cuda):
    import torch

    from oxen_amd import _capi
    from oxen_amd.device import fastcdc_device

    buf = torch.zeros(1024, dtype=torch.uint8, device=cuda)
    for mn, av, mx in [(32, 256, 1024), (4096, 128, 8192), (4096, 8192, 512), (4096, 8 << 20, 16 << 20)]:
        with pytest.raises(_capi.OxenError):
            fastcdc_device(buf, [0], [1024], mn, av, mx)


@pytest.mark.gpu
def test_fastcdchunker_pack(cuda, oracle_lib, tmp_path):
    """fastcdchunker.rs pack(): chunk files named by decimal digests + bincode metadata; unpack is the
    reference's stub (writes nothing), restore() rebuilds the file."""
    from oxen_amd import dedup

    rng = np.random.default_rng(8)
    data = rng.integers(0, 256, 1_234_567, dtype=np.uint8)
    src = tmp_path / "blob.parquet"
    src.write_bytes(data.tobytes())
    ch = dedup.FastCDChunker(8192, 1)
    out = ch.pack(str(src), str(tmp_path / "packed"))
    names = ch.get_chunk_hashes(out)
    want = F.chunks(data, 4096, 8192, 16384)
    assert len(names) == len(want)
    for name, (o, l) in zip(names, want):
        lo, hi = oracle_lib.xxh3_128(data[int(o):int(o + l)].tobytes())
        assert name == str((hi << 64) | lo)
        assert os.path.getsize(os.path.join(out, name)) == l
    name, size, _ = dedup.decode_metadata(open(os.path.join(out, "metadata.bin"), "rb").read())
    assert (name, size) == ("blob.parquet", len(data))
    assert ch.unpack(out, str(tmp_path / "restored")) == str(tmp_path / "restored")  # the reference's stub
    assert not (tmp_path / "restored").exists()
    ch.restore(out, str(tmp_path / "restored"))
    assert (tmp_path / "restored").read_bytes() == data.tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("warmup", ["0", None], ids=["nowarmup", "warmup"])
@pytest.mark.parametrize("section", [1024, 4096, 65536])
@pytest.mark.parametrize("cfg", [CONFIGS[0], CONFIGS[2], CONFIGS[3], CONFIGS[4]], ids=lambda c: "-".join(map(str, c)))
def test_fastcdc_small_sections(cuda, oracle_lib, monkeypatch, section, cfg, warmup, cdc_path):
    """Many sections per file (OXH_CDC_SECTION_BYTES, raised to `max` where smaller and rounded up to
    8 KiB: 64 F1 units of whole 128-byte rounds): speculative walks start mid-chunk everywhere, and the
    stitch re-walks wherever a speculative walk has not converged (constant data never does)."""
    monkeypatch.setenv("OXH_CDC_SECTION_BYTES", str(section))
    if warmup is not None:  # no warm-up: most sections fail the check and are re-walked (F3b)
        monkeypatch.setenv("OXH_CDC_WARMUP_BYTES", warmup)
    rng = np.random.default_rng(section + cfg[1])
    text = np.frombuffer(b"".join(b"row %d,%d\n" % (i, i * 7 % 13) for i in range(60_000)), dtype=np.uint8)
    files = [rng.integers(0, 256, s, dtype=np.uint8) for s in (5, 4097, 65_537, 300_001)]
    files += [text.copy(), np.full(70_000, 9, dtype=np.uint8), rng.integers(0, 3, 100_000, dtype=np.uint8)]
    _check(cuda, oracle_lib, files, *cfg)


@pytest.mark.gpu
@pytest.mark.parametrize("avg", [8192, 65536])
def test_fastcdc_many_default_sections(cuda, oracle_lib, avg, cdc_path):
    """Default section / warm-up sizing (sections >= 512 KiB or 8 max chunks, warm-up >= 128 KiB) over
    files spanning many sections: random, text-like and a misaligned start, C5's min/avg/max shape."""
    rng = np.random.default_rng(avg)
    text = np.frombuffer(b"".join(b"row %d,label %d\n" % (i, i % 7) for i in range(600_000)), dtype=np.uint8)
    files = [rng.integers(0, 256, 12_345_679, dtype=np.uint8), text[:9_000_001].copy(),
             rng.integers(0, 256, 3 * (1 << 20) + 5, dtype=np.uint8)]
    assert _check(cuda, oracle_lib, files, 4096, avg, 2 * avg) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("cap", ["1", "3"])
def test_fastcdc_unit_list_overflow(cuda, oracle_lib, monkeypatch, cap):
    """OXH_CDC_UNIT_CAP shrinks F1's per-unit candidate lists so that most units overflow: the walk
    then scans the bytes after a unit's last stored group (the dense fallback). Same chunks as the
    oracle, at default and at small sections."""
    monkeypatch.setenv("OXH_CDC_UNIT_CAP", cap)
    rng = np.random.default_rng(int(cap))
    text = np.frombuffer(b"".join(b"id %d;%d\n" % (i, i % 5) for i in range(120_000)), dtype=np.uint8)
    files = [rng.integers(0, 256, s, dtype=np.uint8) for s in (9, 70_001, 1_300_000)]
    files += [text.copy(), rng.integers(0, 2, 300_000, dtype=np.uint8)]
    _check(cuda, oracle_lib, files, 4096, 8192, 16384)
    _check(cuda, oracle_lib, files, 64, 256, 1024)
    monkeypatch.setenv("OXH_CDC_SECTION_BYTES", "16384")
    _check(cuda, oracle_lib, files, 4096, 8192, 16384)


@pytest.mark.gpu
@pytest.mark.parametrize("avg", [8192, 65536])
def test_fastcdc_gib_files_fully_checked(cuda, oracle_lib, avg, cdc_path):
    """C5's shape scaled to 4 files of 1 GiB + ragged tails (device-generated splitmix data, files at
    4 KiB-aligned starts as bench_fastcdc lays them out): every chunk boundary of every file and every
    chunk digest against the C oracle -- the whole file, not a prefix."""
    import torch
    from concurrent.futures import ThreadPoolExecutor

    from oxen_amd.device import fastcdc_device, fill_splitmix, to_numpy_u64

    sizes = [(1 << 30) + 13, 1 << 30, (1 << 30) - 4097, (1 << 30) + 65_537]
    pitch = ((max(sizes) + 4095) // 4096) * 4096
    arena = torch.empty(pitch * len(sizes), dtype=torch.uint8, device=cuda)
    fill_splitmix(arena, 4242)
    offs = np.arange(len(sizes), dtype=np.uint64) * np.uint64(pitch)
    lens = np.array(sizes, dtype=np.uint64)
    c_off, c_len, dig, first = fastcdc_device(arena, offs, lens, 4096, avg, 2 * avg)
    got_off, got_len = to_numpy_u64(c_off), to_numpy_u64(c_len)
    got_dig = to_numpy_u64(dig).reshape(-1, 2)

    def one(i):
        host = arena[int(offs[i]):int(offs[i]) + sizes[i]].cpu().numpy()
        want = F.chunks(host, 4096, avg, 2 * avg)
        a, b = int(first[i]), int(first[i + 1])
        ok = b - a == len(want) and np.array_equal(got_off[a:b] - offs[i], want[:, 0]) and np.array_equal(got_len[a:b], want[:, 1])
        return bool(ok and np.array_equal(oracle_lib.batch(host, want[:, 0], want[:, 1], threads=4), got_dig[a:b]))

    with ThreadPoolExecutor(4) as ex:
        assert all(ex.map(one, range(len(sizes))))
    del arena
    torch.cuda.empty_cache()


@pytest.mark.gpu
@pytest.mark.parametrize("avg", [8192, 65536])
def test_fastcdc_item_above_4_gib_fully_checked(cuda, oracle_lib, avg, cdc_path):
    """One device-resident item of 4 GiB + 12 345 B (positions inside the item above 2^32, as C5's
    8 GiB files have them; the host entries never hand the device more than a piece) and a small item
    after it in the arena: every boundary and every digest of both against the C oracle."""
    import torch

    from oxen_amd.device import fastcdc_device, fill_splitmix, to_numpy_u64

    sizes = [(4 << 30) + 12_345, 77_777]
    offs = np.array([0, ((sizes[0] + 4095) // 4096) * 4096], dtype=np.uint64)
    arena = torch.empty(int(offs[1]) + sizes[1] + 4096, dtype=torch.uint8, device=cuda)
    fill_splitmix(arena, 4343)
    lens = np.array(sizes, dtype=np.uint64)
    c_off, c_len, dig, first = fastcdc_device(arena, offs, lens, 4096, avg, 2 * avg)
    got_off, got_len = to_numpy_u64(c_off), to_numpy_u64(c_len)
    got_dig = to_numpy_u64(dig).reshape(-1, 2)
    for i in range(2):
        host = arena[int(offs[i]):int(offs[i]) + sizes[i]].cpu().numpy()
        want = F.chunks(host, 4096, avg, 2 * avg)
        a, b = int(first[i]), int(first[i + 1])
        assert b - a == len(want), (i, b - a, len(want))
        assert np.array_equal(got_off[a:b] - offs[i], want[:, 0]) and np.array_equal(got_len[a:b], want[:, 1]), i
        assert np.array_equal(oracle_lib.batch(host, want[:, 0], want[:, 1], threads=8), got_dig[a:b]), i
        del host
    del arena, c_off, c_len, dig
    torch.cuda.empty_cache()


@pytest.mark.gpu
def test_fastcdc_walk_truncated_window_cuts(cuda, oracle_lib, monkeypatch):
    """The walk (W) never tests a chunk's first 47 hashed positions, where cut_gear's hash has not yet
    seen a full 48-byte window; X re-walks exactly the chunks where one of them matches. With
    min = avg = 4 KiB every tested position uses mask_l (11 bits), so ~47 / 2**11 = 2.3 % of chunks are
    cut inside that window: over 64 MiB of random data ~250 of them. Every boundary must equal the
    oracle's, with the walk path forced (OXH_CDC_WALK=1 fails loudly where it cannot be taken)."""
    import torch

    from oxen_amd.device import fastcdc_device, to_numpy_u64

    monkeypatch.setenv("OXH_CDC_WALK", "1")
    rng = np.random.default_rng(47)
    n = 64 << 20
    data = rng.integers(0, 256, n, dtype=np.uint8)
    want = F.chunks(data, 4096, 4096, 8192)
    # how many chunks the relaxed walk would get wrong, from the oracle's own boundaries
    d_arena = torch.from_numpy(data).to(cuda)
    c_off, c_len, dig, first = fastcdc_device(d_arena, [0], [n], 4096, 4096, 8192)
    assert int(first[1]) == len(want)
    assert np.array_equal(to_numpy_u64(c_off), want[:, 0]) and np.array_equal(to_numpy_u64(c_len), want[:, 1])
    short = int(((want[:-1, 1] >= 4096) & (want[:-1, 1] < 4096 + 47)).sum())
    assert short > 50, short  # chunks cut inside the truncated window: the case X exists for


@pytest.mark.gpu
def test_fastcdc_walk_lists_beyond_lds_take_the_scan(cuda, oracle_lib, monkeypatch):
    """X keeps a section's start list in dynamic LDS (2 x speccap u32). With 128 MiB sections at
    min 4 KiB that is 256 KiB, above a workgroup's 160 KiB: the call must take the scan instead of
    failing its X launch, and with the walk forced (OXH_CDC_WALK=1) fail with a message that says why."""
    from oxen_amd import _capi
    from oxen_amd.device import fastcdc_device

    monkeypatch.setenv("OXH_CDC_SECTION_BYTES", str(128 << 20))
    rng = np.random.default_rng(160)
    files = [rng.integers(0, 256, s, dtype=np.uint8) for s in (3_000_001, 70_000, 0)]
    assert _check(cuda, oracle_lib, files, 4096, 8192, 16384) > 0
    monkeypatch.setenv("OXH_CDC_WALK", "1")
    import torch

    with pytest.raises(_capi.OxenError, match="OXH_CDC_WALK=1: X's section lists do not fit"):
        fastcdc_device(torch.from_numpy(files[0]).to(cuda), [0], [len(files[0])], 4096, 8192, 16384)


# ------------------------------------------------------------------------------ host-memory entry points
def _check_table(oracle_lib, tab, datas, mn, av, mx, level=1):
    """A FastCdcTable (dedup.fastcdc_files / fastcdc_host) against the oracle, file by file."""
    assert len(tab.first) == len(datas) + 1 and int(tab.first[0]) == 0
    for i, d in enumerate(datas):
        off, ln, dig = tab.file(i)
        want = F.chunks(d, mn, av, mx, level) if d is not None else np.zeros((0, 2), np.uint64)
        assert len(off) == len(want), (i, len(off), len(want))
        assert np.array_equal(off, want[:, 0]) and np.array_equal(ln, want[:, 1]), i
        if d is not None and len(want):
            assert np.array_equal(dig, oracle_lib.batch(d, want[:, 0], want[:, 1], threads=8)), i


@pytest.mark.gpu
@pytest.mark.parametrize("piece_mib", [None, "32"], ids=["1GiB-pieces", "32MiB-pieces"])
@pytest.mark.parametrize("cfg", [CONFIGS[0], CONFIGS[1], CONFIGS[3], CONFIGS[4]], ids=lambda c: "-".join(map(str, c)))
def test_fastcdc_files_ragged(cuda, oracle_lib, tmp_path, monkeypatch, cfg, piece_mib):
    """oxh_fastcdc_files (the reference's fs::read -> chunk -> xxh3 per chunk, fastcdchunker.rs:75-98,
    starting and ending in host memory): empty, 1 B, < min, == min, odd tails, files that cross the
    piece boundary and (with 32 MiB pieces) files cut into many segments whose carries must land on
    the crate's boundaries. Every boundary and digest equals the oracle's."""
    from oxen_amd import dedup

    if piece_mib:
        monkeypatch.setenv("OXH_CDC_PIECE_MIB", piece_mib)
    mn, av, mx = cfg
    rng = np.random.default_rng(sum(cfg) + (7 if piece_mib else 0))
    sizes = [0, 1, mn - 1, mn, mn + 1, mx + 7, 262_145, 3_000_001, 70_000_003, 5_555, 41_000_000, 17]
    datas, paths = [], []
    for i, s in enumerate(sizes):
        d = rng.integers(0, 256, s, dtype=np.uint8)
        if i == 9:
            d[:] = 0  # constant data: every position matches or none does
        p = tmp_path / f"f{i}"
        p.write_bytes(d.tobytes())
        datas.append(d)
        paths.append(str(p))
    tab = dedup.fastcdc_files(paths, mn, av, mx)
    assert list(tab.status) == [0] * len(sizes) and list(tab.sizes) == sizes
    _check_table(oracle_lib, tab, datas, mn, av, mx)
    # the same bytes from host buffers
    _check_table(oracle_lib, dedup.fastcdc_host(datas, mn, av, mx), datas, mn, av, mx)


@pytest.mark.gpu
@pytest.mark.parametrize("nctx", [2, 3, 13])
def test_files_multi_contexts(cuda, oracle_lib, tmp_path, monkeypatch, nctx):
    """oxh_fastcdc_files_multi / oxh_chunk_digests_files_multi (one context per device; here all on
    device 0, two of them repeated): byte-balanced contiguous shares side by side, every output --
    offsets, lengths, digests, first_chunk, sizes, status, errno -- equal to the one-context call, which
    the oracle checks. 13 contexts for 12 paths leaves shares empty."""
    from oxen_amd import _capi, dedup

    monkeypatch.setenv("OXH_CDC_PIECE_MIB", "32")
    rng = np.random.default_rng(nctx)
    sizes = [0, 70_000_003, 1, 4095, 3_000_001, 41_000_000, 17, 262_145, 9_000_000, 5]
    datas, paths = [], []
    for i, n in enumerate(sizes):
        d = rng.integers(0, 256, n, dtype=np.uint8)
        p = tmp_path / f"m{i}"
        p.write_bytes(d.tobytes())
        datas.append(d)
        paths.append(str(p))
    paths.insert(3, str(tmp_path / "missing"))
    paths.insert(7, str(tmp_path))
    own = [_capi.Context(0) for _ in range(min(nctx, 3))]
    ctxs = [own[k % len(own)] for k in range(nctx)]
    try:
        one = dedup.fastcdc_files(paths, 4096, 8192, 16384, ctx=own[0])
        many = dedup.fastcdc_files(paths, 4096, 8192, 16384, ctxs=ctxs)
        for f in ("offsets", "lens", "digests", "first", "sizes", "status", "os_error"):
            assert np.array_equal(getattr(one, f), getattr(many, f)), f
        k = 0
        for i in range(len(paths)):
            off, ln, dig = one.file(i)
            if i in (3, 7):
                assert len(off) == 0 and int(one.status[i]) != 0
                continue
            want = F.chunks(datas[k], 4096, 8192, 16384)
            assert np.array_equal(off, want[:, 0]) and np.array_equal(ln, want[:, 1]), i
            if len(want):
                assert np.array_equal(dig, oracle_lib.batch(datas[k], want[:, 0], want[:, 1], threads=8)), i
            k += 1
        # a capacity of exactly the chunk count (below the shares' bounds): each share then fills tables
        # of its own and the call joins them -- the same table as the in-place form above
        from oxen_amd.hasher import _PathTable

        tot = int(one.first[-1])
        off = np.zeros(tot, dtype=np.uint64)
        ln = np.zeros(tot, dtype=np.uint64)
        dg = np.zeros((tot, 2), dtype=np.uint64)
        first = np.zeros(len(paths) + 1, dtype=np.uint64)
        arr = (ctypes.c_void_p * len(ctxs))(*[c.handle.value for c in ctxs])
        table = _PathTable(paths)
        _capi.check(_capi.lib().oxh_fastcdc_files_multi(arr, len(ctxs), table.arg, len(paths), 4096, 8192, 16384, 1,
                                                        off.ctypes.data_as(_capi._u64p), ln.ctypes.data_as(_capi._u64p),
                                                        dg.ctypes.data_as(_capi._u64p), tot,
                                                        first.ctypes.data_as(_capi._u64p), None, None, None), "multi exact")
        assert np.array_equal(first, one.first) and np.array_equal(off, one.offsets)
        assert np.array_equal(ln, one.lens) and np.array_equal(dg, one.digests)
        # the host-buffer forms over the same contexts (shares balanced by length)
        hone = dedup.fastcdc_host(datas, 4096, 8192, 16384, ctx=own[0])
        hmany = dedup.fastcdc_host(datas, 4096, 8192, 16384, ctxs=ctxs)
        for f in ("offsets", "lens", "digests", "first"):
            assert np.array_equal(getattr(hone, f), getattr(hmany, f)), f
        assert np.array_equal(dedup.chunk_digests_host(datas, 4096, ctx=own[0]).digests,
                              dedup.chunk_digests_host(datas, 4096, ctxs=ctxs).digests)
        fone = dedup.chunk_digests_files(paths, 65_536, ctx=own[0])
        fmany = dedup.chunk_digests_files(paths, 65_536, ctxs=ctxs)
        for f in ("digests", "first", "sizes", "status", "os_error"):
            assert np.array_equal(getattr(fone, f), getattr(fmany, f)), f
        k = 0
        for i in range(len(paths)):
            if i in (3, 7):
                continue
            assert np.array_equal(fone.file(i), oracle_lib.chunk_digests(datas[k], 65_536, threads=8)), i
            k += 1
    finally:
        for c in own:
            c.close()


def test_files_multi_arguments():
    """Argument errors of the _multi entries before any device work."""
    from oxen_amd import _capi

    L = _capi.lib()
    first = np.zeros(2, dtype=np.uint64)
    assert L.oxh_fastcdc_files_multi(None, 0, None, 0, 4096, 8192, 16384, 1, None, None, None, 0,
                                     first.ctypes.data_as(_capi._u64p), None, None, None) == _capi.OXH_ERR_INVALID
    assert b"no contexts" in L.oxh_last_error()
    arr = (ctypes.c_void_p * 2)(None, None)
    assert L.oxh_chunk_digests_files_multi(arr, 2, None, 0, 0, None, 0, first.ctypes.data_as(_capi._u64p), None, None,
                                           None) == _capi.OXH_ERR_INVALID
    assert b"zero" in L.oxh_last_error()


@pytest.mark.gpu
@pytest.mark.parametrize("avg", [8192, 65536])
def test_fastcdc_files_2_5_gib_default_pieces(cuda, oracle_lib, tmp_path, avg):
    """A 2.5 GiB file through the default 1 GiB pieces (two piece boundaries inside the file, each
    chunked again from its carry), between two small files: the whole file checked, every boundary
    and every digest, against the oracle."""
    from oxen_amd import dedup
    from oxen_amd.workloads import splitmix_bytes

    big = splitmix_bytes(2525, 0, (5 << 29) + 12_345)
    small = [np.frombuffer(b"hello world" * 1000, dtype=np.uint8), splitmix_bytes(7, 3, 9_999)]
    datas = [small[0], big, small[1]]
    paths = []
    for i, d in enumerate(datas):
        p = tmp_path / f"g{i}"
        d.tofile(str(p))
        paths.append(str(p))
    tab = dedup.fastcdc_files(paths, 4096, avg, 2 * avg)
    assert list(tab.status) == [0, 0, 0]
    _check_table(oracle_lib, tab, datas, 4096, avg, 2 * avg)


@pytest.mark.gpu
def test_fastcdc_files_errors_are_per_file(cuda, oracle_lib, tmp_path):
    """A missing path (File::open fails: OXH_ERR_OPEN, ENOENT), a directory (opens, read fails:
    OXH_ERR_IO, EISDIR), a file used as a directory (ENOTDIR) have no chunks; the files around them are
    chunked exactly. A table too small fails the call and names the count needed."""
    import errno

    from oxen_amd import _capi, dedup

    rng = np.random.default_rng(3)
    a = rng.integers(0, 256, 300_000, dtype=np.uint8)
    b = rng.integers(0, 256, 50_000, dtype=np.uint8)
    (tmp_path / "a").write_bytes(a.tobytes())
    (tmp_path / "b").write_bytes(b.tobytes())
    (tmp_path / "d").mkdir()
    paths = [str(tmp_path / "a"), str(tmp_path / "missing"), str(tmp_path / "d"), str(tmp_path / "a" / "x"), str(tmp_path / "b")]
    tab = dedup.fastcdc_files(paths, 4096, 8192, 16384)
    assert list(tab.status) == [0, _capi.OXH_ERR_OPEN, _capi.OXH_ERR_IO, _capi.OXH_ERR_OPEN, 0]
    assert list(tab.os_error) == [0, errno.ENOENT, errno.EISDIR, errno.ENOTDIR, 0]
    _check_table(oracle_lib, tab, [a, None, None, None, b], 4096, 8192, 16384)
    # capacity: the library counts on and reports what it needed
    from oxen_amd.hasher import _PathTable, default_context

    ctx = default_context()
    t = _PathTable(paths)
    off = np.zeros(2, dtype=np.uint64)
    first = np.zeros(len(paths) + 1, dtype=np.uint64)
    rc = _capi.lib().oxh_fastcdc_files(ctx.handle, t.arg, len(paths), 4096, 8192, 16384, 1, off.ctypes.data_as(_capi._u64p),
                                       off.ctypes.data_as(_capi._u64p), None, 2, first.ctypes.data_as(_capi._u64p),
                                       None, None, None)
    assert rc == _capi.OXH_ERR_INVALID
    assert f"need {len(tab.offsets)} entries" in _capi.lib().oxh_last_error().decode()
    # the reference's pack() returns fs::read's io::Error
    with pytest.raises(FileNotFoundError):
        dedup.FastCDChunker(8192, 1).pack(str(tmp_path / "missing"), str(tmp_path / "out"))


def test_oracle_files_driver_matches_buffers(oracle_lib, tmp_path):
    """oxo_fastcdc_files (the CPU baseline of tools/bench_fastcdc_e2e.py: per file read or mmap -> v2020
    -> xxh3_128 per chunk, files over threads) reports for every file the chunk count and the
    fingerprint of exactly the table F.chunks + the per-chunk oracle give; errors per file."""
    rng = np.random.default_rng(12)
    datas, paths = [], []
    for i, s in enumerate([0, 1, 4095, 4097, 300_001, 2_000_000]):
        d = rng.integers(0, 256, s, dtype=np.uint8)
        p = tmp_path / f"o{i}"
        p.write_bytes(d.tobytes())
        datas.append(d)
        paths.append(str(p))
    paths.append(str(tmp_path / "missing"))
    for mm in (False, True):
        counts, fp, st = F.files(paths, 4096, 8192, 16384, threads=3, mmap_files=mm)
        assert list(st) == [0] * len(datas) + [1]
        for i, d in enumerate(datas):
            want = F.chunks(d, 4096, 8192, 16384)
            dig = oracle_lib.batch(d, want[:, 0], want[:, 1]) if len(want) else np.zeros((0, 2), np.uint64)
            assert int(counts[i]) == len(want)
            assert (int(fp[i, 0]), int(fp[i, 1])) == F.record_fingerprint(want[:, 0], want[:, 1], dig)


@pytest.mark.gpu
def test_fastcdc_host_entries_concurrent(cuda, oracle_lib, tmp_path, monkeypatch):
    """Three callers at once on one device: oxh_fastcdc_files on one context, oxh_fastcdc_host on a second
    (each with its own piece pipeline; the device's two scratch buffers are shared by lease), and
    oxh_hash_files on the process's default context's engine -- every result equal to the oracle's,
    three rounds each. Small pieces (32 MiB) make every call cross piece boundaries."""
    import threading

    from oxen_amd import _capi, dedup, hasher

    monkeypatch.setenv("OXH_CDC_PIECE_MIB", "32")
    rng = np.random.default_rng(33)
    datas = [rng.integers(0, 256, s, dtype=np.uint8) for s in (70_000_001, 5_000_000, 123_457, 0, 40_000_000)]
    paths = []
    for i, d in enumerate(datas):
        p = tmp_path / f"c{i}"
        p.write_bytes(d.tobytes())
        paths.append(str(p))
    errs = []

    def files_worker():
        try:
            with _capi.Context(0) as c:
                for _ in range(3):
                    _check_table(oracle_lib, dedup.fastcdc_files(paths, 4096, 8192, 16384, ctx=c), datas, 4096, 8192, 16384)
        except Exception as e:  # noqa: BLE001
            errs.append(("files", repr(e)))

    def host_worker():
        try:
            with _capi.Context(0) as c:
                for _ in range(3):
                    _check_table(oracle_lib, dedup.fastcdc_host(datas, 4096, 65536, 131072, ctx=c), datas, 4096, 65536, 131072)
        except Exception as e:  # noqa: BLE001
            errs.append(("host", repr(e)))

    def hash_worker():
        try:
            from oracle import oracle

            want = [oracle.xxh3_128_int(d.tobytes()) for d in datas]
            for _ in range(3):
                got, sizes, status = hasher.hash_files_128bit(paths)
                assert status == [0] * len(paths) and got == want
        except Exception as e:  # noqa: BLE001
            errs.append(("hash", repr(e)))

    ts = [threading.Thread(target=f) for f in (files_worker, host_worker, hash_worker)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(600)
    assert not errs, errs


@pytest.mark.gpu
def test_fastcdc_files_many_small(cuda, oracle_lib, tmp_path):
    """5 000 small files in one call (more than a round's 2 048 files, each holding a descriptor until it
    is read): every file chunked exactly, in order, no descriptor exhaustion."""
    from oxen_amd import dedup

    rng = np.random.default_rng(5000)
    datas, paths = [], []
    for i in range(5000):
        d = rng.integers(0, 256, int(rng.integers(0, 40_000)), dtype=np.uint8)
        p = tmp_path / f"s{i:05d}"
        p.write_bytes(d.tobytes())
        datas.append(d)
        paths.append(str(p))
    tab = dedup.fastcdc_files(paths, 4096, 8192, 16384)
    assert (tab.status == 0).all()
    _check_table(oracle_lib, tab, datas, 4096, 8192, 16384)


@pytest.mark.gpu
@pytest.mark.parametrize("level", [0, 1, 2, 3])
def test_fastcdc_host_levels(cuda, oracle_lib, monkeypatch, level):
    """The normalization levels (v2020::FastCDC::with_level, Level0..Level3: MASKS[bits +/- level])
    through the host entry, files split over 32 MiB pieces."""
    from oxen_amd import dedup

    monkeypatch.setenv("OXH_CDC_PIECE_MIB", "32")
    rng = np.random.default_rng(100 + level)
    datas = [rng.integers(0, 256, s, dtype=np.uint8) for s in (45_000_003, 9_999, 0, 4096)]
    for mn, av, mx in [(4096, 8192, 16384), (4096, 65536, 131072)]:
        tab = dedup.fastcdc_host(datas, mn, av, mx, level=level)
        _check_table(oracle_lib, tab, datas, mn, av, mx, level=level)


@pytest.mark.gpu
def test_host_chunk_entries_empty_calls(cuda):
    """n = 0 on every host chunk entry (one context and several): first_chunk = [0], nothing read and
    no pipeline buffers made."""
    from oxen_amd import _capi, dedup

    ctxs = [_capi.Context(0), _capi.Context(0)]
    try:
        for kw in ({"ctx": ctxs[0]}, {"ctxs": ctxs}):
            assert list(dedup.fastcdc_files([], 4096, 8192, 16384, **kw).first) == [0]
            assert list(dedup.fastcdc_host([], 4096, 8192, 16384, **kw).first) == [0]
            assert list(dedup.chunk_digests_files([], 4096, **kw).first) == [0]
            assert list(dedup.chunk_digests_host([], 4096, **kw).first) == [0]
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.gpu
def test_host_chunk_entries_low_fd_limit(cuda, oracle_lib, tmp_path):
    """the host chunk entries under a low descriptor limit. 2 000 empty files (which used to
    keep their descriptors to the end of the call), 300 small files and a few missing paths, with the
    soft RLIMIT_NOFILE lowered to what the process holds + 200: every file is chunked (or reported
    missing with ENOENT, like fs::read), no spurious OXH_ERR_OPEN from EMFILE -- on one context and on
    three side by side (the _multi entries split the descriptor budget over their shares)."""
    import errno
    import resource

    from oxen_amd import _capi, dedup

    rng = np.random.default_rng(2300)
    datas, paths = [], []
    for i in range(2320):
        p = tmp_path / f"e{i:05d}"
        if i % 8 == 3 and len([d for d in datas if d is not None and len(d)]) < 300:
            d = rng.integers(0, 256, int(rng.integers(1, 50_000)), dtype=np.uint8)
        elif i % 500 == 7:
            paths.append(str(p) + ".missing")
            datas.append(None)
            continue
        else:
            d = np.zeros(0, np.uint8)
        p.write_bytes(d.tobytes())
        datas.append(d)
        paths.append(str(p))
    missing = [i for i, d in enumerate(datas) if d is None]
    ctxs = [_capi.Context(0) for _ in range(3)]
    one = _capi.Context(0)
    for c in [one] + ctxs:  # pipelines and reader pools made before the limit drops
        dedup.fastcdc_host([np.zeros(10, np.uint8)], 4096, 8192, 16384, ctx=c)
    dedup.fastcdc_host([np.zeros(10, np.uint8)], 4096, 8192, 16384, ctxs=ctxs)
    soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
    low = len(os.listdir("/proc/self/fd")) + 200
    if hard != resource.RLIM_INFINITY and low > hard:
        pytest.skip("hard descriptor limit below the test's")
    try:
        resource.setrlimit(resource.RLIMIT_NOFILE, (low, hard))
        for kw in ({"ctx": one}, {"ctxs": ctxs}):
            tab = dedup.fastcdc_files(paths, 4096, 8192, 16384, **kw)
            fix = dedup.chunk_digests_files(paths, 4096, **kw)
            for t in (tab, fix):
                bad = [i for i in range(len(paths)) if (i in missing) != (t.status[i] != 0)]
                assert not bad, (kw.keys(), bad[:5], [int(t.status[i]) for i in bad[:5]])
                assert all(t.status[i] == _capi.OXH_ERR_OPEN and t.os_error[i] == errno.ENOENT for i in missing)
            _check_table(oracle_lib, tab, datas, 4096, 8192, 16384)
            for i, d in enumerate(datas):
                if d is None or not len(d):
                    assert len(fix.file(i)) == 0
                    continue
                offs = np.arange(0, len(d), 4096, dtype=np.uint64)
                lens = np.minimum(np.uint64(4096), np.uint64(len(d)) - offs)
                assert np.array_equal(fix.file(i), oracle_lib.batch(d, offs, lens)), i
    finally:
        resource.setrlimit(resource.RLIMIT_NOFILE, (soft, hard))
        for c in [one] + ctxs:
            c.close()


@pytest.mark.gpu
def test_file_entries_refuse_a_fifo_without_blocking(cuda, oracle_lib, tmp_path):
    """A FIFO among the paths (no writer): open(2) without O_NONBLOCK would park a reader in the call
    forever (fs::read would wait there too). The host chunk entries and the file engine open it
    non-blocking and refuse it as unreadable -- OXH_ERR_IO with EINVAL -- while the files around it are
    chunked / hashed exactly."""
    import errno
    import os

    from oxen_amd import _capi, dedup, hasher

    rng = np.random.default_rng(99)
    datas = [rng.integers(0, 256, 70_000, dtype=np.uint8), None, rng.integers(0, 256, 5_000, dtype=np.uint8)]
    paths = []
    for i, d in enumerate(datas):
        p = tmp_path / f"p{i}"
        if d is None:
            os.mkfifo(p)
        else:
            p.write_bytes(d.tobytes())
        paths.append(str(p))
    tab = dedup.fastcdc_files(paths, 4096, 8192, 16384)
    assert list(tab.status) == [0, _capi.OXH_ERR_IO, 0] and int(tab.os_error[1]) == errno.EINVAL
    _check_table(oracle_lib, tab, datas, 4096, 8192, 16384)
    fix = dedup.chunk_digests_files(paths, 4096)
    assert list(fix.status) == [0, _capi.OXH_ERR_IO, 0] and int(fix.os_error[1]) == errno.EINVAL
    assert len(fix.file(1)) == 0
    d, _, st, oe = hasher.hash_files_with_errors_128bit(paths)
    assert st == [0, _capi.OXH_ERR_IO, 0] and oe[1] == errno.EINVAL
    assert d[0] == oracle_lib.xxh3_128_int(datas[0].tobytes()) and d[2] == oracle_lib.xxh3_128_int(datas[2].tobytes())
