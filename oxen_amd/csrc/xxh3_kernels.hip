// oxen_amd/csrc/xxh3_kernels.hip -- hand-written gfx950 kernels for the content-hash stage.
//
//   K1   xxh3_wave_kernel     one 64-lane wave per buffer; XXH3-128 long path in 4 KiB rounds.
//   K1s  xxh3_lane_kernel     one lane per buffer (short items, parent-node streams).
//   K1L  xxh3_blocksum_kernel + xxh3_chain_kernel: one huge buffer, block sums chip-wide, then the
//        serial scramble chain on one wave.
//   K2   xxh3_combined_kernel get_combined_hash (hasher.rs:67-80) on (content, metadata) pairs.
//   util fill_splitmix_kernel synthetic, host-reproducible byte stream.
//
// Long-path data layout (K1): a "round" is 4 consecutive 1 KiB XXH3 blocks = 4 KiB. Lane l of the
// wave owns row g = l/16 (block 4r+g of the round), stripe-in-quad q = (l/4)%4 and word pair
// k = l%4. Load j (0..3) of a round reads 16 B at block_base + (4j+q)*64 + 16k, so each 16-lane row
// reads 256 contiguous bytes per instruction (4 x 256 B = 8 full 128-B lines per wave-instruction,
// the same line count as a flat 1 KiB load), and after the 4 loads lane l has summed stripes
// {q, q+4, q+8, q+12} of its block for accumulators (2k, 2k+1). Two DPP row rotations (ror 4,
// ror 8) finish the 16-stripe block sum inside each row; permlane16/32 swaps broadcast the four
// block sums to every row, and every lane then runs the 4-step scramble chain for its 2 accumulators.
// All of it is 32-bit VALU integer work -- no LDS traffic and no MFMA.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "xxh3_device.hpp"

namespace oxh {

static __constant__ uint64_t kInitW[8] = {acc_init(0), acc_init(1), acc_init(2), acc_init(3),
                                          acc_init(4), acc_init(5), acc_init(6), acc_init(7)};
// last-stripe keys: secret + 192 - 64 - 7 = 121
static __constant__ uint64_t kLastW[8] = {S64(121), S64(129), S64(137), S64(145),
                                          S64(153), S64(161), S64(169), S64(177)};
// merge keys: low64 at secret + 11, high64 at secret + 192 - 64 - 11 = 117
static __constant__ uint64_t kMrgLo[8] = {S64(11), S64(19), S64(27), S64(35),
                                          S64(43), S64(51), S64(59), S64(67)};
static __constant__ uint64_t kMrgHi[8] = {S64(117), S64(125), S64(133), S64(141),
                                          S64(149), S64(157), S64(165), S64(173)};

constexpr int DPP_ROW_ROR4 = 0x124;
constexpr int DPP_ROW_ROR8 = 0x128;
constexpr int DPP_QUAD_XOR1 = 0xB1;
constexpr int DPP_QUAD_XOR2 = 0x4E;

template <int CTRL>
__device__ __forceinline__ uint64_t dpp64(uint64_t x) {
    const uint32_t lo = __builtin_amdgcn_update_dpp(0u, (uint32_t)x, CTRL, 0xf, 0xf, false);
    const uint32_t hi = __builtin_amdgcn_update_dpp(0u, (uint32_t)(x >> 32), CTRL, 0xf, 0xf, false);
    return ((uint64_t)hi << 32) | lo;
}

// Broadcast the value held by each 16-lane row r (x_r) so that every lane gets x_0..x_3.
// VARIANT 0: v_permlane16_swap + v_permlane32_swap (gfx950 VALU cross-row moves).
// VARIANT 1: ds_bpermute through __shfl (LDS crossbar) -- reference formulation for A/B.
template <int VARIANT>
__device__ __forceinline__ void bcast_rows32(uint32_t x, uint32_t& b0, uint32_t& b1, uint32_t& b2,
                                             uint32_t& b3, int lane) {
    if constexpr (VARIANT == 0) {
        // permlane16_swap(a, b): swaps odd rows of a with even rows of b.
        //   with a = b = x:  r[0] = (x0, x0, x2, x2), r[1] = (x1, x1, x3, x3)
        // permlane32_swap(a, b): swaps the upper half of a with the lower half of b.
        //   with a = b = y:  r[0] = (y_lo, y_lo),    r[1] = (y_hi, y_hi)
        const auto p16 = __builtin_amdgcn_permlane16_swap(x, x, false, false);
        const auto pa = __builtin_amdgcn_permlane32_swap(p16[0], p16[0], false, false);
        const auto pb = __builtin_amdgcn_permlane32_swap(p16[1], p16[1], false, false);
        b0 = pa[0];
        b2 = pa[1];
        b1 = pb[0];
        b3 = pb[1];
    } else {
        const int c = lane & 15;
        b0 = __shfl((int)x, c, 64);
        b1 = __shfl((int)x, 16 + c, 64);
        b2 = __shfl((int)x, 32 + c, 64);
        b3 = __shfl((int)x, 48 + c, 64);
    }
}

template <int VARIANT>
__device__ __forceinline__ void bcast_rows64(uint64_t x, uint64_t t[4], int lane) {
    uint32_t l0, l1, l2, l3, h0, h1, h2, h3;
    bcast_rows32<VARIANT>((uint32_t)x, l0, l1, l2, l3, lane);
    bcast_rows32<VARIANT>((uint32_t)(x >> 32), h0, h1, h2, h3, lane);
    t[0] = ((uint64_t)h0 << 32) | l0;
    t[1] = ((uint64_t)h1 << 32) | l1;
    t[2] = ((uint64_t)h2 << 32) | l2;
    t[3] = ((uint64_t)h3 << 32) | l3;
}

// Kernel variant knobs (diagnostic A/B through oxh_set_kernel_variant; 0 is the shipped path):
//   bit 0     cross-row broadcast: 0 = permlane16/32 swaps, 1 = ds_bpermute (__shfl)
//   bit 1     0 = non-temporal (nt) loads for the once-read input stream, 1 = default-policy loads
//   bits 2-3  rounds in flight per wave (software pipeline depth): 0 -> 4, 1 -> 3, 2 -> 2, 3 -> 5
//   bit 4     1 = stagger: waves of the first resident generation start 0..15 x ~1 us apart
//   bit 5     1 = block-wise layout: load j of a round reads block j whole (1 KiB contiguous per
//             wave-instruction; lane l holds stripe l/4, piece l%4 of every block, so its keys are
//             fixed), and a reduce-scatter across rows (permlane32/16 swaps) hands row g block g's
//             partial sums before the usual in-row fold. 0 = row-wise: row g reads block g, 256 B per
//             instruction. At a start that is not 128-B aligned a row-wise instruction touches 12
//             lines per KiB, a block-wise one 9 (tools/k1_small_probe.py).
//   bit 6     1 = stripe keys read from an LDS copy of the secret at each use (fewer VGPRs)
//   bit 8     1 = K1R, one 16-lane row per item and four items per wave (rows_item below; bits 1-3
//             as above, the others unused)
//   bit 9     K1R only: 1 = K1H, two rows per item and two items per wave
//   bit 10    1 = rotated start (K1 only): item i visits its first min(nr, 16) full rounds starting at
//             round i % 16, stashing the block sums of the rounds it reads before round 0 in LDS and
//             replaying them into the chain in order -- so the waves in flight, whose items all start
//             on 64 KiB boundaries in C2's arena, read at addresses 4 KiB apart instead of in lockstep
// Measured on MI355X (C2, tools/readbw.py, profiles/r01_readbw*.json): nt loads ~+11 % over
// default-policy loads; 4 rounds in flight (2 waves/SIMD at 180 VGPRs) ~+4 % over 2 rounds (5 waves/SIMD).
template <int V>
struct Cfg {
    static constexpr int BCAST = V & 1;
    static constexpr bool NT = ((V >> 1) & 1) == 0;
    static constexpr int DEPTH = ((V >> 2) & 3) == 0 ? 4 : ((V >> 2) & 3) == 1 ? 3 : ((V >> 2) & 3) == 2 ? 2 : 5;
    static constexpr bool KEYS_LDS = ((V >> 6) & 1) != 0;
    static constexpr bool STAGGER = ((V >> 4) & 1) != 0;
    static constexpr bool BLOCKWISE = ((V >> 5) & 1) != 0;
    static constexpr bool ROWS = ((V >> 8) & 1) != 0;
    static constexpr bool ROWS2 = ((V >> 9) & 1) != 0;
    static constexpr bool ROT = ((V >> 10) & 1) != 0;
};

template <bool ALIGNED, bool NT = false>
__device__ __forceinline__ uint4 load16(const uint8_t* p) {
    if constexpr (ALIGNED && NT) {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
        return make_uint4(v.x, v.y, v.z, v.w);
    } else if constexpr (ALIGNED) {
        return *reinterpret_cast<const uint4*>(p);
    } else {
        uint4 v;
        __builtin_memcpy(&v, p, 16);
        return v;
    }
}

// One 16-byte piece of one stripe: words (2k, 2k+1) with keys (key0, key1).
__device__ __forceinline__ void accum16(const uint4 d, uint64_t key0, uint64_t key1, uint64_t& s0,
                                        uint64_t& s1) {
    const uint64_t w0 = ((uint64_t)d.y << 32) | d.x;
    const uint64_t w1 = ((uint64_t)d.w << 32) | d.z;
    const uint64_t k0 = w0 ^ key0;
    const uint64_t k1 = w1 ^ key1;
    s0 += mul32x32(k0) + w1;  // acc[2k]   += lo*hi of its keyed word, plus word 2k+1 (the i^1 swap)
    s1 += mul32x32(k1) + w0;  // acc[2k+1] += lo*hi of its keyed word, plus word 2k
}

// Text metadata counts fused into the hash pass (repositories/metadata/text.rs:11-20 ->
// util/fs.rs:217-263): newlines (num_lines = 1 + count) and UTF-8 continuation bytes
// (num_chars = len - count, bytecount::num_chars). SWAR over each dword.
__device__ __forceinline__ uint32_t count_nl32(uint32_t w) {
    const uint32_t x = w ^ 0x0A0A0A0Au;                                // newline bytes become 0
    const uint32_t t = ((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x;          // bit 7 set in non-zero bytes
    return (uint32_t)__builtin_popcount(~t & 0x80808080u);
}
__device__ __forceinline__ uint32_t count_cont32(uint32_t w) {
    return (uint32_t)__builtin_popcount(w & ~(w << 1) & 0x80808080u);  // bytes 10xxxxxx
}
__device__ __forceinline__ void count16(const uint4 d, uint32_t& nl, uint32_t& cont) {
    nl += count_nl32(d.x) + count_nl32(d.y) + count_nl32(d.z) + count_nl32(d.w);
    cont += count_cont32(d.x) + count_cont32(d.y) + count_cont32(d.z) + count_cont32(d.w);
}

// Fold a round: in-row stripe reduction, cross-row broadcast, 4 chain steps.
// nfull: how many of the 4 blocks are full (scrambled); block nfull (if < 4) is the partial one.
template <int VARIANT>
__device__ __forceinline__ void fold_round(uint64_t s0, uint64_t s1, uint64_t& a0, uint64_t& a1,
                                           uint64_t sk0, uint64_t sk1, int nfull, int lane) {
    s0 += dpp64<DPP_ROW_ROR4>(s0);
    s1 += dpp64<DPP_ROW_ROR4>(s1);
    s0 += dpp64<DPP_ROW_ROR8>(s0);
    s1 += dpp64<DPP_ROW_ROR8>(s1);
    uint64_t t0[4], t1[4];
    bcast_rows64<VARIANT>(s0, t0, lane);
    bcast_rows64<VARIANT>(s1, t1, lane);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        if (g < nfull) {
            a0 = scramble1(a0 + t0[g], sk0);
            a1 = scramble1(a1 + t1[g], sk1);
        } else if (g == nfull) {
            a0 += t0[g];
            a1 += t1[g];
        }
    }
}

// Block-wise layout: lane (g, q, k) holds, for each block j of the round, the partial sum of
// stripe 4g+q (v[j]). Two swap-and-add steps leave row g with block g's sum over the four rows
// (still split by q; fold_round's in-row adds finish it):
//   permlane32_swap(v0, v2) -> (v0 lower half, v2 lower half), (v0 upper, v2 upper): the sum holds
//   block 0 in rows 0-1 and block 2 in rows 2-3 (likewise blocks 1 / 3); permlane16_swap of those
//   two then leaves (block 0, block 1, block 2, block 3) in rows (0, 1, 2, 3).
__device__ __forceinline__ uint64_t swap32_add(uint64_t a, uint64_t b) {
    const auto lo = __builtin_amdgcn_permlane32_swap((uint32_t)a, (uint32_t)b, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((uint32_t)(a >> 32), (uint32_t)(b >> 32), false, false);
    return (((uint64_t)hi[0] << 32) | lo[0]) + (((uint64_t)hi[1] << 32) | lo[1]);
}
__device__ __forceinline__ uint64_t swap16_add(uint64_t a, uint64_t b) {
    const auto lo = __builtin_amdgcn_permlane16_swap((uint32_t)a, (uint32_t)b, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((uint32_t)(a >> 32), (uint32_t)(b >> 32), false, false);
    return (((uint64_t)hi[0] << 32) | lo[0]) + (((uint64_t)hi[1] << 32) | lo[1]);
}
__device__ __forceinline__ uint64_t rows_from_blocks(const uint64_t (&v)[4]) {
    return swap16_add(swap32_add(v[0], v[2]), swap32_add(v[1], v[3]));
}

// Buffer resource over one item: loads at voffset >= num_records are dropped by the hardware range
// check (no memory traffic, zeros returned), which lets the pipeline issue every prefetch
// unconditionally -- no branch around a load, so the register ring never needs a phi/copy.
constexpr uint32_t kOOB = 0xFFFFF000u;
constexpr int kRsrcFlags = 0x00020000;  // gfx950 raw-buffer descriptor word 3

template <bool NT>
__device__ __forceinline__ uint4 bload16(__amdgpu_buffer_rsrc_t rsrc, uint32_t voff) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, 0, NT ? 2 : 0);
    return make_uint4(v.x, v.y, v.z, v.w);
}

// The long path (len > 240) for one buffer, executed by one full wave. Writes out[0..1] from lane 0.
// All input loads are raw buffer loads (gfx950 supports unaligned buffer access, so any start offset
// is fine); the descriptor is re-based every 1 GiB so 32-bit offsets cover buffers of any length.
//
// BS (byte shift, 1..3; 0 = none): the item starts bs bytes past a dword boundary. Buffer loads at
// such offsets run ~25 % slower than dword-aligned ones (measured: tools/k1_align_probe.py), so the
// loads are issued from the dword-aligned base p - bs and every 16-byte piece is re-aligned in
// registers with v_alignbyte_b32; the dword after a lane's piece comes from the next lane of its row
// (DPP row_ror:15), for a row's last lane from the next load of the row, and for the last lane of
// the last load from one extra dword load per round (4 active lanes).
template <int VARIANT, bool TEXT, bool BS>
__device__ __forceinline__ void wave_long(const uint8_t* __restrict__ p, uint64_t len,
                                          uint64_t* __restrict__ out, int lane, const uint64_t* lds_sec,
                                          uint64_t* __restrict__ counts, uint32_t bs = 0, uint64_t* stash = nullptr,
                                          uint64_t phase = 0) {
    constexpr bool BW = Cfg<VARIANT>::BLOCKWISE;
    constexpr uint32_t JSTRIDE = BW ? 1024u : 256u;  // bytes between a lane's loads j and j+1
    const int g = lane >> 4, q = (lane >> 2) & 3, k = lane & 3;
    uint32_t n_nl = 0, n_cont = 0;  // TEXT only
    // stripe keys: secret words (stripe + 2k, +1); the lane's stripe in load j is 4j + q (row-wise)
    // or 4g + q (block-wise, the same for every j)
    auto keys = [&](int j, uint64_t& k0, uint64_t& k1) {
        int idx = (BW ? 4 * g : 4 * j) + q + 2 * k;
        if constexpr (Cfg<VARIANT>::KEYS_LDS) {
            asm volatile("" : "+v"(idx));  // opaque: keep the LDS reads inside the loop
            k0 = lds_sec[idx];
            k1 = lds_sec[idx + 1];
        } else {
            k0 = kSecW[idx];
            k1 = kSecW[idx + 1];
        }
    };
    const uint64_t sk0 = kSecW[16 + 2 * k], sk1 = kSecW[16 + 2 * k + 1];
    uint64_t a0 = kInitW[2 * k], a1 = kInitW[2 * k + 1];

    const uint64_t nb = (len - 1) >> 10;  // blocks followed by a scramble
    const uint64_t nr = nb >> 2;          // full rounds (4 scrambled blocks each)
    const uint32_t lane_off = (uint32_t)(g * (BW ? 256 : 1024) + q * 64 + k * 16);
    // round rr lives in 1 GiB window rr >> 18; descriptor over that window (wave-uniform, SALU work)
    auto window_rsrc = [&](uint64_t rr) {
        const uint64_t base = (rr >> 18) << 30;
        const uint64_t rem = len - base + (BS ? bs : 0);
        return __builtin_amdgcn_make_buffer_rsrc((void*)(p + base - (BS ? bs : 0)), (short)0,
                                                 (int)(rem < 0x7FFFFFFFull ? rem : 0x7FFFFFFFull), kRsrcFlags);
    };
    // Rounds 0 .. nr-1 are full (4 scrambled blocks); round nr is the partial final round: blocks
    // 4nr .. nb-1 full, block nb with `ns` stripes. The lane's piece of load j (block b, stripe s:
    // row-wise b = 4nr + g, s = 4j + q; block-wise b = 4nr + j, s = 4g + q) is live in round rr if
    // rr < nr, or rr == nr and (b < nb or (b == nb and s < ns)).
    const uint64_t ns = ((len - 1) - (nb << 10)) >> 6;
    // branch-free (bitwise) so that no load ends up inside control flow
    auto fin_full = [&](int j) -> bool { return nr * 4 + (uint64_t)(BW ? j : g) < nb; };
    auto fin_part = [&](int j) -> bool { return nr * 4 + (uint64_t)(BW ? j : g) == nb; };
    auto stripe_of = [&](int j) -> uint64_t { return (uint64_t)((BW ? 4 * g : 4 * j) + q); };
    auto live_j = [&](uint64_t rr, int j) -> bool {
        const bool fp = fin_part(j), ff = fin_full(j);
        const bool in_part = ff | (fp & (stripe_of(j) < ns));
        return (rr < nr) | ((rr == nr) & in_part);
    };
    auto load_round = [&](uint64_t rr, uint4 (&dst)[4], uint32_t& ext) {
        const __amdgpu_buffer_rsrc_t rsrc = window_rsrc(rr);
        const uint32_t vo = (uint32_t)(rr & 0x3FFFF) * 4096u + lane_off;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            // BS: the first lane of the stripe after a partial block's last live stripe loads too (its
            // first dword completes the last live piece; dwords past the item read as 0)
            const bool fp = fin_part(j);
            const bool extra = BS && (rr == nr) & fp & (stripe_of(j) == ns) & (k == 0);
            dst[j] = bload16<Cfg<VARIANT>::NT>(rsrc, (live_j(rr, j) | extra) ? vo + j * JSTRIDE : kOOB);
        }
        if constexpr (BS) {
            // the dword right after the last piece of load 3, for the lane that holds that piece
            // (row-wise: each row's last lane, 15 / 31 / 47 / 63; block-wise: lane 63)
            const bool tail = BW ? lane == 63 : (lane & 15) == 15;
            ext = __builtin_amdgcn_raw_buffer_load_b32(rsrc, (tail && live_j(rr, 3)) ? vo + 3 * JSTRIDE + 16 : kOOB, 0,
                                                       Cfg<VARIANT>::NT ? 2 : 0);
        } else {
            ext = 0;
        }
    };
    // BS: item bytes [o, o+16) of every piece from the aligned pieces (see above)
    auto realign = [&](uint4 (&src)[4], uint32_t ext) {
        if constexpr (BS) {
            // the next lane's first dword: row_ror:15 inside a row (row-wise), wave_rol:1 (block-wise);
            // the lane holding a load's last piece takes it from load j+1 (lane 0 of its row / wave)
            const bool tail = BW ? lane == 63 : (lane & 15) == 15;
            uint32_t nb[4];
#pragma unroll
            for (int j = 0; j < 4; ++j)
                nb[j] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)src[j].x, BW ? 0x134 : 0x12F, 0xf, 0xf, false);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t n0 = tail ? (j < 3 ? nb[j + 1] : ext) : nb[j];
                const uint4 a = src[j];
                src[j] = make_uint4(__builtin_amdgcn_alignbyte(a.y, a.x, bs), __builtin_amdgcn_alignbyte(a.z, a.y, bs),
                                    __builtin_amdgcn_alignbyte(a.w, a.z, bs), __builtin_amdgcn_alignbyte(n0, a.w, bs));
            }
        }
    };
    auto fold4 = [&](uint4 (&src)[4], uint32_t ext, uint64_t rr, bool partial) {
        realign(src, ext);
        uint64_t s0 = 0, s1 = 0;
        if constexpr (BW) {
            uint64_t v0[4] = {0, 0, 0, 0}, v1[4] = {0, 0, 0, 0};
            uint64_t k0, k1;
            keys(0, k0, k1);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (!partial || live_j(rr, j)) {
                    accum16(src[j], k0, k1, v0[j], v1[j]);
                    if constexpr (TEXT) count16(src[j], n_nl, n_cont);
                }
            }
            s0 = rows_from_blocks(v0);
            s1 = rows_from_blocks(v1);
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                uint64_t k0, k1;
                keys(j, k0, k1);
                if (!partial || live_j(rr, j)) {
                    accum16(src[j], k0, k1, s0, s1);
                    if constexpr (TEXT) count16(src[j], n_nl, n_cont);
                }
            }
        }
        fold_round<Cfg<VARIANT>::BCAST>(s0, s1, a0, a1, sk0, sk1, partial ? (int)(nb - nr * 4) : 4, lane);
    };
    // ROT: visit v of the full rounds reads round seq(v). With phi > 0 the first wr - phi visits read
    // rounds phi .. wr-1 and stash their block sums (slot v), the next phi read rounds 0 .. phi-1 into
    // the chain, and the stash is then replayed in order; visits from wr on read round v.
    constexpr bool ROT = Cfg<VARIANT>::ROT && !BW;
    const uint64_t wr = ROT ? (nr < 16 ? nr : 16) : 0;
    const uint64_t phi = (ROT && wr >= 2) ? phase % wr : 0;
    auto seq = [&](uint64_t v) -> uint64_t {
        if (!ROT || phi == 0 || v >= wr) return v;
        return v < wr - phi ? phi + v : v - (wr - phi);
    };
    // a full round's block sums: row g's lanes q == 0 hold block g's, accumulators (2k, 2k + 1)
    auto stash4 = [&](uint4 (&src)[4], uint32_t ext, uint64_t slot) {
        realign(src, ext);
        uint64_t s0 = 0, s1 = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            uint64_t k0, k1;
            keys(j, k0, k1);
            accum16(src[j], k0, k1, s0, s1);
            if constexpr (TEXT) count16(src[j], n_nl, n_cont);
        }
        s0 += dpp64<DPP_ROW_ROR4>(s0);
        s1 += dpp64<DPP_ROW_ROR4>(s1);
        s0 += dpp64<DPP_ROW_ROR8>(s0);
        s1 += dpp64<DPP_ROW_ROR8>(s1);
        if (q == 0) {
            const uint32_t at = (uint32_t)(((slot * 4 + (uint64_t)g) * 4 + (uint64_t)k) * 2);
            stash[at] = s0;
            stash[at + 1] = s1;
        }
    };
    auto replay = [&]() {
        for (uint64_t slot = 0; slot < wr - phi; ++slot) {
#pragma unroll
            for (int gg = 0; gg < 4; ++gg) {
                const uint32_t at = (uint32_t)(((slot * 4 + (uint64_t)gg) * 4 + (uint64_t)k) * 2);
                a0 = scramble1(a0 + stash[at], sk0);
                a1 = scramble1(a1 + stash[at + 1], sk1);
            }
        }
    };
    // fold visit v (a full round), replaying the stash after the window's last visit
    auto visit = [&](uint4 (&src)[4], uint32_t ext, uint64_t v) {
        if (ROT && phi != 0 && v < wr - phi) {
            stash4(src, ext, v);
        } else {
            fold4(src, ext, seq(v), false);
            if (ROT && phi != 0 && v == wr - 1) replay();
        }
    };
    // the last stripe (at len - 64, secret offset 121) is fetched up front with the first rounds
    const __amdgpu_buffer_rsrc_t rsrc_last =
        __builtin_amdgcn_make_buffer_rsrc((void*)(p + len - 64), (short)0, 64, kRsrcFlags);
    const uint4 last = bload16<false>(rsrc_last, 16u * (uint32_t)k);

    {
        // Software pipeline with a static register ring: slot d holds round r + d; the D rounds
        // (4D dwordx4 per lane) and the last stripe are all issued before the first fold, so a
        // short item (an 8 KiB chunk is 2 rounds) costs one memory round trip.
        constexpr int D = Cfg<VARIANT>::DEPTH;
        uint4 ring[D][4];
        uint32_t ext[D];
#pragma unroll
        for (int d = 0; d < D; ++d) load_round(seq((uint64_t)d), ring[d], ext[d]);
        uint64_t r = 0;
        for (; r + D <= nr; r += D) {  // every slot holds a full round
#pragma unroll
            for (int d = 0; d < D; ++d) {
                if constexpr (ROT) visit(ring[d], ext[d], r + d);
                else fold4(ring[d], ext[d], r + d, false);
                load_round(seq(r + d + D), ring[d], ext[d]);
                // keep slot d+1's arithmetic below this point: otherwise the scheduler hoists its
                // data-only adds above the refill and hipcc has to drain every load (vmcnt(0))
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        // rounds r .. nr (at most D, the last one partial) are already in slots 0 .. nr - r
#pragma unroll
        for (int d = 0; d < D; ++d) {
            if (r + d < nr) {
                if constexpr (ROT) visit(ring[d], ext[d], r + d);
                else fold4(ring[d], ext[d], r + d, false);
            } else if (r + d == nr) {
                fold4(ring[d], ext[d], r + d, true);
            }
        }
    }
    // last stripe, at len - 64, with the secret shifted to offset 121
    {
        const uint64_t w0 = ((uint64_t)last.y << 32) | last.x, w1 = ((uint64_t)last.w << 32) | last.z;
        const uint64_t k0 = w0 ^ kLastW[2 * k], k1 = w1 ^ kLastW[2 * k + 1];
        a0 += mul32x32(k0) + w1;
        a1 += mul32x32(k1) + w0;
    }
    if constexpr (TEXT) {
        // bytes [E, len) not covered by the stripes above come from the last stripe, which always
        // spans them (len - E is 1..64); `last` depends only on k, so only lanes 0..3 count it
        const uint64_t E = (nb << 10) + (ns << 6);
        const uint64_t p0 = len - 64 + 16 * (uint64_t)k;
        const uint32_t skip = E > p0 ? (uint32_t)(E - p0 < 16 ? E - p0 : 16) : 0u;
        const uint32_t w[4] = {last.x, last.y, last.z, last.w};
#ifdef OXH_DEBUG_LANES
        const uint32_t dbg_ring = n_nl;
#endif
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const int sd = (int)skip - 4 * d;
            const uint32_t m = sd <= 0 ? 0xFFFFFFFFu : (sd >= 4 ? 0u : (0xFFFFFFFFu << (8 * sd)));
            if (lane < 4) {
                n_nl += count_nl32(w[d] & m);
                n_cont += count_cont32(w[d] & m);
            }
        }
#ifdef OXH_DEBUG_LANES
        counts[2 + 3 * lane] = dbg_ring;
        counts[3 + 3 * lane] = n_nl;
        counts[4 + 3 * lane] = skip;
#endif
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            n_nl += (uint32_t)__shfl_xor((int)n_nl, off, 64);
            n_cont += (uint32_t)__shfl_xor((int)n_cont, off, 64);
        }
        if (lane == 0) {
            counts[0] = 1 + (uint64_t)n_nl;
            counts[1] = len - (uint64_t)n_cont;
        }
    }
    // merge: lane k contributes mix2Accs for accumulator pair k; sum over the quad
    uint64_t mlo = mul_fold64(a0 ^ kMrgLo[2 * k], a1 ^ kMrgLo[2 * k + 1]);
    uint64_t mhi = mul_fold64(a0 ^ kMrgHi[2 * k], a1 ^ kMrgHi[2 * k + 1]);
    mlo += dpp64<DPP_QUAD_XOR1>(mlo);
    mhi += dpp64<DPP_QUAD_XOR1>(mhi);
    mlo += dpp64<DPP_QUAD_XOR2>(mlo);
    mhi += dpp64<DPP_QUAD_XOR2>(mhi);
    if (lane == 0) {
        out[0] = avalanche_xxh3(len * P64_1 + mlo);
        out[1] = avalanche_xxh3(~(len * P64_2) + mhi);
    }
}

// K1: one wave per item. DESC = descriptor table (offsets/lens); otherwise fixed-size chunks.
// TEXT: also write (num_lines, num_chars) per item to `counts` (K1T, text metadata fused).
template <bool DESC, int VARIANT, bool TEXT>
__device__ __forceinline__ void wave_item(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ offsets,
                                          const uint64_t* __restrict__ lens, uint64_t n, uint64_t chunk,
                                          uint64_t total, uint64_t* __restrict__ out, uint64_t* __restrict__ counts) {
    __shared__ uint64_t lds_sec[24];
    // ROT: 16 rounds x 4 blocks x 8 accumulators per wave (4 waves per workgroup at most)
    __shared__ uint64_t rot_stash[Cfg<VARIANT>::ROT ? 4 * 16 * 32 : 1];
    if constexpr (Cfg<VARIANT>::KEYS_LDS) {
        if (threadIdx.x < 24) lds_sec[threadIdx.x] = kSecW[threadIdx.x];
        __syncthreads();
    }
    const int lane = threadIdx.x & 63;
    // one item per wave; launched with 1, 2 or 4 waves per workgroup (blockDim.x = 64 * waves)
    const uint64_t item = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (uint64_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (item >= n) return;
    if constexpr (Cfg<VARIANT>::STAGGER) {
        if (blockIdx.x < 2048) {
            const int steps = (int)(item & 15) * 40;  // s_sleep 1 ~ 64 clocks
            for (int t = 0; t < steps; ++t) __builtin_amdgcn_s_sleep(1);
        }
    }
    uint64_t off, len;
    if constexpr (DESC) {
        off = offsets[item];
        len = lens[item];
    } else {
        off = item * chunk;
        len = (total - off < chunk) ? total - off : chunk;
    }
    const uint8_t* p = arena + off;
    uint64_t* o = out + 2 * item;
    if (len <= 240) {
        if (lane == 0) {
            const U128 h = xxh3_lane_short(p, len);
            o[0] = h.lo;
            o[1] = h.hi;
            if constexpr (TEXT) {
                uint32_t nl = 0, cont = 0;
                for (uint64_t b = 0; b < len; ++b) {
                    nl += p[b] == 0x0A;
                    cont += (p[b] & 0xC0) == 0x80;
                }
                counts[2 * item] = 1 + (uint64_t)nl;
                counts[2 * item + 1] = len - (uint64_t)cont;
            }
        }
        return;
    }
    // byte-shifted items take the dword-aligned load path unless the last full stripe ends within 4 B
    // of the item end (then the dword after it would straddle the end and read as 0)
    const uint32_t bs = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3);
    const uint64_t nb_ = (len - 1) >> 10;
    const uint64_t E = (nb_ << 10) + ((((len - 1) - (nb_ << 10)) >> 6) << 6);
    uint64_t* stash = Cfg<VARIANT>::ROT ? rot_stash + (threadIdx.x >> 6) * (16 * 32) : nullptr;
    if (bs && len - E >= 4)
        wave_long<VARIANT, TEXT, true>(p, len, o, lane, lds_sec, TEXT ? counts + 2 * item : nullptr, bs, stash, item);
    else
        wave_long<VARIANT, TEXT, false>(p, len, o, lane, lds_sec, TEXT ? counts + 2 * item : nullptr, 0, stash, item);
}

__device__ __forceinline__ uint64_t readlane64(uint64_t x, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}

// K1R: one 16-lane row per item, four items per wave -- small items packed back to back (FastCDC
// chunks). Row g = lane/16 owns item 4w + g; inside the row q = (lane/4)%4 and k = lane%4 as in K1.
// One iteration moves every row one 1 KiB block along its own item: load j (0..3) reads 16 B at
// block + (4j+q)*64 + 16k, 256 contiguous bytes of the row's item per instruction, and the lane sums
// stripes {q, q+4, q+8, q+12}; two DPP row rotations finish the block sum inside the row and the
// row's lanes run that block's scramble for their 2 accumulators. Nothing crosses a row. K1 on such
// items issues ~290 VALU instructions per 4 KiB round -- the reduce-scatter and broadcast across rows
// and 4 chain steps per round on every lane -- and is VALU-issue bound there (SQ_ACTIVE_INST_VALU at
// the SIMDs' issue capacity, profiles/r04e_cdc_pmc.txt); here a 4 KiB iteration (one block of each
// of 4 items) takes ~138 (the loop's .s), and packed items become bound by their access pattern.
// RPI = 2 (Cfg bit 9, "K1H"): two rows (32 lanes) per item, two items per wave. Load j (0..1) reads
// 512 contiguous bytes of the item (5 lines when unaligned, against 2 x 3 for two row loads); the lane
// sums stripes {t/4, 8 + t/4} (t = lane % 32); the block sum takes one permlane16 swap more, and each
// item's chain runs once per block on its 32 lanes.
// The items of a wave run in lockstep to the longest one; a row whose item is done idles (its loads
// go to kOOB and are dropped). All rows address their items through ONE buffer descriptor (it is
// wave-uniform) over [lowest start, highest end) of the wave's items; items further apart than that
// allows (not the case in a chunk table) are hashed by one lane each (correct, slow: K1 is the shape
// for such batches). Byte-shifted items load from the dword below their start and re-align in
// registers (the shift is per lane, 0 for aligned items).
//
// FOLDED (K1F, FastCDC's second pass behind the folded walk W2, fastcdc.hip): blocks 4 .. nb-1 of an
// item whose flag is set are not read; their sums (8 u64 per block, stored by W2 at index
// (arena offset of the block) >> 10 of `sums`) are loaded instead -- by the row's quad 0, lane k the
// accumulator pair (2k, 2k + 1), the other quads contributing 0 to the row reduction -- and the chain
// scrambles them as usual. Blocks 0-3, the partial block and the last stripe come from the bytes. A
// byte-shifted item's first data block after the sums takes its w0 from a dword loaded up front.
template <bool DESC, int VARIANT, bool FOLDED = false>
__device__ __forceinline__ void rows_item(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ offsets,
                                          const uint64_t* __restrict__ lens, uint64_t n, uint64_t chunk,
                                          uint64_t total, uint64_t* __restrict__ out,
                                          const uint64_t* __restrict__ sums = nullptr,
                                          const uint8_t* __restrict__ flags = nullptr) {
    constexpr int D = Cfg<VARIANT>::DEPTH;
    constexpr bool NT = Cfg<VARIANT>::NT;
    constexpr int RPI = Cfg<VARIANT>::ROWS2 ? 2 : 1;  // 16-lane rows per item
    constexpr int LPI = 16 * RPI;                      // lanes per item
    constexpr int IPW = 4 / RPI;                       // items per wave
    constexpr int NL = 4 / RPI;                        // loads per 1 KiB block, 256 * RPI bytes each
    const int lane = threadIdx.x & 63;
    const int t = lane & (LPI - 1), k = lane & 3, st0 = t >> 2;  // the lane's stripe in load j: 4*RPI*j + st0
    const bool head = t == 0;
    const uint64_t first =
        ((uint64_t)blockIdx.x * (blockDim.x >> 6) + (uint64_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) * IPW;
    if (first >= n) return;
    const uint64_t item = first + (uint64_t)(lane / LPI);
    const bool valid = item < n;
    uint64_t off = 0, len = 0;
    if (valid) {
        if constexpr (DESC) {
            off = offsets[item];
            len = lens[item];
        } else {
            off = item * chunk;
            len = (total - off < chunk) ? total - off : chunk;
        }
    }
    const bool lng = valid && len > 240;
    const uint64_t start = reinterpret_cast<uint64_t>(arena + off);
    // loads start at the item's dword boundary, bs bytes before the item
    const uint32_t bs = (uint32_t)(start & 3);
    const uint64_t astart = start - bs;
    // the wave's long items under one descriptor: [lowest aligned start, highest end)
    uint64_t wlo = ~0ull, whi = 0;
#pragma unroll
    for (int r = 0; r < IPW; ++r) {
        const uint64_t a = readlane64(lng ? astart : ~0ull, LPI * r);
        const uint64_t e = readlane64(lng ? start + len : 0, LPI * r);
        wlo = a < wlo ? a : wlo;
        whi = e > whi ? e : whi;
    }
    if (whi != 0 && whi - wlo >= (1ull << 32) - (1ull << 20)) {
        // items too far apart for one descriptor (not a chunk table): each item's first lane hashes
        // it alone -- correct for any layout, slow; K1 (one wave per item) is the path for that
        if (valid && head) {
            const U128 h = xxh3_lane_any(arena + off, len);
            out[2 * item] = h.lo;
            out[2 * item + 1] = h.hi;
        }
        return;
    }
    uint64_t key0[NL], key1[NL];
#pragma unroll
    for (int j = 0; j < NL; ++j) {
        key0[j] = kSecW[4 * RPI * j + st0 + 2 * k];
        key1[j] = kSecW[4 * RPI * j + st0 + 2 * k + 1];
    }
    const uint64_t sk0 = kSecW[16 + 2 * k], sk1 = kSecW[16 + 2 * k + 1];
    if (whi != 0) {
        const bool act = lng;
        const uint64_t base = wlo, span = (whi - wlo + 3) & ~3ull;
        const uint32_t vb = act ? (uint32_t)(astart - base) : 0;  // < 4 GiB - 1 MiB
        // blocks followed by a scramble (< 2^32: an item below 4 TiB) and stripes of block nb
        const uint32_t nb = act ? (uint32_t)((len - 1) >> 10) : 0;
        const uint32_t ns = act ? (uint32_t)(((len - 1) - ((uint64_t)nb << 10)) >> 6) : 0;
        uint32_t B = 0;  // the wave's last iteration: its longest item's partial block
#pragma unroll
        for (int r = 0; r < IPW; ++r) {
            const uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)nb, LPI * r);
            B = x > B ? x : B;
        }
        const bool shifted = act && bs != 0;
        // pieces j < jpart of the partial block are live (stripe 4*RPI*j + st0 < ns)
        const uint32_t jpart = act && ns > (uint32_t)st0 ? (ns - (uint32_t)st0 + 4 * RPI - 1) / (4 * RPI) : 0u;
        uint64_t a0 = kInitW[2 * k], a1 = kInitW[2 * k + 1];
        // FOLDED: blocks [4, nb) of a flagged item come from `sums`
        const bool has_w = FOLDED && act && nb > 4 && flags[item] != 0;
        auto wblk = [&](uint32_t b) -> bool { return has_w && b >= 4u && b < nb; };
        // pieces j < live_n(b) of iteration b are live: NL in a full block, jpart in the partial one
        auto live_n = [&](uint32_t b) -> uint32_t {
            return wblk(b) ? 0u : (act & (b < nb)) ? (uint32_t)NL : (b == nb) ? jpart : 0u;
        };
        const __amdgpu_buffer_rsrc_t rsrc =
            __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(base), (short)0, (int)(uint32_t)span, kRsrcFlags);
        // the wave's sums under one descriptor, from the block index of its lowest start
        const uint64_t sidx0 = FOLDED ? (base - reinterpret_cast<uint64_t>(arena)) >> 10 : 0;
        const uint32_t sspan = FOLDED ? (uint32_t)(((span >> 10) + 2) * 64) : 0u;
        const __amdgpu_buffer_rsrc_t srsrc = __builtin_amdgcn_make_buffer_rsrc(
            FOLDED ? (void*)(sums + 8 * sidx0) : (void*)arena, (short)0, (int)sspan, kRsrcFlags);
        const uint32_t sv = FOLDED && act ? (uint32_t)(((off >> 10) - sidx0) * 64) + 16u * (uint32_t)t : 0u;
        // Byte-shifted items load every piece 4 bytes late: the lane then holds dwords w1..w4 of the
        // five its piece spans (w0 = the dword holding the piece's first byte) and takes w0 from the
        // previous lane's w4 (DPP row_ror:1; a row's first lane from the previous row of the item
        // through a permlane16 swap (RPI 2), or from the previous load, for load 0 from the previous
        // iteration (`carry`; before the first, one dword load). No load reads past a live piece, and
        // no extra loads are needed per iteration. v_perm_b32 then picks bytes bs..bs+3 of each dword
        // pair; an aligned item loads on time and picks bytes 4..7 (the loaded dword itself).
        const uint32_t late = shifted ? 4u : 0u;
        const uint32_t psel = 0x03020100u + 0x01010101u * (shifted ? bs : 4u);
        auto load_iter = [&](uint32_t b, uint4 (&dst)[NL]) {
            const uint32_t vo = vb + (b << 10) + 16u * (uint32_t)t + late;
            const uint32_t jn = live_n(b);
#pragma unroll
            for (int j = 0; j < NL; ++j) dst[j] = bload16<NT>(rsrc, (uint32_t)j < jn ? vo + (uint32_t)(256 * RPI * j) : kOOB);
            if constexpr (FOLDED) {
                if (wblk(b)) dst[0] = bload16<false>(srsrc, t < 4 ? sv + (b << 6) : kOOB);
            }
        };
        uint32_t carry = __builtin_amdgcn_raw_buffer_load_b32(rsrc, (shifted & head) ? vb : kOOB, 0, 0);
        // FOLDED: the dword before the partial block, for the head lane of a shifted item with sums
        const uint32_t carry_nb =
            FOLDED ? __builtin_amdgcn_raw_buffer_load_b32(rsrc, (shifted & head & has_w) ? vb + (nb << 10) : kOOB, 0, 0) : 0u;
        auto fold = [&](uint4 (&src)[NL], uint32_t b) {
            if constexpr (FOLDED) {
                if (has_w && b == nb) carry = carry_nb;
            }
            uint32_t w0s[NL];
#pragma unroll
            for (int j = 0; j < NL; ++j) {
                const uint32_t pw = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)src[j].w, 0x121, 0xf, 0xf, false);
                if constexpr (RPI == 1) {
                    w0s[j] = head ? carry : pw;
                    carry = pw;  // lane 0 of the row now holds the row's last w4
                } else {
                    // rows (0, 1) of the item: swap[0] gives row 1 row 0's values, swap[1] row 0 row 1's
                    const auto sw = __builtin_amdgcn_permlane16_swap(pw, pw, false, false);
                    w0s[j] = head ? carry : (t == 16 ? sw[0] : pw);
                    carry = sw[1];  // lane 0 of the item now holds the item's last w4 of this load
                }
            }
            const uint32_t jn = live_n(b);
            uint64_t s0 = 0, s1 = 0;
#pragma unroll
            for (int j = 0; j < NL; ++j) {
                const uint4 a = src[j];
                const uint4 d = make_uint4(__builtin_amdgcn_perm(a.x, w0s[j], psel), __builtin_amdgcn_perm(a.y, a.x, psel),
                                           __builtin_amdgcn_perm(a.z, a.y, psel), __builtin_amdgcn_perm(a.w, a.z, psel));
                if ((uint32_t)j < jn) accum16(d, key0[j], key1[j], s0, s1);
            }
            if constexpr (FOLDED) {
                if (wblk(b)) {  // W2's block sum: quad 0 holds it, the others 0
                    s0 = ((uint64_t)src[0].y << 32) | src[0].x;
                    s1 = ((uint64_t)src[0].w << 32) | src[0].z;
                }
            }
            s0 += dpp64<DPP_ROW_ROR4>(s0);
            s1 += dpp64<DPP_ROW_ROR4>(s1);
            s0 += dpp64<DPP_ROW_ROR8>(s0);
            s1 += dpp64<DPP_ROW_ROR8>(s1);
            if constexpr (RPI == 2) {
                s0 = swap16_add(s0, s0);  // the item's two rows
                s1 = swap16_add(s1, s1);
            }
            const bool full = act & (b < nb), part = act & (b == nb);
            const uint64_t t0 = a0 + s0, t1 = a1 + s1;
            const uint64_t c0 = scramble1(t0, sk0), c1 = scramble1(t1, sk1);
            a0 = full ? c0 : (part ? t0 : a0);
            a1 = full ? c1 : (part ? t1 : a1);
        };
        // the last stripe (at len - 64, secret offset 121), fetched with the first iterations
        const uint4 last = bload16<false>(rsrc, act ? vb + bs + (uint32_t)len - 64 + 16 * (uint32_t)k : kOOB);
        {
            uint4 ring[D][NL];
#pragma unroll
            for (int d = 0; d < D; ++d) load_iter((uint32_t)d, ring[d]);
            // one loop to the end, the last group's folds guarded: with a separate tail after the loop
            // hipcc copied the whole ring at loop entry (an LDS re-alignment form went 108 -> 156 VGPRs)
            for (uint32_t b = 0; b <= B; b += D) {
#pragma unroll
                for (int d = 0; d < D; ++d) {
                    if (b + d <= B) fold(ring[d], b + d);
                    load_iter(b + d + D, ring[d]);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        }
        {
            const uint64_t w0 = ((uint64_t)last.y << 32) | last.x, w1 = ((uint64_t)last.w << 32) | last.z;
            const uint64_t k0 = w0 ^ kLastW[2 * k], k1 = w1 ^ kLastW[2 * k + 1];
            a0 += mul32x32(k0) + w1;
            a1 += mul32x32(k1) + w0;
        }
        uint64_t mlo = mul_fold64(a0 ^ kMrgLo[2 * k], a1 ^ kMrgLo[2 * k + 1]);
        uint64_t mhi = mul_fold64(a0 ^ kMrgHi[2 * k], a1 ^ kMrgHi[2 * k + 1]);
        mlo += dpp64<DPP_QUAD_XOR1>(mlo);
        mhi += dpp64<DPP_QUAD_XOR1>(mhi);
        mlo += dpp64<DPP_QUAD_XOR2>(mlo);
        mhi += dpp64<DPP_QUAD_XOR2>(mhi);
        if (act && head) {
            out[2 * item] = avalanche_xxh3(len * P64_1 + mlo);
            out[2 * item + 1] = avalanche_xxh3(~(len * P64_2) + mhi);
        }
    }
    if (valid && !lng && head) {
        const U128 h = xxh3_lane_short(arena + off, len);
        out[2 * item] = h.lo;
        out[2 * item + 1] = h.hi;
    }
}

#ifdef OXH_PROBE_FOLD
// K1F: FastCDC chunk digests behind the folded walk (rows_item FOLDED), K1R's shape (variant 264). Probe
// build only: measured and not kept (DESIGN §4 "W2").
__global__ __launch_bounds__(128) void xxh3_rows_fold_kernel(const uint8_t* __restrict__ arena,
                                                             const uint64_t* __restrict__ offsets,
                                                             const uint64_t* __restrict__ lens, uint64_t n,
                                                             uint64_t* __restrict__ out, const uint64_t* __restrict__ sums,
                                                             const uint8_t* __restrict__ flags) {
    rows_item<true, 264, true>(arena, offsets, lens, n, 0, 0, out, sums, flags);
}
#endif

template <bool DESC, int VARIANT>
__global__ __launch_bounds__(256) void xxh3_wave_kernel(const uint8_t* __restrict__ arena,
                                                        const uint64_t* __restrict__ offsets,
                                                        const uint64_t* __restrict__ lens, uint64_t n,
                                                        uint64_t chunk, uint64_t total,
                                                        uint64_t* __restrict__ out) {
    if constexpr (Cfg<VARIANT>::ROWS) rows_item<DESC, VARIANT>(arena, offsets, lens, n, chunk, total, out);
    else wave_item<DESC, VARIANT, false>(arena, offsets, lens, n, chunk, total, out, nullptr);
}

// K1T: K1 + text metadata counts in the same HBM pass (descriptor tables only).
template <int VARIANT>
__global__ __launch_bounds__(256) void xxh3_text_wave_kernel(const uint8_t* __restrict__ arena,
                                                             const uint64_t* __restrict__ offsets,
                                                             const uint64_t* __restrict__ lens, uint64_t n,
                                                             uint64_t* __restrict__ out,
                                                             uint64_t* __restrict__ counts) {
    wave_item<true, VARIANT, true>(arena, offsets, lens, n, 0, 0, out, counts);
}

// K1s: one lane per item (any length; intended for short items).
__global__ __launch_bounds__(256) void xxh3_lane_kernel(const uint8_t* __restrict__ arena,
                                                        const uint64_t* __restrict__ offsets,
                                                        const uint64_t* __restrict__ lens, uint64_t n,
                                                        uint64_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const U128 h = xxh3_lane_any(arena + offsets[i], lens[i]);
    out[2 * i] = h.lo;
    out[2 * i + 1] = h.hi;
}

// K2 helper: combined = XXH3-128(content LE16 || metadata LE16) -- the 17..128 path at len 32.
__global__ __launch_bounds__(256) void xxh3_combined_kernel(const uint64_t* __restrict__ content,
                                                            const uint64_t* __restrict__ meta, uint64_t n,
                                                            uint64_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t c0 = content[2 * i], c1 = content[2 * i + 1];
    const uint64_t m0 = meta[2 * i], m1 = meta[2 * i + 1];
    // mix32B(acc, in, in + 16, secret): a = (c0, c1), b = (m0, m1)
    uint64_t lo = 32 * P64_1, hi = 0;
    lo += mul_fold64(c0 ^ S64(0), c1 ^ S64(8));
    lo ^= m0 + m1;
    hi += mul_fold64(m0 ^ S64(16), m1 ^ S64(24));
    hi ^= c0 + c1;
    const U128 h = finish_mid(lo, hi, 32);
    out[2 * i] = h.lo;
    out[2 * i + 1] = h.hi;
}

// K1L phase 1: block sums. Wave w folds blocks [4w, 4w+4) of the buffer (only blocks < nb, i.e.
// those followed by a scramble) and writes each block's 8 accumulator sums (64 B) to `sums`.
template <bool ALIGNED>
__global__ __launch_bounds__(256) void xxh3_blocksum_kernel(const uint8_t* __restrict__ p, uint64_t nb,
                                                            uint64_t* __restrict__ sums) {
    const int lane = threadIdx.x & 63;
    const uint64_t w = (uint64_t)blockIdx.x * 4 + (uint64_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nwaves = (nb + 3) >> 2;
    if (w >= nwaves) return;
    const int g = lane >> 4, q = (lane >> 2) & 3, k = lane & 3;
    const uint64_t b = 4 * w + g;
    uint64_t s0 = 0, s1 = 0;
    if (b < nb) {
        const uint8_t* lp = p + b * 1024 + (uint64_t)q * 64 + (uint64_t)k * 16;
        uint4 d[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) d[j] = load16<ALIGNED>(lp + j * 256);
#pragma unroll
        for (int j = 0; j < 4; ++j)
            accum16(d[j], kSecW[4 * j + q + 2 * k], kSecW[4 * j + q + 2 * k + 1], s0, s1);
    }
    s0 += dpp64<DPP_ROW_ROR4>(s0);
    s1 += dpp64<DPP_ROW_ROR4>(s1);
    s0 += dpp64<DPP_ROW_ROR8>(s0);
    s1 += dpp64<DPP_ROW_ROR8>(s1);
    if (b < nb && q == 0) {
        // block b's sums: 8 u64, lane k stores (2k, 2k+1)
        uint64_t* dst = sums + b * 8 + 2 * k;
        dst[0] = s0;
        dst[1] = s1;
    }
}

// K1L phase 2: the serial chain over nb block sums, then the tail and the merge -- one wave per
// buffer, up to kChainJobs buffers per launch (so the chains of many large files run concurrently on
// different CUs). Lanes 0..7 each own one accumulator; block sums stream in GROUP steps at a time
// with the next group's loads in flight while the current group is chained.
__global__ __launch_bounds__(64) void xxh3_chain_kernel(ChainBatch batch) {
    constexpr int GROUP = 256;
    // the chain is one latency-bound wave per file: give it issue priority over any wave of a
    // concurrent kernel (chunking, K1) that lands on the same SIMD
    __builtin_amdgcn_s_setprio(3);
    const ChainJob job = batch.job[blockIdx.x];
    const uint8_t* __restrict__ p = job.p;
    const uint64_t len = job.len;
    const uint64_t* __restrict__ sums = job.sums;
    const int lane = threadIdx.x;
    const int i = lane & 7;
    const bool partial = (job.flags & kChainPartial) != 0;
    const uint64_t nb = partial ? len >> 10 : (len - 1) >> 10;
    // The chain acc <- scramble(acc + S_b) is carried as x = acc + S_b in 32-bit halves so that the
    // critical path per step is shift -> xor -> v_mad_u64_u32 (which also adds S_{b+1}) -> add:
    //   y = x ^ (x >> 47) ^ key;  x' = y * P32_1 + S_{b+1}
    //   lo(x') = lo(yl * P + S), hi(x') = hi(yl * P + S) + yh * P   (yh * P off the critical path)
    const uint64_t sk = kSecW[16 + i];
    const uint32_t kl = (uint32_t)sk, kh = (uint32_t)(sk >> 32);
    uint64_t acc = (job.flags & kChainResume) ? job.state[i] : kInitW[i];
    auto step = [&](uint32_t& xl, uint32_t& xh, uint64_t s_next) {
        uint32_t yl;  // one 3-input xor (bitop3 0x96) on the critical path; hipcc emits two xors
        asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(yl) : "v"(xl), "v"(kl), "v"(xh >> 15));
        const uint32_t yh = xh ^ kh;
        uint32_t t = yh * P32_1;  // v_mul_lo_u32, in parallel with the mad below
        asm("" : "+v"(t));        // keep hipcc from folding it into a second, dependent v_mad_u64_u32
        const uint64_t m = (uint64_t)yl * P32_1 + s_next;
        xh = (uint32_t)(m >> 32) + t;
        xl = (uint32_t)m;
    };
    if (nb > 0) {
        uint64_t x0 = acc + sums[i];
        uint32_t xl = (uint32_t)x0, xh = (uint32_t)(x0 >> 32);
        uint64_t b = 1;  // x holds acc + S_0; each step scrambles and adds the next block's sum
        // Block sums reach the chain through LDS: all 64 lanes load the next group of GROUP steps
        // (GROUP x 64 B) while lanes 0-7 run the current group's chain from LDS. Loading the sums in
        // the chain lanes themselves let hipcc re-load each one from memory right before its step
        // (the values are invariant), which put an L1 round trip on every step of the chain.
        __shared__ uint64_t buf[2][GROUP * 8];
        constexpr int PER = GROUP * 8 / 64;  // sums per lane per group
        const uint64_t ngroups = (nb - 1) / GROUP;
        uint64_t r[PER];
        auto issue = [&](uint64_t g) {
#pragma unroll
            for (int k = 0; k < PER; ++k) {
                const uint64_t e = (uint64_t)k * 64 + (uint64_t)lane;  // element of the group
                r[k] = sums[(1 + g * GROUP + e / 8) * 8 + (e & 7)];
            }
        };
        auto commit = [&](int sb) {
#pragma unroll
            for (int k = 0; k < PER; ++k) buf[sb][k * 64 + lane] = r[k];
            __syncthreads();
        };
        if (ngroups > 0) {
            issue(0);
            commit(0);
            for (uint64_t gi = 0; gi < ngroups; ++gi) {
                const int sb = (int)(gi & 1);
                if (gi + 1 < ngroups) issue(gi + 1);
                if (lane < 8) {
                    // LDS reads a batch of B steps ahead of the chain (sched_barrier keeps hipcc from
                    // sinking them to their use, which exposed the LDS latency every other step)
                    constexpr int B = 32;
                    uint64_t va[B], vb[B];
#pragma unroll
                    for (int t = 0; t < B; ++t) va[t] = buf[sb][t * 8 + i];
#pragma unroll
                    for (int t0 = 0; t0 < GROUP; t0 += 2 * B) {
#pragma unroll
                        for (int t = 0; t < B; ++t) vb[t] = buf[sb][(t0 + B + t) * 8 + i];
                        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                        for (int t = 0; t < B; ++t) step(xl, xh, va[t]);
                        if (t0 + 2 * B < GROUP) {
#pragma unroll
                            for (int t = 0; t < B; ++t) va[t] = buf[sb][(t0 + 2 * B + t) * 8 + i];
                        }
                        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                        for (int t = 0; t < B; ++t) step(xl, xh, vb[t]);
                    }
                }
                if (gi + 1 < ngroups) commit(sb ^ 1);
            }
            b = 1 + ngroups * GROUP;
        }
        for (; b < nb; ++b) step(xl, xh, sums[b * 8 + i]);
        step(xl, xh, 0);  // the last full block's scramble
        acc = ((uint64_t)xh << 32) | xl;
    }
    if (partial) {  // a piece of a huge file: hand the accumulators to the next piece
        if (lane < 8) job.state[i] = acc;
        return;
    }
    // partial block stripes + last stripe: lane i owns accumulator i here (scalar per lane)
    const uint64_t ns = ((len - 1) - (nb << 10)) >> 6;
    const uint8_t* pb = p + (nb << 10);
    for (uint64_t s = 0; s < ns; ++s) {
        const uint64_t v = ld64u(pb + s * 64 + 8 * i);
        const uint64_t vs = ld64u(pb + s * 64 + 8 * (i ^ 1));
        acc += mul32x32(v ^ kSecW[s + i]) + vs;
    }
    {
        const uint8_t* ls = p + len - 64;
        const uint64_t v = ld64u(ls + 8 * i);
        const uint64_t vs = ld64u(ls + 8 * (i ^ 1));
        acc += mul32x32(v ^ kLastW[i]) + vs;
    }
    // merge: pairs (2m, 2m+1) live in lanes (2m, 2m+1)
    const uint64_t partner = ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)acc, 1, 64)) |
                             ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(acc >> 32), 1, 64) << 32);
    uint64_t mlo = 0, mhi = 0;
    if ((i & 1) == 0) {
        mlo = mul_fold64(acc ^ kMrgLo[i], partner ^ kMrgLo[i + 1]);
        mhi = mul_fold64(acc ^ kMrgHi[i], partner ^ kMrgHi[i + 1]);
    }
    // sum lanes 0,2,4,6
#pragma unroll
    for (int off = 1; off < 8; off <<= 1) {
        const uint64_t ol = ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)mlo, off, 64)) |
                            ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(mlo >> 32), off, 64) << 32);
        const uint64_t oh = ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)mhi, off, 64)) |
                            ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(mhi >> 32), off, 64) << 32);
        mlo += ol;
        mhi += oh;
    }
    if (lane == 0) {
        const uint64_t tl = job.total_len ? job.total_len : len;  // the whole file's length
        job.out[0] = avalanche_xxh3(tl * P64_1 + mlo);
        job.out[1] = avalanche_xxh3(~(tl * P64_2) + mhi);
    }
}

// util::fs::is_utf8 (util/fs.rs:652-668): the first min(len, 4096) bytes are valid UTF-8, or the
// first error is a multi-byte sequence cut off by the end of that prefix (Utf8Error::error_len() ==
// None); an empty file is UTF-8. Restates core::str::from_utf8's validation (ASCII, C2-DF + 1,
// E0 A0-BF, E1-EC/EE-EF 80-BF, ED 80-9F, F0 90-BF, F1-F3 80-BF, F4 80-8F, then 80-BF continuations).
// One lane per item, 16-byte loads; runs beside K1T on the staged bytes, so the data-type sniff
// add.rs:809-810 makes (file_mime_type -> is_utf8) needs no third read of the file.
__device__ __forceinline__ bool utf8_second_ok(uint32_t lead, uint32_t b) {
    if (lead == 0xE0) return b >= 0xA0 && b <= 0xBF;
    if (lead == 0xED) return b >= 0x80 && b <= 0x9F;
    if (lead == 0xF0) return b >= 0x90 && b <= 0xBF;
    if (lead == 0xF4) return b >= 0x80 && b <= 0x8F;
    return (b & 0xC0) == 0x80;
}

__device__ int32_t utf8_prefix_ok(const uint8_t* __restrict__ p, uint64_t len) {
    const uint32_t n = (uint32_t)(len < 4096 ? len : 4096);
    uint32_t need = 0, width = 0, lead = 0;  // continuation bytes still expected for the open sequence
    for (uint32_t base = 0; base < n; base += 16) {
        uint32_t w[4] = {0, 0, 0, 0};
        if (base + 16 <= n) {
            uint4 v;
            __builtin_memcpy(&v, p + base, 16);
            w[0] = v.x;
            w[1] = v.y;
            w[2] = v.z;
            w[3] = v.w;
        } else {
#pragma unroll
            for (int j = 0; j < 16; ++j)
                if (base + j < n) w[j >> 2] |= (uint32_t)p[base + j] << (8 * (j & 3));
        }
        const uint32_t m = n - base < 16 ? n - base : 16;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            if ((uint32_t)j >= m) break;
            const uint32_t b = (w[j >> 2] >> (8 * (j & 3))) & 0xFF;
            if (need) {
                const bool ok = (need == width - 1) ? utf8_second_ok(lead, b) : ((b & 0xC0) == 0x80);
                if (!ok) return 0;
                --need;
                continue;
            }
            if (b < 0x80) continue;
            if (b >= 0xC2 && b <= 0xDF) width = 2;
            else if (b >= 0xE0 && b <= 0xEF) width = 3;
            else if (b >= 0xF0 && b <= 0xF4) width = 4;
            else return 0;  // continuation byte, C0, C1 or F5-FF: error_len Some(1)
            lead = b;
            need = width - 1;
        }
    }
    return 1;  // valid, or a sequence still open at the end of the prefix (error_len None)
}

__global__ __launch_bounds__(256) void utf8_prefix_kernel(const uint8_t* __restrict__ arena,
                                                          const uint64_t* __restrict__ offsets,
                                                          const uint64_t* __restrict__ lens, uint64_t n,
                                                          int32_t* __restrict__ flags) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    flags[i] = utf8_prefix_ok(arena + offsets[i], lens[i]);
}

// Text counts of one large buffer without hashing it (oversize text files, whose digest comes from
// K1L): counts[0] += newlines, counts[1] += UTF-8 continuation bytes (caller zeroes counts first).
__global__ __launch_bounds__(256) void text_count_kernel(const uint8_t* __restrict__ p, uint64_t len,
                                                         unsigned long long* __restrict__ counts) {
    uint32_t nl = 0, cont = 0;
    const uint64_t n16 = len / 16;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
        uint4 d;
        __builtin_memcpy(&d, p + 16 * i, 16);
        count16(d, nl, cont);
    }
    if (blockIdx.x == 0 && threadIdx.x < (len & 15)) {
        const uint8_t b = p[16 * n16 + threadIdx.x];
        nl += b == 0x0A;
        cont += (b & 0xC0) == 0x80;
    }
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        nl += (uint32_t)__shfl_xor((int)nl, off, 64);
        cont += (uint32_t)__shfl_xor((int)cont, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&counts[0], (unsigned long long)nl);
        atomicAdd(&counts[1], (unsigned long long)cont);
    }
}

__global__ void text_count_finish_kernel(const unsigned long long* __restrict__ raw, CountFix fix,
                                        uint64_t* __restrict__ counts) {
    const int q = threadIdx.x;
    if (q < fix.n) {
        counts[2 * fix.j[q]] = 1 + raw[2 * q];
        counts[2 * fix.j[q] + 1] = fix.len[q] - raw[2 * q + 1];
    }
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void fill_splitmix_kernel(uint64_t* __restrict__ dst, uint64_t nwords,
                                                            uint64_t seed) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nwords; w += stride)
        dst[w] = splitmix64(seed + (w + 1) * 0x9E3779B97F4A7C15ULL);
}

__global__ void fill_splitmix_tail_kernel(uint8_t* __restrict__ dst, uint64_t word, uint64_t nbytes,
                                          uint64_t seed) {
    const uint64_t v = splitmix64(seed + (word + 1) * 0x9E3779B97F4A7C15ULL);
    for (uint64_t j = 0; j < nbytes; ++j) dst[j] = (uint8_t)(v >> (8 * j));
}

// explicit instantiations used by the host runtime (variants: see Cfg). The shipped library carries
// the shapes the dispatch picks (8, 72, 104, 264) and the fallback 0; the experiments that lost their
// A/Bs only in the probe build (tools/build_probe_lib.sh, -DOXH_PROBE_VARIANTS).
template __global__ void xxh3_wave_kernel<true, 0>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<false, 0>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<true, 8>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<false, 8>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<true, 72>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<false, 72>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<true, 104>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<false, 104>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<true, 264>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<false, 264>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
#ifdef OXH_PROBE_VARIANTS
template __global__ void xxh3_wave_kernel<true, 1>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<false, 1>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<true, 2>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<false, 2>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<true, 4>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<false, 4>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<true, 12>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<false, 12>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<true, 40>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<false, 40>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<true, 64>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<false, 64>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<true, 74>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<false, 74>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<true, 256>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<false, 256>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<true, 260>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<false, 260>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<true, 768>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<false, 768>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<true, 772>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<false, 772>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<true, 776>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<false, 776>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<true, 1032>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<false, 1032>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<true, 1024>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
template __global__ void xxh3_wave_kernel<false, 1024>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
#endif
template __global__ void xxh3_text_wave_kernel<72>(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t*, uint64_t*);
template __global__ void xxh3_blocksum_kernel<true>(const uint8_t*, uint64_t, uint64_t*);
template __global__ void xxh3_blocksum_kernel<false>(const uint8_t*, uint64_t, uint64_t*);

}  // namespace oxh
