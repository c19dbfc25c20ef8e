// oxen_amd/csrc/fastcdc.hip -- FastCDC v2020 content-defined chunk boundaries on gfx950
// (block-level dedup), and the chunk digests behind them.
//
// Reference: experiments/block-level-dedup/src/chunker/fastcdchunker.rs:83-98 calls
// `fastcdc::v2020::FastCDC::new(&content, 4096, chunk, 2 * chunk)` (crate fastcdc 3.2.1, not
// vendored) and names every chunk by the decimal xxh3_128 of its bytes. The crate's cut_gear rolls
// a 64-bit gear hash `h = (h << 1) + GEAR[b]` from index `min` of every chunk and cuts at the first
// position whose hash has no bit of mask_s (before `avg`) or mask_l (after it); else at `max`.
//
// The walk is serial per file (each cut decides where the next chunk's hash starts). The GPU
// formulation splits it into three kernels:
//   F1 cdc_scan_kernel    chip-wide, one wave per section (>= 512 KiB), lane-major: lane l rolls
//                         the gear hash through unit l (section / 64 bytes) from 48 bytes before it,
//                         so it has the FULL-window hash at every byte (all mask bits are below bit
//                         48: the hash of position p is a function of b[p-47 .. p]), and records a
//                         position-ordered list of candidate 16-byte groups per unit (a position with
//                         none of the bits both masks share clear).
//   F2 cdc_walk_kernel    one lane per section: a speculative walk that starts 6 max-sized chunks
//                         before the section (by then it has almost surely met the true walk) and
//                         cuts chunks from the candidate lists until it passes the section end,
//                         recording the starts inside the section. The first 47 positions after a chunk's `min` see a hash
//                         that started from 0 (truncated window); the walk recomputes those from the
//                         bytes, everything later comes from the candidates.
//   F3 stitch             cdc_check_kernel (one lane per section): the last start section i-1's
//                         walk recorded is the true entry of section i; if section i's own walk
//                         produced that start too, the rest of its list is the true walk (cut
//                         points depend only on the chunk start). cdc_fixup_kernel re-walks the
//                         sections where that failed; a prefix sum and cdc_emit_kernel write the
//                         chunk table.
// Then K1 hashes every chunk (oxh_xxh3_128_batch_device).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <map>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/oxen_hash.h"
#include "fastcdc_gear.h"
#include "scratch.hpp"
#include "xxh3_device.hpp"

namespace oxh {

int set_error(int code, const std::string& msg);  // capi_context.hip: oxh_last_error() text
int k1_packed(const void* d_arena, const uint64_t* d_offsets, const uint64_t* d_lens, uint64_t n, uint64_t* d_out,
              uint64_t mean_len, hipStream_t st);  // capi_dispatch.hip
__global__ void xxh3_rows_fold_kernel(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t*,
                                      const uint64_t*, const uint8_t*);  // xxh3_kernels.hip (K1F)

// fastcdc::v2020::MASKS, indexed by the number of one bits (entries 0..4 are padding)
static constexpr uint64_t kCdcMasks[26] = {
    0, 0, 0, 0, 0,
    0x0000000001804110ULL, 0x0000000001803110ULL, 0x0000000018035100ULL, 0x0000001800035300ULL,
    0x0000019000353000ULL, 0x0000590003530000ULL, 0x0000d90003530000ULL, 0x0000d90103530000ULL,
    0x0000d90303530000ULL, 0x0000d90313530000ULL, 0x0000d90f03530000ULL, 0x0000d90303537000ULL,
    0x0000d90703537000ULL, 0x0000d90707537000ULL, 0x0000d91707537000ULL, 0x0000d91747537000ULL,
    0x0000d91767537000ULL, 0x0000d93767537000ULL, 0x0000d93777537000ULL, 0x0000d93777577000ULL,
    0x0000db3777577000ULL,
};

constexpr uint32_t kSecDefault = 512 * 1024;  // minimum section bytes (F1 wave / F2 lane unit)
constexpr int kHashSpan = 47;          // positions after a chunk's start index with a truncated window
constexpr uint64_t kXStaticLds = 256 * 8;  // the X kernels' static LDS (their gear table), beside the dynamic lists
constexpr int kEntryShift = 47;        // candidate entry: group index (17 bits: units up to 2 MiB) << 47 | hash
constexpr uint64_t kEntryHash = (1ull << kEntryShift) - 1;

struct CdcParams {
    uint64_t min, avg, max;
    uint64_t mask_s, mask_l;
    uint64_t sec;      // section bytes: a multiple of 8 KiB (F1 wave / F2 lane unit)
    uint64_t unit;     // sec / 64: the candidate list unit (F1 lane)
    uint64_t warmup;   // bytes a speculative walk runs before its section (unrecorded)
    uint32_t cap;      // candidate entries stored per unit
    uint32_t speccap;  // speculative chunk starts stored per section
};

// One recorded candidate group: its entry (group index in the unit << 47 | the full-window hash
// before its first byte mod 2^47; bit 47 and up never reach a masked bit once the walk shifts it, so
// 47 bits suffice) and its 16 bytes (the walk resolves exact flags from these), in one 32-byte record:
// F1's two stores and the walk's two loads of a candidate touch one cache line, not one in each of
// two arrays.
// The first record of a unit's list also carries the unit's true candidate count in `n` (> cap: the
// list was truncated and the walk scans the rest of the unit's bytes), so a walk entering a unit
// gets the count and the first candidate from one line.
struct alignas(16) CandRec {
    uint64_t e;
    uint64_t n;  // record 0 of a unit: the unit's count; unused in the others
    uint4 b;
};

struct CdcFiles {
    const uint8_t* arena;
    const uint64_t* foff;      // [n] arena offset of each file
    const uint64_t* flen;      // [n]
    const uint64_t* sec_base;  // [n+1] first global section of each file
    const uint32_t* sec_file;  // [n_sec] file of each section
    CandRec* cand;             // [n_sec * 64 * cap] candidate groups per unit, in position order
    uint64_t* cand_occ;        // [n_sec] bit u: unit u of the section has a non-empty list
    uint32_t* spec;            // [n_sec * speccap] speculative starts, relative to section start
    uint32_t* spec_cnt;        // [n_sec]
};

__device__ __forceinline__ uint64_t gear_of(const uint64_t* __restrict__ g, uint32_t b) { return g[b]; }

// DPP wave_shr:1 (GFX9): lane l gets x from lane l-1; lane 0 keeps `old`
__device__ __forceinline__ uint32_t wave_shr1(uint32_t x, uint32_t old) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)x, 0x138, 0xf, 0xf, false);
}
// (a & b) | c in one VALU op
__device__ __forceinline__ uint32_t and_or(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(b), "v"(c));
    return r;
}
__device__ __forceinline__ uint32_t min_u32(uint32_t a, uint32_t b) { return a < b ? a : b; }
// min of three: the backend forms v_min3_u32 from the nested umin. (An inline-asm v_min3 made the
// compiler put an `s_nop 0` between every two asm blocks -- it cannot see their hazards -- one wasted
// issue slot per 4 bytes in F1, ~5 % of its issue-bound loop.)
__device__ __forceinline__ uint32_t min3_u32(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_elementwise_min(__builtin_elementwise_min(a, b), c);
}

// 16 bytes at p[pos .. pos+16) of a file of length flen as four little-endian words (zeros past the
// end): one unaligned global_load_dwordx4 (gfx950 runs in unaligned-access mode) instead of 16
// dependent byte loads -- the walk's latency is made of these. Not a buffer load: every lane of the
// walk has its own address, and a buffer resource built from a per-lane pointer is not wave-uniform,
// so the compiler wrapped each such load in a readfirstlane loop that issued it once per lane (64x;
// the walk took 3.7 ms of C5 at 8 KiB chunks with it).
__device__ __forceinline__ uint4 load16_file(const uint8_t* __restrict__ fbase, uint64_t pos, uint64_t flen) {
    if (pos >= flen) return make_uint4(0, 0, 0, 0);
    if (flen - pos >= 16) {
        typedef unsigned int u32x4u __attribute__((ext_vector_type(4), aligned(1)));
        const u32x4u v = *(const u32x4u*)(fbase + pos);
        return make_uint4(v.x, v.y, v.z, v.w);
    }
    uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 16; ++j)
        if (pos + (uint64_t)j < flen) w[j >> 2] |= (uint32_t)fbase[pos + j] << (8 * (j & 3));
    return make_uint4(w[0], w[1], w[2], w[3]);
}
__device__ __forceinline__ uint32_t byte_of(const uint4& v, int j) {
    const uint32_t w = j < 4 ? v.x : j < 8 ? v.y : j < 12 ? v.z : v.w;
    return (w >> (8 * (j & 3))) & 0xFF;
}

// ---------------------------------------------------------------- F1: candidates
// Lane-major scan. A section of S bytes is split into 64 list units of U = S/64 bytes; lane l owns
// unit l and rolls ONE hash through it, starting from the 48 bytes before the unit (warm-up; only
// the last 48 bytes reach the masked bits, so the rolled hash is the full-window hash from the unit's
// first byte on). Per byte: one v_perm_b32 (the LDS address: byte << 8 | copy offset), one
// ds_read_b64, one v_lshl_add_u64, one AND and a share of a v_min3 -- against ~6.4 VALU per byte for
// the wave-cooperative form this replaces, which rolled every byte twice (the lane-local hash, then
// again from the carry of the three lanes before it).
//
// The bytes reach the lanes through LDS without a VGPR round trip: a round is 128 B of every unit;
// 8 `buffer_load_dwordx4 ... lds` per round (lanes 8m..8m+7 of DMA k fetch the whole 128-B line of
// unit 8k+m, so every line is fetched once, coalesced) land unit r's bytes at slot + 128 r, and lane
// r reads them back with 8 ds_read_b128. The DMA lanes fetch their pieces rotated (piece q of unit r
// at position (q + (r >> 1)) & 7 of its line) so that the 16 lanes of every ds_read_b128 group cover
// the 64 banks exactly once. The gear table is stored 32 times (entry k of copy c at byte 256 k + 8 c,
// lane l reads copy l % 32): the 32 lanes of a ds_read_b64 group never share a bank.
// LDS: 64 KiB table + one 8 KiB slot per wave (the round being rolled sits in VGPRs while the next
// round's DMA is in flight): 160 KiB at 12 waves per workgroup. tools/cdc_segment_probe.hip has the variants this was chosen from.
//
// Candidates: a lane records a 16-byte group of its unit when one of its positions has none of the
// bits both masks share (offset in the unit, the hash before the group, its 16 bytes); the walk
// resolves exact mask_s / mask_l flags from those. Lists are per unit, in position order.
//
// SH: the whole hash runs 16 bits to the left (table entries GEAR << 16, masks << 16; only bits below
// 48 matter). When the bits both masks share are all >= 16 they then sit in the high 32-bit word and
// the per-byte test is one AND; otherwise (avg < ~2 KiB) the low word is tested too (v_and_or).
// 12 waves per workgroup: the 64 KiB table + 12 x 8 KiB slots fill the 160 KiB of LDS, 3 waves per
// SIMD (119 VGPRs) instead of 2. The roll is one dependent v_lshl_add_u64 chain per lane, so the
// third wave's chain fills issue slots (C5 at 8 KiB: F1 26.6 vs 28.2 ms with 8 waves, r02). 16 waves
// with 64-byte rounds (4 KiB slots, half-line DMA) measured far slower (73 vs 52 ms end to end).
// OXH_CDC_SCAN_WAVES=8 selects the 8-wave form for A/B.
constexpr int kScanWaves = 12;
#ifndef OXH_SCAN_DMA_AUX
#define OXH_SCAN_DMA_AUX 2
#endif
constexpr int kScanDmaAux = OXH_SCAN_DMA_AUX;  // cache policy of the scan's LDS-DMA loads (2 = nt)

template <bool SH, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void cdc_scan_kernel(CdcFiles f, CdcParams prm, uint64_t n_sec) {
    // one LDS block: the table at address 0 (a gather address is then a single v_perm), slots after it
    __shared__ __attribute__((aligned(16))) uint64_t lds[256 * 32 + WAVES * 1024];
    for (int i = threadIdx.x; i < 256 * 32; i += blockDim.x) lds[i] = kGear[i >> 5] << (SH ? 16 : 0);
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint4* const slot = (uint4*)(lds + 256 * 32) + w * 512;
    const uint64_t sec = (uint64_t)blockIdx.x * WAVES + (uint64_t)w;
    if (sec >= n_sec) return;
    const uint32_t file = f.sec_file[sec];
    const uint64_t flen = f.flen[file];
    const uint64_t sec_start = (sec - f.sec_base[file]) * prm.sec;
    const uint32_t sec_len = (uint32_t)(flen - sec_start < prm.sec ? flen - sec_start : prm.sec);
    const uint8_t* __restrict__ base = f.arena + f.foff[file] + sec_start;
    const uint32_t unit = (uint32_t)prm.unit, rounds = unit / 128;
    const uint32_t us = (uint32_t)lane * unit;  // this lane's unit, section-relative
    // the resource covers the 48 bytes before the section (none at a file start) and every whole
    // 16-byte piece of the section: loads past it return zeros without touching memory
    const uint32_t pre = sec_start > 0 ? 48u : 0u, full16 = sec_len & ~15u;
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void*)(base - pre), (short)0, (int)(pre + full16), 0x00020000);
    const uint64_t mask_s = prm.mask_s << (SH ? 16 : 0), mask_l = prm.mask_l << (SH ? 16 : 0);
    const uint64_t common = mask_s & mask_l;
    const uint32_t ch = (uint32_t)(common >> 32), cl = (uint32_t)common;  // SH: cl == 0 (host checks)
    const uint32_t copy_off = (uint32_t)(lane & 31) * 8;
    const char* const tab = (const char*)lds;
    auto gear = [&](uint32_t word, int j) -> uint64_t {
        const uint32_t a = __builtin_amdgcn_perm(word, copy_off, 0x0c0c0000u | ((4u + (uint32_t)j) << 8));
        return *(const uint64_t*)(tab + a);
    };
    const uint64_t ubase = sec * 64 + (uint64_t)lane;  // global unit index
    CandRec* __restrict__ out_c = f.cand + ubase * prm.cap;
    uint32_t count = 0;  // per lane

    // warm-up over the 48 bytes before the unit (lane 0 at a file start: none, the hash starts at 0)
    uint64_t h = 0;
    {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        uint32_t wv[12];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, pre + us - 48 + 16 * k, 0, 0);
            wv[4 * k] = v.x, wv[4 * k + 1] = v.y, wv[4 * k + 2] = v.z, wv[4 * k + 3] = v.w;
        }
#pragma unroll
        for (int i = 0; i < 12; ++i)
#pragma unroll
            for (int b = 0; b < 4; ++b) h = (h << 1) + gear(wv[i], b);
        if (pre + us < 48) h = 0;
    }
    // round t of every unit into this wave's slot (DMA k, lane 8m + j: unit 8k + m, rotated piece)
    const int dm = lane >> 3, dj = lane & 7;
    // the round moves the resource (SGPR arithmetic: its base by 128 B, its size down by as much) rather
    // than the 8 per-lane offsets (8 VALU adds per round); the whole offset stays in the VGPR operand,
    // so the range check sees it: a piece at or past the section's last whole 16 bytes reads zeros
    uint32_t voff[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t r = 8 * k + dm;
        voff[k] = pre + r * unit + 16 * ((uint32_t)(dj - (int)((r >> 1) & 7)) & 7);
    }
    auto dma_round = [&](uint32_t t) {
        // wave-uniform by construction; readfirstlane keeps the compiler from treating the resource
        // as per-lane (which would wrap every DMA in a readfirstlane loop)
        const int left = __builtin_amdgcn_readfirstlane((int)(pre + full16 > t * 128 ? pre + full16 - t * 128 : 0u));
        const uint64_t a = (uint64_t)(base - pre) + (uint64_t)t * 128;
        const uint64_t au = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a) |
                            ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32)) << 32);
        const __amdgpu_buffer_rsrc_t rt = __builtin_amdgcn_make_buffer_rsrc((void*)au, (short)0, left, 0x00020000);
#pragma unroll
        for (int k = 0; k < 8; ++k)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rt, (__attribute__((address_space(3))) void*)(slot + 64 * k), 16, voff[k],
                                                     0, 0, kScanDmaAux);
    };
    dma_round(0);
    const int rot = (lane >> 1) & 7;
    // the round (if any) whose 128 B hold the section's partial last 16 bytes, for this lane
    const uint32_t t_part = (sec_len != full16 && us <= full16 && full16 < us + unit) ? (full16 - us) >> 7 : 0xFFFFFFFFu;
#pragma unroll 1
    for (uint32_t t = 0; t < rounds; ++t) {
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this round's DMA has landed
        uint32_t wv[32];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const uint4 v = slot[lane * 8 + ((q + rot) & 7)];
            wv[4 * q] = v.x, wv[4 * q + 1] = v.y, wv[4 * q + 2] = v.z, wv[4 * q + 3] = v.w;
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the slot is free for the next DMA
        if (t + 1 < rounds) dma_round(t + 1);
        const uint32_t rb = us + t * 128;  // section-relative start of this lane's 128 B
        // the section's partial last 16 B (outside the resource): byte loads, in the one lane that has it
        if (t == t_part) {
            const int pi = (int)((full16 - rb) >> 4);
            uint32_t pw[4] = {0, 0, 0, 0};
#pragma unroll
            for (uint32_t q = 0; q < 16; ++q)
                if (full16 + q < sec_len) pw[q >> 2] |= (uint32_t)base[full16 + q] << (8 * (q & 3));
#pragma unroll
            for (int q = 0; q < 8; ++q)
                if (q == pi) wv[4 * q] = pw[0], wv[4 * q + 1] = pw[1], wv[4 * q + 2] = pw[2], wv[4 * q + 3] = pw[3];
        }
        // roll the 128 bytes; the gathers of word i + P are issued before word i is rolled
        constexpr int P = 3;
        uint64_t G[P + 1][4];
#pragma unroll
        for (int i = 0; i < P; ++i)
#pragma unroll
            for (int b = 0; b < 4; ++b) G[i][b] = gear(wv[i], b);
        uint64_t hb = h;  // the hash before the current group
        // opaque copy: kept in two VGPRs (otherwise hipcc may re-derive it inside the rare record
        // branch from the rolled hashes, which costs hundreds of extra shift-adds per round)
        asm volatile("" : "+v"(hb));
        uint32_t anyz = 0xFFFFFFFFu;
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            if (i + P < 32) {
#pragma unroll
                for (int b = 0; b < 4; ++b) G[(i + P) % (P + 1)][b] = gear(wv[i + P], b);
            }
            __builtin_amdgcn_sched_barrier(0);
            uint32_t tt[4];
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                h = (h << 1) + G[i % (P + 1)][b];
                if constexpr (SH) tt[b] = (uint32_t)(h >> 32) & ch;
                else tt[b] = ((uint32_t)h & cl) | ((uint32_t)(h >> 32) & ch);
            }
            anyz = min3_u32(min3_u32(anyz, tt[0], tt[1]), tt[2], tt[3]);  // two v_min3 per 4 bytes
            if ((i & 3) == 3) {
                // one VALU compare and a uniform branch when no lane of the wave has a candidate here
                if (__builtin_amdgcn_ballot_w64(anyz == 0)) {
                    const uint32_t g = rb + 16 * (uint32_t)(i >> 2);  // the group, section-relative
                    if (anyz == 0 && g < sec_len) {
#ifndef OXH_F1_NOSTORE  // diagnostic builds only: the cost of the candidate stores (output invalid)
                        if (count < prm.cap) {
                            out_c[count].e = ((uint64_t)((g - us) >> 4) << kEntryShift) | ((SH ? (hb >> 16) : hb) & kEntryHash);
                            out_c[count].b = make_uint4(wv[i - 3], wv[i - 2], wv[i - 1], wv[i]);
                        }
#endif
                        ++count;
                    }
                }
                anyz = 0xFFFFFFFFu;
                hb = h;
                asm volatile("" : "+v"(hb));
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    out_c[0].n = count;
    const uint64_t occ = __builtin_amdgcn_ballot_w64(count != 0);
    if (lane == 0) f.cand_occ[sec] = occ;
}

// ---------------------------------------------------------------- the walk (F2, F3)
// Cursor over the candidate lists of one file, monotone in position. Lists are per unit (sec / 64
// bytes, one F1 lane); unit u of global section s has global index 64 s + u.
struct CandCursor {
    uint64_t sec;   // global unit index of the cursor
    uint32_t idx;   // group index within that unit's list
    uint32_t rsec_idx = 0xFFFFFFFFu;  // the last resolved group (unit + idx) and its flags
    uint64_t rsec = ~0ull;
    uint64_t occ_sec = ~0ull, occ = 0;  // the occupancy mask of section occ_sec (F1's ballot)
    uint32_t rflag = 0, rbits = 0;  // the flag the resolved group's bits are for, and the bits
};

// Full-window hash test of positions [lo, hi) (all inside one file, lo >= 47) by direct byte scan:
// used where a unit's candidate list overflowed. Returns the first position with
// (hash & mask) == 0, or hi.
__device__ uint64_t scan_bytes(const uint8_t* __restrict__ fbase, uint64_t lo, uint64_t hi, uint64_t mask,
                               const uint64_t* __restrict__ gear) {
    // hi <= the file length (queries never pass it)
    uint64_t h = 0;
    for (uint64_t p = lo - kHashSpan; p < hi; p += 16) {
        const uint4 v = load16_file(fbase, p, hi);
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint64_t q = p + (uint64_t)j;
            if (q >= hi) return hi;
            h = (h << 1) + gear_of(gear, byte_of(v, j));
            if (q >= lo && (h & mask) == 0) return q;
        }
    }
    return hi;
}

// Exact flags of a candidate group for ONE mask (bit j: position g + j has (hash & mask) == 0): roll
// the 16 bytes F1 stored with it from the hash F1 recorded before it (no re-read of the file: the
// walk is latency-bound and the lists stay in the L2 / Infinity Cache). The tests fold into one
// minimum first; the bits are assembled only when some position hit (always for mask_l, whose bits
// are the ones F1 filtered on; rarely for the stricter mask_s).
__device__ __forceinline__ uint32_t and_or_v(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ uint32_t resolve_group(const uint4 v, uint64_t g, uint64_t H, uint64_t flen, uint64_t mask,
                                                  const uint64_t* __restrict__ gear) {
    const uint32_t mlo = (uint32_t)mask, mhi = (uint32_t)(mask >> 32);
    uint64_t h = H;
    uint32_t t[16];
    uint32_t z = 0xFFFFFFFFu;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        h = (h << 1) + gear_of(gear, byte_of(v, j));
        t[j] = and_or_v((uint32_t)h, mlo, (uint32_t)(h >> 32) & mhi);
        if (j & 1) z = min3_u32(z, t[j - 1], t[j]);
    }
    uint32_t bits = 0;
    if (z == 0) {
#pragma unroll
        for (int j = 0; j < 16; ++j) bits |= (t[j] == 0 ? 1u : 0u) << j;
    }
    const uint32_t live = flen - g < 16 ? (uint32_t)(flen - g) : 16u;
    return live >= 16 ? bits : bits & ((1u << live) - 1u);
}

// First position in [lo, hi) (file-relative) whose full-window hash matches `flag` (1: mask_s,
// 2: mask_l), or hi. Advances the cursor (callers query increasing positions).
__device__ uint64_t first_cand(const CdcFiles& f, const CdcParams& prm, uint64_t sec0, uint64_t nsec_file,
                               const uint8_t* fbase, uint64_t flen, CandCursor& cur, uint64_t lo, uint64_t hi,
                               uint32_t flag, const uint64_t* gear) {
    if (lo >= hi) return hi;
    // units: the file's sections [sec0, sec0 + nsec_file) hold units [64 sec0, 64 (sec0 + nsec_file))
    const uint64_t u0 = 64 * sec0, nu = 64 * nsec_file;
    const uint64_t s = lo / prm.unit;
    if (cur.sec < u0 + s) {
        cur.sec = u0 + s;
        cur.idx = 0;
    }
    if (cur.sec >= u0 + nu) return hi;
    while (true) {
        // skip the units F1 found no candidate in without loading their counts
        const uint64_t gsec = cur.sec >> 6;
        if (cur.occ_sec != gsec) {
            cur.occ = f.cand_occ[gsec];
            cur.occ_sec = gsec;
        }
        const uint64_t rest = cur.occ >> (cur.sec & 63);
        if (rest == 0) {
            const uint64_t next = (gsec + 1) * 64;  // the next section's first unit
            if (next >= u0 + nu || (next - u0) * prm.unit >= hi) return hi;
            cur.sec = next;
            cur.idx = 0;
            continue;
        }
        if (!(rest & 1)) {
            cur.sec += (uint64_t)__builtin_ctzll(rest);
            cur.idx = 0;
        }
        const uint64_t sec_start = (cur.sec - u0) * prm.unit;  // the unit's start, file-relative
        if (sec_start >= hi) return hi;
        const CandRec* cs = f.cand + cur.sec * prm.cap;
        // an entry and its 16 bytes are loaded together (the bytes before the entry says whether they
        // are needed), and the first pair together with the count (speculatively: slots past the
        // count are scratch, read but never used)
        const uint32_t cnt = (uint32_t)cs[0].n;
        uint64_t e_nx = cur.idx < prm.cap ? cs[cur.idx].e : 0;
        uint4 b_nx = cur.idx < prm.cap ? cs[cur.idx].b : make_uint4(0, 0, 0, 0);
        const uint32_t stored = cnt < prm.cap ? cnt : prm.cap;
        for (bool first = true; cur.idx < stored; first = false) {
            if (!first) {
                e_nx = cs[cur.idx].e;
                b_nx = cs[cur.idx].b;
            }
            const uint64_t e = e_nx;
            const uint4 bv = b_nx;
            const uint64_t g = sec_start + (e >> kEntryShift) * 16;
            if (g >= hi) return hi;
            if (g + 16 > lo) {  // the group overlaps [lo, hi)
                if (cur.rsec != cur.sec || cur.rsec_idx != cur.idx || cur.rflag != flag) {
                    cur.rbits = resolve_group(bv, g, e & kEntryHash, flen, flag == 1 ? prm.mask_s : prm.mask_l, gear);
                    cur.rsec = cur.sec;
                    cur.rsec_idx = cur.idx;
                    cur.rflag = flag;
                }
                uint32_t m = cur.rbits;
                if (lo > g) m &= ~0u << (uint32_t)(lo - g);                  // positions >= lo
                if (hi < g + 16) m &= (1u << (uint32_t)(hi - g)) - 1u;       // positions < hi
                if (m) return g + (uint64_t)__builtin_ctz(m);
                // the rest of the group lies beyond hi: the next query (from hi on) needs it again
                if (g + 16 > hi) return hi;
            }
            // below lo, or done with: later queries start at or after this one's end (an L query
            // follows an S query from eS on), so the group is never needed again
            ++cur.idx;
        }
        const uint64_t sec_end = sec_start + prm.unit;
        if (cnt > prm.cap) {
            // overflowed list: positions after the last stored group were not recorded
            const uint64_t after = stored ? sec_start + (cs[stored - 1].e >> kEntryShift) * 16 + 16 : sec_start;
            const uint64_t a = lo > after ? lo : after;
            const uint64_t b = hi < sec_end ? hi : sec_end;
            if (a < b) {
                const uint64_t m = scan_bytes(fbase, a, b, flag == 1 ? prm.mask_s : prm.mask_l, gear);
                if (m < b) return m;
            }
        }
        // move to the next section only if the query reaches into it: a later query (the L range
        // after an S range) may still need this section
        if (sec_end >= hi || cur.sec + 1 >= u0 + nu) return hi;
        ++cur.sec;
        cur.idx = 0;
    }
}

// Length of the chunk that starts at file-relative position s (cut_gear on content[s..]).
__device__ uint64_t cdc_cut(const CdcFiles& f, const CdcParams& prm, uint64_t sec0, uint64_t nsec_file,
                            const uint8_t* fbase, uint64_t flen, uint64_t s, CandCursor& cur,
                            const uint64_t* gear) {
    uint64_t rem = flen - s;
    if (rem <= prm.min) return rem;
    uint64_t center = prm.avg;
    if (rem > prm.max) rem = prm.max;
    else if (rem < center) center = rem;
    const uint64_t a0 = (prm.min / 2) * 2, eS = (center / 2) * 2, eL = (rem / 2) * 2;
    // truncated window: the hash restarts from 0 at a0
    // the 47 bytes from a0: three 16-byte loads issued together
    const uint4 t0 = load16_file(fbase, s + a0, flen), t1 = load16_file(fbase, s + a0 + 16, flen),
                t2 = load16_file(fbase, s + a0 + 32, flen);
    bool exact = true;
    if (a0 + kHashSpan <= eS) {
        // Common case: all 47 positions test mask_s. Roll them with no branch per position (the
        // table reads do not depend on the hash, so they go out ahead) and fold the tests into one
        // minimum; only lanes with a zero test (2^-popcount(mask_s) per position) run the exact loop
        // below to find the first one. The per-position branch with two masks cost ~16 VALU and an
        // LDS round trip per position.
        const uint32_t mlo = (uint32_t)prm.mask_s, mhi = (uint32_t)(prm.mask_s >> 32);
        uint64_t hh = 0;
        uint32_t anyz = 0xFFFFFFFFu, tprev = 0xFFFFFFFFu;
#pragma unroll
        for (int k = 0; k < kHashSpan; ++k) {
            const uint32_t b = k < 16 ? byte_of(t0, k) : k < 32 ? byte_of(t1, k - 16) : byte_of(t2, k - 32);
            hh = (hh << 1) + gear_of(gear, b);
            const uint32_t t = and_or((uint32_t)hh, mlo, (uint32_t)(hh >> 32) & mhi);
            if (k & 1) anyz = min3_u32(anyz, tprev, t);
            else tprev = t;
        }
        exact = min_u32(anyz, tprev) == 0;
    }
    if (exact) {
        uint64_t h = 0;
        const uint64_t tend = a0 + kHashSpan < eL ? a0 + kHashSpan : eL;
#pragma unroll
        for (int k = 0; k < kHashSpan; ++k) {
            const uint64_t q = a0 + (uint64_t)k;
            if (q >= tend) break;
            const uint32_t b = k < 16 ? byte_of(t0, k) : k < 32 ? byte_of(t1, k - 16) : byte_of(t2, k - 32);
            h = (h << 1) + gear_of(gear, b);
            if ((h & (q < eS ? prm.mask_s : prm.mask_l)) == 0) return q;
        }
    }
    // [qs, eS) against mask_s, then [max(qs, eS), eL) against mask_l, through ONE first_cand site: the
    // lanes of a wave in either range run it together, and the walk's code (and its register
    // pressure) is half the size of two inlined copies
    const uint64_t qs = a0 + kHashSpan;
#pragma unroll 1
    for (uint32_t flag = 1; flag <= 2; ++flag) {
        const uint64_t lo = flag == 1 ? qs : (qs > eS ? qs : eS);
        const uint64_t hi = flag == 1 ? eS : eL;
        if (lo < hi) {
            const uint64_t p = first_cand(f, prm, sec0, nsec_file, fbase, flen, cur, s + lo, s + hi, flag, gear);
            if (p < s + hi) return p - s;
        }
    }
    return rem;
}

// F2: speculative walk of one section from its start, recording chunk starts (relative to the
// section start) until a start reaches the section end or the file end (that start is recorded too).
__global__ __launch_bounds__(256) void cdc_walk_kernel(CdcFiles f, CdcParams prm, uint64_t n_sec) {
    __shared__ uint64_t lds_gear[256];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) lds_gear[i] = kGear[i];
    __syncthreads();
    const uint64_t sec = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (sec >= n_sec) return;
    const uint32_t file = f.sec_file[sec];
    const uint64_t flen = f.flen[file];
    const uint64_t sec0 = f.sec_base[file], nsec_file = f.sec_base[file + 1] - sec0;
    const uint64_t sec_start = (sec - sec0) * prm.sec;
    const uint64_t sec_end = sec_start + prm.sec < flen ? sec_start + prm.sec : flen;
    const uint8_t* fbase = f.arena + f.foff[file];
    uint32_t* out = f.spec + sec * prm.speccap;
    // warm up over the `warmup` bytes before the section (unrecorded): a walk started anywhere meets
    // the true walk within a few chunks, so the recorded starts are almost always the true ones
    // One loop for the warm-up and the recorded part (one cdc_cut site): each lane moves from one to
    // the other on its own, instead of the wave finishing every lane's warm-up first.
    uint64_t s = sec_start > prm.warmup ? sec_start - prm.warmup : 0;
    CandCursor cur{64 * sec0 + s / prm.unit, 0};
    uint32_t n = 0;
    while (true) {
        if (s >= sec_start) {
            if (n < prm.speccap) out[n] = (uint32_t)(s - sec_start);
            ++n;
            if ((s >= sec_end && n > 1) || s >= flen) break;
        }
        s += cdc_cut(f, prm, sec0, nsec_file, fbase, flen, s, cur, lds_gear);
    }
    f.spec_cnt[sec] = n;
}

// ---------------------------------------------------------------- F3: stitch
// Sections are at least `max` bytes, so every chunk that starts before a section ends at or before
// the next section's end: the true walk's first start in section i, entry(i), is < sec_end(i).
// If section i-1 is right, entry(i) is the last start its list recorded (the first >= its end). When
// that start also appears in section i's speculative list, everything after it in that list is the
// true walk (a cut depends only on where its chunk starts) -- section i "converged". Induction from
// section 0 (which starts at the file start, so its walk is the true one) makes every converged
// section right, except after a section that did not converge; those are re-walked serially (F3b).
enum : uint32_t { kConverged = 0, kFailed = 1, kFixed = 2 };

struct CdcStitch {
    uint32_t* status;   // [n_sec]
    uint32_t* k0;       // [n_sec] first speculative entry of the true walk (converged)
    uint32_t* count;    // [n_sec] true starts inside the section
    uint64_t* exit;     // [n_sec] file-relative entry of the next section (or the file length)
    uint32_t* fix;      // [n_sec * speccap] re-walked starts, relative to the section start
    uint64_t* out_base; // [n_sec + 1] exclusive prefix of count (global chunk index)
};

__device__ __forceinline__ uint64_t spec_last_abs(const CdcFiles& f, const CdcParams& prm, uint64_t sec,
                                                  uint64_t sec_start) {
    return sec_start + f.spec[sec * prm.speccap + (f.spec_cnt[sec] - 1)];
}

// F3a: one lane per section.
__global__ __launch_bounds__(256) void cdc_check_kernel(CdcFiles f, CdcParams prm, CdcStitch s, uint64_t n_sec) {
    const uint64_t sec = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (sec >= n_sec) return;
    const uint32_t file = f.sec_file[sec];
    const uint64_t sec0 = f.sec_base[file];
    const uint64_t sec_start = (sec - sec0) * prm.sec;
    const uint32_t cnt = f.spec_cnt[sec];
    const uint32_t* spec = f.spec + sec * prm.speccap;
    uint32_t status = kFailed, k0 = 0;
    if (cnt <= prm.speccap) {
        if (sec == sec0) {
            status = kConverged;
        } else if (f.spec_cnt[sec - 1] <= prm.speccap) {
            const uint64_t e = spec_last_abs(f, prm, sec - 1, sec_start - prm.sec);
            // binary search e - sec_start in the sorted list
            uint32_t lo = 0, hi = cnt;
            const uint64_t key = e - sec_start;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if ((uint64_t)spec[mid] < key) lo = mid + 1;
                else hi = mid;
            }
            if (lo < cnt && (uint64_t)spec[lo] == key) {
                status = kConverged;
                k0 = lo;
            }
        }
    }
    s.status[sec] = status;
    s.k0[sec] = k0;
    if (status == kConverged) {
        s.count[sec] = cnt - 1 - k0;  // every entry but the last is a start inside the section
        s.exit[sec] = sec_start + spec[cnt - 1];
    }
}

// F3b: one wave per file finds the sections that did not converge (64 statuses per step) and its
// lane 0 re-walks them: from the true entry, cut chunks until a start lands on the section's
// speculative list (the rest of the list is then right) or the walk leaves the section (then the
// next section's check is void and it is re-walked too).
__global__ __launch_bounds__(64) void cdc_fixup_kernel(CdcFiles f, CdcParams prm, CdcStitch s, uint64_t n_files) {
    __shared__ uint64_t lds_gear[256];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) lds_gear[i] = kGear[i];
    __syncthreads();
    const uint64_t file = blockIdx.x;
    if (file >= n_files) return;
    const int lane = threadIdx.x;
    const uint64_t flen = f.flen[file];
    const uint64_t sec0 = f.sec_base[file], nsec_file = f.sec_base[file + 1] - sec0;
    const uint8_t* fbase = f.arena + f.foff[file];
    uint64_t i = 1;  // section 0 always converges
    while (i < nsec_file) {
        // next failed section at or after i
        const uint64_t j = i + (uint64_t)lane;
        const bool failed = j < nsec_file && s.status[sec0 + j] == kFailed;
        const uint64_t m = __builtin_amdgcn_ballot_w64(failed);
        if (m == 0) {
            i += 64;
            continue;
        }
        i += (uint64_t)__builtin_ctzll(m);
        // lane 0 re-walks from section i; the others wait at the next ballot
        uint64_t next = i;
        if (lane == 0) {
            uint64_t pos = s.exit[sec0 + i - 1];
            CandCursor cur{64 * (sec0 + i), 0};
            for (uint64_t t = i; t < nsec_file; ++t) {
                const uint64_t sec = sec0 + t;
                const uint64_t sec_start = t * prm.sec;
                const uint64_t sec_end = sec_start + prm.sec < flen ? sec_start + prm.sec : flen;
                const uint32_t cnt = f.spec_cnt[sec];
                const uint32_t* spec = f.spec + sec * prm.speccap;
                const bool spec_ok = cnt <= prm.speccap;
                uint32_t* fix = s.fix + sec * prm.speccap;
                uint32_t n = 0, k = 0;
                bool landed = false;
                while (pos < sec_end) {
                    if (spec_ok) {
                        while (k < cnt && sec_start + spec[k] < pos) ++k;
                        if (k < cnt && sec_start + spec[k] == pos) {
                            for (; k + 1 < cnt; ++k) fix[n++] = spec[k];
                            pos = sec_start + spec[cnt - 1];
                            landed = true;
                            break;
                        }
                    }
                    fix[n++] = (uint32_t)(pos - sec_start);
                    if (cur.sec < 64 * sec) cur = CandCursor{64 * sec, 0};
                    pos += cdc_cut(f, prm, sec0, nsec_file, fbase, flen, pos, cur, lds_gear);
                }
                s.status[sec] = kFixed;
                s.count[sec] = n;
                s.exit[sec] = pos;
                next = t + 1;
                // a converged next section is right only if its check saw this exit
                if (landed && (t + 1 >= nsec_file || s.status[sec + 1] == kConverged)) break;
            }
        }
        i = (uint64_t)__builtin_amdgcn_readfirstlane((int)next) | ((uint64_t)__builtin_amdgcn_readfirstlane((int)(next >> 32)) << 32);
    }
}

// F3c: exclusive prefix of the per-section counts (one block; n_sec is ~ bytes / 512 KiB). Every
// thread owns a run of `per` counts (a multiple of 4, so the run starts 16-B aligned: count is a
// 256-B aligned scratch part) and sums it with independent 16-byte loads; one load per count, each
// waiting on the one before through the running sum, took 0.43 ms for C5's 262 144 sections.
__global__ __launch_bounds__(1024) void cdc_prefix_kernel(CdcStitch s, uint64_t n_sec) {
    __shared__ uint64_t part[1024];
    const uint64_t per = ((n_sec + 1023) / 1024 + 3) & ~3ull;
    const uint64_t b = (uint64_t)threadIdx.x * per < n_sec ? (uint64_t)threadIdx.x * per : n_sec;
    const uint64_t e = b + per < n_sec ? b + per : n_sec;
    const uint4* __restrict__ c4 = (const uint4*)s.count;
    uint64_t sum = 0, i = b;
#pragma unroll 8
    for (; i + 4 <= e; i += 4) {
        const uint4 v = c4[i >> 2];
        sum += (uint64_t)v.x + v.y + v.z + v.w;
    }
    for (; i < e; ++i) sum += s.count[i];
    part[threadIdx.x] = sum;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const uint64_t v = threadIdx.x >= (unsigned)o ? part[threadIdx.x - o] : 0;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    uint64_t run = threadIdx.x ? part[threadIdx.x - 1] : 0;
    // four counts per 16-byte load, four bases per two 16-byte stores (out_base + b is 32-B aligned)
    ulonglong2* __restrict__ o2 = (ulonglong2*)s.out_base;
    i = b;
#pragma unroll 4
    for (; i + 4 <= e; i += 4) {
        const uint4 v = c4[i >> 2];
        const uint64_t r1 = run + v.x, r2 = r1 + v.y, r3 = r2 + v.z;
        o2[i >> 1] = make_ulonglong2(run, r1);
        o2[(i >> 1) + 1] = make_ulonglong2(r2, r3);
        run = r3 + v.w;
    }
    for (; i < e; ++i) {
        s.out_base[i] = run;
        run += s.count[i];
    }
    if (threadIdx.x == 1023) s.out_base[n_sec] = part[1023];
}

// F3d: the chunk table. One lane per chunk start, grouped by section (a wave per section).
// c_flag (W2's fold, may be NULL): 1 for a chunk of a section whose list is W's own (its block sums in
// geo.sums are the chunk's), 0 for the sections X re-walked.
__global__ __launch_bounds__(256) void cdc_emit_kernel(CdcFiles f, CdcParams prm, CdcStitch s, uint64_t n_sec,
                                                       uint64_t* __restrict__ c_off, uint64_t* __restrict__ c_len,
                                                       uint8_t* __restrict__ c_flag) {
    const uint64_t sec = (uint64_t)blockIdx.x * 4 + (uint64_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (sec >= n_sec) return;
    const int lane = threadIdx.x & 63;
    const uint32_t file = f.sec_file[sec];
    const uint64_t sec_start = (sec - f.sec_base[file]) * prm.sec;
    const uint64_t foff = f.foff[file];
    const uint32_t cnt = s.count[sec];
    const uint32_t* src = s.status[sec] == kFixed ? s.fix + sec * prm.speccap : f.spec + sec * prm.speccap + s.k0[sec];
    const uint64_t base = s.out_base[sec];
    const uint64_t ex = s.exit[sec];
    const uint8_t own = s.status[sec] == kFixed ? 0 : 1;
    for (uint32_t k = lane; k < cnt; k += 64) {
        const uint64_t a = sec_start + src[k];
        const uint64_t b = k + 1 < cnt ? sec_start + src[k + 1] : ex;
        c_off[base + k] = foff + a;
        c_len[base + k] = b - a;
        // a chunk that starts within `max` of its section start may overlap the previous section's
        // last chunk, whose blocks that lane stored too (and a lane that had not yet met the true walk
        // there stored blocks of chunks that are not the crate's): K1F hashes those from the bytes
        if (c_flag) c_flag[base + k] = own && src[k] >= prm.max;
    }
}

// per-file first chunk index
__global__ void cdc_first_kernel(const uint64_t* __restrict__ sec_base, const uint64_t* __restrict__ out_base,
                                 uint64_t n_files, uint64_t* __restrict__ first) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i <= n_files) first[i] = out_base[sec_base[i]];
}

// File of every section (sec_base is the exclusive prefix of per-file section counts): built on the
// device so no section-sized table is copied from pageable host memory.
__global__ void cdc_sec_file_kernel(const uint64_t* __restrict__ sec_base, uint64_t n_files, uint64_t n_sec,
                                    uint32_t* __restrict__ sec_file) {
    const uint64_t sec = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (sec >= n_sec) return;
    uint64_t lo = 0, hi = n_files;  // last file with sec_base[file] <= sec
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) >> 1;
        if (sec_base[mid] <= sec) lo = mid;
        else hi = mid;
    }
    sec_file[sec] = (uint32_t)lo;
}


// ---------------------------------------------------------------- W: the walk itself, skipping `min`
// fastcdc v2020's cut_gear never hashes a chunk's first `min` bytes: the hash starts from 0 at
// index a0 = min & ~1 of every chunk (fastcdchunker.rs:83-98 -> crate fastcdc 3.2.1 cut_gear). F1
// rolls every byte of the input; at 8 KiB chunks (min 4 KiB, mean chunk 10.5 KB) only 61 % of the
// bytes are ever hashed by the crate. W walks the chunks themselves, one lane per section, and reads
// and rolls only those bytes.
//
// One lane per section (sections sized so the whole input is one generation of waves), every lane
// walking its own chunks from `warmup` bytes before its section and recording the starts inside it
// (the spec list F3 consumes). The bytes reach the lanes exactly as in F1: a round is one 128-B
// line of every lane's stream, fetched by 8 LDS-DMA loads per wave (lanes 8m..8m+7 of DMA k fetch
// the line of lane 8k+m, its address taken from that lane with ds_bpermute; pieces rotated so the
// ds_read_b128 back are conflict-free), the 32-copy gear table (no bank conflicts), the same
// per-byte v_perm + ds_read_b64 + v_lshl_add_u64 + AND + min3. Per lane the round's mask is the
// exact one for its position in its chunk (mask_s before center, mask_l after, their common bits in
// the round that crosses center, all bits -- nothing passes -- before the first tested position),
// so a group with a zero test is almost always a cut; the ballot-guarded branch resolves the
// position, records the new chunk start and points the lane's next fetch at the line holding its
// next `a0` (the round already in flight for the lane is skipped: one bubble per chunk).
//
// The walk is RELAXED: a chunk's first 47 hashed positions (a0 .. a0+46) see a hash that started
// from 0, not the full 48-byte window, and W does not test them (its hash there includes the bytes
// before a0 of the line it starts rolling from -- harmless from a0+47 on, where those have shifted
// past bit 63). So W's cut of chunk c equals the crate's unless one of those 47 truncated positions
// matches (0.29 % of chunks at 8 KiB, measured against the C restatement): the X pass below checks
// every recorded start for exactly that and re-walks exactly where it happened. Masks must sit at
// bit 16 or above (they do for avg <= 16 KiB at level 1), so with the hash kept 16 bits to the left
// every test is one AND on the high word.
constexpr uint32_t kWalkOob = 0xFFFFFF00u;   // DMA offset of a lane with nothing to fetch (past the range)
constexpr uint32_t kWalkFull = 0xFFFFFFFFu;  // the round mask that lets nothing pass
constexpr uint32_t kNoCut = 0xFFFFFFFFu;

struct WalkGeom {
    uint64_t arena_bytes;  // the arena holds file bytes up to here (the DMA range stops at it, 16-B rounded)
    uint64_t* sums;        // FOLD: XXH3 block sums, 8 u64 per 1 KiB of arena (block at arena offset A -> A >> 10)
};

// The chunk that starts at m-space position cs: its test window [lo, tL), the mask switch tS and the
// relaxed cut cutm (= cs + rem when nothing in the window matches). Chunks with nothing to test (at
// most `min` bytes left, or the window empty at a file's tail) are cut at once; the starts at or after
// the section start are recorded; the start that reaches the section end (or the file end) is the
// lane's last record and ends its walk.
struct WalkLane {
    uint32_t cs, lo, tS, tL, cutm;
    uint32_t mS, mE, mF;  // section start, section end, file end (m-space)
    uint32_t n;           // starts recorded
    bool done;
};

__device__ __forceinline__ void walk_begin_chunk(WalkLane& L, const CdcParams& prm, uint32_t* __restrict__ out) {
    for (;;) {
        if (L.cs >= L.mS) {
            if (L.n < prm.speccap) out[L.n] = L.cs - L.mS;
            ++L.n;
            if ((L.cs >= L.mE && L.n > 1) || L.cs >= L.mF) {
                L.done = true;
                return;
            }
        }
        const uint32_t len = L.mF - L.cs;
        if (len <= (uint32_t)prm.min) {
            L.cs += len;
            continue;
        }
        const uint32_t rem = len > (uint32_t)prm.max ? (uint32_t)prm.max : len;
        uint32_t center = (uint32_t)prm.avg;
        if (len <= (uint32_t)prm.max && len < center) center = len;
        const uint32_t a0 = (uint32_t)(prm.min & ~1ull);
        L.lo = L.cs + a0 + (uint32_t)kHashSpan;
        L.tS = L.cs + (center & ~1u);
        L.tL = L.cs + (rem & ~1u);
        L.cutm = L.cs + rem;
        if (L.lo >= L.tL) {  // only truncated positions to test: X checks those
            L.cs = L.cutm;
            continue;
        }
        return;
    }
}

// LATE: the next round's DMA goes out after this round is rolled, when each lane's next line is known
// (no stale round after a cut, but the DMA's latency is left to the other waves of the SIMD to hide);
// otherwise it goes out before the roll, for the line after the current one.
//
// FOLD (W2, min = 4 KiB, DESIGN §4 "W2"): the walk also folds XXH3's stripe accumulation into the bytes
// it streams. XXH3-128's long path sums 64-B stripes into 8 accumulators per 1 KiB block and scrambles
// them between blocks; a block's sum (acc[i] += lo32(w ^ key) * hi32(w ^ key), acc[i ^ 1] += w over its
// 128 words) does not depend on the accumulators, so W can produce the sums of a chunk's blocks 4..
// (the bytes after its `min` = 4 blocks, the only ones W reads) and a second pass (K1F) adds blocks 0-3,
// the partial last block and the last stripe from the bytes and runs each chunk's chain over the stored
// sums. For that, a lane's lines are chunk-relative: line k of a chunk starting at cs is fetched from
// (cs + min + 128 k) & ~3 (dword aligned; W proper fetches 128-B aligned lines), so every 8 lines are one
// block, word q of a line is bytes [cs + min + 128 k + 8 q, + 8) at line byte (cs & 3) + 8 q, realigned
// with v_alignbyte, and its key is secret word 2 (k % 8) + (q >> 3) + (q & 7) (taken from the lanes that
// hold the secret, by ds_bpermute: W's LDS is full). Word 15 needs the next line's first dword, so it is
// folded at the start of the next round. A block's sum goes to geo.sums once its last word is folded;
// blocks of chunks that start before the lane's section (warm-up) are not stored, and K1F uses a chunk's
// sums only where the stitch kept W's list (X marks fixed sections).
template <int WAVES, bool LATE, bool FOLD = false>
__global__ __launch_bounds__(64 * WAVES) void cdc_walk_scan_kernel(CdcFiles f, CdcParams prm, uint64_t n_sec, WalkGeom geo) {
    __shared__ __attribute__((aligned(16))) uint64_t lds[256 * 32 + WAVES * 1024];
    for (int i = threadIdx.x; i < 256 * 32; i += blockDim.x) lds[i] = kGear[i >> 5] << 16;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint4* const slot = (uint4*)(lds + 256 * 32) + w * 512;
    const uint64_t sec0 = ((uint64_t)blockIdx.x * WAVES + (uint64_t)w) * 64;
    if (sec0 >= n_sec) return;
    const uint64_t sec = sec0 + (uint64_t)lane;
    const bool live = sec < n_sec;
    const uint64_t secq = live ? sec : n_sec - 1;
    const uint32_t file = f.sec_file[secq];
    const uint64_t flen = f.flen[file];
    const uint64_t s_start = (secq - f.sec_base[file]) * prm.sec;
    const uint64_t s_end = s_start + prm.sec < flen ? s_start + prm.sec : flen;
    const uint64_t w0 = s_start > prm.warmup ? s_start - prm.warmup : 0;
    // the wave's DMA window: from the lowest address any lane starts at (a 128-B line), so every lane's
    // positions are 32-bit offsets into one buffer resource (the host checked the wave spans < 4 GiB)
    const uint64_t a_file = (uint64_t)f.arena + f.foff[file];
    uint64_t a_min = live ? a_file + w0 : ~0ull;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t other = ((uint64_t)(uint32_t)__shfl_xor((int)(a_min >> 32), o) << 32) | (uint32_t)__shfl_xor((int)(uint32_t)a_min, o);
        a_min = other < a_min ? other : a_min;
    }
    const uint64_t base = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a_min) |
                           ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a_min >> 32)) << 32)) & ~127ull;
    const uint64_t a_end = ((uint64_t)f.arena + geo.arena_bytes + 15) & ~15ull;
    const uint64_t span = a_end - base;
    const int nrec = __builtin_amdgcn_readfirstlane((int)(uint32_t)(span < 0xFFFFFF00ull ? span : 0xFFFFFF00ull));
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, nrec, 0x00020000);

    WalkLane L;
    const uint32_t mfile = (uint32_t)(a_file - base);  // only positions >= w0 are ever used
    L.mS = mfile + (uint32_t)s_start;
    L.mE = mfile + (uint32_t)s_end;
    // the walk never looks past its section end + one chunk, so the file end is clamped to a point
    // beyond that (every chunk it cuts there still sees more than `max` bytes left: the same cut) and
    // every position fits 32 bits
    const uint64_t f_lim = s_start + prm.sec + 2 * prm.max + 4096;
    L.mF = mfile + (uint32_t)(flen < f_lim ? flen : f_lim);
    L.n = 0;
    L.done = !live;
    L.cs = mfile + (uint32_t)w0;
    uint32_t* __restrict__ out = f.spec + secq * prm.speccap;
    if (live) walk_begin_chunk(L, prm, out);
    const uint32_t a0 = (uint32_t)(prm.min & ~1ull);
    constexpr uint32_t kLineMask = FOLD ? ~3u : ~127u;  // FOLD: chunk-relative, dword-aligned lines
    uint32_t NL = L.done ? kWalkOob : ((L.cs + a0) & kLineMask);  // next line to fetch
    const uint64_t ms64 = prm.mask_s << 16, ml64 = prm.mask_l << 16;
    const uint32_t ms = (uint32_t)(ms64 >> 32), ml = (uint32_t)(ml64 >> 32), mc = ms & ml;  // host: all bits >= 16
    const uint32_t copy_off = (uint32_t)(lane & 31) * 8;
    const char* const tab = (const char*)lds;
    auto gear = [&](uint32_t word, int j) -> uint64_t {
        const uint32_t a = __builtin_amdgcn_perm(word, copy_off, 0x0c0c0000u | ((4u + (uint32_t)j) << 8));
        return *(const uint64_t*)(tab + a);
    };
    // DMA k, lane 8m + j: piece (j - rot(r)) & 7 of the line of lane r = 8k + m; rot(r) = (r >> 1) & 7 =
    // (4 (k & 1) + (m >> 1)) & 7, so the offset takes two values (odd and even k)
    const int dm = lane >> 3, dj = lane & 7;
    const uint32_t poff0 = 16 * ((uint32_t)(dj - (dm >> 1)) & 7), poff1 = 16 * ((uint32_t)(dj - ((4 + (dm >> 1)) & 7)) & 7);
    auto dma = [&](uint32_t line) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t src = (uint32_t)__builtin_amdgcn_ds_bpermute((8 * k + dm) * 4, (int)line);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void*)(slot + 64 * k), 16,
                                                     src + ((k & 1) ? poff1 : poff0), 0, 0, kScanDmaAux);
        }
    };
    uint32_t RL = NL;  // the line the DMA in flight fetches for this lane
    bool RV = !L.done;  // ... and whether it still belongs to the lane's current chunk
    if (!L.done) NL += 128;
    dma(RL);
    const int rot = (lane >> 1) & 7;
    uint64_t h = 0;
    // FOLD state: the chunk's block accumulators, its line count, byte shift, the previous line's last
    // two dwords and its word 15's key (that word is folded next round), whether the chunk's first valid
    // round is still to come (xfresh: the accumulators restart there), and the secret word this lane
    // holds for the others' ds_bpermute. The fold itself runs on every round with the whole wave active
    // (ds_bpermute reads nothing from inactive lanes): what a stale round (the one in flight at a cut)
    // adds is wiped when the next chunk's first valid round restarts the accumulators.
    uint64_t xa[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t xk = 0, xbs = 0, lag0 = 0, lag1 = 0, klag_lo = 0, klag_hi = 0;
    bool xlag = false, xfresh = true;
    const uint64_t sec_w = kSecW[lane < 24 ? lane : 0];
    const uint32_t sec_lo = (uint32_t)sec_w, sec_hi = (uint32_t)(sec_w >> 32);
    const uint64_t mbase = base - (uint64_t)f.arena;  // arena offset of m-space 0
    auto fold_word = [&](uint32_t lo, uint32_t hi, uint32_t klo, uint32_t khi, int i) {
        xa[i] += (uint64_t)(lo ^ klo) * (uint64_t)(hi ^ khi);
        xa[i ^ 1] += ((uint64_t)hi << 32) | lo;
    };
    // the sum of the chunk's block 4 + (xk - 1) / 8 is complete: store it (recorded chunks only), restart
    auto fold_store = [&]() {
        // only chunks starting `max` or more into the lane's section: the previous lane's last chunk
        // ends within `max` of the section start, and its sums must not be overwritten by a chunk this
        // lane walked before meeting the true walk (emit flags the chunks in between for K1F's bytes)
        if (L.cs >= L.mS + (uint32_t)prm.max) {
            const uint64_t blk = (mbase + (uint64_t)L.cs + (uint64_t)a0 + 1024ull * ((xk - 1) >> 3)) >> 10;
            uint4* dst = reinterpret_cast<uint4*>(geo.sums + 8 * blk);
            dst[0] = make_uint4((uint32_t)xa[0], (uint32_t)(xa[0] >> 32), (uint32_t)xa[1], (uint32_t)(xa[1] >> 32));
            dst[1] = make_uint4((uint32_t)xa[2], (uint32_t)(xa[2] >> 32), (uint32_t)xa[3], (uint32_t)(xa[3] >> 32));
            dst[2] = make_uint4((uint32_t)xa[4], (uint32_t)(xa[4] >> 32), (uint32_t)xa[5], (uint32_t)(xa[5] >> 32));
            dst[3] = make_uint4((uint32_t)xa[6], (uint32_t)(xa[6] >> 32), (uint32_t)xa[7], (uint32_t)(xa[7] >> 32));
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) xa[i] = 0;
    };
    auto fold_reset = [&]() { xk = 0, xlag = false, xfresh = true, xbs = L.cs & 3u; };
    if constexpr (FOLD) fold_reset();
#pragma unroll 1
    for (;;) {
        if (__builtin_amdgcn_ballot_w64(!L.done) == 0) break;
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this round's DMA has landed
        uint32_t wv[32];
        // (FOLD: the 8 slot addresses are recomputed every round rather than held in registers)
        int rr = rot;
        if constexpr (FOLD) asm volatile("" : "+v"(rr));
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const uint4 v = slot[lane * 8 + ((q + rr) & 7)];
            wv[4 * q] = v.x, wv[4 * q + 1] = v.y, wv[4 * q + 2] = v.z, wv[4 * q + 3] = v.w;
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the slot is free for the next DMA
        const uint32_t CL = RL;
        const bool CV = RV && !L.done;
        if constexpr (FOLD) {
            // a valid round (CV; not the stale one after a cut) is line xk of the chunk at L.cs: keys
            // 2 (xk % 8) + 0..8 (words q < 8 take key q, words q >= 8 key q - 7), whole wave active
            const uint32_t kb = (xk & 7u) * 8u;  // bpermute byte address of key 2 (xk % 8)
            auto key = [&](int j, uint32_t& lo, uint32_t& hi) {
                lo = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(kb + 4u * (uint32_t)j), (int)sec_lo);
                hi = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(kb + 4u * (uint32_t)j), (int)sec_hi);
            };
            // word 15 of the previous line; its block may then be complete
            fold_word(__builtin_amdgcn_alignbyte(lag1, lag0, xbs), __builtin_amdgcn_alignbyte(wv[0], lag1, xbs), klag_lo,
                      klag_hi, 7);
            if (CV && xlag && ((xk - 1) & 7u) == 7u) fold_store();
            if (CV && xfresh) {  // the chunk's first valid round: the accumulators start here
#pragma unroll
                for (int i = 0; i < 8; ++i) xa[i] = 0;
                xfresh = false;
            }
            // key j serves word j (j < 8) and word j + 7 (1 <= j <= 7); key 8 is word 15's, next round.
            // One key in flight ahead of its use keeps the registers down (W2 sits at 3 waves per SIMD).
            auto word = [&](int q, uint32_t klo, uint32_t khi) {
                fold_word(__builtin_amdgcn_alignbyte(wv[2 * q + 1], wv[2 * q], xbs),
                          __builtin_amdgcn_alignbyte(wv[2 * q + 2], wv[2 * q + 1], xbs), klo, khi, q & 7);
            };
            uint32_t kl, kh, nkl, nkh;
            key(0, kl, kh);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                key(j + 1, nkl, nkh);
                word(j, kl, kh);
                if (j >= 1) word(j + 7, kl, kh);
                kl = nkl, kh = nkh;
            }
            if (CV) {
                lag0 = wv[30], lag1 = wv[31], klag_lo = kl, klag_hi = kh;
                xlag = true;
                ++xk;
            }
        }
        if constexpr (!LATE) {
            RL = L.done ? kWalkOob : NL;
            RV = !L.done;
            if (!L.done) NL += 128;
            dma(RL);
        }
        // this round's mask (see above); tests at positions < lo or >= tL are rejected when resolved
        uint32_t m;
        if (!CV || CL + 128 <= L.lo) m = kWalkFull;
        else if (CL + 128 <= L.tS) m = ms;
        else if (CL >= L.tS) m = ml;
        else m = mc;
        bool cut_now = false;
        constexpr int P = FOLD ? 2 : 3;
        uint64_t G[P + 1][4];
#pragma unroll
        for (int i = 0; i < P; ++i)
#pragma unroll
            for (int b = 0; b < 4; ++b) G[i][b] = gear(wv[i], b);
        uint32_t hh[16];  // the high words of the hash at the current group's 16 positions
        uint32_t anyz = 0xFFFFFFFFu;
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            if (i + P < 32) {
#pragma unroll
                for (int b = 0; b < 4; ++b) G[(i + P) % (P + 1)][b] = gear(wv[i + P], b);
            }
            __builtin_amdgcn_sched_barrier(0);
            uint32_t tt[4];
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                h = (h << 1) + G[i % (P + 1)][b];
                hh[4 * (i & 3) + b] = (uint32_t)(h >> 32);
                tt[b] = hh[4 * (i & 3) + b] & m;
            }
            anyz = min3_u32(min3_u32(anyz, tt[0], tt[1]), tt[2], tt[3]);
            if ((i & 3) == 3) {
                if (__builtin_amdgcn_ballot_w64(anyz == 0)) {
                    if (anyz == 0) {
                        // the group's zero tests, in position order; the first valid one is the cut
                        const uint32_t g = CL + 16 * (uint32_t)(i >> 2);
                        uint32_t bits = 0;  // (built high position first: no shifted-constant registers)
#pragma unroll
                        for (int j = 15; j >= 0; --j) bits = (bits << 1) | ((hh[j] & m) == 0 ? 1u : 0u);
                        while (bits) {
                            const int j = __builtin_ctz(bits);
                            bits &= bits - 1;
                            const uint32_t p = g + (uint32_t)j;
                            if (p < L.lo || p >= L.tL) continue;
                            if (m == mc) {  // the round that crosses center: mask_s before it, mask_l after
                                uint32_t hj = 0;
#pragma unroll
                                for (int k = 0; k < 16; ++k) hj = k == j ? hh[k] : hj;
                                if ((hj & (p < L.tS ? ms : ml)) != 0) continue;
                            }
                            // a cut: the next chunk starts at p (cut_gear returns the matching index)
                            L.cs = p;
                            walk_begin_chunk(L, prm, out);
                            if constexpr (FOLD) fold_reset();
                            if (!L.done) NL = (L.cs + a0) & kLineMask;
                            RV = false;  // the line in flight belonged to the old chunk
                            m = kWalkFull;
                            cut_now = true;
                            break;
                        }
                    }
                }
                anyz = 0xFFFFFFFFu;
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        // no cut before the end of the test window: the chunk ends at cs + rem (max, or the file end)
        if (CV && !cut_now && CL + 128 >= L.tL) {
            if constexpr (FOLD) {
                // the walk reads no further line of this chunk: a block that ended with the line just
                // folded (a chunk of 1024 m + 1 bytes at a dword-aligned start) still lacks its word 15,
                // which then lies wholly in this line (shift 0)
                if (xlag && xbs == 0 && ((xk - 1) & 7u) == 7u) {
                    fold_word(lag0, lag1, (uint32_t)S64(176), (uint32_t)(S64(176) >> 32), 7);  // key word 22
                    fold_store();
                }
            }
            L.cs = L.cutm;
            walk_begin_chunk(L, prm, out);
            if constexpr (FOLD) fold_reset();
            if (!L.done) NL = (L.cs + a0) & kLineMask;
            RV = false;
        }
        if constexpr (LATE) {
            RL = L.done ? kWalkOob : NL;
            RV = !L.done;
            if (!L.done) NL += 128;
            dma(RL);
        }
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // the last (empty) DMA has landed before the slot goes away
    if (live) f.spec_cnt[sec] = L.n;
}

// ---------------------------------------------------------------- X: exact walk over W's lists
// X works in W's shifted form: table entries GEAR << 16 and masks << 16, so every mask bit sits in the
// high word of the hash and a test is one AND of that word (the walk path's masks are all at bit 16 or
// above; the host checks).
struct XMasks {
    uint32_t s, l;  // high words of mask_s << 16, mask_l << 16
};

// Truncated-window check of the chunk that starts at file position c: the first position in
// [c + a0, min(c + a0 + 47, c + eL)) whose hash -- started from 0 at a0, as cut_gear's is --
// matches its mask, or ~0 (then W's relaxed cut of c is the crate's cut).
__device__ uint64_t trunc_cut(const uint8_t* __restrict__ fbase, uint64_t flen, uint64_t c, const CdcParams& prm,
                              XMasks xm, const uint64_t* __restrict__ gear) {
    const uint64_t len = flen - c;
    if (len <= prm.min) return ~0ull;
    const uint64_t rem = len > prm.max ? prm.max : len;
    uint64_t center = prm.avg;
    if (len <= prm.max && len < center) center = len;
    const uint64_t a0 = prm.min & ~1ull, eS = center & ~1ull, eL = rem & ~1ull;
    const uint64_t tend = a0 + kHashSpan < eL ? a0 + kHashSpan : eL;
    const uint4 t0 = load16_file(fbase, c + a0, flen), t1 = load16_file(fbase, c + a0 + 16, flen),
                t2 = load16_file(fbase, c + a0 + 32, flen);
    uint64_t hsh = 0;
    uint32_t first = 0xFFFFFFFFu;
#pragma unroll
    for (int g = 0; g < 3; ++g) {  // 16 table reads together, then their rolls (bounded hoisting)
        const uint4 tw = g == 0 ? t0 : g == 1 ? t1 : t2;
        uint64_t G[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) G[j] = gear[byte_of(tw, j)];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int k = 16 * g + j;
            if (k < kHashSpan) {
                const uint64_t q = a0 + (uint64_t)k;
                hsh = (hsh << 1) + G[j];
                const uint32_t t = (uint32_t)(hsh >> 32) & (q < eS ? xm.s : xm.l);
                first = (t == 0 && q < tend && first == 0xFFFFFFFFu) ? (uint32_t)k : first;
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    return first == 0xFFFFFFFFu ? ~0ull : c + a0 + first;
}

// The exact length of the chunk that starts at file position p (cut_gear on content[p..]), computed by
// one wave: 4 KiB of positions per step (a chunk takes ~2 steps at 8 KiB), 64 per lane. A lane rolls
// the 48 bytes before its positions (the full window; lane 0 of the first step starts at a0 from 0,
// where cut_gear's hash starts), tests each position with one AND and keeps its first match.
__device__ uint64_t cut_coop(const uint8_t* __restrict__ fbase, uint64_t flen, uint64_t p, const CdcParams& prm,
                             XMasks xm, const uint64_t* __restrict__ gear) {
    const int lane = threadIdx.x & 63;
    const uint64_t len = flen - p;
    if (len <= prm.min) return len;
    const uint64_t rem = len > prm.max ? prm.max : len;
    uint64_t center = prm.avg;
    if (len <= prm.max && len < center) center = len;
    const uint64_t a0 = prm.min & ~1ull, eS = center & ~1ull, eL = rem & ~1ull;
    constexpr int kW = 64;  // positions per lane and step
    for (uint64_t W = a0; W < eL; W += 64 * kW) {
        const uint64_t q0 = W + (uint64_t)(kW * lane);
        // positions q0 .. q0+63 of this lane: mask_s below kS, tested below kL; the 48 bytes before
        // them give the full window (a0 >= 64: never before the chunk)
        const int kS = q0 >= eS ? 0 : (eS - q0 >= kW ? kW : (int)(eS - q0));
        const int kL = q0 >= eL ? 0 : (eL - q0 >= kW ? kW : (int)(eL - q0));
        const bool from0 = W == a0 && lane == 0;  // lane 0 of the first step: the hash starts at a0
        uint4 cur[7];
#pragma unroll
        for (int k = 0; k < 7; ++k) cur[k] = load16_file(fbase, p + q0 - 48 + 16 * (uint64_t)k, flen);
        // 16 bytes at a time: the word's 16 table reads go out together, then its 16 rolls (bounded
        // hoisting keeps the register count down)
        uint64_t h = 0;
        int zfirst = -1;
#pragma unroll
        for (int g = 0; g < 7; ++g) {
            uint64_t G[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) G[j] = gear[byte_of(cur[g], j)];
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                h = (h << 1) + G[j];
                const int k = 16 * g + j - 48;
                if (k >= 0) {
                    const uint32_t t = ((uint32_t)(h >> 32) & (k < kS ? xm.s : xm.l)) | (k < kL ? 0u : 1u);
                    zfirst = (t == 0 && zfirst < 0) ? k : zfirst;
                }
            }
            if (g == 2 && from0) h = 0;
            __builtin_amdgcn_sched_barrier(0);
        }
        const uint64_t any = __builtin_amdgcn_ballot_w64(zfirst >= 0);
        if (any) {
            const int first = __builtin_ctzll(any);
            const int k = __shfl(zfirst, first);
            return W + (uint64_t)(kW * first) + (uint64_t)k;
        }
    }
    return rem;
}

// One wave: the true chunk starts of section `sec` given its true entry e (file-relative, e >= the
// section start): W's list from e on wherever it is exact, cut_gear itself (cut_coop) where it is not.
// When e is on the list and every entry from there is exact, the section converged (emit reads W's
// list from k0, as in F3); otherwise the starts are written to `fix`.
__device__ void x_section(const CdcFiles& f, const CdcParams& prm, const CdcStitch& s, uint64_t sec, uint64_t e,
                          uint32_t* __restrict__ entry_used, const uint64_t* __restrict__ gear, XMasks xm,
                          uint32_t* __restrict__ lst, uint32_t* __restrict__ tcl) {
    const int lane = threadIdx.x & 63;
    const uint32_t file = f.sec_file[sec];
    const uint64_t flen = f.flen[file];
    const uint64_t sec0 = f.sec_base[file];
    const uint64_t S = (sec - sec0) * prm.sec;
    const uint64_t E = S + prm.sec < flen ? S + prm.sec : flen;
    const uint8_t* fbase = f.arena + f.foff[file];
    const uint32_t cnt = f.spec_cnt[sec];
    const uint32_t* spec = f.spec + sec * prm.speccap;
    const uint32_t nl = cnt < prm.speccap ? cnt : prm.speccap;  // W's lists never overflow (speccap bound)
    __syncthreads();  // lst / tcl of the previous section this wave walked are no longer read
    // every entry but the last (the exit): its truncated window
    for (uint32_t k = (uint32_t)lane; k < nl; k += 64) {
        const uint32_t rel = spec[k];
        lst[k] = rel;
        uint32_t tc = kNoCut;
        if (k + 1 < nl) {
            const uint64_t t = trunc_cut(fbase, flen, S + rel, prm, xm, gear);
            if (t != ~0ull) tc = (uint32_t)(t - S);
        }
        tcl[k] = tc;
    }
    __syncthreads();
    const uint32_t re = (uint32_t)(e - S);
    // e on the list? and the first inexact entry at or after it
    uint32_t k0 = kNoCut, kb = kNoCut;
    for (uint32_t b = 0; b < nl; b += 64) {
        const uint32_t k = b + (uint32_t)lane;
        const uint64_t hitm = __builtin_amdgcn_ballot_w64(k < nl && lst[k] == re);
        if (hitm && k0 == kNoCut) k0 = b + (uint32_t)__builtin_ctzll(hitm);
    }
    if (k0 != kNoCut) {
        for (uint32_t b = 0; b < nl; b += 64) {
            const uint32_t k = b + (uint32_t)lane;
            const uint64_t badm = __builtin_amdgcn_ballot_w64(k >= k0 && k + 1 < nl && tcl[k] != kNoCut);
            if (badm && kb == kNoCut) kb = b + (uint32_t)__builtin_ctzll(badm);
        }
    }
    if (lane == 0) entry_used[sec] = re;
    if (k0 != kNoCut && kb == kNoCut && cnt <= prm.speccap) {
        if (lane == 0) {
            s.status[sec] = kConverged;
            s.k0[sec] = k0;
            s.count[sec] = nl - 1 - k0;
            s.exit[sec] = S + lst[nl - 1];
        }
        return;
    }
    // the exact walk: follow W's list while it is exact, cut_gear where it is not
    uint32_t* fix = s.fix + sec * prm.speccap;
    auto lookup = [&](uint64_t pos) -> uint32_t {  // index of pos on the list, or kNoCut
        const uint32_t r = (uint32_t)(pos - S);
        uint32_t lo2 = 0, hi2 = nl;
        while (lo2 < hi2) {
            const uint32_t mid = (lo2 + hi2) >> 1;
            if (lst[mid] < r) lo2 = mid + 1;
            else hi2 = mid;
        }
        return lo2 < nl && lst[lo2] == r ? lo2 : kNoCut;
    };
    uint64_t p = e;
    uint32_t j = k0, n = 0;
    while (p < E) {
        if (j != kNoCut && j + 1 < nl) {
            // p = list entry j: entries j .. r-1 up to the next inexact one (r), all inside the section
            // (only the list's last entry, the exit, is past its end), are true starts: copied at once
            uint32_t r = nl - 1;
            for (uint32_t b = j; b < nl - 1; b += 64) {
                const uint32_t k = b + (uint32_t)lane;
                const uint64_t badm = __builtin_amdgcn_ballot_w64(k < nl - 1 && tcl[k] != kNoCut);
                if (badm) {
                    r = b + (uint32_t)__builtin_ctzll(badm);
                    break;
                }
            }
            for (uint32_t k = j + (uint32_t)lane; k < r; k += 64)
                if (n + (k - j) < prm.speccap) fix[n + (k - j)] = lst[k];
            n += r - j;
            p = S + lst[r];
            if (r == nl - 1) break;  // the exit
            // entry r is a true start whose truncated window cuts it short
            if (lane == 0 && n < prm.speccap) fix[n] = lst[r];
            ++n;
            p = S + tcl[r];
        } else {
            if (lane == 0 && n < prm.speccap) fix[n] = (uint32_t)(p - S);
            ++n;
            p += cut_coop(fbase, flen, p, prm, xm, gear);
        }
        j = lookup(p);
    }
    if (lane == 0) {
        s.status[sec] = kFixed;
        s.count[sec] = n;
        s.exit[sec] = p;
    }
}

__device__ __forceinline__ XMasks x_masks(const CdcParams& prm) {
    return XMasks{(uint32_t)((prm.mask_s << 16) >> 32), (uint32_t)((prm.mask_l << 16) >> 32)};
}

// X, first pass: every section (a grid-stride loop of one-wave workgroups), from the entry W's previous
// section ends at (0 for a file's first).
__global__ __launch_bounds__(64) void cdc_xwalk_kernel(CdcFiles f, CdcParams prm, CdcStitch s, uint64_t n_sec,
                                                       uint32_t* __restrict__ entry_used) {
    __shared__ uint64_t lds_gear[256];
    extern __shared__ uint32_t xl[];  // 2 * speccap u32: the list and each entry's truncated cut
    for (int i = threadIdx.x; i < 256; i += blockDim.x) lds_gear[i] = kGear[i] << 16;
    const XMasks xm = x_masks(prm);
    for (uint64_t sec = blockIdx.x; sec < n_sec; sec += gridDim.x) {
        const uint32_t file = f.sec_file[sec];
        const uint64_t sec0 = f.sec_base[file];
        const uint64_t e =
            sec == sec0 ? 0 : ((sec - 1 - sec0) * prm.sec + f.spec[(sec - 1) * prm.speccap + f.spec_cnt[sec - 1] - 1]);
        x_section(f, prm, s, sec, e, entry_used, lds_gear, xm, xl, xl + prm.speccap);
    }
}

// X, second pass: one wave per 64 sections finds those whose assumed entry is not the exit the first
// pass found for the section before them, and walks each of them again from that exit.
__global__ __launch_bounds__(64) void cdc_xretry_kernel(CdcFiles f, CdcParams prm, CdcStitch s, uint64_t n_sec,
                                                        uint32_t* __restrict__ entry_used) {
    __shared__ uint64_t lds_gear[256];
    extern __shared__ uint32_t xl[];
    const int lane = threadIdx.x;
    const uint64_t sec = (uint64_t)blockIdx.x * 64 + (uint64_t)lane;
    bool redo = false;
    if (sec < n_sec) {
        const uint32_t file = f.sec_file[sec];
        const uint64_t sec0 = f.sec_base[file];
        if (sec != sec0) redo = s.exit[sec - 1] != (sec - sec0) * prm.sec + entry_used[sec];
    }
    uint64_t m = __builtin_amdgcn_ballot_w64(redo);
    if (m == 0) return;
    for (int i = threadIdx.x; i < 256; i += blockDim.x) lds_gear[i] = kGear[i] << 16;
    const XMasks xm = x_masks(prm);
    while (m) {
        const uint64_t t = (uint64_t)blockIdx.x * 64 + (uint64_t)__builtin_ctzll(m);
        m &= m - 1;
        x_section(f, prm, s, t, s.exit[t - 1], entry_used, lds_gear, xm, xl, xl + prm.speccap);
    }
}

// X, last resort: one wave per file walks its sections in order and redoes every one whose entry is
// not the exit the section before it ended at (after a redo, the next section is checked again).
__global__ __launch_bounds__(64) void cdc_xfix_kernel(CdcFiles f, CdcParams prm, CdcStitch s, uint64_t n_files,
                                                      uint32_t* __restrict__ entry_used) {
    __shared__ uint64_t lds_gear[256];
    extern __shared__ uint32_t xl[];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) lds_gear[i] = kGear[i] << 16;
    __syncthreads();
    const uint64_t file = blockIdx.x;
    if (file >= n_files) return;
    const XMasks xm = x_masks(prm);
    const int lane = threadIdx.x;
    const uint64_t sec0 = f.sec_base[file], nsec = f.sec_base[file + 1] - sec0;
    uint64_t i = 1;
    while (i < nsec) {
        const uint64_t j = i + (uint64_t)lane;
        bool bad = false;
        if (j < nsec) {
            const uint64_t ex = __atomic_load_n(&s.exit[sec0 + j - 1], __ATOMIC_RELAXED);
            const uint32_t eu = __atomic_load_n(&entry_used[sec0 + j], __ATOMIC_RELAXED);
            bad = ex != j * prm.sec + eu;
        }
        const uint64_t mbad = __builtin_amdgcn_ballot_w64(bad);
        if (mbad == 0) {
            i += 64;
            continue;
        }
        i += (uint64_t)__builtin_ctzll(mbad);
        const uint64_t e = __atomic_load_n(&s.exit[sec0 + i - 1], __ATOMIC_RELAXED);
        x_section(f, prm, s, sec0 + i, e, entry_used, lds_gear, xm, xl, xl + prm.speccap);
        __threadfence();
        ++i;
    }
}

}  // namespace oxh

// ---------------------------------------------------------------- host side
namespace {

int cdc_fail(int code, const std::string& msg) { return oxh::set_error(code, msg); }

#define CDC_HIP(expr)                                                                          \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess) return cdc_fail(OXH_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

uint32_t log2_round(uint32_t v) {
    const uint32_t b = 31 - (uint32_t)__builtin_clz(v);
    const double x = (double)v, lo = (double)(1u << b);
    return (x * x >= 2.0 * lo * lo) ? b + 1 : b;
}

// Per-call scratch (candidate lists, speculative starts, stitch tables) carved out of the device's
// cached scratch buffer (scratch.hpp).
struct Scratch {
    oxh::ScratchLease lease;
    std::vector<std::pair<void**, uint64_t>> parts;
    explicit Scratch(hipStream_t s) : lease(s) {}
    template <class T>
    void want(T** p, uint64_t count) {
        parts.push_back({(void**)p, (std::max<uint64_t>(count, 1) * sizeof(T) + 255) & ~255ull});
    }
    hipError_t commit() {
        uint64_t total = 0;
        for (auto& q : parts) total += q.second;
        void* base = nullptr;
        const hipError_t e = lease.get(total, &base);
        if (e != hipSuccess) return e;
        uint64_t off = 0;
        for (auto& q : parts) {
            *q.first = (uint8_t*)base + off;
            off += q.second;
        }
        return hipSuccess;
    }
};

}  // namespace

extern "C" {

int oxh_fastcdc_gear(uint64_t* out256) {
    if (!out256) return cdc_fail(OXH_ERR_INVALID, "null output");
    memcpy(out256, oxh::kGear, sizeof(oxh::kGear));
    return OXH_OK;
}

int oxh_fastcdc_masks(uint32_t avg_size, uint32_t level, uint64_t* mask_s, uint64_t* mask_l) {
    if (avg_size < 256 || avg_size > 4194304 || level > 3)
        return cdc_fail(OXH_ERR_INVALID, "avg_size must be in [256, 4194304] and level in 0..3");
    const uint32_t bits = log2_round(avg_size);
    if (mask_s) *mask_s = oxh::kCdcMasks[bits + level];
    if (mask_l) *mask_l = oxh::kCdcMasks[bits - level];
    return OXH_OK;
}

uint64_t oxh_fastcdc_max_chunks(const uint64_t* lens, uint64_t n, uint32_t min_size) {
    uint64_t t = 0;
    for (uint64_t i = 0; i < n; ++i) t += lens[i] ? (lens[i] + min_size - 1) / std::max<uint32_t>(min_size, 1) : 0;
    return t;
}

int oxh_fastcdc_device(const void* d_arena, const uint64_t* offsets, const uint64_t* lens, uint64_t n,
                       uint32_t min_size, uint32_t avg_size, uint32_t max_size, uint32_t level,
                       uint64_t* d_chunk_offsets, uint64_t* d_chunk_lens, uint64_t* d_digests, uint64_t capacity,
                       uint64_t* first_chunk, void* stream) {
    // v2020::FastCDC::with_level asserts (crate fastcdc 3.2.1)
    if (min_size < 64 || min_size > 1048576) return cdc_fail(OXH_ERR_INVALID, "min_size must be in [64, 1048576]");
    if (avg_size < 256 || avg_size > 4194304) return cdc_fail(OXH_ERR_INVALID, "avg_size must be in [256, 4194304]");
    if (max_size < 1024 || max_size > 16777216) return cdc_fail(OXH_ERR_INVALID, "max_size must be in [1024, 16777216]");
    if (level > 3) return cdc_fail(OXH_ERR_INVALID, "normalization level must be 0..3");
    if (n > 0 && (!d_arena || !offsets || !lens || !first_chunk)) return cdc_fail(OXH_ERR_INVALID, "null argument");
    if (!first_chunk) return cdc_fail(OXH_ERR_INVALID, "null first_chunk");
    hipStream_t st = (hipStream_t)stream;
    first_chunk[0] = 0;
    if (n == 0) return OXH_OK;

    oxh::CdcParams prm{};
    prm.min = min_size;
    prm.avg = avg_size;
    prm.max = max_size;
    int rc = oxh_fastcdc_masks(avg_size, level, &prm.mask_s, &prm.mask_l);
    if (rc) return rc;
    // F1 records a 16-byte group wherever the bits both masks share are clear at one of its bytes:
    // ~16 * 2^-popcount(common) groups per 16 bytes. Store 8x the expected count (+8) per list unit
    // (sec / 64 bytes), at most one per group; a denser unit keeps a truncated list and the walk
    // scans its bytes (C5 at 8 KiB: 2 expected per 8 KiB unit, 24 stored: P(overflow) ~ 1e-16).
    const double dens = std::min(1.0, 16.0 * std::ldexp(1.0, -__builtin_popcountll(prm.mask_s & prm.mask_l))) / 16.0;
    // sections of at least `max` bytes: a chunk never spans a whole section (F3's invariant)
    // Speculative walks meet the true walk after ~1.5 chunks (median) and within 6 chunks in 99 % of
    // random starts (measured with the oracle). Warm-up: 6 max-sized chunks, at least 128 KiB (r02
    // sweep, walk + fixup: 64 KiB chunks 2.57 / 2.09 / 2.18 ms at 512 / 768 / 1024 KiB; 8 KiB chunks
    // 3.95 / 3.89 / 4.06 / 4.43 ms at 96 / 128 / 192 / 256 KiB);
    // sections: at least 8 max-sized chunks and 512 KiB. Every section whose walk has not met the
    // true one is re-walked serially by F3, so at small chunk sizes the longer warm-up pays for itself
    // (C5 at 8 KiB: 57.2 ms vs 63.8 ms with 256 KiB sections and 64 KiB of warm-up; at 64 KiB: 53.8
    // vs 54.9 ms with 1 MiB sections; tools/bench_fastcdc.py sweeps).
    const uint64_t max_rounded = ((uint64_t)max_size + 1023) / 1024 * 1024;
    uint64_t total_bytes = 0, arena_bytes = 0;
    for (uint64_t i = 0; i < n; ++i) {
        total_bytes += lens[i];
        arena_bytes = std::max<uint64_t>(arena_bytes, offsets[i] + lens[i]);
    }
    // The walk path (W + X, DESIGN §4 "F1 -> W"): chosen where it rolls fewer bytes than F1 -- small
    // chunks, where the skipped `min` bytes are a large share (61 % rolled at 8 KiB, 94 % at 64 KiB) --
    // and where its layout rules hold: masks at bit 16 or above, a 128-B aligned arena, every wave's 64
    // sections inside one 4 GiB window, and X's per-section lists within a workgroup's LDS (checked
    // below; where one does not hold the call takes the scan). OXH_CDC_WALK=0 / 1 forces it off / on.
    const char* walk_env = getenv("OXH_CDC_WALK");
    const bool walk_forced = walk_env && atoi(walk_env) != 0;
    bool walk = (((prm.mask_s | prm.mask_l) & 0xFFFFull) == 0) && (((uintptr_t)d_arena & 127) == 0) &&
                (walk_env ? walk_forced : (avg_size <= 16384));
    if (walk_forced && !walk) return cdc_fail(OXH_ERR_INVALID, "OXH_CDC_WALK=1: masks below bit 16 or an unaligned arena");
    int dev = 0;
    (void)hipGetDevice(&dev);
    int max_lds = 0;
    if (hipDeviceGetAttribute(&max_lds, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess) max_lds = 64 * 1024;
    std::vector<uint64_t> sec_base(n + 1);
    uint64_t n_sec = 0;
    for (;;) {
        prm.sec = oxh::kSecDefault;
        if (const char* e = getenv("OXH_CDC_SECTION_BYTES")) {  // tests: many small sections per file
            const uint64_t v = strtoull(e, nullptr, 10);
            if (v >= 1024 && v % 1024 == 0 && v <= (1u << 30)) prm.sec = v;
        }
        prm.warmup = std::max<uint64_t>(6 * (uint64_t)max_size, 128 * 1024);
        if (walk) {
            // one lane per section, one generation of 12-wave workgroups on every CU: sections as large
            // as that allows (fewer sections = less warm-up and stitching), whole 8 KiB, at least 4 max
            int cus = 256;
            if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
            const uint64_t lanes = (uint64_t)cus * oxh::kScanWaves * 64;
            const uint64_t want = (total_bytes + lanes - 1) / std::max<uint64_t>(lanes, 1);
            if (!getenv("OXH_CDC_SECTION_BYTES")) prm.sec = std::max<uint64_t>({want, 4 * max_rounded, 64 * 1024});
            // warm-up: a relaxed walk started anywhere lands on the true one within 14 / 37 / 67 KB in 50 /
            // 90 / 99 % of starts at 8 KiB chunks (C restatement, 1 GiB); X re-walks the sections whose
            // warm-up was too short, so it is kept short: two max-sized chunks
            prm.warmup = 2 * (uint64_t)max_size;
        }
        if (prm.sec < max_rounded) prm.sec = max_rounded;
        if (!walk && !getenv("OXH_CDC_SECTION_BYTES") && prm.sec < 8 * max_rounded) prm.sec = 8 * max_rounded;
        prm.sec = (prm.sec + 8191) / 8192 * 8192;  // 64 F1 units of whole 128-byte rounds
        // a candidate entry holds the group index in 17 bits: units of at most 2 MiB (sections of 128 MiB,
        // 8 chunks of the crate's largest max); the test-only section override is clamped to that
        prm.sec = std::min<uint64_t>(prm.sec, 128ull << 20);
        if (prm.sec < max_rounded) return cdc_fail(OXH_ERR_INVALID, "section override below max_size");
        prm.unit = prm.sec / 64;
        if (const char* e = getenv("OXH_CDC_WARMUP_BYTES")) prm.warmup = strtoull(e, nullptr, 10);  // tests
        prm.cap = (uint32_t)std::min<double>(prm.unit / 16, 8.0 * dens * prm.unit + 8);
        if (const char* e = getenv("OXH_CDC_UNIT_CAP")) prm.cap = std::max(1, atoi(e));  // tests: force overflow
        prm.speccap = (uint32_t)(prm.sec / min_size + 2 + (max_size + min_size - 1) / min_size);

        sec_base[0] = 0;
        for (uint64_t i = 0; i < n; ++i) sec_base[i + 1] = sec_base[i] + (lens[i] + prm.sec - 1) / prm.sec;
        n_sec = sec_base[n];
        if (!walk) break;
        // X keeps a section's start list and fix list in dynamic LDS beside its static gear table
        std::string why;
        if (2 * (uint64_t)prm.speccap * sizeof(uint32_t) + oxh::kXStaticLds > (uint64_t)max_lds)
            why = "X's section lists do not fit the workgroup's LDS";
        // every wave's lanes must address their streams from one buffer resource: the lowest start
        // (warm-up included) to the highest byte a lane may read (its section end + two max chunks,
        // or its file end) within 4 GiB - 1 MiB
        for (uint64_t w0s = 0, f = 0; w0s < n_sec && why.empty(); w0s += 64) {
            uint64_t lo = ~0ull, hi = 0;
            for (uint64_t sct = w0s; sct < std::min<uint64_t>(n_sec, w0s + 64); ++sct) {
                while (sec_base[f + 1] <= sct) ++f;
                const uint64_t ss = (sct - sec_base[f]) * prm.sec;
                const uint64_t a = offsets[f] + (ss > prm.warmup ? ss - prm.warmup : 0);
                const uint64_t b = offsets[f] + std::min<uint64_t>(lens[f], ss + prm.sec + 2 * prm.max + 4096);
                lo = std::min(lo, a);
                hi = std::max(hi, b);
            }
            if (hi - (lo & ~127ull) + 256 >= 0xFFFFFF00ull - (1ull << 20)) why = "a wave's sections span 4 GiB";
        }
        if (why.empty()) break;
        if (walk_forced) return cdc_fail(OXH_ERR_INVALID, "OXH_CDC_WALK=1: " + why);
        walk = false;  // the scan, with its own section plan
    }

    // OXH_TRACE=1: host-side stage times of this call on stderr
    static const bool trace = getenv("OXH_TRACE") != nullptr;
    const auto t_start = std::chrono::steady_clock::now();
    auto since = [&] { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count(); };
    Scratch sc(st);
    uint64_t *d_foff, *d_flen, *d_sec_base, *d_first, *d_exit, *d_out_base;
    uint32_t *d_sec_file, *d_spec, *d_spec_cnt, *d_status, *d_k0, *d_count, *d_fix;
    uint64_t* d_cand_occ;
    oxh::CandRec* d_cand;
    sc.want(&d_foff, n);
    sc.want(&d_flen, n);
    sc.want(&d_sec_base, n + 1);
    sc.want(&d_first, n + 1);
    uint32_t* d_entry = nullptr;
    sc.want(&d_sec_file, n_sec);
    if (walk) {
        d_cand = nullptr, d_cand_occ = nullptr;
        sc.want(&d_entry, n_sec);
    } else {
        sc.want(&d_cand, n_sec * 64 * prm.cap);
        sc.want(&d_cand_occ, n_sec);
    }
    sc.want(&d_spec, n_sec * prm.speccap);
    sc.want(&d_spec_cnt, n_sec);
    sc.want(&d_status, n_sec);
    sc.want(&d_k0, n_sec);
    sc.want(&d_count, n_sec);
    sc.want(&d_exit, n_sec);
    sc.want(&d_fix, n_sec * prm.speccap);
    sc.want(&d_out_base, n_sec + 1);
    // W2 (the walk with K1's block sums folded in) + K1F: OXH_CDC_FOLD=1 in the probe build
    // (tools/build_probe_lib.py, -DOXH_PROBE_FOLD), on the walk path with digests asked for and `min` a
    // whole number of 1 KiB blocks (C5: min 4 KiB). Sums: 64 B per KiB of arena. It measured 55.4 ms
    // for C5 at 8 KiB against 43.5 for W + K1R (DESIGN §4 "W2"), so the shipped library does not take it.
#ifdef OXH_PROBE_FOLD
    const bool fold_env = getenv("OXH_CDC_FOLD") && atoi(getenv("OXH_CDC_FOLD")) != 0;
#else
    const bool fold_env = false;  // measured and not kept (DESIGN §4 "W2"): the probe build has it
#endif
    const bool fold = fold_env && walk && d_digests && capacity && min_size % 1024 == 0;
    uint64_t* d_sums = nullptr;
    uint8_t* d_flag = nullptr;
    if (fold) {
        sc.want(&d_sums, ((arena_bytes >> 10) + 4) * 8);
        sc.want(&d_flag, capacity);
    }
    CDC_HIP(sc.commit());
    const double t_malloc = since();
    CDC_HIP(hipMemcpyAsync(d_foff, offsets, n * 8, hipMemcpyHostToDevice, st));
    CDC_HIP(hipMemcpyAsync(d_flen, lens, n * 8, hipMemcpyHostToDevice, st));
    CDC_HIP(hipMemcpyAsync(d_sec_base, sec_base.data(), (n + 1) * 8, hipMemcpyHostToDevice, st));
    if (n_sec) {
        hipLaunchKernelGGL(oxh::cdc_sec_file_kernel, dim3((unsigned)((n_sec + 255) / 256)), dim3(256), 0, st, d_sec_base, n,
                           n_sec, d_sec_file);
        CDC_HIP(hipGetLastError());
    }

    const double t_alloc = since();
    oxh::CdcFiles f{(const uint8_t*)d_arena, d_foff, d_flen, d_sec_base, d_sec_file, d_cand, d_cand_occ, d_spec, d_spec_cnt};
    oxh::CdcStitch sti{d_status, d_k0, d_count, d_exit, d_fix, d_out_base};
    if (n_sec && walk) {
        // W: one lane per section; X twice (every section, then the ones whose assumed entry turned out
        // wrong); the serial pass for whatever is left; then the chunk counts' prefix
        const uint64_t nwaves = (n_sec + 63) / 64;
        static const bool late = getenv("OXH_CDC_WALK_LATE") && atoi(getenv("OXH_CDC_WALK_LATE")) != 0;
        auto walk_kernel = late ? oxh::cdc_walk_scan_kernel<oxh::kScanWaves, true> : oxh::cdc_walk_scan_kernel<oxh::kScanWaves, false>;
#ifdef OXH_PROBE_FOLD
        if (fold) walk_kernel = oxh::cdc_walk_scan_kernel<oxh::kScanWaves, false, true>;
#endif
        hipLaunchKernelGGL(walk_kernel,
                           dim3((unsigned)((nwaves + oxh::kScanWaves - 1) / oxh::kScanWaves)), dim3(64 * oxh::kScanWaves), 0, st,
                           f, prm, n_sec, oxh::WalkGeom{arena_bytes, d_sums});
        CDC_HIP(hipGetLastError());
        const size_t xlds = 2 * (size_t)prm.speccap * sizeof(uint32_t);
        static const unsigned xgrid = getenv("OXH_CDC_X_WGS") ? (unsigned)atoi(getenv("OXH_CDC_X_WGS")) : 16384u;
        hipLaunchKernelGGL(oxh::cdc_xwalk_kernel, dim3((unsigned)std::min<uint64_t>(n_sec, xgrid)), dim3(64), xlds, st, f, prm,
                           sti, n_sec, d_entry);
        CDC_HIP(hipGetLastError());
        hipLaunchKernelGGL(oxh::cdc_xretry_kernel, dim3((unsigned)((n_sec + 63) / 64)), dim3(64), xlds, st, f, prm, sti, n_sec,
                           d_entry);
        CDC_HIP(hipGetLastError());
        hipLaunchKernelGGL(oxh::cdc_xfix_kernel, dim3((unsigned)n), dim3(64), xlds, st, f, prm, sti, n, d_entry);
        CDC_HIP(hipGetLastError());
        hipLaunchKernelGGL(oxh::cdc_prefix_kernel, dim3(1), dim3(1024), 0, st, sti, n_sec);
        CDC_HIP(hipGetLastError());
    } else if (n_sec) {
        // F1: one wave per section (kScanWaves per workgroup, 160 KiB of LDS); SH when the bits both
        // masks share are all >= 16
        const bool sh = (((prm.mask_s & prm.mask_l) << 16) & 0xFFFFFFFFull) == 0;
        static const int waves = getenv("OXH_CDC_SCAN_WAVES") ? atoi(getenv("OXH_CDC_SCAN_WAVES")) : oxh::kScanWaves;
        auto scan = waves == 8 ? (sh ? oxh::cdc_scan_kernel<true, 8> : oxh::cdc_scan_kernel<false, 8>)
                               : (sh ? oxh::cdc_scan_kernel<true, 12> : oxh::cdc_scan_kernel<false, 12>);
        const int wv = waves == 8 ? 8 : 12;
        hipLaunchKernelGGL(scan, dim3((unsigned)((n_sec + wv - 1) / wv)), dim3(64 * wv), 0, st, f, prm, n_sec);
        CDC_HIP(hipGetLastError());
        hipLaunchKernelGGL(oxh::cdc_walk_kernel, dim3((unsigned)((n_sec + 255) / 256)), dim3(256), 0, st, f, prm, n_sec);
        CDC_HIP(hipGetLastError());
        hipLaunchKernelGGL(oxh::cdc_check_kernel, dim3((unsigned)((n_sec + 255) / 256)), dim3(256), 0, st, f, prm, sti, n_sec);
        CDC_HIP(hipGetLastError());
        hipLaunchKernelGGL(oxh::cdc_fixup_kernel, dim3((unsigned)n), dim3(64), 0, st, f, prm, sti, n);
        CDC_HIP(hipGetLastError());
        hipLaunchKernelGGL(oxh::cdc_prefix_kernel, dim3(1), dim3(1024), 0, st, sti, n_sec);
        CDC_HIP(hipGetLastError());
    } else {
        CDC_HIP(hipMemsetAsync(d_out_base, 0, 8, st));
    }
    hipLaunchKernelGGL(oxh::cdc_first_kernel, dim3((unsigned)((n + 256) / 256)), dim3(256), 0, st, d_sec_base, d_out_base, n,
                       d_first);
    CDC_HIP(hipGetLastError());
    CDC_HIP(hipMemcpyAsync(first_chunk, d_first, (n + 1) * 8, hipMemcpyDeviceToHost, st));
    const double t_launch = since();
    CDC_HIP(hipStreamSynchronize(st));
    if (trace)
        fprintf(stderr, "[oxh] fastcdc: %s sections=%llu (%llu B, warm-up %llu B) malloc=%.4fs copy=%.4fs launch=%.4fs "
                "chunking=%.4fs scratch=%.2fGiB\n", walk ? "walk" : "scan", (unsigned long long)n_sec,
                (unsigned long long)prm.sec, (unsigned long long)prm.warmup, t_malloc, t_alloc - t_malloc, t_launch - t_alloc,
                since(), sc.lease.size() / 1073741824.0);
    const uint64_t total = first_chunk[n];
    if (total > capacity)
        return cdc_fail(OXH_ERR_INVALID, "chunk capacity too small: need " + std::to_string(total) + " entries");
    if (total && (!d_chunk_offsets || !d_chunk_lens)) return cdc_fail(OXH_ERR_INVALID, "null chunk table");
    if (n_sec) {
        hipLaunchKernelGGL(oxh::cdc_emit_kernel, dim3((unsigned)((n_sec + 3) / 4)), dim3(256), 0, st, f, prm, sti, n_sec,
                           d_chunk_offsets, d_chunk_lens, fold ? d_flag : nullptr);
        CDC_HIP(hipGetLastError());
    }
    if (d_digests && total) {
        // chunks sit back to back at arbitrary byte offsets: K1R at small chunks, the block-wise K1
        // otherwise (oxh::k1_packed)
        uint64_t bytes = 0;
        for (uint64_t i = 0; i < n; ++i) bytes += lens[i];
        if (fold) {  // K1F: blocks 0-3 and the tail from the bytes, blocks 4.. from W2's sums
#ifdef OXH_PROBE_FOLD
            hipLaunchKernelGGL(oxh::xxh3_rows_fold_kernel, dim3((unsigned)((total + 7) / 8)), dim3(128), 0, st,
                               (const uint8_t*)d_arena, d_chunk_offsets, d_chunk_lens, total, d_digests, d_sums, d_flag);
#endif
            rc = hipGetLastError() == hipSuccess ? OXH_OK : OXH_ERR_HIP;
            if (rc) oxh::set_error(rc, "K1F launch");
        } else {
            rc = oxh::k1_packed(d_arena, d_chunk_offsets, d_chunk_lens, total, d_digests, bytes / total, st);
        }
        if (rc) return cdc_fail(rc, std::string("chunk digests: ") + oxh_last_error());
    }
    CDC_HIP(hipStreamSynchronize(st));
    return OXH_OK;
}

}  // extern "C"

