// tools/cdc_segment_probe.hip -- FastCDC scan (F1) redesign probe: per-lane segments, no transpose.
//
// F1 today folds 16 bytes per lane of a 1 KiB sub-block: every byte pays two 64-bit shift-adds (the
// lane-local hash and the chained one) and ~6.4 VALU in all. Here lane l owns a contiguous segment of
// S bytes of its wave's 64*S-byte sub-block and rolls ONE hash through it, starting 48 bytes before
// the segment (warm-up, untested: only the last 48 bytes reach the masked bits), so a byte costs
//   1 v_perm_b32 (LDS address = byte << 8 | copy offset, the table is stored 32 times, entry k of copy
//     c at byte 256k + 8c, so the 32 lanes of a ds_read_b64 group never share a bank)
// + 1 ds_read_b64 + 1 v_lshl_add_u64 + 1 v_and_b32 + 1/2 v_min3_u32,
// with a (48 / S) warm-up overhead. Loads: lane l reads its own 128 B per chunk (8 x 16 B); each
// wave-load instruction touches 64 lines that the next 7 reuse (L1 hits unless the load is
// non-temporal), so FLAG selects the cache policy. Counts candidate groups only (the scan rate).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/cdc_segment_probe.hip -o /tmp/seg && /tmp/seg [GiB]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "../oxen_amd/csrc/fastcdc_gear.h"

constexpr uint32_t kSec = 512 * 1024;
constexpr uint32_t kPad = 256;  // bytes before the first section (warm-up reads of section 0)

__global__ void fill(uint64_t* p, uint64_t n, uint64_t seed) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// S: segment bytes per lane (multiple of 128). FLAG: buffer-load cache policy (0 default, 2 nt).
// D: chunks (128 B per lane) in flight. COMPUTE=false: loads only (the access pattern's rate).
template <uint32_t S, int WAVES, int FLAG, int D, bool COMPUTE>
__global__ __launch_bounds__(64 * WAVES) void seg_scan(const uint8_t* __restrict__ data, uint64_t n_sec, uint32_t ch,
                                                     unsigned long long* __restrict__ count) {
    __shared__ uint64_t gear_tab[256 * 32];
    for (int i = threadIdx.x; i < 256 * 32; i += blockDim.x) gear_tab[i] = oxh::kGear[i >> 5] << 16;
    __syncthreads();
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t sec = (uint64_t)blockIdx.x * WAVES + w;
    if (sec >= n_sec) return;
    constexpr uint32_t kSub = 64 * S, nsub = kSec / kSub, nch = S / 128, nchunks = nsub * nch;
    // the resource starts kPad bytes before the section so that warm-up offsets stay unsigned
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void*)(data + sec * kSec - kPad), (short)0, (int)(kSec + kPad), 0x00020000);
    const uint32_t copy_off = (uint32_t)(lane & 31) * 8;
    auto load_chunk = [&](uint32_t c, uint4 (&dst)[8]) {
        const uint32_t sub = c / nch, r = c % nch;
        const uint32_t seg = sub * kSub + (uint32_t)lane * S + kPad;
        const bool live = c < nchunks;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, live ? seg + r * 128 + 16 * k : 0xFFFFF000u, 0, FLAG);
            dst[k] = make_uint4(v.x, v.y, v.z, v.w);
        }
    };
    // the 48 bytes before the lane's segment of sub-block `sub` (loaded when the segment starts)
    auto load_warm = [&](uint32_t sub, uint4 (&dst)[3]) {
        const uint32_t seg = sub * kSub + (uint32_t)lane * S + kPad;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, seg - 48 + 16 * k, 0, FLAG);
            dst[k] = make_uint4(v.x, v.y, v.z, v.w);
        }
    };
    const char* tab = (const char*)gear_tab;
    auto gear = [&](uint32_t word, int j) -> uint64_t {
        const uint32_t a = __builtin_amdgcn_perm(word, copy_off, 0x0c0c0000u | ((4u + (uint32_t)j) << 8));
        return *(const uint64_t*)(tab + a);
    };
    uint64_t h = 0;
    uint32_t cnt = 0, sink = 0;
    uint4 ring[D][8];
#pragma unroll
    for (int d = 0; d < D; ++d) load_chunk((uint32_t)d, ring[d]);
#pragma unroll 1
    for (uint32_t c = 0; c < nchunks; c += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const uint32_t r = (c + d) % nch;
            if constexpr (COMPUTE) {
                // the gathers of word i + P are issued before word i is rolled (P words = 4P reads in
                // flight, lgkmcnt <= 15), so the LDS latency hides behind the roll
                constexpr int P = 3;
                auto roll_words = [&](auto nw_tag, const uint32_t* wv, bool test) {
                    constexpr int NW = decltype(nw_tag)::value;
                    uint64_t G[P + 1][4];
#pragma unroll
                    for (int i = 0; i < P && i < NW; ++i)
#pragma unroll
                        for (int b = 0; b < 4; ++b) G[i][b] = gear(wv[i], b);
                    uint32_t anyz = 0xFFFFFFFFu;
#pragma unroll
                    for (int i = 0; i < NW; ++i) {
                        if (i + P < NW) {
#pragma unroll
                            for (int b = 0; b < 4; ++b) G[(i + P) % (P + 1)][b] = gear(wv[i + P], b);
                        }
                        __builtin_amdgcn_sched_barrier(0);
                        const uint64_t* g = G[i % (P + 1)];
                        h = (h << 1) + g[0];
                        const uint32_t t0 = (uint32_t)(h >> 32) & ch;
                        h = (h << 1) + g[1];
                        const uint32_t t1 = (uint32_t)(h >> 32) & ch;
                        h = (h << 1) + g[2];
                        const uint32_t t2 = (uint32_t)(h >> 32) & ch;
                        h = (h << 1) + g[3];
                        const uint32_t t3 = (uint32_t)(h >> 32) & ch;
                        if (test) {
                            const uint32_t m01 = t0 < t1 ? t0 : t1, m23 = t2 < t3 ? t2 : t3;
                            const uint32_t m = m01 < m23 ? m01 : m23;
                            anyz = anyz < m ? anyz : m;
                            if ((i & 3) == 3) {
                                cnt += anyz == 0;
                                anyz = 0xFFFFFFFFu;
                            }
                        }
                        __builtin_amdgcn_sched_barrier(0);
                    }
                };
                if (r == 0) {
                    h = 0;
                    uint4 wq[3];
                    load_warm((c + d) / nch, wq);
                    uint32_t wv[12];
#pragma unroll
                    for (int k = 0; k < 3; ++k) {
                        wv[4 * k] = wq[k].x, wv[4 * k + 1] = wq[k].y;
                        wv[4 * k + 2] = wq[k].z, wv[4 * k + 3] = wq[k].w;
                    }
                    roll_words(std::integral_constant<int, 12>{}, wv, false);
                }
                uint32_t wv[32];
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    wv[4 * k] = ring[d][k].x, wv[4 * k + 1] = ring[d][k].y;
                    wv[4 * k + 2] = ring[d][k].z, wv[4 * k + 3] = ring[d][k].w;
                }
                roll_words(std::integral_constant<int, 32>{}, wv, true);
            } else {
#pragma unroll
                for (int g = 0; g < 8; ++g) sink ^= ring[d][g].x ^ ring[d][g].w;
                if (r == 0) {
                    uint4 wq[3];
                    load_warm((c + d) / nch, wq);
                    sink ^= wq[0].x ^ wq[2].w;
                }
            }
            load_chunk(c + d + D, ring[d]);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    if (!COMPUTE) cnt = sink == 0x12345678u;
    atomicAdd(count, (unsigned long long)cnt);
}

// Lane-major with LDS-DMA staging: lane l owns region l (8 KiB) of its wave's 512 KiB section. A round
// is 128 B of every region: 8 `buffer_load_dwordx4 ... lds` (lanes 8m..8m+7 of DMA k fetch one whole
// 128-B line of region 8k+m, so every line is fetched once and the loads stay coalesced) land region
// r's bytes at slot + 128 r; lane r then reads its 128 B with 8 conflict-free ds_read_b128 (piece q of
// lane r sits at position (q + (r >> 1)) & 7 of its line: the DMA lanes fetch their pieces rotated so
// that the 16 lanes of every ds_read_b128 group cover the 64 banks once). No VGPR round trip for the
// staging (a ds_write_b128 costs 13 cycles), and the LDS beside the slots holds the 32-copy gear table.
template <int W, int SLOTS>
__global__ __launch_bounds__(64 * W) void lm_dma(const uint8_t* __restrict__ data, uint64_t n_sec, uint32_t ch,
                                                 unsigned long long* __restrict__ count) {
    // one LDS block: the gear table at address 0 (so a gather address is a single v_perm), the slots after
    __shared__ __attribute__((aligned(16))) uint64_t lds_raw[256 * 32 + W * SLOTS * 1024];
    uint64_t* gear_tab = lds_raw;
    typedef uint4 Slot[512];
    Slot* stage_w = (Slot*)(lds_raw + 256 * 32) + W * 0;
    for (int i = threadIdx.x; i < 256 * 32; i += blockDim.x) gear_tab[i] = oxh::kGear[i >> 5] << 16;
    __syncthreads();
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t sec = (uint64_t)blockIdx.x * W + w;
    if (sec >= n_sec) return;
    constexpr uint32_t kReg = kSec / 64, kRounds = kReg / 128;
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void*)(data + sec * kSec - kPad), (short)0, (int)(kSec + kPad), 0x00020000);
    const uint32_t copy_off = (uint32_t)(lane & 31) * 8;
    // DMA k, lane i = 8m + j: region r = 8k + m, piece (j - ((r >> 1) & 7)) & 7
    const int m = lane >> 3, j = lane & 7;
    auto dma_round = [&](uint32_t t, int slot) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t r = 8 * k + m;
            const uint32_t piece = (uint32_t)(j - (int)((r >> 1) & 7)) & 7;
            const uint32_t off = kPad + r * kReg + 16 * piece;
            // rounds past the end: a uniform soffset beyond the range makes the DMA a no-op
            const uint32_t soff = t < kRounds ? t * 128 : 0x40000000u;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void*)&stage_w[w * SLOTS + slot][64 * k],
                                                     16, off, soff, 0, 0);
        }
    };
    const char* tab = (const char*)gear_tab;
    auto gear = [&](uint32_t word, int jj) -> uint64_t {
        const uint32_t a = __builtin_amdgcn_perm(word, copy_off, 0x0c0c0000u | ((4u + (uint32_t)jj) << 8));
        return *(const uint64_t*)(tab + a);
    };
    uint64_t h = 0;
    uint32_t cnt = 0;
    // warm-up: the 48 bytes before the region
    {
        uint32_t wv[12];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, kPad + (uint32_t)lane * kReg - 48 + 16 * k, 0, 0);
            wv[4 * k] = v.x, wv[4 * k + 1] = v.y, wv[4 * k + 2] = v.z, wv[4 * k + 3] = v.w;
        }
#pragma unroll
        for (int i = 0; i < 12; ++i)
#pragma unroll
            for (int b = 0; b < 4; ++b) h = (h << 1) + gear(wv[i], b);
    }
#pragma unroll
    for (int s = 0; s < SLOTS; ++s) dma_round((uint32_t)s, s);
    const int rot = (lane >> 1) & 7;
#pragma unroll 1
    for (uint32_t t = 0; t < kRounds; t += SLOTS) {
#pragma unroll 1
        for (int s = 0; s < SLOTS; ++s) {
            // this slot's DMA is the oldest outstanding group: leave the other slots' 8 each in flight
            if constexpr (SLOTS == 1) __builtin_amdgcn_s_waitcnt(0x0F70);       // vmcnt(0)
            else __builtin_amdgcn_s_waitcnt(0x0F70 | (8 * (SLOTS - 1)));        // vmcnt(8 (SLOTS-1))
            uint32_t wv[32];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const uint4 v = stage_w[w * SLOTS + s][lane * 8 + ((q + rot) & 7)];
                wv[4 * q] = v.x, wv[4 * q + 1] = v.y, wv[4 * q + 2] = v.z, wv[4 * q + 3] = v.w;
            }
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the slot is in registers
            dma_round(t + s + SLOTS, s);
            constexpr int P = 3;
            uint64_t G[P + 1][4];
#pragma unroll
            for (int i = 0; i < P; ++i)
#pragma unroll
                for (int b = 0; b < 4; ++b) G[i][b] = gear(wv[i], b);
            uint32_t anyz = 0xFFFFFFFFu;
#pragma unroll
            for (int i = 0; i < 32; ++i) {
                if (i + P < 32) {
#pragma unroll
                    for (int b = 0; b < 4; ++b) G[(i + P) % (P + 1)][b] = gear(wv[i + P], b);
                }
                __builtin_amdgcn_sched_barrier(0);
                const uint64_t* g = G[i % (P + 1)];
                h = (h << 1) + g[0];
                const uint32_t t0 = (uint32_t)(h >> 32) & ch;
                h = (h << 1) + g[1];
                const uint32_t t1 = (uint32_t)(h >> 32) & ch;
                h = (h << 1) + g[2];
                const uint32_t t2 = (uint32_t)(h >> 32) & ch;
                h = (h << 1) + g[3];
                const uint32_t t3 = (uint32_t)(h >> 32) & ch;
                const uint32_t m01 = t0 < t1 ? t0 : t1, m23 = t2 < t3 ? t2 : t3;
                const uint32_t mm = m01 < m23 ? m01 : m23;
                anyz = anyz < mm ? anyz : mm;
                if ((i & 3) == 3) {
                    cnt += anyz == 0;
                    anyz = 0xFFFFFFFFu;
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    }
    atomicAdd(count, (unsigned long long)cnt);
}

// Shared roll of NW words (4 bytes each) with gathers issued P words ahead; counts candidate groups
// (every 16 bytes) when TEST.
template <int NW, bool TEST>
__device__ __forceinline__ void roll_words(const uint32_t* wv, uint64_t& h, uint32_t& cnt, uint32_t ch,
                                           const char* tab, uint32_t copy_off) {
    auto gear = [&](uint32_t word, int jj) -> uint64_t {
        const uint32_t a = __builtin_amdgcn_perm(word, copy_off, 0x0c0c0000u | ((4u + (uint32_t)jj) << 8));
        return *(const uint64_t*)(tab + a);
    };
    constexpr int P = 3;
    uint64_t G[P + 1][4];
#pragma unroll
    for (int i = 0; i < P && i < NW; ++i)
#pragma unroll
        for (int b = 0; b < 4; ++b) G[i][b] = gear(wv[i], b);
    uint32_t anyz = 0xFFFFFFFFu;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        if (i + P < NW) {
#pragma unroll
            for (int b = 0; b < 4; ++b) G[(i + P) % (P + 1)][b] = gear(wv[i + P], b);
        }
        __builtin_amdgcn_sched_barrier(0);
        const uint64_t* g = G[i % (P + 1)];
        h = (h << 1) + g[0];
        const uint32_t t0 = (uint32_t)(h >> 32) & ch;
        h = (h << 1) + g[1];
        const uint32_t t1 = (uint32_t)(h >> 32) & ch;
        h = (h << 1) + g[2];
        const uint32_t t2 = (uint32_t)(h >> 32) & ch;
        h = (h << 1) + g[3];
        const uint32_t t3 = (uint32_t)(h >> 32) & ch;
        if (TEST) {
            const uint32_t m01 = t0 < t1 ? t0 : t1, m23 = t2 < t3 ? t2 : t3;
            const uint32_t mm = m01 < m23 ? m01 : m23;
            anyz = anyz < mm ? anyz : mm;
            if ((i & 3) == 3) {
                cnt += anyz == 0;
                anyz = 0xFFFFFFFFu;
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

// LDS-DMA lane-major, rounds of RB bytes per lane (RB/16 pieces; one DMA covers 64/(RB/16) regions),
// one slot per wave. Piece q of lane r sits at position (q + (r >> SH)) % NP of its RB-byte chunk.
template <int W, int RB>
__global__ __launch_bounds__(64 * W) void lm_dma2(const uint8_t* __restrict__ data, uint64_t n_sec, uint32_t ch,
                                                  unsigned long long* __restrict__ count) {
    constexpr int NP = RB / 16, RPD = 64 / NP, SH = NP == 8 ? 1 : 2;  // pieces, regions per DMA
    __shared__ __attribute__((aligned(16))) uint64_t lds_raw[256 * 32 + W * RB * 8];
    for (int i = threadIdx.x; i < 256 * 32; i += blockDim.x) lds_raw[i] = oxh::kGear[i >> 5] << 16;
    __syncthreads();
    uint4* slot = (uint4*)(lds_raw + 256 * 32);
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    slot += w * RB * 4;  // RB * 64 bytes per wave = RB * 4 uint4
    const uint64_t sec = (uint64_t)blockIdx.x * W + w;
    if (sec >= n_sec) return;
    constexpr uint32_t kReg = kSec / 64, kRounds = kReg / RB;
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void*)(data + sec * kSec - kPad), (short)0, (int)(kSec + kPad), 0x00020000);
    const uint32_t copy_off = (uint32_t)(lane & 31) * 8;
    const char* tab = (const char*)lds_raw;
    const int m = lane / NP, j = lane % NP;
    auto dma_round = [&](uint32_t t) {
#pragma unroll
        for (int k = 0; k < NP; ++k) {
            const uint32_t r = RPD * k + m;
            const uint32_t piece = (uint32_t)(j - (int)((r >> SH) % NP) + NP) % NP;
            const uint32_t off = kPad + r * kReg + 16 * piece;
            const uint32_t soff = t < kRounds ? t * RB : 0x40000000u;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void*)&slot[64 * k], 16, off, soff, 0, 0);
        }
    };
    uint64_t h = 0;
    uint32_t cnt = 0;
    {
        uint32_t wv[12];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, kPad + (uint32_t)lane * kReg - 48 + 16 * k, 0, 0);
            wv[4 * k] = v.x, wv[4 * k + 1] = v.y, wv[4 * k + 2] = v.z, wv[4 * k + 3] = v.w;
        }
        roll_words<12, false>(wv, h, cnt, ch, tab, copy_off);
    }
    dma_round(0);
    const int rot = (lane >> SH) % NP;
#pragma unroll 1
    for (uint32_t t = 0; t < kRounds; ++t) {
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
        uint32_t wv[RB / 4];
#pragma unroll
        for (int q = 0; q < NP; ++q) {
            const uint4 v = slot[lane * NP + (q + rot) % NP];
            wv[4 * q] = v.x, wv[4 * q + 1] = v.y, wv[4 * q + 2] = v.z, wv[4 * q + 3] = v.w;
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
        dma_round(t + 1);
        roll_words<RB / 4, true>(wv, h, cnt, ch, tab, copy_off);
    }
    atomicAdd(count, (unsigned long long)cnt);
}

// Register-staged lane-major: coalesced buffer loads into a DEPTH-round VGPR ring (rounds in flight
// without LDS), then ds_write_b128 into the wave's 8 KiB slot and conflict-free ds_read_b128 back
// (the transpose). Costs 8 ds_write_b128 (13 cycles each) per round but keeps DEPTH x 8 KiB in flight.
template <int W, int DEPTH>
__global__ __launch_bounds__(64 * W) void lm_vgpr(const uint8_t* __restrict__ data, uint64_t n_sec, uint32_t ch,
                                                  unsigned long long* __restrict__ count) {
    __shared__ __attribute__((aligned(16))) uint64_t lds_raw[256 * 32 + W * 1024];
    for (int i = threadIdx.x; i < 256 * 32; i += blockDim.x) lds_raw[i] = oxh::kGear[i >> 5] << 16;
    __syncthreads();
    uint4* slot = (uint4*)(lds_raw + 256 * 32);
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    slot += w * 512;
    const uint64_t sec = (uint64_t)blockIdx.x * W + w;
    if (sec >= n_sec) return;
    constexpr uint32_t kReg = kSec / 64, kRounds = kReg / 128;
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void*)(data + sec * kSec - kPad), (short)0, (int)(kSec + kPad), 0x00020000);
    const uint32_t copy_off = (uint32_t)(lane & 31) * 8;
    const char* tab = (const char*)lds_raw;
    const int m = lane >> 3, j = lane & 7;
    auto load_round = [&](uint32_t t, uint4 (&dst)[8]) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t r = 8 * k + m;
            const uint32_t piece = (uint32_t)(j - (int)((r >> 1) & 7)) & 7;
            const uint32_t soff = t < kRounds ? t * 128 : 0x40000000u;
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, kPad + r * kReg + 16 * piece, soff, 0);
            dst[k] = make_uint4(v.x, v.y, v.z, v.w);
        }
    };
    uint64_t h = 0;
    uint32_t cnt = 0;
    {
        uint32_t wv[12];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, kPad + (uint32_t)lane * kReg - 48 + 16 * k, 0, 0);
            wv[4 * k] = v.x, wv[4 * k + 1] = v.y, wv[4 * k + 2] = v.z, wv[4 * k + 3] = v.w;
        }
        roll_words<12, false>(wv, h, cnt, ch, tab, copy_off);
    }
    uint4 ring[DEPTH][8];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) load_round((uint32_t)d, ring[d]);
    const int rot = (lane >> 1) & 7;
#pragma unroll 1
    for (uint32_t t = 0; t < kRounds; t += DEPTH) {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
#pragma unroll
            for (int k = 0; k < 8; ++k) slot[64 * k + lane] = ring[d][k];
            uint32_t wv[32];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const uint4 v = slot[lane * 8 + ((q + rot) & 7)];
                wv[4 * q] = v.x, wv[4 * q + 1] = v.y, wv[4 * q + 2] = v.z, wv[4 * q + 3] = v.w;
            }
            load_round(t + d + DEPTH, ring[d]);
            roll_words<32, true>(wv, h, cnt, ch, tab, copy_off);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    atomicAdd(count, (unsigned long long)cnt);
}

int main(int argc, char** argv) {
    const double gib = argc > 1 ? atof(argv[1]) : 16.0;
    const uint64_t bytes = (uint64_t)(gib * 1073741824.0) / kSec * kSec, n_sec = bytes / kSec;
    uint8_t* d;
    unsigned long long* c;
    if (hipMalloc(&d, bytes + kPad) != hipSuccess || hipMalloc(&c, 8) != hipSuccess) return 1;
    hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, (uint64_t*)d, (bytes + kPad) / 8, 77);
    const uint64_t common = 0x0000d90103530000ull << 16;  // mask_s & mask_l at 8 KiB chunks, shifted
    const uint32_t ch = (uint32_t)(common >> 32);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char* only = argc > 2 ? argv[2] : nullptr;  // run only variants whose name contains this
    auto run = [&](auto kern, int waves, const char* name) {
        if (only && !strstr(name, only)) return;
        const dim3 grid((unsigned)((n_sec + waves - 1) / waves));
        float best = 1e30f, sum = 0;
        unsigned long long got = 0;
        for (int it = 0; it < 11; ++it) {
            hipMemset(c, 0, 8);
            hipEventRecord(e0);
            hipLaunchKernelGGL(kern, grid, dim3(64 * waves), 0, 0, d + kPad, n_sec, ch, c);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (it) {
                best = ms < best ? ms : best;
                sum += ms;
            }
            hipMemcpy(&got, c, 8, hipMemcpyDeviceToHost);
        }
        if (hipGetLastError() != hipSuccess) printf("launch error in %s\n", name);
        printf("{\"variant\": \"%s\", \"bytes\": %llu, \"best_ms\": %.3f, \"mean_ms\": %.3f, \"TB_s_best\": %.3f, "
               "\"cand_per_group\": %.3e, \"expected_per_group\": %.3e}\n",
               name, (unsigned long long)bytes, best, sum / 10, bytes / (best * 1e-3) / 1e12, got / (bytes / 16.0),
               16.0 / 4096.0);
        fflush(stdout);
    };
#define RUN(S, W, F, D, C) run(seg_scan<S, W, F, D, C>, W, "S" #S "_w" #W "_f" #F "_d" #D "_" #C)
    RUN(8192, 8, 0, 2, false);
    RUN(8192, 16, 0, 2, true);
    RUN(256, 8, 0, 2, true);
    run(lm_dma<8, 1>, 8, "dma_w8_slots1");
    run(lm_dma2<8, 128>, 8, "dma2_w8_rb128");
    run(lm_dma2<16, 64>, 16, "dma2_w16_rb64");
    run(lm_dma2<12, 64>, 12, "dma2_w12_rb64");
    run(lm_vgpr<8, 2>, 8, "vgpr_w8_d2");
    run(lm_vgpr<8, 4>, 8, "vgpr_w8_d4");
    run(lm_vgpr<12, 2>, 12, "vgpr_w12_d2");
    run(lm_vgpr<12, 3>, 12, "vgpr_w12_d3");
    return 0;
}
