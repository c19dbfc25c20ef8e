// tools/cdc_lanemajor_probe.hip -- throughput of a lane-major FastCDC scan (F1 redesign probe).
//
// F1 today (oxen_amd/csrc/fastcdc.hip) is VALU-bound at ~4.4 TB/s: lane l folds 16 bytes of a
// 1 KiB sub-block and needs the hash of the 48 bytes before them, so every byte pays two 64-bit
// shift-adds (the lane-local tree and the chained hash) plus the DPP carries. Lane-major: lane l owns
// a contiguous 8 KiB region of a 512 KiB section and rolls ONE hash through it (one v_lshl_add_u64
// per byte, a 47-byte warm-up per region). Loads stay coalesced (each wave load instruction reads 8
// whole 128-B lines: lanes 8m..8m+7 read one line of region 8k+m) and an LDS transpose (pitch 144 B,
// conflict-free for ds_read_b128 in 8-lane passes) hands every lane its own 128 B per round.
// This probe only counts candidate groups (no list output) to measure the scan rate.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/cdc_lanemajor_probe.hip -o /tmp/lm && /tmp/lm [GiB]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "../oxen_amd/csrc/fastcdc_gear.h"

constexpr uint32_t kSec = 512 * 1024, kRegion = kSec / 64, kRounds = kRegion / 128, kPitch = 144;

__global__ void fill(uint64_t* p, uint64_t n, uint64_t seed) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

__device__ __forceinline__ uint32_t byte_of(const uint4& v, int j) {
    const uint32_t w = j < 4 ? v.x : j < 8 ? v.y : j < 12 ? v.z : v.w;
    return (w >> (8 * (j & 3))) & 0xFF;
}

// COPIES: bank-private copies of the gear table (entry b of copy c at b * COPIES + c; lane l reads copy l % COPIES)
template <int kWaves, int COPIES>
__global__ __launch_bounds__(64 * kWaves) void lanemajor(const uint8_t* __restrict__ data, uint64_t n_sec, uint32_t ch,
                                                       unsigned long long* __restrict__ count) {
    __shared__ uint64_t gear_tab[256 * COPIES];
    __shared__ uint4 stage[kWaves][64 * kPitch / 16];
    for (int i = threadIdx.x; i < 256 * COPIES; i += blockDim.x) gear_tab[i] = oxh::kGear[i / COPIES] << 16;
    __syncthreads();
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t* gear = gear_tab + (lane & (COPIES - 1));
    const uint64_t sec = (uint64_t)blockIdx.x * kWaves + w;
    if (sec >= n_sec) return;
    const uint8_t* base = data + sec * kSec;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)kSec, 0x00020000);
    const int m = (lane >> 3) & 7, j = lane & 7;
    auto load_round = [&](uint32_t r, uint4 (&dst)[8]) {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t off = (uint32_t)(8 * k + m) * kRegion + r * 128 + 16 * j;
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, r < kRounds ? off : 0xFFFFF000u, 0, 2);
            dst[k] = make_uint4(v.x, v.y, v.z, v.w);
        }
    };
    uint4* st = stage[w];
    uint64_t h = 0;
    uint32_t cnt = 0;
    uint4 ring[2][8];
    load_round(0, ring[0]);
    load_round(1, ring[1]);
    for (uint32_t r = 0; r < kRounds; r += 2) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
#pragma unroll
            for (int k = 0; k < 8; ++k) st[((8 * k + m) * kPitch) / 16 + j] = ring[q][k];
            uint4 mine[8];
#pragma unroll
            for (int g = 0; g < 8; ++g) mine[g] = st[(lane * kPitch) / 16 + g];
            load_round(r + q + 2, ring[q]);
#pragma unroll
            for (int g = 0; g < 8; ++g) {
                uint32_t anyz = 0xFFFFFFFFu;
#pragma unroll
                for (int b = 0; b < 16; ++b) {
                    h = (h << 1) + gear[byte_of(mine[g], b) * COPIES];
                    const uint32_t t = (uint32_t)(h >> 32) & ch;
                    anyz = anyz < t ? anyz : t;
                }
                cnt += anyz == 0;
            }
        }
    }
    atomicAdd(count, (unsigned long long)cnt);
}

// CH independent chains per lane: the section is 64 * CH regions; lane l rolls regions l, l + 64, ...
// interleaved byte by byte (a single chain per lane is bound by the v_lshl_add_u64 dependency).
template <int kWaves, int CH>
__global__ __launch_bounds__(64 * kWaves) void lanemajor_ilp(const uint8_t* __restrict__ data, uint64_t n_sec,
                                                           uint32_t ch, unsigned long long* __restrict__ count) {
    constexpr uint32_t kReg = kSec / (64 * CH), kRnd = kReg / 128;
    __shared__ uint64_t gear[256];
    __shared__ uint4 stage[kWaves][CH * 64 * kPitch / 16];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) gear[i] = oxh::kGear[i] << 16;
    __syncthreads();
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t sec = (uint64_t)blockIdx.x * kWaves + w;
    if (sec >= n_sec) return;
    const uint8_t* base = data + sec * kSec;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)kSec, 0x00020000);
    const int m = (lane >> 3) & 7, j = lane & 7;
    auto load_round = [&](uint32_t r, uint4 (&dst)[8 * CH]) {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int k = 0; k < 8 * CH; ++k) {
            const uint32_t off = (uint32_t)(8 * k + m) * kReg + r * 128 + 16 * j;
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, r < kRnd ? off : 0xFFFFF000u, 0, 2);
            dst[k] = make_uint4(v.x, v.y, v.z, v.w);
        }
    };
    uint4* st = stage[w];
    uint64_t h[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) h[c] = 0;
    uint32_t cnt = 0;
    uint4 ring[8 * CH];
    load_round(0, ring);
    for (uint32_t r = 0; r < kRnd; ++r) {
#pragma unroll
        for (int k = 0; k < 8 * CH; ++k) st[((8 * k + m) * kPitch) / 16 + j] = ring[k];
        load_round(r + 1, ring);  // LDS writes above precede the reloads; group reads follow just in time
#pragma unroll
        for (int g = 0; g < 8; ++g) {
            uint4 mine[CH];
#pragma unroll
            for (int c = 0; c < CH; ++c) mine[c] = st[((64 * c + lane) * kPitch) / 16 + g];
            uint32_t anyz[CH];
#pragma unroll
            for (int c = 0; c < CH; ++c) anyz[c] = 0xFFFFFFFFu;
#pragma unroll
            for (int b = 0; b < 16; ++b)
#pragma unroll
                for (int c = 0; c < CH; ++c) {
                    h[c] = (h[c] << 1) + gear[byte_of(mine[c], b)];
                    const uint32_t t = (uint32_t)(h[c] >> 32) & ch;
                    anyz[c] = anyz[c] < t ? anyz[c] : t;
                }
#pragma unroll
            for (int c = 0; c < CH; ++c) cnt += anyz[c] == 0;
        }
    }
    atomicAdd(count, (unsigned long long)cnt);
}

// No LDS transpose: lane l loads its own region 128 B per round (8 x 16 B, one whole line per lane;
// each wave load instruction touches 64 lines, the next 7 reuse them). Frees the LDS for COPIES
// bank-private gear tables (32 copies: the 32 lanes of a ds_read_b64 group never share a bank).
template <int kWaves, int COPIES>
__global__ __launch_bounds__(64 * kWaves) void lanemajor_direct(const uint8_t* __restrict__ data, uint64_t n_sec,
                                                              uint32_t ch, unsigned long long* __restrict__ count) {
    __shared__ uint64_t gear_tab[256 * COPIES];
    for (int i = threadIdx.x; i < 256 * COPIES; i += blockDim.x) gear_tab[i] = oxh::kGear[i / COPIES] << 16;
    __syncthreads();
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t* gear = gear_tab + (lane & (COPIES - 1));
    const uint64_t sec = (uint64_t)blockIdx.x * kWaves + w;
    if (sec >= n_sec) return;
    const uint8_t* base = data + sec * kSec;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)kSec, 0x00020000);
    auto load_round = [&](uint32_t r, uint4 (&dst)[8]) {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t off = (uint32_t)lane * kRegion + r * 128 + 16 * k;
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, r < kRounds ? off : 0xFFFFF000u, 0, 2);
            dst[k] = make_uint4(v.x, v.y, v.z, v.w);
        }
    };
    uint64_t h = 0;
    uint32_t cnt = 0;
    uint4 ring[2][8];
    load_round(0, ring[0]);
    load_round(1, ring[1]);
    for (uint32_t r = 0; r < kRounds; r += 2) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
#pragma unroll
            for (int g = 0; g < 8; ++g) {
                uint32_t anyz = 0xFFFFFFFFu;
#pragma unroll
                for (int b = 0; b < 16; ++b) {
                    h = (h << 1) + gear[byte_of(ring[q][g], b) * COPIES];
                    const uint32_t t = (uint32_t)(h >> 32) & ch;
                    anyz = anyz < t ? anyz : t;
                }
                cnt += anyz == 0;
            }
            load_round(r + q + 2, ring[q]);
        }
    }
    atomicAdd(count, (unsigned long long)cnt);
}

int main(int argc, char** argv) {
    const double gib = argc > 1 ? atof(argv[1]) : 16.0;
    const uint64_t bytes = (uint64_t)(gib * 1073741824.0) / kSec * kSec, n_sec = bytes / kSec;
    uint8_t* d;
    unsigned long long* c;
    if (hipMalloc(&d, bytes) != hipSuccess || hipMalloc(&c, 8) != hipSuccess) return 1;
    hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, (uint64_t*)d, bytes / 8, 77);
    const uint64_t common = 0x0000d90103530000ull << 16;  // mask_s & mask_l at 8 KiB chunks, shifted
    const uint32_t ch = (uint32_t)(common >> 32);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](auto kern, int waves, const char* name) {
        const dim3 grid((unsigned)((n_sec + waves - 1) / waves));
        float best = 1e30f, sum = 0;
        unsigned long long got = 0;
        for (int it = 0; it < 11; ++it) {
            hipMemset(c, 0, 8);
            hipEventRecord(e0);
            hipLaunchKernelGGL(kern, grid, dim3(64 * waves), 0, 0, d, n_sec, ch, c);
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
        printf("{\"variant\": \"%s\", \"bytes\": %llu, \"best_ms\": %.3f, \"mean_ms\": %.3f, \"TB_s_best\": %.3f, "
               "\"cand_per_group\": %.3e, \"expected_per_group\": %.3e}\n",
               name, (unsigned long long)bytes, best, sum / 10, bytes / (best * 1e-3) / 1e12, got / (bytes / 16.0),
               16.0 / 4096.0);
        fflush(stdout);
    };
    run(lanemajor<4, 1>, 4, "waves4_copies1");
    run(lanemajor_direct<4, 1>, 4, "direct_waves4_copies1");
    run(lanemajor_direct<16, 32>, 16, "direct_waves16_copies32");
    run(lanemajor_direct<8, 32>, 8, "direct_waves8_copies32");
    run(lanemajor_direct<16, 16>, 16, "direct_waves16_copies16");
    return 0;
}
