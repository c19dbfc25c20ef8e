// Probe for folding K1's block sums into the FastCDC walk (DESIGN §4 "W + X"):
//  (1) issue cost of v_mad_u64_u32 (XXH3's 32x32->64 multiply-accumulate) against v_lshl_add_u64 and
//      v_add_u32: 8 independent chains per lane, cycles per wave-instruction;
//  (2) LDS-DMA (buffer_load_dwordx4 ... lds, as W's rounds) from line starts that are only dword
//      aligned (a chunk-relative line) against 128-B aligned ones: the bytes that land, and the rate of
//      a W-shaped stream (8 DMAs of 64 x 16 B per round per wave, 12 waves per CU) over 8 GiB.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/fold_probe.hip -o tools/fold_probe && tools/fold_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
            return 1;                                                              \
        }                                                                          \
    } while (0)

template <int OP>
__global__ void rate_kernel(uint64_t* out, int iters, uint64_t seed, long long* cyc) {
    uint64_t a[8];
    uint32_t b[8];
    for (int i = 0; i < 8; ++i) {
        a[i] = seed + threadIdx.x * 8 + i;
        b[i] = (uint32_t)(seed >> 7) + i * 77 + threadIdx.x;
    }
    const long long t0 = clock64();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if (OP == 0) {
                    asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(a[i]) : "v"(b[i]), "v"(b[(i + 1) & 7]) : "vcc");
                } else if (OP == 1) {
                    asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a[i]) : "v"(a[(i + 1) & 7]));
                } else {
                    asm volatile("v_add_u32 %0, %0, %1" : "+v"(b[i]) : "v"(b[(i + 1) & 7]));
                }
            }
    }
    const long long t1 = clock64();
    uint64_t s = 0;
    for (int i = 0; i < 8; ++i) s += a[i] + b[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

constexpr uint32_t kAux = 0;
// W-shaped stream: every lane walks its own region of `per_lane` bytes from base + lane_region + shift,
// one 128-B line per round, fetched by 8 DMAs of 16 B per lane (lanes 8m..8m+7 of DMA k fetch the line
// of lane 8k+m); the lane then reads its 128 B back and xors them into a sum (so nothing is dead).
template <int WAVES>
__global__ __launch_bounds__(64 * WAVES) void dma_stream(const uint8_t* base, uint64_t region, uint32_t per_lane,
                                                        uint32_t shift, uint32_t* out) {
    __shared__ __attribute__((aligned(16))) uint4 slot_all[WAVES * 512];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint4* slot = slot_all + w * 512;
    const uint64_t gl = ((uint64_t)blockIdx.x * WAVES + w) * 64;
    const uint8_t* wb = base + gl * region;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)wb, (short)0, (int)(64 * region + 256), 0x00020000);
    const int dm = lane >> 3, dj = lane & 7;
    uint32_t acc = 0;
    const uint32_t my = (uint32_t)lane * (uint32_t)region + shift;
    for (uint32_t r = 0; r < per_lane; r += 128) {
        const uint32_t line = my + r;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t src = (uint32_t)__builtin_amdgcn_ds_bpermute((8 * k + dm) * 4, (int)line);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void*)(slot + 64 * k), 16,
                                                     src + 16 * dj, 0, 0, kAux);
        }
        __builtin_amdgcn_s_waitcnt(0x0F70);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            // line of lane L = 8k+m sits at slot + 64k + 8m .. : piece dj at + dj
            const int k = lane >> 3, m = lane & 7;
            const uint4 v = slot[64 * k + 8 * m + q];
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);
    }
    out[gl + lane] = acc;
}

// the same stream's expected xor, on the host
uint32_t expect(const std::vector<uint8_t>& h, uint64_t region, uint32_t per_lane, uint32_t shift, uint64_t lanes) {
    uint32_t x = 0;
    for (uint64_t l = 0; l < lanes; ++l) {
        const uint8_t* p = h.data() + l * region + shift;
        for (uint32_t i = 0; i + 4 <= per_lane; i += 4) {
            uint32_t v;
            memcpy(&v, p + i, 4);
            x ^= v;
        }
    }
    return x;
}

int main() {
    // (1) rates
    {
        uint64_t* d_out;
        long long* d_cyc;
        CK(hipMalloc(&d_out, 1024 * 256 * 8));
        CK(hipMalloc(&d_cyc, 8));
        const int iters = 2000;
        const char* names[3] = {"v_mad_u64_u32", "v_lshl_add_u64", "v_add_u32"};
        for (int op = 0; op < 3; ++op) {
            for (int rep = 0; rep < 2; ++rep) {
                if (op == 0) hipLaunchKernelGGL(rate_kernel<0>, dim3(1024), dim3(256), 0, 0, d_out, iters, 12345ull, d_cyc);
                if (op == 1) hipLaunchKernelGGL(rate_kernel<1>, dim3(1024), dim3(256), 0, 0, d_out, iters, 12345ull, d_cyc);
                if (op == 2) hipLaunchKernelGGL(rate_kernel<2>, dim3(1024), dim3(256), 0, 0, d_out, iters, 12345ull, d_cyc);
                CK(hipDeviceSynchronize());
            }
            long long cyc = 0;
            CK(hipMemcpy(&cyc, d_cyc, 8, hipMemcpyDeviceToHost));
            // one wave of block 0 (4 waves per CU-quarter... 16 waves / CU): cycles per instruction of that wave
            printf("{\"op\": \"%s\", \"cycles_per_wave_instr_at_16_waves_per_CU\": %.3f}\n", names[op],
                   (double)cyc / (iters * 16.0 * 8.0));
        }
        CK(hipFree(d_out));
        CK(hipFree(d_cyc));
    }
    // (2) DMA from dword-aligned line starts
    {
        constexpr int WAVES = 12;
        const uint64_t region = 256 * 1024 + 256;  // per lane
        const uint32_t per_lane = 256 * 1024;
        int cus = 256;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
        const uint64_t blocks = (uint64_t)cus * 1;  // one generation, one workgroup per CU
        const uint64_t lanes = blocks * WAVES * 64;
        const uint64_t bytes = lanes * region + 4096;
        std::vector<uint8_t> h(bytes);
        uint64_t z = 0x9E3779B97F4A7C15ull;
        for (uint64_t i = 0; i < bytes; i += 8) {
            z += 0x9E3779B97F4A7C15ull;
            uint64_t v = z;
            v = (v ^ (v >> 30)) * 0xBF58476D1CE4E5B9ull;
            v = (v ^ (v >> 27)) * 0x94D049BB133111EBull;
            v ^= v >> 31;
            memcpy(h.data() + i, &v, std::min<uint64_t>(8, bytes - i));
        }
        uint8_t* d;
        uint32_t* d_o;
        CK(hipMalloc(&d, bytes));
        CK(hipMalloc(&d_o, lanes * 4));
        CK(hipMemcpy(d, h.data(), bytes, hipMemcpyHostToDevice));
        std::vector<uint32_t> o(lanes);
        for (uint32_t shift : {0u, 4u, 64u, 100u, 128u}) {
            hipEvent_t e0, e1;
            CK(hipEventCreate(&e0));
            CK(hipEventCreate(&e1));
            float best = 1e9f;
            for (int rep = 0; rep < 5; ++rep) {
                CK(hipEventRecord(e0));
                hipLaunchKernelGGL(dma_stream<WAVES>, dim3((unsigned)blocks), dim3(64 * WAVES), 0, 0, d, region, per_lane, shift, d_o);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                best = std::min(best, ms);
            }
            CK(hipMemcpy(o.data(), d_o, lanes * 4, hipMemcpyDeviceToHost));
            uint32_t got = 0;
            for (uint32_t v : o) got ^= v;
            const uint32_t want = expect(h, region, per_lane, shift, lanes);
            printf("{\"dma_line_shift\": %u, \"bytes\": %llu, \"ms\": %.3f, \"TB_s\": %.3f, \"bytes_ok\": %s}\n", shift,
                   (unsigned long long)(lanes * per_lane), best, lanes * (double)per_lane / (best * 1e-3) / 1e12,
                   got == want ? "true" : "false");
        }
        CK(hipFree(d));
        CK(hipFree(d_o));
    }
    return 0;
}
