// VALU issue-rate probe (gfx950): 64-bit shift-add (v_lshl_add_u64) vs 32-bit add / and, and the
// cross-lane moves K1's realign uses (DPP wave_rol:1, DPP row_ror:15, v_permlane16_swap), 8
// chains per lane. ops: 0 lshl_add_u64, 1 add_u32, 2 and_b32, 3 wave_rol, 4 row_ror, 5 permlane16_swap. hipcc --offload-arch=gfx950 -O3 tools/valu_rate_probe.hip -o /tmp/rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
// Throughput of v_lshl_add_u64 vs v_add_u32 vs v_mad_u64_u32: 8 independent chains per lane.
template <int OP>
__global__ void k(uint64_t* out, int iters, uint64_t seed) {
    uint64_t a[8];
    for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x * 8 + i;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if (OP == 0) asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(a[i]) : "v"(a[(i + 1) & 7]));
                else if (OP == 1) {
                    uint32_t lo = (uint32_t)a[i];
                    asm volatile("v_add_u32 %0, %0, %1" : "+v"(lo) : "v"((uint32_t)a[(i + 1) & 7]));
                    a[i] = (a[i] & 0xFFFFFFFF00000000ull) | lo;
                } else if (OP == 2) {
                    uint32_t lo = (uint32_t)a[i];
                    asm volatile("v_and_b32 %0, %0, %1" : "+v"(lo) : "v"((uint32_t)a[(i + 1) & 7]));
                    a[i] = (a[i] & 0xFFFFFFFF00000000ull) | lo;
                } else if (OP == 3 || OP == 4) {
                    // K1 block-wise byte-shift realign: next lane's dword by wave_rol:1 vs row_ror:15
                    uint32_t lo = (uint32_t)a[i];
                    if (OP == 3)
                        asm volatile("v_mov_b32_dpp %0, %1 wave_rol:1 row_mask:0xf bank_mask:0xf" : "+v"(lo) : "v"((uint32_t)a[(i + 1) & 7]));
                    else
                        asm volatile("v_mov_b32_dpp %0, %1 row_ror:15 row_mask:0xf bank_mask:0xf" : "+v"(lo) : "v"((uint32_t)a[(i + 1) & 7]));
                    a[i] = (a[i] & 0xFFFFFFFF00000000ull) | lo;
                } else if (OP == 5) {
                    uint32_t lo = (uint32_t)a[i], hi = (uint32_t)a[(i + 1) & 7];
                    asm volatile("v_permlane16_swap_b32 %0, %1" : "+v"(lo), "+v"(hi));
                    a[i] = ((uint64_t)hi << 32) | lo;
                }
            }
    }
    uint64_t s = 0;
    for (int i = 0; i < 8; ++i) s ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
int main() {
    uint64_t* d; hipMalloc(&d, 1 << 26);
    const int blocks = 256 * 8, threads = 256, iters = 2000;
    for (int op = 0; op < 6; ++op) {
        auto fn = op == 0 ? k<0> : op == 1 ? k<1> : op == 2 ? k<2> : op == 3 ? k<3> : op == 4 ? k<4> : k<5>;
        hipLaunchKernelGGL(fn, dim3(blocks), dim3(threads), 0, 0, d, 10, 1);
        hipDeviceSynchronize();
        hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
        hipEventRecord(e0);
        hipLaunchKernelGGL(fn, dim3(blocks), dim3(threads), 0, 0, d, iters, 1);
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        const double ops = (double)blocks * threads * iters * 16 * 8;  // lane-ops
        printf("op %d: %.3f ms, %.2f T lane-ops/s, %.3f cycles/wave-instr/SIMD at 2.4GHz\n", op, ms, ops / ms / 1e9,
               (ms * 1e-3 * 2.4e9) / ((double)blocks * threads / 64 * iters * 16 * 8 / (256 * 4)));
    }
    return 0;
}
