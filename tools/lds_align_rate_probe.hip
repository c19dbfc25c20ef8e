// ds_read_b128 throughput by address alignment (16 B, 4 B, 1 B) on gfx950: every lane of 16 waves per
// CU reads 16 B from LDS at lane*16 + shift, 4096 times; the chip-wide rate is printed per shift.
// Build: hipcc --offload-arch=gfx950 -O3 tools/lds_align_rate_probe.hip -o /tmp/lds_align_rate_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k(uint32_t* out, uint32_t shift, int iters) {
    __shared__ __attribute__((aligned(16))) uint8_t buf[4 * 1024 + 64];
    for (int i = threadIdx.x; i < 4 * 1024 + 64; i += blockDim.x) buf[i] = (uint8_t)(i * 13 + 1);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t base = (uint32_t)(uintptr_t)buf + (threadIdx.x >> 6) * 1024 + lane * 16 + shift;
    uint32_t acc = 0;
    for (int it = 0; it < iters; it += 4) {
        u32x4 v0, v1, v2, v3;  // four reads in flight per wave, then one wait
        asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4\n\tds_read_b128 %2, %4\n\tds_read_b128 %3, %4\n\t"
                     "s_waitcnt lgkmcnt(0)"
                     : "=&v"(v0), "=&v"(v1), "=&v"(v2), "=&v"(v3) : "v"(base) : "memory");
        acc += v0.x ^ v1.y ^ v2.z ^ v3.w;
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

int main() {
    uint32_t* d;
    (void)hipMalloc(&d, 1 << 20);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int iters = 4096, blocks = 256 * 4;  // 4 workgroups of 4 waves per CU
    for (uint32_t shift : {0u, 16u, 4u, 8u, 12u, 1u, 2u, 3u}) {
        hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, shift, iters);
        (void)hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, shift, iters);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double bytes = 5.0 * blocks * 256 * 16.0 * iters;
        printf("{\"shift\": %u, \"ms\": %.3f, \"TB_s\": %.2f}\n", shift, ms, bytes / (ms * 1e-3) / 1e12);
    }
    return 0;
}
