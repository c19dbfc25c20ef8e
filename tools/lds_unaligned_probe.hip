#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__global__ void k(uint32_t* out, int mode) {
    __shared__ __attribute__((aligned(16))) uint8_t buf[2048];
    const int t = threadIdx.x;
    for (int i = t; i < 2048; i += 64) buf[i] = (uint8_t)(i * 7 + 3);
    __syncthreads();
    const uint32_t a = (uint32_t)(uintptr_t)buf + (uint32_t)(t * 16 + (t % 16));  // byte offsets 0..15 + 16t
    u32x4 v;
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
    out[4 * t + 0] = v.x; out[4 * t + 1] = v.y; out[4 * t + 2] = v.z; out[4 * t + 3] = v.w;
}
int main() {
    uint32_t* d; hipMalloc(&d, 64 * 16);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, 0);
    uint32_t h[256]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int t = 0; t < 64; ++t) {
        const int o = t * 16 + (t % 16);
        for (int w = 0; w < 4; ++w) {
            uint32_t want = 0;
            for (int b = 3; b >= 0; --b) want = (want << 8) | (uint8_t)((o + 4 * w + b) * 7 + 3);
            if (h[4 * t + w] != want) { if (bad < 8) printf("lane %d off %d word %d got %08x want %08x\n", t, o, w, h[4*t+w], want); ++bad; }
        }
    }
    printf("unaligned ds_read_b128: %s (%d bad words)\n", bad ? "MISMATCH" : "ok", bad);
    return 0;
}
