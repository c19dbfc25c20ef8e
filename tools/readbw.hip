// tools/readbw.hip -- diagnostic HBM read-stream microbenchmarks (not part of the product ABI).
//
// `attainable` read bandwidth for the roofline discussion in DESIGN.md:
//   read_flat     grid-stride dwordx4 read of one large buffer (xor-reduced, one store per thread)
//   read_items    the K1 access pattern (one wave per item, 4 KiB rounds, 4 x 256-B row segments per
//                 wave-instruction) with the hash arithmetic replaced by an xor -- memory pattern alone
#include <hip/hip_runtime.h>
#include <stdint.h>

template <int UNROLL>
__global__ __launch_bounds__(256) void read_flat(const uint4* __restrict__ p, uint64_t n16, uint32_t* __restrict__ sink) {
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t acc = 0;
    uint64_t i = tid;
    for (; i + (UNROLL - 1) * stride < n16; i += UNROLL * stride) {
        uint4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) v[u] = p[i + u * stride];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    for (; i < n16; i += stride) {
        uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9E3779B1u) sink[tid & 1023] = acc;
}

__global__ __launch_bounds__(256) void read_items(const uint8_t* __restrict__ arena, uint64_t n, uint64_t item,
                                                  uint32_t* __restrict__ sink) {
    const int lane = threadIdx.x & 63;
    const uint64_t w = (uint64_t)blockIdx.x * 4 + (uint64_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (w >= n) return;
    const int g = lane >> 4, q = (lane >> 2) & 3, k = lane & 3;
    const uint8_t* lp = arena + w * item + g * 1024 + q * 64 + k * 16;
    const uint64_t nr = item / 4096;
    uint32_t acc = 0;
    for (uint64_t r = 0; r < nr; r += 2) {
        uint4 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = *(const uint4*)(lp + (r + j / 4) * 4096 + (j % 4) * 256);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
    }
    if (acc == 0x9E3779B1u) sink[lane] = acc;
}

extern "C" int readbw_flat(const void* p, uint64_t nbytes, void* sink, int blocks, int unroll, void* stream) {
    const uint64_t n16 = nbytes / 16;
    if (unroll == 8)
        hipLaunchKernelGGL(read_flat<8>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const uint4*)p, n16, (uint32_t*)sink);
    else if (unroll == 4)
        hipLaunchKernelGGL(read_flat<4>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const uint4*)p, n16, (uint32_t*)sink);
    else
        hipLaunchKernelGGL(read_flat<1>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const uint4*)p, n16, (uint32_t*)sink);
    return (int)hipGetLastError();
}

extern "C" int readbw_items(const void* arena, uint64_t n, uint64_t item, void* sink, void* stream) {
    hipLaunchKernelGGL(read_items, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, (hipStream_t)stream, (const uint8_t*)arena,
                       n, item, (uint32_t*)sink);
    return (int)hipGetLastError();
}
