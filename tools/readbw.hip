// tools/readbw.hip -- diagnostic HBM read-stream microbenchmarks (not part of the product ABI).
//
// `attainable` read bandwidth for the roofline discussion in DESIGN.md:
//   read_flat     grid-stride dwordx4 read of one large buffer (xor-reduced, one store per thread)
//   read_items    the K1 access pattern (one wave per item, 4 KiB rounds, 4 x 256-B row segments per
//                 wave-instruction) with the hash arithmetic replaced by an xor -- memory pattern alone
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int UNROLL, bool NT>
__device__ __forceinline__ uint4 ld(const uint4* p) {
    if constexpr (NT) {
        const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
        return make_uint4(v.x, v.y, v.z, v.w);
    } else {
        return *p;
    }
}

template <int UNROLL, bool NT = false>
__global__ __launch_bounds__(256) void read_flat(const uint4* __restrict__ p, uint64_t n16, uint32_t* __restrict__ sink) {
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t acc = 0;
    uint64_t i = tid;
    for (; i + (UNROLL - 1) * stride < n16; i += UNROLL * stride) {
        uint4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) v[u] = ld<UNROLL, NT>(p + i + u * stride);
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    for (; i < n16; i += stride) {
        uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9E3779B1u) sink[tid & 1023] = acc;
}

// MAPPING 0: K1's round layout (4 x 256-B row segments per wave-instruction);
// MAPPING 1: one contiguous 1 KiB block per wave-instruction.
template <int MAPPING, bool NT>
__global__ __launch_bounds__(256) void read_items(const uint8_t* __restrict__ arena, uint64_t n, uint64_t item,
                                                  uint64_t pitch, uint32_t* __restrict__ sink) {
    const int lane = threadIdx.x & 63;
    const uint64_t w = (uint64_t)blockIdx.x * 4 + (uint64_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (w >= n) return;
    const int g = lane >> 4, q = (lane >> 2) & 3, k = lane & 3;
    const uint8_t* lp = MAPPING == 0 ? arena + w * pitch + g * 1024 + q * 64 + k * 16 : arena + w * pitch + lane * 16;
    const uint64_t nr = item / 4096;
    uint32_t acc = 0;
    for (uint64_t r = 0; r < nr; r += 2) {
        uint4 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint64_t off = MAPPING == 0 ? (r + j / 4) * 4096 + (j % 4) * 256 : (r * 4 + j) * 1024;
            v[j] = ld<1, NT>((const uint4*)(lp + off));
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) acc ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
    }
    if (acc == 0x9E3779B1u) sink[lane] = acc;
}

extern "C" int readbw_flat(const void* p, uint64_t nbytes, void* sink, int blocks, int unroll, void* stream) {
    const uint64_t n16 = nbytes / 16;
    if (unroll == 108)
        hipLaunchKernelGGL((read_flat<8, true>), dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const uint4*)p, n16, (uint32_t*)sink);
    else if (unroll == 8)
        hipLaunchKernelGGL(read_flat<8>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const uint4*)p, n16, (uint32_t*)sink);
    else if (unroll == 4)
        hipLaunchKernelGGL(read_flat<4>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const uint4*)p, n16, (uint32_t*)sink);
    else
        hipLaunchKernelGGL(read_flat<1>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const uint4*)p, n16, (uint32_t*)sink);
    return (int)hipGetLastError();
}

extern "C" int readbw_items(const void* arena, uint64_t n, uint64_t item, uint64_t pitch, int kind, void* sink,
                            void* stream) {
    const dim3 grid((unsigned)((n + 3) / 4));
    const uint8_t* a = (const uint8_t*)arena;
    if (kind == 0) hipLaunchKernelGGL((read_items<0, false>), grid, dim3(256), 0, (hipStream_t)stream, a, n, item, pitch, (uint32_t*)sink);
    if (kind == 1) hipLaunchKernelGGL((read_items<1, false>), grid, dim3(256), 0, (hipStream_t)stream, a, n, item, pitch, (uint32_t*)sink);
    if (kind == 2) hipLaunchKernelGGL((read_items<0, true>), grid, dim3(256), 0, (hipStream_t)stream, a, n, item, pitch, (uint32_t*)sink);
    if (kind == 3) hipLaunchKernelGGL((read_items<1, true>), grid, dim3(256), 0, (hipStream_t)stream, a, n, item, pitch, (uint32_t*)sink);
    return (int)hipGetLastError();
}
