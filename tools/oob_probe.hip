#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(const unsigned char* p, unsigned* out, int nrec, unsigned off) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, nrec, 0x00020000);
    u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
    unsigned d = __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
    if (threadIdx.x == 0) { out[0] = v.x; out[1] = v.y; out[2] = v.z; out[3] = v.w; out[4] = d; }
}
int main() {
    unsigned char h[64]; for (int i = 0; i < 64; ++i) h[i] = i + 1;
    unsigned char* d; unsigned* o; unsigned ho[5];
    hipMalloc(&d, 64); hipMalloc(&o, 20); hipMemcpy(d, h, 64, hipMemcpyHostToDevice);
    int cases[][2] = {{16, 0}, {6, 0}, {8, 0}, {12, 0}, {10, 2}, {9, 1}, {5, 1}, {20, 4}, {19, 4}, {18, 4}};
    for (auto& c : cases) {
        hipLaunchKernelGGL(k, 1, 64, 0, 0, d, o, c[0], (unsigned)c[1]);
        hipMemcpy(ho, o, 20, hipMemcpyDeviceToHost);
        printf("nrec=%2d off=%d : x4 = %08x %08x %08x %08x   b32 = %08x\n", c[0], c[1], ho[0], ho[1], ho[2], ho[3], ho[4]);
    }
    return 0;
}
