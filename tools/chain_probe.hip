// K1L chain probe (gfx950): the XXH3 long-path accumulator chain acc <- scramble(acc + S_b), one
// step per 1 KiB block, run three ways over the same synthetic block sums:
//   v 0  VALU, lanes 0-7 of one wave own the 8 accumulators (the shipped xxh3_chain_kernel's step:
//        shift, v_bitop3, v_mul_lo_u32, v_mad_u64_u32, add -- in-order issue of two quarter-rate
//        multiplies per step)
//   v 1  SALU, one wave per accumulator: every value is wave-uniform, so the step is ~10 scalar
//        instructions (s_mul_i32 / s_mul_hi_u32 for the 32x32 products) and the sums arrive by
//        s_load (accumulator-major layout)
// Prints ns per step and checks every variant's final accumulators against the host.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/chain_probe.hip -o tools/chain_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

constexpr uint32_t P = 0x9E3779B1u;

__host__ __device__ inline uint64_t step_ref(uint64_t x, uint64_t s, uint64_t key) {
    x ^= x >> 47;
    x ^= key;
    x *= (uint64_t)P;
    return x + s;
}

// v0: lanes 0-7, sums [b][8] staged through LDS in groups (as the shipped kernel does)
template <int MODE, bool FULL = false>
__global__ __launch_bounds__(64) void chain_valu(const uint64_t* __restrict__ sums, uint64_t nb, const uint64_t* keys,
                                                 const uint64_t* init, uint64_t* out) {
    constexpr int GROUP = 256;
    const int lane = threadIdx.x, i = lane & 7;
    const uint64_t sk = keys[i];
    const uint32_t kl = (uint32_t)sk, kh = (uint32_t)(sk >> 32);
    auto step = [&](uint32_t& xl, uint32_t& xh, uint64_t s_next) {
        uint32_t yl;
        asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(yl) : "v"(xl), "v"(kl), "v"(xh >> 15));
        const uint32_t yh = xh ^ kh;
        uint32_t t;
        if constexpr (MODE == 0) t = yh * P;
        else if constexpr (MODE == 1) asm("v_mul_u32_u24 %0, %1, %2" : "=v"(t) : "v"(yh), "v"(kl));  // timing only
        else t = yh;  // timing only
        asm("" : "+v"(t));
        const uint64_t m = (uint64_t)yl * P + s_next;
        xh = (uint32_t)(m >> 32) + t;
        xl = (uint32_t)m;
    };
    uint64_t x0 = init[i] + sums[i];
    uint32_t xl = (uint32_t)x0, xh = (uint32_t)(x0 >> 32);
    __shared__ uint64_t buf[2][GROUP * 8];
    constexpr int PER = GROUP * 8 / 64;
    const uint64_t ngroups = (nb - 1) / GROUP;
    uint64_t r[PER];
    auto issue = [&](uint64_t g) {
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const uint64_t e = (uint64_t)k * 64 + (uint64_t)lane;
            r[k] = sums[(1 + g * GROUP + e / 8) * 8 + (e & 7)];
        }
    };
    auto commit = [&](int sb) {
#pragma unroll
        for (int k = 0; k < PER; ++k) buf[sb][k * 64 + lane] = r[k];
        __syncthreads();
    };
    uint64_t b = 1;
    if (ngroups > 0) {
        issue(0);
        commit(0);
        for (uint64_t gi = 0; gi < ngroups; ++gi) {
            const int sb = (int)(gi & 1);
            if (gi + 1 < ngroups) issue(gi + 1);
            if (FULL || lane < 8) {
                constexpr int B = 32;
                uint64_t va[B], vb[B];
#pragma unroll
                for (int t = 0; t < B; ++t) va[t] = buf[sb][t * 8 + i];
#pragma unroll
                for (int t0 = 0; t0 < GROUP; t0 += 2 * B) {
#pragma unroll
                    for (int t = 0; t < B; ++t) vb[t] = buf[sb][(t0 + B + t) * 8 + i];
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int t = 0; t < B; ++t) step(xl, xh, va[t]);
                    if (t0 + 2 * B < GROUP) {
#pragma unroll
                        for (int t = 0; t < B; ++t) va[t] = buf[sb][(t0 + 2 * B + t) * 8 + i];
                    }
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int t = 0; t < B; ++t) step(xl, xh, vb[t]);
                }
            }
            if (gi + 1 < ngroups) commit(sb ^ 1);
        }
        b = 1 + ngroups * GROUP;
    }
    for (; b < nb; ++b) step(xl, xh, sums[b * 8 + i]);
    if (lane < 8) out[i] = ((uint64_t)xh << 32) | xl;
}


// v-packed: 8 independent jobs per wave (lanes 8g..8g+7 = job g), each with its own sums array
// (job-major: sums_j = sums + j * nb * 8), staged through LDS in groups of GROUP steps of every job.
// PAD: u64 of padding between the jobs' LDS regions (bank spread).
template <int GROUP, int PAD>
__global__ __launch_bounds__(64) void chain_packed(const uint64_t* __restrict__ sums, uint64_t nb, const uint64_t* keys,
                                                   const uint64_t* init, uint64_t* out) {
    constexpr int JW = 8;
    constexpr int JS = GROUP * 8 + PAD;  // u64 per job region
    const int lane = threadIdx.x, i = lane & 7, jw = lane >> 3;
    const uint64_t* js = sums + (uint64_t)jw * nb * 8;
    const uint64_t sk = keys[i];
    const uint32_t kl = (uint32_t)sk, kh = (uint32_t)(sk >> 32);
    auto step = [&](uint32_t& xl, uint32_t& xh, uint64_t s_next) {
        uint32_t yl;
        asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(yl) : "v"(xl), "v"(kl), "v"(xh >> 15));
        const uint32_t yh = xh ^ kh;
        uint32_t t = yh * P;
        asm("" : "+v"(t));
        const uint64_t m = (uint64_t)yl * P + s_next;
        xh = (uint32_t)(m >> 32) + t;
        xl = (uint32_t)m;
    };
    uint64_t x0 = init[i] + js[i];
    uint32_t xl = (uint32_t)x0, xh = (uint32_t)(x0 >> 32);
    __shared__ uint64_t buf[2][JW * JS];
    constexpr int PER = JW * GROUP * 8 / 64;
    uint64_t r[PER];
    const uint64_t ngroups = (nb - 1) / GROUP;
    auto issue = [&](uint64_t g) {
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int j = k / (GROUP * 8 / 64);
            const int w = (k % (GROUP * 8 / 64)) * 64 + lane;  // element within the job's group
            r[k] = sums[(uint64_t)j * nb * 8 + (1 + g * GROUP) * 8 + (uint64_t)w];
        }
    };
    auto commit = [&](int sb) {
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int j = k / (GROUP * 8 / 64);
            const int w = (k % (GROUP * 8 / 64)) * 64 + lane;
            buf[sb][j * JS + w] = r[k];
        }
        __syncthreads();
    };
    uint64_t b = 1;
    if (ngroups > 0) {
        issue(0);
        commit(0);
        for (uint64_t gi = 0; gi < ngroups; ++gi) {
            const int sb = (int)(gi & 1);
            if (gi + 1 < ngroups) issue(gi + 1);
            constexpr int B = GROUP < 64 ? GROUP / 2 : 32;
            const uint64_t* jb = &buf[sb][jw * JS];
            uint64_t va[B], vb[B];
#pragma unroll
            for (int t = 0; t < B; ++t) va[t] = jb[t * 8 + i];
#pragma unroll
            for (int t0 = 0; t0 < GROUP; t0 += 2 * B) {
#pragma unroll
                for (int t = 0; t < B; ++t) vb[t] = jb[(t0 + B + t) * 8 + i];
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int t = 0; t < B; ++t) step(xl, xh, va[t]);
                if (t0 + 2 * B < GROUP) {
#pragma unroll
                    for (int t = 0; t < B; ++t) va[t] = jb[(t0 + 2 * B + t) * 8 + i];
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int t = 0; t < B; ++t) step(xl, xh, vb[t]);
            }
            if (gi + 1 < ngroups) commit(sb ^ 1);
        }
        b = 1 + ngroups * GROUP;
    }
    for (; b < nb; ++b) step(xl, xh, js[b * 8 + i]);
    out[jw * 8 + i] = ((uint64_t)xh << 32) | xl;
}

// v1: one wave per accumulator, all scalar. sums_t is accumulator-major: [8][nb].
typedef const __attribute__((address_space(4))) uint64_t* const_u64p;
template <int U>
__global__ __launch_bounds__(64) void chain_salu(const uint64_t* __restrict__ sums_t, uint64_t nb, const uint64_t* keys,
                                                 const uint64_t* init, uint64_t* out) {
    const int i = blockIdx.x;
    const_u64p s = (const_u64p)(sums_t + (uint64_t)i * nb);
    const_u64p kp = (const_u64p)keys;
    const_u64p ip = (const_u64p)init;
    const uint64_t key = kp[i];
    const uint32_t kl = (uint32_t)key, kh = (uint32_t)(key >> 32);
    uint64_t x = ip[i] + s[0];
    uint32_t xl = (uint32_t)x, xh = (uint32_t)(x >> 32);
    auto step = [&](uint64_t sn) {
        const uint32_t yl = xl ^ (xh >> 15) ^ kl;
        const uint32_t yh = xh ^ kh;
        const uint64_t m = (uint64_t)yl * P + sn;
        xh = (uint32_t)(m >> 32) + yh * P;
        xl = (uint32_t)m;
    };
    uint64_t b = 1;
    uint64_t cur[U], nxt[U];
    if (nb >= 1 + 2 * (uint64_t)U) {
#pragma unroll
        for (int k = 0; k < U; ++k) cur[k] = s[b + k];
        for (; b + 2 * (uint64_t)U <= nb; b += U) {
#pragma unroll
            for (int k = 0; k < U; ++k) nxt[k] = s[b + U + k];
#pragma unroll
            for (int k = 0; k < U; ++k) step(cur[k]);
#pragma unroll
            for (int k = 0; k < U; ++k) cur[k] = nxt[k];
        }
#pragma unroll
        for (int k = 0; k < U; ++k) step(cur[k]);
        b += U;
    }
    for (; b < nb; ++b) step(s[b]);
    if (threadIdx.x == 0) out[i] = ((uint64_t)xh << 32) | xl;
}

int main(int argc, char** argv) {
    const uint64_t nb = argc > 1 ? strtoull(argv[1], nullptr, 10) : (1ull << 21);
    std::vector<uint64_t> sums(nb * 8), sums_t(nb * 8), keys(8), init(8), want(8);
    uint64_t z = 0x12345678abcdefull;
    auto rnd = [&] {
        z += 0x9E3779B97F4A7C15ull;
        uint64_t r = z;
        r = (r ^ (r >> 30)) * 0xBF58476D1CE4E5B9ull;
        r = (r ^ (r >> 27)) * 0x94D049BB133111EBull;
        return r ^ (r >> 31);
    };
    for (auto& v : sums) v = rnd();
    for (int i = 0; i < 8; ++i) keys[i] = rnd(), init[i] = rnd();
    for (uint64_t b = 0; b < nb; ++b)
        for (int i = 0; i < 8; ++i) sums_t[i * nb + b] = sums[b * 8 + i];
    for (int i = 0; i < 8; ++i) {
        uint64_t x = init[i] + sums[i];
        for (uint64_t b = 1; b < nb; ++b) x = step_ref(x, sums[b * 8 + i], keys[i]);
        want[i] = x;
    }
    uint64_t *d_s, *d_st, *d_k, *d_i, *d_o;
    hipMalloc(&d_s, nb * 64);
    hipMalloc(&d_st, nb * 64);
    hipMalloc(&d_k, 64);
    hipMalloc(&d_i, 64);
    hipMalloc(&d_o, 64 * 4);
    hipMemcpy(d_s, sums.data(), nb * 64, hipMemcpyHostToDevice);
    hipMemcpy(d_st, sums_t.data(), nb * 64, hipMemcpyHostToDevice);
    hipMemcpy(d_k, keys.data(), 64, hipMemcpyHostToDevice);
    hipMemcpy(d_i, init.data(), 64, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    if (argc > 2 && !strcmp(argv[2], "packed")) {  // 8 jobs per wave: job j's sums = the base sums rotated by j steps
        std::vector<uint64_t> s8(nb * 8 * 8);
        for (int j = 0; j < 8; ++j)
            for (uint64_t b = 0; b < nb; ++b)
                for (int a = 0; a < 8; ++a) s8[((uint64_t)j * nb + b) * 8 + a] = sums[((b + j) % nb) * 8 + a];
        std::vector<uint64_t> want8(64);
        for (int j = 0; j < 8; ++j)
            for (int a = 0; a < 8; ++a) {
                uint64_t x = init[a] + s8[((uint64_t)j * nb) * 8 + a];
                for (uint64_t b = 1; b < nb; ++b) x = step_ref(x, s8[((uint64_t)j * nb + b) * 8 + a], keys[a]);
                want8[j * 8 + a] = x;
            }
        uint64_t *d8, *o8;
        hipMalloc(&d8, s8.size() * 8);
        hipMalloc(&o8, 64 * 8 * 4);
        hipMemcpy(d8, s8.data(), s8.size() * 8, hipMemcpyHostToDevice);
        auto run = [&](const char* name, void (*k)(const uint64_t*, uint64_t, const uint64_t*, const uint64_t*, uint64_t*), int waves) {
            float best = 1e30f;
            for (int rep = 0; rep < 2; ++rep) {
                hipEventRecord(e0);
                for (int w = 0; w < waves; ++w) hipLaunchKernelGGL(k, dim3(1), dim3(64), 20 * 1024, 0, d8, nb, d_k, d_i, o8 + 64 * w);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                if (ms < best) best = ms;
            }
            std::vector<uint64_t> got(64);
            hipMemcpy(got.data(), o8, 64 * 8, hipMemcpyDeviceToHost);
            printf("{\"packed\": \"%s\", \"ms\": %.3f, \"ns_per_step\": %.3f, \"exact\": %s}\n", name, best,
                   best * 1e6 / (double)nb, got == want8 ? "true" : "false");
        };
        run("g64_pad0", chain_packed<64, 0>, 1);
        run("g64_pad8", chain_packed<64, 8>, 1);
        run("g32_pad8", chain_packed<32, 8>, 1);
        run("g128_pad8", chain_packed<128, 8>, 1);
        return 0;
    }
    if (argc > 2) {  // concurrency sweep: N independent copies of the v0 chain, one workgroup per CU
        const size_t pad = 50 * 1024;  // as the shipped launch: > half a CU's LDS per workgroup
        for (int n : {1, 2, 4, 8, 16, 32, 64, 128, -1, -2, -4}) {  // -k: k waves with all 64 lanes chaining
            const bool full = n < 0;
            const int nw = full ? -n : n;
            float best = 1e30f;
            for (int rep = 0; rep < 2; ++rep) {
                hipEventRecord(e0);
                if (full) hipLaunchKernelGGL((chain_valu<0, true>), dim3(nw), dim3(64), pad, 0, d_s, nb, d_k, d_i, d_o);
                else hipLaunchKernelGGL(chain_valu<0>, dim3(nw), dim3(64), pad, 0, d_s, nb, d_k, d_i, d_o);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                if (ms < best) best = ms;
            }
            printf("{\"sweep_waves\": %d, \"chains_per_wave\": %d, \"steps\": %llu, \"ms\": %.3f, \"ns_per_step\": %.3f}\n", nw, full ? 8 : 1,
                   (unsigned long long)nb, best, best * 1e6 / (double)nb);
        }
        return 0;
    }
    for (int v = 0; v < 6; ++v) {
        float best = 1e30f;
        for (int rep = 0; rep < 3; ++rep) {
            hipMemset(d_o, 0, 64);
            hipEventRecord(e0);
            if (v == 0) hipLaunchKernelGGL(chain_valu<0>, dim3(1), dim3(64), 0, 0, d_s, nb, d_k, d_i, d_o);
            if (v == 1) hipLaunchKernelGGL(chain_salu<8>, dim3(8), dim3(64), 0, 0, d_st, nb, d_k, d_i, d_o);
            if (v == 2) hipLaunchKernelGGL(chain_salu<16>, dim3(8), dim3(64), 0, 0, d_st, nb, d_k, d_i, d_o);
            if (v == 4) hipLaunchKernelGGL(chain_valu<1>, dim3(1), dim3(64), 0, 0, d_s, nb, d_k, d_i, d_o);
            if (v == 5) hipLaunchKernelGGL(chain_valu<2>, dim3(1), dim3(64), 0, 0, d_s, nb, d_k, d_i, d_o);
            if (v == 3) hipLaunchKernelGGL(chain_salu<32>, dim3(8), dim3(64), 0, 0, d_st, nb, d_k, d_i, d_o);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        std::vector<uint64_t> got(8);
        hipMemcpy(got.data(), d_o, 64, hipMemcpyDeviceToHost);
        bool ok = true;
        for (int i = 0; i < 8; ++i) ok = ok && got[i] == want[i];
        printf("{\"variant\": %d, \"steps\": %llu, \"ms\": %.3f, \"ns_per_step\": %.3f, \"exact\": %s}\n", v,
               (unsigned long long)nb, best, best * 1e6 / (double)nb, ok ? "true" : "false");
    }
    return 0;
}
