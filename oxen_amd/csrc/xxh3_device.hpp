// oxen_amd/csrc/xxh3_device.hpp -- XXH3-128 (seed 0, default secret) primitives for gfx950.
//
// This is the content hash behind liboxen `util/hasher.rs:28-30` (`hash_buffer_128bit` ->
// xxhash-rust 0.8.15 `xxh3_128`). Integer-only: 32x32->64 multiplies, 64-bit add/xor/shift and
// 64x64->128 folds; no MFMA anywhere (this is byte work, not a contraction).
//
// Two device-side formulations live here:
//   * `xxh3_lane_*`  -- one lane computes one whole digest (short inputs, K2 parent streams).
//   * the wave-cooperative long path in xxh3_kernels.hip (one wave per buffer, 4 KiB rounds).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace oxh {

// The XXH3 default secret (192 B). Part of the algorithm's definition.
struct SecretBytes { uint8_t b[192]; };
constexpr SecretBytes kSecret = {{
    0xb8, 0xfe, 0x6c, 0x39, 0x23, 0xa4, 0x4b, 0xbe, 0x7c, 0x01, 0x81, 0x2c, 0xf7, 0x21, 0xad, 0x1c,
    0xde, 0xd4, 0x6d, 0xe9, 0x83, 0x90, 0x97, 0xdb, 0x72, 0x40, 0xa4, 0xa4, 0xb7, 0xb3, 0x67, 0x1f,
    0xcb, 0x79, 0xe6, 0x4e, 0xcc, 0xc0, 0xe5, 0x78, 0x82, 0x5a, 0xd0, 0x7d, 0xcc, 0xff, 0x72, 0x21,
    0xb8, 0x08, 0x46, 0x74, 0xf7, 0x43, 0x24, 0x8e, 0xe0, 0x35, 0x90, 0xe6, 0x81, 0x3a, 0x26, 0x4c,
    0x3c, 0x28, 0x52, 0xbb, 0x91, 0xc3, 0x00, 0xcb, 0x88, 0xd0, 0x65, 0x8b, 0x1b, 0x53, 0x2e, 0xa3,
    0x71, 0x64, 0x48, 0x97, 0xa2, 0x0d, 0xf9, 0x4e, 0x38, 0x19, 0xef, 0x46, 0xa9, 0xde, 0xac, 0xd8,
    0xa8, 0xfa, 0x76, 0x3f, 0xe3, 0x9c, 0x34, 0x3f, 0xf9, 0xdc, 0xbb, 0xc7, 0xc7, 0x0b, 0x4f, 0x1d,
    0x8a, 0x51, 0xe0, 0x4b, 0xcd, 0xb4, 0x59, 0x31, 0xc8, 0x9f, 0x7e, 0xc9, 0xd9, 0x78, 0x73, 0x64,
    0xea, 0xc5, 0xac, 0x83, 0x34, 0xd3, 0xeb, 0xc3, 0xc5, 0x81, 0xa0, 0xff, 0xfa, 0x13, 0x63, 0xeb,
    0x17, 0x0d, 0xdd, 0x51, 0xb7, 0xf0, 0xda, 0x49, 0xd3, 0x16, 0x55, 0x26, 0x29, 0xd4, 0x68, 0x9e,
    0x2b, 0x16, 0xbe, 0x58, 0x7d, 0x47, 0xa1, 0xfc, 0x8f, 0xf8, 0xb8, 0xd1, 0x7a, 0xd0, 0x31, 0xce,
    0x45, 0xcb, 0x3a, 0x8f, 0x95, 0x16, 0x04, 0x28, 0xaf, 0xd7, 0xfb, 0xca, 0xbb, 0x4b, 0x40, 0x7e,
}};

// Little-endian secret words at any byte offset, folded at compile time.
__host__ __device__ constexpr uint64_t S64(int off) {
    uint64_t v = 0;
    for (int i = 7; i >= 0; --i) v = (v << 8) | kSecret.b[off + i];
    return v;
}
__host__ __device__ constexpr uint32_t S32(int off) {
    uint32_t v = 0;
    for (int i = 3; i >= 0; --i) v = (v << 8) | kSecret.b[off + i];
    return v;
}

constexpr uint32_t P32_1 = 0x9E3779B1U;
constexpr uint32_t P32_2 = 0x85EBCA77U;
constexpr uint32_t P32_3 = 0xC2B2AE3DU;
constexpr uint64_t P64_1 = 0x9E3779B185EBCA87ULL;
constexpr uint64_t P64_2 = 0xC2B2AE3D27D4EB4FULL;
constexpr uint64_t P64_3 = 0x165667B19E3779F9ULL;
constexpr uint64_t P64_4 = 0x85EBCA77C2B2AE63ULL;
constexpr uint64_t P64_5 = 0x27D4EB2F165667C5ULL;
constexpr uint64_t MX1 = 0x165667919E3779F9ULL;
constexpr uint64_t MX2 = 0x9FB21C651E98DF25ULL;

// Initial accumulators of the long path.
__host__ __device__ constexpr uint64_t acc_init(int i) {
    return i == 0 ? (uint64_t)P32_3 : i == 1 ? P64_1 : i == 2 ? P64_2 : i == 3 ? P64_3
         : i == 4 ? P64_4 : i == 5 ? (uint64_t)P32_2 : i == 6 ? P64_5 : (uint64_t)P32_1;
}

__device__ __forceinline__ uint64_t mul_hi64(uint64_t a, uint64_t b) { return __umul64hi(a, b); }
__device__ __forceinline__ uint64_t mul_fold64(uint64_t a, uint64_t b) { return (a * b) ^ __umul64hi(a, b); }
__device__ __forceinline__ uint64_t mul32x32(uint64_t k) { return (uint64_t)(uint32_t)k * (uint64_t)(uint32_t)(k >> 32); }

__device__ __forceinline__ uint64_t avalanche_xxh64(uint64_t h) {
    h ^= h >> 33; h *= P64_2; h ^= h >> 29; h *= P64_3; h ^= h >> 32; return h;
}
__device__ __forceinline__ uint64_t avalanche_xxh3(uint64_t h) {
    h ^= h >> 37; h *= MX1; h ^= h >> 32; return h;
}
// scramble one accumulator lane with key word `key` (= secret[128 + 8i])
__device__ __forceinline__ uint64_t scramble1(uint64_t a, uint64_t key) {
    a ^= a >> 47; a ^= key; a *= (uint64_t)P32_1; return a;
}

// Unaligned-safe little-endian reads (byte-assembled by the compiler where alignment is unknown).
__device__ __forceinline__ uint64_t ld64u(const uint8_t* p) { uint64_t v; __builtin_memcpy(&v, p, 8); return v; }
__device__ __forceinline__ uint32_t ld32u(const uint8_t* p) { uint32_t v; __builtin_memcpy(&v, p, 4); return v; }

struct U128 { uint64_t lo, hi; };

// K1L chain launch: one job (one large buffer) per wave, passed by value as kernel arguments.
// One buffer's K1L chain. Whole-buffer jobs: total_len == len, state == nullptr, flags == 0.
// A huge file is chained in pieces of whole 1 KiB blocks: every piece but the last has
// kChainPartial set (all its len / 1024 blocks are scrambled, the 8 accumulators go to `state`),
// every piece but the first has kChainResume (the accumulators come from `state`); the last piece
// (len > 1024) takes the tail and merges with total_len.
constexpr uint32_t kChainResume = 1, kChainPartial = 2;
struct ChainJob {
    const uint8_t* p;
    uint64_t len;
    const uint64_t* sums;  // 8 u64 block sums per scrambled block
    uint64_t* out;         // 2 u64 (lo, hi)
    uint64_t total_len = 0;
    uint64_t* state = nullptr;
    uint32_t flags = 0;
};
constexpr int kChainJobs = 32;
struct ChainBatch {
    ChainJob job[kChainJobs];
};
// The text counts of up to kChainJobs large items of a staged batch (text_count_kernel's raw newline and
// continuation-byte sums, raw[2q], raw[2q + 1]) written in MetadataText's form to counts[2 j[q]] and
// counts[2 j[q] + 1]: num_lines = 1 + newlines, num_chars = len - continuation bytes.
struct CountFix {
    uint64_t j[kChainJobs], len[kChainJobs];
    int n;
};

// The 24 aligned secret words, for lane-dependent (runtime) indexing on the device.
static __constant__ uint64_t kSecW[24] = {
    S64(0), S64(8), S64(16), S64(24), S64(32), S64(40), S64(48), S64(56),
    S64(64), S64(72), S64(80), S64(88), S64(96), S64(104), S64(112), S64(120),
    S64(128), S64(136), S64(144), S64(152), S64(160), S64(168), S64(176), S64(184)};

__device__ __forceinline__ uint64_t mix16(const uint8_t* in, uint64_t s0, uint64_t s1) {
    return mul_fold64(ld64u(in) ^ s0, ld64u(in + 8) ^ s1);
}
template <int SOFF>
__device__ __forceinline__ void mix32(uint64_t& lo, uint64_t& hi, const uint8_t* a, const uint8_t* b) {
    lo += mix16(a, S64(SOFF), S64(SOFF + 8));
    lo ^= ld64u(b) + ld64u(b + 8);
    hi += mix16(b, S64(SOFF + 16), S64(SOFF + 24));
    hi ^= ld64u(a) + ld64u(a + 8);
}
__device__ __forceinline__ void mix32_rt(uint64_t& lo, uint64_t& hi, const uint8_t* a, const uint8_t* b,
                                         uint64_t s0, uint64_t s1, uint64_t s2, uint64_t s3) {
    lo += mix16(a, s0, s1);
    lo ^= ld64u(b) + ld64u(b + 8);
    hi += mix16(b, s2, s3);
    hi ^= ld64u(a) + ld64u(a + 8);
}

__device__ __forceinline__ U128 finish_mid(uint64_t lo, uint64_t hi, uint64_t len) {
    U128 r;
    r.lo = avalanche_xxh3(lo + hi);
    r.hi = 0 - avalanche_xxh3(lo * P64_1 + hi * P64_4 + len * P64_2);
    return r;
}

// len 0..16
__device__ __forceinline__ U128 xxh3_lane_0to16(const uint8_t* in, uint64_t len) {
    U128 r;
    if (len > 8) {
        const uint64_t ilo = ld64u(in);
        uint64_t ihi = ld64u(in + len - 8);
        uint64_t m = (ilo ^ ihi ^ (S64(32) ^ S64(40)));
        uint64_t mlo = m * P64_1;
        uint64_t mhi = mul_hi64(m, P64_1);
        mlo += (len - 1) << 54;
        ihi ^= (S64(48) ^ S64(56));
        mhi += ihi + (uint64_t)(uint32_t)ihi * (uint64_t)(P32_2 - 1);
        mlo ^= __builtin_bswap64(mhi);
        uint64_t hlo = mlo * P64_2;
        uint64_t hhi = mul_hi64(mlo, P64_2) + mhi * P64_2;
        r.lo = avalanche_xxh3(hlo);
        r.hi = avalanche_xxh3(hhi);
    } else if (len >= 4) {
        const uint64_t in64 = (uint64_t)ld32u(in) + ((uint64_t)ld32u(in + len - 4) << 32);
        const uint64_t keyed = in64 ^ (S64(16) ^ S64(24));
        const uint64_t mul = P64_1 + (len << 2);
        uint64_t mlo = keyed * mul;
        uint64_t mhi = mul_hi64(keyed, mul);
        mhi += mlo << 1;
        mlo ^= mhi >> 3;
        mlo ^= mlo >> 35;
        mlo *= MX2;
        mlo ^= mlo >> 28;
        r.lo = mlo;
        r.hi = avalanche_xxh3(mhi);
    } else if (len) {
        const uint32_t c1 = in[0], c2 = in[len >> 1], c3 = in[len - 1];
        const uint32_t cl = (c1 << 16) | (c2 << 24) | c3 | ((uint32_t)len << 8);
        const uint32_t sw = __builtin_bswap32(cl);
        const uint32_t ch = (sw << 13) | (sw >> 19);
        r.lo = avalanche_xxh64((uint64_t)cl ^ (uint64_t)(S32(0) ^ S32(4)));
        r.hi = avalanche_xxh64((uint64_t)ch ^ (uint64_t)(S32(8) ^ S32(12)));
    } else {
        r.lo = avalanche_xxh64(S64(64) ^ S64(72));
        r.hi = avalanche_xxh64(S64(80) ^ S64(88));
    }
    return r;
}

__device__ __forceinline__ U128 xxh3_lane_17to128(const uint8_t* in, uint64_t len) {
    uint64_t lo = len * P64_1, hi = 0;
    if (len > 32) {
        if (len > 64) {
            if (len > 96) mix32<96>(lo, hi, in + 48, in + len - 64);
            mix32<64>(lo, hi, in + 32, in + len - 48);
        }
        mix32<32>(lo, hi, in + 16, in + len - 32);
    }
    mix32<0>(lo, hi, in, in + len - 16);
    return finish_mid(lo, hi, len);
}

// secret words for the 129..240 tail rounds: offset 3 + 32*t (t = 0..2) -> need S64(3+32t+{0,8,16,24})
__device__ __forceinline__ U128 xxh3_lane_129to240(const uint8_t* in, uint64_t len) {
    uint64_t lo = len * P64_1, hi = 0;
    mix32<0>(lo, hi, in + 0, in + 16);
    mix32<32>(lo, hi, in + 32, in + 48);
    mix32<64>(lo, hi, in + 64, in + 80);
    mix32<96>(lo, hi, in + 96, in + 112);
    lo = avalanche_xxh3(lo);
    hi = avalanche_xxh3(hi);
    // i = 160, 192, 224 while i <= len: secret offset 3 + i - 160
    if (len >= 160) mix32<3>(lo, hi, in + 128, in + 144);
    if (len >= 192) mix32<35>(lo, hi, in + 160, in + 176);
    if (len >= 224) mix32<67>(lo, hi, in + 192, in + 208);
    mix32<103>(lo, hi, in + len - 16, in + len - 32);
    return finish_mid(lo, hi, len);
}

// Scalar (one lane) long path: correct for any len > 240; used only where a lane owns a long item
// (the lane-per-item kernel); the throughput path is the wave-cooperative kernel.
__device__ __noinline__ U128 xxh3_lane_long(const uint8_t* in, uint64_t len) {
    uint64_t acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = acc_init(i);
    const uint64_t nb = (len - 1) / 1024;
    for (uint64_t b = 0; b <= nb; ++b) {
        const uint64_t ns = (b < nb) ? 16 : ((len - 1) - 1024 * nb) / 64;
        for (uint64_t s = 0; s < ns; ++s) {
            const uint8_t* p = in + b * 1024 + s * 64;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const uint64_t v = ld64u(p + 8 * i);
                const uint64_t k = v ^ kSecW[s + i];
                acc[i ^ 1] += v;
                acc[i] += mul32x32(k);
            }
        }
        if (b < nb) {
#pragma unroll
            for (int i = 0; i < 8; ++i) acc[i] = scramble1(acc[i], S64(128 + 8 * i));
        }
    }
    const uint8_t* p = in + len - 64;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint64_t v = ld64u(p + 8 * i);
        const uint64_t k = v ^ S64(121 + 8 * i);
        acc[i ^ 1] += v;
        acc[i] += mul32x32(k);
    }
    uint64_t lo = len * P64_1, hi = ~(len * P64_2);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        lo += mul_fold64(acc[2 * i] ^ S64(11 + 16 * i), acc[2 * i + 1] ^ S64(19 + 16 * i));
        hi += mul_fold64(acc[2 * i] ^ S64(117 + 16 * i), acc[2 * i + 1] ^ S64(125 + 16 * i));
    }
    U128 r;
    r.lo = avalanche_xxh3(lo);
    r.hi = avalanche_xxh3(hi);
    return r;
}

__device__ __forceinline__ U128 xxh3_lane_short(const uint8_t* in, uint64_t len) {
    if (len <= 16) return xxh3_lane_0to16(in, len);
    if (len <= 128) return xxh3_lane_17to128(in, len);
    return xxh3_lane_129to240(in, len);
}

__device__ __forceinline__ U128 xxh3_lane_any(const uint8_t* in, uint64_t len) {
    if (len <= 240) return xxh3_lane_short(in, len);
    return xxh3_lane_long(in, len);
}

}  // namespace oxh
