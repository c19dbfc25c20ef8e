// oxen_amd/csrc/capi_dispatch.hip -- K1 launch shapes and the device-resident entry points of the C ABI
// (include/oxen_hash.h): HBM in, HBM out, asynchronous on the caller's stream; errors and the ABI's
// library-level calls. The other runtime pieces are listed in capi_internal.hpp.
#include "capi_internal.hpp"

using namespace oxh::capi;

namespace oxh::capi {

thread_local std::string g_err;
std::atomic<int> g_variant{0};

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

// ---------------------------------------------------------------- kernel launch helpers
using WaveKernel = void (*)(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);

// The shipped library instantiates the shapes the dispatch below picks (8, 72, 104, 264) and the
// 4-round ring (0) as the fallback for any other forced variant. The experiments that lost their A/Bs
//  are compiled only into the probe build (tools/build_probe_lib.sh, -DOXH_PROBE_VARIANTS).
template <bool DESC>
WaveKernel wave_kernel_for(int variant) {
    switch (variant) {
        case 8: return oxh::xxh3_wave_kernel<DESC, 8>;
        case 72: return oxh::xxh3_wave_kernel<DESC, 72>;
        case 104: return oxh::xxh3_wave_kernel<DESC, 104>;
        case 264: return oxh::xxh3_wave_kernel<DESC, 264>;
#ifdef OXH_PROBE_VARIANTS
        case 1: return oxh::xxh3_wave_kernel<DESC, 1>;
        case 2: return oxh::xxh3_wave_kernel<DESC, 2>;
        case 4: return oxh::xxh3_wave_kernel<DESC, 4>;
        case 12: return oxh::xxh3_wave_kernel<DESC, 12>;
        case 64: return oxh::xxh3_wave_kernel<DESC, 64>;
        case 74: return oxh::xxh3_wave_kernel<DESC, 74>;
        case 40: return oxh::xxh3_wave_kernel<DESC, 40>;
        case 256: return oxh::xxh3_wave_kernel<DESC, 256>;
        case 260: return oxh::xxh3_wave_kernel<DESC, 260>;
        case 768: return oxh::xxh3_wave_kernel<DESC, 768>;
        case 772: return oxh::xxh3_wave_kernel<DESC, 772>;
        case 776: return oxh::xxh3_wave_kernel<DESC, 776>;
        case 1032: return oxh::xxh3_wave_kernel<DESC, 1032>;
        case 1024: return oxh::xxh3_wave_kernel<DESC, 1024>;
#endif
        default: return oxh::xxh3_wave_kernel<DESC, 0>;
    }
}

// K1 register/pipeline shape by item size (measured): items of a few KiB want many
// resident waves (2-round ring, keys in LDS: 77 VGPRs, 6 waves/SIMD, every load issued up front);
// larger items a 2-round ring with the keys in registers (variant 8). The 4-round ring (variant 0,
// 201 VGPRs, 2 waves/SIMD) matches it on equal 64 KiB items but loses 13 % on ragged, packed items
// (FastCDC chunks: tools/k1_align_probe.py) and 4 % of the C2 step rate. An explicit
// oxh_set_kernel_variant() overrides the choice.
//
// Items packed back to back (FastCDC chunks) start at arbitrary byte offsets: a row-wise
// instruction (256 B per row) then touches 3 lines where an aligned one touches 2, 12 lines per KiB
// instead of 8, which costs 6-8 % at 8-64 KiB items; the block-wise layout (variant bit 5) reads a
// whole KiB per instruction, 9 lines. tools/k1_small_probe.py (profiles/r02_k1_small_probe.json):
// packed [4, 16) KiB items 6.17-6.23 TB/s block-wise vs 5.90-5.93 row-wise, packed [4, 128) KiB
// 6.72 vs 6.25; on aligned items the row-wise variants stay ahead (6.75 vs 6.66 at 8 KiB).
// (kShortItemBytes, the variant numbers and ItemShape: capi_internal.hpp)
int pick_variant(ItemShape shape) {
    const int v = g_variant.load();
    if (v != 0) return v;
    return shape == ItemShape::Packed ? kVariantPacked : shape == ItemShape::Short ? kVariantShort : kVariantLong;
}
int pick_variant(bool short_items) { return pick_variant(short_items ? ItemShape::Short : ItemShape::Long); }
// K1R variants (bit 8) hash four items per wave, one per 16-lane row; K1H (bits 8 and 9) two, one per
// pair of rows
uint64_t items_per_wave(int variant) { return (variant & 256) ? ((variant & 512) ? 2 : 4) : 1; }
// a variant wave_kernel_for instantiates, else 0 (its default kernel), so the launch geometry always
// matches the kernel that runs
int known_variant(int v) {
    switch (v) {
        case 8: case 72: case 104: case 264: return v;
#ifdef OXH_PROBE_VARIANTS
        case 1: case 2: case 4: case 12: case 40: case 64: case 74:
        case 256: case 260: case 768: case 772: case 776: case 1024: case 1032: return v;
#endif
        default: return 0;
    }
}

// K1 over a descriptor table: one 64-lane wave per item, 4 waves per 256-thread workgroup.
int launch_wave(const uint8_t* arena, const uint64_t* offs, const uint64_t* lens, uint64_t n, uint64_t* out,
                hipStream_t st, ItemShape shape, int waves, int variant) {
    if (n == 0) return OXH_OK;
    // waves (items) per workgroup: 4, or the caller's choice; OXH_K1_WG_WAVES (1, 2 or 4) overrides
    // both for A/B. A workgroup's slot is freed only when its longest item is done.
    const char* wg = getenv("OXH_K1_WG_WAVES");
    const int e = wg ? atoi(wg) : 0;
    const int w = (e == 1 || e == 2 || e == 4) ? e : (waves == 1 || waves == 2) ? waves : 4;
    const int v = known_variant((variant && g_variant.load() == 0) ? variant : pick_variant(shape));
    const uint64_t per_wg = (uint64_t)w * items_per_wave(v);
    const uint64_t blocks = (n + per_wg - 1) / per_wg;
    hipLaunchKernelGGL(wave_kernel_for<true>(v), dim3((unsigned)blocks), dim3(64 * w), 0, st, arena, offs,
                       lens, n, (uint64_t)0, (uint64_t)0, out);
    HIP_TRY(hipGetLastError());
    return OXH_OK;
}

// K1T: K1 plus text counts in the same pass.
int launch_text(const uint8_t* arena, const uint64_t* offs, const uint64_t* lens, uint64_t n, uint64_t* out,
                uint64_t* counts, hipStream_t st, bool short_items) {
    if (n == 0) return OXH_OK;
    const uint64_t blocks = (n + 3) / 4;
    // K1T keeps the 2-round ring with the keys in LDS at every item size: the counting needs the
    // registers (tools/k1t_probe.py: 6.41 TB/s on C2 and 5.55 on ragged items, against 5.42 / 4.40
    // with variant 8 and 4.32 / 2.56 with the 4-round ring); only that shape ships
    (void)short_items;
    hipLaunchKernelGGL(oxh::xxh3_text_wave_kernel<kVariantShort>, dim3((unsigned)blocks), dim3(256), 0, st, arena, offs, lens,
                       n, out, counts);
    HIP_TRY(hipGetLastError());
    return OXH_OK;
}

// Fixed-size chunks of one buffer (no descriptor table): chunk i = [i*chunk, min((i+1)*chunk, total)).
int launch_chunks(const uint8_t* buf, uint64_t n, uint64_t chunk, uint64_t total, uint64_t* out, hipStream_t st) {
    if (n == 0) return OXH_OK;
    const int v = known_variant(pick_variant(chunk <= kShortItemBytes));
    const uint64_t per_wg = 4 * items_per_wave(v);
    const uint64_t blocks = (n + per_wg - 1) / per_wg;
    hipLaunchKernelGGL(wave_kernel_for<false>(v), dim3((unsigned)blocks), dim3(256), 0, st, buf,
                       (const uint64_t*)nullptr, (const uint64_t*)nullptr, n, chunk, total, out);
    HIP_TRY(hipGetLastError());
    return OXH_OK;
}

int launch_lane(const uint8_t* arena, const uint64_t* offs, const uint64_t* lens, uint64_t n, uint64_t* out,
                hipStream_t st) {
    if (n == 0) return OXH_OK;
    hipLaunchKernelGGL(oxh::xxh3_lane_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, arena, offs, lens, n, out);
    HIP_TRY(hipGetLastError());
    return OXH_OK;
}

}  // namespace oxh::capi

namespace oxh {
// FastCDC's K1 pass (fastcdc.hip) over the packed chunk table. Below a 16 KiB mean chunk K1R (four
// chunks per wave, one per 16-lane row: tools/k1_small_probe.py, profiles/r04g_k1_small_probe.json),
// otherwise the block-wise K1 (one chunk per wave; K1R's four streams per wave lose 10 % on 16-128 KiB
// items); 2 waves per workgroup below 16 KiB, else 4. OXH_K1_PACKED_VARIANT forces a K1 shape (A/B).
int k1_packed(const void* d_arena, const uint64_t* d_offsets, const uint64_t* d_lens, uint64_t n, uint64_t* d_out,
              uint64_t mean_len, hipStream_t st) {
    const bool small = mean_len < kShortItemBytes;
    const char* e = getenv("OXH_K1_PACKED_VARIANT");
    const int v = (e && atoi(e)) ? atoi(e) : small ? kVariantRows : kVariantPacked;
    return launch_wave((const uint8_t*)d_arena, d_offsets, d_lens, n, d_out, st, ItemShape::Packed, small ? 2 : 4, v);
}
}  // namespace oxh

extern "C" {

int oxh_abi_version(void) { return OXH_ABI_VERSION; }

const char* oxh_last_error(void) { return g_err.c_str(); }

int oxh_device_count(int* count) {
    if (!count) return fail(OXH_ERR_INVALID, "count is NULL");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return OXH_OK;
}

int oxh_set_kernel_variant(int variant) { return g_variant.exchange(variant); }

int oxh_xxh3_128_batch_device(const void* d_arena, const uint64_t* d_offsets, const uint64_t* d_lens, uint64_t n,
                              uint64_t* d_out, int mode, void* stream) {
    if (n == 0) return OXH_OK;
    if (!d_arena || !d_offsets || !d_lens || !d_out) return fail(OXH_ERR_INVALID, "NULL device pointer");
    hipStream_t st = (hipStream_t)stream;
    const uint8_t* a = (const uint8_t*)d_arena;
    if (mode == OXH_MODE_LANE) return launch_lane(a, d_offsets, d_lens, n, d_out, st);
    if (mode == OXH_MODE_AUTO || mode == OXH_MODE_WAVE) return launch_wave(a, d_offsets, d_lens, n, d_out, st);
    if (mode == OXH_MODE_WAVE_SHORT) return launch_wave(a, d_offsets, d_lens, n, d_out, st, ItemShape::Short);
    if (mode == OXH_MODE_WAVE_PACKED) return launch_wave(a, d_offsets, d_lens, n, d_out, st, ItemShape::Packed);
    return fail(OXH_ERR_INVALID, "unknown mode");
}

int oxh_chunk_digests_device(const void* d_buf, uint64_t len, uint64_t chunk, uint64_t* d_out, void* stream) {
    if (len == 0) return OXH_OK;
    if (!d_buf || !d_out || chunk == 0) return fail(OXH_ERR_INVALID, "bad chunk arguments");
    return launch_chunks((const uint8_t*)d_buf, (len + chunk - 1) / chunk, chunk, len, d_out, (hipStream_t)stream);
}

int oxh_xxh3_128_large_device(oxh_ctx* c, const void* d_buf, uint64_t len, uint64_t* d_out, void* stream) {
    if (!c || !d_out || (!d_buf && len)) return fail(OXH_ERR_INVALID, "bad large-buffer arguments");
    std::lock_guard<std::mutex> g(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t st = (hipStream_t)stream;  // NULL = the null stream, as for every device entry point
    return large_device(c, (const uint8_t*)d_buf, len, d_out, st);
}

int oxh_xxh3_128_large_batch_device(const void* const* d_bufs, const uint64_t* lens, uint64_t n, uint64_t* d_out,
                                    void* stream) {
    if (n == 0) return OXH_OK;
    if (!d_bufs || !lens || !d_out) return fail(OXH_ERR_INVALID, "bad large-batch arguments");
    for (uint64_t i = 0; i < n; ++i)
        if (!d_bufs[i] && lens[i]) return fail(OXH_ERR_INVALID, "NULL buffer with nonzero length");
    return large_batch_device((const uint8_t* const*)d_bufs, lens, n, d_out, (hipStream_t)stream);
}

int oxh_combined_hash_device(const uint64_t* d_content, const uint64_t* d_metadata, uint64_t n, uint64_t* d_out,
                             void* stream) {
    if (n == 0) return OXH_OK;
    if (!d_content || !d_metadata || !d_out) return fail(OXH_ERR_INVALID, "NULL device pointer");
    hipLaunchKernelGGL(oxh::xxh3_combined_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       d_content, d_metadata, n, d_out);
    HIP_TRY(hipGetLastError());
    return OXH_OK;
}

int oxh_xxh3_128_text_batch_device(const void* d_arena, const uint64_t* d_offsets, const uint64_t* d_lens, uint64_t n,
                                   uint64_t* d_out, uint64_t* d_counts, void* stream) {
    if (n == 0) return OXH_OK;
    if (!d_arena || !d_offsets || !d_lens || !d_out || !d_counts) return fail(OXH_ERR_INVALID, "NULL device pointer");
    return launch_text((const uint8_t*)d_arena, d_offsets, d_lens, n, d_out, d_counts, (hipStream_t)stream);
}

int oxh_utf8_prefix_device(const void* d_arena, const uint64_t* d_offsets, const uint64_t* d_lens, uint64_t n,
                           int32_t* d_flags, void* stream) {
    if (n == 0) return OXH_OK;
    if (!d_arena || !d_offsets || !d_lens || !d_flags) return fail(OXH_ERR_INVALID, "NULL device pointer");
    hipLaunchKernelGGL(oxh::utf8_prefix_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       (const uint8_t*)d_arena, d_offsets, d_lens, n, d_flags);
    HIP_TRY(hipGetLastError());
    return OXH_OK;
}

int oxh_fill_splitmix(void* d_buf, uint64_t nbytes, uint64_t seed, void* stream) {
    if (!d_buf && nbytes) return fail(OXH_ERR_INVALID, "NULL buffer");
    if ((reinterpret_cast<uintptr_t>(d_buf) & 7) != 0) return fail(OXH_ERR_INVALID, "buffer must be 8-byte aligned");
    const uint64_t nwords = nbytes / 8;
    if (nwords) {
        const uint64_t blocks = std::min<uint64_t>((nwords + 255) / 256, 256ull * 64);
        hipLaunchKernelGGL(oxh::fill_splitmix_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                           (uint64_t*)d_buf, nwords, seed);
        HIP_TRY(hipGetLastError());
    }
    if (nbytes % 8) {
        hipLaunchKernelGGL(oxh::fill_splitmix_tail_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream,
                           (uint8_t*)d_buf + nwords * 8, nwords, nbytes % 8, seed);
        HIP_TRY(hipGetLastError());
    }
    return OXH_OK;
}

int oxh_format_hex(uint64_t lo, uint64_t hi, char* out) {
    if (!out) return 0;
    unsigned __int128 v = ((unsigned __int128)hi << 64) | lo;
    char tmp[33];
    int n = 0;
    do {
        tmp[n++] = "0123456789abcdef"[(int)(v & 15)];
        v >>= 4;
    } while (v);
    for (int i = 0; i < n; ++i) out[i] = tmp[n - 1 - i];
    out[n] = 0;
    return n;
}

int oxh_format_dec(uint64_t lo, uint64_t hi, char* out) {
    if (!out) return 0;
    unsigned __int128 v = ((unsigned __int128)hi << 64) | lo;
    char tmp[40];
    int n = 0;
    do {
        tmp[n++] = (char)('0' + (int)(v % 10));
        v /= 10;
    } while (v);
    for (int i = 0; i < n; ++i) out[i] = tmp[n - 1 - i];
    out[n] = 0;
    return n;
}

}  // extern "C"
