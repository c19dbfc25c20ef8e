/*
 * oracle/fastcdc_oracle.c -- TEST INFRASTRUCTURE ONLY. NOT PART OF THE PRODUCT PATH.
 *
 * Scalar CPU restatement of FastCDC "v2020" content-defined chunking as the block-level dedup
 * experiment calls it: experiments/block-level-dedup/src/chunker/fastcdchunker.rs:83-88
 * `v2020::FastCDC::new(&file_content, min_chunk_size, avg_chunk_size, max_chunk_size)` with
 * min = 4096, avg = chunk_size, max = 2 * chunk_size (:55-57), then xxh3_128 of every chunk (:98).
 *
 * The algorithm lives in the third-party crate `fastcdc` 3.2.1 (experiments/block-level-dedup/
 * Cargo.lock), which is NOT vendored under /root/reference. This file restates its published
 * v2020 algorithm:
 *   - FastCDC::new = with_level(.., Normalization::Level1); bits = round(log2(avg));
 *     mask_s = MASKS[bits + 1], mask_l = MASKS[bits - 1]; mask_*_ls = mask_* << 1;
 *   - cut_gear: `remaining <= min` -> whole remainder; center = avg, clamped to remaining;
 *     remaining clamped to max; hash = 0 at index = min/2; the loop rolls TWO bytes per step
 *     (hash = (hash << 2) + GEAR_LS[b[2i]], test mask_*_ls, return 2i; hash += GEAR[b[2i+1]],
 *     test mask_*, return 2i+1) with mask_s while index < center/2, mask_l while < remaining/2;
 *     otherwise the chunk is `remaining` long;
 *   - the iterator emits (offset, length = cutpoint) and advances by the cutpoint.
 * The 256-entry GEAR table is an INPUT here: tests derive it from the crate's documented rule (the
 * high 8 bytes of MD5 over 64 copies of the byte value, oracle/fastcdc.py), independently of the
 * product's compiled-in copy. Parity against a reference run is UNPINNED: the reference's tests
 * hold no FastCDC fixtures and the crate cannot be built here (no cargo, no network).
 */
#include <stdint.h>
#include <string.h>

typedef uint64_t u64;
typedef uint32_t u32;
typedef uint8_t u8;

/* fastcdc::v2020::MASKS -- index = number of one bits (entries 0..4 padding) */
static const u64 kMasks[26] = {
    0, 0, 0, 0, 0,
    0x0000000001804110ULL, 0x0000000001803110ULL, 0x0000000018035100ULL, 0x0000001800035300ULL,
    0x0000019000353000ULL, 0x0000590003530000ULL, 0x0000d90003530000ULL, 0x0000d90103530000ULL,
    0x0000d90303530000ULL, 0x0000d90313530000ULL, 0x0000d90f03530000ULL, 0x0000d90303537000ULL,
    0x0000d90703537000ULL, 0x0000d90707537000ULL, 0x0000d91707537000ULL, 0x0000d91747537000ULL,
    0x0000d91767537000ULL, 0x0000d93767537000ULL, 0x0000d93777537000ULL, 0x0000d93777577000ULL,
    0x0000db3777577000ULL,
};

static u32 log2_round(u32 v) {
    /* (v as f64).log2().round() as u32 */
    u32 b = 31 - (u32)__builtin_clz(v);
    /* round up when v >= 2^b * sqrt(2) */
    const double x = (double)v, lo = (double)(1u << b);
    return (x * x >= 2.0 * lo * lo) ? b + 1 : b;
}

int oxo_fastcdc_masks(u32 avg, u32 level, u64 out[2]) {
    const u32 bits = log2_round(avg);
    if (bits + level > 25 || bits < level + 5) return -1;
    out[0] = kMasks[bits + level];
    out[1] = kMasks[bits - level];
    return 0;
}

/* cut_gear over src[0..len): returns the cutpoint (chunk length). */
static u64 cut_gear(const u8* src, u64 len, u64 min, u64 avg, u64 max, u64 mask_s, u64 mask_l,
                    const u64* gear) {
    u64 remaining = len;
    if (remaining <= min) return remaining;
    u64 center = avg;
    if (remaining > max) remaining = max;
    else if (remaining < center) center = remaining;
    const u64 mask_s_ls = mask_s << 1, mask_l_ls = mask_l << 1;
    u64 index = min / 2;
    u64 hash = 0;
    while (index < center / 2) {
        const u64 a = index * 2;
        hash = (hash << 2) + (gear[src[a]] << 1);
        if ((hash & mask_s_ls) == 0) return a;
        hash = hash + gear[src[a + 1]];
        if ((hash & mask_s) == 0) return a + 1;
        index += 1;
    }
    while (index < remaining / 2) {
        const u64 a = index * 2;
        hash = (hash << 2) + (gear[src[a]] << 1);
        if ((hash & mask_l_ls) == 0) return a;
        hash = hash + gear[src[a + 1]];
        if ((hash & mask_l) == 0) return a + 1;
        index += 1;
    }
    return remaining;
}

/* All chunks of src[0..len): writes up to cap (offset, length) pairs, returns the chunk count
 * (which may exceed cap; then only the first cap were written). */
u64 oxo_fastcdc(const u8* src, u64 len, u32 min, u32 avg, u32 max, u32 level, const u64* gear,
                u64* offsets, u64* lengths, u64 cap) {
    u64 m[2];
    if (oxo_fastcdc_masks(avg, level, m) != 0) return 0;
    u64 processed = 0, n = 0;
    while (processed < len) {
        const u64 cut = cut_gear(src + processed, len - processed, min, avg, max, m[0], m[1], gear);
        if (cut == 0) break;
        if (n < cap) {
            offsets[n] = processed;
            lengths[n] = cut;
        }
        ++n;
        processed += cut;
    }
    return n;
}
