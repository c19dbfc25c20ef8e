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
#define _GNU_SOURCE
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

/* ---- files: the reference's pack() loop minus the chunk-file writes, one thread per file ----
 * fastcdchunker.rs:75-98 per file: fs::read(input_file) (mode 0: read() of the whole file into a
 * malloc'd buffer, as fs::read does; mode 1: a read-only mmap, for sets whose whole-file buffers would
 * not fit in host memory beside the page cache), v2020 chunking, xxh3_128 of every chunk. Files are
 * taken by `nthreads` threads from a shared counter (the reference's pack is single-threaded per file;
 * the files of a set are independent). Per file: the chunk count and fp = XXH3-128 of its records
 * (offset, length, digest lo, digest hi as u64 LE per chunk) -- the GPU table is fingerprinted the
 * same way by the caller -- and status 0 / 1 open / 2 read / 3 memory. */
#include <fcntl.h>
#include <pthread.h>
#include <stdlib.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

void oxo_xxh3_128(const void* data, uint64_t len, uint64_t out[2]);

typedef struct {
    const char* const* paths;
    u64 n;
    u32 min, avg, max, level;
    const u64* gear;
    int mode;
    u64 fixed;  /* > 0: fixed-size chunks of this many bytes instead of FastCDC */
    u64* counts;
    u64* fp;
    int32_t* status;
    u64 next;  /* shared file counter (atomic) */
} cdc_files_job;

static int cdc_one_file(cdc_files_job* j, u64 i) {
    const int fd = open(j->paths[i], O_RDONLY | O_CLOEXEC);
    if (fd < 0) return 1;
    struct stat sb;
    if (fstat(fd, &sb) != 0) { close(fd); return 2; }
    const u64 sz = (u64)sb.st_size;
    u8* buf = NULL;
    int mapped = 0;
    if (sz && j->mode == 1) {
        void* m = mmap(NULL, sz, PROT_READ, MAP_PRIVATE, fd, 0);
        if (m == MAP_FAILED) { close(fd); return 3; }
        buf = (u8*)m;
        mapped = 1;
    } else {
        buf = (u8*)malloc(sz ? sz : 1);
        if (!buf) { close(fd); return 3; }
        u64 got = 0;
        while (got < sz) {
            const ssize_t r = read(fd, buf + got, sz - got);
            if (r <= 0) { free(buf); close(fd); return 2; }
            got += (u64)r;
        }
    }
    close(fd);
    u64 m[2] = {0, 0};
    if (!j->fixed) oxo_fastcdc_masks(j->avg, j->level, m);
    const u64 cap = sz / (j->fixed ? j->fixed : j->min ? j->min : 1) + 2;
    u64* rec = (u64*)malloc(cap * 4 * sizeof(u64));
    if (!rec) { if (mapped) munmap(buf, sz); else free(buf); return 3; }
    u64 processed = 0, k = 0;
    while (processed < sz) {
        const u64 cut = j->fixed ? (sz - processed < j->fixed ? sz - processed : j->fixed)
                                 : cut_gear(buf + processed, sz - processed, j->min, j->avg, j->max, m[0], m[1], j->gear);
        if (cut == 0 || k >= cap) break;
        u64 d[2];
        oxo_xxh3_128(buf + processed, cut, d);
        rec[4 * k] = processed;
        rec[4 * k + 1] = cut;
        rec[4 * k + 2] = d[0];
        rec[4 * k + 3] = d[1];
        ++k;
        processed += cut;
    }
    j->counts[i] = k;
    oxo_xxh3_128(rec, k * 4 * sizeof(u64), j->fp + 2 * i);
    free(rec);
    if (mapped) munmap(buf, sz); else free(buf);
    return 0;
}

static void* cdc_files_worker(void* arg) {
    cdc_files_job* j = (cdc_files_job*)arg;
    for (;;) {
        const u64 i = __atomic_fetch_add(&j->next, 1, __ATOMIC_RELAXED);
        if (i >= j->n) break;
        j->counts[i] = 0;
        j->fp[2 * i] = j->fp[2 * i + 1] = 0;
        j->status[i] = cdc_one_file(j, i);
    }
    return NULL;
}

void oxo_fastcdc_files(const char* const* paths, u64 n, u32 min, u32 avg, u32 max, u32 level, const u64* gear,
                       int mode, int nthreads, u64* counts, u64* fp, int32_t* status) {
    cdc_files_job j;
    memset(&j, 0, sizeof j);
    j.paths = paths, j.n = n, j.min = min, j.avg = avg, j.max = max, j.level = level, j.gear = gear, j.mode = mode;
    j.counts = counts, j.fp = fp, j.status = status;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    for (int t = 1; t < nthreads; ++t) pthread_create(&th[t], NULL, cdc_files_worker, &j);
    cdc_files_worker(&j);
    for (int t = 1; t < nthreads; ++t) pthread_join(th[t], NULL);
}

/* fixedsize_multithreaded.rs:78-110 per file: chunk i = [i*chunk, min((i+1)*chunk, size)), xxh3_128 of
 * each; the same per-file records / fingerprint as oxo_fastcdc_files. */
void oxo_fixed_files(const char* const* paths, u64 n, u64 chunk, int mode, int nthreads, u64* counts, u64* fp,
                     int32_t* status) {
    cdc_files_job j;
    memset(&j, 0, sizeof j);
    j.paths = paths, j.n = n, j.fixed = chunk ? chunk : 1, j.mode = mode;
    j.counts = counts, j.fp = fp, j.status = status;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    for (int t = 1; t < nthreads; ++t) pthread_create(&th[t], NULL, cdc_files_worker, &j);
    cdc_files_worker(&j);
    for (int t = 1; t < nthreads; ++t) pthread_join(th[t], NULL);
}
