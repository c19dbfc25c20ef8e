// oxen_amd/csrc/oxen_hash_capi.hip -- host runtime + extern "C" boundary (include/oxen_hash.h).
//
// The runtime replaces the per-file hashing inside liboxen's add loop
// (core/v_latest/add.rs:444-545 -> util/hasher.rs:56-65) with batched device work:
//   * a context owns a compute stream, a copy stream and NSLOT pinned/device staging slots;
//   * host-resident batches are packed into a slot at 256-B aligned offsets (file readers pread
//     straight into pinned memory), copied H2D on the copy stream, hashed by K1 on the compute
//     stream, and the 16-B digests come back D2H -- while the next slot is being filled;
//   * device-resident batches go straight to the kernels.
// There is no CPU hashing path here: every digest this library returns was computed on the GPU.
#include <hip/hip_runtime.h>
#include <dirent.h>
#include <sched.h>
#include <errno.h>
#include <fcntl.h>
#include <ftw.h>
#include <stdint.h>
#include <string.h>
#include <sys/resource.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "../../include/oxen_hash.h"
#include "pool.hpp"
#include "scratch.hpp"
#include "xxh3_device.hpp"

namespace oxh {
template <bool DESC, int VARIANT>
__global__ void xxh3_wave_kernel(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*);
__global__ void xxh3_lane_kernel(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t*);
__global__ void xxh3_combined_kernel(const uint64_t*, const uint64_t*, uint64_t, uint64_t*);
template <bool ALIGNED>
__global__ void xxh3_blocksum_kernel(const uint8_t*, uint64_t, uint64_t*);
__global__ void xxh3_chain_kernel(ChainBatch);
__global__ void fill_splitmix_kernel(uint64_t*, uint64_t, uint64_t);
template <int VARIANT>
__global__ void xxh3_text_wave_kernel(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, uint64_t*, uint64_t*);
__global__ void text_count_kernel(const uint8_t*, uint64_t, unsigned long long*);
__global__ void utf8_prefix_kernel(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, int32_t*);
__global__ void fill_splitmix_tail_kernel(uint8_t*, uint64_t, uint64_t, uint64_t);
}  // namespace oxh

namespace {

thread_local std::string g_err;
std::atomic<int> g_variant{0};

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                      \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess)                                                              \
            return fail(OXH_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));  \
    } while (0)

constexpr uint64_t kAlign = 256;
constexpr int NSLOT = 3;
inline uint64_t align_up(uint64_t x) { return (x + kAlign - 1) & ~(kAlign - 1); }

int check_device(int device) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(OXH_ERR_NODEVICE, "no HIP device visible");
    if (device < 0 || device >= n) return fail(OXH_ERR_INVALID, "device index out of range");
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return fail(OXH_ERR_NODEVICE, "hipGetDeviceProperties failed");
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(OXH_ERR_NODEVICE, std::string("device is ") + prop.gcnArchName + ", this library is built for gfx950");
    return OXH_OK;
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
constexpr uint64_t kShortItemBytes = 16384;
constexpr int kVariantShort = 72;    // Cfg: row-wise, depth 2, keys in LDS
constexpr int kVariantLong = 8;      // Cfg: row-wise, depth 2, keys from the constant table
constexpr int kVariantPacked = 104;  // Cfg: block-wise, depth 2, keys in LDS
constexpr int kVariantRows = 264;    // Cfg: K1R (a 16-lane row per item), depth 2

enum class ItemShape { Long, Short, Packed };

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
                hipStream_t st, ItemShape shape = ItemShape::Long, int waves = 4, int variant = 0) {
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
                uint64_t* counts, hipStream_t st, bool short_items = false) {
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

// CPUs this process may use: the affinity mask, capped by a cgroup-v2 CPU quota (a container's
// cpu.max, e.g. "1600000 100000" = 16 CPUs); hardware_concurrency() sees the whole machine.
int usable_cpus() {
    unsigned n = std::thread::hardware_concurrency();
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0 && CPU_COUNT(&set) > 0) n = (unsigned)CPU_COUNT(&set);
    if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char quota[32] = {0};
        unsigned long long period = 0;
        if (fscanf(f, "%31s %llu", quota, &period) == 2 && strcmp(quota, "max") != 0 && period > 0) {
            const unsigned long long q = strtoull(quota, nullptr, 10);
            const unsigned cap = (unsigned)std::max<unsigned long long>(1, (q + period - 1) / period);
            n = n ? std::min(n, cap) : cap;
        }
        fclose(f);
    }
    return (int)(n ? n : 4);
}

int default_threads() {
    const char* e = getenv("OXH_NUM_THREADS");  // cf. OXEN_NUM_THREADS (util/concurrency.rs:1-45)
    if (e && atoi(e) > 0) return atoi(e);
    return std::max(1, std::min(usable_cpus(), 16));
}



}  // namespace

namespace oxh {
// for the other translation units of the library (fastcdc.hip, fastcdc_host.cpp, comm.cpp)
int set_error(int code, const std::string& msg) { return fail(code, msg); }
int cpu_quota() { return usable_cpus(); }
int default_reader_threads() { return default_threads(); }
}  // namespace oxh

// ---------------------------------------------------------------- context
struct oxh_ctx {
    int device = 0;
    hipStream_t stream = nullptr, copy_stream = nullptr;
    hipStream_t copy_stream2 = nullptr;  // large items: every other bounce window's H2D (created on first use)
    hipEvent_t ev_copy2_join = nullptr;  // copy_stream waits for copy_stream2's windows of a piece
    std::atomic<const char*> where{"-"};  // where the engine / large-item path last blocked (stall reports)
    uint64_t stage_bytes = 0, max_items = 0;
    uint8_t* h_stage[NSLOT] = {};
    uint8_t* d_stage[NSLOT] = {};
    uint64_t* h_desc[NSLOT] = {};  // [offsets(max_items) | lens(max_items)]
    uint64_t* d_desc[NSLOT] = {};
    uint64_t* h_out[NSLOT] = {};
    uint64_t* d_out[NSLOT] = {};
    uint64_t* h_cnt[NSLOT] = {};  // text counts (num_lines, num_chars) per item, K1T
    uint64_t* d_cnt[NSLOT] = {};
    int32_t* h_utf8[NSLOT] = {};  // is_utf8 of each item's first 4 KiB (util/fs.rs:652-668)
    int32_t* d_utf8[NSLOT] = {};
    // streaming file engine (see run_stream): file calls queue requests here; the engine thread runs
    // them, and requests arriving while it runs join the live pipeline
    std::mutex qmu;
    std::condition_variable qcv;  // a request was queued (or the engine must stop)
    std::vector<struct FileRequest*> queue;
    bool stop = false;
    std::thread engine;
    uint64_t flush_bytes = 0;  // seal a partly filled slot at this many bytes when the next slot is free
    // files larger than a staging slot (see big_file): a device buffer kept at the largest size seen
    // and two pinned bounce buffers the file is read into in pieces
    uint8_t* d_big = nullptr;
    uint64_t d_big_size = 0;
    uint64_t d_big_allocs = 0;   // times d_big was (re)allocated (oxh_ctx_counters)
    uint8_t* h_bounce[8] = {};   // kNBounce pinned bounce buffers, used as a ring
    hipEvent_t ev_bounce[8] = {};
    bool bounce_used[8] = {};
    uint64_t bounce_next = 0;    // the ring position (kept across pieces and files)
    hipEvent_t ev_piece_free[2] = {};
    void* live = nullptr;  // the engine's current run (a FileStream, for diagnostics), under qmu
    std::vector<struct FileRequest*> rq[NSLOT];  // per staged item: its request and index in it
    std::vector<uint64_t> loc[NSLOT];
    hipEvent_t ev_copied[NSLOT] = {}, ev_done[NSLOT] = {};
    oxh::Pool* pool = nullptr;   // readers / copiers (fill)
    oxh::Pool* wpool = nullptr;  // consumers of hashed bytes (fused publish), created on first use
    oxh::Pool* rpool = nullptr;  // streaming-pipeline file readers (stream_files)
    std::mutex mu;
    void* cdc = nullptr;                 // FastCDC host pipeline (fastcdc_host.cpp), created on first use
    void (*cdc_free)(void*) = nullptr;
};

namespace {

void engine_main(oxh_ctx* c);  // the streaming file engine's thread (below)

// The chain kernel is VALU-issue-bound per wave (every wave64 instruction takes 4 cycles whatever
// the exec mask), so two chains on one SIMD run at half speed each. Unused dynamic LDS on top of the
// kernel's 32 KiB makes every chain workgroup need more than half a CU's 160 KiB: one chain per CU.
constexpr size_t kChainLdsPad = 50 * 1024;

// K1L over n device buffers. Buffers below ~1 MiB take one K1 wave. The others are processed in
// rounds of 1 GiB pieces (OXH_BIG_PIECE_MIB): round r computes the block sums of every buffer's
// piece r chip-wide on `st` while the serial chains of round r-1 run on the scratch buffer's own
// stream, up to kChainJobs chains per launch (ChainJob resume / partial flags carry each buffer's 8
// accumulators from piece to piece), so a chain starts one piece's block sums after its buffer does
// instead of after every buffer's, and the block-sum scratch is two rounds of pieces, not the whole
// input. Returns after `st` has finished.
int large_batch_device(const uint8_t* const* bufs, const uint64_t* lens, uint64_t n, uint64_t* d_out, hipStream_t st) {
    const char* pe = getenv("OXH_BIG_PIECE_MIB");
    const uint64_t P = std::max<uint64_t>(1, pe ? strtoull(pe, nullptr, 10) : 1024) << 20;
    std::vector<uint64_t> big;  // buffers on the chained path
    uint64_t rounds = 0;
    auto pieces_of = [&](uint64_t len) { return (len > P + 1024 ? (len - 1025) / P : 0) + 1; };
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t len = lens[i];
        const uint64_t nb = len > 0 ? (len - 1) >> 10 : 0;
        if (nb < 1024) {
            if (int rc = launch_chunks(bufs[i], 1, len, len, d_out + 2 * i, st)) return rc;
            continue;
        }
        big.push_back(i);
        rounds = std::max(rounds, pieces_of(len));
    }
    if (big.empty()) return OXH_OK;
    oxh::ScratchLease lease(st);  // the device's cached scratch (scratch.hpp); synchronises st at the end
    const uint64_t per_buf = ((P + 1024) >> 10) * 8;  // block-sum u64 per buffer per round
    uint64_t* scratch = nullptr;
    HIP_TRY(lease.get((2 * per_buf * big.size() + 8 * big.size()) * 8, (void**)&scratch));
    uint64_t* state = scratch + 2 * per_buf * big.size();  // 8 accumulators per buffer
    hipStream_t aux = nullptr;
    hipEvent_t* ev = nullptr;
    HIP_TRY(lease.aux(&aux, &ev));
    hipEvent_t* ev_sums = ev;       // [2] block sums of round r (parity) are ready
    hipEvent_t* ev_chain = ev + 2;  // [2] chains of round r (parity) are done with them
    for (uint64_t r = 0; r < rounds; ++r) {
        const int b = (int)(r & 1);
        if (r >= 2) HIP_TRY(hipStreamWaitEvent(st, ev_chain[b], 0));  // round r-2 read these sums
        oxh::ChainBatch batch;
        int nj = 0;
        auto flush = [&]() -> int {
            if (!nj) return OXH_OK;
            hipLaunchKernelGGL(oxh::xxh3_chain_kernel, dim3(nj), dim3(64), kChainLdsPad, aux, batch);
            HIP_TRY(hipGetLastError());
            nj = 0;
            return OXH_OK;
        };
        std::vector<oxh::ChainJob> jobs;
        for (uint64_t q = 0; q < big.size(); ++q) {
            const uint64_t i = big[q], len = lens[i], k = pieces_of(len) - 1;
            if (r > k) continue;
            const uint64_t off = r * P, plen = r < k ? P : len - off;
            const bool last = r == k;
            const uint64_t nb = last ? (plen - 1) >> 10 : plen >> 10;
            uint64_t* s_q = scratch + ((uint64_t)b * big.size() + q) * per_buf;
            const uint8_t* p = bufs[i] + off;
            const bool aligned = (reinterpret_cast<uintptr_t>(p) & 15) == 0;
            const uint64_t nwaves = (nb + 3) / 4, blocks = (nwaves + 3) / 4;
            if (aligned)
                hipLaunchKernelGGL(oxh::xxh3_blocksum_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, st, p, nb, s_q);
            else
                hipLaunchKernelGGL(oxh::xxh3_blocksum_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, st, p, nb, s_q);
            HIP_TRY(hipGetLastError());
            jobs.push_back({p, plen, s_q, d_out + 2 * i, len, state + 8 * q,
                            (r > 0 ? oxh::kChainResume : 0u) | (last ? 0u : oxh::kChainPartial)});
        }
        HIP_TRY(hipEventRecord(ev_sums[b], st));
        HIP_TRY(hipStreamWaitEvent(aux, ev_sums[b], 0));
        for (const oxh::ChainJob& j : jobs) {
            batch.job[nj++] = j;
            if (nj == oxh::kChainJobs)
                if (int rc = flush()) return rc;
        }
        if (int rc = flush()) return rc;
        HIP_TRY(hipEventRecord(ev_chain[b], aux));
    }
    HIP_TRY(hipStreamWaitEvent(st, ev_chain[(rounds - 1) & 1], 0));  // st continues after every chain
    return OXH_OK;
}

int large_device(oxh_ctx*, const uint8_t* d_buf, uint64_t len, uint64_t* d_out, hipStream_t st) {
    return large_batch_device(&d_buf, &len, 1, d_out, st);
}

// OXH_DEBUG_STEPS=1: one stderr line per runtime step (locating stalls without a debugger)
static const bool g_steps = getenv("OXH_DEBUG_STEPS") != nullptr;
#define STEP(...)                                  \
    do {                                           \
        if (g_steps) {                             \
            fprintf(stderr, "[oxh-step] " __VA_ARGS__); \
            fputc('\n', stderr);                   \
        }                                          \
    } while (0)

// One staged batch: items [0, cnt) already in h_stage[s] at h_desc offsets; launch and queue D2H.
int submit_slot(oxh_ctx* c, int s, uint64_t bytes, uint64_t cnt, bool any_short_only, bool short_items, bool text,
                bool utf8 = false) {
    const uint64_t M = c->max_items;
    STEP("submit s=%d bytes=%llu cnt=%llu lane=%d short=%d", s, (unsigned long long)bytes, (unsigned long long)cnt,
         (int)any_short_only, (int)short_items);
    c->where.store("submit_slot: H2D stage");
    HIP_TRY(hipMemcpyAsync(c->d_stage[s], c->h_stage[s], bytes, hipMemcpyHostToDevice, c->copy_stream));
    c->where.store("submit_slot: H2D desc");
    HIP_TRY(hipMemcpyAsync(c->d_desc[s], c->h_desc[s], cnt * 8, hipMemcpyHostToDevice, c->copy_stream));
    HIP_TRY(hipMemcpyAsync(c->d_desc[s] + M, c->h_desc[s] + M, cnt * 8, hipMemcpyHostToDevice, c->copy_stream));
    c->where.store("submit_slot: record / wait");
    HIP_TRY(hipEventRecord(c->ev_copied[s], c->copy_stream));
    HIP_TRY(hipStreamWaitEvent(c->stream, c->ev_copied[s], 0));
    STEP("copies queued s=%d", s);
    c->where.store("submit_slot: launch");
    int rc = text ? launch_text(c->d_stage[s], c->d_desc[s], c->d_desc[s] + M, cnt, c->d_out[s], c->d_cnt[s], c->stream,
                                short_items)
             : any_short_only ? launch_lane(c->d_stage[s], c->d_desc[s], c->d_desc[s] + M, cnt, c->d_out[s], c->stream)
                              : launch_wave(c->d_stage[s], c->d_desc[s], c->d_desc[s] + M, cnt, c->d_out[s], c->stream,
                                            short_items ? ItemShape::Short : ItemShape::Long);
    if (rc) return rc;
    STEP("launched s=%d", s);
    c->where.store("submit_slot: D2H");
    HIP_TRY(hipMemcpyAsync(c->h_out[s], c->d_out[s], cnt * 16, hipMemcpyDeviceToHost, c->stream));
    if (text) HIP_TRY(hipMemcpyAsync(c->h_cnt[s], c->d_cnt[s], cnt * 16, hipMemcpyDeviceToHost, c->stream));
    if (utf8) {  // is_utf8 sniff of the same staged bytes
        hipLaunchKernelGGL(oxh::utf8_prefix_kernel, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, c->stream, c->d_stage[s],
                           c->d_desc[s], c->d_desc[s] + M, cnt, c->d_utf8[s]);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(c->h_utf8[s], c->d_utf8[s], cnt * 4, hipMemcpyDeviceToHost, c->stream));
    }
    c->where.store("submit_slot: record done");
    HIP_TRY(hipEventRecord(c->ev_done[s], c->stream));
    STEP("submitted s=%d", s);
    return OXH_OK;
}

// OXH_TRACE=1: per-call stage times on stderr (host-side wall clock)
struct Trace {
    bool on = getenv("OXH_TRACE") != nullptr;
    double fill = 0, drain = 0, submit = 0;
    int batches = 0;
    static double now() {
        return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
    }
};

// Consumer of the exact bytes that were hashed (the fused version-store copy of oxh_add_files).
//  * put(): an item whose digest is known, with its staged (pinned) bytes still in place; called
//    from several threads at once for the items of a drained slot;
//  * open_stream() / close_stream(): a file larger than a staging slot, whose bytes pass through
//    bounce buffers piece by piece: the engine writes each piece to the returned fd while the
//    digest is still being computed, then hands over the digest (or ok = false);
//  * commit(): everything put / closed so far is to be made durable and visible; the engine calls it
//    once per drained slot. The sink may do that work asynchronously; its owner waits for it before
//    reading outcomes.
// Publish failures are the sink's own business (oxh_add_files turns them into per-item statuses).
struct ItemSink {
    virtual ~ItemSink() = default;
    virtual void put(uint64_t id, const uint8_t* bytes, uint64_t len, uint64_t lo, uint64_t hi) = 0;
    virtual int open_stream(uint64_t id, std::string& tmp) = 0;
    virtual void close_stream(uint64_t id, int fd, const std::string& tmp, bool ok, uint64_t lo, uint64_t hi) = 0;
    virtual void commit() = 0;
};

struct Pending {
    bool busy = false;
    std::vector<uint64_t> ids;  // caller indices of the staged items
};

// Wait for slot s's digests. Polls (a slot is at most a few hundred MiB: milliseconds of work) and,
// after OXH_WAIT_LIMIT_S seconds (default 60), reports which stage never finished instead of
// blocking forever.
int wait_slot(oxh_ctx* c, int s, const Pending& p) {
    static const double limit = getenv("OXH_WAIT_LIMIT_S") ? atof(getenv("OXH_WAIT_LIMIT_S")) : 60.0;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t spin = 0;; ++spin) {
        const hipError_t q = hipEventQuery(c->ev_done[s]);
        if (q == hipSuccess) return OXH_OK;
        if (q != hipErrorNotReady) return fail(OXH_ERR_HIP, std::string("slot event: ") + hipGetErrorString(q));
        if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(20));
        if ((spin & 1023) == 0 &&
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit) {
            const uint64_t M = c->max_items;
            fprintf(stderr, "[oxh] slot %d stalled: items=%zu copied=%s copy_stream=%s stream=%s first lens:", s,
                    p.ids.size(), hipGetErrorName(hipEventQuery(c->ev_copied[s])),
                    hipGetErrorName(hipStreamQuery(c->copy_stream)), hipGetErrorName(hipStreamQuery(c->stream)));
            for (size_t j = 0; j < std::min<size_t>(p.ids.size(), 16); ++j)
                fprintf(stderr, " %llu@%llu", (unsigned long long)c->h_desc[s][M + j], (unsigned long long)c->h_desc[s][j]);
            fprintf(stderr, "\n");
            return fail(OXH_ERR_HIP, "timed out waiting for a staged batch (see stderr)");
        }
    }
}

// Scatter slot s's digests to the caller's table (host-buffer batches: oxh_hash_buffers/_streams).
int drain_slot(oxh_ctx* c, int s, Pending& p, uint64_t* out) {
    if (!p.busy) return OXH_OK;
    STEP("drain s=%d", s);
    if (int rc = wait_slot(c, s, p)) return rc;
    for (size_t j = 0; j < p.ids.size(); ++j) {
        out[2 * p.ids[j]] = c->h_out[s][2 * j];
        out[2 * p.ids[j] + 1] = c->h_out[s][2 * j + 1];
    }
    p.busy = false;
    p.ids.clear();
    return OXH_OK;
}

// Digest (+ text counts, + is_utf8) of one buffer already on the device (stream-ordered on
// c->stream): d holds align_up(len) + 256 bytes, the tail is the results area. Synchronises c->stream.
int device_item(oxh_ctx* c, uint8_t* d, uint64_t len, uint64_t* out2, uint64_t* cnt2, int32_t* utf8_1) {
    const uint64_t tail = align_up(len);
    struct Res {  // mirrored at d + tail: digest, text counts, a one-item descriptor, is_utf8
        uint64_t out[2], cnt[2], off, len;
        int32_t utf8, pad;
    } h{};
    h.len = len;
    uint64_t* d_res = reinterpret_cast<uint64_t*>(d + tail);
    int rc = OXH_OK;
    auto ok = [&](hipError_t e, const char* what) {
        if (rc == OXH_OK && e != hipSuccess) rc = fail(OXH_ERR_HIP, what);
        return rc == OXH_OK;
    };
    ok(hipMemcpyAsync(d_res, &h, sizeof h, hipMemcpyHostToDevice, c->stream), "results area H2D failed");
    if (rc == OXH_OK) rc = large_device(c, d, len, d_res, c->stream);
    if (rc == OXH_OK && cnt2) {
        hipLaunchKernelGGL(oxh::text_count_kernel, dim3(2048), dim3(256), 0, c->stream, d, len,
                           (unsigned long long*)(d_res + 2));
        ok(hipGetLastError(), "text_count_kernel launch");
    }
    if (rc == OXH_OK && utf8_1) {
        hipLaunchKernelGGL(oxh::utf8_prefix_kernel, dim3(1), dim3(64), 0, c->stream, d, d_res + 4, d_res + 5, (uint64_t)1,
                           (int32_t*)(d_res + 6));
        ok(hipGetLastError(), "utf8_prefix_kernel launch");
    }
    ok(hipMemcpyAsync(&h, d_res, sizeof h, hipMemcpyDeviceToHost, c->stream), "results D2H failed");
    ok(hipStreamSynchronize(c->stream), "sync failed");
    if (rc == OXH_OK) {
        out2[0] = h.out[0];
        out2[1] = h.out[1];
        if (cnt2) {
            cnt2[0] = 1 + h.cnt[0];
            cnt2[1] = len - h.cnt[1];
        }
        if (utf8_1) *utf8_1 = h.utf8;
    }
    return rc;
}

// Hash one oversize host item (> a staging slot) through a device buffer of its own (the staging
// slots may belong to a live pipeline); with `cnt2`, also its text counts (num_lines, num_chars),
// with `utf8_1` its is_utf8 sniff.
int oversize_item(oxh_ctx* c, const uint8_t* src, uint64_t len, uint64_t* out2, uint64_t* cnt2 = nullptr,
                  int32_t* utf8_1 = nullptr) {
    uint8_t* d = nullptr;
    if (hipMalloc(&d, align_up(len) + 256) != hipSuccess) {
        (void)hipGetLastError();
        return fail(OXH_ERR_NOMEM, "oversize hipMalloc failed");
    }
    int rc = OXH_OK;
    if (hipMemcpyAsync(d, src, len, hipMemcpyHostToDevice, c->stream) != hipSuccess) rc = fail(OXH_ERR_HIP, "oversize H2D failed");
    if (rc == OXH_OK) rc = device_item(c, d, len, out2, cnt2, utf8_1);
    (void)hipFree(d);
    return rc;
}

// Items larger than a staging slot (K1L). A file larger than a slot takes the reference's streaming
// branch (hasher.rs:150-174); a host buffer that large (oxh_hash_buffers / _streams) the same path.
// The item is hashed in device pieces of OXH_BIG_PIECE_MIB (default 1 GiB) through two piece
// buffers, so device memory stays bounded whatever the item size and piece j+1's transfer overlaps
// piece j's K1L chain: each piece's block sums are computed chip-wide and the serial chain continues
// from the previous piece's accumulators (ChainJob kChainResume / kChainPartial); the last piece
// (> 1 KiB) takes the tail and the merge. A file piece reaches the device copy-free when its pages
// are in the page cache (mincore) and can be pinned (mmap + hipHostRegister read-only, ~2 ms per GiB;
// the DMA engine then reads them at 46-57 GB/s, tools/mmap_register_probe.hip); otherwise pieces pass
// through two pinned 64 MiB bounce buffers filled by the worker pool (parallel 4 MiB reads). Text
// counts accumulate over the pieces; is_utf8 reads the first 4 KiB of piece 0. With a sink (fused
// add) every bounce part is also written to the sink's temp as it is read, and the temp is published
// once the digest is known: the item never has to fit in host memory.
// Stall reports (dump_engine): the live contexts, and where context creation / destruction and the
// streaming Xxh3 last were -- the threads that call those are not engine threads.
std::mutex g_live_mu;
std::vector<oxh_ctx*> g_live;
std::atomic<const char*> g_life{"-"}, g_stream_where{"-"};

constexpr uint64_t kBounce = 64ull << 20, kBigRead = 4ull << 20;
constexpr int kNBounce = 8;  // bounce buffers in the ring: up to 7 windows read while earlier H2Ds drain

// Bounce windows a large item reads at once (OXH_BIG_WINDOWS, 1 .. kNBounce - 1; 1 is the r03-r04 form)
int big_windows() {
    static const int v = [] {
        const char* e = getenv("OXH_BIG_WINDOWS");
        const int k = e ? atoi(e) : kNBounce - 1;
        return std::max(1, std::min(k, kNBounce - 1));
    }();
    return v;
}

// H2D copy streams a large item's bounce windows alternate over (OXH_BIG_COPY_STREAMS, 1 or 2; default 2)
int big_copy_streams() {
    static const int v = [] {
        const char* e = getenv("OXH_BIG_COPY_STREAMS");
        return e && atoi(e) == 1 ? 1 : 2;
    }();
    return v;
}

// Where a large item's bytes come from.
struct LargeSource {
    virtual ~LargeSource() = default;
    // Pin [off, off + n) in place for an asynchronous H2D copy (no bounce buffer) if this source can:
    // the host pointer to copy from, or nullptr. unpin() once the copy has completed.
    virtual const uint8_t* pin(uint64_t, uint64_t) { return nullptr; }
    virtual void unpin(const uint8_t*) {}
    // [off, off + n) will be read soon.
    virtual void will_need(uint64_t, uint64_t) {}
    // Read [off, off + n) into dst; called from several threads for disjoint ranges. false = I/O error
    // (os_error then holds the errno of the failed read, 0 for a file that ended early).
    virtual bool read(uint64_t off, uint64_t n, uint8_t* dst) = 0;
    std::atomic<int> os_error{0};
};

// A regular file: preads, or mmap pages pinned in place for the copy-free path.
struct FileSource final : LargeSource {
    int fd = -1;
    uint8_t* map = nullptr;
    uint64_t len = 0;
    std::vector<unsigned char> resident;
    FileSource(const char* path, uint64_t L, bool allow_direct)
        : FileSource(path ? open(path, O_RDONLY | O_CLOEXEC | O_NONBLOCK) : -1, L, allow_direct) {}
    // an open descriptor (owned from here on) whose file holds L bytes
    FileSource(int fd_, uint64_t L, bool allow_direct) : fd(fd_), len(L) {
        if (fd >= 0 && allow_direct) {
            void* m = mmap(nullptr, L, PROT_READ, MAP_SHARED, fd, 0);
            if (m != MAP_FAILED) {
                map = (uint8_t*)m;
                (void)madvise(m, L, MADV_SEQUENTIAL);
            }
        }
    }
    ~FileSource() override {
        if (map) munmap(map, len);
        if (fd >= 0) close(fd);
    }
    // pinning faults missing pages in one thread, so a piece that is mostly on disk is read by the
    // parallel preads instead
    bool mostly_resident(uint64_t off, uint64_t n) {
        const uint64_t pg = (uint64_t)sysconf(_SC_PAGESIZE), npg = (n + pg - 1) / pg;
        resident.resize(npg);
        if (mincore(map + off, n, resident.data()) != 0) return false;
        uint64_t in = 0;
        for (unsigned char v : resident) in += v & 1;
        return in * 10 >= npg * 9;
    }
    const uint8_t* pin(uint64_t off, uint64_t n) override {
        if (!map || !mostly_resident(off, n) || hipHostRegister(map + off, n, hipHostRegisterReadOnly) != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
        return map + off;
    }
    void unpin(const uint8_t* p) override {
        (void)hipHostUnregister((void*)p);
        (void)hipGetLastError();
    }
    void will_need(uint64_t off, uint64_t n) override { (void)posix_fadvise(fd, (off_t)off, (off_t)n, POSIX_FADV_WILLNEED); }
    bool read(uint64_t off, uint64_t n, uint8_t* dst) override {
        for (uint64_t got = 0; got < n;) {
            const ssize_t x = pread(fd, dst + got, n - got, (off_t)(off + got));
            if (x < 0) os_error.store(errno);
            if (x <= 0) return false;
            got += (uint64_t)x;
        }
        return true;
    }
};

// A caller's host buffer (pageable): copied into the pinned bounce buffers by the pool.
struct MemSource final : LargeSource {
    const uint8_t* p;
    explicit MemSource(const uint8_t* q) : p(q) {}
    bool read(uint64_t off, uint64_t n, uint8_t* dst) override {
        memcpy(dst, p + off, n);
        return true;
    }
};

struct LargeResult {
    uint64_t out[2] = {0, 0}, cnt[2] = {0, 0};  // digest; text counts (num_lines, num_chars)
    int32_t utf8 = 0;
    int status = OXH_OK;  // this item's status: OXH_OK, OXH_ERR_IO or OXH_ERR_NOMEM
    int os_error = 0;     // errno of a failed read (OXH_ERR_IO)
};

// One large item of a large_items() batch: its source and what the caller wants, then the outcome.
struct LargeJob {
    uint64_t L = 0;
    LargeSource* src = nullptr;
    bool want_counts = false, want_utf8 = false;
    ItemSink* sink = nullptr;
    uint64_t id = 0;
    LargeResult res;
};

// Files up to this many at a time share one large-item pipeline (OXH_BIG_FILES overrides; device
// memory: 2 piece buffers of OXH_BIG_PIECE_MIB + 1 KiB per file).
int big_files_at_once() {
    const char* e = getenv("OXH_BIG_FILES");
    const int v = e && atoi(e) > 0 ? atoi(e) : 4;
    return std::min(v, (int)oxh::kChainJobs);
}

// Hash n (<= kChainJobs) large items side by side (see above). Round r moves piece r of every item
// that has one to the device (the copies are PCIe-bound and serial on the copy stream), launches its
// block sums chip-wide, and then ONE chain launch continues every item's serial chain over its piece
// (the chains are latency-bound: 16 files' chains cost about what one does). The chains of round r
// run on the device while the host moves round r+1's pieces, so the chain time hides behind the
// copies of the next round instead of adding up file after file. Returns a run-level error code only
// for HIP failures; each item's own outcome (I/O error, allocation failure) is its res.status.
int large_items(oxh_ctx* c, LargeJob* jobs, int n) {
    if (n <= 0) return OXH_OK;
    if (n > (int)oxh::kChainJobs) return fail(OXH_ERR_INVALID, "too many large items in one batch");
    const uint64_t P = std::max<uint64_t>(
        1, getenv("OXH_BIG_PIECE_MIB") ? strtoull(getenv("OXH_BIG_PIECE_MIB"), nullptr, 10) : 1024) << 20;
    const uint64_t cap = P + 1024;  // bytes per piece buffer
    const uint64_t slot = align_up(cap) + 256;
    constexpr uint64_t kRes = 256;  // per item: [digest 2 | counts 2 | desc off, len | utf8 | state 8]
    // an allocation that fails is these items' failure (OXH_ERR_NOMEM), not the engine run's: the
    // other requests in the live pipeline carry on
    auto nomem = [&]() {
        (void)hipGetLastError();
        for (int q = 0; q < n; ++q) jobs[q].res.status = OXH_ERR_NOMEM;
        return OXH_OK;
    };
    auto bytes_for = [&](int items) { return (uint64_t)items * (2 * slot + kRes) + 4096; };
    const uint64_t need = bytes_for(n);
    c->where.store("large_items: d_big");
    if (c->d_big_size < need) {
        // Regrow: every earlier large_items call on this context finished its work on d_big before it
        // returned (its streams are synchronised at the end), so the old buffer is idle. Plain
        // hipFree / hipMalloc: the stream-ordered allocator (hipMallocAsync / hipFreeAsync on
        // c->stream, r04) was AVOIDED after a stall under concurrent contexts (threads parked in
        // hipMallocAsync beside others in hipEventRecord / hipHostMalloc, every stream idle;
        // tools/engine_soak.py --regrow, profiles/r05/r05s6_*) -- not proven faulty, no reduced
        // reproducer. hipFree synchronises the whole device, so a regrow waits on every other
        // context's work: the buffer is sized for the most items the engine batches
        // (big_files_at_once(), or n if more) at once, so a context pays this once per piece size,
        // not once per new n (oxh_ctx_counters counts it; DESIGN §5 "Soak").
        if (c->d_big) {
            (void)hipFree(c->d_big);
            c->d_big = nullptr;
            c->d_big_size = 0;
        }
        void* m = nullptr;
        uint64_t size = std::max(need, bytes_for(big_files_at_once()));
        bool ok = hipMalloc(&m, size) == hipSuccess && m != nullptr;
        if (!ok && size > need) {  // the full batch does not fit: just these n items
            (void)hipGetLastError();
            size = need;
            ok = hipMalloc(&m, size) == hipSuccess && m != nullptr;
        }
        if (ok) ++c->d_big_allocs;
        if (!ok) {
            (void)hipGetLastError();
            // 2 piece buffers per file side by side did not fit: fewer files at a time (each item's
            // result does not depend on its batch), down to one before the items fail with NOMEM
            if (n > 1) {
                const int h = n / 2;
                if (int rc = large_items(c, jobs, h)) return rc;
                return large_items(c, jobs + h, n - h);
            }
            return nomem();
        }
        c->d_big = (uint8_t*)m;
        c->d_big_size = size;
    }
    auto dbuf = [&](int q, int b) { return c->d_big + ((uint64_t)q * 2 + b) * slot; };
    uint8_t* d_res_all = c->d_big + (uint64_t)n * 2 * slot;
    auto d_res = [&](int q) { return reinterpret_cast<uint64_t*>(d_res_all + (uint64_t)q * kRes); };
    struct Res {
        uint64_t out[2], cnt[2], off, len;
        int32_t utf8, pad;
    };
    static_assert(sizeof(Res) + 64 <= kRes, "results area");
    std::vector<uint8_t> h_res((size_t)n * kRes, 0);
    for (int q = 0; q < n; ++q) reinterpret_cast<Res*>(h_res.data() + (size_t)q * kRes)->len = jobs[q].L;
    c->where.store("large_items: bounce alloc");
    for (int b = 0; b < kNBounce; ++b) {
        if (!c->h_bounce[b] && hipHostMalloc(&c->h_bounce[b], kBounce, hipHostMallocDefault) != hipSuccess) {
            c->h_bounce[b] = nullptr;
            return nomem();
        }
        if (!c->ev_bounce[b]) HIP_TRY(hipEventCreateWithFlags(&c->ev_bounce[b], hipEventDisableTiming));
    }
    for (int b = 0; b < 2; ++b)
        if (!c->ev_piece_free[b]) HIP_TRY(hipEventCreateWithFlags(&c->ev_piece_free[b], hipEventDisableTiming));
    c->where.store("large_items: events / copy_stream2");
    if (!c->copy_stream2) HIP_TRY(hipStreamCreateWithFlags(&c->copy_stream2, hipStreamNonBlocking));
    if (!c->ev_copy2_join) HIP_TRY(hipEventCreateWithFlags(&c->ev_copy2_join, hipEventDisableTiming));
    uint64_t* sums = nullptr;
    c->where.store("large_items: scratch lease");
    oxh::ScratchLease lease(c->stream);  // block sums of the two rounds in flight
    c->where.store("large_items: scratch get");
    const uint64_t sums_per = (cap >> 10) * 8;
    if (lease.get(2 * sums_per * 8 * (uint64_t)n, (void**)&sums) != hipSuccess) return nomem();
    HIP_TRY(hipMemcpyAsync(d_res_all, h_res.data(), h_res.size(), hipMemcpyHostToDevice, c->stream));

    // one copy-done event per item (created before any sink temp exists: a failure here leaves nothing behind)
    std::vector<hipEvent_t> ev_copy(n, nullptr);
    for (int q = 0; q < n; ++q)
        if (hipEventCreateWithFlags(&ev_copy[q], hipEventDisableTiming) != hipSuccess) {
            (void)hipGetLastError();
            for (hipEvent_t e : ev_copy)
                if (e) (void)hipEventDestroy(e);
            return fail(OXH_ERR_HIP, "large-item events");
        }
    struct State {
        uint64_t k = 0;  // pieces 0 .. k-1 hold P bytes each; the last one L - k*P bytes, in [1025, P + 1024]
        std::string sink_tmp;
        int sfd = -1;
        std::atomic<bool> sink_ok{true};
        bool io_ok = true;
    };
    std::vector<State> st(n);
    uint64_t rounds = 0;
    for (int q = 0; q < n; ++q) {
        const uint64_t L = jobs[q].L;
        st[q].k = L > P + 1024 ? (L - 1025) / P : 0;
        rounds = std::max(rounds, st[q].k + 1);
        if (jobs[q].sink) {
            st[q].sfd = jobs[q].sink->open_stream(jobs[q].id, st[q].sink_tmp);
            if (st[q].sfd < 0) st[q].sink_ok.store(false);
        }
    }
    int rc = OXH_OK;
    // piece [off, off + plen) of item q -> device buffer d on the copy stream; false on an I/O error.
    // The piece goes through the bounce ring in windows of kBounce: up to kNBounce - 1 windows are read
    // at once (their 4 MiB parts queued on the pool without a barrier between windows), and a window's
    // H2D is issued as soon as its own parts are done (r05; r03-r04 read one window at a time).
    struct Window {
        int bb = 0;
        uint64_t o = 0, m = 0;
        std::atomic<bool> bad{false};
        std::function<void(int)> fn;
        oxh::Pool::Group grp;
    };
    auto copy_piece = [&](int q, uint64_t off, uint64_t plen, uint8_t* d) -> bool {
        LargeSource& src = *jobs[q].src;
        State& S = st[q];
        std::vector<std::unique_ptr<Window>> wins;
        std::deque<Window*> inflight;
        bool ok = true;
        auto finish = [&](Window& W) {
            c->where.store("copy_piece: window reads");
            W.grp.wait();
            c->where.store("copy_piece: window H2D");
            if (W.bad.load()) ok = false;
            if (!ok) return;
            // windows alternate over two copy streams: two DMA queues keep the PCIe link busier (the
            // FastCDC host pipeline measured 53.5 vs 47 GB/s)
            hipStream_t cs = (big_copy_streams() == 2 && ((W.o / kBounce) & 1)) ? c->copy_stream2 : c->copy_stream;
            if (hipMemcpyAsync(d + W.o, c->h_bounce[W.bb], W.m, hipMemcpyHostToDevice, cs) != hipSuccess ||
                hipEventRecord(c->ev_bounce[W.bb], cs) != hipSuccess) {
                ok = false;
                return;
            }
            c->bounce_used[W.bb] = true;
        };
        for (uint64_t o = 0; o < plen && ok; o += kBounce) {
            wins.emplace_back(new Window);
            Window& W = *wins.back();
            W.bb = (int)(c->bounce_next++ % kNBounce);
            W.o = o;
            W.m = std::min(kBounce, plen - o);
            c->where.store("copy_piece: bounce event");
            if (c->bounce_used[W.bb] && hipEventSynchronize(c->ev_bounce[W.bb]) != hipSuccess) {
                ok = false;
                break;
            }
            c->where.store("copy_piece: start window");
            c->bounce_used[W.bb] = false;
            src.will_need(off + o + W.m, 2 * kBounce);  // two windows ahead of the ones being read
            uint8_t* buf = c->h_bounce[W.bb];
            const uint64_t base = off + o, m = W.m;
            W.fn = [&src, &S, &W, buf, base, m](int t) {
                const uint64_t lo = (uint64_t)t * kBigRead, hi = std::min(m, lo + kBigRead);
                if (!src.read(base + lo, hi - lo, buf + lo)) {
                    W.bad.store(true);
                    return;
                }
                if (S.sfd >= 0 && S.sink_ok.load(std::memory_order_relaxed))  // the same bytes to the temp blob
                    for (uint64_t put = lo; put < hi;) {
                        const ssize_t x = pwrite(S.sfd, buf + put, hi - put, (off_t)(base + put));
                        if (x <= 0) {
                            S.sink_ok.store(false);
                            break;
                        }
                        put += (uint64_t)x;
                    }
            };
            c->pool->start((int)((m + kBigRead - 1) / kBigRead), W.fn, W.grp);
            inflight.push_back(&W);
            if ((int)inflight.size() >= big_windows()) {
                finish(*inflight.front());
                inflight.pop_front();
            }
        }
        while (!inflight.empty()) {  // every started window is waited for, also after a failure
            finish(*inflight.front());
            inflight.pop_front();
        }
        // the piece's event is recorded on copy_stream: it waits for copy_stream2's windows first
        if (ok && (hipEventRecord(c->ev_copy2_join, c->copy_stream2) != hipSuccess ||
                   hipStreamWaitEvent(c->copy_stream, c->ev_copy2_join, 0) != hipSuccess))
            ok = false;
        // no wait for the copies here: the piece's kernels wait for the copy stream through ev_copy,
        // and a bounce buffer is refilled only after its own H2D (ev_bounce), so the next piece's reads
        // overlap this piece's last copies
        return ok;
    };
    // With OXH_BIG_DIRECT=1, pieces whose pages are in the page cache are pinned in place and copied
    // asynchronously; the next round's pieces are pinned while this round's copies run, and a round's
    // pins are released once its copies are done.
    std::vector<const uint8_t*> pinned(n, nullptr), next_pin(n, nullptr);
    std::vector<std::pair<int, const uint8_t*>> to_unpin;  // (item, pinned range) of copies in flight
    auto piece_len = [&](int q, uint64_t r) { return r < st[q].k ? P : jobs[q].L - r * P; };
    // Pinning page-cache pages in place (OXH_BIG_DIRECT=1) measured 10-27 ms per GiB to register and
    // ~10 ms per GiB to release on the MI355X boxes (r03, OXH_TRACE), more than the 16 pool threads take
    // to copy the same bytes into the pinned bounce buffers; the bounce path is the default.
    const bool may_pin = getenv("OXH_BIG_DIRECT") && atoi(getenv("OXH_BIG_DIRECT")) != 0;
    auto pin_round = [&](uint64_t r, std::vector<const uint8_t*>& into) {
        if (!may_pin) return;
        for (int q = 0; q < n; ++q) {
            if (into[q]) jobs[q].src->unpin(into[q]);
            into[q] = (!jobs[q].sink && st[q].io_ok && r <= st[q].k) ? jobs[q].src->pin(r * P, piece_len(q, r)) : nullptr;
        }
    };
    Trace tr;  // OXH_TRACE=1: where a batch's host time goes
    double t_pin = 0, t_wait = 0, t_unpin = 0, t_bounce = 0;
    const double t_start = Trace::now();
    {
        const double t0 = Trace::now();
        pin_round(0, next_pin);
        t_pin += Trace::now() - t0;
    }
    bool round_used[2] = {false, false};
    for (uint64_t r = 0; r < rounds && rc == OXH_OK; ++r) {
        const int b = (int)(r & 1);
        pinned.swap(next_pin);
        // the chains of round r-2 (which read buffers b and their block sums) are done
        c->where.store("large_items: piece free");
        if (round_used[b] && hipEventSynchronize(c->ev_piece_free[b]) != hipSuccess) {
            rc = fail(OXH_ERR_HIP, "large-item piece wait");
            break;
        }
        oxh::ChainBatch batch;
        int nj = 0;
        for (int q = 0; q < n; ++q) {
            State& S = st[q];
            if (!S.io_ok || r > S.k) {
                if (pinned[q]) jobs[q].src->unpin(pinned[q]);  // pinned ahead, before the item failed
                pinned[q] = nullptr;
                continue;
            }
            const uint64_t off = r * P, plen = piece_len(q, r);
            uint8_t* d = dbuf(q, b);
            if (pinned[q]) {  // copy-free: the DMA engine reads the page cache (a sink must see host bytes)
                if (hipMemcpyAsync(d, pinned[q], plen, hipMemcpyHostToDevice, c->copy_stream) != hipSuccess ||
                    hipEventRecord(ev_copy[q], c->copy_stream) != hipSuccess) {
                    rc = fail(OXH_ERR_HIP, "large-item piece copy");
                    break;
                }
                to_unpin.push_back({q, pinned[q]});
                pinned[q] = nullptr;
            } else {
                const double t0 = Trace::now();
                const bool copied = copy_piece(q, off, plen, d);
                t_bounce += Trace::now() - t0;
                if (!copied) {
                    S.io_ok = false;  // its earlier chains finish harmlessly; the item is reported as unreadable
                    continue;
                }
                if (hipEventRecord(ev_copy[q], c->copy_stream) != hipSuccess) {
                    rc = fail(OXH_ERR_HIP, "large-item piece event");
                    break;
                }
            }
            if (hipStreamWaitEvent(c->stream, ev_copy[q], 0) != hipSuccess) {
                rc = fail(OXH_ERR_HIP, "large-item piece wait");
                break;
            }
            uint64_t* s_q = sums + ((uint64_t)b * n + q) * sums_per;
            const bool last = r == S.k;
            const uint64_t nb = last ? (plen - 1) >> 10 : plen >> 10;
            const uint64_t nwaves = (nb + 3) / 4, blocks = (nwaves + 3) / 4;
            hipLaunchKernelGGL(oxh::xxh3_blocksum_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, c->stream, d, nb, s_q);
            if (jobs[q].want_counts)
                hipLaunchKernelGGL(oxh::text_count_kernel, dim3(2048), dim3(256), 0, c->stream, d, plen,
                                   (unsigned long long*)(d_res(q) + 2));
            if (r == 0 && jobs[q].want_utf8)
                hipLaunchKernelGGL(oxh::utf8_prefix_kernel, dim3(1), dim3(64), 0, c->stream, d, d_res(q) + 4, d_res(q) + 5,
                                   (uint64_t)1, (int32_t*)(d_res(q) + 6));
            batch.job[nj++] = {d, plen, s_q, d_res(q), jobs[q].L, d_res(q) + 7,
                               (r > 0 ? oxh::kChainResume : 0u) | (last ? 0u : oxh::kChainPartial)};
        }
        if (rc) break;
        if (nj) hipLaunchKernelGGL(oxh::xxh3_chain_kernel, dim3(nj), dim3(64), kChainLdsPad, c->stream, batch);
        if (hipGetLastError() != hipSuccess || hipEventRecord(c->ev_piece_free[b], c->stream) != hipSuccess)
            rc = fail(OXH_ERR_HIP, "large-item piece launch");
        round_used[b] = true;
        double t0 = Trace::now();
        if (r + 1 < rounds) pin_round(r + 1, next_pin);  // while this round's copies run
        t_pin += Trace::now() - t0;
        if (!to_unpin.empty()) {
            t0 = Trace::now();
            if (hipStreamSynchronize(c->copy_stream) != hipSuccess && rc == OXH_OK) rc = fail(OXH_ERR_HIP, "large-item copy");
            t_wait += Trace::now() - t0;
            t0 = Trace::now();
            for (const auto& u : to_unpin) jobs[u.first].src->unpin(u.second);
            t_unpin += Trace::now() - t0;
            to_unpin.clear();
        }
    }
    // a failure mid-way: release what is still pinned
    c->where.store("large_items: final copy sync");
    if (hipStreamSynchronize(c->copy_stream) != hipSuccess && rc == OXH_OK) rc = fail(OXH_ERR_HIP, "large-item copy");
    if (hipStreamSynchronize(c->copy_stream2) != hipSuccess && rc == OXH_OK) rc = fail(OXH_ERR_HIP, "large-item copy");
    for (int q = 0; q < n; ++q) {
        if (pinned[q]) jobs[q].src->unpin(pinned[q]);
        if (next_pin[q]) jobs[q].src->unpin(next_pin[q]);
    }
    for (const auto& u : to_unpin) jobs[u.first].src->unpin(u.second);
    if (rc == OXH_OK && hipMemcpyAsync(h_res.data(), d_res_all, h_res.size(), hipMemcpyDeviceToHost, c->stream) != hipSuccess)
        rc = fail(OXH_ERR_HIP, "large-item results D2H");
    const double t_tail0 = Trace::now();
    c->where.store("large_items: results sync");
    if (hipStreamSynchronize(c->stream) != hipSuccess && rc == OXH_OK) rc = fail(OXH_ERR_HIP, "large-item sync");
    c->where.store("large_items: publish");
    if (tr.on)
        fprintf(stderr, "[oxh] large_items n=%d rounds=%llu piece=%llu MiB: total %.1f ms, pin %.1f, copy wait %.1f, unpin %.1f, "
                "bounce %.1f, chain tail %.1f\n", n, (unsigned long long)rounds, (unsigned long long)(P >> 20),
                1e3 * (Trace::now() - t_start), 1e3 * t_pin, 1e3 * t_wait, 1e3 * t_unpin, 1e3 * t_bounce,
                1e3 * (Trace::now() - t_tail0));
    std::vector<ItemSink*> sinks;
    for (int q = 0; q < n; ++q) {
        const Res& h = *reinterpret_cast<const Res*>(h_res.data() + (size_t)q * kRes);
        if (jobs[q].sink) {  // publish (or drop) the temp blob now that the digest is known
            jobs[q].sink->close_stream(jobs[q].id, st[q].sfd, st[q].sink_tmp,
                                       rc == OXH_OK && st[q].io_ok && st[q].sink_ok.load(), h.out[0], h.out[1]);
            if (std::find(sinks.begin(), sinks.end(), jobs[q].sink) == sinks.end()) sinks.push_back(jobs[q].sink);
        }
        LargeResult& res = jobs[q].res;
        if (rc) continue;
        if (!st[q].io_ok) {
            res.status = OXH_ERR_IO;
            res.os_error = jobs[q].src->os_error.load();
            continue;
        }
        res.out[0] = h.out[0];
        res.out[1] = h.out[1];
        res.cnt[0] = 1 + h.cnt[0];
        res.cnt[1] = jobs[q].L - h.cnt[1];
        res.utf8 = h.utf8;
    }
    for (ItemSink* k : sinks) k->commit();
    for (hipEvent_t e : ev_copy) (void)hipEventDestroy(e);
    return rc;
}

// One large item (host buffers of oxh_hash_buffers / _streams, and the single-file case).
int large_item(oxh_ctx* c, uint64_t L, LargeSource& src, bool want_counts, bool want_utf8, ItemSink* sink, uint64_t id,
               LargeResult& res) {
    LargeJob j;
    j.L = L, j.src = &src, j.want_counts = want_counts, j.want_utf8 = want_utf8, j.sink = sink, j.id = id;
    const int rc = large_items(c, &j, 1);
    res = j.res;
    return rc;
}

}  // namespace

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

int oxh_ctx_counters(oxh_ctx* c, uint64_t* out, int n) {
    if (!c || (n > 0 && !out)) return fail(OXH_ERR_INVALID, "null argument");
    const uint64_t v[2] = {c->d_big_allocs, c->d_big_size};
    for (int i = 0; i < n; ++i) out[i] = i < 2 ? v[i] : 0;
    return OXH_OK;
}
const char* oxh_last_error(void) { return g_err.c_str(); }

int oxh_device_count(int* count) {
    if (!count) return fail(OXH_ERR_INVALID, "count is NULL");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return OXH_OK;
}

int oxh_set_kernel_variant(int variant) { return g_variant.exchange(variant); }

int oxh_ctx_create(int device, uint64_t staging_bytes, oxh_ctx** out) {
    if (!out) return fail(OXH_ERR_INVALID, "out is NULL");
    *out = nullptr;
    // a slot's reservation word packs the byte offset into 31 bits and the item count into 19
    // (stream_files below): both must hold a full slot
    if (staging_bytes > OXH_MAX_STAGING_BYTES)
        return fail(OXH_ERR_INVALID, "staging_bytes exceeds OXH_MAX_STAGING_BYTES (2 GiB - 256)");
    int rc = check_device(device);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(device));
    oxh_ctx* c = new oxh_ctx();
    c->device = device;
    {
        std::lock_guard<std::mutex> g(g_live_mu);
        g_live.push_back(c);
    }
    g_life.store("create: streams");
    c->stage_bytes = align_up(staging_bytes ? staging_bytes : (256ull << 20));
    c->max_items = std::max<uint64_t>(1024, c->stage_bytes / 4096);
    auto cleanup = [&](int code, const char* m) { oxh_ctx_destroy(c); return fail(code, m); };
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) return cleanup(OXH_ERR_HIP, "stream");
    if (hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking) != hipSuccess) return cleanup(OXH_ERR_HIP, "copy stream");
    g_life.store("create: slot buffers");
    for (int s = 0; s < NSLOT; ++s) {
        if (hipHostMalloc(&c->h_stage[s], c->stage_bytes, hipHostMallocDefault) != hipSuccess) return cleanup(OXH_ERR_NOMEM, "pinned staging");
        if (hipMalloc(&c->d_stage[s], c->stage_bytes) != hipSuccess) return cleanup(OXH_ERR_NOMEM, "device staging");
        if (hipHostMalloc(&c->h_desc[s], c->max_items * 16, hipHostMallocDefault) != hipSuccess) return cleanup(OXH_ERR_NOMEM, "pinned desc");
        if (hipMalloc(&c->d_desc[s], c->max_items * 16) != hipSuccess) return cleanup(OXH_ERR_NOMEM, "device desc");
        if (hipHostMalloc(&c->h_out[s], c->max_items * 16, hipHostMallocDefault) != hipSuccess) return cleanup(OXH_ERR_NOMEM, "pinned out");
        if (hipMalloc(&c->d_out[s], c->max_items * 16) != hipSuccess) return cleanup(OXH_ERR_NOMEM, "device out");
        if (hipHostMalloc(&c->h_cnt[s], c->max_items * 16, hipHostMallocDefault) != hipSuccess) return cleanup(OXH_ERR_NOMEM, "pinned counts");
        if (hipMalloc(&c->d_cnt[s], c->max_items * 16) != hipSuccess) return cleanup(OXH_ERR_NOMEM, "device counts");
        if (hipHostMalloc(&c->h_utf8[s], c->max_items * 4, hipHostMallocDefault) != hipSuccess) return cleanup(OXH_ERR_NOMEM, "pinned utf8");
        if (hipMalloc(&c->d_utf8[s], c->max_items * 4) != hipSuccess) return cleanup(OXH_ERR_NOMEM, "device utf8");
        if (hipEventCreateWithFlags(&c->ev_copied[s], hipEventDisableTiming) != hipSuccess) return cleanup(OXH_ERR_HIP, "event");
        if (hipEventCreateWithFlags(&c->ev_done[s], hipEventDisableTiming) != hipSuccess) return cleanup(OXH_ERR_HIP, "event");
    }
    for (int s = 0; s < NSLOT; ++s) {
        c->rq[s].resize(c->max_items);
        c->loc[s].resize(c->max_items);
    }
    const char* fl = getenv("OXH_FLUSH_MIB");
    c->flush_bytes = std::min<uint64_t>(c->stage_bytes, (fl ? (uint64_t)atoll(fl) : 16ull) << 20);
    c->pool = new oxh::Pool(default_threads());
    c->rpool = new oxh::Pool(default_threads(), /*private_fds=*/true);  // readers use only their own fds
    c->engine = std::thread(engine_main, c);
    g_life.store("create: done");
    *out = c;
    return OXH_OK;
}

int oxh_ctx_destroy(oxh_ctx* c) {
    if (!c) return OXH_OK;
    {
        std::lock_guard<std::mutex> g(g_live_mu);
        g_live.erase(std::remove(g_live.begin(), g_live.end(), c), g_live.end());
    }
    g_life.store("destroy: engine join");
    if (c->engine.joinable()) {  // finishes what is queued, then exits
        {
            std::lock_guard<std::mutex> g(c->qmu);
            c->stop = true;
        }
        c->qcv.notify_all();
        c->engine.join();
    }
    (void)hipSetDevice(c->device);
    g_life.store("destroy: buffers");
    if (c->cdc && c->cdc_free) c->cdc_free(c->cdc);
    c->cdc = nullptr;
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->copy_stream) (void)hipStreamSynchronize(c->copy_stream);
    for (int s = 0; s < NSLOT; ++s) {
        if (c->h_stage[s]) (void)hipHostFree(c->h_stage[s]);
        if (c->d_stage[s]) (void)hipFree(c->d_stage[s]);
        if (c->h_desc[s]) (void)hipHostFree(c->h_desc[s]);
        if (c->d_desc[s]) (void)hipFree(c->d_desc[s]);
        if (c->h_out[s]) (void)hipHostFree(c->h_out[s]);
        if (c->d_out[s]) (void)hipFree(c->d_out[s]);
        if (c->h_cnt[s]) (void)hipHostFree(c->h_cnt[s]);
        if (c->d_cnt[s]) (void)hipFree(c->d_cnt[s]);
        if (c->h_utf8[s]) (void)hipHostFree(c->h_utf8[s]);
        if (c->d_utf8[s]) (void)hipFree(c->d_utf8[s]);
        if (c->ev_copied[s]) (void)hipEventDestroy(c->ev_copied[s]);
        if (c->ev_done[s]) (void)hipEventDestroy(c->ev_done[s]);
    }
    g_life.store("destroy: d_big");
    if (c->d_big) {  // large_items' piece buffers
        (void)hipStreamSynchronize(c->stream);
        (void)hipFree(c->d_big);
    }
    g_life.store("destroy: bounce / streams");
    for (int b = 0; b < kNBounce; ++b) {
        if (c->h_bounce[b]) (void)hipHostFree(c->h_bounce[b]);
        if (c->ev_bounce[b]) (void)hipEventDestroy(c->ev_bounce[b]);
    }
    for (int b = 0; b < 2; ++b)
        if (c->ev_piece_free[b]) (void)hipEventDestroy(c->ev_piece_free[b]);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
    if (c->copy_stream2) {
        (void)hipStreamSynchronize(c->copy_stream2);
        (void)hipStreamDestroy(c->copy_stream2);
    }
    if (c->ev_copy2_join) (void)hipEventDestroy(c->ev_copy2_join);
    g_life.store("destroy: pools");
    delete c->pool;
    delete c->wpool;
    delete c->rpool;
    delete c;
    g_life.store("destroy: done");
    return OXH_OK;
}

void* oxh_ctx_stream(oxh_ctx* c) { return c ? (void*)c->stream : nullptr; }
}  // extern "C"

namespace oxh {
int ctx_device(oxh_ctx* c) { return c->device; }
std::mutex& ctx_call_mutex(oxh_ctx* c) { return c->mu; }
void*& ctx_cdc_state(oxh_ctx* c, void (*deleter)(void*)) {
    c->cdc_free = deleter;
    return c->cdc;
}
}  // namespace oxh

extern "C" {

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

// ---------------------------------------------------------------- streaming XXH3 (Xxh3)
// xxhash-rust's Xxh3::new / update / digest128 (hasher.rs:9,73-76,157-173, 183-244), with the device
// doing the hashing: bytes collect in a pinned buffer (grown on demand) of up to S + 1025 bytes (S = OXH_STREAM_PIECE_MIB,
// default 16 MiB, whole 1 KiB blocks); each time it fills, its first S bytes go to the device as one
// K1L piece (block sums chip-wide, then the chain resumed from the stream's 8 accumulators, which stay
// in device memory) and the last 1025 bytes move to the front. XXH3 scrambles every block but the
// last and reads the last stripe at len - 64, so keeping > 1 KiB back means the digest always has
// the item's tail on hand. digest128() hashes what is pending as the final piece without changing
// the state (updates may continue). Memory stays bounded whatever the stream's length.
struct oxh_xxh3_stream {
    int device = 0;
    uint64_t piece = 0;           // S
    uint8_t* h_pend = nullptr;    // pinned, grown on demand up to S + 1025
    uint64_t h_cap = 0;
    uint64_t fill = 0, total = 0, pieces = 0;
    uint8_t* d_mem = nullptr;     // [piece 0 | piece 1 | sums 0 | sums 1 | state 8 | out 2], from the first piece on
    uint8_t* d_piece[2] = {};
    uint64_t* d_sums[2] = {};
    uint64_t *d_state = nullptr, *d_out = nullptr;
    uint8_t* d_one = nullptr;     // a stream that never reached a piece: its bytes + out, grown on demand
    uint64_t d_one_cap = 0;
    hipStream_t st = nullptr;
    hipEvent_t ev_copied = nullptr, ev_free[2] = {};
    bool used[2] = {};
};

namespace {

// the stream and its events are created on first device use: a short-lived Xxh3 over a small blob
// (HashingReader / AtomicFile over one received file) pays for neither until its digest
int stream_queue(oxh_xxh3_stream* s) {
    if (s->st) return OXH_OK;
    if (hipStreamCreateWithFlags(&s->st, hipStreamNonBlocking) != hipSuccess) {
        s->st = nullptr;
        (void)hipGetLastError();
        return fail(OXH_ERR_NOMEM, "stream queue");
    }
    return OXH_OK;
}

int stream_device(oxh_xxh3_stream* s) {
    if (s->d_mem) return OXH_OK;
    if (int rc = stream_queue(s)) return rc;
    if (hipEventCreateWithFlags(&s->ev_copied, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&s->ev_free[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&s->ev_free[1], hipEventDisableTiming) != hipSuccess) {
        (void)hipGetLastError();
        return fail(OXH_ERR_NOMEM, "stream events");
    }
    const uint64_t pb = align_up(s->piece + 1025) + 256, sb = ((s->piece >> 10) + 1) * 64;
    if (hipMalloc(&s->d_mem, 2 * pb + 2 * sb + 256) != hipSuccess) {
        s->d_mem = nullptr;
        (void)hipGetLastError();
        return fail(OXH_ERR_NOMEM, "stream device buffers");
    }
    s->d_piece[0] = s->d_mem;
    s->d_piece[1] = s->d_mem + pb;
    s->d_sums[0] = reinterpret_cast<uint64_t*>(s->d_mem + 2 * pb);
    s->d_sums[1] = reinterpret_cast<uint64_t*>(s->d_mem + 2 * pb + sb);
    s->d_state = reinterpret_cast<uint64_t*>(s->d_mem + 2 * pb + 2 * sb);
    s->d_out = s->d_state + 8;
    return OXH_OK;
}

// room for `need` pending bytes (pinned; grown x4 from 64 KiB, capped at S + 1025)
int stream_reserve(oxh_xxh3_stream* s, uint64_t need) {
    if (need <= s->h_cap) return OXH_OK;
    const uint64_t full = s->piece + 1025;
    const uint64_t cap = std::min(full, std::max({need, 4 * s->h_cap, (uint64_t)64 << 10}));
    uint8_t* h = nullptr;
    if (hipHostMalloc(&h, cap, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        return fail(OXH_ERR_NOMEM, "stream pending buffer");
    }
    if (s->fill) memcpy(h, s->h_pend, s->fill);
    if (s->h_pend) (void)hipHostFree(s->h_pend);
    s->h_pend = h;
    s->h_cap = cap;
    return OXH_OK;
}

// the next device piece buffer, once the chain that last read it is done
int stream_take_piece(oxh_xxh3_stream* s, int& b) {
    b = (int)(s->pieces & 1);
    if (s->used[b]) HIP_TRY(hipEventSynchronize(s->ev_free[b]));
    return OXH_OK;
}

// block sums + chain of `len` bytes already in d_piece[b]
int stream_chain(oxh_xxh3_stream* s, int b, uint64_t len, bool partial) {
    const uint64_t nb = partial ? len >> 10 : (len - 1) >> 10;
    const uint64_t nwaves = (nb + 3) / 4, blocks = (nwaves + 3) / 4;
    if (blocks)
        hipLaunchKernelGGL(oxh::xxh3_blocksum_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, s->st, s->d_piece[b], nb,
                           s->d_sums[b]);
    oxh::ChainBatch batch;
    batch.job[0] = {s->d_piece[b], len, s->d_sums[b], s->d_out, s->total, s->d_state,
                    (s->pieces > 0 ? oxh::kChainResume : 0u) | (partial ? oxh::kChainPartial : 0u)};
    hipLaunchKernelGGL(oxh::xxh3_chain_kernel, dim3(1), dim3(64), kChainLdsPad, s->st, batch);
    HIP_TRY(hipGetLastError());
    return OXH_OK;
}

// the first S pending bytes become a piece; the last 1025 move to the front
int stream_flush(oxh_xxh3_stream* s) {
    if (int rc = stream_device(s)) return rc;
    int b = 0;
    if (int rc = stream_take_piece(s, b)) return rc;
    HIP_TRY(hipMemcpyAsync(s->d_piece[b], s->h_pend, s->piece, hipMemcpyHostToDevice, s->st));
    HIP_TRY(hipEventRecord(s->ev_copied, s->st));
    if (int rc = stream_chain(s, b, s->piece, true)) return rc;
    HIP_TRY(hipEventRecord(s->ev_free[b], s->st));
    s->used[b] = true;
    s->pieces++;
    HIP_TRY(hipEventSynchronize(s->ev_copied));  // the pinned bytes were read: reuse the buffer
    memmove(s->h_pend, s->h_pend + s->piece, 1025);
    s->fill = 1025;
    return OXH_OK;
}

}  // namespace

int oxh_xxh3_stream_create(oxh_ctx* ctx, oxh_xxh3_stream** out) {
    if (!ctx || !out) return fail(OXH_ERR_INVALID, "bad stream arguments");
    *out = nullptr;
    oxh_xxh3_stream* s = new oxh_xxh3_stream();
    s->device = ctx->device;
    const char* e = getenv("OXH_STREAM_PIECE_MIB");
    const uint64_t kib = e && strtoull(e, nullptr, 10) ? strtoull(e, nullptr, 10) << 10 : 16ull << 10;
    s->piece = kib << 10;  // whole 1 KiB blocks
    *out = s;              // nothing is allocated until bytes arrive
    return OXH_OK;
}

int oxh_xxh3_stream_update(oxh_xxh3_stream* s, const void* data, uint64_t len) {
    if (!s || (len && !data)) return fail(OXH_ERR_INVALID, "bad stream update");
    if (!len) return OXH_OK;
    HIP_TRY(hipSetDevice(s->device));
    const uint8_t* p = (const uint8_t*)data;
    const uint64_t cap = s->piece + 1025;
    while (len) {
        const uint64_t take = std::min(len, cap - s->fill);
        g_stream_where.store("update: reserve");
        if (int rc = stream_reserve(s, s->fill + take)) return rc;
        g_stream_where.store("update: copy");
        memcpy(s->h_pend + s->fill, p, take);
        s->fill += take;
        s->total += take;
        p += take;
        len -= take;
        if (s->fill == cap) {
            g_stream_where.store("update: flush");
            if (int rc = stream_flush(s)) return rc;
        }
    }
    g_stream_where.store("update: done");
    return OXH_OK;
}

int oxh_xxh3_stream_digest(oxh_xxh3_stream* s, uint64_t* out2) {
    if (!s || !out2) return fail(OXH_ERR_INVALID, "bad stream digest");
    HIP_TRY(hipSetDevice(s->device));
    g_stream_where.store("digest: queue");
    if (int rc = stream_queue(s)) return rc;
    g_stream_where.store("digest: final piece");
    uint64_t* d_out = nullptr;
    if (s->pieces == 0) {  // the whole stream is pending: a one-shot digest (K1, or K1L above 1 MiB)
        const uint64_t need = align_up(s->fill + 1) + 256;
        if (need > s->d_one_cap) {
            if (s->d_one) (void)hipFree(s->d_one);
            s->d_one = nullptr, s->d_one_cap = 0;
            const uint64_t cap = std::max<uint64_t>(need, 64 << 10);
            if (hipMalloc(&s->d_one, cap) != hipSuccess) {
                s->d_one = nullptr;
                (void)hipGetLastError();
                return fail(OXH_ERR_NOMEM, "stream device buffer");
            }
            s->d_one_cap = cap;
        }
        d_out = reinterpret_cast<uint64_t*>(s->d_one + s->d_one_cap - 256);
        if (s->fill) HIP_TRY(hipMemcpyAsync(s->d_one, s->h_pend, s->fill, hipMemcpyHostToDevice, s->st));
        const uint8_t* d = s->d_one;
        if (int rc = large_batch_device(&d, &s->fill, 1, d_out, s->st)) return rc;
    } else {  // fill >= 1025: the final piece
        int b = 0;
        if (int rc = stream_take_piece(s, b)) return rc;
        HIP_TRY(hipMemcpyAsync(s->d_piece[b], s->h_pend, s->fill, hipMemcpyHostToDevice, s->st));
        if (int rc = stream_chain(s, b, s->fill, false)) return rc;
        HIP_TRY(hipEventRecord(s->ev_free[b], s->st));
        s->used[b] = true;
        d_out = s->d_out;
    }
    uint64_t h[2];
    HIP_TRY(hipMemcpyAsync(h, d_out, 16, hipMemcpyDeviceToHost, s->st));
    HIP_TRY(hipStreamSynchronize(s->st));
    out2[0] = h[0];
    out2[1] = h[1];
    return OXH_OK;
}

int oxh_xxh3_stream_reset(oxh_xxh3_stream* s) {
    if (!s) return fail(OXH_ERR_INVALID, "stream is NULL");
    if (s->st) HIP_TRY(hipStreamSynchronize(s->st));
    s->fill = s->total = s->pieces = 0;
    return OXH_OK;
}

int oxh_xxh3_stream_destroy(oxh_xxh3_stream* s) {
    if (!s) return OXH_OK;
    (void)hipSetDevice(s->device);
    g_stream_where.store("destroy: sync");
    if (s->st) (void)hipStreamSynchronize(s->st);
    g_stream_where.store("destroy: free");
    if (s->d_mem) (void)hipFree(s->d_mem);
    if (s->d_one) (void)hipFree(s->d_one);
    if (s->h_pend) (void)hipHostFree(s->h_pend);
    if (s->ev_copied) (void)hipEventDestroy(s->ev_copied);
    for (hipEvent_t e : s->ev_free)
        if (e) (void)hipEventDestroy(e);
    if (s->st) (void)hipStreamDestroy(s->st);
    delete s;
    g_stream_where.store("destroy: done");
    return OXH_OK;
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

// Host-resident buffers (oxh_hash_buffers / oxh_hash_streams): item i (lens[i] bytes) is copied by
// copy(i, dst) straight into a pinned slot; slots are packed greedily in order, hashed on the GPU
// while the next one fills, and items larger than a slot go through the oversize path.
// Items of the short XXH3 paths (<= 240 B: paths, metadata JSON, most parent-node streams) are packed
// back to back: their kernels load unaligned bytes anyway, and 256-B slots would move ~8x their bytes
// over PCIe (a commit's 200 000 bucket paths: 6.3 MB instead of 51 MB). Longer items start on 256 B.
// OXH_HOST_ALIGN_ALL=1: every item on 256 B (the r02 packing, for A/B).
static uint64_t place(uint64_t off, uint64_t len) {
    static const bool all = getenv("OXH_HOST_ALIGN_ALL") && atoi(getenv("OXH_HOST_ALIGN_ALL")) != 0;
    return (len > 240 || all) ? align_up(off) : off;
}

static int hash_host_items(oxh_ctx* c, uint64_t n, const uint64_t* lens,
                           const std::function<const uint8_t*(uint64_t)>& src, uint64_t* out, bool short_only_lane) {
    Trace tr;
    Pending pend[NSLOT];
    int slot = 0;
    uint64_t i = 0;
    std::vector<uint64_t> batch;
    while (i < n) {
        batch.clear();
        uint64_t bytes = 0;
        while (i < n && batch.size() < c->max_items) {
            const uint64_t L = lens[i];
            if (L > c->stage_bytes) {  // straight from the caller's buffer, in pieces (large_item)
                if (!batch.empty()) break;
                MemSource ms(src(i));
                LargeResult res;
                if (int rc = large_item(c, L, ms, false, false, nullptr, i, res)) return rc;
                if (res.status != OXH_OK) return fail(res.status, "large host buffer: device or pinned memory unavailable");
                out[2 * i] = res.out[0];
                out[2 * i + 1] = res.out[1];
                ++i;
                continue;
            }
            if (place(bytes, L) + L > c->stage_bytes) break;
            bytes = place(bytes, L) + L;
            batch.push_back(i);
            ++i;
        }
        if (batch.empty()) continue;
        const int s = slot;
        slot = (slot + 1) % NSLOT;
        const double t0 = Trace::now();
        if (int rc = drain_slot(c, s, pend[s], out)) return rc;  // the slot's previous batch
        const double t1 = Trace::now();
        tr.drain += t1 - t0;
        const uint64_t M = c->max_items;
        uint64_t* hoff = c->h_desc[s];
        uint64_t* hlen = c->h_desc[s] + M;
        uint64_t off = 0;
        bool all_short = true;
        for (size_t j = 0; j < batch.size(); ++j) {
            off = place(off, lens[batch[j]]);
            hoff[j] = off;
            hlen[j] = lens[batch[j]];
            if (hlen[j] > 240) all_short = false;
            off += hlen[j];
        }
        STEP("fill s=%d items=%zu", s, batch.size());
        const int ntasks = (int)std::min<size_t>(batch.size(), (size_t)c->pool->size() * 4);
        c->pool->parallel_for(ntasks, [&](int t) {
            for (size_t j = (size_t)t; j < batch.size(); j += (size_t)ntasks)
                if (hlen[j]) memcpy(c->h_stage[s] + hoff[j], src(batch[j]), hlen[j]);
        });
        const double t2 = Trace::now();
        tr.fill += t2 - t1;
        if (int rc = submit_slot(c, s, off, batch.size(), short_only_lane && all_short,
                                 off / std::max<uint64_t>(1, batch.size()) <= kShortItemBytes, false))
            return rc;
        tr.submit += Trace::now() - t2;
        tr.batches++;
        pend[s].busy = true;
        pend[s].ids = batch;
    }
    const double t3 = Trace::now();
    STEP("final drain");
    for (int s = 0; s < NSLOT; ++s)
        if (int rc = drain_slot(c, s, pend[s], out)) return rc;
    tr.drain += Trace::now() - t3;
    if (tr.on)
        fprintf(stderr, "[oxh] items=%llu batches=%d fill=%.3fs drain-wait=%.3fs submit=%.3fs threads=%d\n",
                (unsigned long long)n, tr.batches, tr.fill, tr.drain, tr.submit, c->pool->size());
    return OXH_OK;
}

int oxh_hash_buffers(oxh_ctx* c, const uint8_t* const* bufs, const uint64_t* lens, uint64_t n, uint64_t* out) {
    if (!c || (n && (!bufs || !lens || !out))) return fail(OXH_ERR_INVALID, "bad arguments");
    std::lock_guard<std::mutex> g(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    return hash_host_items(c, n, lens, [&](uint64_t i) { return bufs[i]; }, out, false);
}

// oxh_hash_streams over an arena whose items run forward (offsets non-decreasing, gaps at most as
// large as the items): each batch is ONE span of the arena, copied into the pinned slot in large
// pieces by the pool, with the items' offsets rebased onto it -- no per-item copy. A commit's
// 200 000 bucket paths are such an arena (the serialised streams of commit_writer); a per-item copy
// of them costs ~12 ns an item on the host. Items larger than a slot go the oversize path as before.
static int hash_stream_spans(oxh_ctx* c, const uint8_t* streams, const uint64_t* offsets, const uint64_t* lens, uint64_t n,
                             uint64_t* out) {
    Trace tr;
    Pending pend[NSLOT];
    int slot = 0;
    uint64_t i = 0;
    std::vector<uint64_t> batch;
    while (i < n) {
        if (lens[i] > c->stage_bytes) {  // straight from the caller's buffer, in pieces (large_item)
            MemSource ms(streams + offsets[i]);
            LargeResult res;
            if (int rc = large_item(c, lens[i], ms, false, false, nullptr, i, res)) return rc;
            if (res.status != OXH_OK) return fail(res.status, "large host buffer: device or pinned memory unavailable");
            out[2 * i] = res.out[0];
            out[2 * i + 1] = res.out[1];
            ++i;
            continue;
        }
        const uint64_t base = offsets[i];
        uint64_t end = base, k = i;
        bool all_short = true;
        batch.clear();
        while (k < n && batch.size() < c->max_items && lens[k] <= c->stage_bytes &&
               std::max(end, offsets[k] + lens[k]) - base <= c->stage_bytes) {
            end = std::max(end, offsets[k] + lens[k]);
            if (lens[k] > 240) all_short = false;
            batch.push_back(k++);
        }
        const int s = slot;
        slot = (slot + 1) % NSLOT;
        const double t0 = Trace::now();
        if (int rc = drain_slot(c, s, pend[s], out)) return rc;  // the slot's previous batch
        const double t1 = Trace::now();
        tr.drain += t1 - t0;
        const uint64_t M = c->max_items;
        uint64_t* hoff = c->h_desc[s];
        uint64_t* hlen = c->h_desc[s] + M;
        for (size_t j = 0; j < batch.size(); ++j) {
            hoff[j] = offsets[batch[j]] - base;
            hlen[j] = lens[batch[j]];
        }
        const uint64_t span = end - base, piece = 1ull << 20;
        const int ntasks = (int)std::min<uint64_t>((span + piece - 1) / piece, (uint64_t)c->pool->size() * 4);
        if (ntasks > 1) {
            c->pool->parallel_for(ntasks, [&](int t) {
                const uint64_t lo = span * (uint64_t)t / (uint64_t)ntasks, hi = span * (uint64_t)(t + 1) / (uint64_t)ntasks;
                memcpy(c->h_stage[s] + lo, streams + base + lo, hi - lo);
            });
        } else if (span) {
            memcpy(c->h_stage[s], streams + base, span);
        }
        const double t2 = Trace::now();
        tr.fill += t2 - t1;
        if (int rc = submit_slot(c, s, span, batch.size(), all_short, span / std::max<uint64_t>(1, batch.size()) <= kShortItemBytes,
                                 false))
            return rc;
        tr.submit += Trace::now() - t2;
        tr.batches++;
        pend[s].busy = true;
        pend[s].ids = batch;
        i = k;
    }
    const double t3 = Trace::now();
    for (int s = 0; s < NSLOT; ++s)
        if (int rc = drain_slot(c, s, pend[s], out)) return rc;
    tr.drain += Trace::now() - t3;
    if (tr.on)
        fprintf(stderr, "[oxh] streams (spans)=%llu batches=%d fill=%.3fs drain-wait=%.3fs submit=%.3fs\n",
                (unsigned long long)n, tr.batches, tr.fill, tr.drain, tr.submit);
    return OXH_OK;
}

int oxh_hash_streams(oxh_ctx* c, const uint8_t* streams, const uint64_t* offsets, const uint64_t* lens, uint64_t n,
                     uint64_t* out) {
    if (!c || (n && (!streams || !offsets || !lens || !out))) return fail(OXH_ERR_INVALID, "bad arguments");
    STEP("hash_streams n=%llu", (unsigned long long)n);
    std::lock_guard<std::mutex> g(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    STEP("hash_streams locked");
    // spans when the items run forward through the arena without large gaps (OXH_STREAM_SPANS=0: per item)
    static const bool spans_on = !(getenv("OXH_STREAM_SPANS") && atoi(getenv("OXH_STREAM_SPANS")) == 0);
    bool forward = spans_on && n > 0;
    uint64_t total = 0, maxend = 0;
    for (uint64_t i = 0; forward && i < n; ++i) {
        total += lens[i];
        maxend = std::max(maxend, offsets[i] + lens[i]);
        if (i && offsets[i] < offsets[i - 1]) forward = false;
    }
    if (forward && maxend - offsets[0] > 2 * total + 4096) forward = false;  // a sparse arena: copy items
    if (forward) return hash_stream_spans(c, streams, offsets, lens, n, out);
    return hash_host_items(c, n, lens, [&](uint64_t i) { return streams + offsets[i]; }, out, true);
}

// ---------------------------------------------------------------- streaming file engine
// The reference reads, stats and hashes each file inside one per-file closure (add.rs:462-539 ->
// hasher.rs:126-148), and liboxen calls it for 64-file batches from up to 2 x ncpu tokio tasks at
// once (add.rs:41, 422-425): a few MB per call, far too small for one launch each. Here every file
// call on a context becomes a REQUEST on the context's queue, and one engine thread per context
// runs a continuous pipeline over all queued requests: requests that arrive while it runs join the
// live pipeline (their files go into the slot being filled), and each request completes, and its
// caller returns, as soon as its own last file is drained.
//
// Inside the pipeline T reader threads run without barriers or per-file locks: each claims the next
// 8 files of the current request, opens + fstats one (one path walk), reserves its bytes in the slot
// being filled with ONE CAS (item count in the high bits, 256-B-rounded bytes in the low bits),
// preads straight into the pinned slot and closes it. Reservations are monotone, so the first one
// that does not fit seals the slot: every earlier one fits and every later one fails. The reader
// that seals opens the next slot of the ring once the engine has freed it. The engine also seals a
// partly filled slot when it holds OXH_FLUSH_MIB (default 16 MiB) and the next slot is free, or
// when every reader is idle, so small requests never wait for a full 256 MiB slot. It submits a
// sealed slot when all its writers are done (H2D on the copy stream, K1/K1T (+ is_utf8), D2H) and
// drains submitted slots, oldest first, as their events complete.
namespace {

// One 64-bit word per slot: bytes (31 bits) | items (19) | sealed (1) | generation (13). Every
// reservation is a CAS on it, so a reader that read an older generation (the slot was sealed,
// submitted and reopened meanwhile) can never act on the new one.
constexpr int kWBytes = 31, kWItems = 19;
constexpr uint64_t kBytesMask = (1ull << kWBytes) - 1, kItemsMask = (1ull << kWItems) - 1;
constexpr uint64_t kSealedBit = 1ull << (kWBytes + kWItems);
constexpr int kGenShift = kWBytes + kWItems + 1;
static_assert(OXH_MAX_STAGING_BYTES <= kBytesMask, "a full slot's byte offset must fit the word");
static_assert(OXH_MAX_STAGING_BYTES / 4096 <= kItemsMask, "a full slot's item count must fit the word");
inline uint64_t w_bytes(uint64_t w) { return w & kBytesMask; }
inline uint64_t w_items(uint64_t w) { return (w >> kWBytes) & kItemsMask; }

struct SlotFill {
    std::atomic<int> state{0};         // 0 free, 1 filling (or sealed, not yet submitted), 2 submitted
    std::atomic<uint64_t> word{0};
    std::atomic<uint64_t> done{0};     // writers finished
};

struct SlotRun {  // a submitted slot
    uint64_t cnt = 0;
    bool text = false, utf8 = false;
};

}  // namespace

// One file call (oxh_hash_files / _text / _text_utf8 / oxh_add_files / fsck). Lives on its caller's
// stack; the engine writes its outputs in place and wakes the caller when the last item is done.
struct FileRequest {
    const char* const* paths = nullptr;
    const uint64_t* meta = nullptr;  // sizes the caller already has (get_hash_given_metadata), or null
    uint64_t n = 0;
    uint64_t* out = nullptr;
    uint64_t* sizes = nullptr;
    int32_t* status = nullptr;
    uint64_t* counts = nullptr;
    int32_t* utf8 = nullptr;
    int32_t* os_err = nullptr;  // per item: errno of a failed open (OXH_ERR_OPEN) or read (OXH_ERR_IO)
    ItemSink* sink = nullptr;
    std::vector<uint64_t> lens;
    std::vector<int32_t> st;
    std::vector<int32_t> eno;
    uint64_t next = 0;                   // claim cursor (under ctx->qmu)
    size_t idx = 0;                      // index in the run's request table
    std::atomic<uint64_t> remaining{0};  // items not yet accounted for
    int rc = OXH_OK;
    std::string msg;
    bool done = false;  // under mu
    std::mutex mu;
    std::condition_variable cv;
};

namespace {

struct FileStream {
    oxh_ctx* c;
    SlotFill slot[NSLOT];
    std::atomic<int> cur{0};
    std::atomic<int> readers_left{0};
    std::atomic<int> idle{0};            // readers waiting for new requests (changed under c->qmu)
    int nreaders = 0;
    std::atomic<bool> abort{false};
    bool closing = false;                // under c->qmu
    std::vector<FileRequest*> reqs;      // joined requests; nullptr once complete (under c->qmu)
    size_t cur_req = 0;                  // under c->qmu
    std::atomic<bool> want_text{false}, want_utf8{false};
    std::atomic<int> claimed_out{0};     // requests with every file claimed, not yet complete
    std::mutex omu;
    std::vector<std::pair<FileRequest*, uint64_t>> oversize;
    std::atomic<uint64_t> n_oversize{0};
    std::vector<std::pair<FileRequest*, uint64_t>> changed;  // meta size != file size: re-read
    std::atomic<uint64_t> n_changed{0};
    std::mutex cmu;  // the engine sleeps on ccv between events
    std::condition_variable ccv;
    uint64_t files = 0, slots = 0;
    void wake() {
        std::lock_guard<std::mutex> g(cmu);
        ccv.notify_all();
    }
};

inline void pause_us(int us) { std::this_thread::sleep_for(std::chrono::microseconds(us)); }

// Request r is complete: zero the outputs of failed items (add.rs:533-544 skips them), report sizes
// and statuses, retire it from the run and wake its caller.
void finish_request(FileStream& fs, FileRequest* r) {
    for (uint64_t i = 0; i < r->n; ++i) {
        if (r->st[i] != OXH_OK) {
            r->out[2 * i] = r->out[2 * i + 1] = 0;
            if (r->counts) r->counts[2 * i] = r->counts[2 * i + 1] = 0;
            if (r->utf8) r->utf8[i] = 0;  // read_first_n_bytes failed -> is_utf8 false (fs.rs:655-658)
        }
        if (r->sizes) r->sizes[i] = r->lens[i];
        if (r->status) r->status[i] = r->st[i];
        if (r->os_err) r->os_err[i] = r->st[i] == OXH_OK ? 0 : r->eno[i];
    }
    {
        std::lock_guard<std::mutex> g(fs.c->qmu);
        fs.reqs[r->idx] = nullptr;
    }
    fs.claimed_out.fetch_sub(1);
    std::lock_guard<std::mutex> g(r->mu);  // notify under the lock: the caller frees r once it sees done
    r->done = true;
    r->cv.notify_all();
}

// Item i of r could not be hashed. `code` says which call of the reference's hash_small_file_contents
// failed (hasher.rs:126-146): File::open (OXH_ERR_OPEN) or the read (OXH_ERR_IO); `e` is the errno its
// io::Error carries (0: the file ended before the size it was read at).
inline void item_failed(FileRequest* r, uint64_t i, int code, int e) {
    r->st[i] = code;
    r->eno[i] = e;
}
// The errno of an opened file that is not hashed: the fstat's own failure, or, for a file that is not
// regular, what its read reports -- open(2) of a directory succeeds on Linux and the read fails with
// EISDIR, as File::open + read_to_end do in the reference; other non-regular files are refused as
// unreadable (EINVAL). Call right after the failed fstat / S_ISREG test on fd.
inline int unreadable_errno(int fd, struct stat& sb) {
    if (fstat(fd, &sb) != 0) return errno;
    return S_ISDIR(sb.st_mode) ? EISDIR : EINVAL;
}

// k more items of r are fully written; the thread that accounts the last one completes r.
inline void account(FileStream& fs, FileRequest* r, uint64_t k) {
    if (k && r->remaining.fetch_sub(k, std::memory_order_acq_rel) == k) finish_request(fs, r);
}

// Next files to read: [i0, i1) of request *r. Moves queued requests into the run; an idle reader
// sleeps until a request arrives or the engine closes the run. False = stop.
bool claim(FileStream& fs, FileRequest*& r, uint64_t& i0, uint64_t& i1) {
    constexpr uint64_t kClaim = 8;
    oxh_ctx* c = fs.c;
    std::unique_lock<std::mutex> lk(c->qmu);
    for (;;) {
        if (fs.abort.load(std::memory_order_relaxed) || fs.closing) return false;
        for (; fs.cur_req < fs.reqs.size(); ++fs.cur_req) {
            FileRequest* q = fs.reqs[fs.cur_req];
            if (q && q->next < q->n) {
                r = q;
                i0 = q->next;
                i1 = std::min(q->n, i0 + kClaim);
                q->next = i1;
                if (i1 == q->n) fs.claimed_out.fetch_add(1);  // its caller may be waiting on a partial slot
                return true;
            }
        }
        if (!c->queue.empty()) {
            for (FileRequest* q : c->queue) {
                q->idx = fs.reqs.size();
                fs.reqs.push_back(q);
                fs.files += q->n;
                if (q->counts) fs.want_text.store(true);
                if (q->utf8) fs.want_utf8.store(true);
            }
            c->queue.clear();
            continue;
        }
        if (fs.idle.fetch_add(1) + 1 == fs.nreaders) fs.wake();  // the engine may flush or close now
        c->qcv.wait(lk, [&] { return fs.abort.load() || fs.closing || !c->queue.empty(); });
        fs.idle.fetch_sub(1);
    }
}

// Open slot t for filling (generation + 1, empty, unsealed) once the engine has freed it.
bool open_slot(FileStream& fs, int t) {
    SlotFill& nx = fs.slot[t];
    while (nx.state.load(std::memory_order_acquire) != 0) {
        if (fs.abort.load(std::memory_order_relaxed)) return false;
        pause_us(5);
    }
    const uint64_t gen = (nx.word.load(std::memory_order_relaxed) >> kGenShift) + 1;
    nx.done.store(0, std::memory_order_relaxed);
    nx.word.store((gen << kGenShift) & ~0ull, std::memory_order_release);
    nx.state.store(1, std::memory_order_release);
    fs.cur.store(t, std::memory_order_release);
    return true;
}

// Reserve L bytes for item i of r; returns the slot (and offset), or -1 on abort.
int reserve(FileStream& fs, FileRequest* r, uint64_t i, uint64_t L, uint64_t room, uint64_t& off, uint64_t& jout) {
    oxh_ctx* c = fs.c;
    const uint64_t M = c->max_items, cap = c->stage_bytes;
    const uint64_t need = align_up(room);
    for (;;) {
        if (fs.abort.load(std::memory_order_relaxed)) return -1;
        const int s = fs.cur.load(std::memory_order_acquire);
        SlotFill& sl = fs.slot[s];
        uint64_t w = sl.word.load(std::memory_order_acquire);
        if (w & kSealedBit) {  // full: wait for the sealer to open the next slot
            // ... or for this slot's word to change: while this reader sleeps, the ring can go all
            // the way round (small slots flushed early) and reopen slot s with cur == s again, and
            // waiting on `cur` alone would then never end
            while (fs.cur.load(std::memory_order_acquire) == s && sl.word.load(std::memory_order_acquire) == w &&
                   !fs.abort.load(std::memory_order_relaxed))
                pause_us(2);
            continue;
        }
        const uint64_t o = w_bytes(w), j = w_items(w);
        if (o + room <= cap && j < M) {
            if (!sl.word.compare_exchange_weak(w, w + (1ull << kWBytes) + need, std::memory_order_acq_rel)) continue;
            off = o;
            jout = j;
            c->h_desc[s][j] = o;
            c->h_desc[s][M + j] = L;
            c->rq[s][j] = r;
            c->loc[s][j] = i;
            return s;
        }
        // does not fit: seal it (one reader wins) and open the next slot of the ring
        if (!sl.word.compare_exchange_strong(w, w | kSealedBit, std::memory_order_acq_rel)) continue;
        if (sl.done.load(std::memory_order_acquire) == j) fs.wake();  // its writers are all done
        if (!open_slot(fs, (s + 1) % NSLOT)) return -1;
    }
}

void reader_loop(FileStream& fs) {
    oxh_ctx* c = fs.c;
    FileRequest* r = nullptr;
    uint64_t i0 = 0, i1 = 0;
    bool stop = false;
    while (!stop && claim(fs, r, i0, i1)) {
        uint64_t failed = 0;  // items of this claim that never reach a slot
        for (uint64_t i = i0; i < i1; ++i) {
            struct stat sb;
            const int fd = r->paths[i] ? open(r->paths[i], O_RDONLY | O_CLOEXEC | O_NONBLOCK) : -1;
            if (fd < 0) {
                item_failed(r, i, OXH_ERR_OPEN, r->paths[i] ? errno : EINVAL);
                ++failed;
                continue;
            }
            // with the caller's metadata size no fstat is needed. Either way the reader asks for one
            // byte more than the expected size L and re-reads the file (fstat + whole read) if it
            // gets a different count: a file that grew or shrank since its size was taken is hashed
            // as it is at read time, like the reference's read_to_end (hasher.rs:126-148)
            const bool meta = r->meta != nullptr && r->meta[i] < c->stage_bytes;
            if (!meta && (fstat(fd, &sb) != 0 || !S_ISREG(sb.st_mode))) {
                item_failed(r, i, OXH_ERR_IO, unreadable_errno(fd, sb));
                close(fd);
                ++failed;
                continue;
            }
            const uint64_t L = meta ? r->meta[i] : (uint64_t)sb.st_size;
            r->lens[i] = L;
            if (L >= c->stage_bytes) {  // the engine reads it through the oversize path (L + 1 > a slot)
                close(fd);
                {
                    std::lock_guard<std::mutex> g(fs.omu);
                    fs.oversize.push_back({r, i});
                }
                fs.n_oversize.fetch_add(1);
                fs.wake();
                continue;
            }
            uint64_t off = 0, j = 0;
            const int s = reserve(fs, r, i, L, L + 1, off, j);
            if (s < 0) {
                close(fd);
                stop = true;  // aborted: the engine fails every open request
                break;
            }
            uint8_t* dst = c->h_stage[s] + off;
            const uint64_t want = L + 1;
            uint64_t got = 0;
            while (got < want) {
                const ssize_t k = pread(fd, dst + got, want - got, (off_t)got);
                if (k < 0) {
                    item_failed(r, i, OXH_ERR_IO, errno);
                    break;
                }
                if (k == 0) break;  // EOF
                got += (uint64_t)k;
                // a short read of a regular file ends at its EOF: once the expected L bytes are in,
                // that settles the size without the extra pread that would return 0
                if (got >= L && (uint64_t)k < want - (got - (uint64_t)k)) break;
            }
            close(fd);
            if (r->st[i] == OXH_OK && got != L) {  // the file is not the size the stat / the caller saw
                c->rq[s][j] = nullptr;                     // drain skips this slot entry
                {
                    std::lock_guard<std::mutex> g(fs.omu);
                    fs.changed.push_back({r, i});
                }
                fs.n_changed.fetch_add(1);
                fs.wake();
            }
            // the last writer of a sealed slot wakes the engine
            const uint64_t d = fs.slot[s].done.fetch_add(1, std::memory_order_acq_rel) + 1;
            const uint64_t w = fs.slot[s].word.load(std::memory_order_acquire);
            if ((w & kSealedBit) && d == w_items(w)) fs.wake();
        }
        if (!stop) account(fs, r, failed);
    }
    if (fs.readers_left.fetch_sub(1, std::memory_order_acq_rel) == 1) fs.wake();
}

// Scatter a completed slot's digests (+ counts, is_utf8) into the requests, run the sinks over the
// staged bytes (fused publish), then account the items.
void drain_files(FileStream& fs, int s, const SlotRun& p) {
    oxh_ctx* c = fs.c;
    const uint64_t M = c->max_items, cnt = p.cnt;
    FileRequest* const* rq = c->rq[s].data();
    const uint64_t* loc = c->loc[s].data();
    std::vector<ItemSink*> sinks;  // the distinct sinks of this slot's requests
    for (uint64_t j = 0; j < cnt; ++j) {
        FileRequest* r = rq[j];
        if (!r) continue;  // re-read later (its size changed)
        const uint64_t i = loc[j];
        r->out[2 * i] = c->h_out[s][2 * j];
        r->out[2 * i + 1] = c->h_out[s][2 * j + 1];
        if (r->counts && p.text) {
            r->counts[2 * i] = c->h_cnt[s][2 * j];
            r->counts[2 * i + 1] = c->h_cnt[s][2 * j + 1];
        }
        if (r->utf8 && p.utf8) r->utf8[i] = c->h_utf8[s][j];
        if (r->sink && std::find(sinks.begin(), sinks.end(), r->sink) == sinks.end()) sinks.push_back(r->sink);
    }
    if (!sinks.empty()) {
        if (!c->wpool) c->wpool = new oxh::Pool(c->pool->size());
        const int ntasks = (int)std::min<uint64_t>(cnt, (uint64_t)c->wpool->size() * 4);
        c->wpool->parallel_for(ntasks, [&](int t) {
            for (uint64_t j = (uint64_t)t; j < cnt; j += (uint64_t)ntasks) {
                FileRequest* r = rq[j];
                if (!r) continue;
                const uint64_t i = loc[j];
                if (!r->sink || r->st[i] != OXH_OK) continue;
                r->sink->put(i, c->h_stage[s] + c->h_desc[s][j], c->h_desc[s][M + j], c->h_out[s][2 * j], c->h_out[s][2 * j + 1]);
            }
        });
        for (ItemSink* k : sinks) k->commit();  // one durability barrier per slot, not per file
    }
    for (uint64_t j = 0; j < cnt;) {  // one atomic per run of items of the same request
        uint64_t k = j + 1;
        while (k < cnt && rq[k] == rq[j]) ++k;
        if (rq[j]) account(fs, rq[j], k - j);
        j = k;
    }
}

// Files of the engine larger than a staging slot, up to big_files_at_once() side by side.
int refresh_file(FileStream& fs, FileRequest* r, uint64_t i);

int big_files(FileStream& fs, const std::vector<std::pair<FileRequest*, uint64_t>>& items) {
    const int n = (int)items.size();
    std::vector<std::unique_ptr<FileSource>> srcs(n);
    std::vector<LargeJob> jobs;
    std::vector<int> who;              // jobs[k] is items[who[k]]
    std::vector<bool> shrunk(n, false);  // now below a staging slot: read whole by refresh_file
    for (int q = 0; q < n; ++q) {
        FileRequest* r = items[q].first;
        const uint64_t i = items[q].second;
        // The pieces are planned from the size of the file THIS descriptor reads: the path may name a
        // different file than the reader's stat saw (replaced since, e.g. by an editor's rename), and the
        // reference reads whatever the file holds when it opens it (hasher.rs:150-174).
        const int fd = open(r->paths[i], O_RDONLY | O_CLOEXEC | O_NONBLOCK);
        struct stat sb;
        if (fd < 0) {
            item_failed(r, i, OXH_ERR_OPEN, errno);
            continue;
        }
        if (fstat(fd, &sb) != 0 || !S_ISREG(sb.st_mode)) {
            item_failed(r, i, OXH_ERR_IO, unreadable_errno(fd, sb));
            close(fd);
            continue;
        }
        r->lens[i] = (uint64_t)sb.st_size;
        if (r->lens[i] < fs.c->stage_bytes) {
            close(fd);
            shrunk[q] = true;
            continue;
        }
        srcs[q].reset(new FileSource(fd, r->lens[i], r->sink == nullptr));
        LargeJob j;
        j.L = r->lens[i], j.src = srcs[q].get(), j.want_counts = r->counts != nullptr, j.want_utf8 = r->utf8 != nullptr;
        j.sink = r->sink, j.id = i;
        jobs.push_back(j);
        who.push_back(q);
    }
    if (int rc = large_items(fs.c, jobs.data(), (int)jobs.size())) return rc;
    for (size_t k = 0; k < jobs.size(); ++k) {
        FileRequest* r = items[who[k]].first;
        const uint64_t i = items[who[k]].second;
        const LargeResult& res = jobs[k].res;
        if (res.status != OXH_OK) {
            item_failed(r, i, res.status, res.os_error);
            continue;
        }
        r->out[2 * i] = res.out[0];
        r->out[2 * i + 1] = res.out[1];
        if (r->counts) {
            r->counts[2 * i] = res.cnt[0];
            r->counts[2 * i + 1] = res.cnt[1];
        }
        if (r->utf8) r->utf8[i] = res.utf8;
    }
    for (int q = 0; q < n; ++q) {
        if (!shrunk[q]) {
            account(fs, items[q].first, 1);
        } else if (int rc = refresh_file(fs, items[q].first, items[q].second)) {  // accounts the item itself
            return rc;  // a HIP error: the run fails every open request
        }
    }
    return OXH_OK;
}

// A file larger than a staging slot, with or without a sink: streamed in pieces (big_files).
int oversize_file(FileStream& fs, FileRequest* r, uint64_t i) { return big_files(fs, {{r, i}}); }

// A file whose size changed between the stat (or the caller's metadata) and the read: stat and read
// it afresh (the reference reads whatever the file holds, hasher.rs:126-148). It fits a staging
// slot, so the host copy is bounded by the slot size.
int refresh_file(FileStream& fs, FileRequest* r, uint64_t i) {
    oxh_ctx* c = fs.c;
    struct stat sb;
    const int fd = open(r->paths[i], O_RDONLY | O_CLOEXEC | O_NONBLOCK);
    if (fd < 0 || fstat(fd, &sb) != 0 || !S_ISREG(sb.st_mode)) {
        if (fd < 0) item_failed(r, i, OXH_ERR_OPEN, errno);
        else item_failed(r, i, OXH_ERR_IO, unreadable_errno(fd, sb));
        if (fd >= 0) close(fd);
        account(fs, r, 1);
        return OXH_OK;
    }
    const uint64_t L = (uint64_t)sb.st_size;
    r->lens[i] = L;
    if (L >= c->stage_bytes) {
        close(fd);
        return oversize_file(fs, r, i);
    }
    // read to EOF (read_to_end), whatever the stat said: st_size is a hint (a file still being
    // written, or one whose size the stat does not report, like /proc files with st_size 0)
    std::vector<uint8_t> tmp(std::max<uint64_t>(L + 1, 4096));
    uint64_t got = 0;
    bool bad = false;
    int bad_errno = 0;
    for (;;) {
        if (got == tmp.size()) {
            if (tmp.size() >= c->stage_bytes) break;  // grew past a staging slot meanwhile
            tmp.resize(std::min<uint64_t>(2 * tmp.size(), c->stage_bytes));
        }
        const ssize_t k = pread(fd, tmp.data() + got, tmp.size() - got, (off_t)got);
        if (k < 0) bad = true, bad_errno = errno;
        if (k <= 0) break;
        got += (uint64_t)k;
    }
    if (!bad && got == tmp.size()) {  // larger than a slot now: the streamed large-file path
        close(fd);
        struct stat sb2;
        r->lens[i] = stat(r->paths[i], &sb2) == 0 ? std::max<uint64_t>((uint64_t)sb2.st_size, got) : got;
        return oversize_file(fs, r, i);
    }
    close(fd);
    r->lens[i] = got;
    if (bad) {
        item_failed(r, i, OXH_ERR_IO, bad_errno);
    } else {
        const uint64_t L = got;
        int32_t u8 = 0;
        const int rc = oversize_item(c, tmp.data(), L, r->out + 2 * i, r->counts ? r->counts + 2 * i : nullptr,
                                     r->utf8 ? &u8 : nullptr);
        if (rc == OXH_ERR_NOMEM) {
            item_failed(r, i, OXH_ERR_NOMEM, 0);  // this file's failure, not the run's; os_error 0 (no open / read failed), as large_items reports it
        } else if (rc) {
            return rc;
        } else {
            if (r->utf8) r->utf8[i] = u8;
            if (r->sink) {
                r->sink->put(i, tmp.data(), L, r->out[2 * i], r->out[2 * i + 1]);
                r->sink->commit();
            }
        }
    }
    account(fs, r, 1);
    return OXH_OK;
}

// One run of the engine: from the first queued request until the readers are idle, the queue is
// empty and every submitted slot is drained.
void run_stream(oxh_ctx* c) {
    FileStream fs;
    fs.c = c;
    {
        std::lock_guard<std::mutex> g(c->qmu);
        c->live = &fs;
    }
    struct Unlive {
        oxh_ctx* c;
        ~Unlive() {
            std::lock_guard<std::mutex> g(c->qmu);
            c->live = nullptr;
        }
    } unlive{c};
    fs.slot[0].state.store(1);
    fs.slot[0].word.store(1ull << kGenShift);
    fs.nreaders = c->rpool->size();
    fs.readers_left.store(fs.nreaders);
    Trace tr;
    const double t_start = Trace::now();
    oxh::Pool::Group readers;  // the readers run on the context's persistent reader pool
    const std::function<void(int)> reader_fn = [&fs](int) { reader_loop(fs); };
    c->rpool->start(fs.nreaders, reader_fn, readers);
    SlotRun pend[NSLOT];
    const uint64_t M = c->max_items;
    int rc = hipSetDevice(c->device) == hipSuccess ? OXH_OK : fail(OXH_ERR_HIP, "hipSetDevice failed");
    int s = 0, nbusy = 0;  // s: the slot being filled; the nbusy slots before it are submitted
    static const double wait_limit = getenv("OXH_WAIT_LIMIT_S") ? atof(getenv("OXH_WAIT_LIMIT_S")) : 60.0;
    double last_progress = Trace::now();
    double big_wait_since = 0;  // when the oldest waiting large file was first seen
    while (rc == OXH_OK) {
        // 1. drain submitted slots whose digests are back, oldest first, and free them
        bool progressed = false;
        while (nbusy) {
            const int t = (s + NSLOT - nbusy) % NSLOT;
            const hipError_t q = hipEventQuery(c->ev_done[t]);
            if (q == hipErrorNotReady) break;
            if (q != hipSuccess) {
                rc = fail(OXH_ERR_HIP, std::string("slot event: ") + hipGetErrorString(q));
                break;
            }
            const double td = Trace::now();
            drain_files(fs, t, pend[t]);
            tr.drain += Trace::now() - td;
            fs.slot[t].state.store(0, std::memory_order_release);
            --nbusy;
            progressed = true;
        }
        if (rc) break;
        // 2. files larger than a slot, and files whose size changed, one at a time
        if (fs.n_changed.load(std::memory_order_acquire)) {
            std::pair<FileRequest*, uint64_t> it;
            {
                std::lock_guard<std::mutex> g(fs.omu);
                it = fs.changed.back();
                fs.changed.pop_back();
            }
            fs.n_changed.fetch_sub(1);
            c->where.store("engine: refresh_file");
            rc = refresh_file(fs, it.first, it.second);
            c->where.store("engine: loop");
            continue;
        }
        if (const uint64_t no = fs.n_oversize.load(std::memory_order_acquire)) {
            // several large files share one piece pipeline (their chains overlap the next pieces'
            // copies): while readers are still claiming files, give more of them a moment to arrive
            const double now = Trace::now();
            if (big_wait_since == 0) big_wait_since = now;
            const bool readers_done = fs.idle.load(std::memory_order_acquire) == fs.nreaders;
            if ((int)no >= big_files_at_once() || readers_done || now - big_wait_since > 0.002) {
                std::vector<std::pair<FileRequest*, uint64_t>> items;
                {
                    std::lock_guard<std::mutex> g(fs.omu);
                    while (!fs.oversize.empty() && (int)items.size() < big_files_at_once()) {
                        items.push_back(fs.oversize.back());
                        fs.oversize.pop_back();
                    }
                }
                fs.n_oversize.fetch_sub(items.size());
                big_wait_since = 0;
                c->where.store("engine: big_files");
                rc = big_files(fs, items);
                c->where.store("engine: loop");
                continue;
            }
        }
        // 3. the slot being filled: seal it early (flush) when it holds enough bytes or every reader
        //    is idle and the next slot is free; submit it once sealed and its writers are done
        SlotFill& sl = fs.slot[s];
        // Idle count FIRST, then the slot: a reader counts itself idle (in claim(), under qmu) only
        // after its reservations in the slot word, so a word read after seeing every reader idle holds
        // all of them. Read the other way round, a reader could reserve an item between the word load
        // and the idle load, and step 4 closed the run over a slot it still saw empty: that item's
        // request never completed (found by tools/engine_soak.py, once in ~157 000 requests).
        const bool all_idle = fs.idle.load(std::memory_order_acquire) == fs.nreaders;
        // state before word: a slot seen open (state 1) shows its current generation's word
        const int sst = sl.state.load(std::memory_order_acquire);
        uint64_t w = sl.word.load(std::memory_order_acquire);
        // (early flushes only help while some caller is waiting on a partial slot: a request whose
        // files are all claimed; a lone whole-list call keeps full slots until its last files)
        if (sst == 1 && !(w & kSealedBit) && w_items(w) > 0 &&
            (all_idle || (w_bytes(w) >= c->flush_bytes && fs.claimed_out.load(std::memory_order_relaxed) > 0)) &&
            fs.slot[(s + 1) % NSLOT].state.load(std::memory_order_acquire) == 0) {
            if (!sl.word.compare_exchange_strong(w, w | kSealedBit, std::memory_order_acq_rel)) continue;
            w |= kSealedBit;
            open_slot(fs, (s + 1) % NSLOT);
        }
        if (sst == 1 && (w & kSealedBit) && sl.done.load(std::memory_order_acquire) == w_items(w) &&
            sl.word.load(std::memory_order_acquire) == w) {
            const uint64_t cnt = w_items(w);
            uint64_t bytes = 0;
            for (uint64_t j = 0; j < cnt; ++j) bytes = std::max(bytes, c->h_desc[s][j] + c->h_desc[s][M + j]);
            const double t0 = Trace::now();
            pend[s].cnt = cnt;
            pend[s].text = fs.want_text.load();
            pend[s].utf8 = fs.want_utf8.load();
            sl.state.store(2, std::memory_order_release);
            c->where.store("engine: submit_slot");
            rc = submit_slot(c, s, bytes, cnt, false, bytes / cnt <= kShortItemBytes, pend[s].text, pend[s].utf8);
            c->where.store("engine: loop");
            if (nbusy == 0) last_progress = Trace::now();
            tr.submit += Trace::now() - t0;
            tr.batches++;
            ++nbusy;
            s = (s + 1) % NSLOT;
            continue;
        }
        // 4. nothing left: close the run (requests arriving later start the next one)
        if (all_idle && sst == 1 && !(w & kSealedBit) && w_items(w) == 0 && nbusy == 0 && fs.n_oversize.load() == 0 &&
            fs.n_changed.load() == 0) {
            std::lock_guard<std::mutex> g(c->qmu);
            // still nothing: no request queued, every reader idle, the slot still empty (re-read
            // under the lock the readers take to go idle)
            if (c->queue.empty() && fs.idle.load() == fs.nreaders && w_items(sl.word.load(std::memory_order_acquire)) == 0 &&
                fs.n_oversize.load() == 0 && fs.n_changed.load() == 0) {
                fs.closing = true;
                c->qcv.notify_all();
                break;
            }
            continue;
        }
        if (progressed) {
            last_progress = Trace::now();
            continue;
        }
        if (nbusy && Trace::now() - last_progress > wait_limit) {  // report a stalled GPU instead of hanging
            fprintf(stderr, "[oxh] slot %d stalled: copy_stream=%s stream=%s\n", (s + NSLOT - nbusy) % NSLOT,
                    hipGetErrorName(hipStreamQuery(c->copy_stream)), hipGetErrorName(hipStreamQuery(c->stream)));
            rc = fail(OXH_ERR_HIP, "timed out waiting for a staged batch (see stderr)");
            break;
        }
        // 5. sleep until a reader reports an event; poll the GPU while slots are in flight
        std::unique_lock<std::mutex> lk(fs.cmu);
        fs.ccv.wait_for(lk, std::chrono::microseconds(nbusy ? 20 : 100));
    }
    if (rc) {
        const std::string msg = g_err;
        {
            std::lock_guard<std::mutex> g(c->qmu);
            fs.abort.store(true);
            c->qcv.notify_all();
        }
        readers.wait();
        (void)hipStreamSynchronize(c->stream);
        (void)hipStreamSynchronize(c->copy_stream);
        std::vector<FileRequest*> open;
        {
            std::lock_guard<std::mutex> g(c->qmu);
            for (FileRequest*& r : fs.reqs)
                if (r) open.push_back(r), r = nullptr;
        }
        for (FileRequest* r : open) {
            std::lock_guard<std::mutex> g(r->mu);
            r->rc = rc;
            r->msg = msg;
            r->done = true;
            r->cv.notify_all();
        }
    } else {
        readers.wait();
    }
    if (tr.on)
        fprintf(stderr, "[oxh] run: requests=%zu files=%llu slots=%d total=%.3fs submit=%.3fs drain=%.3fs readers=%d rc=%d\n",
                fs.reqs.size(), (unsigned long long)fs.files, tr.batches, Trace::now() - t_start, tr.submit,
                tr.drain, fs.nreaders, rc);
}

// The context's engine thread: one run per burst of requests.
void engine_main(oxh_ctx* c) {
    std::unique_lock<std::mutex> lk(c->qmu);
    for (;;) {
        c->qcv.wait(lk, [&] { return c->stop || !c->queue.empty(); });
        if (c->queue.empty()) return;  // stopping, nothing left
        lk.unlock();
        {
            std::lock_guard<std::mutex> g(c->mu);  // the staging slots are the run's
            run_stream(c);
        }
        lk.lock();
    }
}

}  // namespace

// A caller that has waited OXH_WAIT_LIMIT_S (default 60 s) for its request prints the engine's state
// (once per period) and keeps waiting: the engine may still write into the request.
static void dump_engine(oxh_ctx* c, const FileRequest& r) {
    std::lock_guard<std::mutex> g(c->qmu);
    fprintf(stderr, "[oxh] request stalled: n=%llu claimed=%llu remaining=%llu queue=%zu live=%d\n",
            (unsigned long long)r.n, (unsigned long long)r.next, (unsigned long long)r.remaining.load(), c->queue.size(),
            c->live != nullptr);
    // where each live context's engine thread last blocked, and which of its streams still hold work;
    // where context creation / destruction and the streaming Xxh3 last were
    fprintf(stderr, "[oxh]   this ctx %p; ctx create/destroy at \"%s\", Xxh3 stream at \"%s\"\n", (void*)c, g_life.load(),
            g_stream_where.load());
    {
        std::lock_guard<std::mutex> g(g_live_mu);
        for (oxh_ctx* x : g_live)
            fprintf(stderr, "[oxh]   ctx %p at \"%s\": stream=%s copy_stream=%s copy_stream2=%s\n", (void*)x, x->where.load(),
                    x->stream ? hipGetErrorName(hipStreamQuery(x->stream)) : "-",
                    x->copy_stream ? hipGetErrorName(hipStreamQuery(x->copy_stream)) : "-",
                    x->copy_stream2 ? hipGetErrorName(hipStreamQuery(x->copy_stream2)) : "-");
    }
    if (FileStream* fs = static_cast<FileStream*>(c->live)) {
        fprintf(stderr, "[oxh]   run: readers=%d left=%d idle=%d closing=%d abort=%d cur=%d reqs=%zu cur_req=%zu oversize=%llu changed=%llu\n",
                fs->nreaders, fs->readers_left.load(), fs->idle.load(), (int)fs->closing, (int)fs->abort.load(), fs->cur.load(),
                fs->reqs.size(), fs->cur_req, (unsigned long long)fs->n_oversize.load(), (unsigned long long)fs->n_changed.load());
        for (int k = 0; k < NSLOT; ++k) {
            const uint64_t w = fs->slot[k].word.load();
            fprintf(stderr, "[oxh]   slot %d: state=%d bytes=%llu items=%llu sealed=%d gen=%llu done=%llu\n", k,
                    fs->slot[k].state.load(), (unsigned long long)w_bytes(w), (unsigned long long)w_items(w),
                    (int)((w & kSealedBit) != 0), (unsigned long long)(w >> kGenShift), (unsigned long long)fs->slot[k].done.load());
        }
    }
}

static int hash_files_impl(oxh_ctx* c, const char* const* paths, uint64_t n, uint64_t* out, uint64_t* sizes, int32_t* status,
                           uint64_t* counts, ItemSink* sink = nullptr, int32_t* utf8 = nullptr,
                           const uint64_t* meta = nullptr, int32_t* os_error = nullptr) {
    if (!c || (n && (!paths || !out))) return fail(OXH_ERR_INVALID, "bad arguments");
    if (n == 0) return OXH_OK;
    FileRequest r;
    r.paths = paths;
    r.meta = meta;
    r.n = n;
    r.out = out;
    r.sizes = sizes;
    r.status = status;
    r.counts = counts;
    r.utf8 = utf8;
    r.os_err = os_error;
    r.sink = sink;
    r.lens.assign(n, 0);
    r.st.assign(n, OXH_OK);
    r.eno.assign(n, 0);
    r.remaining.store(n);
    {
        std::lock_guard<std::mutex> g(c->qmu);
        c->queue.push_back(&r);
        c->qcv.notify_all();  // the engine (idle) or the live run's idle readers
    }
    static const double limit = getenv("OXH_WAIT_LIMIT_S") ? atof(getenv("OXH_WAIT_LIMIT_S")) : 60.0;
    std::unique_lock<std::mutex> lk(r.mu);
    while (!r.cv.wait_for(lk, std::chrono::duration<double>(limit), [&] { return r.done; })) {
        lk.unlock();
        dump_engine(c, r);
        // No engine run and the request not queued: no thread will ever complete it (the run that held
        // it has ended and its readers are gone). An internal error, reported instead of a hang.
        bool orphaned;
        {
            std::lock_guard<std::mutex> g(c->qmu);
            orphaned = c->live == nullptr && std::find(c->queue.begin(), c->queue.end(), &r) == c->queue.end();
        }
        lk.lock();
        if (orphaned && !r.done)
            return fail(OXH_ERR_HIP, "internal error: the file engine ended its run with items of this request unfinished");
    }
    return r.rc ? fail(r.rc, r.msg) : OXH_OK;
}

int oxh_hash_files(oxh_ctx* c, const char* const* paths, uint64_t n, uint64_t* out, uint64_t* sizes, int32_t* status) {
    return hash_files_impl(c, paths, n, out, sizes, status, nullptr);
}

int oxh_hash_files_meta(oxh_ctx* c, const char* const* paths, const uint64_t* meta_sizes, uint64_t n, uint64_t* out,
                        uint64_t* sizes, int32_t* status) {
    if (n && !meta_sizes) return fail(OXH_ERR_INVALID, "meta_sizes is NULL");
    return hash_files_impl(c, paths, n, out, sizes, status, nullptr, nullptr, nullptr, meta_sizes);
}

int oxh_hash_files_text(oxh_ctx* c, const char* const* paths, uint64_t n, uint64_t* out, uint64_t* sizes, int32_t* status,
                        uint64_t* counts) {
    if (n && !counts) return fail(OXH_ERR_INVALID, "counts is NULL");
    return hash_files_impl(c, paths, n, out, sizes, status, counts);
}

int oxh_hash_files_text_utf8(oxh_ctx* c, const char* const* paths, uint64_t n, uint64_t* out, uint64_t* sizes,
                             int32_t* status, uint64_t* counts, int32_t* is_utf8) {
    if (n && (!counts || !is_utf8)) return fail(OXH_ERR_INVALID, "counts / is_utf8 is NULL");
    for (uint64_t i = 0; i < n; ++i) is_utf8[i] = 0;
    return hash_files_impl(c, paths, n, out, sizes, status, counts, nullptr, is_utf8);
}

int oxh_hash_files_ex(oxh_ctx* c, const char* const* paths, const uint64_t* meta_sizes, uint64_t n, uint64_t* out,
                      uint64_t* sizes, int32_t* status, int32_t* os_error, uint64_t* counts, int32_t* is_utf8) {
    if (is_utf8 && !counts) return fail(OXH_ERR_INVALID, "is_utf8 needs counts");
    if (is_utf8)
        for (uint64_t i = 0; i < n; ++i) is_utf8[i] = 0;
    return hash_files_impl(c, paths, n, out, sizes, status, counts, nullptr, is_utf8, meta_sizes, os_error);
}

// util::fs::classify_modified_from_node_with_metadata (util/fs.rs:1580-1619) x n: the size and mtime
// verdicts and a caller-computed metadata-hash verdict are decided on the host from what the caller's
// walk holds; every item that still needs its file read is read ONCE, all of them in ONE engine request
// (oxh_hash_files_meta semantics), with the text counts of K1T when an item's metadata is MetadataText.
int oxh_files_modified(oxh_ctx* c, const char* const* paths, const uint64_t* sizes, const uint64_t* node_bytes,
                       const uint8_t* mtime_matched, const uint64_t* node_hashes, const uint8_t* node_meta_present,
                       const uint64_t* node_meta_hashes, const uint8_t* file_meta_kind, const uint64_t* file_meta_hashes,
                       uint64_t n, uint8_t* modified, int32_t* status, uint64_t* n_hashed) {
    return oxh_files_modified_ex(c, paths, sizes, node_bytes, mtime_matched, node_hashes, node_meta_present, node_meta_hashes,
                                 file_meta_kind, file_meta_hashes, n, modified, status, nullptr, n_hashed);
}

int oxh_files_modified_ex(oxh_ctx* c, const char* const* paths, const uint64_t* sizes, const uint64_t* node_bytes,
                          const uint8_t* mtime_matched, const uint64_t* node_hashes, const uint8_t* node_meta_present,
                          const uint64_t* node_meta_hashes, const uint8_t* file_meta_kind, const uint64_t* file_meta_hashes,
                          uint64_t n, uint8_t* modified, int32_t* status, int32_t* os_error, uint64_t* n_hashed) {
    if (!c || (n && (!paths || !sizes || !node_bytes || !mtime_matched || !node_hashes || !modified)))
        return fail(OXH_ERR_INVALID, "bad arguments");
    if ((node_meta_present == nullptr) != (node_meta_hashes == nullptr))
        return fail(OXH_ERR_INVALID, "node_meta_present and node_meta_hashes go together");
    std::vector<uint64_t> idx;
    bool any_text = false;
    for (uint64_t i = 0; i < n; ++i) {
        const int kind = file_meta_kind ? file_meta_kind[i] : OXH_META_NONE;
        if (kind > OXH_META_ERROR) return fail(OXH_ERR_INVALID, "file_meta_kind out of range");
        if (kind == OXH_META_GIVEN && !file_meta_hashes) return fail(OXH_ERR_INVALID, "file_meta_hashes is NULL");
    }
    for (uint64_t i = 0; i < n; ++i) {
        modified[i] = sizes[i] != node_bytes[i] ? 1 : 0;  // fs.rs:1590-1592: no hashing needed
        if (status) status[i] = OXH_OK;
        if (os_error) os_error[i] = 0;
        if (modified[i] || mtime_matched[i]) continue;     // fs.rs:1595-1597: a matched mtime is trusted
        const int kind = file_meta_kind ? file_meta_kind[i] : OXH_META_NONE;
        const bool node_has = node_meta_present && node_meta_present[i];
        if (kind == OXH_META_ERROR) {  // fs.rs:1605-1606: the extraction's `?`
            if (status) status[i] = OXH_ERR_META;
            continue;
        }
        if (kind == OXH_META_GIVEN && node_has &&
            (file_meta_hashes[2 * i] != node_meta_hashes[2 * i] || file_meta_hashes[2 * i + 1] != node_meta_hashes[2 * i + 1])) {
            modified[i] = 1;  // fs.rs:1609-1614, before any read
            continue;
        }
        any_text |= kind == OXH_META_TEXT;
        idx.push_back(i);
    }
    if (n_hashed) *n_hashed = idx.size();
    if (idx.empty()) return OXH_OK;
    const uint64_t m = idx.size();
    std::vector<const char*> p(m);
    std::vector<uint64_t> ms(m), out(2 * m), cnt(any_text ? 2 * m : 0);
    std::vector<int32_t> st(m, OXH_OK), eno(m, 0);
    for (uint64_t k = 0; k < m; ++k) p[k] = paths[idx[k]], ms[k] = sizes[idx[k]];
    int rc = hash_files_impl(c, p.data(), m, out.data(), nullptr, st.data(), any_text ? cnt.data() : nullptr, nullptr,
                             nullptr, ms.data(), eno.data());
    if (rc) return rc;
    // MetadataText of the text items whose node has a metadata hash: serde_json of GenericMetadata
    // (model/metadata/generic_metadata.rs, untagged; MetadataText's field order) hashed in one batch
    std::vector<uint64_t> tk, toff, tlen;
    std::string json;
    for (uint64_t k = 0; k < m; ++k) {
        const uint64_t i = idx[k];
        if (st[k] != OXH_OK || !file_meta_kind || file_meta_kind[i] != OXH_META_TEXT) continue;
        if (!(node_meta_present && node_meta_present[i])) continue;  // None on the node side: no comparison
        char buf[96];
        const int len = snprintf(buf, sizeof buf, "{\"text\":{\"num_lines\":%llu,\"num_chars\":%llu}}",
                                 (unsigned long long)cnt[2 * k], (unsigned long long)cnt[2 * k + 1]);
        tk.push_back(k), toff.push_back(json.size()), tlen.push_back((uint64_t)len);
        json.append(buf, (size_t)len);
    }
    std::vector<uint64_t> mh(2 * tk.size());
    if (!tk.empty()) {
        rc = oxh_hash_streams(c, (const uint8_t*)json.data(), toff.data(), tlen.data(), tk.size(), mh.data());
        if (rc) return rc;
    }
    std::vector<uint8_t> meta_differs(m, 0);
    for (size_t j = 0; j < tk.size(); ++j) {
        const uint64_t i = idx[tk[j]];
        meta_differs[tk[j]] = mh[2 * j] != node_meta_hashes[2 * i] || mh[2 * j + 1] != node_meta_hashes[2 * i + 1];
    }
    for (uint64_t k = 0; k < m; ++k) {
        const uint64_t i = idx[k];
        if (st[k] != OXH_OK) {  // the reference returns the open / read error for this path
            if (status) status[i] = st[k];
            if (os_error) os_error[i] = eno[k];
            continue;
        }
        if (meta_differs[k]) {  // fs.rs:1609-1614
            modified[i] = 1;
            continue;
        }
        // fs.rs:1616-1618: node.hash() against get_hash_given_metadata(path, metadata)
        modified[i] = (out[2 * k] != node_hashes[2 * i] || out[2 * k + 1] != node_hashes[2 * i + 1]) ? 1 : 0;
    }
    return OXH_OK;
}

namespace {

// mkdir -p (std::fs::create_dir_all)
bool mkdir_p(const std::string& dir) {
    if (mkdir(dir.c_str(), 0755) == 0 || errno == EEXIST) return true;
    if (errno != ENOENT) return false;
    for (size_t i = 1; i <= dir.size(); ++i)
        if (i == dir.size() || dir[i] == '/') {
            const std::string part = dir.substr(0, i);
            if (mkdir(part.c_str(), 0755) != 0 && errno != EEXIST) return false;
        }
    return true;
}

// A new temp file `{dir}/data.oxentmp.<random>` (AtomicTempFile's `<target_basename>.oxentmp.<random>`,
// util/fs/atomic_file.rs:21-25,58-96, so liboxen's leftover handling recognises it); -1 on failure.
int make_temp(const std::string& dir, std::string& tmp) {
    static const char an[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789";
    thread_local uint64_t x = [] {
        std::random_device rd;
        return ((uint64_t)rd() << 32) ^ rd() ^ (uint64_t)std::hash<std::thread::id>()(std::this_thread::get_id());
    }();
    for (int attempt = 0; attempt < 32; ++attempt) {
        tmp = dir + "/data.oxentmp.";
        for (int k = 0; k < 8; ++k) {  // splitmix64 steps
            uint64_t z = (x += 0x9E3779B97F4A7C15ull);
            z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
            z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
            tmp += an[(z ^ (z >> 31)) % 62];
        }
        const int fd = open(tmp.c_str(), O_RDWR | O_CREAT | O_EXCL | O_CLOEXEC, 0644);
        if (fd >= 0 || errno != EEXIST) return fd;
    }
    return -1;
}

// The version-store half of the fused add: LocalVersionStore::store_version_from_reader
// (storage/local.rs:104-121) publishing through AtomicTempFile (util/fs/atomic_file.rs:54-159) --
// write a `data.oxentmp.<random>` sibling, make the data durable, rename it to
// {root}/{hex[..2]}/{hex[2..]}/data (local.rs:66-75), make the rename durable; a blob already in the
// store is not rewritten (local.rs:112). AtomicTempFile::commit fsyncs each file and its parent; here
// one syncfs() covers every temp of a drained slot before any of them is renamed, and a second one
// covers the renames -- the same ordering, two barriers per slot instead of two per file.
// The barriers run on a committer thread: commit() hands the slot's temps over and returns, so the
// engine reads, hashes and writes the next slots while the disk takes the last ones (a committer
// that falls behind takes every queued slot under one pair of barriers). wait() returns once every
// handed-over temp is published; oxh_add_files calls it before it reads the outcomes.
// OXH_PUBLISH_INLINE=1 publishes inside commit() instead (the r02 form, for A/B).
// OXH_PUBLISH_SYNC=fsync replaces the two syncfs barriers with the reference's own per-blob steps
// (fsync the temp, rename, fsync its parent), run by the committer's threads: for filesystems where
// syncfs is costly (one shared with other tenants' dirty data).
// Identical content twice in one call is published once; every duplicate shares that publish's
// outcome (finish()).
class VersionPublisher final : public ItemSink {
   public:
    VersionPublisher(oxh_ctx* c, std::string root, uint64_t n)
        : c_(c), root_(std::move(root)), owner_(n, kNone), result_(n, 0),
          inline_(env_flag("OXH_PUBLISH_INLINE")),
          fsync_each_(getenv("OXH_PUBLISH_SYNC") && !strcmp(getenv("OXH_PUBLISH_SYNC"), "fsync")) {}
    ~VersionPublisher() override {
        {
            std::lock_guard<std::mutex> g(cq_mu_);
            quit_ = true;
        }
        cq_cv_.notify_all();
        if (committer_.joinable()) committer_.join();  // publishes whatever is still queued first
        if (trace_)
            fprintf(stderr, "[oxh] publish: put=%.3fs (thread time) publish=%.3fs batches=%d wait=%.3fs inline=%d fsync=%d\n",
                    put_s_.load() * 1e-9, publish_s_ * 1e-9, nbatches_, wait_s_ * 1e-9, (int)inline_, (int)fsync_each_);
        delete rpool_;
        if (root_fd_ >= 0) close(root_fd_);
    }

    void put(uint64_t id, const uint8_t* bytes, uint64_t len, uint64_t lo, uint64_t hi) override {
        const Clock t0(trace_);
        put_impl(id, bytes, len, lo, hi);
        put_s_.fetch_add(t0.ns(), std::memory_order_relaxed);
    }
    void put_impl(uint64_t id, const uint8_t* bytes, uint64_t len, uint64_t lo, uint64_t hi) {
        if (!claim(id, lo, hi)) return;
        std::string dir, path;
        target(lo, hi, dir, path);
        struct stat sb;
        if (stat(path.c_str(), &sb) == 0) {
            result_[id] = kExisted;
            return;
        }
        std::string tmp;
        const int fd = mkdir_p(dir) ? make_temp(dir, tmp) : -1;
        if (fd < 0) {
            result_[id] = kFailed;
            return;
        }
        bool ok = true;
        for (uint64_t done = 0; ok && done < len;) {
            const ssize_t w = write(fd, bytes + done, len - done);
            if (w <= 0) ok = false;
            else done += (uint64_t)w;
        }
        if (close(fd) != 0) ok = false;
        if (!ok) {
            unlink(tmp.c_str());
            result_[id] = kFailed;
            return;
        }
        stage(id, tmp, path);
    }

    // a streamed file's temp lives in the root until its digest names the target directory
    int open_stream(uint64_t, std::string& tmp) override { return mkdir_p(root_) ? make_temp(root_, tmp) : -1; }

    void close_stream(uint64_t id, int fd, const std::string& tmp, bool ok, uint64_t lo, uint64_t hi) override {
        if (fd >= 0 && close(fd) != 0) ok = false;
        if (!ok || fd < 0) {
            if (!tmp.empty()) unlink(tmp.c_str());
            owner_[id] = id;
            result_[id] = kFailed;
            return;
        }
        if (!claim(id, lo, hi)) {
            unlink(tmp.c_str());
            return;
        }
        std::string dir, path;
        target(lo, hi, dir, path);
        struct stat sb;
        if (stat(path.c_str(), &sb) == 0) {
            unlink(tmp.c_str());
            result_[id] = kExisted;
        } else if (!mkdir_p(dir)) {
            unlink(tmp.c_str());
            result_[id] = kFailed;
        } else {
            stage(id, tmp, path);
        }
    }

    void commit() override {
        std::vector<Staged> batch;
        {
            std::lock_guard<std::mutex> g(mu_);
            batch.swap(staged_);
        }
        if (batch.empty()) return;
        if (inline_) {
            publish(batch);
            return;
        }
        {
            std::lock_guard<std::mutex> g(cq_mu_);
            cq_.push_back(std::move(batch));
            if (!committer_.joinable()) committer_ = std::thread([this] { committer(); });
        }
        cq_cv_.notify_all();
    }

    // every temp handed to commit() so far is published (or failed)
    void wait() {
        const Clock t0(trace_);
        std::unique_lock<std::mutex> g(cq_mu_);
        cq_cv_.wait(g, [&] { return cq_.empty() && !publishing_; });
        wait_s_ += t0.ns();
    }

    // Per-item outcome into the caller's arrays: a file whose content failed to publish (its own
    // publish or the one its duplicate claimed) fails with OXH_ERR_IO and digest 0, like the
    // reference's add of that file (add.rs:533-544).
    void finish(uint64_t n, uint64_t* out, int32_t* status, int32_t* stored) const {
        for (uint64_t i = 0; i < n; ++i) {
            stored[i] = 0;
            if (status[i] != OXH_OK) continue;
            const uint64_t o = owner_[i];
            if (o == kNone || result_[o] == kFailed) {
                status[i] = OXH_ERR_IO;
                out[2 * i] = out[2 * i + 1] = 0;
                continue;
            }
            stored[i] = (o == i && result_[o] == kWritten) ? 1 : 0;
        }
    }

   private:
    static constexpr uint64_t kNone = ~0ull;
    static constexpr int8_t kExisted = 0, kWritten = 1, kFailed = -1;
    struct Staged {
        uint64_t id;
        std::string tmp, path;
    };
    struct Clock {  // OXH_TRACE: wall time of a section, 0 when tracing is off
        std::chrono::steady_clock::time_point t;
        bool on;
        explicit Clock(bool o) : on(o) {
            if (on) t = std::chrono::steady_clock::now();
        }
        uint64_t ns() const {
            return on ? (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t).count() : 0;
        }
    };
    static bool env_flag(const char* name) {
        const char* e = getenv(name);
        return e && atoi(e) != 0;
    }

    void committer() {
        std::unique_lock<std::mutex> g(cq_mu_);
        for (;;) {
            cq_cv_.wait(g, [&] { return quit_ || !cq_.empty(); });
            if (cq_.empty()) return;  // quit, nothing left
            std::vector<Staged> batch = std::move(cq_.front());
            for (size_t k = 1; k < cq_.size(); ++k)
                for (Staged& st : cq_[k]) batch.push_back(std::move(st));
            cq_.clear();
            publishing_ = true;
            g.unlock();
            publish(batch);
            g.lock();
            publishing_ = false;
            cq_cv_.notify_all();
        }
    }

    void publish(std::vector<Staged>& batch) {
        const Clock t0(trace_);
        publish_impl(batch);
        publish_s_ += t0.ns();
        ++nbatches_;
    }
    void publish_impl(std::vector<Staged>& batch) {
        // 1. the data of every temp is durable before any rename (AtomicTempFile::commit's sync_all,
        //    atomic_file.rs:122); should syncfs fail, each temp is fsynced on its own
        const bool synced = !fsync_each_ && sync_fs();
        auto each = [&](const std::function<void(Staged&)>& fn) {
            if (batch.size() < 64) {
                for (Staged& s : batch) fn(s);
                return;
            }
            if (!rpool_) rpool_ = new oxh::Pool(c_->pool->size());  // the publisher's own: wpool may be busy with put()
            const int ntasks = (int)std::min<size_t>(batch.size(), (size_t)rpool_->size() * 4);
            rpool_->parallel_for(ntasks, [&](int t) {
                for (size_t k = (size_t)t; k < batch.size(); k += (size_t)ntasks) fn(batch[k]);
            });
        };
        each([&](Staged& s) {
            bool ok = true;
            if (!synced) {
                const int fd = open(s.tmp.c_str(), O_RDONLY | O_CLOEXEC);
                ok = fd >= 0 && fsync(fd) == 0;
                if (fd >= 0) close(fd);
            }
            // 2. publish (atomic_file.rs:132-139): a failed rename removes the temp
            if (ok && rename(s.tmp.c_str(), s.path.c_str()) == 0) {
                result_[s.id] = kWritten;
                if (fsync_each_) {  // 3. the rename, best effort: the parent's fsync (:141-156)
                    const int dfd = open(s.path.substr(0, s.path.rfind('/')).c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
                    if (dfd >= 0) {
                        (void)fsync(dfd);
                        close(dfd);
                    }
                }
            } else {
                unlink(s.tmp.c_str());
                result_[s.id] = kFailed;
            }
        });
        // 3. the renames themselves, best effort like the reference's parent fsync (:141-156)
        if (!fsync_each_) (void)sync_fs();
    }

    // the first item with this digest publishes it; the others share its outcome
    bool claim(uint64_t id, uint64_t lo, uint64_t hi) {
        std::lock_guard<std::mutex> g(mu_);
        const auto it = owner_of_.emplace(std::make_pair(lo, hi), id).first;
        owner_[id] = it->second;
        return it->second == id;
    }
    void target(uint64_t lo, uint64_t hi, std::string& dir, std::string& path) const {
        char hex[40];
        const int hl = oxh_format_hex(lo, hi, hex);
        const int p = std::min(hl, 2);
        dir = root_ + "/" + std::string(hex, p) + "/" + std::string(hex + p);
        path = dir + "/data";
    }
    void stage(uint64_t id, const std::string& tmp, const std::string& path) {
        std::lock_guard<std::mutex> g(mu_);
        staged_.push_back({id, tmp, path});
    }
    bool sync_fs() {
        if (root_fd_ < 0) root_fd_ = open(root_.c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
        return root_fd_ >= 0 && syncfs(root_fd_) == 0;
    }

    oxh_ctx* c_;
    std::string root_;
    std::mutex mu_;
    std::map<std::pair<uint64_t, uint64_t>, uint64_t> owner_of_;
    std::vector<uint64_t> owner_;  // per item: the item that publishes its content (itself if first)
    std::vector<int8_t> result_;   // per publishing item: kWritten / kExisted / kFailed
    std::vector<Staged> staged_;   // temps written, waiting for commit()
    int root_fd_ = -1;             // the committer's only (syncfs)
    const bool inline_, fsync_each_;
    std::mutex cq_mu_;
    std::condition_variable cq_cv_;
    std::vector<std::vector<Staged>> cq_;  // committed slots waiting for the committer
    bool publishing_ = false, quit_ = false;
    std::thread committer_;
    oxh::Pool* rpool_ = nullptr;  // renames / fallback fsyncs
    const bool trace_ = getenv("OXH_TRACE") != nullptr;
    std::atomic<uint64_t> put_s_{0};
    uint64_t publish_s_ = 0, wait_s_ = 0;  // committer thread / owner thread
    int nbatches_ = 0;
};

}  // namespace

int oxh_add_files(oxh_ctx* c, const char* const* paths, uint64_t n, const char* versions_root, uint64_t* out,
                  uint64_t* sizes, int32_t* status, int32_t* stored) {
    return oxh_add_files_ex(c, paths, n, versions_root, out, sizes, status, stored, nullptr);
}

int oxh_add_files_ex(oxh_ctx* c, const char* const* paths, uint64_t n, const char* versions_root, uint64_t* out,
                     uint64_t* sizes, int32_t* status, int32_t* stored, int32_t* os_error) {
    if (n && (!versions_root || !stored || !status)) return fail(OXH_ERR_INVALID, "versions_root/status/stored is NULL");
    for (uint64_t i = 0; i < n; ++i) stored[i] = 0;
    VersionPublisher pub(c, versions_root ? versions_root : "", n);
    const int rc = hash_files_impl(c, paths, n, out, sizes, status, nullptr, &pub, nullptr, nullptr, os_error);
    if (rc) return rc;
    pub.wait();
    pub.finish(n, out, status, stored);
    return OXH_OK;
}

static int remove_tree_cb(const char* p, const struct stat*, int, struct FTW*) { return remove(p); }

// std::fs::remove_dir_all: depth-first, does not follow symlinks.
static bool remove_dir_all(const std::string& dir) {
    return nftw(dir.c_str(), remove_tree_cb, 64, FTW_DEPTH | FTW_PHYS) == 0;
}

int oxh_clean_corrupted_versions(oxh_ctx* c, const char* versions_root, int dry_run, uint64_t* result) {
    if (!c || !versions_root || !result) return fail(OXH_ERR_INVALID, "bad arguments");
    uint64_t errors = 0, scanned = 0, corrupted = 0, cleaned = 0;
    // prefix dirs (local.rs:461-474): anything that is not a directory counts as an error
    // 1 = directory, 0 = not, -1 = file_type() failed (an error in the reference's counts)
    auto is_dir = [](const std::string& path, unsigned char d_type) {
        if (d_type != DT_UNKNOWN) return d_type == DT_DIR ? 1 : 0;  // readdir's type, like DirEntry::file_type
        struct stat sb;
        if (lstat(path.c_str(), &sb) != 0) return -1;
        return S_ISDIR(sb.st_mode) ? 1 : 0;
    };
    std::vector<std::string> prefixes;
    {
        DIR* d = opendir(versions_root);
        if (!d) return fail(OXH_ERR_IO, std::string("cannot read ") + versions_root);
        while (struct dirent* e = readdir(d)) {
            if (!strcmp(e->d_name, ".") || !strcmp(e->d_name, "..")) continue;
            if (is_dir(std::string(versions_root) + "/" + e->d_name, e->d_type) == 1)
                prefixes.push_back(e->d_name);
            else
                ++errors;
        }
        closedir(d);
    }
    std::sort(prefixes.begin(), prefixes.end());
    // suffix dirs (local.rs:480-518), one task per prefix as in the reference: non-directories are
    // skipped; expected hash = prefix + suffix
    struct Found {
        std::vector<std::string> dirs, expected;
        uint64_t errors = 0;
    };
    std::vector<Found> found(prefixes.size());
    c->pool->parallel_for((int)prefixes.size(), [&](int t) {
        const std::string pdir = std::string(versions_root) + "/" + prefixes[t];
        DIR* d = opendir(pdir.c_str());
        if (!d) {
            ++found[t].errors;
            return;
        }
        while (struct dirent* e = readdir(d)) {
            if (!strcmp(e->d_name, ".") || !strcmp(e->d_name, "..")) continue;
            std::string sdir = pdir + "/" + e->d_name;
            const int k = is_dir(sdir, e->d_type);
            if (k < 0) ++found[t].errors;
            if (k != 1) continue;
            found[t].dirs.push_back(std::move(sdir));
            found[t].expected.push_back(prefixes[t] + e->d_name);
        }
        closedir(d);
    });
    std::vector<std::string> dirs, expected, data;
    for (Found& f : found) {
        errors += f.errors;
        for (size_t k = 0; k < f.dirs.size(); ++k) {
            data.push_back(f.dirs[k] + "/data");
            dirs.push_back(std::move(f.dirs[k]));
            expected.push_back(std::move(f.expected[k]));
        }
    }
    const uint64_t n = dirs.size();
    std::vector<const char*> paths(n);
    for (uint64_t i = 0; i < n; ++i) paths[i] = data[i].c_str();
    std::vector<uint64_t> out(2 * n), sizes(n);
    std::vector<int32_t> status(n);
    const int rc = hash_files_impl(c, paths.data(), n, out.data(), sizes.data(), status.data(), nullptr);
    if (rc) return rc;
    for (uint64_t i = 0; i < n; ++i) {
        bool remove_it = false;
        if (status[i] != OXH_OK) {  // fs::read failed: an error, not scanned (local.rs:527-537)
            ++errors;
            remove_it = !dry_run;
            if (remove_it && remove_dir_all(dirs[i])) ++cleaned;
            continue;
        }
        ++scanned;
        char hex[40];
        const int hl = oxh_format_hex(out[2 * i], out[2 * i + 1], hex);
        if (expected[i].size() == (size_t)hl && memcmp(expected[i].data(), hex, hl) == 0) continue;
        ++corrupted;  // local.rs:561-581
        if (!dry_run) {
            if (remove_dir_all(dirs[i]))
                ++cleaned;
            else
                ++errors;
        }
    }
    result[0] = scanned;
    result[1] = corrupted;
    result[2] = cleaned;
    result[3] = errors;
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
