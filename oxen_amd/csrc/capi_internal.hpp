// oxen_amd/csrc/capi_internal.hpp -- what the translation units of the C ABI runtime share
// (include/oxen_hash.h is the public side). Not installed; no caller outside oxen_amd/csrc includes it.
//
// The runtime replaces the per-file hashing inside liboxen's add loop
// (core/v_latest/add.rs:444-545 -> util/hasher.rs:56-65) with batched device work. Its pieces:
//   capi_dispatch.hip  K1 launch shapes and the device-resident entries (HBM in, HBM out)
//   capi_context.hip   oxh_ctx: streams, pinned/device staging slots, reader pools, lifetime
//   staging.hip        host-buffer batches through the staging slots (oxh_hash_buffers / _streams)
//   large_items.hip    items larger than a slot: device pieces, K1L block sums + serial chains
//   xxh3_stream.hip    the streaming Xxh3 (update / digest128) over K1L pieces
//   engine.hip         the streaming file engine behind every file call (oxh_hash_files*)
//   modified.hip       util::fs modified checks over one engine request (oxh_files_modified*)
//   publish.hip        the fused add's version-store publisher and the fsck (oxh_add_files*, clean)
// There is no CPU hashing path: every digest this library returns was computed on the GPU.
#pragma once

#include <hip/hip_runtime.h>
#include <dirent.h>
#include <errno.h>
#include <fcntl.h>
#include <sched.h>
#include <stdint.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/resource.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <array>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/oxen_hash.h"
#include "pool.hpp"
#include "scratch.hpp"
#include "xxh3_device.hpp"

// ---------------------------------------------------------------- kernels (xxh3_kernels.hip)
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
__global__ void text_count_finish_kernel(const unsigned long long*, CountFix, uint64_t*);
__global__ void utf8_prefix_kernel(const uint8_t*, const uint64_t*, const uint64_t*, uint64_t, int32_t*);
__global__ void fill_splitmix_tail_kernel(uint8_t*, uint64_t, uint64_t, uint64_t);
}  // namespace oxh

struct FileRequest;  // one file call on the engine's queue (engine.hip)

namespace oxh::capi {

// ---------------------------------------------------------------- errors (capi_dispatch.hip)
extern thread_local std::string g_err;  // oxh_last_error()
extern std::atomic<int> g_variant;      // oxh_set_kernel_variant()
int fail(int code, const std::string& msg);

#define HIP_TRY(expr)                                                                      \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess)                                                              \
            return ::oxh::capi::fail(OXH_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));  \
    } while (0)

// OXH_DEBUG_STEPS=1: one stderr line per runtime step (locating stalls without a debugger)
inline const bool g_steps = getenv("OXH_DEBUG_STEPS") != nullptr;
#define STEP(...)                                  \
    do {                                           \
        if (::oxh::capi::g_steps) {                \
            fprintf(stderr, "[oxh-step] " __VA_ARGS__); \
            fputc('\n', stderr);                   \
        }                                          \
    } while (0)

constexpr uint64_t kAlign = 256;
constexpr int NSLOT = 3;
inline uint64_t align_up(uint64_t x) { return (x + kAlign - 1) & ~(kAlign - 1); }

// ---------------------------------------------------------------- K1 launches (capi_dispatch.hip)
// K1 register/pipeline shape by item size (the measurements are at the definitions)
constexpr uint64_t kShortItemBytes = 16384;
constexpr int kVariantShort = 72;    // Cfg: row-wise, depth 2, keys in LDS
constexpr int kVariantLong = 8;      // Cfg: row-wise, depth 2, keys from the constant table
constexpr int kVariantPacked = 104;  // Cfg: block-wise, depth 2, keys in LDS
constexpr int kVariantRows = 264;    // Cfg: K1R (a 16-lane row per item), depth 2

enum class ItemShape { Long, Short, Packed };

// K1 over a descriptor table: one 64-lane wave per item, 4 waves per 256-thread workgroup.
int launch_wave(const uint8_t* arena, const uint64_t* offs, const uint64_t* lens, uint64_t n, uint64_t* out,
                hipStream_t st, ItemShape shape = ItemShape::Long, int waves = 4, int variant = 0);
// K1T: K1 plus text counts in the same pass.
int launch_text(const uint8_t* arena, const uint64_t* offs, const uint64_t* lens, uint64_t n, uint64_t* out,
                uint64_t* counts, hipStream_t st, bool short_items = false);
// Fixed-size chunks of one buffer (no descriptor table): chunk i = [i*chunk, min((i+1)*chunk, total)).
int launch_chunks(const uint8_t* buf, uint64_t n, uint64_t chunk, uint64_t total, uint64_t* out, hipStream_t st);
int launch_lane(const uint8_t* arena, const uint64_t* offs, const uint64_t* lens, uint64_t n, uint64_t* out,
                hipStream_t st);

// ---------------------------------------------------------------- host resources (capi_context.hip)
int usable_cpus();
int default_threads();
int check_device(int device);

}  // namespace oxh::capi

// ---------------------------------------------------------------- context
struct oxh_ctx {
    int device = 0;
    hipStream_t stream = nullptr, copy_stream = nullptr;
    hipStream_t copy_stream2 = nullptr;  // large items: every other bounce window's H2D (created on first use)
    hipEvent_t ev_copy2_join = nullptr;  // copy_stream waits for copy_stream2's windows of a piece
    std::atomic<const char*> where{"-"};  // where the engine / large-item path last blocked (stall reports)
    uint64_t stage_bytes = 0, max_items = 0;
    uint8_t* h_stage[oxh::capi::NSLOT] = {};
    uint8_t* d_stage[oxh::capi::NSLOT] = {};
    uint64_t* h_desc[oxh::capi::NSLOT] = {};  // [offsets(max_items) | lens(max_items)]
    uint64_t* d_desc[oxh::capi::NSLOT] = {};
    uint64_t* h_out[oxh::capi::NSLOT] = {};
    uint64_t* d_out[oxh::capi::NSLOT] = {};
    uint64_t* h_cnt[oxh::capi::NSLOT] = {};  // text counts (num_lines, num_chars) per item, K1T
    uint64_t* d_cnt[oxh::capi::NSLOT] = {};
    int32_t* h_utf8[oxh::capi::NSLOT] = {};  // is_utf8 of each item's first 4 KiB (util/fs.rs:652-668)
    int32_t* d_utf8[oxh::capi::NSLOT] = {};
    // a slot's large items on K1L (submit_slot): the lens the K1 wave launch sees (those items zeroed),
    // and their block sums (8 u64 per KiB: at most a sixteenth of the slot), then kSlotCountRaw u64 of
    // raw text counts (K1T batches)
    uint64_t* h_klen[oxh::capi::NSLOT] = {};
    uint64_t* d_klen[oxh::capi::NSLOT] = {};
    uint64_t* d_sums[oxh::capi::NSLOT] = {};
    // streaming file engine (engine.hip): file calls queue requests here; the engine thread runs
    // them, and requests arriving while it runs join the live pipeline
    std::mutex qmu;
    std::condition_variable qcv;  // a request was queued (or the engine must stop)
    std::vector<FileRequest*> queue;
    bool stop = false;
    std::thread engine;
    uint64_t flush_bytes = 0;  // seal a partly filled slot at this many bytes when the next slot is free
    // files larger than a staging slot (large_items.hip): device piece buffers sized for a full batch
    // of large files, and pinned bounce buffers the files are read into in windows
    uint8_t* d_big = nullptr;
    uint64_t d_big_size = 0;
    uint64_t d_big_allocs = 0;   // times d_big was (re)allocated (oxh_ctx_counters)
    std::atomic<uint64_t> n_direct{0}, n_runs{0};  // file requests on the caller's thread / engine runs
    uint8_t* h_bounce[8] = {};   // kNBounce pinned bounce buffers, used as a ring
    hipEvent_t ev_bounce[8] = {};
    bool bounce_used[8] = {};
    uint64_t bounce_next = 0;    // the ring position (kept across pieces and files)
    hipEvent_t ev_piece_free[2] = {};
    void* live = nullptr;  // the engine's current run (a FileStream, for diagnostics), under qmu
    std::vector<FileRequest*> rq[oxh::capi::NSLOT];  // per staged item: its request and index in it
    std::vector<uint64_t> loc[oxh::capi::NSLOT];
    hipEvent_t ev_copied[oxh::capi::NSLOT] = {}, ev_done[oxh::capi::NSLOT] = {};
    oxh::Pool* pool = nullptr;   // readers / copiers (fill)
    oxh::Pool* wpool = nullptr;  // consumers of hashed bytes (fused publish), created on first use
    oxh::Pool* rpool = nullptr;  // streaming-pipeline file readers (stream_files)
    std::mutex mu;
    void* cdc = nullptr;                 // FastCDC host pipeline (fastcdc_host.cpp), created on first use
    void (*cdc_free)(void*) = nullptr;
};

namespace oxh::capi {

// Stall reports (engine.hip dump_engine): the live contexts, and where context creation /
// destruction and the streaming Xxh3 last were -- the threads that call those are not engine threads.
extern std::mutex g_live_mu;
extern std::vector<oxh_ctx*> g_live;
extern std::atomic<const char*> g_life, g_stream_where;

void engine_main(oxh_ctx* c);  // the streaming file engine's thread (engine.hip)

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

// ---------------------------------------------------------------- staging slots (staging.hip)
struct Pending {
    bool busy = false;
    std::vector<uint64_t> ids;  // caller indices of the staged items
};

// One staged batch: items [0, cnt) already in h_stage[s] at h_desc offsets; launch and queue D2H.
int submit_slot(oxh_ctx* c, int s, uint64_t bytes, uint64_t cnt, bool any_short_only, bool short_items, bool text,
                bool utf8 = false);
// A small batch of items below kSlotChainBytes with its descriptors packed after its bytes: one H2D on the
// compute stream (engine.hip direct_files). `done` false: not taken (does not fit, or disabled).
int submit_packed(oxh_ctx* c, int s, uint64_t bytes, uint64_t cnt, bool short_items, bool text, bool utf8, bool& done,
                  bool lane = false);
// Wait for slot s's digests (bounded by OXH_WAIT_LIMIT_S, which reports the stalled stage).
int wait_slot(oxh_ctx* c, int s, const Pending& p);
// Scatter slot s's digests to the caller's table (host-buffer batches: oxh_hash_buffers/_streams).
int drain_slot(oxh_ctx* c, int s, Pending& p, uint64_t* out);

// ---------------------------------------------------------------- large items (large_items.hip)
// The chain kernel is VALU-issue-bound per wave, so two chains on one SIMD run at half speed each.
// Unused dynamic LDS on top of the kernel's 32 KiB makes every chain workgroup need more than half a
// CU's 160 KiB: one chain per CU.
constexpr size_t kChainLdsPad = 50 * 1024;
// Items of a staged batch at least this long (the kChainJobs largest) take K1L instead of a K1 wave
// (submit_slot). OXH_SLOT_CHAINS=0: every item on a wave (the r01-r06 form, for A/B).
constexpr uint64_t kSlotChainBytes = 1ull << 20;
constexpr uint64_t kSlotCountRaw = 2 * oxh::kChainJobs;
inline uint64_t slot_sums_words(uint64_t stage_bytes) { return ((stage_bytes >> 10) + 1) * 8; }
constexpr uint64_t kBounce = 64ull << 20, kBigRead = 4ull << 20;
constexpr int kNBounce = 8;  // bounce buffers in the ring: up to 7 windows read while earlier H2Ds drain

// K1L over n device buffers (pieces of OXH_BIG_PIECE_MIB, block sums chip-wide + serial chains);
// returns after `st` has finished.
int large_batch_device(const uint8_t* const* bufs, const uint64_t* lens, uint64_t n, uint64_t* d_out, hipStream_t st);
int large_device(oxh_ctx*, const uint8_t* d_buf, uint64_t len, uint64_t* d_out, hipStream_t st);
// Digest (+ text counts, + is_utf8) of one buffer already on the device; synchronises c->stream.
int device_item(oxh_ctx* c, uint8_t* d, uint64_t len, uint64_t* out2, uint64_t* cnt2, int32_t* utf8_1);
// One oversize host item through a device buffer of its own.
int oversize_item(oxh_ctx* c, const uint8_t* src, uint64_t len, uint64_t* out2, uint64_t* cnt2 = nullptr,
                  int32_t* utf8_1 = nullptr);

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

// Files up to this many at a time share one large-item pipeline (OXH_BIG_FILES, default 4).
int big_files_at_once();
// Hash n (<= kChainJobs) large items side by side; run-level errors only for HIP failures, each
// item's own outcome in its res.
int large_items(oxh_ctx* c, LargeJob* jobs, int n);
// One large item (host buffers of oxh_hash_buffers / _streams, and the single-file case).
int large_item(oxh_ctx* c, uint64_t L, LargeSource& src, bool want_counts, bool want_utf8, ItemSink* sink, uint64_t id,
               LargeResult& res);

// ---------------------------------------------------------------- file engine (engine.hip)
// One file request through the context's engine: returns once every item is hashed (and handed to
// `sink`), outputs in place; per-item statuses in `status` / `os_error`.
int hash_files_impl(oxh_ctx* c, const char* const* paths, uint64_t n, uint64_t* out, uint64_t* sizes, int32_t* status,
                    uint64_t* counts, ItemSink* sink = nullptr, int32_t* utf8 = nullptr,
                    const uint64_t* meta = nullptr, int32_t* os_error = nullptr);

}  // namespace oxh::capi
