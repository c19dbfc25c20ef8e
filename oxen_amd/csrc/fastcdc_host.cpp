// oxen_amd/csrc/fastcdc_host.cpp -- FastCDC chunking that starts and ends in host memory
// (include/oxen_hash.h: oxh_fastcdc_files, oxh_fastcdc_host).
//
// The reference chunker reads a whole file into memory (`fs::read(input_file)`,
// experiments/block-level-dedup/src/chunker/fastcdchunker.rs:75), runs fastcdc v2020 over it (:83-88)
// and hashes every chunk with xxh3_128 (:95-98). Here the bytes go through a bounded pipeline instead:
//
//   readers (pool threads, pread / memcpy)  ->  pinned bounce ring (4 x 64 MiB)  --H2D, copy stream-->
//   device piece buffer b (2 x 1 GiB)  --oxh_fastcdc_device on the compute stream: W + X (or F1-F3),
//   then K1R over the chunks-->  chunk table + digests  --D2H-->  the caller's arrays
//
// Files are taken in order and packed into pieces; a file larger than what is left of a piece is
// cut into segments. A chunk's cut depends only on its start and on the `max` bytes after it
// (cut_gear scans at most `max` bytes, and the hash restarts at every chunk start), so a chunk of a
// segment that starts at s with s + max <= segment end is exactly the crate's chunk; the first chunk
// that is not is the CARRY, the exact start the file's next segment is chunked from. The next segment
// is read from `max` bytes before the previous segment's end (the carry always lies in that tail), so
// its bytes can be uploaded before the previous segment is chunked; the device call then starts the
// segment's chunking at the carry. Two piece buffers let round r+1's reads and copies run while
// round r is chunked on a worker thread.
#include <hip/hip_runtime_api.h>
#include <errno.h>
#include <fcntl.h>
#include <dirent.h>
#include <string.h>
#include <sys/resource.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/oxen_hash.h"
#include "pool.hpp"

namespace oxh {
int set_error(int code, const std::string& msg);            // capi_context.hip
int ctx_device(oxh_ctx* c);                                 // capi_context.hip
std::mutex& ctx_call_mutex(oxh_ctx* c);                     // ... serialises a context's non-engine calls
void*& ctx_cdc_state(oxh_ctx* c, void (*deleter)(void*));   // ... a slot the context frees on destroy
int default_reader_threads();                               // ... OXH_NUM_THREADS / the CPU quota, <= 16
}  // namespace oxh

namespace {

constexpr int kCdcMaxBounce = 16;
// one pinned bounce buffer (a window of the piece): OXH_CDC_BOUNCE_MIB, 16..256 (a power of two),
// default 64
uint64_t cdc_bounce() {
    static const uint64_t v = [] {
        const char* e = getenv("OXH_CDC_BOUNCE_MIB");
        const long k = e ? atol(e) : 64;
        uint64_t m = 16;
        while (m < 256 && (long)m < k) m <<= 1;
        return m << 20;
    }();
    return v;
}
// the ring: reads of the next windows run while earlier H2Ds drain (OXH_CDC_NBOUNCE, 2..16, default 8:
// 47.7 vs 43.6 GiB/s for 4 on 16 x 1 GiB from the page cache, profiles/r05/r05a_e2e_*)
// H2D copy streams the windows alternate over (OXH_CDC_COPY_STREAMS, 1 or 2; default 2: C5 from the
// page cache 2.57-2.64 s against 2.91-2.92 s with one, alternating on one box, profiles/r05/r05e_shm_cs*)
int cdc_copy_streams() {
    static const int v = [] {
        const char* e = getenv("OXH_CDC_COPY_STREAMS");
        return e && atoi(e) == 1 ? 1 : 2;
    }();
    return v;
}
// Fixed-size rounds of at most this many segments hash each segment as one implied chunk grid
// (oxh_chunk_digests_device: no descriptor tables built on the host or copied over the link); more
// segments (many small files) take one launch over descriptors. OXH_FIXED_IMPLICIT_SEGS, 0 = always
// descriptors.
int fixed_implicit_segs() {
    static const int v = [] {
        const char* e = getenv("OXH_FIXED_IMPLICIT_SEGS");
        return e ? std::max(0, atoi(e)) : 8;
    }();
    return v;
}
int cdc_nbounce() {
    static const int v = [] {
        const char* e = getenv("OXH_CDC_NBOUNCE");
        const int k = e ? atoi(e) : 8;
        return std::max(2, std::min(k, kCdcMaxBounce));
    }();
    return v;
}
constexpr uint64_t kCdcPart = 4ull << 20;     // one reader task
constexpr uint64_t kCdcAlign = 256;           // segment placement in a piece
constexpr uint64_t kProbeWindow = 256;        // files opened (and stat'ed) ahead of the planner, at most
// segments per round, at most: every planned file holds its descriptor until its last segment is read
constexpr size_t kMaxSegsPerRound = 2048;

// Descriptors one call may hold at once: files probed ahead of the planner plus the files of the round
// being read (FileSrc only; host buffers hold none). Half of what the soft RLIMIT_NOFILE leaves free
// when the call starts, split over the `shares` calls an _multi entry runs side by side -- so a tree of
// many small (or empty) files never meets EMFILE under a 1024 default limit.
struct FdBudget {
    uint64_t window = kProbeWindow;
    size_t segs = kMaxSegsPerRound;
};
FdBudget fd_budget(int shares) {
    FdBudget b;
    struct rlimit rl;
    if (getrlimit(RLIMIT_NOFILE, &rl) != 0 || rl.rlim_cur == RLIM_INFINITY) return b;
    uint64_t open_now = 0;
    if (DIR* d = opendir("/proc/self/fd")) {
        while (readdir(d)) ++open_now;
        closedir(d);
    }
    const uint64_t lim = (uint64_t)rl.rlim_cur;
    const uint64_t free_fds = lim > open_now ? lim - open_now : 0;
    const uint64_t mine = std::max<uint64_t>(16, free_fds / 2 / (uint64_t)std::max(1, shares));
    b.window = std::min<uint64_t>(kProbeWindow, std::max<uint64_t>(4, mine / 8));
    b.segs = (size_t)std::min<uint64_t>(kMaxSegsPerRound, std::max<uint64_t>(8, mine - b.window));
    return b;
}

inline uint64_t align_up(uint64_t x) { return (x + kCdcAlign - 1) & ~(kCdcAlign - 1); }

// Per-context state, created on first use and kept: the two device piece buffers, the pinned ring,
// the chunk-table buffers, streams and a reader pool of its own (the context's engine keeps its
// pools busy independently).
struct CdcHost {
    int device = 0;
    hipStream_t copy = nullptr, comp = nullptr;
    hipStream_t copy2 = nullptr;  // a second copy stream (OXH_CDC_COPY_STREAMS=2): windows alternate
    int ncopy = 1;
    uint64_t piece = 0;
    uint8_t* d_piece[2] = {};
    hipEvent_t ev_copied[2] = {}, ev_copied2[2] = {};
    int nbounce = 0;
    uint8_t* h_bounce[kCdcMaxBounce] = {};
    hipEvent_t ev_bounce[kCdcMaxBounce] = {};
    bool bounce_used[kCdcMaxBounce] = {};
    uint64_t tab_cap = 0;  // entries of the chunk-table buffers below
    uint64_t *d_off = nullptr, *d_len = nullptr, *d_dig = nullptr;
    uint64_t *h_off = nullptr, *h_len = nullptr, *h_dig = nullptr;
    oxh::Pool* pool = nullptr;

    ~CdcHost() {
        (void)hipSetDevice(device);
        for (hipStream_t st : {copy, copy2, comp})  // every stream that touches d_piece, before it goes
            if (st) (void)hipStreamSynchronize(st);
        for (auto* p : d_piece)
            if (p) (void)hipFree(p);
        for (auto e : ev_copied)
            if (e) (void)hipEventDestroy(e);
        for (auto e : ev_copied2)
            if (e) (void)hipEventDestroy(e);
        for (int i = 0; i < kCdcMaxBounce; ++i) {
            if (h_bounce[i]) (void)hipHostFree(h_bounce[i]);
            if (ev_bounce[i]) (void)hipEventDestroy(ev_bounce[i]);
        }
        free_tables();
        if (copy) (void)hipStreamDestroy(copy);
        if (copy2) (void)hipStreamDestroy(copy2);
        if (comp) (void)hipStreamDestroy(comp);
        delete pool;
    }
    void free_tables() {
        for (auto* p : {d_off, d_len, d_dig})
            if (p) (void)hipFree(p);
        for (auto* p : {h_off, h_len, h_dig})
            if (p) (void)hipHostFree(p);
        d_off = d_len = d_dig = h_off = h_len = h_dig = nullptr;
        tab_cap = 0;
    }
    // chunk-table buffers of at least `need` entries
    int tables(uint64_t need) {
        if (need <= tab_cap) return OXH_OK;
        free_tables();
        const uint64_t cap = std::max<uint64_t>(need + need / 4, 1 << 16);
        bool ok = hipMalloc(&d_off, cap * 8) == hipSuccess && hipMalloc(&d_len, cap * 8) == hipSuccess &&
                  hipMalloc(&d_dig, cap * 16) == hipSuccess &&
                  hipHostMalloc(&h_off, cap * 8, hipHostMallocDefault) == hipSuccess &&
                  hipHostMalloc(&h_len, cap * 8, hipHostMallocDefault) == hipSuccess &&
                  hipHostMalloc(&h_dig, cap * 16, hipHostMallocDefault) == hipSuccess;
        if (!ok) {
            (void)hipGetLastError();
            free_tables();
            return oxh::set_error(OXH_ERR_NOMEM, "host chunk pipeline: chunk-table buffers");
        }
        tab_cap = cap;
        return OXH_OK;
    }
};

void free_cdc_host(void* p) { delete static_cast<CdcHost*>(p); }

// the context's CdcHost with pieces of `piece` bytes (re-made if the size changed)
int cdc_host(oxh_ctx* ctx, uint64_t piece, CdcHost** out) {
    void*& slot = oxh::ctx_cdc_state(ctx, free_cdc_host);
    CdcHost* h = static_cast<CdcHost*>(slot);
    if (h && h->piece == piece && h->nbounce == cdc_nbounce() && h->ncopy == cdc_copy_streams()) {
        *out = h;
        return OXH_OK;
    }
    delete h;
    slot = nullptr;
    h = new CdcHost;
    h->device = oxh::ctx_device(ctx);
    h->piece = piece;
    auto bad = [&](int code, const char* what) {
        (void)hipGetLastError();
        delete h;
        return oxh::set_error(code, std::string("FastCDC host pipeline: ") + what);
    };
    if (hipStreamCreateWithFlags(&h->copy, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&h->comp, hipStreamNonBlocking) != hipSuccess)
        return bad(OXH_ERR_HIP, "streams");
    h->ncopy = cdc_copy_streams();
    if (h->ncopy == 2 && hipStreamCreateWithFlags(&h->copy2, hipStreamNonBlocking) != hipSuccess) return bad(OXH_ERR_HIP, "streams");
    for (int b = 0; b < 2; ++b) {
        if (hipMalloc(&h->d_piece[b], piece + 4096) != hipSuccess) return bad(OXH_ERR_NOMEM, "device piece buffers");
        if (hipEventCreateWithFlags(&h->ev_copied[b], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&h->ev_copied2[b], hipEventDisableTiming) != hipSuccess)
            return bad(OXH_ERR_HIP, "events");
    }
    h->nbounce = cdc_nbounce();
    for (int i = 0; i < h->nbounce; ++i) {
        if (hipHostMalloc(&h->h_bounce[i], cdc_bounce(), hipHostMallocDefault) != hipSuccess)
            return bad(OXH_ERR_NOMEM, "pinned bounce buffers");
        if (hipEventCreateWithFlags(&h->ev_bounce[i], hipEventDisableTiming) != hipSuccess) return bad(OXH_ERR_HIP, "events");
    }
    h->pool = new oxh::Pool(oxh::default_reader_threads());
    slot = h;
    *out = h;
    return OXH_OK;
}

// Where item i's bytes come from.
struct CdcSource {
    virtual ~CdcSource() = default;
    // OXH_OK with its size, or the item's status (OXH_ERR_OPEN / OXH_ERR_IO) and errno
    virtual int open(uint64_t i, uint64_t& size, int& oserr) = 0;
    // [off, off + n) into dst; false with errno (0: the file ended early); called from many threads
    virtual bool read(uint64_t i, uint64_t off, uint64_t n, uint8_t* dst, int& oserr) = 0;
    virtual void close(uint64_t) {}
    virtual bool holds_fds() const { return false; }  // open() keeps a descriptor until close()
};

// fs::read(input_file) (fastcdchunker.rs:75): File::open, then the whole file. A directory opens and
// fails its read with EISDIR, as read_to_end does; the size is the open file's fstat. Files open
// with O_NONBLOCK, so a FIFO cannot park a pool thread in open(2) waiting for a writer (where fs::read
// would wait, and then read whatever arrives); like the file engine, anything that is not a regular
// file or a directory is refused as unreadable (EINVAL) -- the chunk pipeline preads.
struct FileSrc final : CdcSource {
    const char* const* paths;
    std::vector<int> fds;
    FileSrc(const char* const* p, uint64_t n) : paths(p), fds(n, -1) {}
    ~FileSrc() override {
        for (int fd : fds)
            if (fd >= 0) ::close(fd);
    }
    int open(uint64_t i, uint64_t& size, int& oserr) override {
        size = 0;
        const int fd = ::open(paths[i], O_RDONLY | O_CLOEXEC | O_NONBLOCK);
        if (fd < 0) {
            oserr = errno;
            return OXH_ERR_OPEN;
        }
        struct stat sb;
        if (fstat(fd, &sb) != 0) {
            oserr = errno;
            ::close(fd);
            return OXH_ERR_IO;
        }
        if (!S_ISREG(sb.st_mode)) {
            oserr = S_ISDIR(sb.st_mode) ? EISDIR : EINVAL;
            ::close(fd);
            return OXH_ERR_IO;
        }
        fds[i] = fd;
        size = (uint64_t)sb.st_size;
        return OXH_OK;
    }
    bool read(uint64_t i, uint64_t off, uint64_t n, uint8_t* dst, int& oserr) override {
        for (uint64_t got = 0; got < n;) {
            const ssize_t k = pread(fds[i], dst + got, n - got, (off_t)(off + got));
            if (k < 0 && errno == EINTR) continue;
            if (k < 0) oserr = errno;
            if (k <= 0) return false;
            got += (uint64_t)k;
        }
        return true;
    }
    void close(uint64_t i) override {
        if (fds[i] >= 0) ::close(fds[i]);
        fds[i] = -1;
    }
    bool holds_fds() const override { return true; }
};

struct MemSrc final : CdcSource {
    const uint8_t* const* bufs;
    const uint64_t* lens;
    MemSrc(const uint8_t* const* b, const uint64_t* l) : bufs(b), lens(l) {}
    int open(uint64_t i, uint64_t& size, int&) override {
        size = lens[i];
        return OXH_OK;
    }
    bool read(uint64_t i, uint64_t off, uint64_t n, uint8_t* dst, int&) override {
        memcpy(dst, bufs[i] + off, n);
        return true;
    }
};

struct FileState {
    uint64_t size = 0;
    std::atomic<int> status{OXH_OK}, oserr{0};
    bool probed = false;
    uint64_t carry = 0;      // the exact chunk start the next segment is chunked from (stitcher)
    uint64_t next_lo = 0;    // where the next segment's read starts (planner)
    uint64_t first = 0;      // output index of the file's first chunk (stitcher)
    int segs_left = 0;       // segments planned but not yet read (planner / reader; closes the fd)
};

struct Seg {
    uint64_t file, lo, hi, poff;  // file bytes [lo, hi) at piece offset poff
    bool first, last;             // the file's first / last segment
};

struct Round {
    int b = 0;
    std::vector<Seg> segs;
    bool io_done = false;
};

struct Call {
    CdcHost* h;
    CdcSource* src;
    uint64_t n;
    uint32_t mn, av, mx, lv;
    uint64_t fixed = 0;  // fixed-size chunking (oxh_chunk_digests_files / _host): the chunk size; 0 = FastCDC
    uint64_t* c_off;
    uint64_t* c_len;
    uint64_t* dig;
    uint64_t capacity;
    uint64_t* first_chunk;
    std::vector<FileState> files;
    uint64_t total = 0;  // chunks emitted (written while < capacity)
    std::atomic<int> rc{OXH_OK};
    std::string err;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<Round> ready;   // rounds whose bytes are on the device, for the chunking thread
    bool planner_done = false;
    bool buf_busy[2] = {false, false};
    double t_read = 0, t_chunk = 0, t_wait = 0, t_read_wait = 0, t_h2d_wait = 0;

    void fail(int code, const std::string& m) {
        int z = OXH_OK;
        if (rc.compare_exchange_strong(z, code)) {
            std::lock_guard<std::mutex> g(mu);
            err = m;
        }
        cv.notify_all();
    }
};

double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

// Stitch one round's chunk table into the caller's arrays (round order = file order = output order).
void stitch(Call& C, const Round& R, const std::vector<uint64_t>& first, const std::vector<uint64_t>& item_off) {
    CdcHost& h = *C.h;
    for (size_t j = 0; j < R.segs.size(); ++j) {
        const Seg& s = R.segs[j];
        FileState& F = C.files[s.file];
        if (s.first) F.first = C.total;
        if (F.status.load() != OXH_OK) {  // a read of this file failed (this round or before): drop its chunks
            C.total = F.first;
            if (s.last) C.first_chunk[s.file + 1] = C.total;
            continue;
        }
        const uint64_t a = first[j], e = first[j + 1];
        const uint64_t start = s.first ? s.lo : F.carry;
        bool carried = false;
        for (uint64_t k = a; k < e; ++k) {
            const uint64_t pos = start + (h.h_off[k] - item_off[j]);  // the chunk's offset in its file
            if (!s.last && pos + C.mx > s.hi) {  // not certain before the file's next bytes: chunk it again
                F.carry = pos;
                carried = true;
                break;
            }
            if (C.total < C.capacity) {
                C.c_off[C.total] = pos;
                C.c_len[C.total] = h.h_len[k];
                if (C.dig) {
                    C.dig[2 * C.total] = h.h_dig[2 * k];
                    C.dig[2 * C.total + 1] = h.h_dig[2 * k + 1];
                }
            }
            ++C.total;
        }
        if (!s.last && !carried) F.carry = s.hi;  // every chunk final: the next one starts at the segment end
        if (s.last) C.first_chunk[s.file + 1] = C.total;
    }
}

// Fixed-size chunking of one round: every segment starts at a multiple of the chunk size in its file,
// so its chunks are [poff + k*chunk, + min(chunk, rest)) of the piece. A few segments: one implied-grid
// K1 launch each; many: one K1 launch over the round's chunk descriptors. The digests come back and are
// appended per file. false = the call failed.
bool fixed_round(Call& C, const Round& R) {
    CdcHost& h = *C.h;
    const uint64_t ck = C.fixed;
    std::vector<uint64_t> first(R.segs.size() + 1, 0);
    for (size_t j = 0; j < R.segs.size(); ++j) {
        const Seg& s = R.segs[j];
        const bool ok = C.files[s.file].status.load() == OXH_OK;
        first[j + 1] = first[j] + (ok ? (s.hi - s.lo + ck - 1) / ck : 0);
    }
    const uint64_t m = first.back();
    int rc = h.tables(m);
    // a segment starts on a chunk boundary of its file, so its chunks are the implied grid of ck-byte
    // chunks over [poff, poff + hi - lo) of the piece: with few segments, one grid launch each
    size_t live = 0;
    for (size_t j = 0; j < R.segs.size(); ++j) live += first[j + 1] > first[j];
    const bool implicit = live <= (size_t)fixed_implicit_segs();
    for (size_t j = 0; rc == OXH_OK && !implicit && j < R.segs.size(); ++j) {
        const Seg& s = R.segs[j];
        for (uint64_t k = first[j], o = s.lo; k < first[j + 1]; ++k, o += ck) {
            h.h_off[k] = s.poff + (o - s.lo);
            h.h_len[k] = std::min(ck, s.hi - o);
        }
    }
    if (rc == OXH_OK && m && !implicit &&
        (hipMemcpyAsync(h.d_off, h.h_off, m * 8, hipMemcpyHostToDevice, h.comp) != hipSuccess ||
         hipMemcpyAsync(h.d_len, h.h_len, m * 8, hipMemcpyHostToDevice, h.comp) != hipSuccess))
        rc = oxh::set_error(OXH_ERR_HIP, "chunk descriptors H2D");
    if (rc == OXH_OK && (hipStreamWaitEvent(h.comp, h.ev_copied[R.b], 0) != hipSuccess ||
                         (h.ncopy == 2 && hipStreamWaitEvent(h.comp, h.ev_copied2[R.b], 0) != hipSuccess)))
        rc = oxh::set_error(OXH_ERR_HIP, "wait copies");
    if (rc == OXH_OK && m && !implicit)
        rc = oxh_xxh3_128_batch_device(h.d_piece[R.b], h.d_off, h.d_len, m, h.d_dig,
                                       ck <= 16384 ? OXH_MODE_WAVE_SHORT : OXH_MODE_WAVE, h.comp);
    for (size_t j = 0; rc == OXH_OK && implicit && j < R.segs.size(); ++j) {
        const Seg& s = R.segs[j];
        if (first[j + 1] > first[j])
            rc = oxh_chunk_digests_device(h.d_piece[R.b] + s.poff, s.hi - s.lo, ck, h.d_dig + 2 * first[j], h.comp);
    }
    if (rc == OXH_OK && m && hipMemcpyAsync(h.h_dig, h.d_dig, m * 16, hipMemcpyDeviceToHost, h.comp) != hipSuccess)
        rc = oxh::set_error(OXH_ERR_HIP, "digests D2H");
    if (rc == OXH_OK && hipStreamSynchronize(h.comp) != hipSuccess) rc = oxh::set_error(OXH_ERR_HIP, "chunking stream");
    if (rc != OXH_OK) {
        C.fail(rc, oxh_last_error());
        return false;
    }
    {
        std::lock_guard<std::mutex> g(C.mu);
        C.buf_busy[R.b] = false;
    }
    C.cv.notify_all();
    for (size_t j = 0; j < R.segs.size(); ++j) {
        const Seg& s = R.segs[j];
        FileState& F = C.files[s.file];
        if (s.first) F.first = C.total;
        if (F.status.load() != OXH_OK) {  // a read of this file failed: drop what it emitted
            C.total = F.first;
        } else {
            for (uint64_t k = first[j]; k < first[j + 1]; ++k, ++C.total)
                if (C.total < C.capacity && C.dig) {
                    C.dig[2 * C.total] = h.h_dig[2 * k];
                    C.dig[2 * C.total + 1] = h.h_dig[2 * k + 1];
                }
        }
        if (s.last) C.first_chunk[s.file + 1] = C.total;
    }
    return true;
}

// The chunking thread: rounds in order; each waits for its copies, is chunked on the device, its table
// comes back, and its piece buffer is handed back to the planner.
void chunk_rounds(Call& C) {
    CdcHost& h = *C.h;
    (void)hipSetDevice(h.device);
    std::vector<uint64_t> offs, lens, first, item_off;
    for (;;) {
        Round R;
        {
            std::unique_lock<std::mutex> lk(C.mu);
            const double t0 = now();
            C.cv.wait(lk, [&] { return !C.ready.empty() || C.planner_done || C.rc.load() != OXH_OK; });
            C.t_wait += now() - t0;
            if (C.rc.load() != OXH_OK) return;
            if (C.ready.empty()) return;  // planner done, nothing left
            R = std::move(C.ready.front());
            C.ready.pop_front();
        }
        const double t0 = now();
        if (C.fixed) {
            if (!fixed_round(C, R)) return;
            C.t_chunk += now() - t0;
            continue;
        }
        const size_t m = R.segs.size();
        offs.assign(m, 0), lens.assign(m, 0), item_off.assign(m, 0), first.assign(m + 1, 0);
        for (size_t j = 0; j < m; ++j) {
            const Seg& s = R.segs[j];
            const FileState& F = C.files[s.file];
            if (F.status.load() != OXH_OK) continue;  // an empty item keeps the indices
            const uint64_t start = s.first ? s.lo : F.carry;
            if (start < s.lo || start > s.hi) {
                C.fail(OXH_ERR_HIP, "FastCDC host pipeline: carry outside its segment");
                return;
            }
            offs[j] = item_off[j] = s.poff + (start - s.lo);
            lens[j] = s.hi - start;
        }
        const uint64_t need = oxh_fastcdc_max_chunks(lens.data(), m, C.mn) + 1;
        int rc = h.tables(need);
        if (rc == OXH_OK && (hipStreamWaitEvent(h.comp, h.ev_copied[R.b], 0) != hipSuccess ||
                             (h.ncopy == 2 && hipStreamWaitEvent(h.comp, h.ev_copied2[R.b], 0) != hipSuccess)))
            rc = oxh::set_error(OXH_ERR_HIP, "wait copies");
        if (rc == OXH_OK)
            rc = oxh_fastcdc_device(h.d_piece[R.b], offs.data(), lens.data(), m, C.mn, C.av, C.mx, C.lv, h.d_off, h.d_len,
                                    C.dig ? h.d_dig : nullptr, h.tab_cap, first.data(), h.comp);
        const uint64_t tot = first[m];
        if (rc == OXH_OK && tot) {
            if (hipMemcpyAsync(h.h_off, h.d_off, tot * 8, hipMemcpyDeviceToHost, h.comp) != hipSuccess ||
                hipMemcpyAsync(h.h_len, h.d_len, tot * 8, hipMemcpyDeviceToHost, h.comp) != hipSuccess ||
                (C.dig && hipMemcpyAsync(h.h_dig, h.d_dig, tot * 16, hipMemcpyDeviceToHost, h.comp) != hipSuccess))
                rc = oxh::set_error(OXH_ERR_HIP, "chunk table D2H");
        }
        if (rc == OXH_OK && hipStreamSynchronize(h.comp) != hipSuccess) rc = oxh::set_error(OXH_ERR_HIP, "chunking stream");
        if (rc != OXH_OK) {
            C.fail(rc, oxh_last_error());
            return;
        }
        {
            std::lock_guard<std::mutex> g(C.mu);
            C.buf_busy[R.b] = false;  // the piece buffer may take the next round's bytes
        }
        C.cv.notify_all();
        stitch(C, R, first, item_off);
        C.t_chunk += now() - t0;
    }
}

// Read one round's segments into the piece buffer through the bounce ring (windows of cdc_bounce() of
// the piece, read by the pool in kCdcPart tasks, each window's H2D once its reads are done; up to
// kCdcNBounce - 1 windows reading while the oldest one's copy is issued).
int upload_round(Call& C, const Round& R) {
    CdcHost& h = *C.h;
    struct Part {
        uint64_t file, off, n, boff;
    };
    struct Window {
        int bb = 0;
        uint64_t base = 0, used = 0;
        std::vector<Part> parts;
        std::function<void(int)> fn;
        oxh::Pool::Group grp;
    };
    std::vector<std::unique_ptr<Window>> wins;
    const uint64_t bounce = cdc_bounce();
    for (const Seg& s : R.segs) {
        if (C.files[s.file].status.load() != OXH_OK) continue;
        for (uint64_t o = s.lo; o < s.hi;) {
            const uint64_t p = s.poff + (o - s.lo), w = p / bounce;
            const uint64_t n = std::min({s.hi - o, kCdcPart, (w + 1) * bounce - p});
            while (wins.size() <= w) {
                wins.emplace_back(new Window);
                wins.back()->base = (uint64_t)(wins.size() - 1) * bounce;
            }
            Window& W = *wins[w];
            W.parts.push_back({s.file, o, n, p - W.base});
            W.used = std::max(W.used, p - W.base + n);
            o += n;
        }
    }
    std::deque<Window*> inflight;
    uint64_t next_bb = 0;
    auto finish = [&](Window& W) -> int {
        const double tw = now();
        W.grp.wait();
        C.t_read_wait += now() - tw;
        if (W.used == 0) return OXH_OK;
        hipStream_t cs = (h.ncopy == 2 && (W.base / bounce) % 2) ? h.copy2 : h.copy;
        if (hipMemcpyAsync(h.d_piece[R.b] + W.base, h.h_bounce[W.bb], W.used, hipMemcpyHostToDevice, cs) != hipSuccess ||
            hipEventRecord(h.ev_bounce[W.bb], cs) != hipSuccess)
            return oxh::set_error(OXH_ERR_HIP, "piece H2D");
        h.bounce_used[W.bb] = true;
        return OXH_OK;
    };
    int rc = OXH_OK;
    for (auto& wp : wins) {
        Window& W = *wp;
        if (W.parts.empty()) continue;
        W.bb = (int)(next_bb++ % (uint64_t)h.nbounce);
        const double tw = now();
        if (h.bounce_used[W.bb] && hipEventSynchronize(h.ev_bounce[W.bb]) != hipSuccess) {
            rc = oxh::set_error(OXH_ERR_HIP, "bounce buffer wait");
            break;
        }
        C.t_h2d_wait += now() - tw;
        h.bounce_used[W.bb] = false;
        uint8_t* dst = h.h_bounce[W.bb];
        W.fn = [&C, &W, dst](int t) {
            const Part& P = W.parts[(size_t)t];
            FileState& F = C.files[P.file];
            if (F.status.load(std::memory_order_relaxed) != OXH_OK) return;
            int e = 0;
            if (!C.src->read(P.file, P.off, P.n, dst + P.boff, e)) {
                int z = OXH_OK;
                if (F.status.compare_exchange_strong(z, OXH_ERR_IO)) F.oserr.store(e);
            }
        };
        h.pool->start((int)W.parts.size(), W.fn, W.grp);
        inflight.push_back(&W);
        if ((int)inflight.size() >= h.nbounce - 1) {
            rc = finish(*inflight.front());
            inflight.pop_front();
            if (rc) break;
        }
    }
    while (!inflight.empty()) {  // (after an error too: no task may outlive its window)
        const int r2 = finish(*inflight.front());
        inflight.pop_front();
        if (rc == OXH_OK) rc = r2;
    }
    if (rc == OXH_OK && (hipEventRecord(h.ev_copied[R.b], h.copy) != hipSuccess ||
                         (h.ncopy == 2 && hipEventRecord(h.ev_copied2[R.b], h.copy2) != hipSuccess)))
        rc = oxh::set_error(OXH_ERR_HIP, "copy event");
    return rc;
}

// fixed-size chunks per round: bounds the descriptor / digest buffers (32 B a chunk) for tiny chunks
constexpr uint64_t kMaxFixedChunksPerRound = 4ull << 20;
// largest fixed chunk: a chunk must fit a piece, and pieces stop at 3 GiB
constexpr uint64_t kMaxFixedChunk = (3ull << 30) - (64ull << 20);

// the crate's asserts (v2020::FastCDC::with_level) or the fixed chunk size's range, before any I/O
int check_params(uint32_t mn, uint32_t av, uint32_t mx, uint32_t lv, uint64_t fixed) {
    if (fixed) return fixed > kMaxFixedChunk ? oxh::set_error(OXH_ERR_INVALID, "chunk_size above 3 GiB - 64 MiB") : OXH_OK;
    uint64_t ms = 0, ml = 0;
    if (mn < 64 || mn > 1048576) return oxh::set_error(OXH_ERR_INVALID, "min_size must be in [64, 1048576]");
    if (mx < 1024 || mx > 16777216) return oxh::set_error(OXH_ERR_INVALID, "max_size must be in [1024, 16777216]");
    return oxh_fastcdc_masks(av, lv, &ms, &ml);
}

int run(oxh_ctx* ctx, CdcSource& src, uint64_t n, uint32_t mn, uint32_t av, uint32_t mx, uint32_t lv, uint64_t fixed,
        uint64_t* c_off, uint64_t* c_len, uint64_t* dig, uint64_t capacity, uint64_t* first_chunk, uint64_t* sizes,
        int32_t* status, int32_t* os_error, uint64_t* total_out = nullptr, int shares = 1) {
    if (!ctx) return oxh::set_error(OXH_ERR_INVALID, "null context");
    if (!first_chunk) return oxh::set_error(OXH_ERR_INVALID, "null first_chunk");
    if (capacity && !fixed && (!c_off || !c_len)) return oxh::set_error(OXH_ERR_INVALID, "null chunk table");
    if (capacity && fixed && !dig) return oxh::set_error(OXH_ERR_INVALID, "null digests");
    if (int rc = check_params(mn, av, mx, lv, fixed)) return rc;
    if (n == 0) {  // nothing to read: no pipeline buffers for an empty call
        first_chunk[0] = 0;
        if (total_out) *total_out = 0;
        return OXH_OK;
    }
    uint64_t min_seg = 0;
    if (fixed) {
        // a segment is whole chunks: at least one, and 16 MiB when the chunks are smaller (within the
        // round's chunk budget)
        min_seg = fixed * std::max<uint64_t>(1, std::min<uint64_t>((16ull << 20) / fixed, kMaxFixedChunksPerRound));
    } else {
        // a segment is at least 16 MiB and 4 max chunks
        min_seg = std::max<uint64_t>(16ull << 20, 4ull * mx + kCdcAlign);
    }
    std::lock_guard<std::mutex> call_lock(oxh::ctx_call_mutex(ctx));
    (void)hipSetDevice(oxh::ctx_device(ctx));
    // pieces of OXH_CDC_PIECE_MIB (default 1 GiB), at least two minimal segments (one for a fixed chunk
    // size above 1 GiB)
    const char* pe = getenv("OXH_CDC_PIECE_MIB");
    uint64_t piece = (pe && atoll(pe) > 0 ? (uint64_t)atoll(pe) : 1024ull) << 20;
    piece = std::max<uint64_t>(piece, fixed > (1ull << 30) ? min_seg + kCdcAlign : 2 * min_seg);
    piece = std::min<uint64_t>(piece, 3ull << 30);
    piece = (piece + cdc_bounce() - 1) / cdc_bounce() * cdc_bounce();
    CdcHost* h = nullptr;
    if (int rc = cdc_host(ctx, piece, &h)) return rc;

    Call C;
    C.h = h, C.src = &src, C.n = n, C.mn = mn, C.av = av, C.mx = mx, C.lv = lv, C.fixed = fixed;
    C.c_off = c_off, C.c_len = c_len, C.dig = dig, C.capacity = capacity, C.first_chunk = first_chunk;
    C.files = std::vector<FileState>(n);
    first_chunk[0] = 0;
    const FdBudget fdb = src.holds_fds() ? fd_budget(shares) : FdBudget{};
    static const bool trace = getenv("OXH_TRACE") != nullptr;
    const double t_start = now();
    std::thread chunker(chunk_rounds, std::ref(C));

    // probe (open + fstat) the files [lo, hi) in parallel
    uint64_t probed = 0;
    auto probe_to = [&](uint64_t hi) {
        hi = std::min(hi, n);
        if (hi <= probed) return;
        const uint64_t lo = probed;
        h->pool->parallel_for((int)(hi - lo), [&](int t) {
            FileState& F = C.files[lo + (uint64_t)t];
            int e = 0;
            const int st = src.open(lo + (uint64_t)t, F.size, e);
            F.status.store(st);
            F.oserr.store(e);
            F.probed = true;
        });
        probed = hi;
    };

    int rc = OXH_OK;
    uint64_t cur = 0;  // the planner's file
    int round_no = 0;
    while (cur < n && C.rc.load() == OXH_OK) {
        Round R;
        R.b = round_no & 1;
        // plan: files in order into this piece; a file that does not fit whole takes the rest of the
        // piece (if at least min_seg) and continues in the next round from `max` before its end
        uint64_t off = 0, nchunks = 0;  // (nchunks: fixed-size chunks planned this round)
        while (cur < n && R.segs.size() < fdb.segs) {
            if (cur >= probed) probe_to(cur + fdb.window);
            FileState& F = C.files[cur];
            if (F.status.load() != OXH_OK || F.size == 0) {  // no (more) chunks: an error, or an empty file
                // (a file whose read failed in an earlier round keeps its first output index: the
                // stitcher drops what it emitted for it). Nothing more is read from it: its descriptor
                // closes now (its earlier segments, if any, were read in rounds already uploaded).
                R.segs.push_back({cur, 0, 0, 0, F.next_lo == 0, true});
                if (F.segs_left == 0) src.close(cur);
                ++cur;
                continue;
            }
            const uint64_t lo = F.next_lo, left = F.size - lo;
            const uint64_t at = align_up(off);
            uint64_t room = at < piece ? piece - at : 0;
            if (fixed) {  // whole chunks, and the round's chunk budget
                room = std::min(room, (kMaxFixedChunksPerRound - nchunks) * fixed);
                if (left <= room) {
                    R.segs.push_back({cur, lo, F.size, at, lo == 0, true});
                    ++F.segs_left;
                    off = at + left;
                    nchunks += (left + fixed - 1) / fixed;
                    ++cur;
                    continue;
                }
                const uint64_t take = room / fixed * fixed;
                if (take >= min_seg) {  // the next segment starts where this one ends: no chunk straddles
                    R.segs.push_back({cur, lo, lo + take, at, lo == 0, false});
                    ++F.segs_left;
                    F.next_lo = lo + take;
                }
                break;
            }
            if (left <= room) {
                R.segs.push_back({cur, lo, F.size, at, lo == 0, true});
                ++F.segs_left;
                off = at + left;
                ++cur;
                continue;
            }
            if (room >= min_seg) {
                R.segs.push_back({cur, lo, lo + room, at, lo == 0, false});
                ++F.segs_left;
                F.next_lo = lo + room - mx;  // the carry lies in (end - max, end]
            }
            break;
        }
        // the piece buffer: free once the chunking thread is done with round - 2
        {
            std::unique_lock<std::mutex> lk(C.mu);
            const double t0 = now();
            C.cv.wait(lk, [&] { return !C.buf_busy[R.b] || C.rc.load() != OXH_OK; });
            C.t_wait += now() - t0;
            if (C.rc.load() != OXH_OK) break;
            C.buf_busy[R.b] = true;
        }
        const double t0 = now();
        rc = upload_round(C, R);
        C.t_read += now() - t0;
        for (const Seg& s : R.segs)  // a file's descriptor closes after its last segment's reads
            if (s.hi > s.lo && --C.files[s.file].segs_left == 0 && s.last) src.close(s.file);
        if (rc) {
            C.fail(rc, oxh_last_error());
            break;
        }
        {
            std::lock_guard<std::mutex> g(C.mu);
            C.ready.push_back(std::move(R));
        }
        C.cv.notify_all();
        ++round_no;
    }
    {
        std::lock_guard<std::mutex> g(C.mu);
        C.planner_done = true;
    }
    C.cv.notify_all();
    chunker.join();
    (void)hipStreamSynchronize(h->copy);
    if (h->copy2) (void)hipStreamSynchronize(h->copy2);
    for (uint64_t i = 0; i < n; ++i) src.close(i);
    if (C.rc.load() != OXH_OK) return oxh::set_error(C.rc.load(), "FastCDC host pipeline: " + C.err);
    for (uint64_t i = 0; i < n; ++i) {
        const FileState& F = C.files[i];
        const bool ok = F.status.load() == OXH_OK;
        if (sizes) sizes[i] = F.size;  // fstat's size (0 when the open failed)
        if (status) status[i] = F.status.load();
        if (os_error) os_error[i] = ok ? 0 : F.oserr.load();
    }
    if (trace)
        fprintf(stderr, "[oxh] fastcdc_host: %llu items, %d rounds of %llu MiB, %llu chunks: total %.1f ms, reads+H2D %.1f, "
                "chunking+D2H+stitch %.1f, waits %.1f (of them: reads %.1f, bounce H2D %.1f), %d bounce x %llu MiB, %d readers\n",
                (unsigned long long)n, round_no, (unsigned long long)(piece >> 20), (unsigned long long)C.total,
                1e3 * (now() - t_start), 1e3 * C.t_read, 1e3 * C.t_chunk, 1e3 * C.t_wait, 1e3 * C.t_read_wait,
                1e3 * C.t_h2d_wait, h->nbounce, (unsigned long long)(cdc_bounce() >> 20), h->pool->size());
    if (total_out) *total_out = C.total;
    if (C.total > capacity)
        return oxh::set_error(OXH_ERR_INVALID, "chunk capacity too small: need " + std::to_string(C.total) + " entries");
    return OXH_OK;
}

// One call over several contexts (one per device: each its own PCIe link, pipeline and readers): the
// files split into nctx contiguous shares balanced by bytes, the shares run side by side, and their
// tables are concatenated in file order -- the multi-GPU form of SURVEY §8e for files in host memory,
// no collective (the tables meet in host memory).
// (files: paths; host buffers: paths == nullptr, bufs / lens)
int run_sharded(oxh_ctx* const* ctxs, int nctx, const char* const* paths, const uint8_t* const* bufs, const uint64_t* lens,
                uint64_t n, uint32_t mn, uint32_t av, uint32_t mx, uint32_t lv, uint64_t fixed, uint64_t* c_off,
                uint64_t* c_len, uint64_t* dig, uint64_t capacity, uint64_t* first_chunk, uint64_t* sizes, int32_t* status,
                int32_t* os_error) {
    if (!ctxs || nctx < 1) return oxh::set_error(OXH_ERR_INVALID, "no contexts");
    for (int k = 0; k < nctx; ++k)
        if (!ctxs[k]) return oxh::set_error(OXH_ERR_INVALID, "null context");
    if (!first_chunk) return oxh::set_error(OXH_ERR_INVALID, "null first_chunk");
    const bool files = paths != nullptr || bufs == nullptr;
    if (files) {
        if (n && !paths) return oxh::set_error(OXH_ERR_INVALID, "null paths");
        for (uint64_t i = 0; i < n; ++i)
            if (!paths[i]) return oxh::set_error(OXH_ERR_INVALID, "null path");
    } else {
        if (n && !lens) return oxh::set_error(OXH_ERR_INVALID, "null buffers");
        for (uint64_t i = 0; i < n; ++i)
            if (lens[i] && !bufs[i]) return oxh::set_error(OXH_ERR_INVALID, "null buffer");
    }
    if (int rc = check_params(mn, av, mx, lv, fixed)) return rc;
    if (capacity && !fixed && (!c_off || !c_len)) return oxh::set_error(OXH_ERR_INVALID, "null chunk table");
    if (capacity && fixed && !dig) return oxh::set_error(OXH_ERR_INVALID, "null digests");
    auto source = [&](uint64_t a, uint64_t m) -> std::unique_ptr<CdcSource> {
        if (files) return std::unique_ptr<CdcSource>(new FileSrc(paths + a, m));
        return std::unique_ptr<CdcSource>(new MemSrc(bufs + a, lens + a));
    };
    if (nctx == 1 || n <= 1) {
        auto src = source(0, n);
        return run(ctxs[0], *src, n, mn, av, mx, lv, fixed, c_off, c_len, dig, capacity, first_chunk, sizes, status, os_error);
    }
    // sizes for the split (a file that cannot be stat'ed weighs nothing; its share reports it)
    std::vector<uint64_t> sz(n, 0);
    if (!files) {
        for (uint64_t i = 0; i < n; ++i) sz[i] = lens[i];
    } else {
        std::vector<std::thread> th;
        const int nt = std::min<int>(nctx * 2, 16);
        for (int t = 0; t < nt; ++t)
            th.emplace_back([&, t] {
                for (uint64_t i = (uint64_t)t; i < n; i += (uint64_t)nt) {
                    struct stat sb;
                    if (stat(paths[i], &sb) == 0 && S_ISREG(sb.st_mode)) sz[i] = (uint64_t)sb.st_size;
                }
            });
        for (auto& t : th) t.join();
    }
    // contiguous shares, cut where the running byte count (+1 per file) passes k/nctx of the total
    std::vector<uint64_t> lo(nctx + 1, n);
    {
        uint64_t total = 0, run_w = 0;
        for (uint64_t i = 0; i < n; ++i) total += sz[i] + 1;
        int k = 1;
        lo[0] = 0;
        for (uint64_t i = 0; i < n && k < nctx; ++i) {
            run_w += sz[i] + 1;
            while (k < nctx && run_w * (uint64_t)nctx >= total * (uint64_t)k) lo[k++] = i + 1;
        }
        while (k < nctx) lo[k++] = n;
    }
    // Each share writes its chunks straight into the caller's arrays, into a region of its own bound
    // (the same bound the one-context call is sized by), when the capacity holds every share's
    // bound; the regions are then moved down into one contiguous table. A share whose files grew past
    // their bound (or a capacity below the bounds' sum) uses tables of its own instead.
    struct Share {
        std::vector<uint64_t> off, len, dig, first, sizes;
        std::vector<int32_t> st, oe;
        uint64_t cap = 0, start = 0, total = 0;
        bool inplace = false;
        int rc = OXH_OK;
        std::string err;
    };
    std::vector<Share> sh(nctx);
    uint64_t bound_sum = 0;
    for (int k = 0; k < nctx; ++k) {
        Share& S = sh[k];
        const uint64_t a = lo[k], m = lo[k + 1] - a;
        if (fixed) {
            for (uint64_t i = a; i < a + m; ++i) S.cap += (sz[i] + fixed - 1) / fixed;
        } else {
            S.cap += oxh_fastcdc_max_chunks(sz.data() + a, m, mn);
        }
        S.start = bound_sum;
        bound_sum += S.cap;
    }
    const bool inplace = bound_sum <= capacity;
    auto work = [&](int k) {
        Share& S = sh[k];
        const uint64_t a = lo[k], m = lo[k + 1] - a;
        S.first.assign(m + 1, 0);
        if (m == 0) return;  // (more contexts than files)
        uint64_t cap = S.cap;
        S.inplace = inplace;
        for (int attempt = 0; attempt < 3; ++attempt) {  // a file that grew since its stat: retry with the count
            uint64_t *o = nullptr, *l = nullptr, *d = nullptr;
            if (S.inplace) {
                if (!fixed) o = c_off + S.start, l = c_len + S.start;
                if (dig) d = dig + 2 * S.start;
            } else {
                if (!fixed) S.off.assign(cap, 0), S.len.assign(cap, 0), o = S.off.data(), l = S.len.data();
                if (dig) S.dig.assign(2 * cap, 0), d = S.dig.data();
            }
            S.first.assign(m + 1, 0), S.sizes.assign(m, 0), S.st.assign(m, 0), S.oe.assign(m, 0);
            auto src = source(a, m);
            S.total = 0;
            S.rc = run(ctxs[k], *src, m, mn, av, mx, lv, fixed, o, l, d, cap, S.first.data(), S.sizes.data(), S.st.data(),
                       S.oe.data(), &S.total, nctx);
            if (S.rc == OXH_ERR_INVALID && S.total > cap) {
                cap = S.total;
                S.inplace = false;  // past its region: tables of its own
                continue;
            }
            break;
        }
        if (S.rc != OXH_OK) S.err = oxh_last_error();
    };
    {
        std::vector<std::thread> th;
        for (int k = 1; k < nctx; ++k) th.emplace_back(work, k);
        work(0);
        for (auto& t : th) t.join();
    }
    for (int k = 0; k < nctx; ++k)
        if (sh[k].rc != OXH_OK)
            return oxh::set_error(sh[k].rc, "share " + std::to_string(k) + " (files " + std::to_string(lo[k]) + ".." +
                                                std::to_string(lo[k + 1]) + "): " + sh[k].err);
    // a share that left its region may overrun the next one's while the tables are joined: then every
    // in-place share's chunks are copied out first
    bool any_own = false;
    for (const Share& S : sh) any_own = any_own || (!S.inplace && S.total);
    if (inplace && any_own)
        for (Share& S : sh)
            if (S.inplace && S.total) {
                if (!fixed) {
                    S.off.assign(c_off + S.start, c_off + S.start + S.total);
                    S.len.assign(c_len + S.start, c_len + S.start + S.total);
                }
                if (dig) S.dig.assign(dig + 2 * S.start, dig + 2 * (S.start + S.total));
                S.inplace = false;
            }
    uint64_t base = 0;
    for (int k = 0; k < nctx; ++k) {
        const Share& S = sh[k];
        const uint64_t a = lo[k], m = lo[k + 1] - a;
        for (uint64_t i = 0; i < m; ++i) {
            first_chunk[a + i] = base + S.first[i];
            if (sizes) sizes[a + i] = S.sizes[i];
            if (status) status[a + i] = S.st[i];
            if (os_error) os_error[a + i] = S.oe[i];
        }
        const uint64_t keep = base < capacity ? std::min(S.total, capacity - base) : 0;
        if (keep && S.inplace) {  // down to its place in the joined table (base <= start: memmove)
            if (base != S.start) {
                if (!fixed) {
                    memmove(c_off + base, c_off + S.start, keep * 8);
                    memmove(c_len + base, c_len + S.start, keep * 8);
                }
                if (dig) memmove(dig + 2 * base, dig + 2 * S.start, keep * 16);
            }
        } else if (keep) {
            if (!fixed) {
                memcpy(c_off + base, S.off.data(), keep * 8);
                memcpy(c_len + base, S.len.data(), keep * 8);
            }
            if (dig) memcpy(dig + 2 * base, S.dig.data(), keep * 16);
        }
        base += S.total;
    }
    first_chunk[n] = base;
    if (base > capacity)
        return oxh::set_error(OXH_ERR_INVALID, "chunk capacity too small: need " + std::to_string(base) + " entries");
    return OXH_OK;
}

}  // namespace

extern "C" {

int oxh_fastcdc_files(oxh_ctx* ctx, const char* const* paths, uint64_t n, uint32_t min_size, uint32_t avg_size,
                      uint32_t max_size, uint32_t level, uint64_t* chunk_offsets, uint64_t* chunk_lens, uint64_t* digests,
                      uint64_t capacity, uint64_t* first_chunk, uint64_t* sizes, int32_t* status, int32_t* os_error) {
    if (n && !paths) return oxh::set_error(OXH_ERR_INVALID, "null paths");
    for (uint64_t i = 0; i < n; ++i)
        if (!paths[i]) return oxh::set_error(OXH_ERR_INVALID, "null path");
    FileSrc src(paths, n);
    return run(ctx, src, n, min_size, avg_size, max_size, level, 0, chunk_offsets, chunk_lens, digests, capacity, first_chunk,
               sizes, status, os_error);
}

int oxh_fastcdc_host(oxh_ctx* ctx, const uint8_t* const* bufs, const uint64_t* lens, uint64_t n, uint32_t min_size,
                     uint32_t avg_size, uint32_t max_size, uint32_t level, uint64_t* chunk_offsets, uint64_t* chunk_lens,
                     uint64_t* digests, uint64_t capacity, uint64_t* first_chunk) {
    if (n && (!bufs || !lens)) return oxh::set_error(OXH_ERR_INVALID, "null buffers");
    for (uint64_t i = 0; i < n; ++i)
        if (lens[i] && !bufs[i]) return oxh::set_error(OXH_ERR_INVALID, "null buffer");
    MemSrc src(bufs, lens);
    return run(ctx, src, n, min_size, avg_size, max_size, level, 0, chunk_offsets, chunk_lens, digests, capacity, first_chunk,
               nullptr, nullptr, nullptr);
}

// Fixed-size chunk digests from host memory: the block-level dedup's fixed-size chunkers
// (fixedsize_multithreaded.rs:78-110: chunk i = [i*chunk, min((i+1)*chunk, size)), xxh3_128 of each;
// fixedsize.rs:67-91 reads the same chunks through a BufReader) over n files or host buffers.
int oxh_chunk_digests_files(oxh_ctx* ctx, const char* const* paths, uint64_t n, uint64_t chunk_size, uint64_t* digests,
                            uint64_t capacity, uint64_t* first_chunk, uint64_t* sizes, int32_t* status, int32_t* os_error) {
    if (chunk_size == 0) return oxh::set_error(OXH_ERR_INVALID, "Chunk size cannot be zero");
    if (n && !paths) return oxh::set_error(OXH_ERR_INVALID, "null paths");
    for (uint64_t i = 0; i < n; ++i)
        if (!paths[i]) return oxh::set_error(OXH_ERR_INVALID, "null path");
    FileSrc src(paths, n);
    return run(ctx, src, n, 0, 0, 0, 0, chunk_size, nullptr, nullptr, digests, capacity, first_chunk, sizes, status,
               os_error);
}

int oxh_chunk_digests_host(oxh_ctx* ctx, const uint8_t* const* bufs, const uint64_t* lens, uint64_t n,
                           uint64_t chunk_size, uint64_t* digests, uint64_t capacity, uint64_t* first_chunk) {
    if (chunk_size == 0) return oxh::set_error(OXH_ERR_INVALID, "Chunk size cannot be zero");
    if (n && (!bufs || !lens)) return oxh::set_error(OXH_ERR_INVALID, "null buffers");
    for (uint64_t i = 0; i < n; ++i)
        if (lens[i] && !bufs[i]) return oxh::set_error(OXH_ERR_INVALID, "null buffer");
    MemSrc src(bufs, lens);
    return run(ctx, src, n, 0, 0, 0, 0, chunk_size, nullptr, nullptr, digests, capacity, first_chunk, nullptr, nullptr,
               nullptr);
}

// The file entries over several contexts (devices): run_sharded above.
int oxh_fastcdc_files_multi(oxh_ctx* const* ctxs, int nctx, const char* const* paths, uint64_t n, uint32_t min_size,
                            uint32_t avg_size, uint32_t max_size, uint32_t level, uint64_t* chunk_offsets,
                            uint64_t* chunk_lens, uint64_t* digests, uint64_t capacity, uint64_t* first_chunk,
                            uint64_t* sizes, int32_t* status, int32_t* os_error) {
    return run_sharded(ctxs, nctx, paths, nullptr, nullptr, n, min_size, avg_size, max_size, level, 0, chunk_offsets,
                       chunk_lens, digests, capacity, first_chunk, sizes, status, os_error);
}

int oxh_fastcdc_host_multi(oxh_ctx* const* ctxs, int nctx, const uint8_t* const* bufs, const uint64_t* lens, uint64_t n,
                           uint32_t min_size, uint32_t avg_size, uint32_t max_size, uint32_t level, uint64_t* chunk_offsets,
                           uint64_t* chunk_lens, uint64_t* digests, uint64_t capacity, uint64_t* first_chunk) {
    if (n && !bufs) return oxh::set_error(OXH_ERR_INVALID, "null buffers");
    return run_sharded(ctxs, nctx, nullptr, bufs, lens, n, min_size, avg_size, max_size, level, 0, chunk_offsets, chunk_lens,
                       digests, capacity, first_chunk, nullptr, nullptr, nullptr);
}

int oxh_chunk_digests_files_multi(oxh_ctx* const* ctxs, int nctx, const char* const* paths, uint64_t n,
                                  uint64_t chunk_size, uint64_t* digests, uint64_t capacity, uint64_t* first_chunk,
                                  uint64_t* sizes, int32_t* status, int32_t* os_error) {
    if (chunk_size == 0) return oxh::set_error(OXH_ERR_INVALID, "Chunk size cannot be zero");
    return run_sharded(ctxs, nctx, paths, nullptr, nullptr, n, 0, 0, 0, 0, chunk_size, nullptr, nullptr, digests, capacity,
                       first_chunk, sizes, status, os_error);
}

int oxh_chunk_digests_host_multi(oxh_ctx* const* ctxs, int nctx, const uint8_t* const* bufs, const uint64_t* lens, uint64_t n,
                                 uint64_t chunk_size, uint64_t* digests, uint64_t capacity, uint64_t* first_chunk) {
    if (chunk_size == 0) return oxh::set_error(OXH_ERR_INVALID, "Chunk size cannot be zero");
    if (n && !bufs) return oxh::set_error(OXH_ERR_INVALID, "null buffers");
    return run_sharded(ctxs, nctx, nullptr, bufs, lens, n, 0, 0, 0, 0, chunk_size, nullptr, nullptr, digests, capacity,
                       first_chunk, nullptr, nullptr, nullptr);
}

}  // extern "C"
