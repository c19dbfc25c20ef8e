// oxen_amd/csrc/engine.hip -- the streaming file engine behind every file call (oxh_hash_files*,
// oxh_add_files*, the modified check, fsck): one engine thread per context runs a continuous
// pipeline over every queued request. See capi_internal.hpp for the pieces.
#include "capi_internal.hpp"

#include <sys/syscall.h>

using namespace oxh::capi;

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
namespace oxh::capi {

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

// A file of at least kSplitBytes in a slot is read in kPartBytes parts by several readers: one pread
// stream from the page cache copies ~5-10 GB/s, so a slot holding one 200 MiB file waited ~30 ms on
// its reader. The parts together read [0, L + 1), one byte past the expected size, as read_expected does.
// Readers have file-descriptor tables of their own (pool.hpp), so a part reopens the first reader's
// open file through /proc/self/task/<tid>/fd/<fd>: the same inode even if the path was replaced or
// unlinked since, as the reference's one File handle reads it (hasher.rs:126-148). The first reader
// keeps its descriptor until every part has opened its own (reading parts meanwhile). Without /proc a
// part opens the path and checks device + inode; a replaced file is then re-read whole by the engine.
// OXH_SPLIT_READS=0: one pread per file (the r01-r06 form, for A/B).
constexpr uint64_t kPartBytes = 4ull << 20, kSplitBytes = 8ull << 20;
inline bool split_reads() {
    static const bool on = !(getenv("OXH_SPLIT_READS") && atoi(getenv("OXH_SPLIT_READS")) == 0);
    return on;
}

struct PartFile {  // one split file, shared by its parts: the reader that finishes the last one completes it
    FileRequest* r = nullptr;
    uint64_t i = 0, j = 0, L = 0;
    dev_t dev = 0;
    ino_t ino = 0;
    int s = 0;
    uint8_t* dst = nullptr;
    char link[64] = {};                 // /proc/self/task/<first reader's tid>/fd/<its descriptor>
    std::atomic<int> opened{0};         // parts (other than part 0) that have opened their descriptor
    std::atomic<int> refs{2};           // the completing reader and the first reader: the last one deletes
    std::atomic<int> left{0};
    std::atomic<int> err{0};            // errno of a failed pread (the first one recorded)
    std::atomic<bool> failed{false};
    std::atomic<bool> resized{false};   // fewer or more than L bytes: its size changed since the stat
};
struct PartTask {
    PartFile* f = nullptr;
    uint64_t lo = 0, hi = 0;  // file bytes [lo, hi) into f->dst + lo
};

}  // namespace oxh::capi

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

namespace oxh::capi {

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
    std::deque<PartTask> parts;          // parts of split files not yet claimed (under c->qmu)
    std::atomic<uint64_t> n_parts{0};    // parts.size(), read without the lock by waiting readers
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

// Zero the outputs of r's failed items (add.rs:533-544 skips them), report sizes and statuses.
void write_outputs(FileRequest* r) {
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
}

// Request r is complete: write its outputs, retire it from the run and wake its caller.
void finish_request(FileStream& fs, FileRequest* r) {
    write_outputs(r);
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

// pread a file expected to hold L bytes into dst, asking for one byte more (a file that grew since its
// size was taken shows as a longer count): the count read, or -1 with the read's errno in e
inline int64_t read_expected(int fd, uint8_t* dst, uint64_t L, int& e) {
    const uint64_t want = L + 1;
    uint64_t got = 0;
    while (got < want) {
        const ssize_t k = pread(fd, dst + got, want - got, (off_t)got);
        if (k < 0) {
            e = errno;
            return -1;
        }
        if (k == 0) break;  // EOF
        got += (uint64_t)k;
        // a short read of a regular file ends at its EOF: once the expected L bytes are in,
        // that settles the size without the extra pread that would return 0
        if (got >= L && (uint64_t)k < want - (got - (uint64_t)k)) break;
    }
    return (int64_t)got;
}

// k more items of r are fully written; the thread that accounts the last one completes r.
inline void account(FileStream& fs, FileRequest* r, uint64_t k) {
    if (k && r->remaining.fetch_sub(k, std::memory_order_acq_rel) == k) finish_request(fs, r);
}

// Next work: a part of a split file (pt.f set), else files [i0, i1) of request *r. Moves queued
// requests into the run; an idle reader sleeps until a request or a part arrives or the engine closes
// the run. False = stop.
bool claim(FileStream& fs, FileRequest*& r, uint64_t& i0, uint64_t& i1, PartTask& pt) {
    constexpr uint64_t kClaim = 8;
    oxh_ctx* c = fs.c;
    std::unique_lock<std::mutex> lk(c->qmu);
    for (;;) {
        if (fs.abort.load(std::memory_order_relaxed) || fs.closing) return false;
        if (!fs.parts.empty()) {
            pt = fs.parts.front();
            fs.parts.pop_front();
            fs.n_parts.fetch_sub(1);
            return true;
        }
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
        c->qcv.wait(lk, [&] { return fs.abort.load() || fs.closing || !c->queue.empty() || !fs.parts.empty(); });
        fs.idle.fetch_sub(1);
    }
}

// A reader waiting for a slot reads queued parts meanwhile: the slot it waits for may be held by a
// split file whose parts only readers can finish.
bool help_with_a_part(FileStream& fs);

// Open slot t for filling (generation + 1, empty, unsealed) once the engine has freed it.
bool open_slot(FileStream& fs, int t) {
    SlotFill& nx = fs.slot[t];
    while (nx.state.load(std::memory_order_acquire) != 0) {
        if (fs.abort.load(std::memory_order_relaxed)) return false;
        if (!help_with_a_part(fs)) pause_us(5);
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
                if (!help_with_a_part(fs)) pause_us(2);
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

// Item j of slot s is fully written: the last writer of a sealed slot wakes the engine.
inline void slot_item_done(FileStream& fs, int s) {
    const uint64_t d = fs.slot[s].done.fetch_add(1, std::memory_order_acq_rel) + 1;
    const uint64_t w = fs.slot[s].word.load(std::memory_order_acquire);
    if ((w & kSealedBit) && d == w_items(w)) fs.wake();
}

// The file in slot s, item j is not the size its stat / its caller gave: the engine re-reads it.
inline void item_resized(FileStream& fs, FileRequest* r, uint64_t i, int s, uint64_t j) {
    fs.c->rq[s][j] = nullptr;  // drain skips this slot entry
    {
        std::lock_guard<std::mutex> g(fs.omu);
        fs.changed.push_back({r, i});
    }
    fs.n_changed.fetch_add(1);
    fs.wake();
}

// Read one part of a split file (through `own_fd`, the first reader's descriptor, or a descriptor of
// its own); the reader that finishes the file's last part completes the item.
void run_part(FileStream& fs, const PartTask& t, int own_fd = -1) {
    PartFile* f = t.f;
    const uint64_t n = t.hi - t.lo;
    const bool last = t.hi == f->L + 1;
    uint64_t got = 0;
    int fd = own_fd;
    if (fd < 0) {
        fd = open(f->link, O_RDONLY | O_CLOEXEC | O_NONBLOCK);
        f->opened.fetch_add(1, std::memory_order_acq_rel);  // the first reader may close its descriptor now
        if (fd < 0) fd = open(f->r->paths[f->i], O_RDONLY | O_CLOEXEC | O_NONBLOCK);  // no /proc
        struct stat sb;
        if (fd >= 0 && (fstat(fd, &sb) != 0 || sb.st_dev != f->dev || sb.st_ino != f->ino)) {
            close(fd);
            fd = -1;
        }
        if (fd < 0) f->resized.store(true);  // gone or replaced since the first open: the engine re-reads it
    }
    while (fd >= 0 && got < n && !f->failed.load(std::memory_order_relaxed)) {
        const ssize_t k = pread(fd, f->dst + t.lo + got, n - got, (off_t)(t.lo + got));
        if (k < 0) {
            int zero = 0;
            f->err.compare_exchange_strong(zero, errno);
            f->failed.store(true);
            break;
        }
        if (k == 0) break;  // EOF
        got += (uint64_t)k;
        // the last part asks for one byte past L: a short read once L is reached is the EOF
        if (last && t.lo + got >= f->L && (uint64_t)k < n - (got - (uint64_t)k)) break;
    }
    // a part that ends before L, or the last one reaching L + 1: the file changed size
    if (fd >= 0 && !f->failed.load() && (last ? t.lo + got != f->L : got != n)) f->resized.store(true);
    if (fd >= 0 && fd != own_fd) close(fd);
    if (f->left.fetch_sub(1, std::memory_order_acq_rel) != 1) return;
    if (f->failed.load()) item_failed(f->r, f->i, OXH_ERR_IO, f->err.load());
    else if (f->resized.load()) item_resized(fs, f->r, f->i, f->s, f->j);
    const int s = f->s;
    if (f->refs.fetch_sub(1, std::memory_order_acq_rel) == 1) delete f;
    slot_item_done(fs, s);
}

bool help_with_a_part(FileStream& fs) {
    if (fs.n_parts.load(std::memory_order_acquire) == 0) return false;
    PartTask t;
    {
        std::lock_guard<std::mutex> g(fs.c->qmu);
        if (fs.parts.empty()) return false;
        t = fs.parts.front();
        fs.parts.pop_front();
        fs.n_parts.fetch_sub(1);
    }
    run_part(fs, t);
    return true;
}

void reader_loop(FileStream& fs) {
    oxh_ctx* c = fs.c;
    FileRequest* r = nullptr;
    uint64_t i0 = 0, i1 = 0;
    bool stop = false;
    PartTask pt;
    while (!stop && claim(fs, r, i0, i1, pt)) {
        if (pt.f) {
            run_part(fs, pt);
            pt = PartTask{};
            continue;
        }
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
            struct stat fsb;
            if (L >= kSplitBytes && fs.nreaders > 1 && split_reads() && fstat(fd, &fsb) == 0) {  // parts for the
                // other readers; part 0 here
                auto* f = new PartFile;
                f->r = r, f->i = i, f->j = j, f->L = L, f->s = s, f->dst = c->h_stage[s] + off;
                f->dev = fsb.st_dev, f->ino = fsb.st_ino;
                snprintf(f->link, sizeof f->link, "/proc/self/task/%ld/fd/%d", (long)syscall(SYS_gettid), fd);
                const uint64_t nparts = (L + kPartBytes) / kPartBytes;  // over [0, L + 1)
                f->left.store((int)nparts);
                {
                    std::lock_guard<std::mutex> g(c->qmu);
                    for (uint64_t k = 1; k < nparts; ++k)
                        fs.parts.push_back({f, k * kPartBytes, std::min(L + 1, (k + 1) * kPartBytes)});
                    fs.n_parts.fetch_add(nparts - 1);
                }
                c->qcv.notify_all();
                run_part(fs, {f, 0, kPartBytes}, fd);
                // the descriptor stays open until every other part has reopened it (this reader reads
                // queued parts meanwhile, its own among them, so the wait always ends)
                while (f->opened.load(std::memory_order_acquire) < (int)nparts - 1 && !fs.abort.load(std::memory_order_relaxed))
                    if (!help_with_a_part(fs)) pause_us(2);
                close(fd);
                if (f->refs.fetch_sub(1, std::memory_order_acq_rel) == 1) delete f;
                continue;
            }
            int e = 0;
            const int64_t got = read_expected(fd, c->h_stage[s] + off, L, e);
            close(fd);
            if (got < 0) item_failed(r, i, OXH_ERR_IO, e);
            if (got >= 0 && (uint64_t)got != L) item_resized(fs, r, i, s, j);  // not the size the stat / the caller saw
            slot_item_done(fs, s);
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
    c->n_runs.fetch_add(1, std::memory_order_relaxed);
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
        {  // parts no reader took (the run aborted): their files' descriptors and state
            std::vector<PartFile*> left;
            for (const PartTask& t : fs.parts)
                if (std::find(left.begin(), left.end(), t.f) == left.end()) left.push_back(t.f);
            fs.parts.clear();
            for (PartFile* f : left) delete f;
        }
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
    oxh::runtime_thread_timer_slack();  // pool.hpp: the engine's 20 us polls are not stretched to 70
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

}  // namespace oxh::capi

namespace oxh::capi {

// A caller that has waited OXH_WAIT_LIMIT_S (default 60 s) for its request prints the engine's state
// (once per period) and keeps waiting: the engine may still write into the request.
void dump_engine(oxh_ctx* c, const FileRequest& r) {
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

// Small requests on an idle context: the caller's own thread does what an engine run would do for them
// -- open + fstat (or the caller's size), pread into staging slot 0, one submit, wait -- with none of a
// run's hand-offs (engine wake-up, reader-pool start, the readers' idle handshake, the engine's 20 us
// drain poll, the caller's wake-up), which cost ~60 of a one-file call's ~100 us (DESIGN §5 "Per-call
// latency"). This is the shape of the per-file callers (hash_file_contents from restore, checkout, the
// metadata CLI). Requests of more files, or more bytes, or arriving while a run is live keep the engine,
// where concurrent requests share slots and reads run in parallel. The outputs are the engine's: the
// same reads (read_expected), statuses, errnos and kernels; a file whose size changed between its stat
// and its read hands the whole request back to the engine, whose refresh path re-reads it.
// OXH_DIRECT_FILES=0 turns it off (A/B, and the tests that compare both forms).
constexpr uint64_t kDirectFiles = 8, kDirectBytes = 2ull << 20;

// OXH_OK / an error: the request is done. kDirectDeclined: the engine runs it (r is as it was).
constexpr int kDirectDeclined = -1;

int direct_files(oxh_ctx* c, FileRequest& r) {
    const uint64_t n = r.n;
    if (n > kDirectFiles || n > c->max_items) return kDirectDeclined;
    const char* env = getenv("OXH_DIRECT_FILES");
    if (env && atoi(env) == 0) return kDirectDeclined;
    {
        std::lock_guard<std::mutex> g(c->qmu);
        if (c->live || !c->queue.empty()) return kDirectDeclined;
    }
    // the slots are the holder's (an engine run, a buffer call, the large-item path): never wait for one
    std::unique_lock<std::mutex> lk(c->mu, std::try_to_lock);
    if (!lk.owns_lock()) return kDirectDeclined;
    int fds[kDirectFiles];
    auto decline = [&](uint64_t upto) {
        for (uint64_t i = 0; i < upto; ++i)
            if (fds[i] >= 0) close(fds[i]);
        r.lens.assign(n, 0);
        r.st.assign(n, OXH_OK);
        r.eno.assign(n, 0);
        return kDirectDeclined;
    };
    // 1. open + fstat, as reader_loop does
    uint64_t room = 0;
    for (uint64_t i = 0; i < n; ++i) {
        fds[i] = -1;
        struct stat sb;
        const int fd = r.paths[i] ? open(r.paths[i], O_RDONLY | O_CLOEXEC | O_NONBLOCK) : -1;
        if (fd < 0) {
            item_failed(&r, i, OXH_ERR_OPEN, r.paths[i] ? errno : EINVAL);
            continue;
        }
        const bool meta = r.meta != nullptr && r.meta[i] < c->stage_bytes;
        if (!meta && (fstat(fd, &sb) != 0 || !S_ISREG(sb.st_mode))) {
            item_failed(&r, i, OXH_ERR_IO, unreadable_errno(fd, sb));
            close(fd);
            continue;
        }
        fds[i] = fd;
        r.lens[i] = meta ? r.meta[i] : (uint64_t)sb.st_size;
        room += align_up(r.lens[i] + 1);
        if (r.lens[i] >= c->stage_bytes || room > kDirectBytes || room > c->stage_bytes) return decline(i + 1);
    }
    const int prev_dev = [] {
        int d = 0;
        (void)hipGetDevice(&d);
        return d;
    }();
    if (hipSetDevice(c->device) != hipSuccess) {
        decline(n);
        return fail(OXH_ERR_HIP, "hipSetDevice failed");
    }
    struct RestoreDevice {  // the caller's thread keeps its current device
        int d;
        ~RestoreDevice() { (void)hipSetDevice(d); }
    } restore{prev_dev};
    // 2. read into slot 0 at the engine's placement (256-B aligned, one spare byte per item)
    const int s = 0;
    const uint64_t M = c->max_items;
    uint64_t* hoff = c->h_desc[s];
    uint64_t* hlen = c->h_desc[s] + M;
    uint64_t idx[kDirectFiles];
    uint64_t off = 0, cnt = 0, bytes = 0;
    for (uint64_t i = 0; i < n; ++i) {
        if (fds[i] < 0) continue;
        const uint64_t L = r.lens[i];
        int e = 0;
        const int64_t got = read_expected(fds[i], c->h_stage[s] + off, L, e);
        close(fds[i]);
        fds[i] = -1;
        if (got < 0) {
            item_failed(&r, i, OXH_ERR_IO, e);
            continue;
        }
        if ((uint64_t)got != L) return decline(n);  // its size changed: the engine's refresh path
        hoff[cnt] = off;
        hlen[cnt] = L;
        idx[cnt++] = i;
        bytes = off + L;
        off += align_up(L + 1);
    }
    // 3. one batch: H2D, K1 / K1T (+ is_utf8), D2H -- the engine's submit
    if (cnt) {
        c->where.store("direct: submit_slot");
        const bool text = r.counts != nullptr, utf8 = r.utf8 != nullptr;
        bool packed = false;
        if (int rc = submit_packed(c, s, bytes, cnt, bytes / cnt <= kShortItemBytes, text, utf8, packed)) return rc;
        if (!packed)
            if (int rc = submit_slot(c, s, bytes, cnt, false, bytes / cnt <= kShortItemBytes, text, utf8)) return rc;
        Pending p;
        p.busy = true;
        p.ids.assign(idx, idx + cnt);
        c->where.store("direct: wait_slot");
        if (int rc = wait_slot(c, s, p)) return rc;
        c->where.store("direct: done");
        for (uint64_t j = 0; j < cnt; ++j) {
            const uint64_t i = idx[j];
            r.out[2 * i] = c->h_out[s][2 * j];
            r.out[2 * i + 1] = c->h_out[s][2 * j + 1];
            if (text) {
                r.counts[2 * i] = c->h_cnt[s][2 * j];
                r.counts[2 * i + 1] = c->h_cnt[s][2 * j + 1];
            }
            if (utf8) r.utf8[i] = c->h_utf8[s][j];
            if (r.sink) r.sink->put(i, c->h_stage[s] + hoff[j], hlen[j], r.out[2 * i], r.out[2 * i + 1]);
        }
        if (r.sink) r.sink->commit();
    }
    write_outputs(&r);
    c->n_direct.fetch_add(1, std::memory_order_relaxed);
    return OXH_OK;
}

int hash_files_impl(oxh_ctx* c, const char* const* paths, uint64_t n, uint64_t* out, uint64_t* sizes, int32_t* status,
                    uint64_t* counts, ItemSink* sink, int32_t* utf8, const uint64_t* meta, int32_t* os_error) {
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
    if (const int d = direct_files(c, r); d != kDirectDeclined) return d;
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

}  // namespace oxh::capi

extern "C" {

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

}  // extern "C"
