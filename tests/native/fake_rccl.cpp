// tests/native/fake_rccl.cpp -- TEST DOUBLE, never shipped: a stand-in "RCCL" that lets the digest
// gather of the C ABI (oxen_amd/csrc/comm.cpp, oxh_gather_digests) run with N ranks as N processes
// that all use device 0 of a one-GPU box, where the real RCCL refuses two ranks on one device
// (profiles/r05/r05i_comm_two_ranks_one_gpu.txt). Loaded through OXH_RCCL_LIB; it exports the eleven
// symbols comm.cpp resolves (ncclGather only when built without -DFAKE_NO_GATHER, so the "RCCL
// without ncclGather" branch is testable too).
//
// Mechanics. ncclGetUniqueId creates a POSIX shared-memory region and writes its name into the id;
// every rank maps it in ncclCommInitRank. A region holds a process-shared barrier, one directory of
// posted buffers per rank and one data slot per rank. An operation (or a whole ncclGroupStart/End
// group) runs in two phases: POST -- the stream is synchronised and every buffer this rank sends is
// copied device-to-host into its own slot with a directory entry {kind, peer, seq, bytes} -- then a
// barrier, then FETCH -- every buffer this rank receives is found in the owner's directory by the
// same matching rule RCCL uses (collectives by issue order, send/recv by per-peer order), checked
// for size and copied host-to-device on the op's stream (not waited for: it lands in stream order,
// as RCCL's kernel would) -- then a barrier. Each entry counts its
// readers; after the second barrier every rank checks that its own entries were read exactly as
// often as the call pattern requires (an all-gather by every rank, a gather by the root, a send by
// its peer). Any mismatch -- unmatched send, size disagreement, wrong root -- is ncclInvalidUsage
// with a line on stderr, so the double is stricter than the real library about call patterns.
// Every rank must enter every group (an empty one included) and every collective, as comm.cpp does.
// Everything else is synchronous; a barrier that waits longer than OXH_FAKE_RCCL_TIMEOUT_S (default 60 s)
// fails with ncclSystemError instead of hanging the test.
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <fcntl.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <cstdint>
#include <string>
#include <vector>

namespace {

constexpr int kMaxRanks = 16;
constexpr int kMaxDir = 512;
constexpr uint64_t kHeaderBytes = 1 << 20;

enum Kind : uint32_t { kAllGather = 1, kGather = 2, kBcast = 3, kSend = 4 };

struct Entry {
    uint32_t kind;
    int32_t peer;   // send: destination; gather/bcast: root
    uint32_t seq;   // collectives: issue index in this communicator; send: per-peer index
    uint32_t pad;
    uint64_t off, bytes;  // in the owner's slot
    std::atomic<uint32_t> reads;
};

struct RankDir {
    uint32_t n;
    Entry e[kMaxDir];
};

struct Header {
    uint64_t magic, slot_bytes;
    std::atomic<uint32_t> nranks, joined, live, bar_count, bar_gen;
    RankDir dir[kMaxRanks];
};
static_assert(sizeof(Header) <= kHeaderBytes, "header");
static_assert(std::atomic<uint32_t>::is_always_lock_free, "process-shared atomics");
constexpr uint64_t kMagic = 0x6f78685f66616b65ull;  // "oxh_fake"

struct Op {
    Kind kind;
    const void* send;
    void* recv;
    uint64_t bytes;  // per rank
    int peer;        // root / send-recv peer
    bool is_recv;
    hipStream_t st;
};

}  // namespace

struct ncclComm {
    Header* h = nullptr;
    uint8_t* data = nullptr;
    size_t map_bytes = 0;
    std::string name;
    int rank = 0, nranks = 1;
    uint32_t coll_seq = 0;
    std::vector<uint32_t> sent, recvd;  // per-peer send/recv indices
};

namespace {

thread_local int g_group = 0;
thread_local std::vector<std::pair<ncclComm*, Op>> g_ops;
// The communicator an EMPTY group synchronises on: NCCL lets a rank with nothing to send or receive
// skip a point-to-point group, but this double runs every group through the region's barriers, so a
// rank that enters a group with no ops (comm.cpp's gather: every rank opens and closes the group, a
// zero-count rank issues nothing in it) still meets the others there -- on the comm it last used.
thread_local ncclComm* g_last = nullptr;

// one stderr line; `fmt` takes a %s (a) and then a %ld (b), either may be unused
void fail(const char* fmt, const std::string& a = "", long b = 0) {
    fprintf(stderr, "fake_rccl: ");
    fprintf(stderr, fmt, a.c_str(), b);
    fprintf(stderr, "\n");
}

double timeout_s() {
    const char* t = getenv("OXH_FAKE_RCCL_TIMEOUT_S");
    return t && *t ? atof(t) : 60.0;
}

double now_s() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

// sense-by-generation barrier over the region's two counters
bool barrier(ncclComm* c) {
    Header* h = c->h;
    const uint32_t gen = h->bar_gen.load(std::memory_order_acquire);
    if (h->bar_count.fetch_add(1, std::memory_order_acq_rel) + 1 == (uint32_t)c->nranks) {
        h->bar_count.store(0, std::memory_order_relaxed);
        h->bar_gen.fetch_add(1, std::memory_order_release);
        return true;
    }
    const double deadline = now_s() + timeout_s();
    for (unsigned spin = 0; h->bar_gen.load(std::memory_order_acquire) == gen; ++spin) {
        if (spin > 1000) {
            if (now_s() > deadline) {
                fail("rank %s: barrier timed out (%ld ranks expected)", std::to_string(c->rank), c->nranks);
                return false;
            }
            usleep(50);
        } else {
            sched_yield();
        }
    }
    return true;
}

size_t type_bytes(ncclDataType_t t) {
    switch (t) {
        case ncclInt8: case ncclUint8: return 1;
        case ncclFloat16: case ncclBfloat16: return 2;
        case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
        case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
        default: return 0;
    }
}

bool check_hip(hipError_t e, const char* what) {
    if (e == hipSuccess) return true;
    fail("%s failed: %ld", what, (long)e);
    return false;
}

Entry* find(ncclComm* c, int owner, Kind kind, int peer, uint32_t seq) {
    RankDir& d = c->h->dir[owner];
    for (uint32_t i = 0; i < d.n; ++i) {
        Entry& e = d.e[i];
        if (e.seq == seq && (kind == kSend ? (e.kind == kSend && e.peer == peer) : e.kind != kSend)) return &e;
    }
    return nullptr;
}

// POST + barrier + FETCH + barrier + read-count check for one op or one group of ops of one comm
ncclResult_t run(ncclComm* c, std::vector<Op>& ops) {
    RankDir& mine = c->h->dir[c->rank];
    mine.n = 0;
    uint64_t used = 0;
    bool ok = true;
    std::vector<uint32_t> coll(ops.size(), 0), pseq(ops.size(), 0);
    // POST
    for (size_t i = 0; i < ops.size() && ok; ++i) {
        Op& o = ops[i];
        const bool coll_op = o.kind != kSend;
        if (coll_op) coll[i] = c->coll_seq++;
        else pseq[i] = o.is_recv ? c->recvd[o.peer]++ : c->sent[o.peer]++;
        const bool posts = o.kind == kAllGather || o.kind == kGather || (o.kind == kBcast && o.peer == c->rank) ||
                           (o.kind == kSend && !o.is_recv);
        if (!posts) continue;
        if (mine.n >= (uint32_t)kMaxDir || used + o.bytes > c->h->slot_bytes) {
            fail("rank %s: slot full (%ld bytes)", std::to_string(c->rank), (long)(used + o.bytes));
            ok = false;
            break;
        }
        Entry& e = mine.e[mine.n];
        e.kind = o.kind, e.peer = o.peer, e.seq = coll_op ? coll[i] : pseq[i], e.off = used, e.bytes = o.bytes;
        e.reads.store(0, std::memory_order_relaxed);
        if (o.bytes) {
            ok = check_hip(hipStreamSynchronize(o.st), "hipStreamSynchronize") &&
                 check_hip(hipMemcpyAsync(c->data + c->rank * c->h->slot_bytes + used, o.send, o.bytes,
                                          hipMemcpyDeviceToHost, o.st), "hipMemcpyAsync D2H") &&
                 check_hip(hipStreamSynchronize(o.st), "hipStreamSynchronize");
        }
        used += (o.bytes + 255) / 256 * 256;
        std::atomic_thread_fence(std::memory_order_release);
        ++mine.n;
    }
    if (!barrier(c)) return ncclSystemError;
    // FETCH (a rank that failed its POST still takes part in both barriers, then reports)
    for (size_t i = 0; i < ops.size() && ok; ++i) {
        Op& o = ops[i];
        std::vector<std::pair<int, uint64_t>> srcs;  // (owner, destination offset)
        if (o.kind == kAllGather || (o.kind == kGather && o.peer == c->rank)) {
            for (int q = 0; q < c->nranks; ++q) srcs.push_back({q, q * o.bytes});
        } else if (o.kind == kBcast) {
            srcs.push_back({o.peer, 0});
        } else if (o.kind == kSend && o.is_recv) {
            srcs.push_back({o.peer, 0});
        }
        for (auto [q, dst] : srcs) {
            Entry* e = o.kind == kSend ? find(c, q, kSend, c->rank, pseq[i]) : find(c, q, o.kind, 0, coll[i]);
            if (!e) {
                fail("rank %s: no matching post from rank %ld", std::to_string(c->rank), q);
                ok = false;
                break;
            }
            if (e->kind != (uint32_t)o.kind || e->bytes != o.bytes || (o.kind != kSend && o.kind != kAllGather && e->peer != o.peer)) {
                fail("rank %s: op disagrees with rank %ld's (kind/root/size)", std::to_string(c->rank), q);
                ok = false;
                break;
            }
            // No wait for the copy to land: like RCCL's kernel, it completes on the op's stream, so a
            // caller that reads the table without ordering after that stream reads stale bytes. A
            // pageable-source copy returns once the source is staged, so the slot may be reused after.
            if (o.bytes)
                ok = check_hip(hipMemcpyAsync((uint8_t*)o.recv + dst, c->data + q * c->h->slot_bytes + e->off, o.bytes,
                                              hipMemcpyHostToDevice, o.st), "hipMemcpyAsync H2D");
            e->reads.fetch_add(1, std::memory_order_acq_rel);
            if (!ok) break;
        }
    }
    if (!barrier(c)) return ncclSystemError;
    // every posted buffer read exactly as the call pattern requires: an all-gather or broadcast
    // buffer by every rank (the root included), a gather buffer by the root, a send by its peer.
    // Only this rank's own directory is read here, and no rank rewrites its directory before the
    // next op's POST, which every other rank's FETCH of this op precedes (the second barrier).
    for (uint32_t i = 0; i < mine.n && ok; ++i) {
        const Entry& e = mine.e[i];
        const uint32_t want = e.kind == kAllGather || e.kind == kBcast ? (uint32_t)c->nranks : 1u;
        const uint32_t got = e.reads.load(std::memory_order_acquire);
        if (got != want) {
            fail("rank %s: a posted buffer was read %ld times", std::to_string(c->rank), (long)got);
            ok = false;
        }
    }
    return ok ? ncclSuccess : ncclInvalidUsage;
}

ncclResult_t submit(ncclComm* c, const Op& o) {
    if (!c || !c->h) return ncclInvalidArgument;
    if (o.peer < 0 || o.peer >= c->nranks) return ncclInvalidArgument;
    g_last = c;
    if (g_group > 0) {
        g_ops.push_back({c, o});
        return ncclSuccess;
    }
    std::vector<Op> one{o};
    return run(c, one);
}

}  // namespace

extern "C" {

__attribute__((visibility("default"))) ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
    if (!id) return ncclInvalidArgument;
    static std::atomic<unsigned> counter{0};
    timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    char name[96];
    snprintf(name, sizeof name, "/oxh_fake_rccl.%d.%u.%lx", (int)getpid(), counter++, (unsigned long)ts.tv_nsec);
    const int fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0) return ncclSystemError;
    const char* sb = getenv("OXH_FAKE_RCCL_SLOT_BYTES");
    const uint64_t slot = sb && *sb ? strtoull(sb, nullptr, 10) : (64ull << 20);
    const uint64_t total = kHeaderBytes + kMaxRanks * slot;
    if (ftruncate(fd, (off_t)total) != 0) {
        close(fd);
        shm_unlink(name);
        return ncclSystemError;
    }
    void* p = mmap(nullptr, kHeaderBytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) {
        shm_unlink(name);
        return ncclSystemError;
    }
    auto* h = static_cast<Header*>(p);  // tmpfs pages start zeroed: the counters are 0
    h->slot_bytes = slot;
    std::atomic_thread_fence(std::memory_order_release);
    h->magic = kMagic;
    munmap(p, kHeaderBytes);
    memset(id->internal, 0, sizeof id->internal);
    memcpy(id->internal, name, strlen(name));
    return ncclSuccess;
}

__attribute__((visibility("default"))) ncclResult_t ncclCommInitRank(ncclComm_t* out, int nranks, ncclUniqueId id, int rank) {
    if (!out || nranks < 1 || nranks > kMaxRanks || rank < 0 || rank >= nranks) return ncclInvalidArgument;
    char name[sizeof id.internal + 1] = {0};
    memcpy(name, id.internal, sizeof id.internal);
    const int fd = shm_open(name, O_RDWR, 0600);
    if (fd < 0) {
        fail("cannot open region %s", name);
        return ncclSystemError;
    }
    struct stat sst;
    if (fstat(fd, &sst) != 0) {
        close(fd);
        return ncclSystemError;
    }
    void* p = mmap(nullptr, (size_t)sst.st_size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) return ncclSystemError;
    auto* c = new ncclComm;
    c->h = static_cast<Header*>(p);
    c->data = static_cast<uint8_t*>(p) + kHeaderBytes;
    c->map_bytes = (size_t)sst.st_size;
    c->name = name;
    c->rank = rank, c->nranks = nranks;
    c->sent.assign(nranks, 0), c->recvd.assign(nranks, 0);
    g_last = c;
    uint32_t expect = 0;
    if (c->h->magic != kMagic ||
        (!c->h->nranks.compare_exchange_strong(expect, (uint32_t)nranks) && expect != (uint32_t)nranks)) {
        fail("region %s: bad magic or rank count", name);
        munmap(p, c->map_bytes);
        delete c;
        return ncclInvalidUsage;
    }
    c->h->joined.fetch_add(1);
    c->h->live.fetch_add(1);
    if (!barrier(c)) {  // like ncclCommInitRank: returns once every rank has joined
        c->h->live.fetch_sub(1);
        munmap(p, c->map_bytes);
        delete c;
        return ncclSystemError;
    }
    *out = c;
    return ncclSuccess;
}

__attribute__((visibility("default"))) ncclResult_t ncclCommDestroy(ncclComm_t c) {
    if (!c) return ncclSuccess;
    if (g_last == c) g_last = nullptr;
    if (c->h->live.fetch_sub(1) == 1) shm_unlink(c->name.c_str());  // the last rank out removes the region
    munmap(c->h, c->map_bytes);
    delete c;
    return ncclSuccess;
}

__attribute__((visibility("default"))) ncclResult_t ncclAllGather(const void* send, void* recv, size_t count, ncclDataType_t t,
                                                                  ncclComm_t c, hipStream_t st) {
    if (!type_bytes(t)) return ncclInvalidArgument;
    return submit(c, Op{kAllGather, send, recv, count * type_bytes(t), 0, false, st});
}

#ifndef FAKE_NO_GATHER
__attribute__((visibility("default"))) ncclResult_t ncclGather(const void* send, void* recv, size_t count, ncclDataType_t t,
                                                               int root, ncclComm_t c, hipStream_t st) {
    if (!type_bytes(t)) return ncclInvalidArgument;
    return submit(c, Op{kGather, send, recv, count * type_bytes(t), root, false, st});
}
#endif

__attribute__((visibility("default"))) ncclResult_t ncclBroadcast(const void* send, void* recv, size_t count, ncclDataType_t t,
                                                                  int root, ncclComm_t c, hipStream_t st) {
    if (!type_bytes(t)) return ncclInvalidArgument;
    return submit(c, Op{kBcast, send, recv, count * type_bytes(t), root, false, st});
}

__attribute__((visibility("default"))) ncclResult_t ncclSend(const void* send, size_t count, ncclDataType_t t, int peer,
                                                             ncclComm_t c, hipStream_t st) {
    if (!type_bytes(t) || (c && peer == c->rank)) return ncclInvalidArgument;
    return submit(c, Op{kSend, send, nullptr, count * type_bytes(t), peer, false, st});
}

__attribute__((visibility("default"))) ncclResult_t ncclRecv(void* recv, size_t count, ncclDataType_t t, int peer,
                                                             ncclComm_t c, hipStream_t st) {
    if (!type_bytes(t) || (c && peer == c->rank)) return ncclInvalidArgument;
    return submit(c, Op{kSend, nullptr, recv, count * type_bytes(t), peer, true, st});
}

__attribute__((visibility("default"))) ncclResult_t ncclGroupStart() {
    ++g_group;
    return ncclSuccess;
}

__attribute__((visibility("default"))) ncclResult_t ncclGroupEnd() {
    if (g_group <= 0) return ncclInvalidUsage;
    if (--g_group > 0) return ncclSuccess;
    auto ops = std::move(g_ops);
    g_ops.clear();
    // one communicator per group in this double (comm.cpp issues one group per gather)
    ncclComm* c = ops.empty() ? g_last : ops[0].first;
    if (!c) return ncclSuccess;
    std::vector<Op> list;
    for (auto& [oc, o] : ops) {
        if (oc != c) return ncclInvalidUsage;
        list.push_back(o);
    }
    return run(c, list);
}

__attribute__((visibility("default"))) const char* ncclGetErrorString(ncclResult_t r) {
    switch (r) {
        case ncclSuccess: return "no error (fake RCCL)";
        case ncclInvalidArgument: return "invalid argument (fake RCCL)";
        case ncclInvalidUsage: return "invalid usage (fake RCCL): ranks disagree on the call pattern";
        case ncclSystemError: return "system error (fake RCCL): shared memory or barrier timeout";
        default: return "error (fake RCCL)";
    }
}

}  // extern "C"
