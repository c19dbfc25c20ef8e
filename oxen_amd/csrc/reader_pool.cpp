// oxen_amd/csrc/reader_pool.cpp -- oxh_pool: a file list hashed by several helper PROCESSES, each with
// its own context (include/oxen_hash.h, "reader-process pool").
//
// Why processes: on the MI355X boxes the warm-cache floor of reading many small files is open() +
// close() themselves, and it belongs to the process -- 200 000 open + close pairs take 0.28 s in one
// process whatever its thread count, 0.16 s in two, 0.13 s in four (tools/open_probe.cpp, PROCS=P,
// profiles/r02e_open_procs.json). One context's engine lives in one process, so it sits on that floor.
// The reference's add loop fans 64-file batches out over num_cpus * 2 tokio tasks of ONE process
// (core/v_latest/add.rs:422-425); a liboxen built on this library creates one pool and hands it the
// whole list (or each batch) instead.
//
// Multi-GPU: helper p runs its context on devices[p % ndevices], so every GPU of a node is fed its
// own contiguous share of the list over its own PCIe link; shares are balanced by
// bytes when the caller passes sizes.
//
// Helpers are started with posix_spawn (fork + exec in the child: nothing of this process's GPU
// state is inherited), get the shared region and their socket as fixed descriptors, and exit when
// the pool is destroyed, when their socket closes, or when this process dies (the helper polls its
// socket and checks getppid(); PR_SET_PDEATHSIG is not used: it fires when the creating THREAD
// exits, so a pool created on a short-lived thread would lose its helpers with that thread).
#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <poll.h>
#include <signal.h>
#include <spawn.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/oxen_hash.h"
#include "reader_pool.hpp"

extern char** environ;

namespace oxh {
int set_error(int code, const std::string& msg);
int cpu_quota();
}  // namespace oxh

using oxh_pool_wire::PoolRep;
using oxh_pool_wire::PoolReq;

struct oxh_pool {
    struct Helper {
        pid_t pid = -1;
        int sock = -1;
        int device = 0;
    };
    std::mutex mu;  // one call at a time (a call already spreads over every helper)
    std::vector<Helper> helpers;
    int memfd = -1;
    uint8_t* map = nullptr;
    uint64_t cap = 0;
    uint64_t seq = 0;
    bool broken = false;
    std::string broken_msg;
};

namespace {

int fail(int code, const std::string& msg) { return oxh::set_error(code, msg); }

// oxh_hash_helper next to this library ($OXH_HELPER overrides)
std::string helper_path() {
    if (const char* e = getenv("OXH_HELPER")) return e;
    Dl_info info;
    if (dladdr((void*)&oxh_pool_create, &info) && info.dli_fname) {
        std::string so = info.dli_fname;
        const size_t slash = so.rfind('/');
        return (slash == std::string::npos ? std::string(".") : so.substr(0, slash)) + "/oxh_hash_helper";
    }
    return "oxh_hash_helper";
}

bool send_all(int fd, const void* p, size_t n) {
    for (;;) {
        const ssize_t k = send(fd, p, n, MSG_NOSIGNAL);
        if (k == (ssize_t)n) return true;
        if (k < 0 && errno == EINTR) continue;
        return false;
    }
}

bool recv_rep(int fd, PoolRep& r) {
    for (;;) {
        const ssize_t k = recv(fd, &r, sizeof r, 0);
        if (k == (ssize_t)sizeof r) return true;
        if (k < 0 && errno == EINTR) continue;
        return false;  // EOF: the helper exited
    }
}

// A call's reply from helper h. A helper that has not answered within OXH_WAIT_LIMIT_S seconds
// (default 60) is reported on stderr, like a stalled request of the in-process engine, and waited
// for further: a share of a large cold list can take that long. OXH_POOL_CALL_LIMIT_S (default 0 =
// no limit) turns the wait into a deadline: the call then fails and the pool is marked unusable.
// false: the helper exited, or the deadline passed.
bool wait_rep(int fd, pid_t pid, uint64_t seq, PoolRep& r) {
    const double report = getenv("OXH_WAIT_LIMIT_S") ? atof(getenv("OXH_WAIT_LIMIT_S")) : 60.0;
    const double limit = getenv("OXH_POOL_CALL_LIMIT_S") ? atof(getenv("OXH_POOL_CALL_LIMIT_S")) : 0.0;
    timespec t0;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    double next_report = report;
    for (;;) {
        pollfd pf{fd, POLLIN, 0};
        const int k = poll(&pf, 1, 1000);
        if (k > 0) return recv_rep(fd, r);
        if (k < 0 && errno != EINTR) return false;
        timespec t;
        clock_gettime(CLOCK_MONOTONIC, &t);
        const double waited = (double)(t.tv_sec - t0.tv_sec) + 1e-9 * (double)(t.tv_nsec - t0.tv_nsec);
        if (limit > 0 && waited >= limit) return false;
        if (report > 0 && waited >= next_report) {
            fprintf(stderr, "[oxh] reader pool: helper pid %d has not answered call %llu after %.0f s\n", (int)pid,
                    (unsigned long long)seq, waited);
            next_report += report;
        }
    }
}

void reap(oxh_pool* p, bool polite) {
    for (auto& h : p->helpers) {
        if (h.sock >= 0) {
            if (polite) {
                PoolReq q{};
                q.quit = 1;
                send_all(h.sock, &q, sizeof q);
            }
            close(h.sock);
            h.sock = -1;
        }
    }
    // helpers exit on quit or on EOF; give them 10 s to release their contexts, then kill
    const timespec step{0, 10 * 1000 * 1000};
    for (int waited = 0; waited < 1000; ++waited) {
        bool alive = false;
        for (auto& h : p->helpers)
            if (h.pid > 0) {
                const pid_t w = waitpid(h.pid, nullptr, WNOHANG);
                if (w == h.pid || (w < 0 && errno == ECHILD)) h.pid = -1;  // ECHILD: SIGCHLD ignored, reaped already
                else alive = true;
            }
        if (!alive) return;
        nanosleep(&step, nullptr);
    }
    for (auto& h : p->helpers)
        if (h.pid > 0) {
            kill(h.pid, SIGKILL);
            while (waitpid(h.pid, nullptr, 0) < 0 && errno == EINTR) {
            }
            h.pid = -1;
        }
}

void destroy(oxh_pool* p, bool polite) {
    reap(p, polite);
    if (p->map) munmap(p->map, p->cap);
    if (p->memfd >= 0) close(p->memfd);
    delete p;
}

int grow(oxh_pool* p, uint64_t need) {
    if (need <= p->cap) return OXH_OK;
    uint64_t cap = std::max<uint64_t>(need, 2 * p->cap);
    cap = (cap + (2u << 20) - 1) & ~((2ull << 20) - 1);
    if (ftruncate(p->memfd, (off_t)cap) != 0) return fail(OXH_ERR_NOMEM, std::string("pool region: ftruncate: ") + strerror(errno));
    void* m = mmap(nullptr, cap, PROT_READ | PROT_WRITE, MAP_SHARED, p->memfd, 0);
    if (m == MAP_FAILED) return fail(OXH_ERR_NOMEM, std::string("pool region: mmap: ") + strerror(errno));
    if (p->map) munmap(p->map, p->cap);
    p->map = (uint8_t*)m;
    p->cap = cap;
    return OXH_OK;
}

int mark_broken(oxh_pool* p, const std::string& why) {
    p->broken = true;
    p->broken_msg = why;
    // a helper may be stuck (the deadline case) or mid-call for another share: none of them is asked
    for (auto& h : p->helpers)
        if (h.pid > 0) kill(h.pid, SIGKILL);
    reap(p, false);
    return fail(OXH_ERR_HIP, why);
}

inline uint64_t al64(uint64_t x) { return (x + 63) & ~63ull; }

}  // namespace

extern "C" {

int oxh_pool_create(const int* devices, int ndevices, int procs, int threads, uint64_t staging_bytes, oxh_pool** out) {
    if (!out || procs < 1 || procs > 64 || ndevices < 0 || (ndevices > 0 && !devices))
        return fail(OXH_ERR_INVALID, "oxh_pool_create: bad arguments");
    if (staging_bytes > OXH_MAX_STAGING_BYTES) return fail(OXH_ERR_INVALID, "staging_bytes above OXH_MAX_STAGING_BYTES");
    *out = nullptr;
    if (threads <= 0) threads = std::max(1, std::min(16, oxh::cpu_quota() / procs));
    const std::string exe = helper_path();
    if (access(exe.c_str(), X_OK) != 0) return fail(OXH_ERR_INVALID, "reader pool helper not found: " + exe);

    oxh_pool* p = new oxh_pool;
    p->memfd = memfd_create("oxh_pool", MFD_CLOEXEC);
    if (p->memfd < 0) {
        delete p;
        return fail(OXH_ERR_NOMEM, std::string("memfd_create: ") + strerror(errno));
    }
    if (int rc = grow(p, 2u << 20)) {
        destroy(p, false);
        return rc;
    }
    // descriptors handed to a child sit above the fixed targets, so no dup2 of the spawn clobbers
    // another's source
    const int memsrc = fcntl(p->memfd, F_DUPFD_CLOEXEC, 300);
    std::string err;
    int err_rc = OXH_OK;
    for (int k = 0; k < procs && !err_rc; ++k) {
        oxh_pool::Helper h;
        h.device = ndevices > 0 ? devices[k % ndevices] : 0;
        int sv[2];
        if (socketpair(AF_UNIX, SOCK_SEQPACKET | SOCK_CLOEXEC, 0, sv) != 0) {
            err_rc = OXH_ERR_NOMEM, err = std::string("socketpair: ") + strerror(errno);
            break;
        }
        const int csrc = fcntl(sv[1], F_DUPFD_CLOEXEC, 300);
        close(sv[1]);
        posix_spawn_file_actions_t fa;
        posix_spawn_file_actions_init(&fa);
        posix_spawn_file_actions_adddup2(&fa, csrc, oxh_pool_wire::kSockFd);  // dup2 clears CLOEXEC
        posix_spawn_file_actions_adddup2(&fa, memsrc, oxh_pool_wire::kMemFd);
        const std::string a_dev = "--device=" + std::to_string(h.device), a_thr = "--threads=" + std::to_string(threads),
                          a_stg = "--staging=" + std::to_string(staging_bytes), a_pp = "--ppid=" + std::to_string(getpid());
        char* argv[] = {(char*)exe.c_str(), (char*)a_dev.c_str(), (char*)a_thr.c_str(), (char*)a_stg.c_str(),
                        (char*)a_pp.c_str(), nullptr};
        pid_t pid = -1;
        const int e = posix_spawn(&pid, exe.c_str(), &fa, nullptr, argv, environ);
        posix_spawn_file_actions_destroy(&fa);
        close(csrc);
        if (e != 0) {
            close(sv[0]);
            err_rc = OXH_ERR_INVALID, err = "posix_spawn " + exe + ": " + strerror(e);
            break;
        }
        h.pid = pid;
        h.sock = sv[0];
        p->helpers.push_back(h);
    }
    if (memsrc >= 0) close(memsrc);
    // every helper reports once its context exists (or why it could not create one)
    for (auto& h : p->helpers) {
        if (err_rc) break;
        PoolRep r{};
        if (!recv_rep(h.sock, r)) {
            err_rc = OXH_ERR_HIP, err = "reader pool helper exited during start-up (device " + std::to_string(h.device) + ")";
        } else if (r.rc != OXH_OK) {
            r.msg[sizeof r.msg - 1] = 0;
            err_rc = r.rc, err = std::string("reader pool helper (device ") + std::to_string(h.device) + "): " + r.msg;
        }
    }
    if (err_rc) {
        destroy(p, true);
        return fail(err_rc, err);
    }
    *out = p;
    return OXH_OK;
}

int oxh_pool_hash_files(oxh_pool* p, const char* const* paths, const uint64_t* meta_sizes, uint64_t n, uint64_t* out,
                        uint64_t* sizes, int32_t* status) {
    return oxh_pool_hash_files_ex(p, paths, meta_sizes, n, out, sizes, status, nullptr);
}

int oxh_pool_hash_files_ex(oxh_pool* p, const char* const* paths, const uint64_t* meta_sizes, uint64_t n, uint64_t* out,
                           uint64_t* sizes, int32_t* status, int32_t* os_error) {
    if (!p || (n && (!paths || !out))) return fail(OXH_ERR_INVALID, "oxh_pool_hash_files: bad arguments");
    std::lock_guard<std::mutex> lk(p->mu);
    if (p->broken) return fail(OXH_ERR_HIP, "reader pool is unusable: " + p->broken_msg);
    if (n == 0) return OXH_OK;
    for (uint64_t i = 0; i < n; ++i)
        if (!paths[i]) return fail(OXH_ERR_INVALID, "NULL path");
    const bool has_meta = meta_sizes != nullptr;
    std::vector<uint64_t> plen(n);
    uint64_t blob = 0;
    for (uint64_t i = 0; i < n; ++i) blob += (plen[i] = strlen(paths[i]) + 1);
    PoolReq q{};
    q.n = n;
    q.has_meta = has_meta;
    q.off_offs = 0;
    q.off_meta = al64(8 * n);
    q.off_out = q.off_meta + (has_meta ? al64(8 * n) : 0);
    q.off_sizes = q.off_out + al64(16 * n);
    q.off_status = q.off_sizes + al64(8 * n);
    q.off_oserr = q.off_status + al64(4 * n);
    q.off_blob = q.off_oserr + al64(4 * n);
    if (int rc = grow(p, q.off_blob + blob)) return rc;
    q.cap = p->cap;
    uint64_t* offs = (uint64_t*)(p->map + q.off_offs);
    uint8_t* b = p->map + q.off_blob;
    for (uint64_t i = 0, o = 0; i < n; o += plen[i], ++i) {
        offs[i] = o;
        memcpy(b + o, paths[i], plen[i]);
    }
    if (has_meta) memcpy(p->map + q.off_meta, meta_sizes, 8 * n);

    // contiguous shares, balanced by bytes (+4 KiB per file for its syscalls) when sizes are known
    const uint64_t P = p->helpers.size();
    std::vector<uint64_t> cut(P + 1, n);
    cut[0] = 0;
    if (has_meta) {
        long double total = 0;
        for (uint64_t i = 0; i < n; ++i) total += (long double)meta_sizes[i] + 4096;
        long double acc = 0;
        uint64_t k = 1, i = 0;
        for (; i < n && k < P; ++i) {
            acc += (long double)meta_sizes[i] + 4096;
            while (k < P && acc >= total * k / P) cut[k++] = i + 1;
        }
    } else {
        for (uint64_t k = 1; k < P; ++k) cut[k] = n * k / P;
    }
    q.seq = ++p->seq;
    std::vector<int> busy;
    for (uint64_t k = 0; k < P; ++k) {
        if (cut[k + 1] <= cut[k]) continue;
        q.lo = cut[k], q.hi = cut[k + 1];
        if (!send_all(p->helpers[k].sock, &q, sizeof q))
            return mark_broken(p, "reader pool helper (pid " + std::to_string(p->helpers[k].pid) + ") is gone");
        busy.push_back((int)k);
    }
    int rc = OXH_OK;
    std::string msg;
    for (int k : busy) {
        PoolRep r{};
        if (!wait_rep(p->helpers[k].sock, p->helpers[k].pid, q.seq, r) || r.seq != q.seq)
            return mark_broken(p, "reader pool helper (pid " + std::to_string(p->helpers[k].pid) +
                                      ") died during a call or missed OXH_POOL_CALL_LIMIT_S");
        if (r.rc != OXH_OK && rc == OXH_OK) {
            r.msg[sizeof r.msg - 1] = 0;
            rc = r.rc, msg = r.msg;
        }
    }
    if (rc) return fail(rc, "reader pool: " + msg);
    memcpy(out, p->map + q.off_out, 16 * n);
    if (sizes) memcpy(sizes, p->map + q.off_sizes, 8 * n);
    if (status) memcpy(status, p->map + q.off_status, 4 * n);
    if (os_error) memcpy(os_error, p->map + q.off_oserr, 4 * n);
    return OXH_OK;
}

int oxh_pool_size(oxh_pool* p, int* procs, int* pids) {
    if (!p || !procs) return fail(OXH_ERR_INVALID, "oxh_pool_size: bad arguments");
    std::lock_guard<std::mutex> lk(p->mu);
    *procs = (int)p->helpers.size();
    if (pids)
        for (size_t k = 0; k < p->helpers.size(); ++k) pids[k] = p->helpers[k].pid;
    return OXH_OK;
}

int oxh_pool_destroy(oxh_pool* p) {
    if (!p) return OXH_OK;
    {
        std::lock_guard<std::mutex> lk(p->mu);
    }
    destroy(p, true);
    return OXH_OK;
}

}  // extern "C"
