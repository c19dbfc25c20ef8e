// oxen_amd/csrc/hash_helper.cpp -> oxen_amd/oxh_hash_helper: one reader process of an oxh_pool
// (reader_pool.cpp). Started by oxh_pool_create with its socket on fd 200 and the pool's shared
// region on fd 201; creates one context on --device with --threads reader threads, reports, then
// serves requests (its share [lo, hi) of a call's list through oxh_hash_files_ex, outputs written
// into the region in place) until told to quit, its socket closes, or its parent process dies.
// Parent death is seen as the socket's hang-up or a changed getppid() (checked every second while
// idle), not through PR_SET_PDEATHSIG, which fires when the spawning THREAD exits: a pool created on
// a short-lived thread (a tokio spawn_blocking worker, a Python thread) must keep its helpers.
#include <errno.h>
#include <poll.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <unistd.h>

#include <string>
#include <vector>

#include "../../include/oxen_hash.h"
#include "reader_pool.hpp"

using oxh_pool_wire::PoolRep;
using oxh_pool_wire::PoolReq;

namespace {

long arg(int argc, char** argv, const char* key, long dflt) {
    const size_t k = strlen(key);
    for (int i = 1; i < argc; ++i)
        if (strncmp(argv[i], key, k) == 0 && argv[i][k] == '=') return atol(argv[i] + k + 1);
    return dflt;
}

bool reply(int sock, uint64_t seq, int rc, const char* msg) {
    PoolRep r{};
    r.seq = seq;
    r.rc = rc;
    r.pid = (int)getpid();
    snprintf(r.msg, sizeof r.msg, "%s", msg ? msg : "");
    return send(sock, &r, sizeof r, MSG_NOSIGNAL) == (ssize_t)sizeof r;
}

}  // namespace

int main(int argc, char** argv) {
    const int sock = oxh_pool_wire::kSockFd, mem = oxh_pool_wire::kMemFd;
    const long ppid = arg(argc, argv, "--ppid", 0);
    if (ppid && getppid() != (pid_t)ppid) return 1;  // the parent died before this helper started
    const int device = (int)arg(argc, argv, "--device", 0);
    const long threads = arg(argc, argv, "--threads", 0);
    const uint64_t staging = (uint64_t)arg(argc, argv, "--staging", 0);
    if (threads > 0) setenv("OXH_NUM_THREADS", std::to_string(threads).c_str(), 1);

    oxh_ctx* ctx = nullptr;
    int rc = oxh_ctx_create(device, staging, &ctx);
    if (!reply(sock, 0, rc, rc ? oxh_last_error() : "")) return 2;
    if (rc) return 3;

    uint8_t* map = nullptr;
    uint64_t cap = 0;
    std::vector<const char*> ptrs;
    for (;;) {
        // idle: wake every second to see whether the parent process is still there (after its death
        // this process is re-parented, and its socket may stay open in a forked child of the parent)
        pollfd pf{sock, POLLIN, 0};
        const int ready = poll(&pf, 1, 1000);
        if (ready < 0 && errno != EINTR) break;
        if (ready <= 0) {
            if (ppid && getppid() != (pid_t)ppid) break;
            continue;
        }
        PoolReq q{};
        const ssize_t k = recv(sock, &q, sizeof q, 0);
        if (k != (ssize_t)sizeof q || q.quit) break;
        if (q.cap != cap) {
            if (map) munmap(map, cap);
            void* m = mmap(nullptr, q.cap, PROT_READ | PROT_WRITE, MAP_SHARED, mem, 0);
            if (m == MAP_FAILED) {
                map = nullptr, cap = 0;
                if (!reply(sock, q.seq, OXH_ERR_NOMEM, "helper: mmap of the pool region failed")) break;
                continue;
            }
            map = (uint8_t*)m, cap = q.cap;
        }
        if (q.hi < q.lo || q.hi > q.n || q.off_blob > cap) {
            if (!reply(sock, q.seq, OXH_ERR_INVALID, "helper: malformed request")) break;
            continue;
        }
        const uint64_t m = q.hi - q.lo;
        const uint64_t* offs = (const uint64_t*)(map + q.off_offs);
        const char* blob = (const char*)(map + q.off_blob);
        ptrs.resize(m);
        for (uint64_t i = 0; i < m; ++i) ptrs[i] = blob + offs[q.lo + i];
        uint64_t* out = (uint64_t*)(map + q.off_out) + 2 * q.lo;
        uint64_t* sizes = (uint64_t*)(map + q.off_sizes) + q.lo;
        int32_t* status = (int32_t*)(map + q.off_status) + q.lo;
        int32_t* os_error = (int32_t*)(map + q.off_oserr) + q.lo;
        rc = oxh_hash_files_ex(ctx, ptrs.data(), q.has_meta ? (const uint64_t*)(map + q.off_meta) + q.lo : nullptr, m, out,
                               sizes, status, os_error, nullptr, nullptr);
        if (!reply(sock, q.seq, rc, rc ? oxh_last_error() : "")) break;
    }
    if (map) munmap(map, cap);
    oxh_ctx_destroy(ctx);
    return 0;
}
