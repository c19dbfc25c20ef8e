// tests/native/fake_pool_helper.cpp -- a stand-in for oxen_amd/oxh_hash_helper that speaks the reader
// pool's wire protocol (oxen_amd/csrc/reader_pool.hpp) without a GPU, so the pool's mechanics --
// spawning, the shared region and its growth, share splitting, per-call sequence numbers, per-file
// statuses, helper death -- are tested on any host (tests/test_procpool.py, OXH_HELPER=<this>).
// Test infrastructure only: it computes no digest; "out" is (size, index of the file in the call)
// so the test can check that every item landed in its own slot. A missing path gets OXH_ERR_OPEN (7)
// with its stat errno, a directory OXH_ERR_IO (3) with EISDIR, like the real helper's engine.
// OXH_FAKE_STALL_S=s: every call's reply is held back s seconds (the pool's deadline test).
// Like the real helper it watches its socket and getppid() instead of PR_SET_PDEATHSIG.
#include <errno.h>
#include <poll.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdint>

#include "../../oxen_amd/csrc/reader_pool.hpp"

using oxh_pool_wire::PoolRep;
using oxh_pool_wire::PoolReq;

static bool reply(int sock, uint64_t seq, int rc, const char* msg) {
    PoolRep r{};
    r.seq = seq;
    r.rc = rc;
    r.pid = (int)getpid();
    snprintf(r.msg, sizeof r.msg, "%s", msg);
    return send(sock, &r, sizeof r, MSG_NOSIGNAL) == (ssize_t)sizeof r;
}

int main(int argc, char** argv) {
    const int sock = oxh_pool_wire::kSockFd, mem = oxh_pool_wire::kMemFd;
    int device = 0;
    long ppid = 0;
    for (int i = 1; i < argc; ++i) {
        if (strncmp(argv[i], "--device=", 9) == 0) device = atoi(argv[i] + 9);
        if (strncmp(argv[i], "--ppid=", 7) == 0) ppid = atol(argv[i] + 7);
    }
    const int stall = getenv("OXH_FAKE_STALL_S") ? atoi(getenv("OXH_FAKE_STALL_S")) : 0;
    // OXH_FAKE_FAIL_DEVICE=d: the helper on device d reports a start-up failure (status 5)
    const char* fd = getenv("OXH_FAKE_FAIL_DEVICE");
    if (fd && atoi(fd) == device) {
        reply(sock, 0, 5, "fake helper: no device");
        return 3;
    }
    if (!reply(sock, 0, 0, "")) return 2;
    uint8_t* map = nullptr;
    uint64_t cap = 0;
    for (;;) {
        pollfd pf{sock, POLLIN, 0};
        const int ready = poll(&pf, 1, 1000);
        if (ready < 0 && errno != EINTR) break;
        if (ready <= 0) {
            if (ppid && getppid() != (pid_t)ppid) break;  // the parent process is gone
            continue;
        }
        PoolReq q{};
        if (recv(sock, &q, sizeof q, 0) != (ssize_t)sizeof q || q.quit) break;
        if (q.cap != cap) {
            if (map) munmap(map, cap);
            map = (uint8_t*)mmap(nullptr, q.cap, PROT_READ | PROT_WRITE, MAP_SHARED, mem, 0);
            cap = map == MAP_FAILED ? 0 : q.cap;
            if (!cap) {
                map = nullptr;
                reply(sock, q.seq, 4, "fake helper: mmap");
                continue;
            }
        }
        const uint64_t* offs = (const uint64_t*)(map + q.off_offs);
        const uint64_t* meta = q.has_meta ? (const uint64_t*)(map + q.off_meta) : nullptr;
        const char* blob = (const char*)(map + q.off_blob);
        uint64_t* out = (uint64_t*)(map + q.off_out);
        uint64_t* sizes = (uint64_t*)(map + q.off_sizes);
        int32_t* status = (int32_t*)(map + q.off_status);
        int32_t* os_error = (int32_t*)(map + q.off_oserr);
        for (uint64_t i = q.lo; i < q.hi; ++i) {
            struct stat sb;
            const bool found = stat(blob + offs[i], &sb) == 0;
            const bool ok = found && S_ISREG(sb.st_mode);
            status[i] = ok ? 0 : found ? 3 : 7;
            os_error[i] = ok ? 0 : found ? EISDIR : errno;
            sizes[i] = ok ? (uint64_t)sb.st_size : 0;
            out[2 * i] = ok ? (uint64_t)sb.st_size : 0;
            out[2 * i + 1] = ok ? i + (meta ? (1ull << 40) : 0) : 0;
        }
        if (stall) sleep((unsigned)stall);
        if (!reply(sock, q.seq, 0, "")) break;
    }
    return 0;
}
