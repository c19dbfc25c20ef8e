// tests/native/fake_pool_helper.cpp -- a stand-in for oxen_amd/oxh_hash_helper that speaks the reader
// pool's wire protocol (oxen_amd/csrc/reader_pool.hpp) without a GPU, so the pool's mechanics --
// spawning, the shared region and its growth, share splitting, per-call sequence numbers, per-file
// statuses, helper death -- are tested on any host (tests/test_procpool.py, OXH_HELPER=<this>).
// Test infrastructure only: it computes no digest; "out" is (size, index of the file in the call)
// so the test can check that every item landed in its own slot.
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/prctl.h>
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
    prctl(PR_SET_PDEATHSIG, SIGKILL);
    const int sock = oxh_pool_wire::kSockFd, mem = oxh_pool_wire::kMemFd;
    int device = 0;
    for (int i = 1; i < argc; ++i)
        if (strncmp(argv[i], "--device=", 9) == 0) device = atoi(argv[i] + 9);
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
        for (uint64_t i = q.lo; i < q.hi; ++i) {
            struct stat sb;
            const bool ok = stat(blob + offs[i], &sb) == 0 && S_ISREG(sb.st_mode);
            status[i] = ok ? 0 : 3;
            sizes[i] = ok ? (uint64_t)sb.st_size : 0;
            out[2 * i] = ok ? (uint64_t)sb.st_size : 0;
            out[2 * i + 1] = ok ? i + (meta ? (1ull << 40) : 0) : 0;
        }
        if (!reply(sock, q.seq, 0, "")) break;
    }
    return 0;
}
