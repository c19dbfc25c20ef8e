// tools/uring_probe.cpp -- can io_uring lower the per-file syscall floor of the C3 host fill?
// Reads a list of files (one path per line on stdin; sizes stat'ed up front, untimed, as the
// caller's walk has them for oxh_hash_files_meta) with T threads into one large buffer, warm cache:
//   sync    open + fstat + pread + close per file (the staging readers today)
//   nostat  open + pread(size + 1) + close (the _meta path: no fstat)
//   uring   one io_uring per thread, per file a hard-linked OPENAT (direct descriptor slot) ->
//           READ (size + 1, fixed file) -> CLOSE, B files per io_uring_enter
// and prints seconds per mode (median of R runs). Raw syscalls, no liburing (not in the image).
//
//   g++ -O2 -std=c++17 -pthread -o tools/uring_probe tools/uring_probe.cpp
//   find DIR -type f | tools/uring_probe [T] [B] [R]
#include <fcntl.h>
#include <linux/io_uring.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <iostream>
#include <string>
#include <thread>
#include <vector>

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Ring {
    int fd = -1;
    unsigned *sq_head, *sq_tail, *sq_mask, *sq_array, *cq_head, *cq_tail, *cq_mask;
    io_uring_sqe* sqes;
    io_uring_cqe* cqes;
    unsigned entries;

    bool init(unsigned n, unsigned slots) {
        io_uring_params p{};
        fd = (int)syscall(__NR_io_uring_setup, n, &p);
        if (fd < 0) return false;
        entries = p.sq_entries;
        const size_t sq_sz = p.sq_off.array + p.sq_entries * sizeof(unsigned);
        const size_t cq_sz = p.cq_off.cqes + p.cq_entries * sizeof(io_uring_cqe);
        const size_t sz = std::max(sq_sz, cq_sz);
        uint8_t* sq = (uint8_t*)mmap(nullptr, sz, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, fd, IORING_OFF_SQ_RING);
        if (sq == MAP_FAILED) return false;
        uint8_t* cq = sq;
        if (!(p.features & IORING_FEAT_SINGLE_MMAP)) {
            cq = (uint8_t*)mmap(nullptr, cq_sz, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, fd, IORING_OFF_CQ_RING);
            if (cq == MAP_FAILED) return false;
        }
        sqes = (io_uring_sqe*)mmap(nullptr, p.sq_entries * sizeof(io_uring_sqe), PROT_READ | PROT_WRITE,
                                   MAP_SHARED | MAP_POPULATE, fd, IORING_OFF_SQES);
        if (sqes == MAP_FAILED) return false;
        sq_head = (unsigned*)(sq + p.sq_off.head);
        sq_tail = (unsigned*)(sq + p.sq_off.tail);
        sq_mask = (unsigned*)(sq + p.sq_off.ring_mask);
        sq_array = (unsigned*)(sq + p.sq_off.array);
        cq_head = (unsigned*)(cq + p.cq_off.head);
        cq_tail = (unsigned*)(cq + p.cq_off.tail);
        cq_mask = (unsigned*)(cq + p.cq_off.ring_mask);
        cqes = (io_uring_cqe*)(cq + p.cq_off.cqes);
        std::vector<int> table(slots, -1);  // sparse direct-descriptor table
        return syscall(__NR_io_uring_register, fd, IORING_REGISTER_FILES, table.data(), slots) == 0;
    }
    io_uring_sqe* next(unsigned k) {  // k-th SQE of the current batch (tail not yet published)
        const unsigned t = __atomic_load_n(sq_tail, __ATOMIC_RELAXED) + k;
        const unsigned i = t & *sq_mask;
        sq_array[i] = i;
        io_uring_sqe* s = &sqes[i];
        memset(s, 0, sizeof *s);
        return s;
    }
    // publish k SQEs, wait for `want` completions; returns the number of failed file reads
    int submit_wait(unsigned k, unsigned want, const std::vector<long>& expect) {
        __atomic_store_n(sq_tail, __atomic_load_n(sq_tail, __ATOMIC_RELAXED) + k, __ATOMIC_RELEASE);
        if (syscall(__NR_io_uring_enter, fd, k, want, IORING_ENTER_GETEVENTS, nullptr, 0) < 0) return -1;
        int bad = 0;
        unsigned got = 0;
        while (got < want) {
            unsigned h = __atomic_load_n(cq_head, __ATOMIC_RELAXED);
            const unsigned t = __atomic_load_n(cq_tail, __ATOMIC_ACQUIRE);
            if (h == t) {
                if (syscall(__NR_io_uring_enter, fd, 0, want - got, IORING_ENTER_GETEVENTS, nullptr, 0) < 0) return -1;
                continue;
            }
            for (; h != t; ++h, ++got) {
                const io_uring_cqe& c = cqes[h & *cq_mask];
                const uint64_t ud = c.user_data;
                if ((ud & 3) == 1 && c.res != expect[ud >> 2]) ++bad;  // READ: whole file, no more
                if ((ud & 3) != 1 && c.res < 0) ++bad;
                static std::atomic<int> shown{0};
                if (c.res < 0 && shown.fetch_add(1) < 3) fprintf(stderr, "op %d res %d\n", (int)(ud & 3), c.res);
            }
            __atomic_store_n(cq_head, h, __ATOMIC_RELEASE);
        }
        return bad;
    }
};

int main(int argc, char** argv) {
    const int T = argc > 1 ? atoi(argv[1]) : 16;
    const unsigned B = argc > 2 ? (unsigned)atoi(argv[2]) : 32;
    const int R = argc > 3 ? atoi(argv[3]) : 5;
    std::vector<std::string> paths;
    std::string line;
    while (std::getline(std::cin, line))
        if (!line.empty()) paths.push_back(line);
    const size_t n = paths.size();
    std::vector<long> sizes(n);
    std::vector<uint64_t> off(n);
    uint64_t total = 0;
    for (size_t i = 0; i < n; ++i) {
        struct stat sb;
        if (stat(paths[i].c_str(), &sb) != 0) return 2;
        sizes[i] = (long)sb.st_size;
        off[i] = total;
        total += ((uint64_t)sb.st_size + 256) & ~255ull;  // room for the one-byte over-read
    }
    uint8_t* big = (uint8_t*)malloc(total + 4096);
    memset(big, 0, total + 4096);

    auto run = [&](int mode) -> double {
        std::atomic<size_t> next{0};
        std::atomic<long> bad{0};
        const double t0 = now();
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back([&] {
                if (mode < 2) {
                    for (;;) {
                        const size_t i0 = next.fetch_add(8);
                        if (i0 >= n) break;
                        for (size_t i = i0; i < std::min(n, i0 + 8); ++i) {
                            const int fd = open(paths[i].c_str(), O_RDONLY | O_CLOEXEC);
                            if (fd < 0) { bad++; continue; }
                            long want = sizes[i];
                            if (mode == 0) {
                                struct stat sb;
                                fstat(fd, &sb);
                                want = sb.st_size;
                            }
                            const ssize_t x = pread(fd, big + off[i], (size_t)want + (mode == 1), 0);
                            if (x != sizes[i]) bad++;
                            close(fd);
                        }
                    }
                    return;
                }
                Ring r;
                if (!r.init(4 * B, B)) { bad += 1000000; return; }
                for (;;) {
                    const size_t i0 = next.fetch_add(B);
                    if (i0 >= n) break;
                    const unsigned m = (unsigned)std::min<size_t>(B, n - i0);
                    for (unsigned j = 0; j < m; ++j) {
                        const size_t i = i0 + j;
                        io_uring_sqe* s = r.next(3 * j);
                        s->opcode = IORING_OP_OPENAT;
                        s->fd = AT_FDCWD;
                        s->addr = (uint64_t)paths[i].c_str();
                        s->open_flags = O_RDONLY;  // O_CLOEXEC is EINVAL with a direct slot
                        s->file_index = j + 1;
                        s->flags = IOSQE_IO_HARDLINK;
                        s->user_data = (uint64_t)i << 2;
                        s = r.next(3 * j + 1);
                        s->opcode = IORING_OP_READ;
                        s->fd = (int)j;
                        s->addr = (uint64_t)(big + off[i]);
                        s->len = (unsigned)sizes[i] + 1;
                        s->off = 0;
                        s->flags = IOSQE_FIXED_FILE | IOSQE_IO_HARDLINK;
                        s->user_data = ((uint64_t)i << 2) | 1;
                        s = r.next(3 * j + 2);
                        s->opcode = IORING_OP_CLOSE;
                        s->file_index = j + 1;
                        s->user_data = ((uint64_t)i << 2) | 2;
                    }
                    const int b = r.submit_wait(3 * m, 3 * m, sizes);
                    if (b) bad += b < 0 ? 1000000 : b;
                }
                close(r.fd);
            });
        for (auto& x : th) x.join();
        const double dt = now() - t0;
        if (bad.load()) fprintf(stderr, "mode %d: %ld failures\n", mode, bad.load());
        return bad.load() ? -dt : dt;
    };
    const char* names[3] = {"sync", "nostat", "uring"};
    printf("{\"files\": %zu, \"bytes\": %llu, \"threads\": %d, \"batch\": %u", n, (unsigned long long)total, T, B);
    for (int mode : {0, 1, 2}) {
        std::vector<double> v;
        for (int k = 0; k < R; ++k) v.push_back(run(mode));
        std::sort(v.begin(), v.end());
        printf(", \"%s_s\": %.4f", names[mode], v[v.size() / 2]);
    }
    printf("}\n");
    return 0;
}
