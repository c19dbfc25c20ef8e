// tools/fill_probe.cpp -- where does the host fill of oxh_hash_files spend its time?
// Reads a list of files (one path per line on stdin) with T threads, warm page cache, into:
//   reuse   a per-thread malloc buffer reused for every file (what the CPU reference loop does)
//   big     successive offsets of one large malloc'ed buffer
//   pinned  successive offsets of one large hipHostMalloc'ed buffer (the staging slots)
// each with and without a separate stat() pass, and reports seconds per mode.
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <emmintrin.h>
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

int main(int argc, char** argv) {
    const int T = argc > 1 ? atoi(argv[1]) : 16;
    std::vector<std::string> paths;
    std::string line;
    while (std::getline(std::cin, line))
        if (!line.empty()) paths.push_back(line);
    const size_t n = paths.size();
    std::vector<uint64_t> sizes(n);
    uint64_t total = 0;
    for (size_t i = 0; i < n; ++i) {
        struct stat sb;
        stat(paths[i].c_str(), &sb);
        sizes[i] = sb.st_size;
        total += (sb.st_size + 255) & ~255ull;
    }
    uint64_t maxsz = 1;
    for (size_t i = 0; i < n; ++i) maxsz = std::max<uint64_t>(maxsz, sizes[i]);
    uint8_t* big = (uint8_t*)malloc(total);
    memset(big, 0, total);
    uint8_t* pinned = nullptr;
    if (hipHostMalloc((void**)&pinned, total, hipHostMallocDefault) != hipSuccess) return 1;
    memset(pinned, 0, total);
    std::vector<uint64_t> off(n);
    uint64_t o = 0;
    for (size_t i = 0; i < n; ++i) {
        off[i] = o;
        o += (sizes[i] + 255) & ~255ull;
    }
    auto run = [&](int mode, bool statpass) {
        const double t0 = now();
        std::vector<uint64_t> sz2(n);
        if (statpass) {
            std::atomic<size_t> next{0};
            std::vector<std::thread> th;
            for (int t = 0; t < T; ++t)
                th.emplace_back([&] {
                    for (size_t i; (i = next.fetch_add(64)) < n;)
                        for (size_t j = i; j < std::min(n, i + 64); ++j) {
                            struct stat sb;
                            stat(paths[j].c_str(), &sb);
                            sz2[j] = sb.st_size;
                        }
                });
            for (auto& x : th) x.join();
        }
        std::atomic<size_t> next{0};
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back([&] {
                std::vector<uint8_t> buf(maxsz);
                for (size_t i; (i = next.fetch_add(64)) < n;)
                    for (size_t j = i; j < std::min(n, i + 64); ++j) {
                        int fd = open(paths[j].c_str(), O_RDONLY | O_CLOEXEC);
                        uint64_t len = sizes[j];
                        if (!statpass) {
                            struct stat sb;
                            fstat(fd, &sb);
                            len = sb.st_size;
                        }
                        uint8_t* dst = (mode == 0 || mode == 3) ? buf.data() : mode == 1 ? big + off[j] : pinned + off[j];
                        uint64_t got = 0;
                        while (got < len) {
                            ssize_t r = pread(fd, dst + got, len - got, got);
                            if (r <= 0) break;
                            got += r;
                        }
                        close(fd);
                        if (mode == 3) {  // bounce buffer -> pinned with non-temporal stores
                            const __m128i* src = (const __m128i*)buf.data();
                            __m128i* d = (__m128i*)(pinned + off[j]);
                            const uint64_t n16 = len / 16;
                            for (uint64_t q = 0; q < n16; ++q) _mm_stream_si128(d + q, _mm_loadu_si128(src + q));
                            memcpy(pinned + off[j] + n16 * 16, buf.data() + n16 * 16, len - n16 * 16);
                        }
                    }
            });
        for (auto& x : th) x.join();
        _mm_sfence();
        return now() - t0;
    };
    // the C oracle's loop: thread t takes files t, t+T, ...; open, fstat, malloc, read, free, close
    auto run_oracle_style = [&](bool interleave) {
        const double t0 = now();
        std::vector<std::thread> th;
        std::atomic<size_t> next{0};
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t] {
                auto one = [&](size_t j) {
                    int fd = open(paths[j].c_str(), O_RDONLY);
                    struct stat sb;
                    fstat(fd, &sb);
                    uint8_t* b = (uint8_t*)malloc(sb.st_size ? sb.st_size : 1);
                    uint64_t got = 0;
                    while (got < (uint64_t)sb.st_size) {
                        ssize_t r = read(fd, b + got, sb.st_size - got);
                        if (r <= 0) break;
                        got += r;
                    }
                    free(b);
                    close(fd);
                };
                if (interleave) {
                    for (size_t j = t; j < n; j += T) one(j);
                } else {
                    for (size_t i; (i = next.fetch_add(64)) < n;)
                        for (size_t j = i; j < std::min(n, i + 64); ++j) one(j);
                }
            });
        for (auto& x : th) x.join();
        return now() - t0;
    };
    const char* names[4] = {"reuse", "big", "pinned", "bounce+nt"};
    for (int rep = 0; rep < 3; ++rep) {
        printf("oracle-style interleaved: %.3f s\n", run_oracle_style(true));
        printf("oracle-style chunked64: %.3f s\n", run_oracle_style(false));
        for (int mode = 0; mode < 4; ++mode)
            for (int sp = 0; sp < 1; ++sp)
                printf("%s statpass=%d: %.3f s\n", names[mode], sp, run(mode, sp));
    }
    return 0;
}
