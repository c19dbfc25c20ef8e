// tools/cold_probe.cpp -- does the cold-page-cache read of many small files (C3 end to end, cold)
// gain from more I/O in flight than the reader threads keep? Reads a list of files (one path per
// line on stdin) after dropping their pages (posix_fadvise DONTNEED), in three shapes:
//   plain T        T threads: open, fstat, pread the whole file into a reused buffer, close
//   willneed T P   the same T readers, plus P prefetch threads that run W files ahead of the readers
//                  issuing open + posix_fadvise(WILLNEED) + close (the kernel reads ahead async)
// Prints one JSON line per run.
//   g++ -O2 -std=c++17 -pthread tools/cold_probe.cpp -o tools/cold_probe
//   find DIR -type f | tools/cold_probe "plain 16" "plain 64" "willneed 16 4 4096"
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <iostream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void drop(const std::vector<std::string>& paths) {
    for (const auto& p : paths) {
        const int fd = open(p.c_str(), O_RDONLY);
        if (fd < 0) continue;
        fdatasync(fd);
        posix_fadvise(fd, 0, 0, POSIX_FADV_DONTNEED);
        close(fd);
    }
}

int main(int argc, char** argv) {
    std::vector<std::string> paths;
    std::string line;
    while (std::getline(std::cin, line))
        if (!line.empty()) paths.push_back(line);
    const size_t n = paths.size();
    for (int a = 1; a < argc; ++a) {
        std::istringstream in(argv[a]);
        std::string mode;
        int T = 16, P = 0, W = 4096;
        in >> mode >> T;
        if (mode == "willneed") in >> P >> W;
        drop(paths);
        std::atomic<size_t> next{0}, done_upto{0};
        std::atomic<uint64_t> bytes{0};
        std::atomic<bool> stop{false};
        const double t0 = now();
        std::vector<std::thread> th;
        for (int p = 0; p < P; ++p)
            th.emplace_back([&, p] {
                // prefetcher p takes every P-th file, staying at most W files ahead of the readers
                for (size_t i = (size_t)p; i < n && !stop.load(); i += (size_t)P) {
                    while (i > next.load(std::memory_order_relaxed) + (size_t)W && !stop.load()) usleep(50);
                    const int fd = open(paths[i].c_str(), O_RDONLY);
                    if (fd < 0) continue;
                    posix_fadvise(fd, 0, 0, POSIX_FADV_WILLNEED);
                    close(fd);
                }
            });
        std::vector<std::thread> rd;
        for (int t = 0; t < T; ++t)
            rd.emplace_back([&] {
                std::vector<char> buf(1 << 20);
                uint64_t mine = 0;
                for (;;) {
                    const size_t i = next.fetch_add(1);
                    if (i >= n) break;
                    const int fd = open(paths[i].c_str(), O_RDONLY);
                    if (fd < 0) continue;
                    struct stat sb;
                    fstat(fd, &sb);
                    if ((size_t)sb.st_size + 1 > buf.size()) buf.resize(sb.st_size + 1);
                    uint64_t got = 0;
                    for (;;) {
                        const ssize_t k = pread(fd, buf.data() + got, buf.size() - got, (off_t)got);
                        if (k <= 0) break;
                        got += (uint64_t)k;
                        if (got >= (uint64_t)sb.st_size) break;
                    }
                    mine += got;
                    close(fd);
                }
                bytes.fetch_add(mine);
            });
        for (auto& t : rd) t.join();
        const double dt = now() - t0;
        stop = true;
        for (auto& t : th) t.join();
        printf("{\"mode\": \"%s\", \"readers\": %d, \"prefetchers\": %d, \"window\": %d, \"files\": %zu, \"bytes\": %llu, "
               "\"s\": %.3f, \"GBs\": %.2f}\n",
               mode.c_str(), T, P, W, n, (unsigned long long)bytes.load(), dt, bytes.load() / dt / 1e9);
        fflush(stdout);
    }
    return 0;
}
