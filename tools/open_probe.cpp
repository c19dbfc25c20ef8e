// tools/open_probe.cpp -- what does the per-file syscall floor of the warm C3 read (200 000 files of
// 49 292 B in 1 000 dirs) consist of, and does opening relative to a cached directory descriptor
// lower it? Reads a list of files (one path per line on stdin, page cache warm) with T threads that
// claim files 8 at a time, in these shapes:
//   full          open(path) + fstat + pread(whole file) + close   (the reference loop, our readers)
//   dirfd         openat(cached fd of the file's directory, basename) + fstat + pread + close
//   nostat        open(path) + read until a short read + close     (no fstat: the size comes from
//                 the read itself; a regular file's short read is its end)
//   dirfd_nostat  both
//   openclose     open(path) + close                               (path walk + fd only)
//   dirfd_oc      openat(dirfd, basename) + close
// PROCS=P in the environment splits the list into P contiguous parts read by P forked processes of
// T/P threads each (separate file tables and address spaces): does the floor belong to one process?
// UNSHARE=1: every reader thread first calls unshare(CLONE_FILES) -- its own file-descriptor table
// (threads still share the address space), so its open/close no longer take the process-wide table
// lock the other threads take.
// Prints one JSON line per run.
//   g++ -O2 -std=c++17 -pthread tools/open_probe.cpp -o tools/open_probe
//   find DIR -type f | tools/open_probe 16 full dirfd nostat dirfd_nostat openclose dirfd_oc
#include <fcntl.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <iostream>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    const int T = argc > 1 ? atoi(argv[1]) : 16;
    std::vector<std::string> paths, base;
    std::vector<int> dir_of;
    std::unordered_map<std::string, int> dir_id;
    std::vector<std::string> dirs;
    std::string line;
    while (std::getline(std::cin, line)) {
        if (line.empty()) continue;
        const size_t s = line.rfind('/');
        const std::string d = s == std::string::npos ? "." : line.substr(0, s);
        auto it = dir_id.find(d);
        if (it == dir_id.end()) {
            it = dir_id.emplace(d, (int)dirs.size()).first;
            dirs.push_back(d);
        }
        paths.push_back(line);
        base.push_back(s == std::string::npos ? line : line.substr(s + 1));
        dir_of.push_back(it->second);
    }
    const size_t n = paths.size();
    std::vector<int> dfd(dirs.size());
    for (size_t i = 0; i < dirs.size(); ++i) dfd[i] = open(dirs[i].c_str(), O_RDONLY | O_DIRECTORY);
    for (int a = 2; a < argc; ++a) {
        const std::string mode = argv[a];
        const bool at = mode.rfind("dirfd", 0) == 0;
        const bool nostat = mode.find("nostat") != std::string::npos;
        const bool oc = mode == "openclose" || mode == "dirfd_oc";
        const int P = getenv("PROCS") ? std::max(1, atoi(getenv("PROCS"))) : 1;
        const int TP = std::max(1, T / P);
        std::atomic<size_t> next{0};
        std::atomic<uint64_t> bytes{0}, errors{0};
        const double t0 = now();
        size_t lo = 0, hi = n;
        std::vector<pid_t> kids;
        for (int p = 1; p < P; ++p) {  // process p reads part p; this process reads part 0
            const pid_t pid = fork();
            if (pid == 0) {
                lo = n * p / P;
                hi = n * (p + 1) / P;
                kids.clear();
                break;
            }
            kids.push_back(pid);
            hi = n / P;
        }
        next = lo;
        std::vector<std::thread> th;
        for (int t = 0; t < (P > 1 ? TP : T); ++t)
            th.emplace_back([&] {
                if (getenv("UNSHARE") && atoi(getenv("UNSHARE"))) unshare(CLONE_FILES);
                std::vector<char> buf(1 << 20);
                uint64_t mine = 0, err = 0;
                for (;;) {
                    const size_t i0 = next.fetch_add(8);
                    if (i0 >= hi) break;
                    for (size_t i = i0; i < i0 + 8 && i < hi; ++i) {
                        const int fd = at ? openat(dfd[dir_of[i]], base[i].c_str(), O_RDONLY) : open(paths[i].c_str(), O_RDONLY);
                        if (fd < 0) {
                            ++err;
                            continue;
                        }
                        if (!oc) {
                            uint64_t want = buf.size(), got = 0;
                            if (!nostat) {
                                struct stat sb;
                                fstat(fd, &sb);
                                want = (uint64_t)sb.st_size + 1;  // one byte over, as the readers do
                                if (want > buf.size()) buf.resize(want);
                            }
                            for (;;) {
                                const ssize_t k = pread(fd, buf.data() + got, want - got, (off_t)got);
                                if (k <= 0) break;
                                got += (uint64_t)k;
                                if (got < want) break;  // short read: end of file
                                if (nostat) {
                                    buf.resize(buf.size() * 2);
                                    want = buf.size();
                                } else {
                                    break;
                                }
                            }
                            mine += got;
                        }
                        close(fd);
                    }
                }
                bytes.fetch_add(mine);
                errors.fetch_add(err);
            });
        for (auto& t : th) t.join();
        if (P > 1 && lo != 0) _exit(errors.load() ? 1 : 0);  // a child: its part is done
        for (const pid_t k : kids) {
            int st = 0;
            waitpid(k, &st, 0);
            if (!WIFEXITED(st) || WEXITSTATUS(st)) errors.fetch_add(1);
        }
        const double dt = now() - t0;
        printf("{\"mode\": \"%s\", \"unshare\": %d, \"procs\": %d, \"threads\": %d, \"files\": %zu, \"bytes\": %llu, \"errors\": %llu, \"s\": %.4f}\n",
               mode.c_str(), getenv("UNSHARE") ? atoi(getenv("UNSHARE")) : 0, P, T, n, (unsigned long long)bytes.load(), (unsigned long long)errors.load(), dt);
        fflush(stdout);
    }
    return 0;
}
