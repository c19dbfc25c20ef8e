// Where the fused add's drain time goes ("the durable add"): 16 threads create, write
// and close N small files (C3's 49 292 B) under a store-like tree, the bytes coming from
// (a) hipHostMalloc'd pinned staging (what VersionPublisher::put writes from) or (b) malloc'd
// memory, each with and without the steps put() adds (stat of the target, mkdir of its directory).
//   hipcc -O2 tools/put_probe.cpp -o /tmp/put_probe && /tmp/put_probe /dev/shm/put_probe 100000
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main(int argc, char** argv) {
    const std::string root = argc > 1 ? argv[1] : "/dev/shm/put_probe";
    const int n = argc > 2 ? atoi(argv[2]) : 100000;
    const int T = 16;
    const size_t sz = 49292, total = (size_t)n * sz;
    const size_t span = std::min(total, (size_t)256 << 20);  // one staging slot, reused
    uint8_t* pinned = nullptr;
    if (hipHostMalloc((void**)&pinned, span, hipHostMallocDefault) != hipSuccess) return 1;
    uint8_t* pageable = (uint8_t*)malloc(span);
    for (size_t i = 0; i < span; ++i) pinned[i] = pageable[i] = (uint8_t)(i * 131 + 7);
    const char* names[] = {"pinned", "pageable", "pinned+stat+mkdir", "pageable+stat+mkdir"};
    for (int mode = 0; mode < 4; ++mode) {
        const uint8_t* src = (mode & 1) ? pageable : pinned;
        const bool extra = mode >= 2;
        const std::string base = root + "/m" + std::to_string(mode);
        mkdir(root.c_str(), 0755);
        mkdir(base.c_str(), 0755);
        for (int d = 0; d < 256; ++d) mkdir((base + "/" + std::to_string(d)).c_str(), 0755);
        std::atomic<int> next{0};
        const double t0 = now();
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back([&] {
                for (int i; (i = next.fetch_add(1)) < n;) {
                    const std::string dir = base + "/" + std::to_string(i & 255) + "/f" + std::to_string(i);
                    const std::string path = dir + "/data";
                    if (extra) {
                        struct stat sb;
                        (void)stat(path.c_str(), &sb);
                        mkdir(dir.c_str(), 0755);
                    } else {
                        mkdir(dir.c_str(), 0755);
                    }
                    const std::string tmp = dir + "/data.oxentmp.x";
                    const int fd = open(tmp.c_str(), O_RDWR | O_CREAT | O_EXCL | O_CLOEXEC, 0644);
                    if (fd < 0) continue;
                    const size_t off = ((size_t)i * sz) % (span - sz + 1);
                    if (write(fd, src + off, sz) != (ssize_t)sz) perror("write");
                    close(fd);
                }
            });
        for (auto& t : th) t.join();
        const double dt = now() - t0;
        printf("{\"mode\": \"%s\", \"files\": %d, \"s\": %.3f, \"us_per_file_thread\": %.1f}\n", names[mode], n, dt,
               dt * T * 1e6 / n);
        fflush(stdout);
        std::string cmd = "rm -rf " + base;
        if (system(cmd.c_str()) != 0) return 2;
    }
    (void)hipHostFree(pinned);
    free(pageable);
    return 0;
}
