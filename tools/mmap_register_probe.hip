// Can a page-cache file be DMA'd to the GPU without a CPU copy? mmap the file, hipHostRegister
// the mapping (pins the page-cache pages), hipMemcpy to the device; times each step against
// pread into a pinned buffer + hipMemcpy. Probe only (tools/, not the product path).
//   hipcc --offload-arch=gfx950 -O2 tools/mmap_register_probe.hip -o /tmp/mrp && /tmp/mrp FILE
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    const int fd = open(argv[argc > 2 && getenv("MRP_SECOND") ? 2 : 1], O_RDONLY);
    struct stat sb;
    if (fd < 0 || fstat(fd, &sb) != 0) return 3;
    const size_t len = (size_t)sb.st_size;
    void* d = nullptr;
    if (hipMalloc(&d, len) != hipSuccess) return 4;
    (void)hipMemset(d, 0, len);  // first touch of the device buffer outside the timings
    (void)hipDeviceSynchronize();
    for (int rep = 0; rep < 3; ++rep) {
        double t0 = now();
        void* m = mmap(nullptr, len, PROT_READ, MAP_SHARED | MAP_POPULATE, fd, 0);
        if (m == MAP_FAILED) { printf("mmap failed\n"); return 5; }
        double t1 = now();
        hipError_t e = hipHostRegister(m, len, hipHostRegisterReadOnly);
        double t2 = now();
        if (e != hipSuccess) {
            printf("hipHostRegister: %s\n", hipGetErrorString(e));
            munmap(m, len);
            break;
        }
        e = hipMemcpy(d, m, len, hipMemcpyHostToDevice);
        double t3 = now();
        (void)hipHostUnregister(m);
        double t4 = now();
        munmap(m, len);
        printf("rep %d: mmap+populate %.3f s, register %.3f s, H2D %.3f s (%.1f GB/s, %s), unregister %.3f s\n", rep, t1 - t0,
               t2 - t1, t3 - t2, len / (t3 - t2) / 1e9, hipGetErrorString(e), t4 - t3);
    }
    // baseline: pread (one thread) into a 256 MiB pinned buffer + H2D
    void* h = nullptr;
    const size_t piece = 256u << 20;
    (void)hipHostMalloc(&h, piece, 0);
    double t0 = now();
    for (size_t off = 0; off < len; off += piece) {
        const size_t n = len - off < piece ? len - off : piece;
        size_t got = 0;
        while (got < n) {
            ssize_t k = pread(fd, (char*)h + got, n - got, (off_t)(off + got));
            if (k <= 0) return 6;
            got += (size_t)k;
        }
        (void)hipMemcpy((char*)d + off, h, n, hipMemcpyHostToDevice);
    }
    printf("pread(1 thread)+H2D in 256 MiB pieces: %.3f s\n", now() - t0);
    return 0;
}
