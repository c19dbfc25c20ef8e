// Stress test of the runtime thread pool (oxen_amd/csrc/pool.hpp): many short parallel_for calls;
// a lost wake-up or lock-order bug shows as a hang (tests/test_host.py runs it under a timeout).
#include "pool.hpp"
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>
int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 200000;
    oxh::Pool pool(16);
    std::vector<char> src(1 << 20), dst(1 << 20);
    auto t0 = std::chrono::steady_clock::now();
    for (int it = 0; it < iters; ++it) {
        int n = 1 + (it * 7919) % 130;
        int ntasks = std::min(n, pool.size() * 4);
        pool.parallel_for(ntasks, [&](int t) {
            for (int j = t; j < n; j += ntasks) memcpy(&dst[j * 100], &src[j * 100], 100);
        });
        if (it % 20000 == 0) { printf("it %d %.1fs\n", it, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count()); fflush(stdout); }
    }
    puts("done");
}
