// oxen_amd/csrc/scratch.hpp -- device scratch kept between calls, one buffer per device.
//
// K1L's block sums (64 B per KiB: 8.6 GB for C5's 16 x 8 GiB) and FastCDC's candidate / stitch
// tables (2.5-8 GB) are too large to allocate per call: stream-ordered allocations of that size
// (hipMallocAsync, from the default pool or a private one with a release threshold) every few calls
// stalled the host for 0.5-2.4 s before the first launch (tools/bench_fastcdc.py, bench_c5.py with
// OXH_TRACE=1 / rocprofv3 kernel traces). A lease holds the device's buffer for one call: it grows
// the buffer when needed, and on release synchronises the call's stream (the kernels must be done
// with it) and frees the buffer only if it exceeds OXH_SCRATCH_KEEP_MIB (default 16 GiB).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <map>
#include <mutex>

namespace oxh {

struct ScratchCache {
    std::mutex mu;
    void* base = nullptr;
    uint64_t size = 0;
};

inline ScratchCache& scratch_cache(int dev) {
    static std::mutex mu;
    static std::map<int, ScratchCache*> caches;  // one per device, for the process lifetime
    std::lock_guard<std::mutex> g(mu);
    ScratchCache*& c = caches[dev];
    if (!c) c = new ScratchCache();
    return *c;
}

class ScratchLease {
   public:
    explicit ScratchLease(hipStream_t st) : st_(st) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        cache_ = &scratch_cache(dev);
        lk_ = std::unique_lock<std::mutex>(cache_->mu);
    }
    ~ScratchLease() {
        (void)hipStreamSynchronize(st_);
        static const uint64_t keep =
            (getenv("OXH_SCRATCH_KEEP_MIB") ? strtoull(getenv("OXH_SCRATCH_KEEP_MIB"), nullptr, 10) : 16384ull) << 20;
        if (cache_->size > keep) {
            (void)hipFree(cache_->base);
            cache_->base = nullptr;
            cache_->size = 0;
        }
    }
    ScratchLease(const ScratchLease&) = delete;
    ScratchLease& operator=(const ScratchLease&) = delete;
    // At least `bytes` of device memory, valid until the lease ends.
    hipError_t get(uint64_t bytes, void** out) {
        if (cache_->size < bytes) {
            if (cache_->base) {
                const hipError_t e = hipDeviceSynchronize();  // an earlier call may still read it
                if (e != hipSuccess) return e;
                (void)hipFree(cache_->base);
                cache_->base = nullptr;
                cache_->size = 0;
            }
            const hipError_t e = hipMalloc(&cache_->base, bytes);
            if (e != hipSuccess) return e;
            cache_->size = bytes;
        }
        *out = cache_->base;
        return hipSuccess;
    }
    uint64_t size() const { return cache_->size; }

   private:
    hipStream_t st_;
    ScratchCache* cache_ = nullptr;
    std::unique_lock<std::mutex> lk_;
};

}  // namespace oxh
