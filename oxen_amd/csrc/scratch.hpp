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
    hipStream_t aux = nullptr;  // a second stream for the lease holder (created on first use)
    hipEvent_t ev[4] = {};
};

// Two buffers per device, so two calls on different streams (say FastCDC chunking and the K1L
// whole-file chains of the same blobs) can run concurrently; a third caller waits for the first.
constexpr int kScratchPerDevice = 2;

inline ScratchCache* scratch_caches(int dev) {
    static std::mutex mu;
    static std::map<int, ScratchCache*> caches;  // kScratchPerDevice per device, process lifetime
    std::lock_guard<std::mutex> g(mu);
    ScratchCache*& c = caches[dev];
    if (!c) c = new ScratchCache[kScratchPerDevice];
    return c;
}

class ScratchLease {
   public:
    explicit ScratchLease(hipStream_t st) : st_(st) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        ScratchCache* cs = scratch_caches(dev);
        for (int k = 0; k < kScratchPerDevice && !lk_.owns_lock(); ++k) {
            std::unique_lock<std::mutex> t(cs[k].mu, std::try_to_lock);
            if (t.owns_lock()) {
                cache_ = &cs[k];
                lk_ = std::move(t);
            }
        }
        if (!lk_.owns_lock()) {
            cache_ = &cs[0];
            lk_ = std::unique_lock<std::mutex>(cache_->mu);
        }
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
            if (cache_->base) {  // idle: the previous holder synchronised its stream before releasing
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
    // A stream of this scratch buffer's own, for work the caller overlaps with its stream, and four
    // events to order the two (created on first use, kept with the buffer).
    hipError_t aux(hipStream_t* s, hipEvent_t** ev) {
        if (!cache_->aux) {
            const hipError_t e = hipStreamCreateWithFlags(&cache_->aux, hipStreamNonBlocking);
            if (e != hipSuccess) return e;
            for (hipEvent_t& x : cache_->ev) {
                const hipError_t f = hipEventCreateWithFlags(&x, hipEventDisableTiming);
                if (f != hipSuccess) return f;
            }
        }
        *s = cache_->aux;
        *ev = cache_->ev;
        return hipSuccess;
    }

   private:
    hipStream_t st_;
    ScratchCache* cache_ = nullptr;
    std::unique_lock<std::mutex> lk_;
};

}  // namespace oxh
