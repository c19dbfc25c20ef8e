// oxen_amd/csrc/capi_context.hip -- oxh_ctx: a device's streams, NSLOT pinned + device staging slots,
// reader pools and the engine thread (oxh_ctx_create / _destroy), and the host-resource queries the
// other pieces share (usable CPUs, the device check). See capi_internal.hpp for the pieces.
#include "capi_internal.hpp"

using namespace oxh::capi;

namespace oxh::capi {

int check_device(int device) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(OXH_ERR_NODEVICE, "no HIP device visible");
    if (device < 0 || device >= n) return fail(OXH_ERR_INVALID, "device index out of range");
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return fail(OXH_ERR_NODEVICE, "hipGetDeviceProperties failed");
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(OXH_ERR_NODEVICE, std::string("device is ") + prop.gcnArchName + ", this library is built for gfx950");
    return OXH_OK;
}

// CPUs this process may use: the affinity mask, capped by a cgroup-v2 CPU quota (a container's
// cpu.max, e.g. "1600000 100000" = 16 CPUs); hardware_concurrency() sees the whole machine.
int usable_cpus() {
    unsigned n = std::thread::hardware_concurrency();
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0 && CPU_COUNT(&set) > 0) n = (unsigned)CPU_COUNT(&set);
    if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char quota[32] = {0};
        unsigned long long period = 0;
        if (fscanf(f, "%31s %llu", quota, &period) == 2 && strcmp(quota, "max") != 0 && period > 0) {
            const unsigned long long q = strtoull(quota, nullptr, 10);
            const unsigned cap = (unsigned)std::max<unsigned long long>(1, (q + period - 1) / period);
            n = n ? std::min(n, cap) : cap;
        }
        fclose(f);
    }
    return (int)(n ? n : 4);
}

int default_threads() {
    const char* e = getenv("OXH_NUM_THREADS");  // cf. OXEN_NUM_THREADS (util/concurrency.rs:1-45)
    if (e && atoi(e) > 0) return atoi(e);
    return std::max(1, std::min(usable_cpus(), 16));
}

// Stall reports (dump_engine): the live contexts, and where context creation / destruction and the
// streaming Xxh3 last were -- the threads that call those are not engine threads.
std::mutex g_live_mu;
std::vector<oxh_ctx*> g_live;
std::atomic<const char*> g_life{"-"}, g_stream_where{"-"};

}  // namespace oxh::capi

namespace oxh {
// for the other translation units of the library (fastcdc.hip, fastcdc_host.cpp, comm.cpp)
int set_error(int code, const std::string& msg) { return fail(code, msg); }
int cpu_quota() { return usable_cpus(); }
int default_reader_threads() { return default_threads(); }
}  // namespace oxh

extern "C" {

int oxh_ctx_counters(oxh_ctx* c, uint64_t* out, int n) {
    if (!c || (n > 0 && !out)) return fail(OXH_ERR_INVALID, "null argument");
    const uint64_t v[4] = {c->d_big_allocs, c->d_big_size, c->n_direct.load(), c->n_runs.load()};
    for (int i = 0; i < n; ++i) out[i] = i < 4 ? v[i] : 0;
    return OXH_OK;
}

int oxh_ctx_create(int device, uint64_t staging_bytes, oxh_ctx** out) {
    if (!out) return fail(OXH_ERR_INVALID, "out is NULL");
    *out = nullptr;
    // a slot's reservation word packs the byte offset into 31 bits and the item count into 19
    // (stream_files below): both must hold a full slot
    if (staging_bytes > OXH_MAX_STAGING_BYTES)
        return fail(OXH_ERR_INVALID, "staging_bytes exceeds OXH_MAX_STAGING_BYTES (2 GiB - 256)");
    int rc = check_device(device);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(device));
    oxh_ctx* c = new oxh_ctx();
    c->device = device;
    {
        std::lock_guard<std::mutex> g(g_live_mu);
        g_live.push_back(c);
    }
    g_life.store("create: streams");
    c->stage_bytes = align_up(staging_bytes ? staging_bytes : (256ull << 20));
    c->max_items = std::max<uint64_t>(1024, c->stage_bytes / 4096);
    auto cleanup = [&](int code, const char* m) { oxh_ctx_destroy(c); return fail(code, m); };
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) return cleanup(OXH_ERR_HIP, "stream");
    if (hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking) != hipSuccess) return cleanup(OXH_ERR_HIP, "copy stream");
    g_life.store("create: slot buffers");
    for (int s = 0; s < NSLOT; ++s) {
        if (hipHostMalloc(&c->h_stage[s], c->stage_bytes, hipHostMallocDefault) != hipSuccess) return cleanup(OXH_ERR_NOMEM, "pinned staging");
        if (hipMalloc(&c->d_stage[s], c->stage_bytes) != hipSuccess) return cleanup(OXH_ERR_NOMEM, "device staging");
        if (hipHostMalloc(&c->h_desc[s], c->max_items * 16, hipHostMallocDefault) != hipSuccess) return cleanup(OXH_ERR_NOMEM, "pinned desc");
        if (hipMalloc(&c->d_desc[s], c->max_items * 16) != hipSuccess) return cleanup(OXH_ERR_NOMEM, "device desc");
        if (hipHostMalloc(&c->h_out[s], c->max_items * 16, hipHostMallocDefault) != hipSuccess) return cleanup(OXH_ERR_NOMEM, "pinned out");
        if (hipMalloc(&c->d_out[s], c->max_items * 16) != hipSuccess) return cleanup(OXH_ERR_NOMEM, "device out");
        if (hipHostMalloc(&c->h_cnt[s], c->max_items * 16, hipHostMallocDefault) != hipSuccess) return cleanup(OXH_ERR_NOMEM, "pinned counts");
        if (hipMalloc(&c->d_cnt[s], c->max_items * 16) != hipSuccess) return cleanup(OXH_ERR_NOMEM, "device counts");
        if (hipHostMalloc(&c->h_utf8[s], c->max_items * 4, hipHostMallocDefault) != hipSuccess) return cleanup(OXH_ERR_NOMEM, "pinned utf8");
        if (hipMalloc(&c->d_utf8[s], c->max_items * 4) != hipSuccess) return cleanup(OXH_ERR_NOMEM, "device utf8");
        if (hipHostMalloc(&c->h_klen[s], c->max_items * 8, hipHostMallocDefault) != hipSuccess) return cleanup(OXH_ERR_NOMEM, "pinned wave lens");
        if (hipMalloc(&c->d_klen[s], c->max_items * 8) != hipSuccess) return cleanup(OXH_ERR_NOMEM, "device wave lens");
        if (hipMalloc(&c->d_sums[s], (slot_sums_words(c->stage_bytes) + kSlotCountRaw) * 8) != hipSuccess)
            return cleanup(OXH_ERR_NOMEM, "device block sums");
        if (hipEventCreateWithFlags(&c->ev_copied[s], hipEventDisableTiming) != hipSuccess) return cleanup(OXH_ERR_HIP, "event");
        if (hipEventCreateWithFlags(&c->ev_done[s], hipEventDisableTiming) != hipSuccess) return cleanup(OXH_ERR_HIP, "event");
    }
    for (int s = 0; s < NSLOT; ++s) {
        c->rq[s].resize(c->max_items);
        c->loc[s].resize(c->max_items);
    }
    const char* fl = getenv("OXH_FLUSH_MIB");
    c->flush_bytes = std::min<uint64_t>(c->stage_bytes, (fl ? (uint64_t)atoll(fl) : 16ull) << 20);
    c->pool = new oxh::Pool(default_threads());
    c->rpool = new oxh::Pool(default_threads(), /*private_fds=*/true);  // readers use only their own fds
    c->engine = std::thread(engine_main, c);
    g_life.store("create: done");
    *out = c;
    return OXH_OK;
}

int oxh_ctx_destroy(oxh_ctx* c) {
    if (!c) return OXH_OK;
    {
        std::lock_guard<std::mutex> g(g_live_mu);
        g_live.erase(std::remove(g_live.begin(), g_live.end(), c), g_live.end());
    }
    g_life.store("destroy: engine join");
    if (c->engine.joinable()) {  // finishes what is queued, then exits
        {
            std::lock_guard<std::mutex> g(c->qmu);
            c->stop = true;
        }
        c->qcv.notify_all();
        c->engine.join();
    }
    (void)hipSetDevice(c->device);
    g_life.store("destroy: buffers");
    if (c->cdc && c->cdc_free) c->cdc_free(c->cdc);
    c->cdc = nullptr;
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->copy_stream) (void)hipStreamSynchronize(c->copy_stream);
    for (int s = 0; s < NSLOT; ++s) {
        if (c->h_stage[s]) (void)hipHostFree(c->h_stage[s]);
        if (c->d_stage[s]) (void)hipFree(c->d_stage[s]);
        if (c->h_desc[s]) (void)hipHostFree(c->h_desc[s]);
        if (c->d_desc[s]) (void)hipFree(c->d_desc[s]);
        if (c->h_out[s]) (void)hipHostFree(c->h_out[s]);
        if (c->d_out[s]) (void)hipFree(c->d_out[s]);
        if (c->h_cnt[s]) (void)hipHostFree(c->h_cnt[s]);
        if (c->d_cnt[s]) (void)hipFree(c->d_cnt[s]);
        if (c->h_utf8[s]) (void)hipHostFree(c->h_utf8[s]);
        if (c->d_utf8[s]) (void)hipFree(c->d_utf8[s]);
        if (c->h_klen[s]) (void)hipHostFree(c->h_klen[s]);
        if (c->d_klen[s]) (void)hipFree(c->d_klen[s]);
        if (c->d_sums[s]) (void)hipFree(c->d_sums[s]);
        if (c->ev_copied[s]) (void)hipEventDestroy(c->ev_copied[s]);
        if (c->ev_done[s]) (void)hipEventDestroy(c->ev_done[s]);
    }
    g_life.store("destroy: d_big");
    if (c->d_big) {  // large_items' piece buffers
        (void)hipStreamSynchronize(c->stream);
        (void)hipFree(c->d_big);
    }
    g_life.store("destroy: bounce / streams");
    for (int b = 0; b < kNBounce; ++b) {
        if (c->h_bounce[b]) (void)hipHostFree(c->h_bounce[b]);
        if (c->ev_bounce[b]) (void)hipEventDestroy(c->ev_bounce[b]);
    }
    for (int b = 0; b < 2; ++b)
        if (c->ev_piece_free[b]) (void)hipEventDestroy(c->ev_piece_free[b]);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
    if (c->copy_stream2) {
        (void)hipStreamSynchronize(c->copy_stream2);
        (void)hipStreamDestroy(c->copy_stream2);
    }
    if (c->ev_copy2_join) (void)hipEventDestroy(c->ev_copy2_join);
    g_life.store("destroy: pools");
    delete c->pool;
    delete c->wpool;
    delete c->rpool;
    delete c;
    g_life.store("destroy: done");
    return OXH_OK;
}

void* oxh_ctx_stream(oxh_ctx* c) { return c ? (void*)c->stream : nullptr; }

}  // extern "C"

namespace oxh {
int ctx_device(oxh_ctx* c) { return c->device; }
std::mutex& ctx_call_mutex(oxh_ctx* c) { return c->mu; }
void*& ctx_cdc_state(oxh_ctx* c, void (*deleter)(void*)) {
    c->cdc_free = deleter;
    return c->cdc;
}
}  // namespace oxh
