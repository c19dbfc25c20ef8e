// oxen_amd/csrc/large_items.hip -- items larger than a staging slot (K1L): device-resident buffers in
// pieces (large_batch_device), and host files / buffers through device piece buffers fed by a pinned
// bounce ring (large_items), each piece's block sums chip-wide and every item's serial chain resumed
// piece to piece. See capi_internal.hpp for the pieces.
#include "capi_internal.hpp"

using namespace oxh::capi;

namespace oxh::capi {

// K1L over n device buffers. Buffers below ~1 MiB take one K1 wave. The others are processed in
// rounds of 1 GiB pieces (OXH_BIG_PIECE_MIB): round r computes the block sums of every buffer's
// piece r chip-wide on `st` while the serial chains of round r-1 run on the scratch buffer's own
// stream, up to kChainJobs chains per launch (ChainJob resume / partial flags carry each buffer's 8
// accumulators from piece to piece), so a chain starts one piece's block sums after its buffer does
// instead of after every buffer's, and the block-sum scratch is two rounds of pieces, not the whole
// input. Returns after `st` has finished.
int large_batch_device(const uint8_t* const* bufs, const uint64_t* lens, uint64_t n, uint64_t* d_out, hipStream_t st) {
    const char* pe = getenv("OXH_BIG_PIECE_MIB");
    const uint64_t P = std::max<uint64_t>(1, pe ? strtoull(pe, nullptr, 10) : 1024) << 20;
    std::vector<uint64_t> big;  // buffers on the chained path
    uint64_t rounds = 0;
    auto pieces_of = [&](uint64_t len) { return (len > P + 1024 ? (len - 1025) / P : 0) + 1; };
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t len = lens[i];
        const uint64_t nb = len > 0 ? (len - 1) >> 10 : 0;
        if (nb < 1024) {
            if (int rc = launch_chunks(bufs[i], 1, len, len, d_out + 2 * i, st)) return rc;
            continue;
        }
        big.push_back(i);
        rounds = std::max(rounds, pieces_of(len));
    }
    if (big.empty()) return OXH_OK;
    oxh::ScratchLease lease(st);  // the device's cached scratch (scratch.hpp); synchronises st at the end
    const uint64_t per_buf = ((P + 1024) >> 10) * 8;  // block-sum u64 per buffer per round
    uint64_t* scratch = nullptr;
    HIP_TRY(lease.get((2 * per_buf * big.size() + 8 * big.size()) * 8, (void**)&scratch));
    uint64_t* state = scratch + 2 * per_buf * big.size();  // 8 accumulators per buffer
    hipStream_t aux = nullptr;
    hipEvent_t* ev = nullptr;
    HIP_TRY(lease.aux(&aux, &ev));
    hipEvent_t* ev_sums = ev;       // [2] block sums of round r (parity) are ready
    hipEvent_t* ev_chain = ev + 2;  // [2] chains of round r (parity) are done with them
    for (uint64_t r = 0; r < rounds; ++r) {
        const int b = (int)(r & 1);
        if (r >= 2) HIP_TRY(hipStreamWaitEvent(st, ev_chain[b], 0));  // round r-2 read these sums
        oxh::ChainBatch batch;
        int nj = 0;
        auto flush = [&]() -> int {
            if (!nj) return OXH_OK;
            hipLaunchKernelGGL(oxh::xxh3_chain_kernel, dim3(nj), dim3(64), kChainLdsPad, aux, batch);
            HIP_TRY(hipGetLastError());
            nj = 0;
            return OXH_OK;
        };
        std::vector<oxh::ChainJob> jobs;
        for (uint64_t q = 0; q < big.size(); ++q) {
            const uint64_t i = big[q], len = lens[i], k = pieces_of(len) - 1;
            if (r > k) continue;
            const uint64_t off = r * P, plen = r < k ? P : len - off;
            const bool last = r == k;
            const uint64_t nb = last ? (plen - 1) >> 10 : plen >> 10;
            uint64_t* s_q = scratch + ((uint64_t)b * big.size() + q) * per_buf;
            const uint8_t* p = bufs[i] + off;
            const bool aligned = (reinterpret_cast<uintptr_t>(p) & 15) == 0;
            const uint64_t nwaves = (nb + 3) / 4, blocks = (nwaves + 3) / 4;
            if (aligned)
                hipLaunchKernelGGL(oxh::xxh3_blocksum_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, st, p, nb, s_q);
            else
                hipLaunchKernelGGL(oxh::xxh3_blocksum_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, st, p, nb, s_q);
            HIP_TRY(hipGetLastError());
            jobs.push_back({p, plen, s_q, d_out + 2 * i, len, state + 8 * q,
                            (r > 0 ? oxh::kChainResume : 0u) | (last ? 0u : oxh::kChainPartial)});
        }
        HIP_TRY(hipEventRecord(ev_sums[b], st));
        HIP_TRY(hipStreamWaitEvent(aux, ev_sums[b], 0));
        for (const oxh::ChainJob& j : jobs) {
            batch.job[nj++] = j;
            if (nj == oxh::kChainJobs)
                if (int rc = flush()) return rc;
        }
        if (int rc = flush()) return rc;
        HIP_TRY(hipEventRecord(ev_chain[b], aux));
    }
    HIP_TRY(hipStreamWaitEvent(st, ev_chain[(rounds - 1) & 1], 0));  // st continues after every chain
    return OXH_OK;
}

int large_device(oxh_ctx*, const uint8_t* d_buf, uint64_t len, uint64_t* d_out, hipStream_t st) {
    return large_batch_device(&d_buf, &len, 1, d_out, st);
}

// Digest (+ text counts, + is_utf8) of one buffer already on the device (stream-ordered on
// c->stream): d holds align_up(len) + 256 bytes, the tail is the results area. Synchronises c->stream.
int device_item(oxh_ctx* c, uint8_t* d, uint64_t len, uint64_t* out2, uint64_t* cnt2, int32_t* utf8_1) {
    const uint64_t tail = align_up(len);
    struct Res {  // mirrored at d + tail: digest, text counts, a one-item descriptor, is_utf8
        uint64_t out[2], cnt[2], off, len;
        int32_t utf8, pad;
    } h{};
    h.len = len;
    uint64_t* d_res = reinterpret_cast<uint64_t*>(d + tail);
    int rc = OXH_OK;
    auto ok = [&](hipError_t e, const char* what) {
        if (rc == OXH_OK && e != hipSuccess) rc = fail(OXH_ERR_HIP, what);
        return rc == OXH_OK;
    };
    ok(hipMemcpyAsync(d_res, &h, sizeof h, hipMemcpyHostToDevice, c->stream), "results area H2D failed");
    if (rc == OXH_OK) rc = large_device(c, d, len, d_res, c->stream);
    if (rc == OXH_OK && cnt2) {
        hipLaunchKernelGGL(oxh::text_count_kernel, dim3(2048), dim3(256), 0, c->stream, d, len,
                           (unsigned long long*)(d_res + 2));
        ok(hipGetLastError(), "text_count_kernel launch");
    }
    if (rc == OXH_OK && utf8_1) {
        hipLaunchKernelGGL(oxh::utf8_prefix_kernel, dim3(1), dim3(64), 0, c->stream, d, d_res + 4, d_res + 5, (uint64_t)1,
                           (int32_t*)(d_res + 6));
        ok(hipGetLastError(), "utf8_prefix_kernel launch");
    }
    ok(hipMemcpyAsync(&h, d_res, sizeof h, hipMemcpyDeviceToHost, c->stream), "results D2H failed");
    ok(hipStreamSynchronize(c->stream), "sync failed");
    if (rc == OXH_OK) {
        out2[0] = h.out[0];
        out2[1] = h.out[1];
        if (cnt2) {
            cnt2[0] = 1 + h.cnt[0];
            cnt2[1] = len - h.cnt[1];
        }
        if (utf8_1) *utf8_1 = h.utf8;
    }
    return rc;
}

// Hash one oversize host item (> a staging slot) through a device buffer of its own (the staging
// slots may belong to a live pipeline); with `cnt2`, also its text counts (num_lines, num_chars),
// with `utf8_1` its is_utf8 sniff.
int oversize_item(oxh_ctx* c, const uint8_t* src, uint64_t len, uint64_t* out2, uint64_t* cnt2, int32_t* utf8_1) {
    uint8_t* d = nullptr;
    if (hipMalloc(&d, align_up(len) + 256) != hipSuccess) {
        (void)hipGetLastError();
        return fail(OXH_ERR_NOMEM, "oversize hipMalloc failed");
    }
    int rc = OXH_OK;
    if (hipMemcpyAsync(d, src, len, hipMemcpyHostToDevice, c->stream) != hipSuccess) rc = fail(OXH_ERR_HIP, "oversize H2D failed");
    if (rc == OXH_OK) rc = device_item(c, d, len, out2, cnt2, utf8_1);
    (void)hipFree(d);
    return rc;
}

// Items larger than a staging slot (K1L). A file larger than a slot takes the reference's streaming
// branch (hasher.rs:150-174); a host buffer that large (oxh_hash_buffers / _streams) the same path.
// The item is hashed in device pieces of OXH_BIG_PIECE_MIB (default 1 GiB) through two piece
// buffers, so device memory stays bounded whatever the item size and piece j+1's transfer overlaps
// piece j's K1L chain: each piece's block sums are computed chip-wide and the serial chain continues
// from the previous piece's accumulators (ChainJob kChainResume / kChainPartial); the last piece
// (> 1 KiB) takes the tail and the merge. A file piece reaches the device copy-free when its pages
// are in the page cache (mincore) and can be pinned (mmap + hipHostRegister read-only, ~2 ms per GiB;
// the DMA engine then reads them at 46-57 GB/s, tools/mmap_register_probe.hip); otherwise pieces pass
// through two pinned 64 MiB bounce buffers filled by the worker pool (parallel 4 MiB reads). Text
// counts accumulate over the pieces; is_utf8 reads the first 4 KiB of piece 0. With a sink (fused
// add) every bounce part is also written to the sink's temp as it is read, and the temp is published
// once the digest is known: the item never has to fit in host memory.

// Bounce windows a large item reads at once (OXH_BIG_WINDOWS, 1 .. kNBounce - 1; 1 is the r03-r04 form)
int big_windows() {
    static const int v = [] {
        const char* e = getenv("OXH_BIG_WINDOWS");
        const int k = e ? atoi(e) : kNBounce - 1;
        return std::max(1, std::min(k, kNBounce - 1));
    }();
    return v;
}

// H2D copy streams a large item's bounce windows alternate over (OXH_BIG_COPY_STREAMS, 1 or 2; default 2)
int big_copy_streams() {
    static const int v = [] {
        const char* e = getenv("OXH_BIG_COPY_STREAMS");
        return e && atoi(e) == 1 ? 1 : 2;
    }();
    return v;
}

// Files up to this many at a time share one large-item pipeline (OXH_BIG_FILES overrides; device
// memory: 2 piece buffers of OXH_BIG_PIECE_MIB + 1 KiB per file).
int big_files_at_once() {
    const char* e = getenv("OXH_BIG_FILES");
    const int v = e && atoi(e) > 0 ? atoi(e) : 4;
    return std::min(v, (int)oxh::kChainJobs);
}

// Hash n (<= kChainJobs) large items side by side (see above). Round r moves piece r of every item
// that has one to the device (the copies are PCIe-bound and serial on the copy stream), launches its
// block sums chip-wide, and then ONE chain launch continues every item's serial chain over its piece
// (the chains are latency-bound: 16 files' chains cost about what one does). The chains of round r
// run on the device while the host moves round r+1's pieces, so the chain time hides behind the
// copies of the next round instead of adding up file after file. Returns a run-level error code only
// for HIP failures; each item's own outcome (I/O error, allocation failure) is its res.status.
int large_items(oxh_ctx* c, LargeJob* jobs, int n) {
    if (n <= 0) return OXH_OK;
    if (n > (int)oxh::kChainJobs) return fail(OXH_ERR_INVALID, "too many large items in one batch");
    const uint64_t P = std::max<uint64_t>(
        1, getenv("OXH_BIG_PIECE_MIB") ? strtoull(getenv("OXH_BIG_PIECE_MIB"), nullptr, 10) : 1024) << 20;
    const uint64_t cap = P + 1024;  // bytes per piece buffer
    const uint64_t slot = align_up(cap) + 256;
    constexpr uint64_t kRes = 256;  // per item: [digest 2 | counts 2 | desc off, len | utf8 | state 8]
    // an allocation that fails is these items' failure (OXH_ERR_NOMEM), not the engine run's: the
    // other requests in the live pipeline carry on
    auto nomem = [&]() {
        (void)hipGetLastError();
        for (int q = 0; q < n; ++q) jobs[q].res.status = OXH_ERR_NOMEM;
        return OXH_OK;
    };
    auto bytes_for = [&](int items) { return (uint64_t)items * (2 * slot + kRes) + 4096; };
    const uint64_t need = bytes_for(n);
    c->where.store("large_items: d_big");
    if (c->d_big_size < need) {
        // Regrow: every earlier large_items call on this context finished its work on d_big before it
        // returned (its streams are synchronised at the end), so the old buffer is idle. Plain
        // hipFree / hipMalloc: the stream-ordered allocator (hipMallocAsync / hipFreeAsync on
        // c->stream, r04) was AVOIDED after a stall under concurrent contexts (threads parked in
        // hipMallocAsync beside others in hipEventRecord / hipHostMalloc, every stream idle;
        // tools/engine_soak.py --regrow, profiles/r05/r05s6_*) -- not proven faulty, no reduced
        // reproducer. hipFree synchronises the whole device, so a regrow waits on every other
        // context's work: the buffer is sized for the most items the engine batches
        // (big_files_at_once(), or n if more) at once, so a context pays this once per piece size,
        // not once per new n (oxh_ctx_counters counts it; DESIGN §5 "Soak").
        if (c->d_big) {
            (void)hipFree(c->d_big);
            c->d_big = nullptr;
            c->d_big_size = 0;
        }
        void* m = nullptr;
        uint64_t size = std::max(need, bytes_for(big_files_at_once()));
        bool ok = hipMalloc(&m, size) == hipSuccess && m != nullptr;
        if (!ok && size > need) {  // the full batch does not fit: just these n items
            (void)hipGetLastError();
            size = need;
            ok = hipMalloc(&m, size) == hipSuccess && m != nullptr;
        }
        if (ok) ++c->d_big_allocs;
        if (!ok) {
            (void)hipGetLastError();
            // 2 piece buffers per file side by side did not fit: fewer files at a time (each item's
            // result does not depend on its batch), down to one before the items fail with NOMEM
            if (n > 1) {
                const int h = n / 2;
                if (int rc = large_items(c, jobs, h)) return rc;
                return large_items(c, jobs + h, n - h);
            }
            return nomem();
        }
        c->d_big = (uint8_t*)m;
        c->d_big_size = size;
    }
    auto dbuf = [&](int q, int b) { return c->d_big + ((uint64_t)q * 2 + b) * slot; };
    uint8_t* d_res_all = c->d_big + (uint64_t)n * 2 * slot;
    auto d_res = [&](int q) { return reinterpret_cast<uint64_t*>(d_res_all + (uint64_t)q * kRes); };
    struct Res {
        uint64_t out[2], cnt[2], off, len;
        int32_t utf8, pad;
    };
    static_assert(sizeof(Res) + 64 <= kRes, "results area");
    std::vector<uint8_t> h_res((size_t)n * kRes, 0);
    for (int q = 0; q < n; ++q) reinterpret_cast<Res*>(h_res.data() + (size_t)q * kRes)->len = jobs[q].L;
    c->where.store("large_items: bounce alloc");
    for (int b = 0; b < kNBounce; ++b) {
        if (!c->h_bounce[b] && hipHostMalloc(&c->h_bounce[b], kBounce, hipHostMallocDefault) != hipSuccess) {
            c->h_bounce[b] = nullptr;
            return nomem();
        }
        if (!c->ev_bounce[b]) HIP_TRY(hipEventCreateWithFlags(&c->ev_bounce[b], hipEventDisableTiming));
    }
    for (int b = 0; b < 2; ++b)
        if (!c->ev_piece_free[b]) HIP_TRY(hipEventCreateWithFlags(&c->ev_piece_free[b], hipEventDisableTiming));
    c->where.store("large_items: events / copy_stream2");
    if (!c->copy_stream2) HIP_TRY(hipStreamCreateWithFlags(&c->copy_stream2, hipStreamNonBlocking));
    if (!c->ev_copy2_join) HIP_TRY(hipEventCreateWithFlags(&c->ev_copy2_join, hipEventDisableTiming));
    uint64_t* sums = nullptr;
    c->where.store("large_items: scratch lease");
    oxh::ScratchLease lease(c->stream);  // block sums of the two rounds in flight
    c->where.store("large_items: scratch get");
    const uint64_t sums_per = (cap >> 10) * 8;
    if (lease.get(2 * sums_per * 8 * (uint64_t)n, (void**)&sums) != hipSuccess) return nomem();
    HIP_TRY(hipMemcpyAsync(d_res_all, h_res.data(), h_res.size(), hipMemcpyHostToDevice, c->stream));

    // one copy-done event per item (created before any sink temp exists: a failure here leaves nothing behind)
    std::vector<hipEvent_t> ev_copy(n, nullptr);
    for (int q = 0; q < n; ++q)
        if (hipEventCreateWithFlags(&ev_copy[q], hipEventDisableTiming) != hipSuccess) {
            (void)hipGetLastError();
            for (hipEvent_t e : ev_copy)
                if (e) (void)hipEventDestroy(e);
            return fail(OXH_ERR_HIP, "large-item events");
        }
    struct State {
        uint64_t k = 0;  // pieces 0 .. k-1 hold P bytes each; the last one L - k*P bytes, in [1025, P + 1024]
        std::string sink_tmp;
        int sfd = -1;
        std::atomic<bool> sink_ok{true};
        bool io_ok = true;
    };
    std::vector<State> st(n);
    uint64_t rounds = 0;
    for (int q = 0; q < n; ++q) {
        const uint64_t L = jobs[q].L;
        st[q].k = L > P + 1024 ? (L - 1025) / P : 0;
        rounds = std::max(rounds, st[q].k + 1);
        if (jobs[q].sink) {
            st[q].sfd = jobs[q].sink->open_stream(jobs[q].id, st[q].sink_tmp);
            if (st[q].sfd < 0) st[q].sink_ok.store(false);
        }
    }
    int rc = OXH_OK;
    // piece [off, off + plen) of item q -> device buffer d on the copy stream; false on an I/O error.
    // The piece goes through the bounce ring in windows of kBounce: up to kNBounce - 1 windows are read
    // at once (their 4 MiB parts queued on the pool without a barrier between windows), and a window's
    // H2D is issued as soon as its own parts are done (r05; r03-r04 read one window at a time).
    struct Window {
        int bb = 0;
        uint64_t o = 0, m = 0;
        std::atomic<bool> bad{false};
        std::function<void(int)> fn;
        oxh::Pool::Group grp;
    };
    auto copy_piece = [&](int q, uint64_t off, uint64_t plen, uint8_t* d) -> bool {
        LargeSource& src = *jobs[q].src;
        State& S = st[q];
        std::vector<std::unique_ptr<Window>> wins;
        std::deque<Window*> inflight;
        bool ok = true;
        auto finish = [&](Window& W) {
            c->where.store("copy_piece: window reads");
            W.grp.wait();
            c->where.store("copy_piece: window H2D");
            if (W.bad.load()) ok = false;
            if (!ok) return;
            // windows alternate over two copy streams: two DMA queues keep the PCIe link busier (the
            // FastCDC host pipeline measured 53.5 vs 47 GB/s)
            hipStream_t cs = (big_copy_streams() == 2 && ((W.o / kBounce) & 1)) ? c->copy_stream2 : c->copy_stream;
            if (hipMemcpyAsync(d + W.o, c->h_bounce[W.bb], W.m, hipMemcpyHostToDevice, cs) != hipSuccess ||
                hipEventRecord(c->ev_bounce[W.bb], cs) != hipSuccess) {
                ok = false;
                return;
            }
            c->bounce_used[W.bb] = true;
        };
        for (uint64_t o = 0; o < plen && ok; o += kBounce) {
            wins.emplace_back(new Window);
            Window& W = *wins.back();
            W.bb = (int)(c->bounce_next++ % kNBounce);
            W.o = o;
            W.m = std::min(kBounce, plen - o);
            c->where.store("copy_piece: bounce event");
            if (c->bounce_used[W.bb] && hipEventSynchronize(c->ev_bounce[W.bb]) != hipSuccess) {
                ok = false;
                break;
            }
            c->where.store("copy_piece: start window");
            c->bounce_used[W.bb] = false;
            src.will_need(off + o + W.m, 2 * kBounce);  // two windows ahead of the ones being read
            uint8_t* buf = c->h_bounce[W.bb];
            const uint64_t base = off + o, m = W.m;
            W.fn = [&src, &S, &W, buf, base, m](int t) {
                const uint64_t lo = (uint64_t)t * kBigRead, hi = std::min(m, lo + kBigRead);
                if (!src.read(base + lo, hi - lo, buf + lo)) {
                    W.bad.store(true);
                    return;
                }
                if (S.sfd >= 0 && S.sink_ok.load(std::memory_order_relaxed))  // the same bytes to the temp blob
                    for (uint64_t put = lo; put < hi;) {
                        const ssize_t x = pwrite(S.sfd, buf + put, hi - put, (off_t)(base + put));
                        if (x <= 0) {
                            S.sink_ok.store(false);
                            break;
                        }
                        put += (uint64_t)x;
                    }
            };
            c->pool->start((int)((m + kBigRead - 1) / kBigRead), W.fn, W.grp);
            inflight.push_back(&W);
            if ((int)inflight.size() >= big_windows()) {
                finish(*inflight.front());
                inflight.pop_front();
            }
        }
        while (!inflight.empty()) {  // every started window is waited for, also after a failure
            finish(*inflight.front());
            inflight.pop_front();
        }
        // the piece's event is recorded on copy_stream: it waits for copy_stream2's windows first
        if (ok && (hipEventRecord(c->ev_copy2_join, c->copy_stream2) != hipSuccess ||
                   hipStreamWaitEvent(c->copy_stream, c->ev_copy2_join, 0) != hipSuccess))
            ok = false;
        // no wait for the copies here: the piece's kernels wait for the copy stream through ev_copy,
        // and a bounce buffer is refilled only after its own H2D (ev_bounce), so the next piece's reads
        // overlap this piece's last copies
        return ok;
    };
    // With OXH_BIG_DIRECT=1, pieces whose pages are in the page cache are pinned in place and copied
    // asynchronously; the next round's pieces are pinned while this round's copies run, and a round's
    // pins are released once its copies are done.
    std::vector<const uint8_t*> pinned(n, nullptr), next_pin(n, nullptr);
    std::vector<std::pair<int, const uint8_t*>> to_unpin;  // (item, pinned range) of copies in flight
    auto piece_len = [&](int q, uint64_t r) { return r < st[q].k ? P : jobs[q].L - r * P; };
    // Pinning page-cache pages in place (OXH_BIG_DIRECT=1) measured 10-27 ms per GiB to register and
    // ~10 ms per GiB to release on the MI355X boxes (r03, OXH_TRACE), more than the 16 pool threads take
    // to copy the same bytes into the pinned bounce buffers; the bounce path is the default.
    const bool may_pin = getenv("OXH_BIG_DIRECT") && atoi(getenv("OXH_BIG_DIRECT")) != 0;
    auto pin_round = [&](uint64_t r, std::vector<const uint8_t*>& into) {
        if (!may_pin) return;
        for (int q = 0; q < n; ++q) {
            if (into[q]) jobs[q].src->unpin(into[q]);
            into[q] = (!jobs[q].sink && st[q].io_ok && r <= st[q].k) ? jobs[q].src->pin(r * P, piece_len(q, r)) : nullptr;
        }
    };
    Trace tr;  // OXH_TRACE=1: where a batch's host time goes
    double t_pin = 0, t_wait = 0, t_unpin = 0, t_bounce = 0;
    const double t_start = Trace::now();
    {
        const double t0 = Trace::now();
        pin_round(0, next_pin);
        t_pin += Trace::now() - t0;
    }
    bool round_used[2] = {false, false};
    for (uint64_t r = 0; r < rounds && rc == OXH_OK; ++r) {
        const int b = (int)(r & 1);
        pinned.swap(next_pin);
        // the chains of round r-2 (which read buffers b and their block sums) are done
        c->where.store("large_items: piece free");
        if (round_used[b] && hipEventSynchronize(c->ev_piece_free[b]) != hipSuccess) {
            rc = fail(OXH_ERR_HIP, "large-item piece wait");
            break;
        }
        oxh::ChainBatch batch;
        int nj = 0;
        for (int q = 0; q < n; ++q) {
            State& S = st[q];
            if (!S.io_ok || r > S.k) {
                if (pinned[q]) jobs[q].src->unpin(pinned[q]);  // pinned ahead, before the item failed
                pinned[q] = nullptr;
                continue;
            }
            const uint64_t off = r * P, plen = piece_len(q, r);
            uint8_t* d = dbuf(q, b);
            if (pinned[q]) {  // copy-free: the DMA engine reads the page cache (a sink must see host bytes)
                if (hipMemcpyAsync(d, pinned[q], plen, hipMemcpyHostToDevice, c->copy_stream) != hipSuccess ||
                    hipEventRecord(ev_copy[q], c->copy_stream) != hipSuccess) {
                    rc = fail(OXH_ERR_HIP, "large-item piece copy");
                    break;
                }
                to_unpin.push_back({q, pinned[q]});
                pinned[q] = nullptr;
            } else {
                const double t0 = Trace::now();
                const bool copied = copy_piece(q, off, plen, d);
                t_bounce += Trace::now() - t0;
                if (!copied) {
                    S.io_ok = false;  // its earlier chains finish harmlessly; the item is reported as unreadable
                    continue;
                }
                if (hipEventRecord(ev_copy[q], c->copy_stream) != hipSuccess) {
                    rc = fail(OXH_ERR_HIP, "large-item piece event");
                    break;
                }
            }
            if (hipStreamWaitEvent(c->stream, ev_copy[q], 0) != hipSuccess) {
                rc = fail(OXH_ERR_HIP, "large-item piece wait");
                break;
            }
            uint64_t* s_q = sums + ((uint64_t)b * n + q) * sums_per;
            const bool last = r == S.k;
            const uint64_t nb = last ? (plen - 1) >> 10 : plen >> 10;
            const uint64_t nwaves = (nb + 3) / 4, blocks = (nwaves + 3) / 4;
            hipLaunchKernelGGL(oxh::xxh3_blocksum_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, c->stream, d, nb, s_q);
            if (jobs[q].want_counts)
                hipLaunchKernelGGL(oxh::text_count_kernel, dim3(2048), dim3(256), 0, c->stream, d, plen,
                                   (unsigned long long*)(d_res(q) + 2));
            if (r == 0 && jobs[q].want_utf8)
                hipLaunchKernelGGL(oxh::utf8_prefix_kernel, dim3(1), dim3(64), 0, c->stream, d, d_res(q) + 4, d_res(q) + 5,
                                   (uint64_t)1, (int32_t*)(d_res(q) + 6));
            batch.job[nj++] = {d, plen, s_q, d_res(q), jobs[q].L, d_res(q) + 7,
                               (r > 0 ? oxh::kChainResume : 0u) | (last ? 0u : oxh::kChainPartial)};
        }
        if (rc) break;
        if (nj) hipLaunchKernelGGL(oxh::xxh3_chain_kernel, dim3(nj), dim3(64), kChainLdsPad, c->stream, batch);
        if (hipGetLastError() != hipSuccess || hipEventRecord(c->ev_piece_free[b], c->stream) != hipSuccess)
            rc = fail(OXH_ERR_HIP, "large-item piece launch");
        round_used[b] = true;
        double t0 = Trace::now();
        if (r + 1 < rounds) pin_round(r + 1, next_pin);  // while this round's copies run
        t_pin += Trace::now() - t0;
        if (!to_unpin.empty()) {
            t0 = Trace::now();
            if (hipStreamSynchronize(c->copy_stream) != hipSuccess && rc == OXH_OK) rc = fail(OXH_ERR_HIP, "large-item copy");
            t_wait += Trace::now() - t0;
            t0 = Trace::now();
            for (const auto& u : to_unpin) jobs[u.first].src->unpin(u.second);
            t_unpin += Trace::now() - t0;
            to_unpin.clear();
        }
    }
    // a failure mid-way: release what is still pinned
    c->where.store("large_items: final copy sync");
    if (hipStreamSynchronize(c->copy_stream) != hipSuccess && rc == OXH_OK) rc = fail(OXH_ERR_HIP, "large-item copy");
    if (hipStreamSynchronize(c->copy_stream2) != hipSuccess && rc == OXH_OK) rc = fail(OXH_ERR_HIP, "large-item copy");
    for (int q = 0; q < n; ++q) {
        if (pinned[q]) jobs[q].src->unpin(pinned[q]);
        if (next_pin[q]) jobs[q].src->unpin(next_pin[q]);
    }
    for (const auto& u : to_unpin) jobs[u.first].src->unpin(u.second);
    if (rc == OXH_OK && hipMemcpyAsync(h_res.data(), d_res_all, h_res.size(), hipMemcpyDeviceToHost, c->stream) != hipSuccess)
        rc = fail(OXH_ERR_HIP, "large-item results D2H");
    const double t_tail0 = Trace::now();
    c->where.store("large_items: results sync");
    if (hipStreamSynchronize(c->stream) != hipSuccess && rc == OXH_OK) rc = fail(OXH_ERR_HIP, "large-item sync");
    c->where.store("large_items: publish");
    if (tr.on)
        fprintf(stderr, "[oxh] large_items n=%d rounds=%llu piece=%llu MiB: total %.1f ms, pin %.1f, copy wait %.1f, unpin %.1f, "
                "bounce %.1f, chain tail %.1f\n", n, (unsigned long long)rounds, (unsigned long long)(P >> 20),
                1e3 * (Trace::now() - t_start), 1e3 * t_pin, 1e3 * t_wait, 1e3 * t_unpin, 1e3 * t_bounce,
                1e3 * (Trace::now() - t_tail0));
    std::vector<ItemSink*> sinks;
    for (int q = 0; q < n; ++q) {
        const Res& h = *reinterpret_cast<const Res*>(h_res.data() + (size_t)q * kRes);
        if (jobs[q].sink) {  // publish (or drop) the temp blob now that the digest is known
            jobs[q].sink->close_stream(jobs[q].id, st[q].sfd, st[q].sink_tmp,
                                       rc == OXH_OK && st[q].io_ok && st[q].sink_ok.load(), h.out[0], h.out[1]);
            if (std::find(sinks.begin(), sinks.end(), jobs[q].sink) == sinks.end()) sinks.push_back(jobs[q].sink);
        }
        LargeResult& res = jobs[q].res;
        if (rc) continue;
        if (!st[q].io_ok) {
            res.status = OXH_ERR_IO;
            res.os_error = jobs[q].src->os_error.load();
            continue;
        }
        res.out[0] = h.out[0];
        res.out[1] = h.out[1];
        res.cnt[0] = 1 + h.cnt[0];
        res.cnt[1] = jobs[q].L - h.cnt[1];
        res.utf8 = h.utf8;
    }
    for (ItemSink* k : sinks) k->commit();
    for (hipEvent_t e : ev_copy) (void)hipEventDestroy(e);
    return rc;
}

// One large item (host buffers of oxh_hash_buffers / _streams, and the single-file case).
int large_item(oxh_ctx* c, uint64_t L, LargeSource& src, bool want_counts, bool want_utf8, ItemSink* sink, uint64_t id,
               LargeResult& res) {
    LargeJob j;
    j.L = L, j.src = &src, j.want_counts = want_counts, j.want_utf8 = want_utf8, j.sink = sink, j.id = id;
    const int rc = large_items(c, &j, 1);
    res = j.res;
    return rc;
}

}  // namespace oxh::capi
