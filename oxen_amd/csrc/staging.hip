// oxen_amd/csrc/staging.hip -- host-resident batches through the context's staging slots: packed into a
// pinned slot, H2D on the copy stream, K1 on the compute stream, digests back D2H while the next slot
// fills (oxh_hash_buffers, oxh_hash_streams); the slot submit / wait the file engine shares.
// See capi_internal.hpp for the pieces.
#include "capi_internal.hpp"

using namespace oxh::capi;

namespace oxh::capi {

// The batch's large items for K1L, at most kChainJobs (the largest): one K1 wave reads ~10 GB/s, so a
// batch holding a few large files waited on their waves -- a 200 MiB file ~20 ms against ~4 ms to copy
// it over PCIe, and one 1 MiB file ~100 us of a single-file call. K1L's block sums run chip-wide and
// its serial chain costs ~17 ns per KiB. In a K1T batch their text counts come from
// text_count_kernel (chip-wide) instead of the wave.
static uint64_t slot_chain_items(const uint64_t* hlen, uint64_t cnt, uint64_t* big) {
    static const bool on = !(getenv("OXH_SLOT_CHAINS") && atoi(getenv("OXH_SLOT_CHAINS")) == 0);
    uint64_t nbig = 0;
    if (!on) return 0;
    for (uint64_t j = 0; j < cnt; ++j) {
        if (hlen[j] < kSlotChainBytes) continue;
        if (nbig < (uint64_t)oxh::kChainJobs) {
            big[nbig++] = j;
            continue;
        }
        uint64_t m = 0;  // the smallest kept item gives way to a larger one
        for (uint64_t q = 1; q < nbig; ++q)
            if (hlen[big[q]] < hlen[big[m]]) m = q;
        if (hlen[j] > hlen[big[m]]) big[m] = j;
    }
    return nbig;
}

// One staged batch: items [0, cnt) already in h_stage[s] at h_desc offsets; launch and queue D2H.
int submit_slot(oxh_ctx* c, int s, uint64_t bytes, uint64_t cnt, bool any_short_only, bool short_items, bool text,
                bool utf8) {
    const uint64_t M = c->max_items;
    uint64_t big[oxh::kChainJobs];
    const uint64_t nbig = any_short_only ? 0 : slot_chain_items(c->h_desc[s] + M, cnt, big);
    STEP("submit s=%d bytes=%llu cnt=%llu lane=%d short=%d", s, (unsigned long long)bytes, (unsigned long long)cnt,
         (int)any_short_only, (int)short_items);
    c->where.store("submit_slot: H2D stage");
    HIP_TRY(hipMemcpyAsync(c->d_stage[s], c->h_stage[s], bytes, hipMemcpyHostToDevice, c->copy_stream));
    c->where.store("submit_slot: H2D desc");
    HIP_TRY(hipMemcpyAsync(c->d_desc[s], c->h_desc[s], cnt * 8, hipMemcpyHostToDevice, c->copy_stream));
    HIP_TRY(hipMemcpyAsync(c->d_desc[s] + M, c->h_desc[s] + M, cnt * 8, hipMemcpyHostToDevice, c->copy_stream));
    const uint64_t* d_wave_lens = c->d_desc[s] + M;
    if (nbig) {  // the wave launch sees the K1L items as empty
        memcpy(c->h_klen[s], c->h_desc[s] + M, cnt * 8);
        for (uint64_t q = 0; q < nbig; ++q) c->h_klen[s][big[q]] = 0;
        HIP_TRY(hipMemcpyAsync(c->d_klen[s], c->h_klen[s], cnt * 8, hipMemcpyHostToDevice, c->copy_stream));
        d_wave_lens = c->d_klen[s];
    }
    c->where.store("submit_slot: record / wait");
    HIP_TRY(hipEventRecord(c->ev_copied[s], c->copy_stream));
    HIP_TRY(hipStreamWaitEvent(c->stream, c->ev_copied[s], 0));
    STEP("copies queued s=%d", s);
    c->where.store("submit_slot: launch");
    int rc = text ? launch_text(c->d_stage[s], c->d_desc[s], d_wave_lens, cnt, c->d_out[s], c->d_cnt[s], c->stream,
                                short_items)
             : any_short_only ? launch_lane(c->d_stage[s], c->d_desc[s], c->d_desc[s] + M, cnt, c->d_out[s], c->stream)
                              : launch_wave(c->d_stage[s], c->d_desc[s], d_wave_lens, cnt, c->d_out[s], c->stream,
                                            short_items ? ItemShape::Short : ItemShape::Long);
    if (rc) return rc;
    if (nbig) {  // K1L: each item's block sums chip-wide, then one launch of their chains (after the
                 // wave kernel on the same stream, so the chains' digests are the ones that stay)
        oxh::ChainBatch batch;
        uint64_t soff = 0;
        for (uint64_t q = 0; q < nbig; ++q) {
            const uint64_t j = big[q], L = c->h_desc[s][M + j], nb = (L - 1) >> 10;
            const uint8_t* p = c->d_stage[s] + c->h_desc[s][j];
            uint64_t* sums = c->d_sums[s] + soff;
            soff += nb * 8;
            const uint64_t blocks = ((nb + 3) / 4 + 3) / 4;
            if ((reinterpret_cast<uintptr_t>(p) & 15) == 0)
                hipLaunchKernelGGL(oxh::xxh3_blocksum_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, c->stream, p, nb, sums);
            else
                hipLaunchKernelGGL(oxh::xxh3_blocksum_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, c->stream, p, nb, sums);
            HIP_TRY(hipGetLastError());
            batch.job[q] = {p, L, sums, c->d_out[s] + 2 * j, L, nullptr, 0};
        }
        hipLaunchKernelGGL(oxh::xxh3_chain_kernel, dim3((unsigned)nbig), dim3(64), kChainLdsPad, c->stream, batch);
        HIP_TRY(hipGetLastError());
        if (text) {  // their counts: chip-wide sums, then MetadataText's form over the wave's (1, 0)
            unsigned long long* raw = (unsigned long long*)(c->d_sums[s] + slot_sums_words(c->stage_bytes));
            HIP_TRY(hipMemsetAsync(raw, 0, nbig * 16, c->stream));
            oxh::CountFix fix{};
            fix.n = (int)nbig;
            for (uint64_t q = 0; q < nbig; ++q) {
                const uint64_t j = big[q], L = c->h_desc[s][M + j];
                fix.j[q] = j, fix.len[q] = L;
                const unsigned grid = (unsigned)std::min<uint64_t>(2048, (L / 16 + 255) / 256 + 1);
                hipLaunchKernelGGL(oxh::text_count_kernel, dim3(grid), dim3(256), 0, c->stream, c->d_stage[s] + c->h_desc[s][j],
                                   L, raw + 2 * q);
                HIP_TRY(hipGetLastError());
            }
            hipLaunchKernelGGL(oxh::text_count_finish_kernel, dim3(1), dim3(64), 0, c->stream, raw, fix, c->d_cnt[s]);
            HIP_TRY(hipGetLastError());
        }
    }
    STEP("launched s=%d", s);
    c->where.store("submit_slot: D2H");
    HIP_TRY(hipMemcpyAsync(c->h_out[s], c->d_out[s], cnt * 16, hipMemcpyDeviceToHost, c->stream));
    if (text) HIP_TRY(hipMemcpyAsync(c->h_cnt[s], c->d_cnt[s], cnt * 16, hipMemcpyDeviceToHost, c->stream));
    if (utf8) {  // is_utf8 sniff of the same staged bytes
        hipLaunchKernelGGL(oxh::utf8_prefix_kernel, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, c->stream, c->d_stage[s],
                           c->d_desc[s], c->d_desc[s] + M, cnt, c->d_utf8[s]);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(c->h_utf8[s], c->d_utf8[s], cnt * 4, hipMemcpyDeviceToHost, c->stream));
    }
    c->where.store("submit_slot: record done");
    HIP_TRY(hipEventRecord(c->ev_done[s], c->stream));
    STEP("submitted s=%d", s);
    return OXH_OK;
}

// One small batch of the caller's thread (engine.hip direct_files), items below kSlotChainBytes: their
// descriptors go into the slot right after their bytes, so ONE H2D on the compute stream carries both
// (no copy-stream hop, no event between the streams), then K1 / K1T (+ is_utf8), D2H and the done
// event. Each host-to-device copy costs ~5 us of a small call's ~40 us round trip. False: it does not
// fit (the caller takes submit_slot). OXH_DIRECT_PACKED=0: always submit_slot.
int submit_packed(oxh_ctx* c, int s, uint64_t bytes, uint64_t cnt, bool short_items, bool text, bool utf8, bool& done,
                  bool lane) {
    static const bool on = !(getenv("OXH_DIRECT_PACKED") && atoi(getenv("OXH_DIRECT_PACKED")) == 0);
    const uint64_t M = c->max_items, doff = align_up(bytes);
    done = false;
    if (!on || doff + 16 * cnt > c->stage_bytes) return OXH_OK;
    for (uint64_t j = 0; j < cnt; ++j)
        if (c->h_desc[s][M + j] >= kSlotChainBytes) return OXH_OK;
    uint64_t* hd = reinterpret_cast<uint64_t*>(c->h_stage[s] + doff);
    memcpy(hd, c->h_desc[s], cnt * 8);
    memcpy(hd + cnt, c->h_desc[s] + M, cnt * 8);
    const uint64_t* d_offs = reinterpret_cast<const uint64_t*>(c->d_stage[s] + doff);
    const uint64_t* d_lens = d_offs + cnt;
    c->where.store("submit_packed: H2D");
    HIP_TRY(hipMemcpyAsync(c->d_stage[s], c->h_stage[s], doff + 16 * cnt, hipMemcpyHostToDevice, c->stream));
    int rc = text   ? launch_text(c->d_stage[s], d_offs, d_lens, cnt, c->d_out[s], c->d_cnt[s], c->stream, short_items)
             : lane ? launch_lane(c->d_stage[s], d_offs, d_lens, cnt, c->d_out[s], c->stream)
                    : launch_wave(c->d_stage[s], d_offs, d_lens, cnt, c->d_out[s], c->stream,
                                  short_items ? ItemShape::Short : ItemShape::Long);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(c->h_out[s], c->d_out[s], cnt * 16, hipMemcpyDeviceToHost, c->stream));
    if (text) HIP_TRY(hipMemcpyAsync(c->h_cnt[s], c->d_cnt[s], cnt * 16, hipMemcpyDeviceToHost, c->stream));
    if (utf8) {
        hipLaunchKernelGGL(oxh::utf8_prefix_kernel, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, c->stream, c->d_stage[s],
                           d_offs, d_lens, cnt, c->d_utf8[s]);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(c->h_utf8[s], c->d_utf8[s], cnt * 4, hipMemcpyDeviceToHost, c->stream));
    }
    HIP_TRY(hipEventRecord(c->ev_done[s], c->stream));
    done = true;
    return OXH_OK;
}

// Wait for slot s's digests. Polls (a slot is at most a few hundred MiB: milliseconds of work) and,
// after OXH_WAIT_LIMIT_S seconds (default 60), reports which stage never finished instead of
// blocking forever.
// OXH_SPIN_US: how long a caller waiting on a staged batch spins before it sleeps (default 200; 0 =
// sleep after 64 polls, the r02-r05 form)
double spin_us() {
    static const double v = getenv("OXH_SPIN_US") ? atof(getenv("OXH_SPIN_US")) : 200.0;
    return v;
}

int wait_slot(oxh_ctx* c, int s, const Pending& p) {
    static const double limit = getenv("OXH_WAIT_LIMIT_S") ? atof(getenv("OXH_WAIT_LIMIT_S")) : 60.0;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t spin = 0;; ++spin) {
        const hipError_t q = hipEventQuery(c->ev_done[s]);
        if (q == hipSuccess) return OXH_OK;
        if (q != hipErrorNotReady) return fail(OXH_ERR_HIP, std::string("slot event: ") + hipGetErrorString(q));
        // a small batch is back within tens of us: spin (yielding) for the first spin_us(), then sleep
        // in 20 us steps (a caller's own thread keeps its timer slack, so a sleep costs ~70 us)
        if (spin > 64 && std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() * 1e6 > spin_us())
            std::this_thread::sleep_for(std::chrono::microseconds(20));
        else
            std::this_thread::yield();
        if ((spin & 1023) == 0 &&
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit) {
            const uint64_t M = c->max_items;
            fprintf(stderr, "[oxh] slot %d stalled: items=%zu copied=%s copy_stream=%s stream=%s first lens:", s,
                    p.ids.size(), hipGetErrorName(hipEventQuery(c->ev_copied[s])),
                    hipGetErrorName(hipStreamQuery(c->copy_stream)), hipGetErrorName(hipStreamQuery(c->stream)));
            for (size_t j = 0; j < std::min<size_t>(p.ids.size(), 16); ++j)
                fprintf(stderr, " %llu@%llu", (unsigned long long)c->h_desc[s][M + j], (unsigned long long)c->h_desc[s][j]);
            fprintf(stderr, "\n");
            return fail(OXH_ERR_HIP, "timed out waiting for a staged batch (see stderr)");
        }
    }
}

// Scatter slot s's digests to the caller's table (host-buffer batches: oxh_hash_buffers/_streams).
int drain_slot(oxh_ctx* c, int s, Pending& p, uint64_t* out) {
    if (!p.busy) return OXH_OK;
    STEP("drain s=%d", s);
    if (int rc = wait_slot(c, s, p)) return rc;
    for (size_t j = 0; j < p.ids.size(); ++j) {
        out[2 * p.ids[j]] = c->h_out[s][2 * j];
        out[2 * p.ids[j] + 1] = c->h_out[s][2 * j + 1];
    }
    p.busy = false;
    p.ids.clear();
    return OXH_OK;
}

}  // namespace oxh::capi

// Host-resident buffers (oxh_hash_buffers / oxh_hash_streams): item i (lens[i] bytes) is copied by
// copy(i, dst) straight into a pinned slot; slots are packed greedily in order, hashed on the GPU
// while the next one fills, and items larger than a slot go through the oversize path.
// Items of the short XXH3 paths (<= 240 B: paths, metadata JSON, most parent-node streams) are packed
// back to back: their kernels load unaligned bytes anyway, and 256-B slots would move ~8x their bytes
// over PCIe (a commit's 200 000 bucket paths: 6.3 MB instead of 51 MB). Longer items start on 256 B.
// OXH_HOST_ALIGN_ALL=1: every item on 256 B (the r02 packing, for A/B).
static uint64_t place(uint64_t off, uint64_t len) {
    static const bool all = getenv("OXH_HOST_ALIGN_ALL") && atoi(getenv("OXH_HOST_ALIGN_ALL")) != 0;
    return (len > 240 || all) ? align_up(off) : off;
}

static int hash_host_items(oxh_ctx* c, uint64_t n, const uint64_t* lens,
                           const std::function<const uint8_t*(uint64_t)>& src, uint64_t* out, bool short_only_lane) {
    Trace tr;
    Pending pend[NSLOT];
    int slot = 0;
    uint64_t i = 0;
    std::vector<uint64_t> batch;
    while (i < n) {
        batch.clear();
        uint64_t bytes = 0;
        while (i < n && batch.size() < c->max_items) {
            const uint64_t L = lens[i];
            if (L > c->stage_bytes) {  // straight from the caller's buffer, in pieces (large_item)
                if (!batch.empty()) break;
                MemSource ms(src(i));
                LargeResult res;
                if (int rc = large_item(c, L, ms, false, false, nullptr, i, res)) return rc;
                if (res.status != OXH_OK) return fail(res.status, "large host buffer: device or pinned memory unavailable");
                out[2 * i] = res.out[0];
                out[2 * i + 1] = res.out[1];
                ++i;
                continue;
            }
            if (place(bytes, L) + L > c->stage_bytes) break;
            bytes = place(bytes, L) + L;
            batch.push_back(i);
            ++i;
        }
        if (batch.empty()) continue;
        const int s = slot;
        slot = (slot + 1) % NSLOT;
        const double t0 = Trace::now();
        if (int rc = drain_slot(c, s, pend[s], out)) return rc;  // the slot's previous batch
        const double t1 = Trace::now();
        tr.drain += t1 - t0;
        const uint64_t M = c->max_items;
        uint64_t* hoff = c->h_desc[s];
        uint64_t* hlen = c->h_desc[s] + M;
        uint64_t off = 0;
        bool all_short = true;
        for (size_t j = 0; j < batch.size(); ++j) {
            off = place(off, lens[batch[j]]);
            hoff[j] = off;
            hlen[j] = lens[batch[j]];
            if (hlen[j] > 240) all_short = false;
            off += hlen[j];
        }
        STEP("fill s=%d items=%zu", s, batch.size());
        // a small batch is copied on this thread: handing 1 MiB or less to the pool costs more in
        // wake-ups than the copy (tools/latency_probe.py, one 4 KiB buffer). Otherwise the pool copies
        // pieces of at most 4 MiB, so one large buffer is not one thread's memcpy (~10 GB/s)
        if (off <= (1u << 20)) {
            for (size_t j = 0; j < batch.size(); ++j)
                if (hlen[j]) memcpy(c->h_stage[s] + hoff[j], src(batch[j]), hlen[j]);
        } else {
            constexpr uint64_t kPiece = 4ull << 20;
            std::vector<std::array<uint64_t, 3>> pieces;  // (j, lo, hi) of item j's bytes
            for (size_t j = 0; j < batch.size(); ++j)
                for (uint64_t lo = 0; lo < hlen[j]; lo += kPiece) pieces.push_back({j, lo, std::min(hlen[j], lo + kPiece)});
            const int ntasks = (int)std::min<size_t>(pieces.size(), (size_t)c->pool->size() * 4);
            c->pool->parallel_for(ntasks, [&](int t) {
                for (size_t k = (size_t)t; k < pieces.size(); k += (size_t)ntasks) {
                    const auto& pc = pieces[k];
                    memcpy(c->h_stage[s] + hoff[pc[0]] + pc[1], src(batch[pc[0]]) + pc[1], pc[2] - pc[1]);
                }
            });
        }
        const double t2 = Trace::now();
        tr.fill += t2 - t1;
        // a call that is one small batch: descriptors packed after the bytes, one H2D (submit_packed)
        bool packed = false;
        const bool short_items = off / std::max<uint64_t>(1, batch.size()) <= kShortItemBytes;
        if (off <= (1u << 20) && i == n && tr.batches == 0)
            if (int rc = submit_packed(c, s, off, batch.size(), short_items, false, false, packed, short_only_lane && all_short))
                return rc;
        if (!packed)
            if (int rc = submit_slot(c, s, off, batch.size(), short_only_lane && all_short, short_items, false)) return rc;
        tr.submit += Trace::now() - t2;
        tr.batches++;
        pend[s].busy = true;
        pend[s].ids = batch;
    }
    const double t3 = Trace::now();
    STEP("final drain");
    for (int s = 0; s < NSLOT; ++s)
        if (int rc = drain_slot(c, s, pend[s], out)) return rc;
    tr.drain += Trace::now() - t3;
    if (tr.on)
        fprintf(stderr, "[oxh] items=%llu batches=%d fill=%.3fs drain-wait=%.3fs submit=%.3fs threads=%d\n",
                (unsigned long long)n, tr.batches, tr.fill, tr.drain, tr.submit, c->pool->size());
    return OXH_OK;
}


extern "C" {

int oxh_hash_buffers(oxh_ctx* c, const uint8_t* const* bufs, const uint64_t* lens, uint64_t n, uint64_t* out) {
    if (!c || (n && (!bufs || !lens || !out))) return fail(OXH_ERR_INVALID, "bad arguments");
    std::lock_guard<std::mutex> g(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    return hash_host_items(c, n, lens, [&](uint64_t i) { return bufs[i]; }, out, false);
}

}  // extern "C"

// oxh_hash_streams over an arena whose items run forward (offsets non-decreasing, gaps at most as
// large as the items): each batch is ONE span of the arena, copied into the pinned slot in large
// pieces by the pool, with the items' offsets rebased onto it -- no per-item copy. A commit's
// 200 000 bucket paths are such an arena (the serialised streams of commit_writer); a per-item copy
// of them costs ~12 ns an item on the host. Items larger than a slot go the oversize path as before.
static int hash_stream_spans(oxh_ctx* c, const uint8_t* streams, const uint64_t* offsets, const uint64_t* lens, uint64_t n,
                             uint64_t* out) {
    Trace tr;
    Pending pend[NSLOT];
    int slot = 0;
    uint64_t i = 0;
    std::vector<uint64_t> batch;
    while (i < n) {
        if (lens[i] > c->stage_bytes) {  // straight from the caller's buffer, in pieces (large_item)
            MemSource ms(streams + offsets[i]);
            LargeResult res;
            if (int rc = large_item(c, lens[i], ms, false, false, nullptr, i, res)) return rc;
            if (res.status != OXH_OK) return fail(res.status, "large host buffer: device or pinned memory unavailable");
            out[2 * i] = res.out[0];
            out[2 * i + 1] = res.out[1];
            ++i;
            continue;
        }
        const uint64_t base = offsets[i];
        uint64_t end = base, k = i;
        bool all_short = true;
        batch.clear();
        while (k < n && batch.size() < c->max_items && lens[k] <= c->stage_bytes &&
               std::max(end, offsets[k] + lens[k]) - base <= c->stage_bytes) {
            end = std::max(end, offsets[k] + lens[k]);
            if (lens[k] > 240) all_short = false;
            batch.push_back(k++);
        }
        const int s = slot;
        slot = (slot + 1) % NSLOT;
        const double t0 = Trace::now();
        if (int rc = drain_slot(c, s, pend[s], out)) return rc;  // the slot's previous batch
        const double t1 = Trace::now();
        tr.drain += t1 - t0;
        const uint64_t M = c->max_items;
        uint64_t* hoff = c->h_desc[s];
        uint64_t* hlen = c->h_desc[s] + M;
        for (size_t j = 0; j < batch.size(); ++j) {
            hoff[j] = offsets[batch[j]] - base;
            hlen[j] = lens[batch[j]];
        }
        const uint64_t span = end - base, piece = 1ull << 20;
        const int ntasks = (int)std::min<uint64_t>((span + piece - 1) / piece, (uint64_t)c->pool->size() * 4);
        if (ntasks > 1) {
            c->pool->parallel_for(ntasks, [&](int t) {
                const uint64_t lo = span * (uint64_t)t / (uint64_t)ntasks, hi = span * (uint64_t)(t + 1) / (uint64_t)ntasks;
                memcpy(c->h_stage[s] + lo, streams + base + lo, hi - lo);
            });
        } else if (span) {
            memcpy(c->h_stage[s], streams + base, span);
        }
        const double t2 = Trace::now();
        tr.fill += t2 - t1;
        // a call that is one small span: descriptors packed after the bytes, one H2D (submit_packed)
        bool packed = false;
        const bool short_items = span / std::max<uint64_t>(1, batch.size()) <= kShortItemBytes;
        if (span <= (1u << 20) && k == n && tr.batches == 0)
            if (int rc = submit_packed(c, s, span, batch.size(), short_items, false, false, packed, all_short)) return rc;
        if (!packed)
            if (int rc = submit_slot(c, s, span, batch.size(), all_short, short_items, false)) return rc;
        tr.submit += Trace::now() - t2;
        tr.batches++;
        pend[s].busy = true;
        pend[s].ids = batch;
        i = k;
    }
    const double t3 = Trace::now();
    for (int s = 0; s < NSLOT; ++s)
        if (int rc = drain_slot(c, s, pend[s], out)) return rc;
    tr.drain += Trace::now() - t3;
    if (tr.on)
        fprintf(stderr, "[oxh] streams (spans)=%llu batches=%d fill=%.3fs drain-wait=%.3fs submit=%.3fs\n",
                (unsigned long long)n, tr.batches, tr.fill, tr.drain, tr.submit);
    return OXH_OK;
}

extern "C" {

int oxh_hash_streams(oxh_ctx* c, const uint8_t* streams, const uint64_t* offsets, const uint64_t* lens, uint64_t n,
                     uint64_t* out) {
    if (!c || (n && (!streams || !offsets || !lens || !out))) return fail(OXH_ERR_INVALID, "bad arguments");
    STEP("hash_streams n=%llu", (unsigned long long)n);
    std::lock_guard<std::mutex> g(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    STEP("hash_streams locked");
    // spans when the items run forward through the arena without large gaps (OXH_STREAM_SPANS=0: per item)
    static const bool spans_on = !(getenv("OXH_STREAM_SPANS") && atoi(getenv("OXH_STREAM_SPANS")) == 0);
    bool forward = spans_on && n > 0;
    uint64_t total = 0, maxend = 0;
    for (uint64_t i = 0; forward && i < n; ++i) {
        total += lens[i];
        maxend = std::max(maxend, offsets[i] + lens[i]);
        if (i && offsets[i] < offsets[i - 1]) forward = false;
    }
    if (forward && maxend - offsets[0] > 2 * total + 4096) forward = false;  // a sparse arena: copy items
    if (forward) return hash_stream_spans(c, streams, offsets, lens, n, out);
    return hash_host_items(c, n, lens, [&](uint64_t i) { return streams + offsets[i]; }, out, true);
}

}  // extern "C"
