// oxen_amd/csrc/xxh3_stream.hip -- the streaming Xxh3 (oxh_xxh3_stream_*): xxhash-rust's Xxh3::new /
// update / digest128 with the device doing the hashing. See capi_internal.hpp for the pieces.
#include "capi_internal.hpp"

using namespace oxh::capi;

// ---------------------------------------------------------------- streaming XXH3 (Xxh3)
// xxhash-rust's Xxh3::new / update / digest128 (hasher.rs:9,73-76,157-173, 183-244), with the device
// doing the hashing: bytes collect in a pinned buffer (grown on demand) of up to S + 1025 bytes (S = OXH_STREAM_PIECE_MIB,
// default 16 MiB, whole 1 KiB blocks); each time it fills, its first S bytes go to the device as one
// K1L piece (block sums chip-wide, then the chain resumed from the stream's 8 accumulators, which stay
// in device memory) and the last 1025 bytes move to the front. XXH3 scrambles every block but the
// last and reads the last stripe at len - 64, so keeping > 1 KiB back means the digest always has
// the item's tail on hand. digest128() hashes what is pending as the final piece without changing
// the state (updates may continue). Memory stays bounded whatever the stream's length.
struct oxh_xxh3_stream {
    int device = 0;
    uint64_t piece = 0;           // S
    uint8_t* h_pend = nullptr;    // pinned, grown on demand up to S + 1025
    uint64_t h_cap = 0;
    uint64_t fill = 0, total = 0, pieces = 0;
    uint8_t* d_mem = nullptr;     // [piece 0 | piece 1 | sums 0 | sums 1 | state 8 | out 2], from the first piece on
    uint8_t* d_piece[2] = {};
    uint64_t* d_sums[2] = {};
    uint64_t *d_state = nullptr, *d_out = nullptr;
    uint8_t* d_one = nullptr;     // a stream that never reached a piece: its bytes + out, grown on demand
    uint64_t d_one_cap = 0;
    hipStream_t st = nullptr;
    hipEvent_t ev_copied = nullptr, ev_free[2] = {};
    bool used[2] = {};
};


namespace oxh::capi {


// the stream and its events are created on first device use: a short-lived Xxh3 over a small blob
// (HashingReader / AtomicFile over one received file) pays for neither until its digest
int stream_queue(oxh_xxh3_stream* s) {
    if (s->st) return OXH_OK;
    if (hipStreamCreateWithFlags(&s->st, hipStreamNonBlocking) != hipSuccess) {
        s->st = nullptr;
        (void)hipGetLastError();
        return fail(OXH_ERR_NOMEM, "stream queue");
    }
    return OXH_OK;
}

int stream_device(oxh_xxh3_stream* s) {
    if (s->d_mem) return OXH_OK;
    if (int rc = stream_queue(s)) return rc;
    if (hipEventCreateWithFlags(&s->ev_copied, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&s->ev_free[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&s->ev_free[1], hipEventDisableTiming) != hipSuccess) {
        (void)hipGetLastError();
        return fail(OXH_ERR_NOMEM, "stream events");
    }
    const uint64_t pb = align_up(s->piece + 1025) + 256, sb = ((s->piece >> 10) + 1) * 64;
    if (hipMalloc(&s->d_mem, 2 * pb + 2 * sb + 256) != hipSuccess) {
        s->d_mem = nullptr;
        (void)hipGetLastError();
        return fail(OXH_ERR_NOMEM, "stream device buffers");
    }
    s->d_piece[0] = s->d_mem;
    s->d_piece[1] = s->d_mem + pb;
    s->d_sums[0] = reinterpret_cast<uint64_t*>(s->d_mem + 2 * pb);
    s->d_sums[1] = reinterpret_cast<uint64_t*>(s->d_mem + 2 * pb + sb);
    s->d_state = reinterpret_cast<uint64_t*>(s->d_mem + 2 * pb + 2 * sb);
    s->d_out = s->d_state + 8;
    return OXH_OK;
}

// room for `need` pending bytes (pinned; grown x4 from 64 KiB, capped at S + 1025)
int stream_reserve(oxh_xxh3_stream* s, uint64_t need) {
    if (need <= s->h_cap) return OXH_OK;
    const uint64_t full = s->piece + 1025;
    const uint64_t cap = std::min(full, std::max({need, 4 * s->h_cap, (uint64_t)64 << 10}));
    uint8_t* h = nullptr;
    if (hipHostMalloc(&h, cap, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        return fail(OXH_ERR_NOMEM, "stream pending buffer");
    }
    if (s->fill) memcpy(h, s->h_pend, s->fill);
    if (s->h_pend) (void)hipHostFree(s->h_pend);
    s->h_pend = h;
    s->h_cap = cap;
    return OXH_OK;
}

// the next device piece buffer, once the chain that last read it is done
int stream_take_piece(oxh_xxh3_stream* s, int& b) {
    b = (int)(s->pieces & 1);
    if (s->used[b]) HIP_TRY(hipEventSynchronize(s->ev_free[b]));
    return OXH_OK;
}

// block sums + chain of `len` bytes already in d_piece[b]
int stream_chain(oxh_xxh3_stream* s, int b, uint64_t len, bool partial) {
    const uint64_t nb = partial ? len >> 10 : (len - 1) >> 10;
    const uint64_t nwaves = (nb + 3) / 4, blocks = (nwaves + 3) / 4;
    if (blocks)
        hipLaunchKernelGGL(oxh::xxh3_blocksum_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, s->st, s->d_piece[b], nb,
                           s->d_sums[b]);
    oxh::ChainBatch batch;
    batch.job[0] = {s->d_piece[b], len, s->d_sums[b], s->d_out, s->total, s->d_state,
                    (s->pieces > 0 ? oxh::kChainResume : 0u) | (partial ? oxh::kChainPartial : 0u)};
    hipLaunchKernelGGL(oxh::xxh3_chain_kernel, dim3(1), dim3(64), kChainLdsPad, s->st, batch);
    HIP_TRY(hipGetLastError());
    return OXH_OK;
}

// the first S pending bytes become a piece; the last 1025 move to the front
int stream_flush(oxh_xxh3_stream* s) {
    if (int rc = stream_device(s)) return rc;
    int b = 0;
    if (int rc = stream_take_piece(s, b)) return rc;
    HIP_TRY(hipMemcpyAsync(s->d_piece[b], s->h_pend, s->piece, hipMemcpyHostToDevice, s->st));
    HIP_TRY(hipEventRecord(s->ev_copied, s->st));
    if (int rc = stream_chain(s, b, s->piece, true)) return rc;
    HIP_TRY(hipEventRecord(s->ev_free[b], s->st));
    s->used[b] = true;
    s->pieces++;
    HIP_TRY(hipEventSynchronize(s->ev_copied));  // the pinned bytes were read: reuse the buffer
    memmove(s->h_pend, s->h_pend + s->piece, 1025);
    s->fill = 1025;
    return OXH_OK;
}


}  // namespace oxh::capi

extern "C" {

int oxh_xxh3_stream_create(oxh_ctx* ctx, oxh_xxh3_stream** out) {
    if (!ctx || !out) return fail(OXH_ERR_INVALID, "bad stream arguments");
    *out = nullptr;
    oxh_xxh3_stream* s = new oxh_xxh3_stream();
    s->device = ctx->device;
    const char* e = getenv("OXH_STREAM_PIECE_MIB");
    const uint64_t kib = e && strtoull(e, nullptr, 10) ? strtoull(e, nullptr, 10) << 10 : 16ull << 10;
    s->piece = kib << 10;  // whole 1 KiB blocks
    *out = s;              // nothing is allocated until bytes arrive
    return OXH_OK;
}

int oxh_xxh3_stream_update(oxh_xxh3_stream* s, const void* data, uint64_t len) {
    if (!s || (len && !data)) return fail(OXH_ERR_INVALID, "bad stream update");
    if (!len) return OXH_OK;
    HIP_TRY(hipSetDevice(s->device));
    const uint8_t* p = (const uint8_t*)data;
    const uint64_t cap = s->piece + 1025;
    while (len) {
        const uint64_t take = std::min(len, cap - s->fill);
        g_stream_where.store("update: reserve");
        if (int rc = stream_reserve(s, s->fill + take)) return rc;
        g_stream_where.store("update: copy");
        memcpy(s->h_pend + s->fill, p, take);
        s->fill += take;
        s->total += take;
        p += take;
        len -= take;
        if (s->fill == cap) {
            g_stream_where.store("update: flush");
            if (int rc = stream_flush(s)) return rc;
        }
    }
    g_stream_where.store("update: done");
    return OXH_OK;
}

int oxh_xxh3_stream_digest(oxh_xxh3_stream* s, uint64_t* out2) {
    if (!s || !out2) return fail(OXH_ERR_INVALID, "bad stream digest");
    HIP_TRY(hipSetDevice(s->device));
    g_stream_where.store("digest: queue");
    if (int rc = stream_queue(s)) return rc;
    g_stream_where.store("digest: final piece");
    uint64_t* d_out = nullptr;
    if (s->pieces == 0) {  // the whole stream is pending: a one-shot digest (K1, or K1L above 1 MiB)
        const uint64_t need = align_up(s->fill + 1) + 256;
        if (need > s->d_one_cap) {
            if (s->d_one) (void)hipFree(s->d_one);
            s->d_one = nullptr, s->d_one_cap = 0;
            const uint64_t cap = std::max<uint64_t>(need, 64 << 10);
            if (hipMalloc(&s->d_one, cap) != hipSuccess) {
                s->d_one = nullptr;
                (void)hipGetLastError();
                return fail(OXH_ERR_NOMEM, "stream device buffer");
            }
            s->d_one_cap = cap;
        }
        d_out = reinterpret_cast<uint64_t*>(s->d_one + s->d_one_cap - 256);
        if (s->fill) HIP_TRY(hipMemcpyAsync(s->d_one, s->h_pend, s->fill, hipMemcpyHostToDevice, s->st));
        const uint8_t* d = s->d_one;
        if (int rc = large_batch_device(&d, &s->fill, 1, d_out, s->st)) return rc;
    } else {  // fill >= 1025: the final piece
        int b = 0;
        if (int rc = stream_take_piece(s, b)) return rc;
        HIP_TRY(hipMemcpyAsync(s->d_piece[b], s->h_pend, s->fill, hipMemcpyHostToDevice, s->st));
        if (int rc = stream_chain(s, b, s->fill, false)) return rc;
        HIP_TRY(hipEventRecord(s->ev_free[b], s->st));
        s->used[b] = true;
        d_out = s->d_out;
    }
    uint64_t h[2];
    HIP_TRY(hipMemcpyAsync(h, d_out, 16, hipMemcpyDeviceToHost, s->st));
    HIP_TRY(hipStreamSynchronize(s->st));
    out2[0] = h[0];
    out2[1] = h[1];
    return OXH_OK;
}

int oxh_xxh3_stream_reset(oxh_xxh3_stream* s) {
    if (!s) return fail(OXH_ERR_INVALID, "stream is NULL");
    if (s->st) HIP_TRY(hipStreamSynchronize(s->st));
    s->fill = s->total = s->pieces = 0;
    return OXH_OK;
}

int oxh_xxh3_stream_destroy(oxh_xxh3_stream* s) {
    if (!s) return OXH_OK;
    (void)hipSetDevice(s->device);
    g_stream_where.store("destroy: sync");
    if (s->st) (void)hipStreamSynchronize(s->st);
    g_stream_where.store("destroy: free");
    if (s->d_mem) (void)hipFree(s->d_mem);
    if (s->d_one) (void)hipFree(s->d_one);
    if (s->h_pend) (void)hipHostFree(s->h_pend);
    if (s->ev_copied) (void)hipEventDestroy(s->ev_copied);
    for (hipEvent_t e : s->ev_free)
        if (e) (void)hipEventDestroy(e);
    if (s->st) (void)hipStreamDestroy(s->st);
    delete s;
    g_stream_where.store("destroy: done");
    return OXH_OK;
}

}  // extern "C"
