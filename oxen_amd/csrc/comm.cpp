// oxen_amd/csrc/comm.cpp -- the digest-table gather of a multi-GPU add (include/oxen_hash.h, oxh_comm_*).
//
// SURVEY.md §8e / BASELINE north_star: files shard across the GPUs of a node with no data-path
// collective (contiguous byte-balanced ranges, each rank hashing its own share with K1), and ONE
// exchange at the end -- the 16-B-per-file digest tables gathered over xGMI with RCCL. This is the
// point where a Rust liboxen replacing the fan-out of add.rs:422-425 with device-resident shards
// collects every rank's FileNode hashes, so it sits behind the C ABI, with plain pointers only.
//
// RCCL is opened at run time (dlopen of librccl.so.1; OXH_RCCL_LIB overrides) rather than linked: a
// single-GPU caller never loads it, and a process that already holds an RCCL (PyTorch's) shares the
// loaded one when the sonames match.
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>
#include <dlfcn.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/oxen_hash.h"

namespace oxh {
int set_error(int code, const std::string& msg);  // capi_context.hip
}

namespace {

struct Rccl {
    void* so = nullptr;
    std::string error;
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*gather)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
};

// the process's RCCL, opened once
Rccl* rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        const char* names[] = {getenv("OXH_RCCL_LIB"), "librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
        for (const char* n : names)
            if (n && *n && (r.so = dlopen(n, RTLD_NOW | RTLD_LOCAL)) != nullptr) break;
        if (!r.so) {
            const char* e = dlerror();
            r.error = std::string("cannot load RCCL (librccl.so.1): ") + (e ? e : "");
            return;
        }
        auto sym = [&](const char* name, auto& fn) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(r.so, name));
            if (!fn && r.error.empty()) r.error = std::string("RCCL lacks ") + name;
        };
        sym("ncclGetUniqueId", r.get_unique_id);
        sym("ncclCommInitRank", r.comm_init_rank);
        sym("ncclCommDestroy", r.comm_destroy);
        sym("ncclAllGather", r.all_gather);
        sym("ncclBroadcast", r.broadcast);
        sym("ncclSend", r.send);
        sym("ncclRecv", r.recv);
        sym("ncclGroupStart", r.group_start);
        sym("ncclGroupEnd", r.group_end);
        sym("ncclGetErrorString", r.error_string);
        r.gather = reinterpret_cast<decltype(r.gather)>(dlsym(r.so, "ncclGather"));  // RCCL extension, optional
    });
    return r.error.empty() ? &r : nullptr;
}

int rccl_fail(const Rccl* r, ncclResult_t e, const char* what) {
    return oxh::set_error(OXH_ERR_HIP, std::string(what) + ": " + (r && r->error_string ? r->error_string(e) : "RCCL error"));
}

}  // namespace

struct oxh_comm {
    ncclComm_t comm = nullptr;
    int rank = 0, nranks = 1, device = 0;
};

extern "C" {

int oxh_comm_unique_id(uint8_t* id) {
    if (!id) return oxh::set_error(OXH_ERR_INVALID, "null id buffer");
    Rccl* r = rccl();
    if (!r) return oxh::set_error(OXH_ERR_NODEVICE, "RCCL unavailable");
    ncclUniqueId u;
    const ncclResult_t e = r->get_unique_id(&u);
    if (e != ncclSuccess) return rccl_fail(r, e, "ncclGetUniqueId");
    static_assert(sizeof(u) == OXH_COMM_ID_BYTES, "ncclUniqueId size");
    memcpy(id, &u, sizeof u);
    return OXH_OK;
}

int oxh_comm_check(int device) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        (void)hipGetLastError();
        return oxh::set_error(OXH_ERR_NODEVICE, "no HIP device visible");
    }
    if (device < 0 || device >= ndev) return oxh::set_error(OXH_ERR_INVALID, "device index out of range");
    if (!rccl()) return oxh::set_error(OXH_ERR_NODEVICE, "RCCL unavailable");
    return OXH_OK;
}

int oxh_comm_create(const uint8_t* id, int rank, int nranks, int device, oxh_comm** out) {
    if (!id || !out) return oxh::set_error(OXH_ERR_INVALID, "null argument");
    *out = nullptr;
    if (nranks < 1 || rank < 0 || rank >= nranks) return oxh::set_error(OXH_ERR_INVALID, "rank out of range");
    if (const int rc = oxh_comm_check(device); rc != OXH_OK) return rc;
    Rccl* r = rccl();
    int prev = 0;
    (void)hipGetDevice(&prev);
    if (hipSetDevice(device) != hipSuccess) return oxh::set_error(OXH_ERR_HIP, "hipSetDevice failed");
    ncclUniqueId u;
    memcpy(&u, id, sizeof u);
    auto* c = new oxh_comm;
    c->rank = rank, c->nranks = nranks, c->device = device;
    // blocks until every rank of the id has called it (RCCL's bootstrap)
    const ncclResult_t e = r->comm_init_rank(&c->comm, nranks, u, rank);
    (void)hipSetDevice(prev);
    if (e != ncclSuccess) {
        delete c;
        return rccl_fail(r, e, "ncclCommInitRank");
    }
    *out = c;
    return OXH_OK;
}

int oxh_comm_destroy(oxh_comm* c) {
    if (!c) return OXH_OK;
    Rccl* r = rccl();
    const ncclResult_t e = r ? r->comm_destroy(c->comm) : ncclSuccess;
    delete c;
    return e == ncclSuccess ? OXH_OK : rccl_fail(r, e, "ncclCommDestroy");
}

int oxh_comm_info(oxh_comm* c, int* rank, int* nranks, int* device) {
    if (!c) return oxh::set_error(OXH_ERR_INVALID, "null comm");
    if (rank) *rank = c->rank;
    if (nranks) *nranks = c->nranks;
    if (device) *device = c->device;
    return OXH_OK;
}

int oxh_gather_digests(oxh_comm* c, const uint64_t* d_local, const uint64_t* counts, uint64_t* d_full, int root,
                       void* stream) {
    if (!c || !counts) return oxh::set_error(OXH_ERR_INVALID, "null argument");
    if (root >= c->nranks) return oxh::set_error(OXH_ERR_INVALID, "root out of range");
    Rccl* r = rccl();
    if (!r) return oxh::set_error(OXH_ERR_NODEVICE, "RCCL unavailable");
    const int P = c->nranks, me = c->rank;
    std::vector<uint64_t> base(P + 1, 0);
    for (int q = 0; q < P; ++q) base[q + 1] = base[q] + counts[q];
    const bool receives = root < 0 || root == me;
    if (counts[me] && !d_local) return oxh::set_error(OXH_ERR_INVALID, "null local table");
    if (receives && base[P] && !d_full) return oxh::set_error(OXH_ERR_INVALID, "null full table");
    hipStream_t st = (hipStream_t)stream;
    // OXH_GATHER_P2P=1 takes the grouped point-to-point form even for equal shares (tests: the ragged
    // path on a one-GPU box)
    const char* pe = getenv("OXH_GATHER_P2P");
    const bool equal = !(pe && atoi(pe) != 0) && std::all_of(counts, counts + P, [&](uint64_t k) { return k == counts[0]; });
    const size_t words = 2 * (size_t)counts[0];  // a digest is two u64 (lo, hi)
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(c->device);
    ncclResult_t e = ncclSuccess;
    const char* what = "";
    if (equal && root < 0) {  // the table on every rank: one all-gather, rank order = table order
        what = "ncclAllGather";
        if (words) e = r->all_gather(d_local, d_full, words, ncclUint64, c->comm, st);
    } else if (equal && r->gather) {  // rank `root` only: RCCL's gather
        what = "ncclGather";
        if (words) e = r->gather(d_local, d_full, words, ncclUint64, root, c->comm, st);
    } else {
        // ragged shares (or an RCCL without ncclGather): point-to-point into each rank's slot of the
        // table, all in one group -- to `root`, or every rank's slot broadcast from its owner
        what = root < 0 ? "grouped ncclBroadcast" : "grouped ncclSend/ncclRecv";
        e = r->group_start();
        for (int q = 0; q < P && e == ncclSuccess; ++q) {
            const size_t n = 2 * (size_t)counts[q];
            if (!n) continue;
            if (root < 0) {
                e = r->broadcast(q == me ? d_local : nullptr, d_full + 2 * base[q], n, ncclUint64, q, c->comm, st);
            } else if (me == root) {
                if (q == me) {
                    if (hipMemcpyAsync(d_full + 2 * base[q], d_local, n * 8, hipMemcpyDeviceToDevice, st) != hipSuccess)
                        e = ncclUnhandledCudaError;
                } else {
                    e = r->recv(d_full + 2 * base[q], n, ncclUint64, q, c->comm, st);
                }
            } else if (q == me) {
                e = r->send(d_local, n, ncclUint64, root, c->comm, st);
            }
        }
        const ncclResult_t e2 = r->group_end();
        if (e == ncclSuccess) e = e2;
    }
    (void)hipSetDevice(prev);
    return e == ncclSuccess ? OXH_OK : rccl_fail(r, e, what);
}

}  // extern "C"
