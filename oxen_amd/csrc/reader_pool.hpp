// oxen_amd/csrc/reader_pool.hpp -- wire format between oxh_pool (reader_pool.cpp, inside
// liboxen_hash.so) and its helper processes (hash_helper.cpp -> oxen_amd/oxh_hash_helper).
//
// One shared-memory region (a memfd the pool creates; every helper maps it MAP_SHARED) holds a call's
// inputs and outputs; requests and replies are fixed-size records on one SOCK_SEQPACKET socket per
// helper. A helper reads paths and sizes of its share [lo, hi) from the region, runs its own context's
// engine over them, and writes digests, sizes and statuses of that share in place.
#pragma once
#include <stdint.h>

namespace oxh_pool_wire {

constexpr int kSockFd = 200;  // the helper's end of its socket, dup2'ed here by posix_spawn
constexpr int kMemFd = 201;   // the shared region

// region layout of one call with n paths (byte offsets, each 64-B aligned, in PoolReq)
//   offs   u64[n]   offset of path i's NUL-terminated bytes inside `blob`
//   meta   u64[n]   the caller's sizes (oxh_hash_files_meta), when has_meta
//   out    u64[2n]  digests (lo, hi)
//   sizes  u64[n]
//   status i32[n]
//   oserr  i32[n]   errno of each failed open / read (oxh_hash_files_ex)
//   blob   the paths, back to back
struct PoolReq {
    uint64_t seq;   // call number; the reply echoes it
    uint64_t cap;   // region size: the helper re-maps when it changed
    uint64_t n, lo, hi;
    uint64_t off_offs, off_meta, off_out, off_sizes, off_status, off_oserr, off_blob;
    int32_t has_meta;
    int32_t quit;   // 1: exit
};

struct PoolRep {
    uint64_t seq;   // 0 = the start-up report
    int32_t rc;     // OXH_* of the call (per-file errors are in status[])
    int32_t pid;
    char msg[240];
};

}  // namespace oxh_pool_wire
