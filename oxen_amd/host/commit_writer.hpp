// oxen_amd/host/commit_writer.hpp -- C++ host mirror of the parent-node hashing in liboxen's commit
// writer (crates/liboxen/src/repositories/commits/commit_writer.rs) over the MI355X C ABI: the K2
// driver. The reference is Rust; this is the host code a liboxen build without the Rust toolchain
// would run above `oxh_hash_streams`.
//
// What it restates (the byte streams commit_writer.rs feeds to `Xxh3::update`, and the bookkeeping
// that decides them):
//   split_into_vnodes  :544-755  child set (:561-638: HEAD's children, then the staged changes;
//                                removals drop the child; defensive prefixing of leaf-only paths
//                                :591-612), num_vnodes in f32 (:657-660), bucket = xxh3_128(path) %
//                                num_vnodes (:669-681, also commit_merkle_tree.rs:813-814), entries
//                                sorted by path (:684-694), vnode id = xxh3("vnode" || dir || child
//                                hashes LE [|| uuid]) (:696-720)
//   compute_dir_node   :995-1165 dir hash = xxh3("dir" || path || for every staged dir that
//                                starts_with(path), in map order: for each vnode: id LE || for each
//                                entry: name || hash LE) (get_children :979-993, :1001-1071)
// Nothing inside one commit chains (a vnode hashes its entries' staged hashes; a dir hashes its
// descendants' vnode ids and the staged dir hashes), so a whole commit is three batched GPU passes:
// every bucket hash, every vnode id, every dir hash. HashMap iteration order and the UUID salt are
// inputs (the caller's order; SaltFn), as in oxen_amd/merkle.py and oracle/commit_oracle.py.
#pragma once

#include <cstdint>
#include <functional>
#include <optional>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "oxen_hasher.hpp"

namespace liboxen::commit_writer {

// model/merkle_tree/node/staged_merkle_tree_node.rs: the status of a staged node
enum class StagedStatus { Added, Modified, Removed, Unmodified };

// A StagedMerkleTreeNode as the commit writer sees it: `path` is maybe_path() (repo-relative),
// `hash` what both parent streams take from it (file_node.combined_hash() for files, node.hash for
// dirs), `name` the node name the dir stream uses (nullopt: the path).
struct StagedNode {
    std::string path;
    u128 hash = 0;
    bool is_dir = false;
    StagedStatus status = StagedStatus::Added;
    std::optional<std::string> name;
    const std::string& node_name() const { return name ? *name : path; }
};

// commit_writer.rs EntryVNode: an id and its entries sorted by path
struct EntryVNode {
    MerkleHash id;
    std::vector<StagedNode> entries;
};

struct DirVNodes {
    std::string dir;
    std::vector<EntryVNode> vnodes;
    std::vector<StagedNode> removed;
};

// The staged changes per directory, in the caller's (HashMap) order; HEAD's children per directory.
using StagedDirs = std::vector<std::pair<std::string, std::vector<StagedNode>>>;
using ExistingDirs = std::unordered_map<std::string, std::vector<StagedNode>>;
// The 16 salt bytes of vnode `vnode_index` of `dir` (Uuid::new_v4().as_bytes(), :713-716)
using SaltFn = std::function<void(const std::string& dir, size_t vnode_index, uint8_t out[16])>;

void uuid_v4_salt(const std::string& dir, size_t vnode_index, uint8_t out[16]);

// std::path::Path::components of a relative unix path ("" and "." dropped), joined by '/': the key
// Path's Ord / starts_with compare by.
std::vector<std::string> path_components(const std::string& p);
std::string normalize(const std::string& p);  // path_components joined by '/'

// commit_writer.rs:660: (total_children as f32 / vnode_size as f32).ceil() as u128
uint64_t num_vnodes(uint64_t total_children, uint64_t vnode_size);

std::vector<DirVNodes> split_into_vnodes(const StagedDirs& entries, const ExistingDirs& existing,
                                         uint64_t vnode_size = 10000, const SaltFn& salt = uuid_v4_salt,
                                         oxh_ctx* ctx = nullptr);

// compute_dir_node's hash for `dirs` (nullptr: "" and every key of `vnodes` with a non-empty path),
// all in one GPU batch. A dir's stream covers every key of `vnodes` that starts_with it,
// component-wise, in `vnodes` order.
std::vector<std::pair<std::string, MerkleHash>> compute_dir_hashes(const std::vector<DirVNodes>& vnodes,
                                                                   const std::vector<std::string>* dirs = nullptr,
                                                                   oxh_ctx* ctx = nullptr);

struct CommitTree {
    std::vector<DirVNodes> vnodes;
    std::vector<std::pair<std::string, MerkleHash>> dir_hashes;  // "" first
};

// Every parent digest of one commit: three batched GPU passes.
CommitTree commit_tree(const StagedDirs& entries, const ExistingDirs& existing, uint64_t vnode_size = 10000,
                       const SaltFn& salt = uuid_v4_salt, oxh_ctx* ctx = nullptr);

// XXH3-128 of caller-serialised streams (arena[offsets[i] .. + lens[i]]) in one oxh_hash_streams call
std::vector<u128> hash_streams(const std::string& arena, const std::vector<uint64_t>& offsets,
                               const std::vector<uint64_t>& lens, oxh_ctx* ctx = nullptr);

}  // namespace liboxen::commit_writer
