// oxen_amd/host/oxen_hasher.hpp -- C++ host mirror of liboxen `util::hasher`
// (crates/liboxen/src/util/hasher.rs) over the MI355X C ABI (include/oxen_hash.h).
//
// The reference is Rust; its toolchain is not in this image, so the host side above the C ABI is
// C++: the same function names, argument meaning and error behaviour as the Rust module, with
// Result<T, OxenError> mapped to "returns T or throws OxenError" and u128 to unsigned __int128
// (MerkleHash, model/merkle_tree/merkle_hash.rs:16). Every digest is computed on the GPU; there is
// no CPU hashing path (without a gfx950 device every call throws OxenError).
#pragma once

#include <sys/stat.h>

#include <cstdint>
#include <functional>
#include <optional>
#include <stdexcept>
#include <string>
#include <string_view>
#include <vector>

#include "../../include/oxen_hash.h"

namespace liboxen {

using u128 = unsigned __int128;

// error/mod.rs: the variants this path raises, with the reference's messages.
class OxenError : public std::runtime_error {
   public:
    enum class Kind { Basic, HashMismatch, NoDevice };
    OxenError(Kind k, const std::string& msg, int code = 0) : std::runtime_error(msg), kind_(k), code_(code) {}
    static OxenError basic_str(const std::string& msg, int code = 0) { return OxenError(Kind::Basic, msg, code); }
    Kind kind() const { return kind_; }
    int code() const { return code_; }  // the C ABI status (OXH_ERR_*) behind it, 0 if none

   private:
    Kind kind_;
    int code_;
};

// model/merkle_tree/merkle_hash.rs:16-131
class MerkleHash {
   public:
    MerkleHash() = default;
    explicit MerkleHash(u128 v) : v_(v) {}
    static MerkleHash from_str(std::string_view hex);  // FromStr, radix 16 (:54-61)
    u128 to_u128() const { return v_; }
    std::string to_string() const;                      // Display "{:x}", unpadded (:73-77)
    std::string to_short_str() const;                   // first 10 hex chars (:79-83)
    void to_le_bytes(uint8_t out[16]) const;            // (:25-27)
    std::string node_db_prefix() const;                 // "{hex[..3]}/{hex[3..]}" (:125-131)
    bool operator==(const MerkleHash& o) const { return v_ == o.v_; }
    bool operator!=(const MerkleHash& o) const { return v_ != o.v_; }

   private:
    u128 v_ = 0;
};

namespace util::hasher {

// The process-wide GPU context (device $OXH_DEVICE, default 0), created on first use.
oxh_ctx* default_context();

std::string format_hex(u128 v);  // format!("{:x}", u128)

std::string hash_buffer(const void* data, size_t len);        // hasher.rs:11-14
std::string hash_str(std::string_view s);                      // hasher.rs:16-19
u128 hash_buffer_128bit(const void* data, size_t len);        // hasher.rs:28-30
inline u128 hash_buffer_128bit(std::string_view s) { return hash_buffer_128bit(s.data(), s.size()); }

u128 get_hash_given_metadata(const std::string& path, const struct stat& metadata);  // hasher.rs:56-65
u128 u128_hash_file_contents(const std::string& path);                               // hasher.rs:102-112
std::string hash_file_contents(const std::string& path);                             // hasher.rs:114-124
// hasher.rs:32-54: exponential backoff 2, 4, 8 ... s; `sleep` is injectable for tests
std::string hash_file_contents_with_retry(const std::string& path, int total_retries = 5,
                                          const std::function<void(int)>& sleep = nullptr);

// hasher.rs:67-80
u128 get_combined_hash(std::optional<u128> oxen_metadata_hash, u128 content_hash);
// hasher.rs:82-100: XXH3-128 of serde_json::to_string(&Option<GenericMetadata>); the caller passes
// the JSON text (nullopt = None, serialised as "null")
u128 get_metadata_hash(const std::optional<std::string>& metadata_json);
std::optional<u128> maybe_get_metadata_hash(const std::optional<std::string>& metadata_json);

// The batched form the add loop calls once per batch (add.rs:422-444): one entry per path, the
// digest and size, or the error hash_small_file_contents would have raised (hasher.rs:126-148).
struct FileHash {
    bool ok = false;
    u128 hash = 0;
    uint64_t size = 0;
    std::string error;
    int code = 0;      // OXH_OK, OXH_ERR_OPEN (File::open failed), OXH_ERR_IO (the read failed), OXH_ERR_NOMEM
    int os_error = 0;  // the errno of the failed open / read
};
// hasher.rs picks its one-shot (< 1e9 B) or streamed branch by the file's size (:56-65, 106)
constexpr uint64_t kLargeFileBytes = 1000000000ull;
// The text of the OxenError hasher.rs returns for a file that could not be hashed: File::open failed
// (OXH_ERR_OPEN: "util::hasher::hash_file_contents Could not open file {path:?} {err:?}", or "Could not
// open file {path:?} due to {err:?}" on the streamed branch), else "Could not read file for hashing".
std::string file_error_text(const std::string& path, int status, int os_error, uint64_t size_hint);
// Rust `{:?}` of a str / Path, and of std::io::Error::from_raw_os_error(e)
std::string rust_str_debug(const std::string& s);
std::string rust_path_debug(const std::string& path);
std::string rust_io_error_debug(int e);
std::vector<FileHash> hash_files(const std::vector<std::string>& paths, oxh_ctx* ctx = nullptr);

// The add loop's hash stage over helper processes (oxh_pool_*): the list split into contiguous
// shares (by bytes when sizes are given), one helper process per share, helper p on
// devices[p % devices.size()]. liboxen's fan-out of 64-file batches over tasks of one process
// (add.rs:422-425) becomes a fan-out over processes and GPUs. Calls serialise; a helper that dies
// makes this and every later call throw.
class ReaderPool {
   public:
    explicit ReaderPool(int procs = 2, const std::vector<int>& devices = {0}, int threads = 0, uint64_t staging_bytes = 0);
    ~ReaderPool();
    ReaderPool(const ReaderPool&) = delete;
    ReaderPool& operator=(const ReaderPool&) = delete;
    // get_hash_given_metadata over every path (meta_sizes: the walk's metadata.len(), or empty)
    std::vector<FileHash> hash_files(const std::vector<std::string>& paths, const std::vector<uint64_t>& meta_sizes = {});
    int procs() const { return procs_; }

   private:
    oxh_pool* p_ = nullptr;
    int procs_ = 0;
};
std::vector<u128> hash_buffers_128bit(const std::vector<std::string_view>& buffers, oxh_ctx* ctx = nullptr);

// xxhash-rust Xxh3 (new / update / digest128 / reset) on the GPU (oxh_xxh3_stream_*).
class Xxh3 {
   public:
    explicit Xxh3(oxh_ctx* ctx = nullptr);
    ~Xxh3();
    Xxh3(const Xxh3&) = delete;
    Xxh3& operator=(const Xxh3&) = delete;
    void update(const void* data, size_t len);
    void update(std::string_view s) { update(s.data(), s.size()); }
    u128 digest128() const;
    void reset();

   private:
    oxh_xxh3_stream* s_ = nullptr;
};

// hasher.rs:183-209. R: size_t read(uint8_t* buf, size_t n) (0 = EOF; throws on error).
template <class R>
class HashingReader {
   public:
    explicit HashingReader(R& inner, oxh_ctx* ctx = nullptr) : inner_(inner), hasher_(ctx) {}
    size_t read(uint8_t* buf, size_t n) {
        const size_t got = inner_.read(buf, n);
        if (got > 0) hasher_.update(buf, got);
        return got;
    }
    u128 digest128() const { return hasher_.digest128(); }

   private:
    R& inner_;
    Xxh3 hasher_;
};

// hasher.rs:214-244. W: size_t write(const uint8_t* buf, size_t n) (bytes accepted), void flush().
template <class W>
class HashingWriter {
   public:
    explicit HashingWriter(W& inner, oxh_ctx* ctx = nullptr) : inner_(inner), hasher_(ctx) {}
    size_t write(const uint8_t* buf, size_t n) {
        const size_t put = inner_.write(buf, n);
        if (put > 0) hasher_.update(buf, put);  // only what the inner writer accepted
        return put;
    }
    void write_all(const uint8_t* buf, size_t n) {
        while (n) {
            const size_t put = write(buf, n);
            if (put == 0) throw OxenError::basic_str("failed to write whole buffer");
            buf += put;
            n -= put;
        }
    }
    void flush() { inner_.flush(); }
    u128 digest128() const { return hasher_.digest128(); }

   private:
    W& inner_;
    Xxh3 hasher_;
};

}  // namespace util::hasher

namespace util::fs {

// One tracked working-tree file as `oxen status`'s walk holds it (core/v_latest/status.rs:690-745):
// metadata.len(), the committed FileNode's num_bytes and hash, and the caller's mtime verdict
// (LocalRepository::mtime_matches, model/repository/local_repository.rs:601-615).
// The working file's side of the metadata-hash comparison (util/fs.rs:1600-1607):
// maybe_get_metadata_hash(get_file_metadata(path, data_type)).
struct FileMetadataHash {
    enum Kind : uint8_t {
        None = OXH_META_NONE,    // no metadata for the file's data type
        Given = OXH_META_GIVEN,  // the caller extracted it: `hash`
        Text = OXH_META_TEXT,    // data type Text: MetadataText counted on the hashing read (K1T)
        Error = OXH_META_ERROR,  // the caller's extraction failed: `error`
    } kind = None;
    u128 hash = 0;
    std::string error;
};
struct TrackedFile {
    std::string path;
    uint64_t size = 0;
    uint64_t node_num_bytes = 0;
    u128 node_hash = 0;
    bool mtime_matched = false;
    std::optional<u128> node_metadata_hash;  // node.metadata_hash()
    FileMetadataHash file_metadata;
};
struct Modified {
    bool ok = true;         // false: metadata extraction failed, or the file had to be read and could not be
    bool modified = false;
    int code = OXH_OK;
    std::string error;
};
// classify_modified_from_node_with_metadata (util/fs.rs:1580-1619) x n through oxh_files_modified:
// size, mtime and a caller-given metadata hash decide first; the files that remain are read once,
// all in one GPU request (text files' MetadataText counted on that read).
std::vector<Modified> classify_modified_batch(const std::vector<TrackedFile>& files, oxh_ctx* ctx = nullptr,
                                              uint64_t* n_hashed = nullptr);
// One file; an extraction or read error throws OxenError, as the reference's `?` does.
bool classify_modified_from_node_with_metadata(const std::string& path, uint64_t node_num_bytes, u128 node_hash,
                                               const struct stat& metadata, bool mtime_matched,
                                               std::optional<u128> node_metadata_hash = std::nullopt,
                                               const FileMetadataHash& file_metadata = FileMetadataHash());

// util/fs/atomic_file.rs: AtomicFile with an expected hash -- verify-before-publish. Bytes go to an
// AtomicTempFile sibling `<target>.oxentmp.<random>` (:54-159) while a GPU Xxh3 stream (oxh_xxh3_stream)
// hashes them; on a digest other than the expected one the temp is unlinked and OxenError
// HashMismatch is thrown (:396-431), else the temp's data is fsynced, renamed over the target and
// the parent fsynced (commit, :116-159). Without with_hash nothing is hashed.
class AtomicFile {
   public:
    // reads up to n bytes into buf, returns 0 at EOF, throws on error
    using Reader = std::function<size_t(uint8_t* buf, size_t n)>;
    explicit AtomicFile(std::string target, oxh_ctx* ctx = nullptr) : target_(std::move(target)), ctx_(ctx) {}
    AtomicFile& with_hash(MerkleHash expected) {
        expected_ = expected;
        verify_ = true;
        return *this;
    }
    void stream(const Reader& reader);          // AtomicFile::stream / stream_async (:271-318, :363-463)
    void write(const void* data, size_t len);   // AtomicFile::write (:161-...)
    // AtomicFile::stream_from_paths (:320-351): the in-order concatenation of `paths`, one source
    // open at a time, verified as it streams (chunked-upload reassembly)
    void stream_from_paths(const std::vector<std::string>& paths);

   private:
    std::string target_;
    oxh_ctx* ctx_;
    MerkleHash expected_;
    bool verify_ = false;
};

}  // namespace util::fs

namespace storage {

// storage/local.rs: LocalVersionStore's content-addressed writes, verified on the GPU.
class LocalVersionStore {
   public:
    explicit LocalVersionStore(std::string root, oxh_ctx* ctx = nullptr) : root_(std::move(root)), ctx_(ctx) {}
    std::string version_dir(const std::string& hash) const;   // {root}/{hash[..2]}/{hash[2..]} (:66-70)
    std::string version_path(const std::string& hash) const;  // + /data (:72-75)
    bool version_exists(const std::string& hash) const;       // (:259-261)
    // (:123-139) skipped when the blob exists; the bytes must hash to `hash` (HashMismatch otherwise)
    void store_version(const std::string& hash, const void* data, size_t len) const;
    // (:104-121) streamed in STREAMING_BUF_SIZE (10 MiB) reads, verified as it streams
    void store_version_from_reader(const std::string& hash, const util::fs::AtomicFile::Reader& reader,
                                   uint64_t size) const;
    // Many received blobs at once (pull / clone downloads, api/client/versions.rs): every buffer hashed
    // in ONE batched GPU pass (oxh_hash_buffers), each verified blob published as store_version
    // would; result i is empty on success, else the error store_version would have thrown.
    std::vector<std::string> store_versions(const std::vector<std::string>& hashes,
                                            const std::vector<std::string_view>& datas) const;
    // Chunked uploads (:78-92, :315-330, :367-413): chunks under {version_dir}/chunks/{offset}/chunk,
    // written unverified; combine_version_chunks reassembles them in offset order, verifies the
    // whole blob on the GPU (HashMismatch: nothing published, chunks kept), then removes the chunks.
    std::string version_chunks_dir(const std::string& hash) const;
    std::string version_chunk_file(const std::string& hash, uint64_t offset) const;
    void store_version_chunk(const std::string& hash, uint64_t offset, const void* data, size_t len) const;
    std::vector<uint64_t> list_version_chunks(const std::string& hash) const;
    void combine_version_chunks(const std::string& hash) const;

   private:
    std::string root_;
    oxh_ctx* ctx_;
};

}  // namespace storage

// experiments/block-level-dedup/src/chunker/fastcdchunker.rs:72-122 over the ABI's host entry points:
// fs::read(input_file) (:75) -> v2020 chunking (:83-88) -> xxh3_128 per chunk (:95-98), the file read
// inside the library and streamed through its piece pipeline (oxh_fastcdc_files / oxh_fastcdc_host).
namespace dedup {
struct Chunk {
    uint64_t offset = 0, length = 0;  // the crate's Chunk.offset / length, relative to the file
    u128 hash = 0;                    // xxh3_128 of the chunk (its file name is hash.to_string())
};
struct ChunkedFile {
    bool ok = false;
    uint64_t size = 0;
    int code = 0, os_error = 0;  // as FileHash: OXH_ERR_OPEN / OXH_ERR_IO with the errno
    std::vector<Chunk> chunks;
};
// One entry per path; min / avg / max as v2020::FastCDC::new (FastCDChunker: 4096, chunk, 2 * chunk).
std::vector<ChunkedFile> fastcdc_files(const std::vector<std::string>& paths, uint32_t min_size, uint32_t avg_size,
                                       uint32_t max_size, oxh_ctx* ctx = nullptr);
// ... over several contexts (one per GPU): oxh_fastcdc_files_multi, the same result
std::vector<ChunkedFile> fastcdc_files(const std::vector<std::string>& paths, uint32_t min_size, uint32_t avg_size,
                                       uint32_t max_size, const std::vector<oxh_ctx*>& ctxs);
std::vector<std::vector<Chunk>> fastcdc_buffers(const std::vector<std::string_view>& buffers, uint32_t min_size,
                                                uint32_t avg_size, uint32_t max_size, oxh_ctx* ctx = nullptr);
std::vector<std::vector<Chunk>> fastcdc_buffers(const std::vector<std::string_view>& buffers, uint32_t min_size,
                                                uint32_t avg_size, uint32_t max_size, const std::vector<oxh_ctx*>& ctxs);
// Fixed-size chunks (fixedsize_multithreaded.rs:78-110: chunk i = [i*chunk_size, min(+chunk_size, size)),
// xxh3_128 of each) through oxh_chunk_digests_files / _host; offsets and lengths are implied.
std::vector<ChunkedFile> fixed_chunk_files(const std::vector<std::string>& paths, uint64_t chunk_size,
                                           oxh_ctx* ctx = nullptr);
std::vector<ChunkedFile> fixed_chunk_files(const std::vector<std::string>& paths, uint64_t chunk_size,
                                           const std::vector<oxh_ctx*>& ctxs);
std::vector<std::vector<Chunk>> fixed_chunk_buffers(const std::vector<std::string_view>& buffers, uint64_t chunk_size,
                                                    oxh_ctx* ctx = nullptr);
std::vector<std::vector<Chunk>> fixed_chunk_buffers(const std::vector<std::string_view>& buffers, uint64_t chunk_size,
                                                    const std::vector<oxh_ctx*>& ctxs);
// Whether the host chunk entries above beat the reference's own CPU loop for host-resident files on
// this node (INTEGRATION.md §2 "When NOT to call the host chunk entries"): every byte crosses a PCIe
// link first, so `links` GPUs move ~49 GiB/s each, against `host_cores` hashing at ~4.2 GiB/s per core
// (fixed-size) or ~2.4 (FastCDC v2020 + XXH3), as measured on the MI355X boxes. Bytes
// already in HBM take the device entries regardless. A routing rule for the caller, not a CPU path.
bool host_entry_pays_off(unsigned host_cores, unsigned links, bool fastcdc);
// u128::to_string() (fastcdchunker.rs:98, the chunk file name)
std::string chunk_name(u128 hash);
}  // namespace dedup

// core/v_latest/index/restore.rs:231-405: may restore / merge overwrite this working file?
namespace core::restore {
struct NodeHashes {  // PartialNode {hash, size} (:231) or FileNode {hash, combined_hash, num_bytes} (:300)
    u128 hash = 0;
    uint64_t num_bytes = 0;
    u128 combined_hash = 0;
};
struct RestoreCheck {
    std::string working_path;
    NodeHashes target;                       // the node being restored / merged in
    std::optional<NodeHashes> base;          // the merge base's node, if any
    bool mtime_matched = false;              // LocalRepository::mtime_matches (local_repository.rs:556)
    util::fs::FileMetadataHash file_metadata;  // combined only: None / Given / Text (Error: the call fails)
};
// should_restore_partial_node (combined = false) or should_restore_file (combined = true) x n: the
// existence and mtime + size short cuts, then every remaining file hashed in one pass (oxh_hash_files_ex;
// its text counts give MetadataText) and compared with the target / base hashes. A path whose stat
// fails reads as absent (Path::exists()): restore. The first file in order whose read or metadata
// fails throws OxenError, as the reference's `?` does.
std::vector<bool> should_restore_batch(const std::vector<RestoreCheck>& files, bool combined, oxh_ctx* ctx = nullptr);
}  // namespace core::restore

// core/v_latest/branches.rs:653-757: the File arm of checkout's target-tree walk, three-way.
namespace core::branches {
enum class CheckoutOutcome {
    Skip,         // the working file already is the target's version
    Restore,      // results.files_to_restore
    Conflict,     // results.cannot_overwrite_entries (OnConflict::Abort)
    KeepDeleted,  // an uncommitted deletion of content both trees hold: preserved
};
struct CheckoutCheck {
    std::string working_path;
    core::restore::NodeHashes target;                // the target FileNode: content hash, num_bytes
    std::optional<core::restore::NodeHashes> from;   // the from tree's PartialNode (hash, size), if any
    bool target_mtime_matched = false;  // repo.mtime_matches(disk mtime, the target's mtime)
    bool from_mtime_matched = false;    // repo.mtime_matches(disk mtime, the PartialNode's last_modified)
};
// Every file of the walk, in its order: missing (from holds the target's hash -> KeepDeleted; a from
// node -> Conflict, or Restore with overwrite; none -> Restore), the target / from mtime + size short
// cuts, then every remaining file hashed in one pass (get_hash_given_metadata with the stat's size,
// oxh_hash_files_ex) and compared with the target's and the from node's hash. The first file in order
// whose stat or read fails throws OxenError, as the reference's `?` does.
std::vector<CheckoutOutcome> classify_checkout_batch(const std::vector<CheckoutCheck>& files, bool overwrite,
                                                     oxh_ctx* ctx = nullptr);
}  // namespace core::branches

// one process per GPU, the digest table gathered once over xGMI (oxh_comm_*).
namespace multigpu {
class DigestGather {
   public:
    static std::vector<uint8_t> unique_id();  // OXH_COMM_ID_BYTES; one rank makes it, every rank gets it
    DigestGather(const std::vector<uint8_t>& id, int rank, int nranks, int device);  // blocks until all join
    ~DigestGather();
    DigestGather(const DigestGather&) = delete;
    DigestGather& operator=(const DigestGather&) = delete;
    // d_local: this rank's 2 * counts[rank] u64 on the device; d_full: 2 * sum(counts) u64 on the device
    // (every rank when root < 0, else rank `root` only); enqueued on `stream` (hipStream_t)
    void gather(const uint64_t* d_local, const std::vector<uint64_t>& counts, uint64_t* d_full, int root,
                void* stream) const;

   private:
    oxh_comm* c_ = nullptr;
};
}  // namespace multigpu
}  // namespace liboxen
