/*
 * include/oxen_hash.h -- C ABI of the MI355X content-hashing stage for `oxen add` / commit.
 *
 * Drop-in boundary for liboxen's `util::hasher` module (crates/liboxen/src/util/hasher.rs) and the
 * per-file hash call in the add loop (crates/liboxen/src/core/v_latest/add.rs:716-718,741-743).
 * Every digest is XXH3-128 with seed 0 and the default secret -- bit-identical to
 * `xxhash_rust::xxh3::xxh3_128` (xxhash-rust 0.8.15) -- returned as two u64 words per item:
 * out[2*i] = low 64 bits, out[2*i+1] = high 64 bits, i.e. the Rust `u128` is
 * `((hi as u128) << 64) | lo as u128` (MerkleHash, model/merkle_tree/merkle_hash.rs:16).
 *
 * Conventions:
 *   - plain pointers and sizes only; no torch / Rust / HIP-runtime types in the signatures
 *     (`stream` is an opaque hipStream_t; NULL = the null stream, as in HIP itself);
 *   - every function returns an int status (OXH_OK == 0); batch calls also fill a per-item
 *     `status[]` so one unreadable file never fails the batch (add.rs:533-544 logs and skips);
 *   - the library never frees caller memory and retains no caller pointer after returning;
 *   - all entry points are thread-safe; file calls on one context are requests to the context's
 *     streaming engine, and concurrent ones share its live pipeline (each caller returns when its
 *     own files are done); other calls on a context serialise;
 *   - there is no CPU fallback: without a usable gfx950 device, calls fail with OXH_ERR_NODEVICE.
 *
 * The Rust-side `extern "C"` block that binds these is in INTEGRATION.md.
 */
#ifndef OXEN_HASH_H
#define OXEN_HASH_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OXH_ABI_VERSION 5

/* status codes (also used per item in status[]) */
#define OXH_OK 0
#define OXH_ERR_INVALID 1   /* bad argument */
#define OXH_ERR_HIP 2       /* HIP runtime error */
#define OXH_ERR_IO 3        /* file opened but its read failed (hasher.rs:135-139, 162-165) */
#define OXH_ERR_NOMEM 4     /* host or device allocation failed */
#define OXH_ERR_NODEVICE 5  /* no usable MI355X (gfx950) device */
#define OXH_ERR_OPEN 7      /* per item: File::open failed (hasher.rs:141-145, 151-154) */

/* kernel selection for the device-resident batch */
#define OXH_MODE_AUTO 0     /* one wave per buffer (K1), lane-per-item for short-only batches */
#define OXH_MODE_WAVE 1     /* force K1: one 64-lane wave per buffer */
#define OXH_MODE_LANE 2     /* force K1s: one lane per buffer (short items, parent-node streams) */
#define OXH_MODE_WAVE_SHORT 3 /* K1 shaped for items of <= ~16 KiB (more resident waves) */
#define OXH_MODE_WAVE_PACKED 4 /* K1 shaped for items packed back to back at arbitrary byte offsets
                                  (FastCDC chunks of one buffer): each wave-instruction reads a
                                  whole 1 KiB block */

typedef struct oxh_ctx oxh_ctx;

/* ---------------------------------------------------------------- library / context */
int oxh_abi_version(void);
/* Thread-local text of the last error on this thread ("" if none). */
const char* oxh_last_error(void);
/* Number of visible HIP devices (0 on a host without a GPU). */
int oxh_device_count(int* count);
/* Create a hashing context on `device`: owns a compute stream, a copy stream, pinned host staging
 * (`staging_bytes` per slot, 0 = default 256 MiB, 3 slots) and matching device slots.
 * staging_bytes above OXH_MAX_STAGING_BYTES fails with OXH_ERR_INVALID (a slot's fill state is one
 * 64-bit word: 31 bits of byte offset, 19 bits of item count at one item per 4 KiB). Files of a
 * slot's size or larger are streamed through the large-file path whatever the setting. */
#define OXH_MAX_STAGING_BYTES 2147483392ull /* 2 GiB - 256 */
int oxh_ctx_create(int device, uint64_t staging_bytes, oxh_ctx** out);
int oxh_ctx_destroy(oxh_ctx* ctx);
/* The context's compute stream (hipStream_t), for callers that want to order against it. */
void* oxh_ctx_stream(oxh_ctx* ctx);

/* ---------------------------------------------------------------- K1 / K1s: device-resident batch
 * Replaces N calls of `hash_buffer_128bit(&[u8]) -> u128` (hasher.rs:28-30) over buffers that are
 * already resident in HBM: item i is d_arena[d_offsets[i] .. d_offsets[i] + d_lens[i]).
 * d_offsets / d_lens / d_out are device pointers; d_out receives 2*n u64. Asynchronous on `stream`.
 * Any start offset and length; starts off a dword boundary are loaded dword-aligned and re-aligned
 * in registers. `mode` (OXH_MODE_*) only picks the kernel shape, never the result: AUTO / WAVE for
 * items placed at 128-B (or coarser) aligned offsets, WAVE_SHORT when they are mostly <= 16 KiB,
 * WAVE_PACKED for items packed back to back at arbitrary offsets (chunks of one buffer). */
int oxh_xxh3_128_batch_device(const void* d_arena, const uint64_t* d_offsets, const uint64_t* d_lens,
                              uint64_t n, uint64_t* d_out, int mode, void* stream);

/* Fixed-size chunk digests of one device-resident buffer (block-level dedup,
 * experiments/block-level-dedup/src/chunker/fixedsize.rs:52-102): chunk i is
 * d_buf[i*chunk .. min((i+1)*chunk, len)); d_out receives 2*ceil(len/chunk) u64. */
int oxh_chunk_digests_device(const void* d_buf, uint64_t len, uint64_t chunk, uint64_t* d_out,
                             void* stream);

/* K1L: whole-buffer digest of one large device-resident buffer (files >= 1e9 B take the streamed
 * branch in hasher.rs:150-174; the digest is the same XXH3-128). Block sums are computed in
 * parallel across the chip, then the serial scramble chain runs on one wave. `d_out` gets 2 u64. */
int oxh_xxh3_128_large_device(oxh_ctx* ctx, const void* d_buf, uint64_t len, uint64_t* d_out,
                              void* stream);

/* K1L over n large device-resident buffers (e.g. the 16 x 8 GiB files of the dedup experiment):
 * d_bufs and lens are HOST arrays of n device pointers / lengths; d_out (device) gets 2n u64.
 * Buffers are processed in rounds of 1 GiB pieces: a round's block sums run chip-wide on `stream`
 * while the previous round's serial chains (up to 32 per launch, resumed from piece to piece) run
 * on a second stream. The block sums live in one of the device's two cached scratch buffers, so
 * both K1L calls return only after `stream` has finished them (a third concurrent caller on the
 * device waits for a buffer). */
int oxh_xxh3_128_large_batch_device(const void* const* d_bufs, const uint64_t* lens, uint64_t n,
                                    uint64_t* d_out, void* stream);

/* ---------------------------------------------------------------- streaming XXH3
 * xxhash-rust's `Xxh3` (new / update / digest128) as used by hasher.rs:73-76, 157-173 (large files),
 * HashingReader / HashingWriter (hasher.rs:183-244) and AtomicFile's verify (atomic_file.rs:396-431).
 * Bytes collect in a pinned buffer; every 16 MiB (OXH_STREAM_PIECE_MIB) of whole 1 KiB blocks go to
 * the device as one K1L piece whose chain resumes from the stream's accumulators, so memory stays
 * bounded whatever the length. digest (2 u64, lo then hi) = xxh3_128 of everything updated so far
 * and leaves the state unchanged. A stream is used by one thread at a time (like `&mut Xxh3`). */
typedef struct oxh_xxh3_stream oxh_xxh3_stream;
int oxh_xxh3_stream_create(oxh_ctx* ctx, oxh_xxh3_stream** out);
int oxh_xxh3_stream_update(oxh_xxh3_stream* s, const void* data, uint64_t len);
int oxh_xxh3_stream_digest(oxh_xxh3_stream* s, uint64_t* out2);
int oxh_xxh3_stream_reset(oxh_xxh3_stream* s);
int oxh_xxh3_stream_destroy(oxh_xxh3_stream* s);

/* ---------------------------------------------------------------- host-resident entry points
 * These block until the digests are in host memory. */

/* hash_buffer_128bit x n over host buffers (pinned staging, H2D on a side stream, K1, D2H). */
int oxh_hash_buffers(oxh_ctx* ctx, const uint8_t* const* bufs, const uint64_t* lens, uint64_t n,
                     uint64_t* out);

/* get_hash_given_metadata / u128_hash_file_contents x n (hasher.rs:56-65,102-112): reads each file
 * whole (parallel readers straight into pinned staging), overlaps H2D with hashing, and returns
 * digests, file sizes and a per-file status (OXH_OK; OXH_ERR_OPEN for a file whose open() fails --
 * File::open in hash_small_file_contents, hasher.rs:141-145; OXH_ERR_IO for a file that opens but
 * cannot be read -- read_to_end, hasher.rs:135-139, e.g. a directory (EISDIR); OXH_ERR_NOMEM for a
 * file larger than a staging slot whose device / pinned buffers cannot be allocated -- the other
 * files of the call are unaffected; digest 0 on error). Files are read to EOF: one whose size
 * differs from its stat (or, below, from the caller's size) is re-read, so the digest covers what
 * the read returned, like read_to_end (hasher.rs:126-148).
 * A call of at most 8 files and 2 MiB on a context with no file request in flight runs on the caller's
 * thread (the same reads and kernels, no engine hand-offs; the thread's current HIP device is restored
 * before return); other calls are requests to the context's engine thread. Either way the results are
 * the same. `sizes` and `status` may be NULL. oxh_hash_files_ex also returns the errno of each failure. */
int oxh_hash_files(oxh_ctx* ctx, const char* const* paths, uint64_t n, uint64_t* out,
                   uint64_t* sizes, int32_t* status);

/* get_hash_given_metadata(path, &metadata) x n (hasher.rs:56-65) with the sizes the caller already
 * holds from its directory walk (add.rs stats every entry): readers skip the fstat and read
 * meta_sizes[i] + 1 bytes; a file whose size differs from meta_sizes[i] is re-read (fstat + whole
 * read), so digests always cover the file's current content. `sizes` returns the sizes read. */
int oxh_hash_files_meta(oxh_ctx* ctx, const char* const* paths, const uint64_t* meta_sizes, uint64_t n,
                        uint64_t* out, uint64_t* sizes, int32_t* status);

/* The add loop's hash and version-store copy, fused (add.rs:507-516, 718, 743;
 * storage/local.rs:104-121; util/fs/atomic_file.rs:363-463): each file is read ONCE into pinned
 * staging and hashed by K1; when its blob is not already in the store it is written from the same
 * pinned bytes to {versions_root}/{hex[..2]}/{hex[2..]}/data (hex = unpadded {:x}) through
 * AtomicTempFile's protocol (util/fs/atomic_file.rs:54-159): a `data.oxentmp.<random>` sibling,
 * data made durable, rename, rename made durable -- with one syncfs() per drained staging slot in
 * place of an fsync per file and per parent. Files larger than a staging slot are streamed: each
 * piece goes to the device and to a temp file in {versions_root} as it is read, and the temp is
 * renamed into place once the digest is known (host memory stays bounded by the bounce buffers).
 * The reference reads a new file three times and hashes it twice (verify-before-publish); here the
 * published bytes are the hashed bytes, so the check holds by construction.
 * Identical content in several items is published once. stored[i] = 1 for the item that wrote the
 * blob, 0 otherwise. status[i] = OXH_ERR_IO (digest 0) for an unreadable file AND for every item
 * whose content could not be published, OXH_ERR_NOMEM as for oxh_hash_files. */
int oxh_add_files(oxh_ctx* ctx, const char* const* paths, uint64_t n, const char* versions_root,
                  uint64_t* out, uint64_t* sizes, int32_t* status, int32_t* stored);
/* oxh_add_files plus os_error[i] as in oxh_hash_files_ex (0 for a failed publish). */
int oxh_add_files_ex(oxh_ctx* ctx, const char* const* paths, uint64_t n, const char* versions_root,
                     uint64_t* out, uint64_t* sizes, int32_t* status, int32_t* stored, int32_t* os_error);

/* Bulk re-hash of a version store: LocalVersionStore::clean_corrupted_versions
 * (storage/local.rs:417-610, `oxen fsck`). Walks {versions_root}/{prefix}/{suffix}/data, hashes every
 * blob on the GPU (files batched exactly as oxh_hash_files) and compares the unpadded hex digest with
 * prefix+suffix. Corrupted or unreadable blobs have their {suffix} directory removed unless dry_run.
 * result[4] = {scanned, corrupted, cleaned, errors} -- the fields of CleanCorruptedVersionsResult
 * (view/versions.rs), counted with the reference's rules: a non-directory under the root is an
 * error; a non-directory under a prefix is skipped; an unreadable blob is an error (not scanned) and
 * is removed unless dry_run; a failed removal is an error. */
int oxh_clean_corrupted_versions(oxh_ctx* ctx, const char* versions_root, int dry_run, uint64_t* result);

/* ---------------------------------------------------------------- reader-process pool
 * oxh_hash_files / oxh_hash_files_meta over a list split across `procs` helper PROCESSES. The warm
 * page-cache floor of reading many small files is open()+close() themselves, and it is per process
 * (200 000 opens: 0.28 s in one process at any thread count, 0.16 s in two, 0.13 s in four;
 * DESIGN.md §5), so one context's engine -- one process -- sits on it. The pool starts helper
 * processes (posix_spawn of `oxh_hash_helper` from this library's directory, $OXH_HELPER overrides),
 * each with its own context on devices[p % ndevices] and `threads` reader threads (<= 0: the
 * process's CPU quota / procs, at most 16); ndevices = 0 means device 0. With devices {0..7} every
 * GPU of a node is fed its own contiguous share over its own PCIe link. Shares are
 * balanced by bytes when meta_sizes is given. Paths and outputs cross the process boundary through
 * one shared-memory region; calls on one pool serialise. Helpers exit on oxh_pool_destroy, or when
 * the creating process exits (whichever thread created the pool: a helper watches its socket and its
 * parent process, not the creating thread). A helper that dies makes the call, and every later call,
 * fail with OXH_ERR_HIP. A helper that is alive but has not answered within OXH_WAIT_LIMIT_S seconds
 * (default 60) is only reported on stderr (the call keeps waiting: a large batch may take that long);
 * OXH_POOL_CALL_LIMIT_S > 0 is the opt-in deadline after which the call, and every later call, fail
 * with OXH_ERR_HIP (default 0 = no deadline). Creation fails with the first helper's error (e.g. OXH_ERR_NODEVICE without a GPU).
 * Replaces the reference's fan-out of 64-file batches over num_cpus*2 tasks of one process
 * (core/v_latest/add.rs:422-425) with a fan-out over processes and devices. */
typedef struct oxh_pool oxh_pool;
int oxh_pool_create(const int* devices, int ndevices, int procs, int threads, uint64_t staging_bytes, oxh_pool** out);
/* oxh_hash_files (meta_sizes == NULL) or oxh_hash_files_meta semantics, per-file status[] included. */
int oxh_pool_hash_files(oxh_pool* pool, const char* const* paths, const uint64_t* meta_sizes, uint64_t n,
                        uint64_t* out, uint64_t* sizes, int32_t* status);
/* oxh_pool_hash_files plus os_error[i] as in oxh_hash_files_ex. */
int oxh_pool_hash_files_ex(oxh_pool* pool, const char* const* paths, const uint64_t* meta_sizes, uint64_t n,
                           uint64_t* out, uint64_t* sizes, int32_t* status, int32_t* os_error);
/* procs = number of helpers; pids (may be NULL) receives their process ids. */
int oxh_pool_size(oxh_pool* pool, int* procs, int* pids);
/* Not while another thread is inside a call on the same pool (the caller owns the pool's lifetime,
 * as with oxh_ctx_destroy). */
int oxh_pool_destroy(oxh_pool* pool);

/* Text-metadata fusion (K1T): the same digests as oxh_hash_files plus, per file, the counts liboxen's
 * text metadata reads in a second full pass (repositories/metadata/text.rs:11-20 ->
 * util/fs.rs:217-263): counts[2i] = num_lines (1 + number of b'\n'), counts[2i+1] = num_chars
 * (bytes that are not UTF-8 continuation bytes, bytecount::num_chars). Computed in the hash's
 * HBM pass; the caller uses them only for files it classifies as text. */
int oxh_hash_files_text(oxh_ctx* ctx, const char* const* paths, uint64_t n, uint64_t* out,
                        uint64_t* sizes, int32_t* status, uint64_t* counts);
/* K1T + the data-type sniff: as oxh_hash_files_text, plus is_utf8[i] = util::fs::is_utf8 of file i
 * (util/fs.rs:652-668: its first min(size, 4096) bytes are UTF-8, or the first error is a sequence cut
 * off by the end of that prefix; 0 for unreadable files), computed on the same staged bytes -- the
 * mime/data-type decision of add.rs:809-810 then needs no third read of the file. */
int oxh_hash_files_text_utf8(oxh_ctx* ctx, const char* const* paths, uint64_t n, uint64_t* out,
                             uint64_t* sizes, int32_t* status, uint64_t* counts, int32_t* is_utf8);
/* The four calls above in one, with the OS error of every failed item: meta_sizes NULL ->
 * oxh_hash_files, else oxh_hash_files_meta semantics; counts non-NULL -> the K1T counts; is_utf8
 * non-NULL (needs counts) -> the sniff. os_error[i] (may be NULL) = the errno of item i's failed open
 * (status OXH_ERR_OPEN) or read (OXH_ERR_IO; 0 when the file ended before the size it was read at),
 * 0 otherwise -- what the io::Error in the reference's message carries: a Rust caller builds
 * `std::io::Error::from_raw_os_error(os_error[i])` and formats hasher.rs's own text with it. */
int oxh_hash_files_ex(oxh_ctx* ctx, const char* const* paths, const uint64_t* meta_sizes, uint64_t n,
                      uint64_t* out, uint64_t* sizes, int32_t* status, int32_t* os_error,
                      uint64_t* counts, int32_t* is_utf8);

/* The modified check of `oxen status` (core/v_latest/status.rs:710,734), add (add.rs:723) and
 * checkout (branches.rs:524,548): util::fs::classify_modified_from_node_with_metadata
 * (util/fs.rs:1580-1619) x n, behind LocalRepository::is_modified_from_node_with_metadata
 * (model/repository/local_repository.rs:601-615). Per item, from the caller's walk: sizes[i] =
 * metadata.len(), node_bytes[i] = node.num_bytes(), mtime_matched[i] = mtime_matches(...) (the
 * caller's tolerance rule), node_hashes[2i..2i+1] = node.hash() (lo, hi);
 * node_meta_present[i] / node_meta_hashes[2i..2i+1] = node.metadata_hash() (Some / its value; both
 * NULL: None for every item); file_meta_kind[i] (OXH_META_*; NULL: OXH_META_NONE for every item) says
 * how the working file's maybe_get_metadata_hash(get_file_metadata(path, data_type)) (fs.rs:1601-1607)
 * is obtained, with file_meta_hashes[2i..2i+1] its value for OXH_META_GIVEN. In the reference's order:
 *   sizes[i] != node_bytes[i]  -> modified[i] = 1, file not read                      (fs.rs:1590-1592)
 *   else mtime_matched[i]      -> modified[i] = 0, file not read                      (fs.rs:1595-1597)
 *   else OXH_META_ERROR        -> status[i] = OXH_ERR_META (the reference's `?`), file not read
 *   else node and file metadata hashes both Some and different -> modified[i] = 1     (fs.rs:1609-1614)
 *        (OXH_META_GIVEN: decided before any read; OXH_META_TEXT: MetadataText {num_lines, num_chars}
 *        is counted on the hashing read itself (K1T, repositories/metadata/text.rs:11-20) and its
 *        serde_json `{"text":{"num_lines":L,"num_chars":C}}` hashed on the device)
 *   else modified[i] = (get_hash_given_metadata(path) != node.hash())                (fs.rs:1616-1618)
 * Every file that has to be read is read once, all of them in one engine request (oxh_hash_files_meta
 * semantics, read to EOF). status[i] = OXH_OK, OXH_ERR_META as above, or the read error of a file
 * that had to be read (modified[i] = 0 then; the reference returns that error). status and n_hashed
 * (the count of files read) may be NULL. */
#define OXH_ERR_META 6      /* the caller's metadata extraction failed (per item, oxh_files_modified) */
#define OXH_META_NONE 0     /* the file's metadata hash is None (no metadata for its data type) */
#define OXH_META_GIVEN 1    /* the caller computed it: file_meta_hashes[2i..2i+1] */
#define OXH_META_TEXT 2     /* data type Text: counted on the hashing read and hashed on the device */
#define OXH_META_ERROR 3    /* the caller's extraction returned an error */
int oxh_files_modified(oxh_ctx* ctx, const char* const* paths, const uint64_t* sizes, const uint64_t* node_bytes,
                       const uint8_t* mtime_matched, const uint64_t* node_hashes, const uint8_t* node_meta_present,
                       const uint64_t* node_meta_hashes, const uint8_t* file_meta_kind, const uint64_t* file_meta_hashes,
                       uint64_t n, uint8_t* modified, int32_t* status, uint64_t* n_hashed);
/* oxh_files_modified plus os_error[i] (may be NULL) as in oxh_hash_files_ex for items whose read failed. */
int oxh_files_modified_ex(oxh_ctx* ctx, const char* const* paths, const uint64_t* sizes, const uint64_t* node_bytes,
                          const uint8_t* mtime_matched, const uint64_t* node_hashes, const uint8_t* node_meta_present,
                          const uint64_t* node_meta_hashes, const uint8_t* file_meta_kind, const uint64_t* file_meta_hashes,
                          uint64_t n, uint8_t* modified, int32_t* status, int32_t* os_error, uint64_t* n_hashed);
/* Device-resident is_utf8 sniff: d_flags[i] (int32) for item i of the arena (first 4 KiB). */
int oxh_utf8_prefix_device(const void* d_arena, const uint64_t* d_offsets, const uint64_t* d_lens, uint64_t n,
                           int32_t* d_flags, void* stream);
/* Device-resident K1T: as oxh_xxh3_128_batch_device plus d_counts (2n u64: num_lines, num_chars). */
int oxh_xxh3_128_text_batch_device(const void* d_arena, const uint64_t* d_offsets, const uint64_t* d_lens,
                                   uint64_t n, uint64_t* d_out, uint64_t* d_counts, void* stream);

/* ---------------------------------------------------------------- content-defined chunking
 * FastCDC v2020 as the block-level dedup experiment runs it (experiments/block-level-dedup/src/
 * chunker/fastcdchunker.rs:83-98: `v2020::FastCDC::new(&content, 4096, chunk, 2 * chunk)`, crate
 * fastcdc 3.2.1, Normalization::Level1, then `xxh3_128` of every chunk).
 *
 * Chunks n device-resident buffers (file i = d_arena[offsets[i] .. offsets[i] + lens[i]); `offsets`
 * and `lens` are HOST arrays). On return first_chunk[0..n] (host, n+1 entries) holds each file's
 * first chunk index; chunk k is d_arena[d_chunk_offsets[k] .. + d_chunk_lens[k]) (device arrays of
 * `capacity` entries; oxh_fastcdc_max_chunks gives a bound). If d_digests is not NULL it receives
 * XXH3-128 (lo, hi) of every chunk (2*capacity u64). Parameter ranges are the crate's asserts
 * (min 64..1 MiB, avg 256..4 MiB, max 1 KiB..16 MiB, level 0..3); out-of-range -> OXH_ERR_INVALID.
 * Blocks until the chunk table is complete. */
int oxh_fastcdc_device(const void* d_arena, const uint64_t* offsets, const uint64_t* lens, uint64_t n,
                       uint32_t min_size, uint32_t avg_size, uint32_t max_size, uint32_t level,
                       uint64_t* d_chunk_offsets, uint64_t* d_chunk_lens, uint64_t* d_digests, uint64_t capacity,
                       uint64_t* first_chunk, void* stream);
/* FastCDC from host memory to host memory: the block-level dedup chunker as the reference runs it --
 * fs::read(input_file), v2020 chunking, xxh3_128 per chunk (fastcdchunker.rs:75-98) -- over n files
 * (oxh_fastcdc_files: paths; each opened and read whole, its size from fstat) or n host buffers
 * (oxh_fastcdc_host). The bytes stream through a bounded pipeline: parallel reads into a pinned
 * bounce ring, H2D on a side stream into one of two device pieces of OXH_CDC_PIECE_MIB (default 1 GiB),
 * chunked by oxh_fastcdc_device while the next piece is read. A file larger than what is left of a
 * piece is chunked in segments; a chunk is kept only once `max_size` bytes after its start are known
 * and the next segment is chunked from the first one that was not (a cut depends only on its start
 * and the max bytes after it), so every boundary is the one the crate finds in the whole file.
 * Output, in host memory: chunk k = bytes [chunk_offsets[k], + chunk_lens[k]) of its file (the
 * crate's Chunk.offset / length), digests[2k..2k+1] its XXH3-128 (lo, hi; NULL = boundaries only);
 * file i's chunks are first_chunk[i] .. first_chunk[i+1]-1 (n+1 entries). A file that cannot be
 * opened (status OXH_ERR_OPEN) or read (OXH_ERR_IO, e.g. EISDIR, or the file ended early: os_error 0)
 * has no chunks; the others are unaffected. sizes / status / os_error may be NULL. More chunks than
 * `capacity` fail the call with OXH_ERR_INVALID (the text holds the count needed); the
 * oxh_fastcdc_max_chunks bound of the sizes always suffices. Parameter ranges as oxh_fastcdc_device. */
int oxh_fastcdc_files(oxh_ctx* ctx, const char* const* paths, uint64_t n, uint32_t min_size, uint32_t avg_size,
                      uint32_t max_size, uint32_t level, uint64_t* chunk_offsets, uint64_t* chunk_lens, uint64_t* digests,
                      uint64_t capacity, uint64_t* first_chunk, uint64_t* sizes, int32_t* status, int32_t* os_error);
int oxh_fastcdc_host(oxh_ctx* ctx, const uint8_t* const* bufs, const uint64_t* lens, uint64_t n, uint32_t min_size,
                     uint32_t avg_size, uint32_t max_size, uint32_t level, uint64_t* chunk_offsets, uint64_t* chunk_lens,
                     uint64_t* digests, uint64_t capacity, uint64_t* first_chunk);
/* Upper bound on the chunk count of files of these lengths (every chunk but a file's last is >= min). */
uint64_t oxh_fastcdc_max_chunks(const uint64_t* lens, uint64_t n, uint32_t min_size);
/* Fixed-size chunk digests from host memory to host memory: the block-level dedup's fixed-size
 * chunkers (fixedsize_multithreaded.rs:78-110 -- chunk i = [i*chunk_size, min((i+1)*chunk_size, size)),
 * xxh3_128 of each -- and fixedsize.rs:67-91, which reads the same chunks through a BufReader) over n
 * files (oxh_chunk_digests_files) or n host buffers (oxh_chunk_digests_host), through the same pipeline
 * as oxh_fastcdc_files (segments of whole chunks, so nothing is carried between them). File i's
 * chunks are first_chunk[i] .. first_chunk[i+1]-1 (n+1 entries), digests[2k..2k+1] = XXH3-128 (lo, hi)
 * of chunk k; an empty file has none. Errors per file as oxh_fastcdc_files. `capacity` entries of
 * `digests`; the count needed is sum(ceil(size_i / chunk_size)) (more fails with OXH_ERR_INVALID,
 * "need N entries"). chunk_size 0 -> OXH_ERR_INVALID ("Chunk size cannot be zero", fixedsize.rs:43-47);
 * chunk_size is at most 3 GiB - 64 MiB (a chunk fits one device piece). */
int oxh_chunk_digests_files(oxh_ctx* ctx, const char* const* paths, uint64_t n, uint64_t chunk_size, uint64_t* digests,
                            uint64_t capacity, uint64_t* first_chunk, uint64_t* sizes, int32_t* status, int32_t* os_error);
int oxh_chunk_digests_host(oxh_ctx* ctx, const uint8_t* const* bufs, const uint64_t* lens, uint64_t n,
                           uint64_t chunk_size, uint64_t* digests, uint64_t capacity, uint64_t* first_chunk);
/* oxh_fastcdc_files / oxh_chunk_digests_files over several contexts (one per device, so one PCIe link,
 * pipeline and reader pool each): the files split into nctx contiguous shares balanced by
 * their stat sizes, the shares run side by side, and the tables come back concatenated in file order --
 * every output exactly as the single-context call gives it. Contexts may repeat (shares on the same
 * context run one after the other). A failing share fails the call with its text ("share k ..."). */
int oxh_fastcdc_files_multi(oxh_ctx* const* ctxs, int nctx, const char* const* paths, uint64_t n, uint32_t min_size,
                            uint32_t avg_size, uint32_t max_size, uint32_t level, uint64_t* chunk_offsets,
                            uint64_t* chunk_lens, uint64_t* digests, uint64_t capacity, uint64_t* first_chunk,
                            uint64_t* sizes, int32_t* status, int32_t* os_error);
int oxh_chunk_digests_files_multi(oxh_ctx* const* ctxs, int nctx, const char* const* paths, uint64_t n,
                                  uint64_t chunk_size, uint64_t* digests, uint64_t capacity, uint64_t* first_chunk,
                                  uint64_t* sizes, int32_t* status, int32_t* os_error);
/* ... and the host-buffer entries (oxh_fastcdc_host / oxh_chunk_digests_host) the same way, the shares
 * balanced by the buffers' lengths. */
int oxh_fastcdc_host_multi(oxh_ctx* const* ctxs, int nctx, const uint8_t* const* bufs, const uint64_t* lens, uint64_t n,
                           uint32_t min_size, uint32_t avg_size, uint32_t max_size, uint32_t level, uint64_t* chunk_offsets,
                           uint64_t* chunk_lens, uint64_t* digests, uint64_t capacity, uint64_t* first_chunk);
int oxh_chunk_digests_host_multi(oxh_ctx* const* ctxs, int nctx, const uint8_t* const* bufs, const uint64_t* lens, uint64_t n,
                                 uint64_t chunk_size, uint64_t* digests, uint64_t capacity, uint64_t* first_chunk);
/* The compiled-in GEAR table (256 u64) and the (mask_s, mask_l) pair for an average size and
 * normalization level (fastcdc v2020 MASKS[bits +/- level], bits = round(log2(avg))). Host only. */
int oxh_fastcdc_gear(uint64_t* out256);
int oxh_fastcdc_masks(uint32_t avg_size, uint32_t level, uint64_t* mask_s, uint64_t* mask_l);

/* ---------------------------------------------------------------- K2: merkle parent nodes */
/* get_combined_hash (hasher.rs:67-80) x n on the device:
 * XXH3-128(content.to_le_bytes() || metadata.to_le_bytes()), inputs as (lo, hi) pairs. */
int oxh_combined_hash_device(const uint64_t* d_content, const uint64_t* d_metadata, uint64_t n,
                             uint64_t* d_out, void* stream);
/* Host-resident batch of caller-serialised parent streams (vnode ids, commit_writer.rs:686-720;
 * dir hashes, commit_writer.rs:995-1147; metadata JSON, hasher.rs:95-100): item i is
 * streams[offsets[i] .. offsets[i] + lens[i]). Blocks until `out` (2n u64) is filled. */
int oxh_hash_streams(oxh_ctx* ctx, const uint8_t* streams, const uint64_t* offsets,
                     const uint64_t* lens, uint64_t n, uint64_t* out);

/* ---------------------------------------------------------------- multi-GPU: the digest gather
 * files shard across the GPUs of a node as contiguous byte-balanced ranges, one process
 * per GPU and no data-path collective; the one exchange is the 16-B-per-file digest table, gathered over
 * xGMI with RCCL. This replaces the reference's in-process fan-out of 64-file batches
 * (core/v_latest/add.rs:422-425) when the shards are device-resident on several GPUs.
 * RCCL is loaded at run time (librccl.so.1; $OXH_RCCL_LIB overrides); without it the calls fail with
 * OXH_ERR_NODEVICE.
 * One rank calls oxh_comm_unique_id and hands the OXH_COMM_ID_BYTES bytes to every rank out of band
 * (as ncclGetUniqueId); each rank then calls oxh_comm_create with its rank and GPU (it blocks until all
 * nranks have). oxh_gather_digests: counts[q] (host, nranks entries, the same on every rank) = rank q's
 * item count; rank q's d_local holds its 2 * counts[q] u64 digests (lo, hi); d_full (2 * sum(counts) u64,
 * device) receives every rank's table in rank order -- on every rank when root < 0 (all-gather), else on
 * rank `root` only (d_full may be NULL on the others). Equal counts take one ncclAllGather / ncclGather,
 * ragged ones a group of point-to-point transfers. Enqueued on `stream` (hipStream_t, NULL = the null
 * stream); returns without waiting. A communicator is used by one thread at a time.
 * oxh_comm_check: OXH_OK when RCCL loads and `device` is a visible HIP device, else the error
 * oxh_comm_create would return for that reason (OXH_ERR_NODEVICE / OXH_ERR_INVALID) without joining
 * anything -- every rank calls it and the job agrees on the result before any rank enters
 * oxh_comm_create, which would otherwise wait in RCCL's bootstrap for a rank that has already failed. */
#define OXH_COMM_ID_BYTES 128
typedef struct oxh_comm oxh_comm;
int oxh_comm_check(int device);
int oxh_comm_unique_id(uint8_t* id);
int oxh_comm_create(const uint8_t* id, int rank, int nranks, int device, oxh_comm** out);
int oxh_comm_info(oxh_comm* comm, int* rank, int* nranks, int* device);
int oxh_gather_digests(oxh_comm* comm, const uint64_t* d_local, const uint64_t* counts, uint64_t* d_full, int root,
                       void* stream);
int oxh_comm_destroy(oxh_comm* comm);

/* ---------------------------------------------------------------- formatting (host only) */
/* MerkleHash Display (merkle_hash.rs:73-77): format!("{:x}") -- lowercase, NOT zero-padded.
 * `out` must hold 33 bytes; returns the string length (1..32). */
int oxh_format_hex(uint64_t lo, uint64_t hi, char* out);
/* u128::to_string() -- the decimal chunk names of the dedup experiment (fixedsize.rs:78).
 * `out` must hold 40 bytes; returns the string length. */
int oxh_format_dec(uint64_t lo, uint64_t hi, char* out);

/* ---------------------------------------------------------------- bench / test utilities */
/* Fill d_buf[0..nbytes) with the counter-based splitmix64 byte stream of `seed` (byte j is byte
 * j%8, little-endian, of splitmix64(seed + (j/8 + 1) * 0x9E3779B97F4A7C15)) so that a host can
 * regenerate any item of a device-resident synthetic workload without copying it back. */
int oxh_fill_splitmix(void* d_buf, uint64_t nbytes, uint64_t seed, void* stream);
/* Diagnostic: select the long-path kernel variant (0 = default). Returns the previous value. */
int oxh_set_kernel_variant(int variant);
/* Diagnostic counters of a context, out[0..n): [0] device allocations of the large-file piece buffers
 * (files above a staging slot; each one synchronises the device), [1] their current bytes, [2] file
 * requests served on the caller's thread (small requests on an idle context), [3] file-engine runs;
 * further entries 0. */
int oxh_ctx_counters(oxh_ctx* ctx, uint64_t* out, int n);

#ifdef __cplusplus
}
#endif
#endif /* OXEN_HASH_H */
