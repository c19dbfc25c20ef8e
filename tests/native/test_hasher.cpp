// tests/native/test_hasher.cpp -- the C++ host mirror of liboxen `util::hasher` on the GPU, tested
// the way the reference tests hasher.rs (hashing_reader_tests / hashing_writer_tests, :246-350), plus
// known-answer digests (the reference's schemas.rs:131 KAT, data/test/text/hello.txt),
// the error behaviour of the file functions, MerkleHash formatting and a long GPU stream.
//
// Built by oxen_amd/build.py (g++ against liboxen_hasher.so + liboxen_hash.so); run by
// tests/test_native_mirror.py on the GPU box. argv[1] = tests/golden. Exit status 0 = all passed.
#include <dirent.h>
#include <errno.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "../../oxen_amd/host/oxen_hasher.hpp"

using liboxen::MerkleHash;
using liboxen::OxenError;
using liboxen::u128;
namespace hasher = liboxen::util::hasher;

static int g_fail = 0, g_pass = 0;
#define CHECK(cond)                                                               \
    do {                                                                          \
        if (cond) {                                                               \
            ++g_pass;                                                             \
        } else {                                                                  \
            ++g_fail;                                                             \
            fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);       \
        }                                                                         \
    } while (0)

template <class F>
static bool throws_oxen(F f, const char* needle = nullptr) {
    try {
        f();
    } catch (const OxenError& e) {
        return !needle || strstr(e.what(), needle) != nullptr;
    }
    return false;
}

// the exact message
template <class F>
static bool throws_oxen(F f, const std::string& exact) {
    try {
        f();
    } catch (const OxenError& e) {
        if (exact != e.what()) fprintf(stderr, "  message: %s\n  expected: %s\n", e.what(), exact.c_str());
        return exact == e.what();
    }
    return false;
}

static u128 hex(const char* s) { return MerkleHash::from_str(s).to_u128(); }

// a `Read` over a byte string, `chunk` bytes per call
struct SliceReader {
    const std::string& data;
    size_t pos = 0, chunk;
    size_t read(uint8_t* buf, size_t n) {
        const size_t k = std::min({n, chunk, data.size() - pos});
        memcpy(buf, data.data() + pos, k);
        pos += k;
        return k;
    }
};

struct VecWriter {
    std::string written;
    size_t write(const uint8_t* b, size_t n) {
        written.append(reinterpret_cast<const char*>(b), n);
        return n;
    }
    void flush() {}
};

struct ShortWriter {  // hasher.rs:323-335: accepts at most 4 bytes per call
    std::string written;
    size_t write(const uint8_t* b, size_t n) {
        const size_t k = std::min<size_t>(n, 4);
        written.append(reinterpret_cast<const char*>(b), k);
        return k;
    }
    void flush() {}
};

static const std::string kPayload = "the quick brown fox jumps over the lazy dog";

static void hashing_reader_tests() {
    {  // sync_reader_matches_one_shot (hasher.rs:250-259)
        SliceReader src{kPayload, 0, 5};
        hasher::HashingReader<SliceReader> hashing(src);
        std::string sink;
        uint8_t buf[64];
        while (size_t n = hashing.read(buf, sizeof buf)) sink.append(reinterpret_cast<char*>(buf), n);
        CHECK(sink == kPayload);
        CHECK(hashing.digest128() == hasher::hash_buffer_128bit(kPayload));
        CHECK(hashing.digest128() == hex("e9a1932627d7f46d15c21eead63fa21f"));
    }
    {  // sync_reader_empty_input (:261-269)
        const std::string empty;
        SliceReader src{empty, 0, 5};
        hasher::HashingReader<SliceReader> hashing(src);
        uint8_t buf[8];
        CHECK(hashing.read(buf, sizeof buf) == 0);
        CHECK(hashing.digest128() == hex("99aa06d3014798d86001c324468d497f"));
    }
}

static void hashing_writer_tests() {
    {  // sync_writer_matches_one_shot (:276-289)
        VecWriter sink;
        u128 digest;
        {
            hasher::HashingWriter<VecWriter> hashing(sink);
            hashing.write_all(reinterpret_cast<const uint8_t*>(kPayload.data()), kPayload.size());
            hashing.flush();
            digest = hashing.digest128();
        }
        CHECK(digest == hasher::hash_buffer_128bit(kPayload));
        CHECK(sink.written == kPayload);
    }
    {  // sync_writer_accumulates_across_writes (:293-308)
        VecWriter sink;
        hasher::HashingWriter<VecWriter> hashing(sink);
        for (const char* chunk : {"hello ", "brave ", "world"})
            hashing.write_all(reinterpret_cast<const uint8_t*>(chunk), strlen(chunk));
        CHECK(hashing.digest128() == hex("6a11bc56dc3c4cce2f81a90bed1a8d2c"));
        CHECK(sink.written == "hello brave world");
    }
    {  // sync_writer_empty_input (:310-317)
        VecWriter sink;
        CHECK(hasher::HashingWriter<VecWriter>(sink).digest128() == hex("99aa06d3014798d86001c324468d497f"));
        CHECK(sink.written.empty());
    }
    {  // sync_writer_hashes_only_accepted_bytes (:321-349)
        ShortWriter inner;
        u128 digest;
        {
            hasher::HashingWriter<ShortWriter> hashing(inner);
            const size_t accepted = hashing.write(reinterpret_cast<const uint8_t*>("0123456789"), 10);
            CHECK(accepted == 4);
            digest = hashing.digest128();
        }
        CHECK(inner.written == "0123");
        CHECK(digest == hex("e7f00c8d576b45ee824b77d5917b737b"));
    }
}

static void known_answers(const std::string& golden) {
    CHECK(hasher::hash_str("") == "99aa06d3014798d86001c324468d497f");
    CHECK(hasher::hash_str("hello") == "b5e9c1ad071b3e7fc779cfaa5e523818");
    CHECK(hasher::hash_str(std::string(65536, 'x')) == "2da4b9c5a75caad3688558138047f8a");  // unpadded
    // repositories/data_frames/schemas.rs:131
    CHECK(hasher::hash_str("filestrlabelstrmin_xf64min_yf64widthi64heighti64") == "b821946753334c083124fd563377d795");
    // add.rs:833-842 on a C1 text file: content, metadata and combined hashes
    const u128 c = hasher::hash_buffer_128bit(std::string_view("File content 0"));
    CHECK(hasher::format_hex(c) == "393ba5849f5590fc5985c4bbcec0003f");
    const auto m = hasher::maybe_get_metadata_hash(std::string("{\"text\":{\"num_lines\":1,\"num_chars\":14}}"));
    CHECK(m && hasher::format_hex(*m) == "5b1951f1adb8e39ebda9b20e8c20a11");
    CHECK(hasher::format_hex(hasher::get_combined_hash(m, c)) == "957a1ebb6676cdb2a326863b0858a474");
    CHECK(hasher::get_combined_hash(std::nullopt, c) == c);
    CHECK(!hasher::maybe_get_metadata_hash(std::nullopt));
    CHECK(hasher::get_metadata_hash(std::nullopt) == hasher::hash_buffer_128bit(std::string_view("null")));
    // the reference's data/test fixture (tests/golden/data_test/text/hello.txt)
    const std::string hello = golden + "/data_test/text/hello.txt";
    CHECK(hasher::hash_file_contents(hello) == "1bfd09d1a433fb78117b4c7b1583d16d");
    struct stat sb;
    CHECK(stat(hello.c_str(), &sb) == 0 && hasher::format_hex(hasher::get_hash_given_metadata(hello, sb)) ==
                                               "1bfd09d1a433fb78117b4c7b1583d16d");
}

static void file_errors(const std::string& golden) {
    const std::string missing = golden + "/no-such-file";
    struct stat sb {};
    // hasher.rs:141-145: File::open's io::Error in its Debug form (the errno crosses the ABI)
    const std::string enoent = "Os { code: 2, kind: NotFound, message: \"No such file or directory\" }";
    // hasher.rs:117 -> util::fs::metadata (fs.rs:593-601) -> OxenError::file_metadata_error (error.rs:1176-1182)
    CHECK(throws_oxen([&] { hasher::hash_file_contents(missing); },
                      "Could not get file metadata: \"" + missing + "\" error " + enoent));
    const std::string notdir = golden + "/data_test/text/hello.txt/x";  // ENOTDIR: root cannot bypass it
    CHECK(throws_oxen([&] { hasher::u128_hash_file_contents(notdir); },
                      "Could not get file metadata: \"" + notdir +
                          "\" error Os { code: 20, kind: NotADirectory, message: \"Not a directory\" }"));
    CHECK(throws_oxen([&] { hasher::get_hash_given_metadata(notdir, sb); },
                      "util::hasher::hash_file_contents Could not open file \"" + notdir +
                          "\" Os { code: 20, kind: NotADirectory, message: \"Not a directory\" }"));
    CHECK(throws_oxen([&] { hasher::get_hash_given_metadata(missing, sb); },
                      "util::hasher::hash_file_contents Could not open file \"" + missing + "\" " + enoent));
    struct stat big {};
    big.st_size = 2000000000;  // the streamed branch's message (hasher.rs:151-154)
    CHECK(throws_oxen([&] { hasher::get_hash_given_metadata(missing, big); },
                      "Could not open file \"" + missing + "\" due to " + enoent));
    CHECK(throws_oxen([&] { hasher::get_hash_given_metadata(golden, sb); }, "Could not read file for hashing"));
    CHECK(hasher::rust_str_debug("a\"b\\c\nd\x01") == "\"a\\\"b\\\\c\\nd\\u{1}\"");
    // Path Debug: a single quote escaped, bytes outside UTF-8 as \xNN, zero-width space and combining
    // acute as \u{..}; str Debug keeps the single quote
    CHECK(hasher::rust_path_debug("a'b\xff\xfe\xe2\x80\x8bx\xcc\x81\xc3\xa9") == "\"a\\'b\\xFF\\xFE\\u{200b}x\\u{301}\xc3\xa9\"");
    CHECK(hasher::rust_str_debug("it's") == "\"it's\"");
    CHECK(hasher::rust_io_error_debug(40) == "Os { code: 40, kind: FilesystemLoop, message: \"Too many levels of symbolic links\" }");
    CHECK(hasher::rust_io_error_debug(24) == "Os { code: 24, kind: Uncategorized, message: \"Too many open files\" }");
    std::vector<int> sleeps;
    CHECK(throws_oxen([&] { hasher::hash_file_contents_with_retry(missing, 5, [&](int s) { sleeps.push_back(s); }); }));
    CHECK((sleeps == std::vector<int>{2, 4, 8, 16, 32, 64}));  // hasher.rs:32-54
    const auto r = hasher::hash_files({golden + "/data_test/text/hello.txt", missing, golden});
    CHECK(r.size() == 3 && r[0].ok && r[0].size == 5 && !r[1].ok && !r[2].ok);
    CHECK(r[1].error == "util::hasher::hash_file_contents Could not open file \"" + missing + "\" " + enoent);
    CHECK(r[1].code == OXH_ERR_OPEN && r[1].os_error == ENOENT);
    CHECK(r[2].error == "Could not read file for hashing" && r[2].code == OXH_ERR_IO && r[2].os_error == EISDIR);
}

// The reader-process pool (oxh_pool_*) through liboxen::util::hasher::ReaderPool: the same outcomes
// as one context's hash_files, per file, with and without the walk's sizes, over 2 and 3 helpers.
static void reader_pool(const std::string& golden) {
    const std::string missing = golden + "/no-such-file";
    std::vector<std::string> paths;
    std::vector<uint64_t> sizes;
    if (DIR* dp = opendir((golden + "/data_test/text").c_str())) {
        while (dirent* e = readdir(dp))
            if (e->d_name[0] != '.') paths.push_back(golden + "/data_test/text/" + e->d_name);
        closedir(dp);
    }
    paths.push_back(missing);
    paths.push_back(golden);  // a directory: cannot be read
    for (const std::string& p : paths) {
        struct stat sb {};
        sizes.push_back(stat(p.c_str(), &sb) == 0 ? (uint64_t)sb.st_size : 0);
    }
    const auto want = hasher::hash_files(paths);
    for (int procs : {2, 3}) {
        hasher::ReaderPool pool(procs, {0});
        CHECK(pool.procs() == procs);
        for (int with_sizes = 0; with_sizes < 2; ++with_sizes) {
            const auto got = pool.hash_files(paths, with_sizes ? sizes : std::vector<uint64_t>{});
            bool same = got.size() == want.size();
            for (size_t i = 0; same && i < got.size(); ++i)
                same = got[i].ok == want[i].ok && got[i].hash == want[i].hash && got[i].error == want[i].error &&
                       (!got[i].ok || got[i].size == want[i].size);
            CHECK(same);
        }
        CHECK(pool.hash_files({}).empty());
    }
    CHECK(throws_oxen([&] { hasher::ReaderPool bad(0); }));
}

static void merkle_hash() {
    const MerkleHash h = MerkleHash::from_str("2da4b9c5a75caad3688558138047f8a");
    CHECK(h.to_string() == "2da4b9c5a75caad3688558138047f8a");
    CHECK(h.to_short_str() == "2da4b9c5a7");
    CHECK(h.node_db_prefix() == "2da/4b9c5a75caad3688558138047f8a");
    uint8_t le[16];
    h.to_le_bytes(le);
    CHECK(le[0] == 0x8a && le[15] == 0x02);
    CHECK(MerkleHash::from_str("FF").to_u128() == 255 && MerkleHash::from_str("+1").to_u128() == 1);
    CHECK(MerkleHash(0).to_string() == "0");
    CHECK(throws_oxen([] { MerkleHash::from_str(""); }));
    CHECK(throws_oxen([] { MerkleHash::from_str("xyz"); }));
    CHECK(throws_oxen([] { MerkleHash::from_str("1ffffffffffffffffffffffffffffffff"); }));  // 33 digits
}

static void long_stream() {
    // 40 MiB + 1234 B in ragged updates: three 16 MiB device pieces with resumed chains + the tail
    std::string data(40u * 1024 * 1024 + 1234, '\0');
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (size_t i = 0; i < data.size(); i += 8) {
        x ^= x << 13, x ^= x >> 7, x ^= x << 17;
        memcpy(&data[i], &x, std::min<size_t>(8, data.size() - i));
    }
    hasher::Xxh3 h;
    size_t pos = 0, step = 1;
    while (pos < data.size()) {
        const size_t k = std::min(step, data.size() - pos);
        h.update(data.data() + pos, k);
        pos += k;
        step = step * 7 % 5000011 + 1;
    }
    const u128 one_shot = hasher::hash_buffer_128bit(data.data(), data.size());
    CHECK(h.digest128() == one_shot);
    CHECK(h.digest128() == one_shot);  // digest128 does not consume the state
    h.reset();
    h.update(std::string_view("hello"));
    CHECK(h.digest128() == hex("b5e9c1ad071b3e7fc779cfaa5e523818"));
}

// util::fs::classify_modified_from_node_with_metadata (util/fs.rs:1580-1619) over oxh_files_modified:
// size differs -> modified without a read; matched mtime -> clean without a read; else content hash.
static void modified_check(const std::string& golden) {
    namespace fs = liboxen::util::fs;
    const std::string hello = golden + "/data_test/text/hello.txt";  // 5 bytes, KAT below
    const u128 h = hex("1bfd09d1a433fb78117b4c7b1583d16d");
    std::vector<fs::TrackedFile> t = {
        {hello, 5, 5, h, false},          // same content, drifted mtime: hashed, clean
        {hello, 5, 5, h + 1, false},      // node hash differs: hashed, modified
        {hello, 5, 5, h + 1, true},       // matched mtime is trusted: not read, clean
        {hello, 5, 6, h, false},          // size differs: not read, modified
        {golden + "/no/such/file", 3, 3, h, false},  // must be hashed, cannot be read
    };
    uint64_t hashed = 0;
    const std::vector<fs::Modified> r = fs::classify_modified_batch(t, nullptr, &hashed);
    CHECK(r.size() == 5 && hashed == 3);
    CHECK(r[0].ok && !r[0].modified);
    CHECK(r[1].ok && r[1].modified);
    CHECK(r[2].ok && !r[2].modified);
    CHECK(r[3].ok && r[3].modified);
    CHECK(!r[4].ok && !r[4].modified && r[4].code == OXH_ERR_OPEN &&
          r[4].error == "util::hasher::hash_file_contents Could not open file \"" + golden +
                            "/no/such/file\" Os { code: 2, kind: NotFound, message: \"No such file or directory\" }");
    struct stat sb;
    CHECK(stat(hello.c_str(), &sb) == 0 && !fs::classify_modified_from_node_with_metadata(hello, 5, h, sb, false));
    CHECK(throws_oxen([&] { fs::classify_modified_from_node_with_metadata(golden + "/no/such/file", (uint64_t)sb.st_size, h, sb, false); },
                      ("Could not open file \"" + golden + "/no/such/file\"").c_str()));

    // the metadata-hash step (fs.rs:1599-1614): hello.txt is MetadataText {1 line, 5 chars}
    const u128 mh = liboxen::util::hasher::get_metadata_hash(std::string("{\"text\":{\"num_lines\":1,\"num_chars\":5}}"));
    fs::FileMetadataHash text, given_stale, err;
    text.kind = fs::FileMetadataHash::Text;
    given_stale.kind = fs::FileMetadataHash::Given, given_stale.hash = mh + 1;
    err.kind = fs::FileMetadataHash::Error, err.error = "no extractor";
    std::vector<fs::TrackedFile> m = {
        {hello, 5, 5, h, false, mh, text},            // counted on the read: equal -> content: clean
        {hello, 5, 5, h, false, mh + 7, text},        // stale node metadata hash, same content: modified
        {hello, 5, 5, h, false, std::nullopt, text},  // node has none: no comparison, clean
        {hello, 5, 5, h, false, mh, given_stale},     // caller-given differs: modified, not read
        {hello, 5, 5, h, false, mh, err},             // extraction error: returned, not read
    };
    const std::vector<fs::Modified> q = fs::classify_modified_batch(m, nullptr, &hashed);
    CHECK(hashed == 3);
    CHECK(q[0].ok && !q[0].modified);
    CHECK(q[1].ok && q[1].modified);
    CHECK(q[2].ok && !q[2].modified);
    CHECK(q[3].ok && q[3].modified);
    CHECK(!q[4].ok && q[4].code == OXH_ERR_META && q[4].error == "no extractor");
    CHECK(fs::classify_modified_from_node_with_metadata(hello, 5, h, sb, false, mh + 7, text));
    CHECK(throws_oxen([&] { fs::classify_modified_from_node_with_metadata(hello, 5, h, sb, false, mh, err); }, "no extractor"));
}

static std::vector<std::string> list_dir(const std::string& d) {
    std::vector<std::string> r;
    if (DIR* dp = opendir(d.c_str())) {
        while (dirent* e = readdir(dp))
            if (strcmp(e->d_name, ".") && strcmp(e->d_name, "..")) r.push_back(e->d_name);
        closedir(dp);
    }
    return r;
}
static std::string read_file(const std::string& p) {
    std::string out;
    if (FILE* f = fopen(p.c_str(), "rb")) {
        char b[65536];
        size_t k;
        while ((k = fread(b, 1, sizeof b, f)) > 0) out.append(b, k);
        fclose(f);
    }
    return out;
}
// a reader over a byte string, in pieces of at most `piece` bytes; throws after `fail_after` bytes
struct StrReader {
    std::string data;
    size_t pos = 0, piece = 1 << 30, fail_after = (size_t)-1;
    size_t operator()(uint8_t* buf, size_t n) {
        if (pos >= fail_after) throw OxenError::basic_str("simulated read failure");
        const size_t k = std::min({n, piece, data.size() - pos, fail_after - pos});
        memcpy(buf, data.data() + pos, k);
        pos += k;
        return k;
    }
};

// util/fs/atomic_file.rs tests (verified stream / write: commits on match, aborts on mismatch with
// HashMismatch and nothing left behind, cleans up on read failure) and storage/version_store.rs's
// verify_suite::assert_rejects_mismatched_content, over the GPU-verified mirror.
static void verified_publish(const std::string& scratch) {
    namespace fs = liboxen::util::fs;
    using liboxen::storage::LocalVersionStore;
    std::string payload;  // (0..50_000u32).flat_map(u32::to_le_bytes)
    for (uint32_t i = 0; i < 50000; ++i) payload.append((const char*)&i, 4);
    const MerkleHash want(hex("290ee6c54069340c8a3c8891ce6b2d9"));  // xxh3_128(payload), oracle + libxxhash
    const MerkleHash bogus((u128)0xdeadbeefdeadbeefull << 64 | 0xdeadbeefdeadbeefull);
    const std::string d1 = scratch + "/commit", d2 = scratch + "/abort", d3 = scratch + "/readfail", d4 = scratch + "/write";
    for (const auto& d : {d1, d2, d3, d4}) mkdir(d.c_str(), 0755);

    StrReader r1{payload, 0, 7777};
    fs::AtomicFile(d1 + "/blob.bin").with_hash(want).stream(std::ref(r1));
    CHECK(read_file(d1 + "/blob.bin") == payload && list_dir(d1).size() == 1);

    StrReader r2{payload};
    bool mism = false;
    try {
        fs::AtomicFile(d2 + "/blob.bin").with_hash(bogus).stream(std::ref(r2));
    } catch (const OxenError& e) {
        mism = e.kind() == OxenError::Kind::HashMismatch && strstr(e.what(), "expected deadbeefdeadbeefdeadbeefdeadbeef") &&
               strstr(e.what(), "got 290ee6c54069340c8a3c8891ce6b2d9");
    }
    CHECK(mism && list_dir(d2).empty());

    StrReader r3{payload, 0, 4096, 100000};
    CHECK(throws_oxen([&] { fs::AtomicFile(d3 + "/blob.bin").with_hash(want).stream(std::ref(r3)); }, "simulated read failure"));
    CHECK(list_dir(d3).empty());

    CHECK(throws_oxen([&] { fs::AtomicFile(d4 + "/blob.bin").with_hash(bogus).write(payload.data(), payload.size()); }, "Hash mismatch"));
    CHECK(list_dir(d4).empty());
    fs::AtomicFile(d4 + "/blob.bin").with_hash(want).write(payload.data(), payload.size());
    CHECK(read_file(d4 + "/blob.bin") == payload && list_dir(d4).size() == 1);

    // verify_suite: DATA under WRONG_HASH is rejected by both content-addressed writes
    const std::string data = "the quick brown fox jumps over the lazy dog";
    const std::string wrong = "deadbeefdeadbeefdeadbeefdeadbeef", right = "e9a1932627d7f46d15c21eead63fa21f";
    LocalVersionStore store(scratch + "/versions");
    CHECK(hasher::hash_buffer(data.data(), data.size()) == right);
    CHECK(throws_oxen([&] { store.store_version(wrong, data.data(), data.size()); }, "mismatch"));
    CHECK(!store.version_exists(wrong));
    StrReader r4{data};
    CHECK(throws_oxen([&] { store.store_version_from_reader(wrong, std::ref(r4), data.size()); }, "mismatch"));
    CHECK(!store.version_exists(wrong));
    StrReader r5{data, 0, 5};
    store.store_version_from_reader(right, std::ref(r5), data.size());
    CHECK(store.version_exists(right) && read_file(store.version_path(right)) == data);
    CHECK(store.version_path(right) == scratch + "/versions/e9/a1932627d7f46d15c21eead63fa21f/data");
    store.store_version(right, "ignored: the blob exists", 24);  // local.rs:127-129
    CHECK(read_file(store.version_path(right)) == data);

    // batched receive: one GPU pass over every buffer
    const std::vector<std::string> hs = {hasher::hash_buffer(payload.data(), payload.size()), wrong, right,
                                         hasher::hash_buffer("", 0), hasher::hash_buffer(payload.data(), payload.size())};
    const std::vector<std::string_view> ds = {payload, data, data, std::string_view(), payload};
    const std::vector<std::string> err = store.store_versions(hs, ds);
    CHECK(err.size() == 5 && err[0].empty() && err[1].find("Hash mismatch") != std::string::npos && err[2].empty() &&
          err[3].empty() && err[4].empty());
    CHECK(read_file(store.version_path(hs[0])) == payload && store.version_exists(hs[3]) &&
          read_file(store.version_path(hs[3])).empty() && !store.version_exists(wrong));
    CHECK(list_dir(store.version_dir(hs[0])).size() == 1);  // no .oxentmp. leftovers

    // chunked upload (local.rs:862-891): chunks at their byte offsets, reassembled in numeric offset
    // order, verified, the chunks directory removed; a wrong hash publishes nothing and keeps them
    const std::string ph = hasher::hash_buffer(payload.data(), payload.size());
    const std::vector<uint64_t> cuts = {0, 7, 100, 150000, payload.size()};  // "100" sorts after "7" only numerically
    LocalVersionStore store2(scratch + "/versions2");
    for (size_t k = 0; k + 1 < cuts.size(); ++k)
        store2.store_version_chunk(ph, cuts[k], payload.data() + cuts[k], cuts[k + 1] - cuts[k]);
    CHECK((store2.list_version_chunks(ph) == std::vector<uint64_t>{0, 7, 100, 150000}));
    store2.combine_version_chunks(ph);
    CHECK(read_file(store2.version_path(ph)) == payload && list_dir(store2.version_dir(ph)).size() == 1);
    store2.store_version_chunk(wrong, 0, data.data(), data.size());
    CHECK(throws_oxen([&] { store2.combine_version_chunks(wrong); }, "Hash mismatch"));
    CHECK(!store2.version_exists(wrong) && store2.list_version_chunks(wrong) == std::vector<uint64_t>{0});
    // names parse as Rust's u64 (an optional '+', ASCII digits, < 2^64); a symlink is not a chunk dir
    const std::string cdir = store2.version_chunks_dir(wrong);
    for (const char* name : {"+5", "-1", "1_0", " 7", "007", "18446744073709551616", "x"})
        CHECK(mkdir((cdir + "/" + name).c_str(), 0755) == 0);
    CHECK(symlink((cdir + "/0").c_str(), (cdir + "/99").c_str()) == 0);
    CHECK((store2.list_version_chunks(wrong) == std::vector<uint64_t>{0, 5, 7}));
}

// dedup::fastcdc_files / fastcdc_buffers (fastcdchunker.rs:75-98 over oxh_fastcdc_files / _host): the two
// entries agree, chunks tile each file within [min, max] (a file's last may be shorter), every chunk's hash
// equals hash_buffer_128bit of its bytes (K1 through the host-buffer path), and a missing path is that
// file's error only. The boundaries against the oracle: tests/test_fastcdc.py.
static void dedup_chunks(const std::string& golden) {
    namespace dd = liboxen::dedup;
    std::string big(3000017, '\0');
    uint64_t z = 12345;
    for (auto& ch : big) {
        z = z * 6364136223846793005ull + 1442695040888963407ull;
        ch = (char)(z >> 56);
    }
    char tmpl[] = "/tmp/oxh_cdc_XXXXXX";
    const char* dir = mkdtemp(tmpl);
    CHECK(dir != nullptr);
    if (!dir) return;
    const std::string p_big = std::string(dir) + "/big.bin";
    if (FILE* f = fopen(p_big.c_str(), "wb")) {
        fwrite(big.data(), 1, big.size(), f);
        fclose(f);
    }
    const std::string hello = golden + "/data_test/text/hello.txt", missing = std::string(dir) + "/missing";
    const auto files = dd::fastcdc_files({p_big, missing, hello}, 4096, 8192, 16384);
    CHECK(files.size() == 3 && files[0].ok && !files[1].ok && files[2].ok);
    CHECK(files[1].code == OXH_ERR_OPEN && files[1].os_error == ENOENT && files[1].chunks.empty());
    CHECK(files[0].size == big.size() && files[2].size == 5 && files[2].chunks.size() == 1);
    const auto bufs = dd::fastcdc_buffers({std::string_view(big), std::string_view("hello")}, 4096, 8192, 16384);
    CHECK(bufs.size() == 2 && bufs[0].size() == files[0].chunks.size());
    uint64_t at = 0;
    bool tiles = true, same = true, hashes = true;
    for (size_t k = 0; k < files[0].chunks.size(); ++k) {
        const auto& c = files[0].chunks[k];
        tiles = tiles && c.offset == at && c.length <= 16384 && (c.length >= 4096 || k + 1 == files[0].chunks.size());
        same = same && k < bufs[0].size() && bufs[0][k].offset == c.offset && bufs[0][k].length == c.length &&
               bufs[0][k].hash == c.hash;
        at += c.length;
    }
    for (size_t k = 0; k < files[0].chunks.size(); k += 37) {
        const auto& c = files[0].chunks[k];
        hashes = hashes && hasher::hash_buffer_128bit(big.data() + c.offset, c.length) == c.hash;
    }
    CHECK(tiles && at == big.size());
    CHECK(same);
    CHECK(hashes);
    CHECK(files[2].chunks[0].hash == hex("1bfd09d1a433fb78117b4c7b1583d16d"));
    CHECK(dd::chunk_name(files[2].chunks[0].hash) == "37203006142592822661058489871983956333");
    // fixed-size chunks (fixedsize_multithreaded.rs:78-110) of the same files and buffers
    const auto fx = dd::fixed_chunk_files({p_big, missing, hello}, 65536);
    const auto fb = dd::fixed_chunk_buffers({std::string_view(big), std::string_view("hello")}, 65536);
    CHECK(fx.size() == 3 && fx[0].ok && !fx[1].ok && fx[1].os_error == ENOENT && fx[2].ok);
    CHECK(fx[0].chunks.size() == (big.size() + 65535) / 65536 && fb[0].size() == fx[0].chunks.size());
    bool fixed_ok = true;
    for (size_t k = 0; k < fx[0].chunks.size(); ++k) {
        const auto& c = fx[0].chunks[k];
        fixed_ok = fixed_ok && c.offset == 65536 * k && c.length == std::min<uint64_t>(65536, big.size() - c.offset) &&
                   c.hash == fb[0][k].hash && c.hash == hasher::hash_buffer_128bit(big.data() + c.offset, c.length);
    }
    CHECK(fixed_ok);
    CHECK(fx[2].chunks.size() == 1 && fx[2].chunks[0].hash == files[2].chunks[0].hash);
    CHECK(fb[1].size() == 1 && fb[1][0].hash == hasher::hash_buffer_128bit("hello", 5));
    // the same over two contexts on device 0 (oxh_*_files_multi): identical tables
    oxh_ctx* c2 = nullptr;
    CHECK(oxh_ctx_create(0, 0, &c2) == OXH_OK);
    const std::vector<oxh_ctx*> two{liboxen::util::hasher::default_context(), c2};
    const auto fx2 = dd::fixed_chunk_files({p_big, missing, hello}, 65536, two);
    const auto cd2 = dd::fastcdc_files({p_big, missing, hello}, 4096, 8192, 16384, two);
    bool multi_same = fx2.size() == 3 && cd2.size() == 3;
    for (size_t i = 0; multi_same && i < 3; ++i) {
        multi_same = fx2[i].ok == fx[i].ok && fx2[i].chunks.size() == fx[i].chunks.size() && cd2[i].ok == files[i].ok &&
                     cd2[i].chunks.size() == files[i].chunks.size() && cd2[i].os_error == files[i].os_error;
        for (size_t k = 0; multi_same && k < fx[i].chunks.size(); ++k) multi_same = fx2[i].chunks[k].hash == fx[i].chunks[k].hash;
        for (size_t k = 0; multi_same && k < files[i].chunks.size(); ++k)
            multi_same = cd2[i].chunks[k].hash == files[i].chunks[k].hash && cd2[i].chunks[k].offset == files[i].chunks[k].offset;
    }
    CHECK(multi_same);
    // ... and the buffer forms (oxh_*_host_multi)
    const std::vector<std::string_view> bv{std::string_view(big), std::string_view("hello"), std::string_view()};
    const auto fb2 = dd::fixed_chunk_buffers(bv, 65536, two);
    const auto cb2 = dd::fastcdc_buffers(bv, 4096, 8192, 16384, two);
    bool multi_bufs = fb2.size() == 3 && cb2.size() == 3 && fb2[2].empty() && cb2[2].empty();
    for (size_t i = 0; multi_bufs && i < 2; ++i) {
        multi_bufs = fb2[i].size() == fb[i].size() && cb2[i].size() == bufs[i].size();
        for (size_t k = 0; multi_bufs && k < fb[i].size(); ++k)
            multi_bufs = fb2[i][k].hash == fb[i][k].hash && fb2[i][k].offset == fb[i][k].offset;
        for (size_t k = 0; multi_bufs && k < bufs[i].size(); ++k)
            multi_bufs = cb2[i][k].hash == bufs[i][k].hash && cb2[i][k].length == bufs[i][k].length;
    }
    CHECK(multi_bufs);
    (void)oxh_ctx_destroy(c2);
    const std::string rm = std::string("rm -rf ") + dir;
    if (system(rm.c_str()) != 0) fprintf(stderr, "could not remove %s\n", dir);
}

// core::restore::should_restore_batch (restore.rs:231-405) against the per-file rules spelled out here
static void restore_checks() {
    namespace rs = liboxen::core::restore;
    char tmpl[] = "/tmp/oxh_restore_XXXXXX";
    const char* dir = mkdtemp(tmpl);
    CHECK(dir != nullptr);
    if (!dir) return;
    auto put = [&](const std::string& name, const std::string& data) {
        const std::string p = std::string(dir) + "/" + name;
        if (FILE* f = fopen(p.c_str(), "wb")) {
            fwrite(data.data(), 1, data.size(), f);
            fclose(f);
        }
        return p;
    };
    const std::string oldv = "line one\nline two\n", newv = "line one\nline two\nchanged\n", other = "something else";
    auto text_meta = [](const std::string& d) {
        uint64_t lines = 1, chars = 0;
        for (unsigned char c : d) lines += c == '\n', chars += (c & 0xC0) != 0x80;
        return hasher::get_metadata_hash(std::string("{\"text\":{\"num_lines\":") + std::to_string(lines) +
                                         ",\"num_chars\":" + std::to_string(chars) + "}}");
    };
    auto node = [&](const std::string& d, bool meta) {
        rs::NodeHashes h;
        h.hash = hasher::hash_buffer_128bit(d);
        h.num_bytes = d.size();
        h.combined_hash = meta ? hasher::get_combined_hash(text_meta(d), h.hash) : h.hash;
        return h;
    };
    for (bool combined : {false, true}) {
        std::vector<rs::RestoreCheck> v;
        std::vector<bool> want;
        auto add = [&](const std::string& path, bool has_base, bool mtime_ok, bool expect) {
            rs::RestoreCheck c;
            c.working_path = path;
            c.target = node(newv, combined);
            if (has_base) c.base = node(oldv, combined);
            c.mtime_matched = mtime_ok;
            if (combined) c.file_metadata.kind = liboxen::util::fs::FileMetadataHash::Text;
            v.push_back(c);
            want.push_back(expect);
        };
        const std::string p_new = put("new.txt", newv), p_old = put("old.txt", oldv), p_other = put("other.txt", other);
        add(std::string(dir) + "/missing", true, false, true);  // nothing to lose
        add(p_new, true, false, true);                          // already the target
        add(p_old, true, false, true);                          // unchanged since the base
        add(p_other, true, false, false);                       // modified: keep it
        add(p_other, false, false, false);                      // untracked and different
        add(p_new, false, false, true);                         // untracked and equal to the target
        add(put("short.txt", std::string(oldv.size(), 'z')), true, true, true);  // mtime + size short cut: no read
        add(p_other + "/x", true, false, true);  // stat fails (ENOTDIR): exists() is false, restore
        const std::string dangling = std::string(dir) + "/dangling" + (combined ? "1" : "0");
        CHECK(symlink((std::string(dir) + "/nowhere").c_str(), dangling.c_str()) == 0);
        add(dangling, false, false, true);  // exists() follows the link: absent, restore
        CHECK(rs::should_restore_batch(v, combined) == want);
    }
    rs::RestoreCheck d;
    d.working_path = dir;  // a directory: the hash's read fails (EISDIR) and the call throws
    d.target = node(newv, false);
    CHECK(throws_oxen([&] { rs::should_restore_batch({d}, false); }, "Could not read file for hashing"));
    // the first failing FILE's error: per file the hash comes before get_file_metadata
    // (restore.rs:334-339), so file 0's read error beats file 1's metadata error, and the other way round
    rs::RestoreCheck bad_meta;
    bad_meta.working_path = put("meta.txt", other);
    bad_meta.target = node(newv, true);
    bad_meta.file_metadata.kind = liboxen::util::fs::FileMetadataHash::Error;
    bad_meta.file_metadata.error = "metadata failed (test)";
    d.target = node(newv, true);
    CHECK(throws_oxen([&] { rs::should_restore_batch({d, bad_meta}, true); }, "Could not read file for hashing"));
    CHECK(throws_oxen([&] { rs::should_restore_batch({bad_meta, d}, true); }, "metadata failed (test)"));
    const std::string rm = std::string("rm -rf ") + dir;
    if (system(rm.c_str()) != 0) fprintf(stderr, "could not remove %s\n", dir);
}

// core::branches::classify_checkout_batch (branches.rs:653-757) against the File arm's rules spelled out here
static void checkout_checks() {
    namespace br = liboxen::core::branches;
    namespace rs = liboxen::core::restore;
    using O = br::CheckoutOutcome;
    char tmpl[] = "/tmp/oxh_checkout_XXXXXX";
    const char* dir = mkdtemp(tmpl);
    CHECK(dir != nullptr);
    if (!dir) return;
    auto put = [&](const std::string& name, const std::string& data) {
        const std::string p = std::string(dir) + "/" + name;
        if (FILE* f = fopen(p.c_str(), "wb")) {
            fwrite(data.data(), 1, data.size(), f);
            fclose(f);
        }
        return p;
    };
    auto node = [](const std::string& d) {
        rs::NodeHashes h;
        h.hash = hasher::hash_buffer_128bit(d);
        h.num_bytes = d.size();
        return h;
    };
    const std::string tgt = "target version\n", frm = "from version\n", other = "edited elsewhere\n";
    for (bool overwrite : {false, true}) {
        std::vector<br::CheckoutCheck> v;
        std::vector<O> want;
        auto add = [&](const std::string& path, const std::string* from, bool t_ok, bool f_ok, O expect) {
            br::CheckoutCheck c;
            c.working_path = path;
            c.target = node(tgt);
            if (from) c.from = node(*from);
            c.target_mtime_matched = t_ok;
            c.from_mtime_matched = f_ok;
            v.push_back(c);
            want.push_back(expect);
        };
        const std::string missing = std::string(dir) + "/missing";
        const std::string p_t = put("t.txt", tgt), p_f = put("f.txt", frm), p_o = put("o.txt", other);
        add(missing, nullptr, false, false, O::Restore);                        // new in the target
        add(missing, &tgt, false, false, O::KeepDeleted);                      // deleted, unchanged in both
        add(missing, &frm, false, false, overwrite ? O::Restore : O::Conflict);  // deleted after a change
        add(p_t, &frm, false, false, O::Skip);                                 // already the target
        add(p_f, &frm, false, false, O::Restore);                              // unchanged since from
        add(p_o, &frm, false, false, overwrite ? O::Restore : O::Conflict);    // diverged from both
        add(p_o, nullptr, false, false, overwrite ? O::Restore : O::Conflict);
        add(put("same_size_t.txt", std::string(tgt.size(), 'z')), &frm, true, false, O::Skip);  // short cuts: no read
        add(put("same_size_f.txt", std::string(frm.size(), 'z')), &frm, false, true, O::Restore);
        add(p_o + "/x", &frm, false, false, overwrite ? O::Restore : O::Conflict);  // ENOTDIR: not on disk
        CHECK(br::classify_checkout_batch(v, overwrite) == want);
    }
    br::CheckoutCheck d;
    d.working_path = dir;  // a directory: the read fails (EISDIR) and the call throws
    d.target = node(tgt);
    CHECK(throws_oxen([&] { br::classify_checkout_batch({d}, false); }, "Could not read file for hashing"));
    const std::string rm = std::string("rm -rf ") + dir;
    if (system(rm.c_str()) != 0) fprintf(stderr, "could not remove %s\n", dir);
}

// liboxen::dedup::host_entry_pays_off: INTEGRATION.md §2's routing rule (the same table as dedup.py)
static void routing_rule_checks() {
    namespace dd = liboxen::dedup;
    CHECK(!dd::host_entry_pays_off(16, 1, false));  // fixed-size: 67.2 GiB/s of cores > 49 of one link
    CHECK(dd::host_entry_pays_off(16, 1, true));    // FastCDC: 38.4 < 49
    CHECK(dd::host_entry_pays_off(8, 1, false));
    CHECK(!dd::host_entry_pays_off(128, 8, false));
    CHECK(dd::host_entry_pays_off(128, 8, true));
    CHECK(!dd::host_entry_pays_off(64, 0, true));
}

int main(int argc, char** argv) {
    const std::string golden = argc > 1 ? argv[1] : "tests/golden";
    try {
        hashing_reader_tests();
        hashing_writer_tests();
        known_answers(golden);
        file_errors(golden);
        reader_pool(golden);
        merkle_hash();
        long_stream();
        modified_check(golden);
        dedup_chunks(golden);
        restore_checks();
        checkout_checks();
        routing_rule_checks();
        char tmpl[] = "/tmp/oxh_native_XXXXXX";
        const char* scratch = mkdtemp(tmpl);
        if (!scratch) throw std::runtime_error("mkdtemp failed");
        verified_publish(scratch);
        const std::string rm = std::string("rm -rf ") + scratch;
        if (system(rm.c_str()) != 0) fprintf(stderr, "could not remove %s\n", scratch);
    } catch (const std::exception& e) {
        fprintf(stderr, "FAIL: unexpected exception: %s\n", e.what());
        ++g_fail;
    }
    printf("%d passed, %d failed\n", g_pass, g_fail);
    return g_fail ? 1 : 0;
}
