// oxen_amd/host/oxen_hasher.cpp -- liboxen `util::hasher` mirror over the C ABI (see the header).
#include "oxen_hasher.hpp"

#include <dirent.h>
#include <errno.h>
#include <fcntl.h>
#include <ftw.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>

#include <chrono>
#include <cstring>
#include <random>
#include <cstdlib>
#include <mutex>
#include <thread>

#include "../../include/oxen_hash.h"
#include "commit_writer.hpp"

namespace liboxen {

namespace {

u128 to_u128(uint64_t lo, uint64_t hi) { return ((u128)hi << 64) | lo; }

[[noreturn]] void raise(int rc, const char* what) {
    const std::string msg = std::string(what) + ": " + oxh_last_error();
    throw OxenError(rc == OXH_ERR_NODEVICE ? OxenError::Kind::NoDevice : OxenError::Kind::Basic, msg, rc);
}

void check(int rc, const char* what) {
    if (rc != OXH_OK) raise(rc, what);
}

}  // namespace

MerkleHash MerkleHash::from_str(std::string_view s) {
    // u128::from_str_radix(s, 16): optional '+', at least one digit, no overflow
    if (!s.empty() && s[0] == '+') s.remove_prefix(1);
    if (s.empty()) throw OxenError::basic_str("cannot parse integer from empty string");
    u128 v = 0;
    for (char ch : s) {
        int d;
        if (ch >= '0' && ch <= '9') d = ch - '0';
        else if (ch >= 'a' && ch <= 'f') d = ch - 'a' + 10;
        else if (ch >= 'A' && ch <= 'F') d = ch - 'A' + 10;
        else throw OxenError::basic_str("invalid digit found in string");
        if (v >> 124) throw OxenError::basic_str("number too large to fit in target type");
        v = (v << 4) | (u128)d;
    }
    return MerkleHash(v);
}

std::string MerkleHash::to_string() const { return util::hasher::format_hex(v_); }

std::string MerkleHash::to_short_str() const {
    const std::string s = to_string();
    return s.size() > 10 ? s.substr(0, 10) : s;
}

void MerkleHash::to_le_bytes(uint8_t out[16]) const {
    for (int i = 0; i < 16; ++i) out[i] = (uint8_t)(v_ >> (8 * i));
}

std::string MerkleHash::node_db_prefix() const {
    const std::string s = to_string();
    return s.substr(0, 3) + "/" + (s.size() > 3 ? s.substr(3) : std::string());
}

namespace util::hasher {

oxh_ctx* default_context() {
    static std::once_flag once;
    static oxh_ctx* ctx = nullptr;
    static int rc = OXH_OK;
    static std::string err;
    std::call_once(once, [] {
        const char* dev = getenv("OXH_DEVICE");
        rc = oxh_ctx_create(dev ? atoi(dev) : 0, 0, &ctx);
        if (rc != OXH_OK) err = oxh_last_error();
    });
    if (rc != OXH_OK)
        throw OxenError(rc == OXH_ERR_NODEVICE ? OxenError::Kind::NoDevice : OxenError::Kind::Basic,
                        "oxh_ctx_create: " + err, rc);
    return ctx;
}

std::string format_hex(u128 v) {
    char buf[40];
    const int n = oxh_format_hex((uint64_t)v, (uint64_t)(v >> 64), buf);
    return std::string(buf, (size_t)n);
}

std::vector<u128> hash_buffers_128bit(const std::vector<std::string_view>& buffers, oxh_ctx* ctx) {
    ctx = ctx ? ctx : default_context();
    const size_t n = buffers.size();
    std::vector<const uint8_t*> ptrs(n);
    std::vector<uint64_t> lens(n), out(2 * n);
    for (size_t i = 0; i < n; ++i) {
        ptrs[i] = reinterpret_cast<const uint8_t*>(buffers[i].data());
        lens[i] = buffers[i].size();
    }
    check(oxh_hash_buffers(ctx, ptrs.data(), lens.data(), n, out.data()), "oxh_hash_buffers");
    std::vector<u128> r(n);
    for (size_t i = 0; i < n; ++i) r[i] = to_u128(out[2 * i], out[2 * i + 1]);
    return r;
}

u128 hash_buffer_128bit(const void* data, size_t len) {
    return hash_buffers_128bit({std::string_view(static_cast<const char*>(data), len)})[0];
}

std::string hash_buffer(const void* data, size_t len) { return format_hex(hash_buffer_128bit(data, len)); }

std::string hash_str(std::string_view s) { return hash_buffer(s.data(), s.size()); }

namespace {
// core::unicode::printable marks as non-printable every code point of general category Cc, Cf, Cs, Co,
// Cn, Zl, Zp or Zs except the space; Grapheme_Extend chars are escaped too. This table holds the
// controls, format chars, separators, surrogates, private use and noncharacters, and the combining
// blocks most file names meet; marks of other scripts and unassigned code points are not in it
// ("Error texts").
bool needs_unicode_escape(uint32_t c) {
    static const uint32_t ranges[][2] = {
        {0x0000, 0x001F}, {0x007F, 0x00A0}, {0x00AD, 0x00AD}, {0x0300, 0x036F}, {0x0483, 0x0489}, {0x0591, 0x05BD},
        {0x0600, 0x0605}, {0x0610, 0x061A}, {0x061C, 0x061C}, {0x064B, 0x065F}, {0x06DD, 0x06DD}, {0x070F, 0x070F},
        {0x1680, 0x1680}, {0x180E, 0x180E}, {0x1AB0, 0x1AFF}, {0x1DC0, 0x1DFF}, {0x2000, 0x200F}, {0x2028, 0x202F},
        {0x205F, 0x2064}, {0x2066, 0x206F}, {0x20D0, 0x20F0}, {0x3000, 0x3000}, {0x302E, 0x302F}, {0x3099, 0x309A},
        {0xD800, 0xF8FF}, {0xFE00, 0xFE0F}, {0xFE20, 0xFE2F}, {0xFEFF, 0xFEFF}, {0xFF9E, 0xFF9F}, {0xFFF0, 0xFFFB},
        {0xFFFE, 0xFFFF}, {0x1D165, 0x1D169}, {0x1D16D, 0x1D182}, {0xE0000, 0xE0FFF}, {0xF0000, 0x10FFFF},
    };
    for (const auto& r : ranges)
        if (c >= r[0] && c <= r[1]) return true;
    return false;
}

// char::escape_debug_ext of one code point, appended to o
void escape_char(std::string& o, uint32_t c, const char* utf8, size_t n, bool escape_single_quote) {
    switch (c) {
        case '"': o += "\\\""; return;
        case '\\': o += "\\\\"; return;
        case '\n': o += "\\n"; return;
        case '\r': o += "\\r"; return;
        case '\t': o += "\\t"; return;
        case '\0': o += "\\0"; return;
        case '\'':
            o += escape_single_quote ? "\\'" : "'";
            return;
        default:
            break;
    }
    if (needs_unicode_escape(c)) {
        char b[16];
        snprintf(b, sizeof b, "\\u{%x}", c);
        o += b;
    } else {
        o.append(utf8, n);
    }
}

// length of the valid UTF-8 sequence at s[i] (core::str::from_utf8's rules), 0 if it is not one
size_t utf8_seq(const std::string& s, size_t i, uint32_t& cp) {
    const unsigned char b0 = (unsigned char)s[i];
    auto cont = [&](size_t k) { return i + k < s.size() && ((unsigned char)s[i + k] & 0xC0) == 0x80; };
    if (b0 < 0x80) {
        cp = b0;
        return 1;
    }
    if (b0 >= 0xC2 && b0 <= 0xDF && cont(1)) {
        cp = ((b0 & 0x1Fu) << 6) | ((unsigned char)s[i + 1] & 0x3Fu);
        return 2;
    }
    if (b0 >= 0xE0 && b0 <= 0xEF && cont(1) && cont(2)) {
        const unsigned char b1 = (unsigned char)s[i + 1];
        if ((b0 == 0xE0 && b1 < 0xA0) || (b0 == 0xED && b1 > 0x9F)) return 0;  // overlong / surrogate
        cp = ((b0 & 0x0Fu) << 12) | ((b1 & 0x3Fu) << 6) | ((unsigned char)s[i + 2] & 0x3Fu);
        return 3;
    }
    if (b0 >= 0xF0 && b0 <= 0xF4 && cont(1) && cont(2) && cont(3)) {
        const unsigned char b1 = (unsigned char)s[i + 1];
        if ((b0 == 0xF0 && b1 < 0x90) || (b0 == 0xF4 && b1 > 0x8F)) return 0;  // overlong / above U+10FFFF
        cp = ((b0 & 0x07u) << 18) | ((b1 & 0x3Fu) << 12) | (((unsigned char)s[i + 2] & 0x3Fu) << 6) |
             ((unsigned char)s[i + 3] & 0x3Fu);
        return 4;
    }
    return 0;
}

std::string rust_debug(const std::string& s, bool path) {
    std::string o = "\"";
    for (size_t i = 0; i < s.size();) {
        uint32_t cp = 0;
        const size_t n = utf8_seq(s, i, cp);
        if (n == 0) {  // a byte outside valid UTF-8: \xNN in a Path (str values are valid UTF-8 by type)
            char b[8];
            snprintf(b, sizeof b, "\\x%02X", (unsigned char)s[i]);
            o += b;
            ++i;
            continue;
        }
        escape_char(o, cp, s.data() + i, n, path);
        i += n;
    }
    return o + "\"";
}
}  // namespace

// `{:?}` of a Rust str: double quotes, char::escape_debug's escapes except the single quote
std::string rust_str_debug(const std::string& s) { return rust_debug(s, false); }

// `{:?}` of a Rust Path on Unix (OsStr Debug -> Utf8Chunks Debug, core/src/str/lossy.rs): valid UTF-8 runs
// escaped by char::escape_debug (the single quote too), each byte of an invalid sequence as \xNN
std::string rust_path_debug(const std::string& path) { return rust_debug(path, true); }

// `{:?}` of std::io::Error::from_raw_os_error(e): Os { code, kind, message }, the kind from Rust std's
// decode_error_kind (sys/pal/unix)
std::string rust_io_error_debug(int e) {
    static const struct {
        int code;
        const char* kind;
    } kinds[] = {
        {E2BIG, "ArgumentListTooLong"}, {EADDRINUSE, "AddrInUse"}, {EADDRNOTAVAIL, "AddrNotAvailable"},
        {EBUSY, "ResourceBusy"}, {ECONNABORTED, "ConnectionAborted"}, {ECONNREFUSED, "ConnectionRefused"},
        {ECONNRESET, "ConnectionReset"}, {EDEADLK, "Deadlock"}, {EDQUOT, "FilesystemQuotaExceeded"},
        {EEXIST, "AlreadyExists"}, {EFBIG, "FileTooLarge"}, {EHOSTUNREACH, "HostUnreachable"}, {EINTR, "Interrupted"},
        {EINVAL, "InvalidInput"}, {EISDIR, "IsADirectory"}, {ELOOP, "FilesystemLoop"}, {ENOENT, "NotFound"},
        {ENOMEM, "OutOfMemory"}, {ENOSPC, "StorageFull"}, {ENOSYS, "Unsupported"}, {EMLINK, "TooManyLinks"},
        {ENAMETOOLONG, "InvalidFilename"}, {ENETDOWN, "NetworkDown"}, {ENETUNREACH, "NetworkUnreachable"},
        {ENOTCONN, "NotConnected"}, {ENOTDIR, "NotADirectory"}, {ENOTEMPTY, "DirectoryNotEmpty"}, {EPIPE, "BrokenPipe"},
        {EROFS, "ReadOnlyFilesystem"}, {ESPIPE, "NotSeekable"}, {ESTALE, "StaleNetworkFileHandle"},
        {ETIMEDOUT, "TimedOut"}, {ETXTBSY, "ExecutableFileBusy"}, {EXDEV, "CrossesDevices"}, {EINPROGRESS, "InProgress"},
        {EACCES, "PermissionDenied"}, {EPERM, "PermissionDenied"}, {EAGAIN, "WouldBlock"},
    };
    const char* kind = "Uncategorized";
    for (const auto& k : kinds)
        if (k.code == e) {
            kind = k.kind;
            break;
        }
    char buf[256];
    const char* msg = strerror_r(e, buf, sizeof buf);  // GNU: returns the text
    return "Os { code: " + std::to_string(e) + ", kind: " + kind + ", message: " + rust_str_debug(msg) + " }";
}

std::string file_error_text(const std::string& path, int status, int os_error, uint64_t size_hint) {
    if (status == OXH_ERR_OPEN) {
        const std::string p = rust_path_debug(path), err = rust_io_error_debug(os_error);
        if (size_hint >= kLargeFileBytes) return "Could not open file " + p + " due to " + err;  // hasher.rs:151-154
        return "util::hasher::hash_file_contents Could not open file " + p + " " + err;       // hasher.rs:141-145
    }
    if (status == OXH_ERR_NOMEM) return "Could not allocate the buffers to hash a large file";
    return "Could not read file for hashing";  // hasher.rs:135-139, 161-165
}

namespace {
// per-file outcomes of a hash_files-shaped call, with hasher.rs's error texts
std::vector<FileHash> file_hashes(const std::vector<std::string>& paths, const std::vector<uint64_t>& out,
                                  const std::vector<uint64_t>& sizes, const std::vector<int32_t>& status,
                                  const std::vector<int32_t>& os_error, const std::vector<uint64_t>& size_hints);
}  // namespace

std::vector<FileHash> hash_files(const std::vector<std::string>& paths, oxh_ctx* ctx) {
    ctx = ctx ? ctx : default_context();
    const size_t n = paths.size();
    std::vector<const char*> cp(n);
    for (size_t i = 0; i < n; ++i) cp[i] = paths[i].c_str();
    std::vector<uint64_t> out(2 * n), sizes(n);
    std::vector<int32_t> status(n), oserr(n);
    check(oxh_hash_files_ex(ctx, cp.data(), nullptr, n, out.data(), sizes.data(), status.data(), oserr.data(), nullptr, nullptr),
          "oxh_hash_files_ex");
    return file_hashes(paths, out, sizes, status, oserr, {});
}

ReaderPool::ReaderPool(int procs, const std::vector<int>& devices, int threads, uint64_t staging_bytes) {
    check(oxh_pool_create(devices.data(), (int)devices.size(), procs, threads, staging_bytes, &p_), "oxh_pool_create");
    procs_ = procs;
}

ReaderPool::~ReaderPool() {
    if (p_) oxh_pool_destroy(p_);
}

std::vector<FileHash> ReaderPool::hash_files(const std::vector<std::string>& paths, const std::vector<uint64_t>& meta_sizes) {
    const size_t n = paths.size();
    if (!meta_sizes.empty() && meta_sizes.size() != n) throw OxenError::basic_str("paths and meta_sizes differ in length", OXH_ERR_INVALID);
    std::vector<const char*> cp(n);
    for (size_t i = 0; i < n; ++i) cp[i] = paths[i].c_str();
    std::vector<uint64_t> out(2 * n), sizes(n);
    std::vector<int32_t> status(n), oserr(n);
    check(oxh_pool_hash_files_ex(p_, cp.data(), meta_sizes.empty() ? nullptr : meta_sizes.data(), n, out.data(), sizes.data(),
                                 status.data(), oserr.data()),
          "oxh_pool_hash_files_ex");
    return file_hashes(paths, out, sizes, status, oserr, meta_sizes);
}

namespace {
std::vector<FileHash> file_hashes(const std::vector<std::string>& paths, const std::vector<uint64_t>& out,
                                  const std::vector<uint64_t>& sizes, const std::vector<int32_t>& status,
                                  const std::vector<int32_t>& os_error, const std::vector<uint64_t>& size_hints) {
    const size_t n = paths.size();
    std::vector<FileHash> r(n);
    for (size_t i = 0; i < n; ++i) {
        r[i].code = status[i];
        if (status[i] == OXH_OK) {
            r[i].ok = true;
            r[i].hash = to_u128(out[2 * i], out[2 * i + 1]);
            r[i].size = sizes[i];
        } else {  // File::open (OXH_ERR_OPEN) or the read (OXH_ERR_IO) failed, with the errno of its io::Error
            r[i].os_error = os_error[i];
            r[i].error = file_error_text(paths[i], status[i], os_error[i], size_hints.empty() ? 0 : size_hints[i]);
        }
    }
    return r;
}
}  // namespace

namespace {
u128 hash_one_file(const std::string& path, uint64_t size_hint) {
    std::vector<FileHash> r = hash_files({path});
    if (!r[0].ok) {
        // the size picks hasher.rs's one-shot or streamed branch, and so which open message
        r[0].error = file_error_text(path, r[0].code, r[0].os_error, size_hint);
        throw OxenError::basic_str(r[0].error, r[0].code);
    }
    return r[0].hash;
}
}  // namespace

// Both size branches (one-shot below 1e9 B, 4 KiB streaming above) give the same XXH3-128; here
// both go through the batched file path (K1, or the K1L piece pipeline above a staging slot).
u128 get_hash_given_metadata(const std::string& path, const struct stat& metadata) {
    return hash_one_file(path, (uint64_t)metadata.st_size);
}

u128 u128_hash_file_contents(const std::string& path) {
    struct stat sb;
    // util::fs::metadata(path)? (hasher.rs:105) -> OxenError::file_metadata_error (util/fs.rs:593-601,
    // error.rs:1176-1182)
    if (stat(path.c_str(), &sb) != 0)
        throw OxenError::basic_str("Could not get file metadata: " + rust_path_debug(path) + " error " +
                                       rust_io_error_debug(errno),
                                   OXH_ERR_IO);
    return hash_one_file(path, (uint64_t)sb.st_size);
}

std::string hash_file_contents(const std::string& path) { return format_hex(u128_hash_file_contents(path)); }

std::string hash_file_contents_with_retry(const std::string& path, int total_retries,
                                          const std::function<void(int)>& sleep) {
    int timeout = 1, retries = 0;
    for (;;) {
        try {
            return hash_file_contents(path);
        } catch (const OxenError&) {
            retries += 1;
            timeout *= 2;
            if (sleep) sleep(timeout);
            else std::this_thread::sleep_for(std::chrono::seconds(timeout));
            if (retries > total_retries) throw;
        }
    }
}

u128 get_combined_hash(std::optional<u128> oxen_metadata_hash, u128 content_hash) {
    if (!oxen_metadata_hash) return content_hash;
    uint8_t buf[32];
    MerkleHash(content_hash).to_le_bytes(buf);
    MerkleHash(*oxen_metadata_hash).to_le_bytes(buf + 16);
    return hash_buffer_128bit(buf, sizeof buf);
}

u128 get_metadata_hash(const std::optional<std::string>& metadata_json) {
    const std::string s = metadata_json ? *metadata_json : std::string("null");
    return hash_buffer_128bit(s.data(), s.size());
}

std::optional<u128> maybe_get_metadata_hash(const std::optional<std::string>& metadata_json) {
    if (!metadata_json) return std::nullopt;
    return get_metadata_hash(metadata_json);
}

Xxh3::Xxh3(oxh_ctx* ctx) {
    check(oxh_xxh3_stream_create(ctx ? ctx : default_context(), &s_), "oxh_xxh3_stream_create");
}

Xxh3::~Xxh3() { oxh_xxh3_stream_destroy(s_); }

void Xxh3::update(const void* data, size_t len) { check(oxh_xxh3_stream_update(s_, data, len), "oxh_xxh3_stream_update"); }

u128 Xxh3::digest128() const {
    uint64_t out[2];
    check(oxh_xxh3_stream_digest(s_, out), "oxh_xxh3_stream_digest");
    return to_u128(out[0], out[1]);
}

void Xxh3::reset() { check(oxh_xxh3_stream_reset(s_), "oxh_xxh3_stream_reset"); }

}  // namespace util::hasher

namespace util::fs {

std::vector<Modified> classify_modified_batch(const std::vector<TrackedFile>& files, oxh_ctx* ctx, uint64_t* n_hashed) {
    ctx = ctx ? ctx : hasher::default_context();
    const size_t n = files.size();
    std::vector<const char*> cp(n);
    std::vector<uint64_t> sizes(n), node_bytes(n), node_hashes(2 * n), nmh(2 * n), fmh(2 * n);
    std::vector<uint8_t> mtime(n), modified(n), nmp(n), fk(n);
    std::vector<int32_t> status(n), oserr(n);
    for (size_t i = 0; i < n; ++i) {
        const TrackedFile& f = files[i];
        cp[i] = f.path.c_str();
        sizes[i] = f.size;
        node_bytes[i] = f.node_num_bytes;
        node_hashes[2 * i] = (uint64_t)f.node_hash;
        node_hashes[2 * i + 1] = (uint64_t)(f.node_hash >> 64);
        mtime[i] = f.mtime_matched ? 1 : 0;
        nmp[i] = f.node_metadata_hash.has_value();
        const u128 h = f.node_metadata_hash.value_or(0);
        nmh[2 * i] = (uint64_t)h, nmh[2 * i + 1] = (uint64_t)(h >> 64);
        fk[i] = f.file_metadata.kind;
        fmh[2 * i] = (uint64_t)f.file_metadata.hash, fmh[2 * i + 1] = (uint64_t)(f.file_metadata.hash >> 64);
    }
    uint64_t hashed = 0;
    check(oxh_files_modified_ex(ctx, cp.data(), sizes.data(), node_bytes.data(), mtime.data(), node_hashes.data(), nmp.data(),
                                nmh.data(), fk.data(), fmh.data(), n, modified.data(), status.data(), oserr.data(), &hashed),
          "oxh_files_modified_ex");
    if (n_hashed) *n_hashed = hashed;
    std::vector<Modified> r(n);
    for (size_t i = 0; i < n; ++i) {
        r[i].modified = modified[i] != 0;
        r[i].code = status[i];
        if (status[i] == OXH_ERR_META) {
            r[i].ok = false;
            r[i].error = files[i].file_metadata.error.empty() ? "could not compute file metadata" : files[i].file_metadata.error;
        } else if (status[i] != OXH_OK) {  // get_hash_given_metadata(path, metadata)? (fs.rs:1616-1618)
            r[i].ok = false;
            r[i].error = hasher::file_error_text(files[i].path, status[i], oserr[i], files[i].size);
        }
    }
    return r;
}

bool classify_modified_from_node_with_metadata(const std::string& path, uint64_t node_num_bytes, u128 node_hash,
                                               const struct stat& metadata, bool mtime_matched,
                                               std::optional<u128> node_metadata_hash, const FileMetadataHash& file_metadata) {
    TrackedFile t{path, (uint64_t)metadata.st_size, node_num_bytes, node_hash, mtime_matched, node_metadata_hash, file_metadata};
    const std::vector<Modified> r = classify_modified_batch({t});
    if (!r[0].ok) throw OxenError::basic_str(r[0].error, r[0].code);
    return r[0].modified;
}

namespace {

constexpr size_t kStreamingBufSize = 10 * 1024 * 1024;  // constants::STREAMING_BUF_SIZE (constants.rs:196)

std::string parent_of(const std::string& p) {
    const size_t k = p.find_last_of('/');
    return k == std::string::npos ? std::string() : p.substr(0, k);
}

bool mkdir_all(const std::string& dir) {  // std::fs::create_dir_all
    if (dir.empty()) return true;
    struct stat sb;
    if (stat(dir.c_str(), &sb) == 0) return S_ISDIR(sb.st_mode);
    if (!mkdir_all(parent_of(dir))) return false;
    return mkdir(dir.c_str(), 0755) == 0 || errno == EEXIST;
}

// AtomicTempFile (atomic_file.rs:54-159): `<target>.oxentmp.<random>` beside the target, unlinked
// unless committed.
class TempFile {
   public:
    explicit TempFile(const std::string& target) : target_(target) {
        const size_t slash = target.find_last_of('/');
        const std::string name = slash == std::string::npos ? target : target.substr(slash + 1);
        if (name.empty())
            throw OxenError::basic_str("Could not create file \"" + target + "\": target path has no filename component", OXH_ERR_IO);
        const std::string parent = parent_of(target);
        if (!mkdir_all(parent)) throw OxenError::basic_str("Could not create directory \"" + parent + "\"", OXH_ERR_IO);
        static const char kAlnum[] = "0123456789ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz";
        thread_local std::mt19937_64 rng{std::random_device{}()};
        for (int attempt = 0; attempt < 64; ++attempt) {
            std::string rnd(6, 'x');
            for (char& c : rnd) c = kAlnum[rng() % (sizeof(kAlnum) - 1)];
            path_ = (parent.empty() ? std::string() : parent + "/") + name + ".oxentmp." + rnd;
            fd_ = open(path_.c_str(), O_CREAT | O_EXCL | O_WRONLY | O_CLOEXEC, 0600);
            if (fd_ >= 0 || errno != EEXIST) break;
        }
        if (fd_ < 0) throw OxenError::basic_str("Could not create file \"" + path_ + "\": " + strerror(errno), OXH_ERR_IO);
    }
    ~TempFile() {
        if (fd_ >= 0) close(fd_);
        if (!committed_) unlink(path_.c_str());
    }
    TempFile(const TempFile&) = delete;
    TempFile& operator=(const TempFile&) = delete;

    void write_all(const uint8_t* p, size_t n) {
        while (n) {
            const ssize_t w = ::write(fd_, p, n);
            if (w < 0 && errno == EINTR) continue;
            if (w <= 0) throw OxenError::basic_str("Could not write file \"" + path_ + "\": " + strerror(errno), OXH_ERR_IO);
            p += w;
            n -= (size_t)w;
        }
    }
    // sync_all, rename over the target, best-effort fsync of the parent (:116-159)
    void commit() {
        if (fsync(fd_) != 0) throw OxenError::basic_str("Could not sync file \"" + path_ + "\": " + strerror(errno), OXH_ERR_IO);
        close(fd_);
        fd_ = -1;
        if (rename(path_.c_str(), target_.c_str()) != 0)
            throw OxenError::basic_str("Could not rename file from \"" + path_ + "\" to \"" + target_ + "\": " + strerror(errno),
                                       OXH_ERR_IO);
        committed_ = true;
        const std::string parent = parent_of(target_);
        const int dfd = open(parent.empty() ? "." : parent.c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
        if (dfd >= 0) {
            (void)fsync(dfd);
            close(dfd);
        }
    }

   private:
    std::string target_, path_;
    int fd_ = -1;
    bool committed_ = false;
};

OxenError hash_mismatch(const std::string& path, MerkleHash expected, MerkleHash actual) {  // error.rs:463-471
    return OxenError(OxenError::Kind::HashMismatch,
                     "Hash mismatch writing \"" + path + "\": expected " + expected.to_string() + ", got " + actual.to_string(),
                     OXH_ERR_IO);
}

}  // namespace

void AtomicFile::stream(const Reader& reader) {
    TempFile tmp(target_);
    std::optional<hasher::Xxh3> h;
    if (verify_) h.emplace(ctx_);
    std::vector<uint8_t> buf(kStreamingBufSize);
    for (;;) {
        const size_t k = reader(buf.data(), buf.size());
        if (k == 0) break;
        if (h) h->update(buf.data(), k);
        tmp.write_all(buf.data(), k);
    }
    if (h) {
        const MerkleHash actual(h->digest128());
        if (actual != expected_) throw hash_mismatch(target_, expected_, actual);  // tmp unlinked
    }
    tmp.commit();
}

void AtomicFile::write(const void* data, size_t len) {
    TempFile tmp(target_);
    tmp.write_all((const uint8_t*)data, len);
    if (verify_) {
        const MerkleHash actual(hasher::hash_buffers_128bit({std::string_view((const char*)data, len)}, ctx_)[0]);
        if (actual != expected_) throw hash_mismatch(target_, expected_, actual);
    }
    tmp.commit();
}

void AtomicFile::stream_from_paths(const std::vector<std::string>& paths) {
    TempFile tmp(target_);
    std::optional<hasher::Xxh3> h;
    if (verify_) h.emplace(ctx_);
    std::vector<uint8_t> buf(kStreamingBufSize);
    for (const std::string& path : paths) {
        const int fd = open(path.c_str(), O_RDONLY | O_CLOEXEC);
        if (fd < 0) throw OxenError::basic_str("Could not open " + path + ": " + strerror(errno), OXH_ERR_IO);
        for (;;) {
            const ssize_t k = read(fd, buf.data(), buf.size());
            if (k < 0) {
                const int e = errno;
                close(fd);
                throw OxenError::basic_str("Could not read " + path + ": " + strerror(e), OXH_ERR_IO);
            }
            if (k == 0) break;
            if (h) h->update(buf.data(), (size_t)k);
            tmp.write_all(buf.data(), (size_t)k);
        }
        close(fd);
    }
    if (h) {
        const MerkleHash actual(h->digest128());
        if (actual != expected_) throw hash_mismatch(target_, expected_, actual);
    }
    tmp.commit();
}

}  // namespace util::fs

namespace storage {

std::string LocalVersionStore::version_dir(const std::string& hash) const {
    if (hash.size() < 3) throw OxenError::basic_str("invalid version hash \"" + hash + "\"", OXH_ERR_INVALID);
    return root_ + "/" + hash.substr(0, 2) + "/" + hash.substr(2);
}

std::string LocalVersionStore::version_path(const std::string& hash) const { return version_dir(hash) + "/data"; }

bool LocalVersionStore::version_exists(const std::string& hash) const {
    struct stat sb;
    return stat(version_path(hash).c_str(), &sb) == 0;
}

void LocalVersionStore::store_version(const std::string& hash, const void* data, size_t len) const {
    if (version_exists(hash)) return;
    util::fs::AtomicFile(version_path(hash), ctx_).with_hash(MerkleHash::from_str(hash)).write(data, len);
}

void LocalVersionStore::store_version_from_reader(const std::string& hash, const util::fs::AtomicFile::Reader& reader,
                                                  uint64_t size) const {
    (void)size;  // `_size` in the reference too
    if (version_exists(hash)) return;
    const MerkleHash expected = MerkleHash::from_str(hash);
    util::fs::AtomicFile(version_path(hash), ctx_).with_hash(expected).stream(reader);
}

std::vector<std::string> LocalVersionStore::store_versions(const std::vector<std::string>& hashes,
                                                           const std::vector<std::string_view>& datas) const {
    if (hashes.size() != datas.size()) throw OxenError::basic_str("hashes and datas differ in length", OXH_ERR_INVALID);
    const std::vector<u128> got = util::hasher::hash_buffers_128bit(datas, ctx_);  // one GPU pass
    std::vector<std::string> err(hashes.size());
    for (size_t i = 0; i < hashes.size(); ++i) {
        try {
            if (version_exists(hashes[i])) continue;
            const MerkleHash expected = MerkleHash::from_str(hashes[i]);
            if (MerkleHash(got[i]) != expected) throw util::fs::hash_mismatch(version_path(hashes[i]), expected, MerkleHash(got[i]));
            util::fs::AtomicFile(version_path(hashes[i]), ctx_).write(datas[i].data(), datas[i].size());  // verified above
        } catch (const OxenError& e) {
            err[i] = e.what();
        }
    }
    return err;
}

std::string LocalVersionStore::version_chunks_dir(const std::string& hash) const { return version_dir(hash) + "/chunks"; }

std::string LocalVersionStore::version_chunk_file(const std::string& hash, uint64_t offset) const {
    return version_chunks_dir(hash) + "/" + std::to_string(offset) + "/chunk";
}

void LocalVersionStore::store_version_chunk(const std::string& hash, uint64_t offset, const void* data, size_t len) const {
    const std::string path = version_chunk_file(hash, offset);
    struct stat sb;
    if (stat(path.c_str(), &sb) == 0) return;
    util::fs::AtomicFile(path, ctx_).write(data, len);
}

std::vector<uint64_t> LocalVersionStore::list_version_chunks(const std::string& hash) const {
    const std::string dir = version_chunks_dir(hash);
    DIR* d = opendir(dir.c_str());
    if (!d) throw OxenError::basic_str("Could not read " + dir + ": " + strerror(errno), OXH_ERR_IO);
    std::vector<uint64_t> out;
    while (struct dirent* e = readdir(d)) {
        // name.parse::<u64>(): an optional '+' then ASCII digits, below 2^64
        const std::string name = e->d_name;
        const std::string digits = !name.empty() && name[0] == '+' ? name.substr(1) : name;
        if (digits.empty() || digits.find_first_not_of("0123456789") != std::string::npos) continue;
        struct stat sb;  // DirEntry::file_type(): the entry itself, a symlink is not a directory
        if (lstat((dir + "/" + name).c_str(), &sb) != 0 || !S_ISDIR(sb.st_mode)) continue;
        errno = 0;
        const unsigned long long v = strtoull(digits.c_str(), nullptr, 10);
        if (errno == 0) out.push_back(v);
    }
    closedir(d);
    std::sort(out.begin(), out.end());
    return out;
}

void LocalVersionStore::combine_version_chunks(const std::string& hash) const {
    const MerkleHash expected = MerkleHash::from_str(hash);
    std::vector<std::string> paths;
    for (uint64_t off : list_version_chunks(hash)) paths.push_back(version_chunk_file(hash, off));
    util::fs::AtomicFile(version_path(hash), ctx_).with_hash(expected).stream_from_paths(paths);
    const std::string dir = version_chunks_dir(hash);
    if (nftw(dir.c_str(), [](const char* p, const struct stat*, int, struct FTW*) { return remove(p); }, 16,
             FTW_DEPTH | FTW_PHYS) != 0)
        throw OxenError::basic_str("Could not remove " + dir + ": " + strerror(errno), OXH_ERR_IO);
}

}  // namespace storage
namespace dedup {
namespace {
std::vector<std::vector<Chunk>> split(const std::vector<uint64_t>& first, const std::vector<uint64_t>& off,
                                      const std::vector<uint64_t>& len, const std::vector<uint64_t>& dig) {
    std::vector<std::vector<Chunk>> r(first.size() - 1);
    for (size_t i = 0; i + 1 < first.size(); ++i)
        for (uint64_t k = first[i]; k < first[i + 1]; ++k) r[i].push_back({off[k], len[k], to_u128(dig[2 * k], dig[2 * k + 1])});
    return r;
}
}  // namespace

std::vector<ChunkedFile> fastcdc_files(const std::vector<std::string>& paths, uint32_t min_size, uint32_t avg_size,
                                       uint32_t max_size, oxh_ctx* ctx) {
    return fastcdc_files(paths, min_size, avg_size, max_size, std::vector<oxh_ctx*>{ctx ? ctx : util::hasher::default_context()});
}

std::vector<ChunkedFile> fastcdc_files(const std::vector<std::string>& paths, uint32_t min_size, uint32_t avg_size,
                                       uint32_t max_size, const std::vector<oxh_ctx*>& ctxs) {
    if (ctxs.empty()) throw OxenError::basic_str("no contexts", OXH_ERR_INVALID);
    const size_t n = paths.size();
    std::vector<const char*> cp(n);
    std::vector<uint64_t> sz(n, 0);
    for (size_t i = 0; i < n; ++i) {
        cp[i] = paths[i].c_str();
        struct stat sb;
        if (stat(cp[i], &sb) == 0) sz[i] = (uint64_t)sb.st_size;
    }
    uint64_t cap = std::max<uint64_t>(1, oxh_fastcdc_max_chunks(sz.data(), n, min_size));
    for (int attempt = 0;; ++attempt) {
        std::vector<uint64_t> off(cap), len(cap), dig(2 * cap), first(n + 1), sizes(n);
        std::vector<int32_t> status(n), oserr(n);
        const int rc = ctxs.size() == 1
                           ? oxh_fastcdc_files(ctxs[0], cp.data(), n, min_size, avg_size, max_size, 1, off.data(), len.data(),
                                               dig.data(), cap, first.data(), sizes.data(), status.data(), oserr.data())
                           : oxh_fastcdc_files_multi(ctxs.data(), (int)ctxs.size(), cp.data(), n, min_size, avg_size, max_size,
                                                     1, off.data(), len.data(), dig.data(), cap, first.data(), sizes.data(),
                                                     status.data(), oserr.data());
        if (rc == OXH_ERR_INVALID && attempt < 2) {  // a file grew since the stat: the text has the count
            const std::string e = oxh_last_error();
            const size_t at = e.find("need ");
            if (at != std::string::npos) {
                cap = std::stoull(e.substr(at + 5));
                continue;
            }
        }
        if (rc != OXH_OK) throw OxenError::basic_str(std::string("oxh_fastcdc_files: ") + oxh_last_error(), rc);
        std::vector<std::vector<Chunk>> per = split(first, off, len, dig);
        std::vector<ChunkedFile> r(n);
        for (size_t i = 0; i < n; ++i) {
            r[i].ok = status[i] == OXH_OK;
            r[i].size = sizes[i];
            r[i].code = status[i];
            r[i].os_error = oserr[i];
            r[i].chunks = std::move(per[i]);
        }
        return r;
    }
}

std::vector<std::vector<Chunk>> fastcdc_buffers(const std::vector<std::string_view>& buffers, uint32_t min_size,
                                                uint32_t avg_size, uint32_t max_size, oxh_ctx* ctx) {
    return fastcdc_buffers(buffers, min_size, avg_size, max_size,
                           std::vector<oxh_ctx*>{ctx ? ctx : util::hasher::default_context()});
}

std::vector<std::vector<Chunk>> fastcdc_buffers(const std::vector<std::string_view>& buffers, uint32_t min_size,
                                                uint32_t avg_size, uint32_t max_size, const std::vector<oxh_ctx*>& ctxs) {
    if (ctxs.empty()) throw OxenError::basic_str("no contexts", OXH_ERR_INVALID);
    const size_t n = buffers.size();
    std::vector<const uint8_t*> ptrs(n);
    std::vector<uint64_t> lens(n);
    for (size_t i = 0; i < n; ++i) {
        ptrs[i] = reinterpret_cast<const uint8_t*>(buffers[i].data());
        lens[i] = buffers[i].size();
    }
    const uint64_t cap = std::max<uint64_t>(1, oxh_fastcdc_max_chunks(lens.data(), n, min_size));
    std::vector<uint64_t> off(cap), len(cap), dig(2 * cap), first(n + 1);
    if (ctxs.size() == 1)
        check(oxh_fastcdc_host(ctxs[0], ptrs.data(), lens.data(), n, min_size, avg_size, max_size, 1, off.data(),
                               len.data(), dig.data(), cap, first.data()),
              "oxh_fastcdc_host");
    else
        check(oxh_fastcdc_host_multi(ctxs.data(), (int)ctxs.size(), ptrs.data(), lens.data(), n, min_size, avg_size,
                                     max_size, 1, off.data(), len.data(), dig.data(), cap, first.data()),
              "oxh_fastcdc_host_multi");
    return split(first, off, len, dig);
}

std::vector<ChunkedFile> fixed_chunk_files(const std::vector<std::string>& paths, uint64_t chunk_size, oxh_ctx* ctx) {
    return fixed_chunk_files(paths, chunk_size, std::vector<oxh_ctx*>{ctx ? ctx : util::hasher::default_context()});
}

std::vector<ChunkedFile> fixed_chunk_files(const std::vector<std::string>& paths, uint64_t chunk_size,
                                           const std::vector<oxh_ctx*>& ctxs) {
    if (ctxs.empty()) throw OxenError::basic_str("no contexts", OXH_ERR_INVALID);
    const size_t n = paths.size();
    std::vector<const char*> cp(n);
    uint64_t cap = 1;
    for (size_t i = 0; i < n; ++i) {
        cp[i] = paths[i].c_str();
        struct stat sb;
        if (chunk_size && stat(cp[i], &sb) == 0) cap += ((uint64_t)sb.st_size + chunk_size - 1) / chunk_size;
    }
    for (int attempt = 0;; ++attempt) {
        std::vector<uint64_t> dig(2 * cap), first(n + 1), sizes(n);
        std::vector<int32_t> status(n), oserr(n);
        const int rc = ctxs.size() == 1
                           ? oxh_chunk_digests_files(ctxs[0], cp.data(), n, chunk_size, dig.data(), cap, first.data(),
                                                     sizes.data(), status.data(), oserr.data())
                           : oxh_chunk_digests_files_multi(ctxs.data(), (int)ctxs.size(), cp.data(), n, chunk_size, dig.data(),
                                                           cap, first.data(), sizes.data(), status.data(), oserr.data());
        if (rc == OXH_ERR_INVALID && attempt < 2) {  // a file grew since the stat: the text has the count
            const std::string e = oxh_last_error();
            const size_t at = e.find("need ");
            if (at != std::string::npos) {
                cap = std::stoull(e.substr(at + 5));
                continue;
            }
        }
        if (rc != OXH_OK) throw OxenError::basic_str(std::string("oxh_chunk_digests_files: ") + oxh_last_error(), rc);
        std::vector<ChunkedFile> r(n);
        for (size_t i = 0; i < n; ++i) {
            r[i].ok = status[i] == OXH_OK;
            r[i].size = sizes[i];
            r[i].code = status[i];
            r[i].os_error = oserr[i];
            for (uint64_t k = first[i], o = 0; k < first[i + 1]; ++k, o += chunk_size)
                r[i].chunks.push_back({o, std::min(chunk_size, sizes[i] - o), to_u128(dig[2 * k], dig[2 * k + 1])});
        }
        return r;
    }
}

std::vector<std::vector<Chunk>> fixed_chunk_buffers(const std::vector<std::string_view>& buffers, uint64_t chunk_size,
                                                    oxh_ctx* ctx) {
    return fixed_chunk_buffers(buffers, chunk_size, std::vector<oxh_ctx*>{ctx ? ctx : util::hasher::default_context()});
}

std::vector<std::vector<Chunk>> fixed_chunk_buffers(const std::vector<std::string_view>& buffers, uint64_t chunk_size,
                                                    const std::vector<oxh_ctx*>& ctxs) {
    if (ctxs.empty()) throw OxenError::basic_str("no contexts", OXH_ERR_INVALID);
    const size_t n = buffers.size();
    std::vector<const uint8_t*> ptrs(n);
    std::vector<uint64_t> lens(n);
    uint64_t cap = 1;
    for (size_t i = 0; i < n; ++i) {
        ptrs[i] = reinterpret_cast<const uint8_t*>(buffers[i].data());
        lens[i] = buffers[i].size();
        if (chunk_size) cap += (lens[i] + chunk_size - 1) / chunk_size;
    }
    std::vector<uint64_t> dig(2 * cap), first(n + 1);
    if (ctxs.size() == 1)
        check(oxh_chunk_digests_host(ctxs[0], ptrs.data(), lens.data(), n, chunk_size, dig.data(), cap, first.data()),
              "oxh_chunk_digests_host");
    else
        check(oxh_chunk_digests_host_multi(ctxs.data(), (int)ctxs.size(), ptrs.data(), lens.data(), n, chunk_size,
                                           dig.data(), cap, first.data()),
              "oxh_chunk_digests_host_multi");
    std::vector<std::vector<Chunk>> r(n);
    for (size_t i = 0; i < n; ++i)
        for (uint64_t k = first[i], o = 0; k < first[i + 1]; ++k, o += chunk_size)
            r[i].push_back({o, std::min(chunk_size, lens[i] - o), to_u128(dig[2 * k], dig[2 * k + 1])});
    return r;
}

bool host_entry_pays_off(unsigned host_cores, unsigned links, bool fastcdc) {
    const double cpu = host_cores * (fastcdc ? 2.4 : 4.2), gpu = links * 49.0;  // GiB/s
    return gpu > cpu;
}

std::string chunk_name(u128 hash) {
    char b[48];
    oxh_format_dec((uint64_t)hash, (uint64_t)(hash >> 64), b);
    return b;
}
}  // namespace dedup

namespace core::restore {
std::vector<bool> should_restore_batch(const std::vector<RestoreCheck>& files, bool combined, oxh_ctx* ctx) {
    ctx = ctx ? ctx : util::hasher::default_context();
    const size_t n = files.size();
    std::vector<bool> out(n, true);
    std::vector<size_t> need;
    for (size_t i = 0; i < n; ++i) {
        const RestoreCheck& f = files[i];
        struct stat sb;
        // working_path.exists() is fs::metadata(..).is_ok(): any stat failure (ENOENT, ENOTDIR, EACCES on a
        // parent, ELOOP ...) reads as "does not exist" -> restore; the reference's metadata(..)? after it
        // fails only if the file changes between the two calls
        if (stat(f.working_path.c_str(), &sb) != 0) continue;
        const NodeHashes& ref = f.base ? *f.base : f.target;
        if (f.mtime_matched && (uint64_t)sb.st_size == ref.num_bytes) continue;
        need.push_back(i);  // (a metadata Error is raised after this file's hash, below, as restore.rs:334-339)
    }
    if (need.empty()) return out;
    const size_t m = need.size();
    std::vector<const char*> cp(m);
    for (size_t j = 0; j < m; ++j) cp[j] = files[need[j]].working_path.c_str();
    std::vector<uint64_t> dig(2 * m), sizes(m), counts(2 * m);
    std::vector<int32_t> status(m), oserr(m);
    check(oxh_hash_files_ex(ctx, cp.data(), nullptr, m, dig.data(), sizes.data(), status.data(), oserr.data(),
                            combined ? counts.data() : nullptr, nullptr),
          "oxh_hash_files_ex");
    // per file in order: u128_hash_file_contents(&working_path)?, then (combined) get_file_metadata(..)?
    // (restore.rs:334-339 / :377-382) -- the first failing file's first failure is the error
    for (size_t j = 0; j < m; ++j) {
        const RestoreCheck& f = files[need[j]];
        if (status[j] != OXH_OK)
            throw OxenError::basic_str(util::hasher::file_error_text(f.working_path, status[j], oserr[j], sizes[j]), status[j]);
        if (combined && f.file_metadata.kind == util::fs::FileMetadataHash::Error)
            throw OxenError::basic_str(f.file_metadata.error.empty() ? "could not compute file metadata" : f.file_metadata.error,
                                       OXH_ERR_META);
    }
    std::vector<u128> h(m);
    for (size_t j = 0; j < m; ++j) h[j] = to_u128(dig[2 * j], dig[2 * j + 1]);
    if (combined) {  // maybe_get_metadata_hash + get_combined_hash (hasher.rs:67-100), batched
        std::string arena;
        std::vector<uint64_t> offs, lens;
        std::vector<size_t> text;
        for (size_t j = 0; j < m; ++j)
            if (files[need[j]].file_metadata.kind == util::fs::FileMetadataHash::Text) {
                const std::string js = "{\"text\":{\"num_lines\":" + std::to_string(counts[2 * j]) + ",\"num_chars\":" +
                                       std::to_string(counts[2 * j + 1]) + "}}";
                offs.push_back(arena.size()), lens.push_back(js.size()), arena += js, text.push_back(j);
            }
        const std::vector<u128> th = commit_writer::hash_streams(arena, offs, lens, ctx);
        std::vector<std::optional<u128>> mh(m);
        for (size_t t = 0; t < text.size(); ++t) mh[text[t]] = th[t];
        for (size_t j = 0; j < m; ++j)
            if (files[need[j]].file_metadata.kind == util::fs::FileMetadataHash::Given) mh[j] = files[need[j]].file_metadata.hash;
        arena.clear(), offs.clear(), lens.clear();
        std::vector<size_t> with;
        for (size_t j = 0; j < m; ++j)
            if (mh[j]) {
                uint8_t b[32];
                for (int k = 0; k < 16; ++k) b[k] = (uint8_t)(h[j] >> (8 * k)), b[16 + k] = (uint8_t)(*mh[j] >> (8 * k));
                offs.push_back(arena.size()), lens.push_back(32), arena.append(reinterpret_cast<char*>(b), 32), with.push_back(j);
            }
        const std::vector<u128> ch = commit_writer::hash_streams(arena, offs, lens, ctx);
        for (size_t t = 0; t < with.size(); ++t) h[with[t]] = ch[t];
    }
    for (size_t j = 0; j < m; ++j) {
        const RestoreCheck& f = files[need[j]];
        const u128 want = combined ? f.target.combined_hash : f.target.hash;
        if (f.base)
            out[need[j]] = h[j] == want || h[j] == (combined ? f.base->combined_hash : f.base->hash);
        else
            out[need[j]] = h[j] == want;
    }
    return out;
}
}  // namespace core::restore

namespace core::branches {
std::vector<CheckoutOutcome> classify_checkout_batch(const std::vector<CheckoutCheck>& files, bool overwrite, oxh_ctx* ctx) {
    ctx = ctx ? ctx : util::hasher::default_context();
    const size_t n = files.size();
    std::vector<CheckoutOutcome> out(n, CheckoutOutcome::Restore);
    std::vector<size_t> need;
    std::vector<uint64_t> meta_sizes;
    for (size_t i = 0; i < n; ++i) {
        const CheckoutCheck& f = files[i];
        struct stat sb;
        // full_path.exists() is fs::metadata(..).is_ok(): a failing stat reads as "not on disk"
        if (stat(f.working_path.c_str(), &sb) != 0) {
            if (f.from && f.from->hash == f.target.hash)
                out[i] = CheckoutOutcome::KeepDeleted;  // branches.rs:664-667
            else if (f.from && !overwrite)
                out[i] = CheckoutOutcome::Conflict;     // :668-673
            else
                out[i] = CheckoutOutcome::Restore;      // :678-686
            continue;
        }
        const uint64_t size = (uint64_t)sb.st_size;
        if (f.target_mtime_matched && size == f.target.num_bytes) {
            out[i] = CheckoutOutcome::Skip;  // :703-705
            continue;
        }
        if (f.from && f.from_mtime_matched && size == f.from->num_bytes) {
            out[i] = CheckoutOutcome::Restore;  // :709-723
            continue;
        }
        need.push_back(i);
        meta_sizes.push_back(size);
    }
    if (need.empty()) return out;
    const size_t m = need.size();
    std::vector<const char*> cp(m);
    for (size_t j = 0; j < m; ++j) cp[j] = files[need[j]].working_path.c_str();
    std::vector<uint64_t> dig(2 * m), sizes(m);
    std::vector<int32_t> status(m), oserr(m);
    check(oxh_hash_files_ex(ctx, cp.data(), meta_sizes.data(), m, dig.data(), sizes.data(), status.data(), oserr.data(),
                            nullptr, nullptr),
          "oxh_hash_files_ex");
    for (size_t j = 0; j < m; ++j)  // get_hash_given_metadata(&full_path, &meta)? -- the first failure in order
        if (status[j] != OXH_OK)
            throw OxenError::basic_str(util::hasher::file_error_text(files[need[j]].working_path, status[j], oserr[j],
                                                                     meta_sizes[j]),
                                       status[j]);
    for (size_t j = 0; j < m; ++j) {  // :726-756
        const CheckoutCheck& f = files[need[j]];
        const u128 h = to_u128(dig[2 * j], dig[2 * j + 1]);
        if (h == f.target.hash)
            out[need[j]] = CheckoutOutcome::Skip;
        else if (f.from && h == f.from->hash)
            out[need[j]] = CheckoutOutcome::Restore;
        else
            out[need[j]] = overwrite ? CheckoutOutcome::Restore : CheckoutOutcome::Conflict;
    }
    return out;
}
}  // namespace core::branches

namespace multigpu {
std::vector<uint8_t> DigestGather::unique_id() {
    std::vector<uint8_t> id(OXH_COMM_ID_BYTES);
    check(oxh_comm_unique_id(id.data()), "oxh_comm_unique_id");
    return id;
}
DigestGather::DigestGather(const std::vector<uint8_t>& id, int rank, int nranks, int device) {
    if (id.size() != OXH_COMM_ID_BYTES) throw OxenError::basic_str("a comm id is OXH_COMM_ID_BYTES bytes", OXH_ERR_INVALID);
    check(oxh_comm_create(id.data(), rank, nranks, device, &c_), "oxh_comm_create");
}
DigestGather::~DigestGather() { (void)oxh_comm_destroy(c_); }
void DigestGather::gather(const uint64_t* d_local, const std::vector<uint64_t>& counts, uint64_t* d_full, int root,
                          void* stream) const {
    check(oxh_gather_digests(c_, d_local, counts.data(), d_full, root, stream), "oxh_gather_digests");
}
}  // namespace multigpu
}  // namespace liboxen
