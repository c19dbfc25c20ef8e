// oxen_amd/csrc/publish.hip -- the version-store half of the fused add (oxh_add_files, _ex: the
// publisher the engine hands hashed bytes to) and the version-store fsck (oxh_clean_corrupted_versions).
// See capi_internal.hpp for the pieces.
#include <ftw.h>

#include <random>

#include "capi_internal.hpp"

using namespace oxh::capi;

namespace {

// mkdir -p (std::fs::create_dir_all)
bool mkdir_p(const std::string& dir) {
    if (mkdir(dir.c_str(), 0755) == 0 || errno == EEXIST) return true;
    if (errno != ENOENT) return false;
    for (size_t i = 1; i <= dir.size(); ++i)
        if (i == dir.size() || dir[i] == '/') {
            const std::string part = dir.substr(0, i);
            if (mkdir(part.c_str(), 0755) != 0 && errno != EEXIST) return false;
        }
    return true;
}

// A new temp file `{dir}/data.oxentmp.<random>` (AtomicTempFile's `<target_basename>.oxentmp.<random>`,
// util/fs/atomic_file.rs:21-25,58-96, so liboxen's leftover handling recognises it); -1 on failure.
int make_temp(const std::string& dir, std::string& tmp) {
    static const char an[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789";
    thread_local uint64_t x = [] {
        std::random_device rd;
        return ((uint64_t)rd() << 32) ^ rd() ^ (uint64_t)std::hash<std::thread::id>()(std::this_thread::get_id());
    }();
    for (int attempt = 0; attempt < 32; ++attempt) {
        tmp = dir + "/data.oxentmp.";
        for (int k = 0; k < 8; ++k) {  // splitmix64 steps
            uint64_t z = (x += 0x9E3779B97F4A7C15ull);
            z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
            z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
            tmp += an[(z ^ (z >> 31)) % 62];
        }
        const int fd = open(tmp.c_str(), O_RDWR | O_CREAT | O_EXCL | O_CLOEXEC, 0644);
        if (fd >= 0 || errno != EEXIST) return fd;
    }
    return -1;
}

// The version-store half of the fused add: LocalVersionStore::store_version_from_reader
// (storage/local.rs:104-121) publishing through AtomicTempFile (util/fs/atomic_file.rs:54-159) --
// write a `data.oxentmp.<random>` sibling, make the data durable, rename it to
// {root}/{hex[..2]}/{hex[2..]}/data (local.rs:66-75), make the rename durable; a blob already in the
// store is not rewritten (local.rs:112). AtomicTempFile::commit fsyncs each file and its parent; here
// one syncfs() covers every temp of a drained slot before any of them is renamed, and a second one
// covers the renames -- the same ordering, two barriers per slot instead of two per file.
// The barriers run on a committer thread: commit() hands the slot's temps over and returns, so the
// engine reads, hashes and writes the next slots while the disk takes the last ones (a committer
// that falls behind takes every queued slot under one pair of barriers). wait() returns once every
// handed-over temp is published; oxh_add_files calls it before it reads the outcomes.
// OXH_PUBLISH_INLINE=1 publishes inside commit() instead (the r02 form, for A/B).
// OXH_PUBLISH_SYNC=fsync replaces the two syncfs barriers with the reference's own per-blob steps
// (fsync the temp, rename, fsync its parent), run by the committer's threads: for filesystems where
// syncfs is costly (one shared with other tenants' dirty data).
// Identical content twice in one call is published once; every duplicate shares that publish's
// outcome (finish()).
class VersionPublisher final : public ItemSink {
   public:
    VersionPublisher(oxh_ctx* c, std::string root, uint64_t n)
        : c_(c), root_(std::move(root)), owner_(n, kNone), result_(n, 0),
          inline_(env_flag("OXH_PUBLISH_INLINE")),
          fsync_each_(getenv("OXH_PUBLISH_SYNC") && !strcmp(getenv("OXH_PUBLISH_SYNC"), "fsync")) {}
    ~VersionPublisher() override {
        {
            std::lock_guard<std::mutex> g(cq_mu_);
            quit_ = true;
        }
        cq_cv_.notify_all();
        if (committer_.joinable()) committer_.join();  // publishes whatever is still queued first
        if (trace_)
            fprintf(stderr, "[oxh] publish: put=%.3fs (thread time) publish=%.3fs batches=%d wait=%.3fs inline=%d fsync=%d\n",
                    put_s_.load() * 1e-9, publish_s_ * 1e-9, nbatches_, wait_s_ * 1e-9, (int)inline_, (int)fsync_each_);
        delete rpool_;
        if (root_fd_ >= 0) close(root_fd_);
    }

    void put(uint64_t id, const uint8_t* bytes, uint64_t len, uint64_t lo, uint64_t hi) override {
        const Clock t0(trace_);
        put_impl(id, bytes, len, lo, hi);
        put_s_.fetch_add(t0.ns(), std::memory_order_relaxed);
    }
    void put_impl(uint64_t id, const uint8_t* bytes, uint64_t len, uint64_t lo, uint64_t hi) {
        if (!claim(id, lo, hi)) return;
        std::string dir, path;
        target(lo, hi, dir, path);
        struct stat sb;
        if (stat(path.c_str(), &sb) == 0) {
            result_[id] = kExisted;
            return;
        }
        std::string tmp;
        const int fd = mkdir_p(dir) ? make_temp(dir, tmp) : -1;
        if (fd < 0) {
            result_[id] = kFailed;
            return;
        }
        bool ok = true;
        for (uint64_t done = 0; ok && done < len;) {
            const ssize_t w = write(fd, bytes + done, len - done);
            if (w <= 0) ok = false;
            else done += (uint64_t)w;
        }
        if (close(fd) != 0) ok = false;
        if (!ok) {
            unlink(tmp.c_str());
            result_[id] = kFailed;
            return;
        }
        stage(id, tmp, path);
    }

    // a streamed file's temp lives in the root until its digest names the target directory
    int open_stream(uint64_t, std::string& tmp) override { return mkdir_p(root_) ? make_temp(root_, tmp) : -1; }

    void close_stream(uint64_t id, int fd, const std::string& tmp, bool ok, uint64_t lo, uint64_t hi) override {
        if (fd >= 0 && close(fd) != 0) ok = false;
        if (!ok || fd < 0) {
            if (!tmp.empty()) unlink(tmp.c_str());
            owner_[id] = id;
            result_[id] = kFailed;
            return;
        }
        if (!claim(id, lo, hi)) {
            unlink(tmp.c_str());
            return;
        }
        std::string dir, path;
        target(lo, hi, dir, path);
        struct stat sb;
        if (stat(path.c_str(), &sb) == 0) {
            unlink(tmp.c_str());
            result_[id] = kExisted;
        } else if (!mkdir_p(dir)) {
            unlink(tmp.c_str());
            result_[id] = kFailed;
        } else {
            stage(id, tmp, path);
        }
    }

    void commit() override {
        std::vector<Staged> batch;
        {
            std::lock_guard<std::mutex> g(mu_);
            batch.swap(staged_);
        }
        if (batch.empty()) return;
        if (inline_) {
            publish(batch);
            return;
        }
        {
            std::lock_guard<std::mutex> g(cq_mu_);
            cq_.push_back(std::move(batch));
            if (!committer_.joinable()) committer_ = std::thread([this] { committer(); });
        }
        cq_cv_.notify_all();
    }

    // every temp handed to commit() so far is published (or failed)
    void wait() {
        const Clock t0(trace_);
        std::unique_lock<std::mutex> g(cq_mu_);
        cq_cv_.wait(g, [&] { return cq_.empty() && !publishing_; });
        wait_s_ += t0.ns();
    }

    // Per-item outcome into the caller's arrays: a file whose content failed to publish (its own
    // publish or the one its duplicate claimed) fails with OXH_ERR_IO and digest 0, like the
    // reference's add of that file (add.rs:533-544).
    void finish(uint64_t n, uint64_t* out, int32_t* status, int32_t* stored) const {
        for (uint64_t i = 0; i < n; ++i) {
            stored[i] = 0;
            if (status[i] != OXH_OK) continue;
            const uint64_t o = owner_[i];
            if (o == kNone || result_[o] == kFailed) {
                status[i] = OXH_ERR_IO;
                out[2 * i] = out[2 * i + 1] = 0;
                continue;
            }
            stored[i] = (o == i && result_[o] == kWritten) ? 1 : 0;
        }
    }

   private:
    static constexpr uint64_t kNone = ~0ull;
    static constexpr int8_t kExisted = 0, kWritten = 1, kFailed = -1;
    struct Staged {
        uint64_t id;
        std::string tmp, path;
    };
    struct Clock {  // OXH_TRACE: wall time of a section, 0 when tracing is off
        std::chrono::steady_clock::time_point t;
        bool on;
        explicit Clock(bool o) : on(o) {
            if (on) t = std::chrono::steady_clock::now();
        }
        uint64_t ns() const {
            return on ? (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t).count() : 0;
        }
    };
    static bool env_flag(const char* name) {
        const char* e = getenv(name);
        return e && atoi(e) != 0;
    }

    void committer() {
        std::unique_lock<std::mutex> g(cq_mu_);
        for (;;) {
            cq_cv_.wait(g, [&] { return quit_ || !cq_.empty(); });
            if (cq_.empty()) return;  // quit, nothing left
            std::vector<Staged> batch = std::move(cq_.front());
            for (size_t k = 1; k < cq_.size(); ++k)
                for (Staged& st : cq_[k]) batch.push_back(std::move(st));
            cq_.clear();
            publishing_ = true;
            g.unlock();
            publish(batch);
            g.lock();
            publishing_ = false;
            cq_cv_.notify_all();
        }
    }

    void publish(std::vector<Staged>& batch) {
        const Clock t0(trace_);
        publish_impl(batch);
        publish_s_ += t0.ns();
        ++nbatches_;
    }
    void publish_impl(std::vector<Staged>& batch) {
        // 1. the data of every temp is durable before any rename (AtomicTempFile::commit's sync_all,
        //    atomic_file.rs:122); should syncfs fail, each temp is fsynced on its own
        const bool synced = !fsync_each_ && sync_fs();
        auto each = [&](const std::function<void(Staged&)>& fn) {
            if (batch.size() < 64) {
                for (Staged& s : batch) fn(s);
                return;
            }
            if (!rpool_) rpool_ = new oxh::Pool(c_->pool->size());  // the publisher's own: wpool may be busy with put()
            const int ntasks = (int)std::min<size_t>(batch.size(), (size_t)rpool_->size() * 4);
            rpool_->parallel_for(ntasks, [&](int t) {
                for (size_t k = (size_t)t; k < batch.size(); k += (size_t)ntasks) fn(batch[k]);
            });
        };
        each([&](Staged& s) {
            bool ok = true;
            if (!synced) {
                const int fd = open(s.tmp.c_str(), O_RDONLY | O_CLOEXEC);
                ok = fd >= 0 && fsync(fd) == 0;
                if (fd >= 0) close(fd);
            }
            // 2. publish (atomic_file.rs:132-139): a failed rename removes the temp
            if (ok && rename(s.tmp.c_str(), s.path.c_str()) == 0) {
                result_[s.id] = kWritten;
                if (fsync_each_) {  // 3. the rename, best effort: the parent's fsync (:141-156)
                    const int dfd = open(s.path.substr(0, s.path.rfind('/')).c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
                    if (dfd >= 0) {
                        (void)fsync(dfd);
                        close(dfd);
                    }
                }
            } else {
                unlink(s.tmp.c_str());
                result_[s.id] = kFailed;
            }
        });
        // 3. the renames themselves, best effort like the reference's parent fsync (:141-156)
        if (!fsync_each_) (void)sync_fs();
    }

    // the first item with this digest publishes it; the others share its outcome
    bool claim(uint64_t id, uint64_t lo, uint64_t hi) {
        std::lock_guard<std::mutex> g(mu_);
        const auto it = owner_of_.emplace(std::make_pair(lo, hi), id).first;
        owner_[id] = it->second;
        return it->second == id;
    }
    void target(uint64_t lo, uint64_t hi, std::string& dir, std::string& path) const {
        char hex[40];
        const int hl = oxh_format_hex(lo, hi, hex);
        const int p = std::min(hl, 2);
        dir = root_ + "/" + std::string(hex, p) + "/" + std::string(hex + p);
        path = dir + "/data";
    }
    void stage(uint64_t id, const std::string& tmp, const std::string& path) {
        std::lock_guard<std::mutex> g(mu_);
        staged_.push_back({id, tmp, path});
    }
    bool sync_fs() {
        if (root_fd_ < 0) root_fd_ = open(root_.c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
        return root_fd_ >= 0 && syncfs(root_fd_) == 0;
    }

    oxh_ctx* c_;
    std::string root_;
    std::mutex mu_;
    std::map<std::pair<uint64_t, uint64_t>, uint64_t> owner_of_;
    std::vector<uint64_t> owner_;  // per item: the item that publishes its content (itself if first)
    std::vector<int8_t> result_;   // per publishing item: kWritten / kExisted / kFailed
    std::vector<Staged> staged_;   // temps written, waiting for commit()
    int root_fd_ = -1;             // the committer's only (syncfs)
    const bool inline_, fsync_each_;
    std::mutex cq_mu_;
    std::condition_variable cq_cv_;
    std::vector<std::vector<Staged>> cq_;  // committed slots waiting for the committer
    bool publishing_ = false, quit_ = false;
    std::thread committer_;
    oxh::Pool* rpool_ = nullptr;  // renames / fallback fsyncs
    const bool trace_ = getenv("OXH_TRACE") != nullptr;
    std::atomic<uint64_t> put_s_{0};
    uint64_t publish_s_ = 0, wait_s_ = 0;  // committer thread / owner thread
    int nbatches_ = 0;
};

}  // namespace

extern "C" {

int oxh_add_files(oxh_ctx* c, const char* const* paths, uint64_t n, const char* versions_root, uint64_t* out,
                  uint64_t* sizes, int32_t* status, int32_t* stored) {
    return oxh_add_files_ex(c, paths, n, versions_root, out, sizes, status, stored, nullptr);
}

int oxh_add_files_ex(oxh_ctx* c, const char* const* paths, uint64_t n, const char* versions_root, uint64_t* out,
                     uint64_t* sizes, int32_t* status, int32_t* stored, int32_t* os_error) {
    if (n && (!versions_root || !stored || !status)) return fail(OXH_ERR_INVALID, "versions_root/status/stored is NULL");
    for (uint64_t i = 0; i < n; ++i) stored[i] = 0;
    VersionPublisher pub(c, versions_root ? versions_root : "", n);
    const int rc = hash_files_impl(c, paths, n, out, sizes, status, nullptr, &pub, nullptr, nullptr, os_error);
    if (rc) return rc;
    pub.wait();
    pub.finish(n, out, status, stored);
    return OXH_OK;
}

static int remove_tree_cb(const char* p, const struct stat*, int, struct FTW*) { return remove(p); }

// std::fs::remove_dir_all: depth-first, does not follow symlinks.
static bool remove_dir_all(const std::string& dir) {
    return nftw(dir.c_str(), remove_tree_cb, 64, FTW_DEPTH | FTW_PHYS) == 0;
}

int oxh_clean_corrupted_versions(oxh_ctx* c, const char* versions_root, int dry_run, uint64_t* result) {
    if (!c || !versions_root || !result) return fail(OXH_ERR_INVALID, "bad arguments");
    uint64_t errors = 0, scanned = 0, corrupted = 0, cleaned = 0;
    // prefix dirs (local.rs:461-474): anything that is not a directory counts as an error
    // 1 = directory, 0 = not, -1 = file_type() failed (an error in the reference's counts)
    auto is_dir = [](const std::string& path, unsigned char d_type) {
        if (d_type != DT_UNKNOWN) return d_type == DT_DIR ? 1 : 0;  // readdir's type, like DirEntry::file_type
        struct stat sb;
        if (lstat(path.c_str(), &sb) != 0) return -1;
        return S_ISDIR(sb.st_mode) ? 1 : 0;
    };
    std::vector<std::string> prefixes;
    {
        DIR* d = opendir(versions_root);
        if (!d) return fail(OXH_ERR_IO, std::string("cannot read ") + versions_root);
        while (struct dirent* e = readdir(d)) {
            if (!strcmp(e->d_name, ".") || !strcmp(e->d_name, "..")) continue;
            if (is_dir(std::string(versions_root) + "/" + e->d_name, e->d_type) == 1)
                prefixes.push_back(e->d_name);
            else
                ++errors;
        }
        closedir(d);
    }
    std::sort(prefixes.begin(), prefixes.end());
    // suffix dirs (local.rs:480-518), one task per prefix as in the reference: non-directories are
    // skipped; expected hash = prefix + suffix
    struct Found {
        std::vector<std::string> dirs, expected;
        uint64_t errors = 0;
    };
    std::vector<Found> found(prefixes.size());
    c->pool->parallel_for((int)prefixes.size(), [&](int t) {
        const std::string pdir = std::string(versions_root) + "/" + prefixes[t];
        DIR* d = opendir(pdir.c_str());
        if (!d) {
            ++found[t].errors;
            return;
        }
        while (struct dirent* e = readdir(d)) {
            if (!strcmp(e->d_name, ".") || !strcmp(e->d_name, "..")) continue;
            std::string sdir = pdir + "/" + e->d_name;
            const int k = is_dir(sdir, e->d_type);
            if (k < 0) ++found[t].errors;
            if (k != 1) continue;
            found[t].dirs.push_back(std::move(sdir));
            found[t].expected.push_back(prefixes[t] + e->d_name);
        }
        closedir(d);
    });
    std::vector<std::string> dirs, expected, data;
    for (Found& f : found) {
        errors += f.errors;
        for (size_t k = 0; k < f.dirs.size(); ++k) {
            data.push_back(f.dirs[k] + "/data");
            dirs.push_back(std::move(f.dirs[k]));
            expected.push_back(std::move(f.expected[k]));
        }
    }
    const uint64_t n = dirs.size();
    std::vector<const char*> paths(n);
    for (uint64_t i = 0; i < n; ++i) paths[i] = data[i].c_str();
    std::vector<uint64_t> out(2 * n), sizes(n);
    std::vector<int32_t> status(n);
    const int rc = hash_files_impl(c, paths.data(), n, out.data(), sizes.data(), status.data(), nullptr);
    if (rc) return rc;
    for (uint64_t i = 0; i < n; ++i) {
        bool remove_it = false;
        if (status[i] != OXH_OK) {  // fs::read failed: an error, not scanned (local.rs:527-537)
            ++errors;
            remove_it = !dry_run;
            if (remove_it && remove_dir_all(dirs[i])) ++cleaned;
            continue;
        }
        ++scanned;
        char hex[40];
        const int hl = oxh_format_hex(out[2 * i], out[2 * i + 1], hex);
        if (expected[i].size() == (size_t)hl && memcmp(expected[i].data(), hex, hl) == 0) continue;
        ++corrupted;  // local.rs:561-581
        if (!dry_run) {
            if (remove_dir_all(dirs[i]))
                ++cleaned;
            else
                ++errors;
        }
    }
    result[0] = scanned;
    result[1] = corrupted;
    result[2] = cleaned;
    result[3] = errors;
    return OXH_OK;
}

}  // extern "C"
