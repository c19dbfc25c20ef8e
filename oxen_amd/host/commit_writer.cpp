// oxen_amd/host/commit_writer.cpp -- the K2 commit driver (see commit_writer.hpp).
#include "commit_writer.hpp"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <map>
#include <random>
#include <thread>

#include "../../include/oxen_hash.h"

namespace liboxen::commit_writer {

namespace {

void put_le(std::string& s, u128 v) {
    char b[16];
    for (int i = 0; i < 16; ++i) b[i] = (char)(uint8_t)(v >> (8 * i));
    s.append(b, 16);
}

std::string join(const std::vector<std::string>& c, size_t n) {
    std::string r;
    for (size_t i = 0; i < n; ++i) {
        if (i) r += '/';
        r += c[i];
    }
    return r;
}

// Path's Ord on a normalised path (components joined by '/') is component-wise: bytewise with '/'
// below every other byte (a component that ends first sorts first). With '/' mapped to '\0' the plain
// (memcmp) string order is that order; paths hold no NUL.
std::string sort_key(std::string k) {
    std::replace(k.begin(), k.end(), '/', '\0');
    return k;
}

// fn(i) for i in [0, n), split over up to 16 threads in contiguous blocks (each dir is independent)
template <class F>
void parallel_for(size_t n, F&& fn) {
    const size_t hw = std::max<size_t>(1, std::min<size_t>(16, std::thread::hardware_concurrency()));
    const size_t nt = std::min(hw, n / 64 + 1);
    if (nt <= 1) {
        for (size_t i = 0; i < n; ++i) fn(i);
        return;
    }
    std::vector<std::thread> pool;
    std::vector<std::exception_ptr> err(nt);
    for (size_t t = 0; t < nt; ++t)
        pool.emplace_back([&, t] {
            try {
                for (size_t i = n * t / nt; i < n * (t + 1) / nt; ++i) fn(i);
            } catch (...) {
                err[t] = std::current_exception();  // rethrown in the caller (e.g. std::bad_alloc)
            }
        });
    for (auto& th : pool) th.join();
    for (auto& e : err)
        if (e) std::rethrow_exception(e);
}

// OXH_TRACE=1: wall time of each driver stage on stderr
struct StageClock {
    const bool on = std::getenv("OXH_TRACE") != nullptr;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void mark(const char* what) {
        if (!on) return;
        const auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[commit] %-16s %.4fs\n", what, std::chrono::duration<double>(now - t).count());
        t = now;
    }
};

}  // namespace

void uuid_v4_salt(const std::string&, size_t, uint8_t out[16]) {
    static thread_local std::random_device rd;
    for (int i = 0; i < 16; i += 4) {
        const uint32_t r = rd();
        for (int k = 0; k < 4; ++k) out[i + k] = (uint8_t)(r >> (8 * k));
    }
    out[6] = (uint8_t)((out[6] & 0x0F) | 0x40);  // version 4
    out[8] = (uint8_t)((out[8] & 0x3F) | 0x80);  // RFC 4122 variant
}

std::vector<std::string> path_components(const std::string& p) {
    std::vector<std::string> c;
    size_t i = 0;
    while (i <= p.size()) {
        const size_t j = std::min(p.find('/', i), p.size());
        if (j > i && !(j == i + 1 && p[i] == '.')) c.emplace_back(p, i, j - i);
        i = j + 1;
    }
    return c;
}

std::string normalize(const std::string& p) {
    // fast path: already normalised (no empty or "." component)
    bool plain = !p.empty() && p.front() != '/' && p.back() != '/';
    for (size_t i = 0; plain && i < p.size(); ++i)
        if ((p[i] == '/' && i + 1 < p.size() && p[i + 1] == '/') ||
            (p[i] == '.' && (i == 0 || p[i - 1] == '/') && (i + 1 == p.size() || p[i + 1] == '/')))
            plain = false;
    if (plain) return p;
    const std::vector<std::string> c = path_components(p);
    return join(c, c.size());
}

uint64_t num_vnodes(uint64_t total_children, uint64_t vnode_size) {
    return (uint64_t)std::ceil((float)total_children / (float)vnode_size);
}

std::vector<u128> hash_streams(const std::string& arena, const std::vector<uint64_t>& offsets,
                               const std::vector<uint64_t>& lens, oxh_ctx* ctx) {
    const size_t n = lens.size();
    if (n == 0) return {};
    ctx = ctx ? ctx : util::hasher::default_context();
    static const uint8_t empty = 0;
    std::vector<uint64_t> out(2 * n);
    const int rc = oxh_hash_streams(ctx, arena.empty() ? &empty : reinterpret_cast<const uint8_t*>(arena.data()),
                                    offsets.data(), lens.data(), n, out.data());
    if (rc != OXH_OK)
        throw OxenError(rc == OXH_ERR_NODEVICE ? OxenError::Kind::NoDevice : OxenError::Kind::Basic,
                        std::string("oxh_hash_streams: ") + oxh_last_error(), rc);
    std::vector<u128> r(n);
    for (size_t i = 0; i < n; ++i) r[i] = ((u128)out[2 * i + 1] << 64) | out[2 * i];
    return r;
}

std::vector<DirVNodes> split_into_vnodes(const StagedDirs& entries, const ExistingDirs& existing, uint64_t vnode_size,
                                         const SaltFn& salt, oxh_ctx* ctx) {
    if (vnode_size == 0) throw OxenError::basic_str("vnode_size must be positive");
    // the child set of every staged dir (:561-638): HEAD's children, then the staged changes (a
    // removal drops the child), keyed by the normalised path. Only the last operation on a path
    // counts, so each dir's operations are sorted by (Path's Ord, arrival) and the last one of every
    // path kept: the surviving children come out in path order with one sort and no hash map.
    struct Op {
        std::string key;  // sort_key of the normalised (possibly prefixed) path
        const StagedNode* src;
        bool put, prefixed;
    };
    struct Dir {
        std::vector<StagedNode> live;  // surviving children in path order
        std::vector<StagedNode> removed;
    };
    StageClock clk;
    std::vector<Dir> dirs(entries.size());
    parallel_for(entries.size(), [&](size_t i) {
        const std::string& directory = entries[i].first;
        const std::vector<std::string> dcomps = path_components(directory);
        const std::string dkey = join(dcomps, dcomps.size());
        Dir& d = dirs[i];
        const auto ex = existing.find(directory);
        std::vector<Op> ops;
        ops.reserve(entries[i].second.size() + (ex != existing.end() ? ex->second.size() : 0));
        if (ex != existing.end())
            for (const StagedNode& c : ex->second) ops.push_back({sort_key(normalize(c.path)), &c, true, false});
        std::unordered_map<std::string, size_t> removed_at;  // a later removal of a path replaces it
        for (const StagedNode& c : entries[i].second) {
            std::string ckey = normalize(c.path);
            if (ckey.empty()) continue;  // child_path != "" (:589)
            bool prefixed = false;
            if (!dkey.empty() && !(ckey.size() > dkey.size() && ckey.compare(0, dkey.size(), dkey) == 0 &&
                                   ckey[dkey.size()] == '/') && ckey != dkey) {  // defensive prefixing (:591-612)
                ckey = dkey + "/" + ckey;
                prefixed = true;
            }
            const bool put = c.status != StagedStatus::Removed;
            if (!put) {
                StagedNode r = c;
                if (prefixed) {
                    r.path = ckey;
                    r.name = ckey;
                }
                auto [it, fresh] = removed_at.emplace(ckey, d.removed.size());
                if (fresh) d.removed.push_back(std::move(r));
                else d.removed[it->second] = std::move(r);
            }
            ops.push_back({sort_key(std::move(ckey)), &c, put, prefixed});
        }
        std::stable_sort(ops.begin(), ops.end(), [](const Op& x, const Op& y) { return x.key < y.key; });
        d.live.reserve(ops.size());
        for (size_t k = 0; k < ops.size(); ++k) {
            if ((k + 1 < ops.size() && ops[k + 1].key == ops[k].key) || !ops[k].put) continue;
            d.live.push_back(*ops[k].src);
            if (ops[k].prefixed) {
                std::string p = std::move(ops[k].key);
                std::replace(p.begin(), p.end(), '\0', '/');
                d.live.back().name = p;
                d.live.back().path = std::move(p);
            }
        }
    });
    clk.mark("child sets");
    // bucket = xxh3_128(path) % num_vnodes (:665-681): every child of every dir in one pass; each
    // dir writes its own slice of the stream arena
    const size_t nd = dirs.size();
    std::vector<size_t> first(nd + 1, 0), at(nd + 1, 0);
    parallel_for(nd, [&](size_t i) {
        for (const StagedNode& c : dirs[i].live) at[i + 1] += c.path.size();
    });
    for (size_t i = 0; i < nd; ++i) {
        first[i + 1] = first[i] + dirs[i].live.size();
        at[i + 1] += at[i];
    }
    std::string arena(at[nd], '\0');
    std::vector<uint64_t> offs(first[nd]), lens(first[nd]);
    parallel_for(nd, [&](size_t i) {
        size_t o = at[i], q = first[i];
        for (const StagedNode& c : dirs[i].live) {
            offs[q] = o;
            lens[q++] = c.path.size();
            std::memcpy(&arena[o], c.path.data(), c.path.size());
            o += c.path.size();
        }
    });
    clk.mark("bucket streams");
    const std::vector<u128> buckets = hash_streams(arena, offs, lens, ctx);
    clk.mark("bucket hash");
    std::vector<DirVNodes> out(nd);
    std::vector<size_t> vfirst(nd + 1, 0);
    parallel_for(nd, [&](size_t i) {
        out[i].dir = entries[i].first;
        out[i].removed = std::move(dirs[i].removed);
        const uint64_t nv = num_vnodes(dirs[i].live.size(), vnode_size);
        out[i].vnodes.resize(nv);
        vfirst[i + 1] = nv;
        std::vector<uint32_t> b(dirs[i].live.size());
        std::vector<size_t> per(nv, 0);
        for (size_t q = 0; q < b.size(); ++q) ++per[b[q] = (uint32_t)(buckets[first[i] + q] % nv)];
        for (uint64_t j = 0; j < nv; ++j) out[i].vnodes[j].entries.reserve(per[j]);
        // path order in, so every vnode's entries come out sorted (:684-694)
        for (size_t q = 0; q < b.size(); ++q) out[i].vnodes[b[q]].entries.push_back(std::move(dirs[i].live[q]));
    });
    for (size_t i = 0; i < nd; ++i) vfirst[i + 1] += vfirst[i];
    clk.mark("vnode fill");
    // vnode id = xxh3("vnode" || dir || child hashes LE [|| uuid]) (:683-720): every vnode in one
    // pass. Stream sizes first (a vnode of a dir HEAD holds is salted when one of its entries
    // changed, :713-716), then every dir fills its slice; the salts are drawn afterwards, on this
    // thread, in vnode order.
    const size_t nvn = vfirst[nd];
    std::vector<char> salted(nvn, 0);
    offs.assign(nvn + 1, 0);
    lens.assign(nvn, 0);
    parallel_for(nd, [&](size_t i) {
        const DirVNodes& d = out[i];
        const bool dir_existed = existing.count(d.dir) != 0;
        for (size_t j = 0; j < d.vnodes.size(); ++j) {
            bool changed = false;
            for (const StagedNode& c : d.vnodes[j].entries) changed = changed || c.status != StagedStatus::Unmodified;
            salted[vfirst[i] + j] = dir_existed && changed;
            lens[vfirst[i] + j] = 5 + d.dir.size() + 16 * d.vnodes[j].entries.size() + (salted[vfirst[i] + j] ? 16 : 0);
        }
    });
    for (size_t v = 0; v < nvn; ++v) offs[v + 1] = offs[v] + lens[v];
    arena.assign(offs[nvn], '\0');
    offs.pop_back();
    parallel_for(nd, [&](size_t i) {
        const DirVNodes& d = out[i];
        for (size_t j = 0; j < d.vnodes.size(); ++j) {
            char* p = &arena[offs[vfirst[i] + j]];
            std::memcpy(p, "vnode", 5);
            std::memcpy(p + 5, d.dir.data(), d.dir.size());
            p += 5 + d.dir.size();
            for (const StagedNode& c : d.vnodes[j].entries) {
                for (int b = 0; b < 16; ++b) p[b] = (char)(uint8_t)(c.hash >> (8 * b));
                p += 16;
            }
        }
    });
    for (size_t i = 0; i < nd; ++i)
        for (size_t j = 0; j < out[i].vnodes.size(); ++j)
            if (salted[vfirst[i] + j]) {
                uint8_t s16[16];
                salt(out[i].dir, j, s16);
                std::memcpy(&arena[offs[vfirst[i] + j] + lens[vfirst[i] + j] - 16], s16, 16);
            }
    clk.mark("vnode streams");
    const std::vector<u128> ids = hash_streams(arena, offs, lens, ctx);
    clk.mark("vnode hash");
    size_t k = 0;
    for (DirVNodes& d : out)
        for (EntryVNode& v : d.vnodes) v.id = MerkleHash(ids[k++]);
    return out;
}

std::vector<std::pair<std::string, MerkleHash>> compute_dir_hashes(const std::vector<DirVNodes>& vnodes,
                                                                   const std::vector<std::string>* dirs, oxh_ctx* ctx) {
    StageClock clk;
    // what compute_dir_node feeds for each staged dir's vnodes (:1042-1071)
    std::vector<std::string> segs(vnodes.size());
    parallel_for(vnodes.size(), [&](size_t i) {
        std::string& s = segs[i];
        size_t bytes = 0;
        for (const EntryVNode& v : vnodes[i].vnodes) {
            bytes += 16;
            for (const StagedNode& c : v.entries) bytes += c.node_name().size() + 16;
        }
        s.reserve(bytes);
        for (const EntryVNode& v : vnodes[i].vnodes) {
            put_le(s, v.id.to_u128());
            for (const StagedNode& c : v.entries) {
                s += c.node_name();
                put_le(s, c.hash);
            }
        }
    });
    clk.mark("dir segments");
    std::unordered_map<std::string, std::vector<size_t>> under;  // ancestor path -> descendants, in order
    for (size_t i = 0; i < vnodes.size(); ++i) {
        const std::vector<std::string> comps = path_components(vnodes[i].dir);
        for (size_t d = 0; d <= comps.size(); ++d) under[join(comps, d)].push_back(i);
    }
    std::vector<std::string> dflt;
    if (!dirs) {
        dflt.push_back("");
        for (const DirVNodes& v : vnodes)
            if (!path_components(v.dir).empty()) dflt.push_back(v.dir);
        dirs = &dflt;
    }
    // each dir's descendants (looked up once), then one arena of the exact size
    std::vector<const std::vector<size_t>*> desc(dirs->size(), nullptr);
    size_t total = 0;
    for (size_t q = 0; q < dirs->size(); ++q) {
        const std::vector<std::string> comps = path_components((*dirs)[q]);
        if (auto it = under.find(join(comps, comps.size())); it != under.end()) desc[q] = &it->second;
        total += 3 + (*dirs)[q].size();
        if (desc[q])
            for (size_t i : *desc[q]) total += segs[i].size();
    }
    std::string arena;
    arena.reserve(total);
    std::vector<uint64_t> offs, lens;
    offs.reserve(dirs->size());
    lens.reserve(dirs->size());
    for (size_t q = 0; q < dirs->size(); ++q) {
        const std::string& d = (*dirs)[q];
        const size_t start = arena.size();
        arena += "dir";
        arena += d;
        if (desc[q])
            for (size_t i : *desc[q]) arena += segs[i];
        offs.push_back(start);
        lens.push_back(arena.size() - start);
    }
    clk.mark("dir streams");
    const std::vector<u128> h = hash_streams(arena, offs, lens, ctx);
    clk.mark("dir hash");
    std::vector<std::pair<std::string, MerkleHash>> r;
    r.reserve(dirs->size());
    for (size_t i = 0; i < dirs->size(); ++i) r.emplace_back((*dirs)[i], MerkleHash(h[i]));
    return r;
}

CommitTree commit_tree(const StagedDirs& entries, const ExistingDirs& existing, uint64_t vnode_size, const SaltFn& salt,
                       oxh_ctx* ctx) {
    CommitTree t;
    t.vnodes = split_into_vnodes(entries, existing, vnode_size, salt, ctx);
    t.dir_hashes = compute_dir_hashes(t.vnodes, nullptr, ctx);
    return t;
}

}  // namespace liboxen::commit_writer
