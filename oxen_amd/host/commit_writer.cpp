// oxen_amd/host/commit_writer.cpp -- the K2 commit driver (see commit_writer.hpp).
#include "commit_writer.hpp"

#include <algorithm>
#include <cmath>
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
std::string sort_key(const std::string& normalised) {
    std::string k = normalised;
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
    // removal drops the child), keyed by the normalised path; ordered by Path's Ord at the end
    struct Dir {
        std::vector<StagedNode> nodes;
        std::vector<std::string> keys;
        std::vector<char> alive;
        std::unordered_map<std::string, size_t> at;  // key -> live slot
        std::vector<StagedNode> removed;
        std::vector<size_t> order;  // live slots in path order
        void put(std::string key, StagedNode&& n) {
            auto it = at.find(key);
            if (it != at.end()) {
                nodes[it->second] = std::move(n);
                return;
            }
            keys.push_back(sort_key(key));
            at.emplace(std::move(key), nodes.size());
            nodes.push_back(std::move(n));
            alive.push_back(1);
        }
        void drop(const std::string& key) {
            auto it = at.find(key);
            if (it == at.end()) return;
            alive[it->second] = 0;
            at.erase(it);
        }
    };
    std::vector<Dir> dirs(entries.size());
    parallel_for(entries.size(), [&](size_t i) {
        const std::string& directory = entries[i].first;
        const std::vector<std::string> dcomps = path_components(directory);
        const std::string dkey = join(dcomps, dcomps.size());
        Dir& d = dirs[i];
        const auto ex = existing.find(directory);
        const size_t expect = entries[i].second.size() + (ex != existing.end() ? ex->second.size() : 0);
        d.nodes.reserve(expect);
        d.keys.reserve(expect);
        d.alive.reserve(expect);
        d.at.reserve(expect);
        if (auto it = ex; it != existing.end())
            for (const StagedNode& c : it->second) d.put(normalize(c.path), StagedNode(c));
        std::unordered_map<std::string, size_t> removed_at;  // a later removal of a path replaces it
        for (StagedNode c : entries[i].second) {
            std::string ckey = normalize(c.path);
            if (ckey.empty()) continue;  // child_path != "" (:589)
            if (!dkey.empty() && !(ckey.size() > dkey.size() && ckey.compare(0, dkey.size(), dkey) == 0 &&
                                   ckey[dkey.size()] == '/') && ckey != dkey) {  // defensive prefixing (:591-612)
                ckey = dkey + "/" + ckey;
                c.path = ckey;
                c.name = ckey;
            }
            if (c.status == StagedStatus::Removed) {
                d.drop(ckey);
                auto [it, fresh] = removed_at.emplace(ckey, d.removed.size());
                if (fresh) d.removed.push_back(std::move(c));
                else d.removed[it->second] = std::move(c);
            } else {
                d.put(std::move(ckey), std::move(c));
            }
        }
        for (size_t k = 0; k < d.nodes.size(); ++k)
            if (d.alive[k]) d.order.push_back(k);
        std::sort(d.order.begin(), d.order.end(), [&](size_t x, size_t y) { return d.keys[x] < d.keys[y]; });
    });
    // bucket = xxh3_128(path) % num_vnodes (:665-681): every child of every dir in one pass
    std::string arena;
    std::vector<uint64_t> offs, lens;
    size_t n_children = 0, path_bytes = 0;
    for (const Dir& d : dirs)
        for (size_t k : d.order) {
            ++n_children;
            path_bytes += d.nodes[k].path.size();
        }
    arena.reserve(path_bytes);
    offs.reserve(n_children);
    lens.reserve(n_children);
    for (const Dir& d : dirs)
        for (size_t k : d.order) {
            offs.push_back(arena.size());
            lens.push_back(d.nodes[k].path.size());
            arena += d.nodes[k].path;
        }
    const std::vector<u128> buckets = hash_streams(arena, offs, lens, ctx);
    std::vector<DirVNodes> out(entries.size());
    size_t k = 0;
    for (size_t i = 0; i < dirs.size(); ++i) {
        out[i].dir = entries[i].first;
        out[i].removed = std::move(dirs[i].removed);
        const uint64_t nv = num_vnodes(dirs[i].order.size(), vnode_size);
        out[i].vnodes.resize(nv);
        std::vector<uint32_t> b(dirs[i].order.size());
        std::vector<size_t> per(nv, 0);
        for (size_t q = 0; q < b.size(); ++q) ++per[b[q] = (uint32_t)(buckets[k + q] % nv)];
        for (uint64_t j = 0; j < nv; ++j) out[i].vnodes[j].entries.reserve(per[j]);
        // path order in, so every vnode's entries come out sorted (:684-694)
        for (size_t q = 0; q < b.size(); ++q) out[i].vnodes[b[q]].entries.push_back(std::move(dirs[i].nodes[dirs[i].order[q]]));
        k += b.size();
    }
    // vnode id = xxh3("vnode" || dir || child hashes LE [|| uuid]) (:683-720): every vnode in one pass
    arena.clear();
    offs.clear();
    lens.clear();
    arena.reserve(n_children * 16 + out.size() * 64);
    for (const DirVNodes& d : out) {
        const bool dir_existed = existing.count(d.dir) != 0;
        for (size_t j = 0; j < d.vnodes.size(); ++j) {
            const size_t start = arena.size();
            arena += "vnode";
            arena += d.dir;
            bool changed = false;
            for (const StagedNode& c : d.vnodes[j].entries) {
                put_le(arena, c.hash);
                changed = changed || c.status != StagedStatus::Unmodified;
            }
            if (dir_existed && changed) {  // :713-716
                uint8_t s[16];
                salt(d.dir, j, s);
                arena.append(reinterpret_cast<const char*>(s), 16);
            }
            offs.push_back(start);
            lens.push_back(arena.size() - start);
        }
    }
    const std::vector<u128> ids = hash_streams(arena, offs, lens, ctx);
    k = 0;
    for (DirVNodes& d : out)
        for (EntryVNode& v : d.vnodes) v.id = MerkleHash(ids[k++]);
    return out;
}

std::vector<std::pair<std::string, MerkleHash>> compute_dir_hashes(const std::vector<DirVNodes>& vnodes,
                                                                   const std::vector<std::string>* dirs, oxh_ctx* ctx) {
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
    const std::vector<u128> h = hash_streams(arena, offs, lens, ctx);
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
