// tests/native/commit_tree_cli.cpp -- drives liboxen::commit_writer::commit_tree (the C++ K2 driver,
// oxen_amd/host/commit_writer.cpp) on a staged commit read from stdin, for tests/test_native_commit.py
// and tools/bench_commit.py. Input, one record per line, tab-separated:
//   vnode_size <n>
//   entries <dir>            following `node` lines are staged changes of <dir> (caller order kept)
//   existing <dir>           following `node` lines are HEAD's children of <dir>
//   node <path> <hash hex> <is_dir 0|1> <added|modified|removed|unmodified> <name, or \x01 for none>
// Salt: (dir + "#" + vnode index) padded with zero bytes / cut to 16 bytes (tests/_commit.py: salt).
// Output: `vnode <dir> <j> <id hex> <n entries> <entry paths...>` per vnode, `removed <dir> <path>`,
// `dir <dir> <hash hex>` per dir hash, and `time <seconds>` (best commit_tree call of --reps).
#include <chrono>
#include <cstdio>
#include <cstring>
#include <iostream>
#include <sstream>
#include <string>

#include "../../oxen_amd/host/commit_writer.hpp"

using namespace liboxen;
using namespace liboxen::commit_writer;

namespace {

std::vector<std::string> split_tabs(const std::string& line) {
    std::vector<std::string> f;
    size_t i = 0;
    while (true) {
        const size_t j = line.find('\t', i);
        f.emplace_back(line, i, j == std::string::npos ? std::string::npos : j - i);
        if (j == std::string::npos) break;
        i = j + 1;
    }
    return f;
}

StagedStatus parse_status(const std::string& s) {
    if (s == "added") return StagedStatus::Added;
    if (s == "modified") return StagedStatus::Modified;
    if (s == "removed") return StagedStatus::Removed;
    if (s == "unmodified") return StagedStatus::Unmodified;
    throw std::runtime_error("bad status " + s);
}

void det_salt(const std::string& dir, size_t j, uint8_t out[16]) {
    const std::string s = dir + "#" + std::to_string(j);
    for (size_t i = 0; i < 16; ++i) out[i] = i < s.size() ? (uint8_t)s[i] : 0;
}

}  // namespace

int main(int argc, char** argv) {
    int reps = 1;
    for (int i = 1; i + 1 < argc; ++i)
        if (!strcmp(argv[i], "--reps")) reps = std::max(1, atoi(argv[i + 1]));
    try {
        std::ios::sync_with_stdio(false);
        StagedDirs entries;
        ExistingDirs existing;
        uint64_t vnode_size = 10000;
        std::vector<StagedNode>* cur = nullptr;
        std::string line;
        while (std::getline(std::cin, line)) {
            const std::vector<std::string> f = split_tabs(line);
            if (f[0] == "vnode_size") {
                vnode_size = std::stoull(f.at(1));
            } else if (f[0] == "entries") {
                entries.emplace_back(f.at(1), std::vector<StagedNode>{});
                cur = &entries.back().second;
            } else if (f[0] == "existing") {
                cur = &existing[f.at(1)];
            } else if (f[0] == "node") {
                if (!cur || f.size() != 6) throw std::runtime_error("bad node line: " + line);
                StagedNode n;
                n.path = f[1];
                n.hash = MerkleHash::from_str(f[2]).to_u128();
                n.is_dir = f[3] == "1";
                n.status = parse_status(f[4]);
                if (f[5] != "\x01") n.name = f[5];
                cur->push_back(std::move(n));
            } else if (!f[0].empty()) {
                throw std::runtime_error("bad line: " + line);
            }
        }
        CommitTree t;
        double best = 1e30;
        for (int r = 0; r < reps; ++r) {
            t = CommitTree();  // the previous rep's tree is freed outside the timed call
            const auto t0 = std::chrono::steady_clock::now();
            t = commit_tree(entries, existing, vnode_size, det_salt);
            best = std::min(best, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
        }
        std::ostringstream os;
        for (const DirVNodes& d : t.vnodes) {
            for (size_t j = 0; j < d.vnodes.size(); ++j) {
                os << "vnode\t" << d.dir << '\t' << j << '\t' << d.vnodes[j].id.to_string() << '\t'
                   << d.vnodes[j].entries.size();
                for (const StagedNode& c : d.vnodes[j].entries) os << '\t' << c.path;
                os << '\n';
            }
            for (const StagedNode& c : d.removed) os << "removed\t" << d.dir << '\t' << c.path << '\n';
        }
        for (const auto& [dir, h] : t.dir_hashes) os << "dir\t" << dir << '\t' << h.to_string() << '\n';
        os << "time\t" << best << '\n';
        std::cout << os.str();
        return 0;
    } catch (const std::exception& e) {
        std::cerr << "commit_tree_cli: " << e.what() << '\n';
        return 1;
    }
}
