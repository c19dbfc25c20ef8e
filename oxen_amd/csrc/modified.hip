// oxen_amd/csrc/modified.hip -- util::fs::classify_modified_from_node_with_metadata x n over one engine
// request (oxh_files_modified, _ex). See capi_internal.hpp for the pieces.
#include "capi_internal.hpp"

using namespace oxh::capi;

extern "C" {

// util::fs::classify_modified_from_node_with_metadata (util/fs.rs:1580-1619) x n: the size and mtime
// verdicts and a caller-computed metadata-hash verdict are decided on the host from what the caller's
// walk holds; every item that still needs its file read is read ONCE, all of them in ONE engine request
// (oxh_hash_files_meta semantics), with the text counts of K1T when an item's metadata is MetadataText.
int oxh_files_modified(oxh_ctx* c, const char* const* paths, const uint64_t* sizes, const uint64_t* node_bytes,
                       const uint8_t* mtime_matched, const uint64_t* node_hashes, const uint8_t* node_meta_present,
                       const uint64_t* node_meta_hashes, const uint8_t* file_meta_kind, const uint64_t* file_meta_hashes,
                       uint64_t n, uint8_t* modified, int32_t* status, uint64_t* n_hashed) {
    return oxh_files_modified_ex(c, paths, sizes, node_bytes, mtime_matched, node_hashes, node_meta_present, node_meta_hashes,
                                 file_meta_kind, file_meta_hashes, n, modified, status, nullptr, n_hashed);
}

int oxh_files_modified_ex(oxh_ctx* c, const char* const* paths, const uint64_t* sizes, const uint64_t* node_bytes,
                          const uint8_t* mtime_matched, const uint64_t* node_hashes, const uint8_t* node_meta_present,
                          const uint64_t* node_meta_hashes, const uint8_t* file_meta_kind, const uint64_t* file_meta_hashes,
                          uint64_t n, uint8_t* modified, int32_t* status, int32_t* os_error, uint64_t* n_hashed) {
    if (!c || (n && (!paths || !sizes || !node_bytes || !mtime_matched || !node_hashes || !modified)))
        return fail(OXH_ERR_INVALID, "bad arguments");
    if ((node_meta_present == nullptr) != (node_meta_hashes == nullptr))
        return fail(OXH_ERR_INVALID, "node_meta_present and node_meta_hashes go together");
    std::vector<uint64_t> idx;
    bool any_text = false;
    for (uint64_t i = 0; i < n; ++i) {
        const int kind = file_meta_kind ? file_meta_kind[i] : OXH_META_NONE;
        if (kind > OXH_META_ERROR) return fail(OXH_ERR_INVALID, "file_meta_kind out of range");
        if (kind == OXH_META_GIVEN && !file_meta_hashes) return fail(OXH_ERR_INVALID, "file_meta_hashes is NULL");
    }
    for (uint64_t i = 0; i < n; ++i) {
        modified[i] = sizes[i] != node_bytes[i] ? 1 : 0;  // fs.rs:1590-1592: no hashing needed
        if (status) status[i] = OXH_OK;
        if (os_error) os_error[i] = 0;
        if (modified[i] || mtime_matched[i]) continue;     // fs.rs:1595-1597: a matched mtime is trusted
        const int kind = file_meta_kind ? file_meta_kind[i] : OXH_META_NONE;
        const bool node_has = node_meta_present && node_meta_present[i];
        if (kind == OXH_META_ERROR) {  // fs.rs:1605-1606: the extraction's `?`
            if (status) status[i] = OXH_ERR_META;
            continue;
        }
        if (kind == OXH_META_GIVEN && node_has &&
            (file_meta_hashes[2 * i] != node_meta_hashes[2 * i] || file_meta_hashes[2 * i + 1] != node_meta_hashes[2 * i + 1])) {
            modified[i] = 1;  // fs.rs:1609-1614, before any read
            continue;
        }
        any_text |= kind == OXH_META_TEXT;
        idx.push_back(i);
    }
    if (n_hashed) *n_hashed = idx.size();
    if (idx.empty()) return OXH_OK;
    const uint64_t m = idx.size();
    std::vector<const char*> p(m);
    std::vector<uint64_t> ms(m), out(2 * m), cnt(any_text ? 2 * m : 0);
    std::vector<int32_t> st(m, OXH_OK), eno(m, 0);
    for (uint64_t k = 0; k < m; ++k) p[k] = paths[idx[k]], ms[k] = sizes[idx[k]];
    int rc = hash_files_impl(c, p.data(), m, out.data(), nullptr, st.data(), any_text ? cnt.data() : nullptr, nullptr,
                             nullptr, ms.data(), eno.data());
    if (rc) return rc;
    // MetadataText of the text items whose node has a metadata hash: serde_json of GenericMetadata
    // (model/metadata/generic_metadata.rs, untagged; MetadataText's field order) hashed in one batch
    std::vector<uint64_t> tk, toff, tlen;
    std::string json;
    for (uint64_t k = 0; k < m; ++k) {
        const uint64_t i = idx[k];
        if (st[k] != OXH_OK || !file_meta_kind || file_meta_kind[i] != OXH_META_TEXT) continue;
        if (!(node_meta_present && node_meta_present[i])) continue;  // None on the node side: no comparison
        char buf[96];
        const int len = snprintf(buf, sizeof buf, "{\"text\":{\"num_lines\":%llu,\"num_chars\":%llu}}",
                                 (unsigned long long)cnt[2 * k], (unsigned long long)cnt[2 * k + 1]);
        tk.push_back(k), toff.push_back(json.size()), tlen.push_back((uint64_t)len);
        json.append(buf, (size_t)len);
    }
    std::vector<uint64_t> mh(2 * tk.size());
    if (!tk.empty()) {
        rc = oxh_hash_streams(c, (const uint8_t*)json.data(), toff.data(), tlen.data(), tk.size(), mh.data());
        if (rc) return rc;
    }
    std::vector<uint8_t> meta_differs(m, 0);
    for (size_t j = 0; j < tk.size(); ++j) {
        const uint64_t i = idx[tk[j]];
        meta_differs[tk[j]] = mh[2 * j] != node_meta_hashes[2 * i] || mh[2 * j + 1] != node_meta_hashes[2 * i + 1];
    }
    for (uint64_t k = 0; k < m; ++k) {
        const uint64_t i = idx[k];
        if (st[k] != OXH_OK) {  // the reference returns the open / read error for this path
            if (status) status[i] = st[k];
            if (os_error) os_error[i] = eno[k];
            continue;
        }
        if (meta_differs[k]) {  // fs.rs:1609-1614
            modified[i] = 1;
            continue;
        }
        // fs.rs:1616-1618: node.hash() against get_hash_given_metadata(path, metadata)
        modified[i] = (out[2 * k] != node_hashes[2 * i] || out[2 * k + 1] != node_hashes[2 * i + 1]) ? 1 : 0;
    }
    return OXH_OK;
}

}  // extern "C"
