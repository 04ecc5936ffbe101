// fragment_engine.hpp — C++ host-side mirror of StorageNode's fragment seam.
//
// The reference is Java (storage-node/src/StorageNode.java, SN:line) and no
// JDK exists in this image, so the host side above the C ABI is C++.  This
// header keeps the reference's method names, argument meaning and error
// behaviour for the fragment pipeline and routes every byte of work through
// libdfsgpu.so (include/dfs_gpu.h):
//   sha256Hex                     SN:603-613   (RuntimeException -> std::runtime_error)
//   handleUpload's split + hashes SN:118-171   (fileId, fragments, log lines)
//   buildFragmentsJson            SN:629-642   (Base64 of each fragment, encoded once)
//   handleInternalStoreFragments  SN:265-293   (decode + hash; IllegalArgumentException)
//   parseResponseHashes check     SN:248-257   ("Hash mismatch on fragment")
//   handleDownload gather+verify  SN:419-461   ("Could not retrieve fragment i",
//                                               "File corrupted")
// A Java build binds the same C ABI through FFM (java.lang.foreign) or JNI.
#pragma once

#include <cstdint>
#include <cstdio>
#include <map>
#include <optional>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../../include/dfs_gpu.h"

namespace dfs {

using Bytes = std::vector<uint8_t>;

// java.lang.IllegalArgumentException from java.util.Base64.Decoder (SN:281).
struct IllegalArgumentException : std::invalid_argument {
    using std::invalid_argument::invalid_argument;
};

// The 500 responses of handleDownload (SN:443-446, 455-458).
struct DownloadError : std::runtime_error {
    int code;
    DownloadError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

inline std::string hex(const uint8_t* d) {  // SN:607-609: String.format("%02x", b)
    static const char* hx = "0123456789abcdef";
    std::string s(64, '0');
    for (int i = 0; i < 32; ++i) {
        s[2 * i] = hx[d[i] >> 4];
        s[2 * i + 1] = hx[d[i] & 15];
    }
    return s;
}

inline Bytes unhex(const std::string& h) {
    Bytes b(h.size() / 2);
    for (size_t i = 0; i < b.size(); ++i) b[i] = static_cast<uint8_t>(std::stoul(h.substr(2 * i, 2), nullptr, 16));
    return b;
}

// StorageNode.Fragment (SN:779-789) plus the Base64 the upload computed once.
struct Fragment {
    int index;
    Bytes data;
    std::string hash;
    std::string b64;
};

class FragmentEngine {
public:
    explicit FragmentEngine(int device = 0) {
        check(dfs_open(&ctx_, device), "dfs_open");
    }
    ~FragmentEngine() {
        if (ctx_) dfs_close(ctx_);
    }
    FragmentEngine(const FragmentEngine&) = delete;
    FragmentEngine& operator=(const FragmentEngine&) = delete;

    // sha256Hex (SN:603-613).
    std::string sha256Hex(const Bytes& data) {
        dfs_span sp{0, data.size()};
        uint8_t d[32];
        check(dfs_sha256_batch(ctx_, data.empty() ? nullptr : data.data(), &sp, 1, d, 0), "sha256Hex");
        return hex(d);
    }

    // handleUpload's hashing and split (SN:127, 138-171) plus the Base64 of
    // each fragment (SN:636), for one file: returns fileId and fragments.
    std::pair<std::string, std::vector<Fragment>> upload(const Bytes& file, int parts) {
        dfs_span sp{0, file.size()};
        std::vector<uint8_t> fd(32), frd(32ull * parts);
        std::vector<uint64_t> off(parts + 1);
        std::vector<dfs_span> split(parts);
        check(dfs_split_plan(file.size(), parts, split.data()), "split");
        uint64_t cap = 0;
        for (auto& s : split) cap += dfs_b64_encoded_len(s.len);
        std::string b64(cap, '\0');
        check(dfs_upload_batch(ctx_, file.empty() ? nullptr : file.data(), &sp, 1, parts, fd.data(), frd.data(),
                               cap ? &b64[0] : nullptr, cap, off.data(), 0),
              "handleUpload");
        std::vector<Fragment> frags;
        for (int i = 0; i < parts; ++i) {
            Fragment f;
            f.index = i;
            f.data.assign(file.begin() + split[i].off, file.begin() + split[i].off + split[i].len);
            f.hash = hex(frd.data() + 32 * i);
            f.b64 = b64.substr(off[i], off[i + 1] - off[i]);
            frags.push_back(std::move(f));
        }
        return {hex(fd.data()), std::move(frags)};
    }

    // handleInternalStoreFragments (SN:265-293): decode every fragment of the
    // body and hash it; returns index -> (data, hash).  Throws
    // IllegalArgumentException where Base64.getDecoder().decode would.
    std::map<int, std::pair<Bytes, std::string>> storeFragments(
        const std::vector<std::pair<int, std::string>>& frags) {
        const uint32_t n = static_cast<uint32_t>(frags.size());
        std::string in;
        std::vector<dfs_span> sp(n);
        std::vector<uint64_t> out_off(n), out_len(n);
        uint64_t o = 0;
        for (uint32_t i = 0; i < n; ++i) {
            sp[i] = dfs_span{in.size(), frags[i].second.size()};
            in += frags[i].second;
            out_off[i] = o;
            o += dfs_b64_decoded_cap(frags[i].second.size());
        }
        Bytes out(o ? o : 1);
        std::vector<uint8_t> dig(32ull * (n ? n : 1));
        std::vector<int32_t> status(n ? n : 1);
        const int rc = dfs_receive_fragments_batch(ctx_, in.empty() ? nullptr : in.data(), sp.data(), n,
                                                   out.data(), out_off.data(), out_len.data(), dig.data(),
                                                   status.data(), 0);
        if (rc == DFS_E_DECODE) throw IllegalArgumentException("Illegal base64 character");
        check(rc, "handleInternalStoreFragments");
        std::map<int, std::pair<Bytes, std::string>> res;
        for (uint32_t i = 0; i < n; ++i)
            res[frags[i].first] = {Bytes(out.begin() + out_off[i], out.begin() + out_off[i] + out_len[i]),
                                   hex(dig.data() + 32 * i)};
        return res;
    }

    // sendFragmentsToPeers + buildFragmentsJson (SN:195-205, 629-642): the
    // storeFragments body for every peer k != uploader (0-based, ascending),
    // built on the device with the Base64 encoded straight into it.
    std::vector<std::string> storeBodies(const Bytes& file, const std::string& fileId, int parts, int uploader) {
        dfs_span sp{0, file.size()};
        const Bytes dig = unhex(fileId);
        std::vector<uint64_t> off(parts);
        check(dfs_store_bodies_build(ctx_, nullptr, &sp, 1, parts, uploader, dig.data(), nullptr, off.data(), 0),
              "buildFragmentsJson (layout)");
        std::string buf(off[parts - 1] ? off[parts - 1] : 1, '\0');
        check(dfs_store_bodies_build(ctx_, file.empty() ? nullptr : file.data(), &sp, 1, parts, uploader, dig.data(),
                                     &buf[0], off.data(), 0),
              "buildFragmentsJson");
        std::vector<std::string> bodies;
        for (int k = 0, j = 0; k < parts; ++k) {
            if (k == uploader) continue;
            bodies.push_back(buf.substr(off[j++], dfs_store_body_len(file.size(), parts, k, (k + 1) % parts)));
        }
        return bodies;
    }

    // handleInternalStoreFragments (SN:265-293) for a body in
    // buildFragmentsJson form, parsed on the device: fileId and index ->
    // (data, hash), in body order.  Returns false for a body in any other
    // form (DFS_E_WIRE: the caller parses it with parseJson); throws
    // IllegalArgumentException where Base64.getDecoder().decode would.
    bool receiveStoreBody(const std::string& body, std::string& fileId,
                          std::vector<std::pair<int, std::pair<Bytes, std::string>>>& frags) {
        dfs_span sp{0, body.size()};
        std::vector<uint64_t> out_off(2), foff(2), flen(2);
        Bytes out(((3 * ((body.size() + 3) / 4) + 16 + 15) & ~size_t(15)) + 1);  // dfs_store_bodies_receive's slot
        uint32_t idx[2];
        uint8_t dig[64];
        char ids[64];
        int32_t st = 0;
        check(dfs_store_bodies_receive(ctx_, body.data(), &sp, 1, out.data(), out_off.data(), idx, foff.data(),
                                       flen.data(), dig, ids, &st, 0),
              "handleInternalStoreFragments");
        if (st == DFS_E_WIRE) return false;
        fileId.assign(ids, 64);
        frags.clear();
        for (int q = 0; q < 2; ++q) {
            if (st == DFS_E_DECODE && flen[q] == 0 && q == 1) break;
            frags.push_back({static_cast<int>(idx[q]),
                             {Bytes(out.begin() + foff[q], out.begin() + foff[q] + flen[q]), hex(dig + 32 * q)}});
        }
        if (st == DFS_E_DECODE) throw IllegalArgumentException("Illegal base64 character");
        return true;
    }

    // handleDownload's ordered gather + verify (SN:419-458).  frags[i] is
    // the fragment i found locally or fetched, or nullopt.
    Bytes reassembleAndVerify(const std::string& fileId, const std::vector<std::optional<Bytes>>& frags) {
        const uint32_t n = static_cast<uint32_t>(frags.size());
        std::vector<const uint8_t*> src(n);
        std::vector<uint64_t> len(n);
        uint64_t total = 0;
        static const uint8_t empty = 0;
        for (uint32_t i = 0; i < n; ++i) {
            if (!frags[i]) throw DownloadError(DFS_E_MISSING, "Could not retrieve fragment " + std::to_string(i));
            src[i] = frags[i]->empty() ? &empty : frags[i]->data();
            len[i] = frags[i]->size();
            total += len[i];
        }
        Bytes out(total ? total : 1);
        uint64_t off = 0;
        const Bytes want = unhex(fileId);
        uint8_t got[32];
        int32_t st = 0;
        const int rc = dfs_reassemble_verify(ctx_, src.data(), len.data(), 1, n, out.data(), &off, want.data(), got,
                                             &st, 0);
        if (rc == DFS_E_CORRUPT) throw DownloadError(DFS_E_CORRUPT, "File corrupted");
        check(rc, "handleDownload");
        out.resize(total);
        return out;
    }

    dfs_ctx* raw() { return ctx_; }

    // ---- the same two handler operations through a process-wide request
    // batcher (dfs_batcher): StorageNode runs one thread per connection
    // (SN:28-31), each handling ONE file; concurrent handlers' files run as
    // one launch.  Results are identical to upload() / reassembleAndVerify().
    static std::pair<std::string, std::vector<Fragment>> upload(dfs_batcher* b, const Bytes& file, int parts) {
        std::vector<uint8_t> fd(32), frd(32ull * parts);
        std::vector<uint64_t> off(parts + 1);
        std::vector<dfs_span> split(parts);
        check(dfs_split_plan(file.size(), parts, split.data()), "split");
        // The Base64 is only forwarded (into the fragments' strings here, into
        // the storeFragments bodies in the reference, SN:226-246): take it as
        // a view of the batch's result buffer and give the view back at once.
        const char* b64 = nullptr;
        dfs_view* view = nullptr;
        check(dfs_submit_upload_view(b, file.empty() ? nullptr : file.data(), file.size(), fd.data(), frd.data(), &b64,
                                     off.data(), &view),
              "handleUpload");
        std::vector<Fragment> frags;
        for (int i = 0; i < parts; ++i) {
            Fragment f;
            f.index = i;
            f.data.assign(file.begin() + split[i].off, file.begin() + split[i].off + split[i].len);
            f.hash = hex(frd.data() + 32 * i);
            f.b64.assign(b64 + off[i], off[i + 1] - off[i]);
            frags.push_back(std::move(f));
        }
        check(dfs_view_release(view), "dfs_view_release");
        return {hex(fd.data()), std::move(frags)};
    }

    static Bytes reassembleAndVerify(dfs_batcher* b, const std::string& fileId,
                                     const std::vector<std::optional<Bytes>>& frags) {
        const uint32_t n = static_cast<uint32_t>(frags.size());
        std::vector<const uint8_t*> src(n);
        std::vector<uint64_t> len(n);
        uint64_t total = 0;
        static const uint8_t empty = 0;
        for (uint32_t i = 0; i < n; ++i) {
            if (!frags[i]) throw DownloadError(DFS_E_MISSING, "Could not retrieve fragment " + std::to_string(i));
            src[i] = frags[i]->empty() ? &empty : frags[i]->data();
            len[i] = frags[i]->size();
            total += len[i];
        }
        Bytes out(total ? total : 1);
        const Bytes want = unhex(fileId);
        const int rc = dfs_submit_reassemble(b, src.data(), len.data(), want.data(), out.data(), nullptr);
        if (rc == DFS_E_CORRUPT) throw DownloadError(DFS_E_CORRUPT, "File corrupted");
        check(rc, "handleDownload");
        out.resize(total);
        return out;
    }

private:
    static void check(int rc, const char* where) {
        if (rc != DFS_OK) throw std::runtime_error(std::string(where) + ": " + dfs_strerror(rc));
    }
    dfs_ctx* ctx_ = nullptr;
};

// buildFragmentsJson (SN:629-642) from Base64 already computed on the GPU.
inline std::string buildFragmentsJson(const std::string& fileId, const std::vector<const Fragment*>& frags) {
    std::string sb = "{\"fileId\":\"" + fileId + "\",\"fragments\":[";
    for (size_t i = 0; i < frags.size(); ++i) {
        sb += "{\"index\":\"" + std::to_string(frags[i]->index) + "\",\"data\":\"" + frags[i]->b64 + "\"}";
        if (i + 1 < frags.size()) sb += ",";
    }
    return sb + "]}";
}

// buildManifestJson (SN:620-626).
inline std::string buildManifestJson(const std::string& fileId, const std::string& name, int total) {
    return "{\"fileId\":\"" + fileId + "\",\"originalName\":\"" + name + "\",\"totalFragments\":" +
           std::to_string(total) + "}";
}

}  // namespace dfs
