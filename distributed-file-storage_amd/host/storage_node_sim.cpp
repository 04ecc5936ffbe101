// storage_node_sim.cpp — BASELINE config 1 replayed in-process on the GPU path.
//
// Five StorageNodes (ids 1..5, TOTAL_NODES = 5, SN:15) share one process;
// the HTTP hops of the reference (SN:226-259 storeFragments, SN:471-483
// getFragment, SN:313-350 announce) become direct calls, everything else
// follows StorageNode.java: node 1 uploads the example files (split, hashes,
// Base64 and the receivers' decode + hash all run in libdfsgpu.so through
// FragmentEngine), node 3 then goes down, and nodes 1, 2, 4 and 5 download
// every file with the reference's fetch order (local, then nodeA = i+1, then
// nodeB = ((i-1+N)%N)+1, SN:422-440) and verify SHA-256(file) == fileId.
// Log lines use the reference's formats (SN:125, 128, 136, 160, 167, 209) so
// config 1's "diff fragment SHA-256s" is a grep + diff.
//
// Fragments are real files: every node's data/node-<id>/<fileId>/fragments/
// <i>.frag (SN:20, 147-166, 273-285), written and read through the library's
// fragment store (dfs_store_write_fragments / dfs_store_read_fragments).
// The data directory is $DFS_SIM_DATA (kept), else a fresh /tmp directory
// removed at exit.
//
// Handlers run as in the reference: one thread per connection (SN:28-31), one
// file per request.  The uploads of all files run concurrently on their own
// threads, then (node 3 down) each node's downloads do; every handler goes
// through the process-wide request batcher (dfs_submit_upload for SN:118-171,
// dfs_submit_reassemble for SN:419-458), which runs the concurrent requests as
// one launch.  A handler writes its log lines to its own buffer; the buffers
// are printed in request order, so the log is the same as a serial run's.
// --serial: the same replay with one handler at a time through the per-call
// ABI (dfs_upload_batch / dfs_reassemble_verify).
//
// usage: storage_node_sim [--serial] <file>...   (prints the log to stdout;
//        exit 0 = all downloads verified bit-exact)
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <filesystem>
#include <fstream>
#include <iterator>
#include <map>
#include <mutex>
#include <optional>
#include <set>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "fragment_engine.hpp"

namespace {

constexpr int TOTAL_NODES = 5;  // SN:15
namespace fs = std::filesystem;

// One handler's log lines (System.out.printf in the reference), printed by
// the main thread in request order.
struct Log {
    std::string text;
    void printf(const char* fmt, ...) __attribute__((format(printf, 2, 3))) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        const int n = std::vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        text.append(buf, n < 0 ? 0 : std::min<size_t>(static_cast<size_t>(n), sizeof buf - 1));
    }
};

std::string basename_of(const std::string& p) {
    const size_t s = p.find_last_of('/');
    return s == std::string::npos ? p : p.substr(s + 1);
}

// parseJson for /internal/storeFragments bodies (SN:704-753): the same
// indexOf / split("},{") / strip-quotes procedure.
std::pair<std::string, std::vector<std::pair<int, std::string>>> parseJson(const std::string& json) {
    std::string fileId;
    std::vector<std::pair<int, std::string>> frags;
    size_t i = json.find("\"fileId\"");
    if (i != std::string::npos) {
        size_t colon = json.find(':', i), q1 = json.find('"', colon + 1), q2 = json.find('"', q1 + 1);
        if (q1 != std::string::npos && q2 != std::string::npos) fileId = json.substr(q1 + 1, q2 - q1 - 1);
    }
    size_t k = json.find("\"fragments\"");
    if (k != std::string::npos) {
        size_t a = json.find('[', k), b = json.find(']', a);
        std::string arr = json.substr(a + 1, b - a - 1);
        size_t pos = 0;
        while (pos <= arr.size() && !arr.empty()) {
            size_t nx = arr.find("},{", pos);
            std::string item = arr.substr(pos, nx == std::string::npos ? std::string::npos : nx - pos);
            std::string clean;
            for (char c : item)
                if (c != '{' && c != '}' && c != '"') clean += c;
            std::map<std::string, std::string> kv;
            std::stringstream ss(clean);
            std::string field;
            while (std::getline(ss, field, ',')) {
                size_t c = field.find(':');
                if (c != std::string::npos) kv[field.substr(0, c)] = field.substr(c + 1);
            }
            if (kv.count("index") && kv.count("data")) frags.emplace_back(std::stoi(kv["index"]), kv["data"]);
            if (nx == std::string::npos) break;
            pos = nx + 3;
        }
    }
    return {fileId, frags};
}

std::vector<uint8_t> raw_id(const std::string& hex) {
    std::vector<uint8_t> d(32, 0);
    for (size_t i = 0; i < 32 && 2 * i + 1 < hex.size(); ++i) d[i] = static_cast<uint8_t>(std::stoi(hex.substr(2 * i, 2), nullptr, 16));
    return d;
}

struct Node {
    int id;
    bool up = true;
    std::string root;                              // dataRoot = data/node-<id> (SN:20)
    std::map<std::string, std::string> manifests;  // data/node-<id>/<fileId>/manifest.json

    // Files.createDirectories + Files.write(<i>.frag) (SN:149, 166; 275, 285)
    void saveFragment(const std::string& fileId, int index, const dfs::Bytes& b) {
        const auto d = raw_id(fileId);
        dfs_frag_ref ref{0, b.size(), 0, static_cast<uint32_t>(index)};
        int32_t st = 0;
        const int rc = dfs_store_write_fragments(nullptr, root.c_str(), d.data(), 1, b.data(), &ref, 1, &st, 0);
        if (rc != DFS_OK) throw std::runtime_error(std::string("Files.write: ") + dfs_strerror(rc));
    }
    // tryLoadFragmentLocal (SN:463-469): the bytes, or nullopt if absent
    std::optional<dfs::Bytes> loadFragment(const std::string& fileId, int index) const {
        std::error_code ec;
        const fs::path p = fs::path(root) / fileId / "fragments" / (std::to_string(index) + ".frag");
        if (!fs::exists(p, ec)) return std::nullopt;
        const uint64_t sz = fs::file_size(p, ec);
        if (ec) throw std::runtime_error("readAllBytes: " + ec.message());
        dfs::Bytes b(sz);
        const auto d = raw_id(fileId);
        dfs_frag_ref ref{0, sz, 0, static_cast<uint32_t>(index)};
        uint64_t len = 0;
        int32_t st = 0;
        const int rc = dfs_store_read_fragments(nullptr, root.c_str(), d.data(), 1, b.data(), &ref, 1, &len, &st, 0);
        if (st == DFS_E_MISSING) return std::nullopt;
        if (rc != DFS_OK) throw std::runtime_error(std::string("readAllBytes: ") + dfs_strerror(rc));
        b.resize(len);
        return b;
    }
};

struct Cluster {
    dfs::FragmentEngine eng;
    dfs_batcher* batcher = nullptr;  // nullptr: --serial, the per-call ABI
    std::mutex mu;                   // the manifests (handlers run concurrently)
    std::vector<Node> nodes;
    ~Cluster() {
        if (batcher) dfs_batcher_destroy(batcher);
    }
    explicit Cluster(const std::string& data, bool threaded) {
        if (threaded) {
            dfs_batcher_opts o{};
            o.max_wait_us = 2000;
            const int rc = dfs_batcher_create(0, TOTAL_NODES, &o, &batcher);
            if (rc != DFS_OK) throw std::runtime_error(std::string("dfs_batcher_create: ") + dfs_strerror(rc));
        }
        for (int i = 1; i <= TOTAL_NODES; ++i) {
            nodes.emplace_back();
            nodes.back().id = i;
            nodes.back().root = data + "/node-" + std::to_string(i);
            fs::create_directories(nodes.back().root);  // SN:24
        }
    }
    Node& node(int id) { return nodes[id - 1]; }

    // What a peer answers: the reply text on the wire (buildHashResponse,
    // SN:644-655) and, for the log lines, the {index -> hash} behind it.
    struct StoreReply {
        std::string json;
        std::map<int, std::string> hashes;
    };

    // buildHashResponse through the ABI (dfs_store_hash_responses_build) for one body's two entries.
    static std::string hashResponse(const std::string& fileId, const std::vector<std::pair<int, std::string>>& put) {
        if (fileId.size() != 64 || put.size() != 2) {
            // not a sendFragmentsToNode body (two entries, a SHA-256 fileId): the reference's builder as text;
            // indices below 16 iterate in ascending order in its HashMap
            std::map<int, std::string> m;
            for (auto& kv : put) m[kv.first] = kv.second;
            std::string out = "{\"fileId\":\"" + fileId + "\",\"received\":[";
            size_t k = 0;
            for (auto& kv : m)
                out += "{\"index\":\"" + std::to_string(kv.first) + "\",\"hash\":\"" + kv.second + "\"}" +
                       (++k < m.size() ? "," : "");
            return out + "]}";
        }
        const uint32_t idx[2] = {static_cast<uint32_t>(put[0].first), static_cast<uint32_t>(put[1].first)};
        dfs::Bytes dig = dfs::unhex(put[0].second), d2 = dfs::unhex(put[1].second);
        dig.insert(dig.end(), d2.begin(), d2.end());
        std::string out(dfs_store_hash_response_cap(), '\0');
        uint64_t off[2] = {0, 0};
        if (dfs_store_hash_responses_build(fileId.data(), idx, dig.data(), nullptr, 1, &out[0], out.size(), off) != DFS_OK)
            throw std::runtime_error("dfs_store_hash_responses_build");
        out.resize(off[1]);
        return out;
    }

    // handleInternalStoreFragments (SN:265-293) on node `id`.
    StoreReply storeFragments(int id, const std::string& body) {
        Node& n = node(id);
        if (!n.up) throw std::runtime_error("Connection refused");
        StoreReply r;
        std::vector<std::pair<int, std::string>> put;  // response.put(index, hash) in body order, SN:287
        std::string fileId;
        std::vector<std::pair<int, std::pair<dfs::Bytes, std::string>>> dev;
        if (eng.receiveStoreBody(body, fileId, dev)) {  // device parse + decode + hash
            for (auto& kv : dev) {
                n.saveFragment(fileId, kv.first, kv.second.first);  // Files.write(<i>.frag), SN:284-285
                r.hashes[kv.first] = kv.second.second;
                put.emplace_back(kv.first, kv.second.second);
            }
        } else {
            auto parsed = parseJson(body);  // any other body form: the reference's parser
            fileId = parsed.first;
            auto got = eng.storeFragments(parsed.second);
            for (auto& kv : got) {
                n.saveFragment(parsed.first, kv.first, kv.second.first);  // Files.write(<i>.frag), SN:284-285
                r.hashes[kv.first] = kv.second.second;
                put.emplace_back(kv.first, kv.second.second);
            }
        }
        r.json = hashResponse(fileId, put);
        return r;
    }

    // handleUpload on node u (SN:118-189).
    std::string upload(int u, const std::string& name, const dfs::Bytes& file, Log& out) {
        out.printf("[%d] Received upload: %zu bytes\n", u, file.size());
        auto up = batcher ? dfs::FragmentEngine::upload(batcher, file, TOTAL_NODES) : eng.upload(file, TOTAL_NODES);
        const std::string& fileId = up.first;
        out.printf("[%d] FileId = %s\n", u, fileId.c_str());
        out.printf("[%d] Original name = %s\n", u, name.c_str());
        const int u0 = u - 1, my1 = u0, my2 = (u0 + 1) % TOTAL_NODES;
        for (const auto& f : up.second) {
            out.printf("[%d] Fragment %d: %zu bytes, hash=%s\n", u, f.index, f.data.size(), f.hash.c_str());
            if (f.index == my1 || f.index == my2) {
                node(u).saveFragment(fileId, f.index, f.data);  // SN:165-166
                out.printf("[%d] Saved fragment %d locally\n", u, f.index);
            }
        }
        // sendFragmentsToPeers (SN:195-224); every peer's body built on the device
        const std::vector<std::string> bodies = eng.storeBodies(file, fileId, TOTAL_NODES, u0);
        for (int k = 0, j = 0; k < TOTAL_NODES; ++k) {
            if (k == u0) continue;
            const int f1 = k, f2 = (k + 1) % TOTAL_NODES;
            bool ok = false;
            for (int attempt = 1; attempt <= 3 && !ok; ++attempt) {
                out.printf("[%d] Sending fragments %d and %d to node %d (attempt %d)\n", u, f1, f2, k + 1, attempt);
                try {
                    const std::string& body = bodies[j];
                    if (body != dfs::buildFragmentsJson(fileId, {&up.second[f1], &up.second[f2]}))
                        throw std::logic_error("device body differs from buildFragmentsJson");
                    const StoreReply remote = storeFragments(k + 1, body);
                    // parseResponseHashes + the comparison of SN:248-257 through the ABI, on the reply text
                    const uint32_t idx[2] = {static_cast<uint32_t>(f1), static_cast<uint32_t>(f2)};
                    dfs::Bytes want = dfs::unhex(up.second[f1].hash), w2 = dfs::unhex(up.second[f2].hash);
                    want.insert(want.end(), w2.begin(), w2.end());
                    const dfs_span sp{0, remote.json.size()};
                    int32_t st = 0;
                    (void)dfs_store_hash_responses_check(remote.json.data(), &sp, 1, idx, want.data(), &st);
                    ok = st == DFS_OK;
                    for (int fi : {f1, f2}) {  // the reference's log line for a mismatch, SN:253-254
                        auto it = remote.hashes.find(fi);
                        const std::string rh = it == remote.hashes.end() ? "null" : it->second;
                        if (!ok && rh != up.second[fi].hash) {
                            out.printf("[%d] Hash mismatch on fragment %d (local=%s, remote=%s)\n", u, fi,
                                        up.second[fi].hash.c_str(), rh.c_str());
                            break;  // return false at the first one, SN:255
                        }
                    }
                } catch (const std::exception&) {
                }
            }
            if (!ok) {
                out.printf("[%d] FAILED sending to node %d\n", u, k + 1);
                return "";  // 500 "Replication failed", SN:174-177
            }
            ++j;
        }
        const std::string manifest = dfs::buildManifestJson(fileId, name, TOTAL_NODES);
        {
            std::lock_guard<std::mutex> lk(mu);
            for (auto& n : nodes) n.manifests[fileId] = manifest;  // save + announce (SN:180-186)
        }
        out.printf("[%d] Uploaded %s\n", u, name.c_str());
        return fileId;
    }

    // handleDownload on node r (SN:399-461): returns the file bytes.
    dfs::Bytes download(int r, const std::string& fileId, std::string& plan) {
        std::vector<std::optional<dfs::Bytes>> frags(TOTAL_NODES);
        plan.clear();
        for (int i = 0; i < TOTAL_NODES; ++i) {
            std::string src = "missing";
            if (auto local = node(r).loadFragment(fileId, i)) {  // SN:421
                frags[i] = std::move(local);
                src = "local";
            } else {
                const int cand[2] = {i + 1, ((i - 1 + TOTAL_NODES) % TOTAL_NODES) + 1};  // SN:427-428
                for (int nd : cand) {
                    if (nd == r) continue;  // SN:433
                    Node& peer = node(nd);
                    if (!peer.up) continue;  // IOException swallowed, SN:439
                    auto got = peer.loadFragment(fileId, i);  // getFragment, SN:471-483
                    if (!got) continue;                        // 404 -> null
                    frags[i] = std::move(got);
                    src = "node" + std::to_string(nd);
                    break;
                }
            }
            plan += (i ? "," : "") + src;
        }
        return batcher ? dfs::FragmentEngine::reassembleAndVerify(batcher, fileId, frags)
                       : eng.reassembleAndVerify(fileId, frags);  // SN:448-458
    }
};

}  // namespace

int main(int argc, char** argv) {
    bool threaded = true;
    std::vector<std::string> paths;
    for (int a = 1; a < argc; ++a) {
        if (std::string(argv[a]) == "--serial") threaded = false;
        else paths.push_back(argv[a]);
    }
    if (paths.empty()) {
        std::fprintf(stderr, "usage: %s [--serial] <file>...\n", argv[0]);
        return 2;
    }
    std::string data;
    bool keep = false;
    if (const char* d = std::getenv("DFS_SIM_DATA")) {
        data = d;
        keep = true;
    } else {
        char tmpl[] = "/tmp/dfs_sim_XXXXXX";
        if (!mkdtemp(tmpl)) {
            std::perror("mkdtemp");
            return 3;
        }
        data = tmpl;
    }
    struct Cleanup {
        std::string dir;
        bool keep;
        ~Cleanup() {
            std::error_code ec;
            if (!keep) fs::remove_all(dir, ec);
        }
    } cleanup{data, keep};
    try {
        Cluster c(data, threaded);
        std::vector<std::pair<std::string, dfs::Bytes>> files;
        for (const std::string& p : paths) {
            std::ifstream in(p, std::ios::binary);
            if (!in) throw std::runtime_error("cannot read " + p);
            dfs::Bytes b((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
            files.emplace_back(basename_of(p), b);
        }
        const size_t nf = files.size();
        // Run fn(k, log) for every file k: one handler thread per request
        // (SN:30) or, with --serial, one after the other; then print the logs
        // in request order.  An exception that escapes a handler is rethrown.
        auto handlers = [&](auto fn) {
            std::vector<Log> logs(nf);
            std::vector<std::string> errs(nf);
            auto run = [&](size_t k) {
                try {
                    fn(k, logs[k]);
                } catch (const std::exception& e) {
                    errs[k] = e.what();
                }
            };
            if (threaded) {
                std::vector<std::thread> th;
                for (size_t k = 0; k < nf; ++k) th.emplace_back(run, k);
                for (auto& t : th) t.join();
            } else {
                for (size_t k = 0; k < nf; ++k) run(k);
            }
            for (size_t k = 0; k < nf; ++k) std::fputs(logs[k].text.c_str(), stdout);
            for (size_t k = 0; k < nf; ++k)
                if (!errs[k].empty()) throw std::runtime_error(errs[k]);
        };
        std::vector<std::string> ids(nf);
        handlers([&](size_t k, Log& log) { ids[k] = c.upload(1, files[k].first, files[k].second, log); });
        for (const std::string& id : ids)
            if (id.empty()) return 1;
        c.node(3).up = false;  // config 1: node 3 down after the uploads
        std::printf("[sim] node 3 is down\n");
        std::vector<int> bad(nf, 0);
        for (int r : {1, 2, 4, 5}) {
            handlers([&](size_t k, Log& log) {
                std::string plan;
                try {
                    dfs::Bytes got = c.download(r, ids[k], plan);
                    const bool same = got == files[k].second;
                    log.printf("[%d] Download %s fileId=%s plan=%s -> %zu bytes %s\n", r, files[k].first.c_str(),
                               ids[k].c_str(), plan.c_str(), got.size(), same ? "OK" : "MISMATCH");
                    bad[k] += !same;
                } catch (const dfs::DownloadError& e) {
                    log.printf("[%d] Download %s -> 500 %s\n", r, files[k].first.c_str(), e.what());
                    ++bad[k];
                }
            });
        }
        int nbad = 0;
        for (int b : bad) nbad += b;
        // both holders of fragment 2 (nodes 3 and 2) down -> SN:443-446
        c.node(2).up = false;
        std::string plan;
        try {
            c.download(1, ids[0], plan);
            std::printf("[1] Download with nodes 2,3 down -> unexpectedly OK\n");
            ++nbad;
        } catch (const dfs::DownloadError& e) {
            std::printf("[1] Download with nodes 2,3 down -> 500 %s\n", e.what());
        }
        if (c.batcher) {
            dfs_batcher_stats_t st{};
            dfs_batcher_stats(c.batcher, &st);
            std::printf("[sim] batcher: %llu requests in %llu batches (largest %llu)\n",
                        (unsigned long long)st.requests, (unsigned long long)st.batches, (unsigned long long)st.max_batch);
        }
        return nbad ? 1 : 0;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "storage_node_sim: %s\n", e.what());
        return 3;
    }
}
