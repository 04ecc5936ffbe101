// wire_host.cpp — the reply half of the storeFragments exchange, on the host.
//
// Reference (StorageNode.java): after a peer has decoded, hashed and stored
// the two fragments of a storeFragments body it answers
//   {"fileId":"<id>","received":[{"index":"k","hash":"<64 hex>"},...]}
// (buildHashResponse, :644-655, over a HashMap<Integer,String> filled by
// put(index, hash), :277-288), and the sender parses that reply
// (parseResponseHashes, :657-701) and compares every fragment it sent with the
// hash it computed itself (:248-257); a mismatch, a missing entry or an
// exception make the attempt fail (:212-215).  A reply is ~200 bytes per
// body, so this is string work for the host, batched over the bodies of one
// dfs_store_bodies_receive / dfs_store_bodies_build call; the digests come
// from the device calls.  The parser restates the reference's own lenient
// one (indexOf / split / replace / trim), so replies from an unmodified
// StorageNode and replies built here are read alike.
#include <algorithm>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "../../include/dfs_gpu.h"

namespace {

const char kHex[] = "0123456789abcdef";

void hex32(const uint8_t* d, char* out) {
    for (int i = 0; i < 32; ++i) {
        out[2 * i] = kHex[d[i] >> 4];
        out[2 * i + 1] = kHex[d[i] & 15];
    }
}

// Iteration order of a HashMap<Integer, ?> holding two keys put in the order
// (a, b): table of 16 buckets, bucket = (k ^ (k >>> 16)) & 15, buckets
// ascending, insertion order within one.
bool b_first(uint32_t a, uint32_t b) {
    const uint32_t ba = (a ^ (a >> 16)) & 15u, bb = (b ^ (b >> 16)) & 15u;
    return bb < ba;
}

// ---- java.lang.String pieces the reference's parser uses --------------------
std::string j_trim(const std::string& s) {
    size_t a = 0, b = s.size();
    while (a < b && static_cast<unsigned char>(s[a]) <= 0x20) ++a;
    while (b > a && static_cast<unsigned char>(s[b - 1]) <= 0x20) --b;
    return s.substr(a, b - a);
}

// String.split(literal) / split(literal, limit): no match -> the string
// itself; limit 0 drops trailing empty strings.
std::vector<std::string> j_split(const std::string& s, const std::string& sep, int limit = 0) {
    std::vector<std::string> out;
    size_t pos = 0, hit = s.find(sep);
    if (hit == std::string::npos) return {s};
    while (hit != std::string::npos && (limit <= 0 || static_cast<int>(out.size()) < limit - 1)) {
        out.push_back(s.substr(pos, hit - pos));
        pos = hit + sep.size();
        hit = s.find(sep, pos);
    }
    out.push_back(s.substr(pos));
    if (limit == 0)
        while (!out.empty() && out.back().empty()) out.pop_back();
    return out;
}

std::string j_remove(std::string s, char c) {
    s.erase(std::remove(s.begin(), s.end(), c), s.end());
    return s;
}

// Integer.parseInt: optional sign, ASCII digits, 32-bit range.
bool j_parse_int(const std::string& s, long long* v) {
    size_t i = (!s.empty() && (s[0] == '-' || s[0] == '+')) ? 1 : 0;
    if (i == s.size()) return false;
    long long x = 0;
    for (size_t k = i; k < s.size(); ++k) {
        if (s[k] < '0' || s[k] > '9') return false;
        x = x * 10 + (s[k] - '0');
        if (x > (1ll << 31)) return false;
    }
    if (s[0] == '-') x = -x;
    if (x < -(1ll << 31) || x > (1ll << 31) - 1) return false;
    *v = x;
    return true;
}

// parseResponseHashes (SN:657-701).  false = the Java code would throw
// (NumberFormatException, StringIndexOutOfBoundsException).
bool parse_response(const std::string& text, std::vector<std::pair<long long, std::string>>& map) {
    const std::string json = j_trim(text);
    size_t start = json.find("\"received\"");
    if (start == std::string::npos) return true;
    start = json.find('[', start);
    const size_t end = json.find(']', start == std::string::npos ? 0 : start);
    if (start == std::string::npos || end == std::string::npos) return true;
    if (end < start + 1) return false;  // substring(start + 1, end)
    const std::string arr = j_trim(json.substr(start + 1, end - start - 1));
    if (arr.empty()) return true;
    for (const std::string& raw : j_split(arr, "},{")) {
        const std::string item = j_trim(j_remove(j_remove(j_remove(raw, '{'), '}'), '"'));
        bool have_i = false, have_h = false;
        long long index = 0;
        std::string hash;
        for (const std::string& field : j_split(item, ",")) {
            const std::vector<std::string> kv = j_split(field, ":", 2);
            if (kv.size() != 2) continue;
            const std::string key = j_trim(kv[0]), value = j_trim(kv[1]);
            if (key == "index") {
                if (!j_parse_int(value, &index)) return false;
                have_i = true;
            } else if (key == "hash") {
                hash = value;
                have_h = true;
            }
        }
        if (have_i && have_h) {  // map.put: a later entry with the same index replaces the earlier
            bool found = false;
            for (auto& e : map)
                if (e.first == index) {
                    e.second = hash;
                    found = true;
                }
            if (!found) map.emplace_back(index, hash);
        }
    }
    return true;
}

}  // namespace

extern "C" {

uint64_t dfs_store_hash_response_cap(void) {
    // {"fileId":" + 64 + ","received":[ + 2 x ({"index":" + 10 digits + ","hash":" + 64 + "}) + , + ]}
    return 11 + 64 + 14 + 2 * (10 + 10 + 10 + 64 + 2) + 1 + 2;
}

int dfs_store_hash_responses_build(const char* file_ids, const uint32_t* frag_index, const uint8_t* digests,
                                   const int32_t* status, uint32_t n, char* out, uint64_t out_cap, uint64_t* out_off) {
    if (!out_off || (n && (!file_ids || !frag_index || !digests))) return DFS_E_ARG;
    uint64_t o = 0;
    for (uint32_t i = 0; i < n; ++i) {
        out_off[i] = o;
        if (status && status[i] != DFS_OK) continue;  // the handler threw before it answered (SN:280-282)
        const uint32_t a = frag_index[2 * i], b = frag_index[2 * i + 1];
        // response.put(a, ..); response.put(b, ..): one entry if a == b (the second hash stays)
        uint32_t key[2] = {a, b};
        int src[2] = {0, 1}, cnt = 2;
        if (a == b) {
            src[0] = 1;
            cnt = 1;
        } else if (b_first(a, b)) {
            std::swap(key[0], key[1]);
            std::swap(src[0], src[1]);
        }
        std::string s = "{\"fileId\":\"";
        s.append(file_ids + 64ull * i, 64);
        s += "\",\"received\":[";
        for (int k = 0; k < cnt; ++k) {
            char hx[64];
            hex32(digests + 64ull * i + 32 * src[k], hx);
            s += "{\"index\":\"" + std::to_string(key[k]) + "\",\"hash\":\"";
            s.append(hx, 64);
            s += "\"}";
            if (k + 1 < cnt) s += ",";
        }
        s += "]}";
        if (out) {
            if (o + s.size() > out_cap) return DFS_E_ARG;
            std::memcpy(out + o, s.data(), s.size());
        }
        o += s.size();
    }
    out_off[n] = o;
    return DFS_OK;
}

int dfs_store_hash_responses_check(const char* responses, const dfs_span* spans, uint32_t n, const uint32_t* frag_index,
                                   const uint8_t* expected, int32_t* status) {
    if (n && (!spans || !frag_index || !expected || !status)) return DFS_E_ARG;
    int worst = DFS_OK;
    for (uint32_t i = 0; i < n; ++i) {
        if (spans[i].len && !responses) return DFS_E_ARG;
        std::vector<std::pair<long long, std::string>> map;
        int st = DFS_OK;
        if (!parse_response(std::string(spans[i].len ? responses + spans[i].off : "", spans[i].len), map)) {
            st = DFS_E_WIRE;  // an exception inside sendFragmentsToNode: the attempt fails (SN:212-215)
        } else {
            for (int q = 0; q < 2 && st == DFS_OK; ++q) {  // for (Fragment f : frags), SN:250-257
                char hx[64];
                hex32(expected + 64ull * i + 32 * q, hx);
                const std::string* remote = nullptr;
                for (const auto& e : map)
                    if (e.first == static_cast<long long>(frag_index[2 * i + q])) remote = &e.second;
                if (!remote || remote->size() != 64 || std::memcmp(remote->data(), hx, 64) != 0) st = DFS_E_FRAG_MISMATCH;
            }
        }
        status[i] = st;
        if (st != DFS_OK && worst == DFS_OK) worst = st;
    }
    return worst;
}

}  // extern "C"
