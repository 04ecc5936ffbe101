// The storeFragments reply parser and builder (csrc/wire_host.cpp) under
// AddressSanitizer + UBSan: replies built by the library, then mutated at
// random (characters replaced, spans cut, brackets and quotes moved), 200,000
// of them through dfs_store_hash_responses_check.  No result is checked here
// beyond "a status comes back" (tests/test_hash_response.py compares the
// statuses with the oracle); this run is for memory errors and overflow.
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../include/dfs_gpu.h"

int main() {
    std::mt19937_64 rng(12345);
    const char pool[] = "{}[]\",:0123456789abcdefx+- \n\t";
    long ok = 0, mismatch = 0, wire = 0;
    for (int round = 0; round < 2000; ++round) {
        const uint32_t n = 100;
        std::string ids(64ull * n, 'a');
        std::vector<uint32_t> idx(2 * n);
        std::vector<uint8_t> dig(64ull * n);
        for (auto& b : dig) b = static_cast<uint8_t>(rng());
        for (auto& c : ids) c = "0123456789abcdef"[rng() % 16];
        for (uint32_t i = 0; i < n; ++i) {
            idx[2 * i] = static_cast<uint32_t>(rng() % 70000);
            idx[2 * i + 1] = rng() % 4 ? (idx[2 * i] + 1) % 10 : idx[2 * i];
        }
        std::vector<uint64_t> off(n + 1);
        std::string out(dfs_store_hash_response_cap() * n, '\0');
        if (dfs_store_hash_responses_build(ids.data(), idx.data(), dig.data(), nullptr, n, &out[0], out.size(), off.data()))
            return 1;
        // mutate each reply in its own copy
        std::string blob;
        std::vector<dfs_span> sp(n);
        for (uint32_t i = 0; i < n; ++i) {
            std::string r = out.substr(off[i], off[i + 1] - off[i]);
            const int edits = static_cast<int>(rng() % 5);
            for (int e = 0; e < edits && !r.empty(); ++e) {
                const size_t p = rng() % r.size();
                switch (rng() % 4) {
                    case 0: r[p] = pool[rng() % (sizeof pool - 1)]; break;
                    case 1: r.erase(p, rng() % 9); break;
                    case 2: r.insert(p, 1, pool[rng() % (sizeof pool - 1)]); break;
                    default: r = r.substr(0, p); break;
                }
            }
            sp[i] = dfs_span{blob.size(), r.size()};
            blob += r;
        }
        std::vector<int32_t> st(n, 99);
        (void)dfs_store_hash_responses_check(blob.empty() ? nullptr : blob.data(), sp.data(), n, idx.data(), dig.data(), st.data());
        for (int32_t s : st) {
            if (s == DFS_OK) ++ok;
            else if (s == DFS_E_FRAG_MISMATCH) ++mismatch;
            else if (s == DFS_E_WIRE) ++wire;
            else return 2;
        }
    }
    std::printf("wire_sanitize_drv: 200000 replies: %ld accepted, %ld mismatch, %ld parser exceptions\n", ok, mismatch, wire);
    return ok > 0 && mismatch > 0 && wire > 0 ? 0 : 3;
}
