// Sanitizer driver (ThreadSanitizer / ASan+UBSan) for the fragment store host mode: pool, latches, chunking.
// Host-only: the ctx accessors are stubbed, no device is touched.  Run tools/store_sanitize.sh.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include "dfs_gpu.h"
#include "dfs_internal.h"
namespace dfs {
hipStream_t ctx_stream(dfs_ctx*) { return nullptr; }
int ctx_device(dfs_ctx*) { return 0; }
std::mutex& ctx_mutex(dfs_ctx*) { static std::mutex m; return m; }
StoreStaging*& ctx_store(dfs_ctx*) { static StoreStaging* s = nullptr; return s; }
}
int main() {
    setenv("DFS_STORE_SLOT_MB", "1", 1);
    const std::string dir = std::string(std::getenv("TMPDIR") ? std::getenv("TMPDIR") : "/tmp") + "/dfs_store_sanitize";
    const int nf = 64;
    std::vector<uint8_t> dig(32 * nf);
    for (size_t i = 0; i < dig.size(); ++i) dig[i] = uint8_t((i % 32) * 13 + i / 32);
    std::vector<dfs_frag_ref> refs;
    uint64_t pos = 0;
    for (int f = 0; f < nf; ++f)
        for (int i = 0; i < 2; ++i) {
            uint64_t len = (f % 7 == 0) ? (3u << 20) + f : 1000u * f + i;
            refs.push_back({pos, len, uint32_t(f), uint32_t(i)});
            pos += len;
        }
    std::vector<uint8_t> data(pos), back(pos);
    for (size_t i = 0; i < pos; ++i) data[i] = uint8_t(i * 131 + (i >> 9));
    std::vector<int32_t> st(refs.size());
    std::vector<uint64_t> len(refs.size());
    for (int it = 0; it < 3; ++it) {
        int rc = dfs_store_write_fragments(nullptr, dir.c_str(), dig.data(), uint32_t(nf), data.data(), refs.data(), refs.size(), st.data(), 0);
        int rc2 = dfs_store_read_fragments(nullptr, dir.c_str(), dig.data(), uint32_t(nf), back.data(), refs.data(), refs.size(), len.data(), st.data(), 0);
        if (rc || rc2 || back != data) { std::printf("FAIL %d %d\n", rc, rc2); return 1; }
    }
    std::printf("store sanitize driver OK (%zu refs, %llu bytes)\n", refs.size(), (unsigned long long)pos);
    return 0;
}
