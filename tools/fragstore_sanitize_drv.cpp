// fragstore_sanitize_drv.cpp — the on-disk fragment store's staging ring and
// I/O thread pool (csrc/fragstore.cpp) under ThreadSanitizer /
// AddressSanitizer + UBSan, without a GPU: built against the host stand-ins
// for the HIP calls (tools/batcher_sanitize/hip), "device" memory is host
// memory.  Fragments from one byte to several staging slots are written in
// device mode and in host mode, read back both ways and compared; then the
// reference's miss cases (tryLoadFragmentLocal returns null, SN:463-469), a
// too-small read buffer, and two threads using two ctxs at once.
//
//   fragstore_sanitize_drv <scratch dir>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../include/dfs_gpu.h"
#include "../distributed-file-storage_amd/csrc/dfs_internal.h"

struct dfs_ctx {
    std::mutex store_mu;
    dfs::StoreStaging* store = nullptr;
};

namespace dfs {
hipStream_t ctx_stream(dfs_ctx*) { return nullptr; }
int ctx_device(dfs_ctx*) { return 0; }
std::mutex& ctx_store_mutex(dfs_ctx* c) { return c->store_mu; }
StoreStaging*& ctx_store(dfs_ctx* c) { return c->store; }
hipError_t quiet_wait(hipEvent_t) { return hipSuccess; }
}  // namespace dfs

namespace {

std::atomic<int> g_fail{0};
#define CHECK(c)                                                                                            \
    do {                                                                                                    \
        if (!(c) && g_fail.fetch_add(1) < 10) std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
    } while (0)

uint8_t byte_of(uint32_t seed, uint64_t i) { return static_cast<uint8_t>(seed * 131 + i * 7 + (i >> 9)); }

void round_trip(dfs_ctx* ctx, const std::string& root, uint32_t seed) {
    // 3 files x 5 fragments, lengths from 0 to a few staging slots (1 MiB slots in this build)
    const uint64_t lens[] = {0, 1, 4095, 65536, (1ull << 20) - 1, 1ull << 20, (1ull << 20) + 1, (3ull << 20) + 17};
    const uint32_t nfiles = 3, nfrag = 5;
    std::vector<uint8_t> dig(32 * nfiles);
    for (size_t i = 0; i < dig.size(); ++i) dig[i] = byte_of(seed + 9, i);
    std::vector<dfs_frag_ref> refs;
    uint64_t total = 0;
    for (uint32_t f = 0; f < nfiles; ++f)
        for (uint32_t k = 0; k < nfrag; ++k) {
            const uint64_t n = lens[(seed + f * nfrag + k) % 8];
            refs.push_back(dfs_frag_ref{total, n, f, k});
            total += n + 3;  // odd gaps: unaligned sources
        }
    std::vector<uint8_t> data(total + 1), back(total + 1, 0xEE);
    for (uint64_t i = 0; i < total; ++i) data[i] = byte_of(seed, i);
    const uint32_t n = static_cast<uint32_t>(refs.size());
    std::vector<int32_t> st(n, 99);
    for (uint32_t flags : {static_cast<uint32_t>(DFS_DEVICE_PTRS), 0u}) {
        const std::string r = root + (flags ? "/dev" : "/host");
        CHECK(dfs_store_write_fragments(ctx, r.c_str(), dig.data(), nfiles, data.data(), refs.data(), n, st.data(), flags) == DFS_OK);
        for (int32_t s : st) CHECK(s == DFS_OK);
        for (uint32_t rflags : {static_cast<uint32_t>(DFS_DEVICE_PTRS), 0u}) {
            std::fill(back.begin(), back.end(), 0xEE);
            std::vector<uint64_t> got(n, 0);
            CHECK(dfs_store_read_fragments(ctx, r.c_str(), dig.data(), nfiles, back.data(), refs.data(), n, got.data(), st.data(), rflags) == DFS_OK);
            for (uint32_t i = 0; i < n; ++i) {
                CHECK(st[i] == DFS_OK && got[i] == refs[i].len);
                CHECK(!std::memcmp(back.data() + refs[i].off, data.data() + refs[i].off, refs[i].len));
                CHECK(back[refs[i].off + refs[i].len] == 0xEE);  // nothing past the fragment
            }
        }
        // a fragment nobody stored, and a read buffer shorter than the file
        std::vector<dfs_frag_ref> odd = {dfs_frag_ref{0, 100, 0, 77}, refs[n - 1]};
        if (odd[1].len) odd[1].len -= 1;
        std::vector<uint64_t> got(2, 0);
        std::vector<int32_t> st2(2, 99);
        const int rc = dfs_store_read_fragments(ctx, r.c_str(), dig.data(), nfiles, back.data(), odd.data(), 2, got.data(), st2.data(), flags);
        CHECK(st2[0] == DFS_E_MISSING);
        CHECK(refs[n - 1].len == 0 || st2[1] == DFS_E_ARG);
        CHECK(rc != DFS_OK);
    }
    // a file index out of range is refused before any I/O
    dfs_frag_ref bad{0, 1, nfiles, 0};
    int32_t s1 = 99;
    CHECK(dfs_store_write_fragments(ctx, root.c_str(), dig.data(), nfiles, data.data(), &bad, 1, &s1, 0) == DFS_E_ARG);
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    const std::string root = argv[1];
    dfs_ctx a, b;
    round_trip(&a, root + "/one", 1);
    std::thread t1([&] { for (uint32_t s = 2; s < 5; ++s) round_trip(&a, root + "/a" + std::to_string(s), s); });
    std::thread t2([&] { for (uint32_t s = 5; s < 8; ++s) round_trip(&b, root + "/b" + std::to_string(s), s); });
    t1.join();
    t2.join();
    dfs::store_staging_free(a.store);
    dfs::store_staging_free(b.store);
    std::printf("fragstore_sanitize_drv: %d failed checks\n", g_fail.load());
    return g_fail.load() ? 1 : 0;
}
