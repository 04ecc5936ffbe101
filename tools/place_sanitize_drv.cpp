// Sanitizer driver (ASan + UBSan) for the pure-host parts of placement.cpp and
// replica.cpp: the transfer schedules (dfs_place_plan), the runner under the
// in-process RCCL stand-in (dfs_place_simulate) and the replica layout
// (dfs_replica_layout), over many world sizes, fragment counts, ragged and
// empty groups and offline masks; then the host-staged communicator's
// mailboxes (hostcomm.cpp) with one thread per rank and host-memory messages
// from one byte to several chunks.  Host-only: the kernel launchers and ctx
// accessors are stubbed, no device is touched.  Run tools/place_sanitize.sh.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <random>
#include <thread>
#include <vector>
#include "dfs_gpu.h"
#include "dfs_internal.h"
#include "placement_internal.h"
namespace dfs {
hipStream_t ctx_stream(dfs_ctx*) { return nullptr; }
int ctx_device(dfs_ctx*) { return 0; }
hipError_t ctx_aux_stream(dfs_ctx*, hipStream_t* aux) { *aux = nullptr; return hipSuccess; }
uint32_t sort_sha_lanes(std::vector<ShaDesc>&) { return 0; }
uint64_t finish_stream_jobs(std::vector<StreamJob>&, const std::vector<uint64_t>&, uint64_t) { return 0; }
uint64_t decode_items(uint64_t, uintptr_t) { return 1; }
hipError_t launch_fill_u32(uint32_t*, uint64_t, uint32_t, hipStream_t) { return hipSuccess; }
hipError_t launch_digest_transpose(const uint8_t*, uint8_t*, uint32_t, uint32_t, hipStream_t) { return hipSuccess; }
hipError_t launch_replica_verdict(const int32_t*, const uint8_t*, const uint8_t*, uint64_t, const uint64_t*, const uint32_t*,
                                  uint32_t, int32_t, int32_t, int32_t*, uint32_t*, hipStream_t) { return hipSuccess; }
hipError_t launch_b64_decode(const char*, const StreamJob*, uint32_t, uint64_t, uint8_t*, int32_t*, uint64_t*, hipStream_t,
                             uint32_t, uint32_t, const StreamAhead*) { return hipSuccess; }
hipError_t launch_sha256(const uint8_t*, const ShaDesc*, uint32_t, uint32_t, uint32_t, uint8_t*, uint8_t*, uint32_t*, int,
                         hipStream_t, uint32_t*, char*, const ShaWait*) { return hipSuccess; }
hipError_t launch_sha256_b64dec(const char*, const DecLane*, uint32_t, uint8_t*, uint8_t*, int32_t*, uint32_t*, int,
                                hipStream_t, uint64_t*) { return hipSuccess; }
}  // namespace dfs

static int fail(const char* what, uint32_t W, uint32_t N) {
    std::printf("FAIL %s W=%u N=%u: %s\n", what, W, N, dfs_comm_last_error());
    return 1;
}

// Every rank sends two messages to every other rank per round and receives
// theirs; message (from, to, k, round) has a length and bytes both sides can
// compute.
static uint64_t msg_len(uint32_t from, uint32_t to, uint32_t k, uint32_t round) {
    static const uint64_t sizes[] = {1, 7, 4096, (4ull << 20) - 1, 4ull << 20, (4ull << 20) + 1, (9ull << 20) + 13, 70000};
    return sizes[(from * 7 + to * 3 + k * 5 + round) % 8];
}
static uint8_t msg_byte(uint32_t from, uint32_t to, uint32_t k, uint32_t round, uint64_t i) {
    return static_cast<uint8_t>(from * 31 + to * 17 + k * 5 + round * 3 + i * 7 + (i >> 11));
}

static int host_comm_cases() {
    int cases = 0;
    for (uint32_t W : {2u, 3u, 5u}) {
        uint8_t id[DFS_COMM_ID_BYTES];
        if (dfs::host_comm_make_id(id) != DFS_OK || !dfs::host_comm_is_id(id)) return -1;
        std::atomic<int> bad{0};
        std::vector<std::thread> th;
        for (uint32_t me = 0; me < W; ++me)
            th.emplace_back([&, me] {
                dfs::HostComm* h = nullptr;
                if (dfs::host_comm_open(id, W, me, &h) != DFS_OK) {
                    ++bad;
                    return;
                }
                for (uint32_t round = 0; round < 3; ++round) {
                    std::vector<std::vector<uint8_t>> out, in;
                    std::vector<dfs::HostOp> ops;
                    for (uint32_t k = 0; k < 2; ++k)
                        for (uint32_t r = 0; r < W; ++r) {
                            if (r == me) continue;
                            out.emplace_back(msg_len(me, r, k, round));
                            for (uint64_t i = 0; i < out.back().size(); ++i) out.back()[i] = msg_byte(me, r, k, round, i);
                            in.emplace_back(msg_len(r, me, k, round), 0xEE);
                        }
                    size_t q = 0;
                    for (uint32_t k = 0; k < 2; ++k)
                        for (uint32_t r = 0; r < W; ++r) {
                            if (r == me) continue;
                            // receives before sends on odd ranks: the order of posting across peers must not matter
                            dfs::HostOp snd{true, out[q].data(), out[q].size(), r, false};
                            dfs::HostOp rcv{false, in[q].data(), in[q].size(), r, false};
                            if (me & 1) ops.push_back(rcv), ops.push_back(snd);
                            else ops.push_back(snd), ops.push_back(rcv);
                            ++q;
                        }
                    if (dfs::host_comm_exchange(h, ops) != DFS_OK) ++bad;
                    q = 0;
                    for (uint32_t k = 0; k < 2; ++k)
                        for (uint32_t r = 0; r < W; ++r) {
                            if (r == me) continue;
                            for (uint64_t i = 0; i < in[q].size(); ++i)
                                if (in[q][i] != msg_byte(r, me, k, round, i)) {
                                    ++bad;
                                    break;
                                }
                            ++q;
                        }
                }
                dfs::host_comm_close(h);
            });
        for (auto& t : th) t.join();
        if (bad.load()) return -1;
        ++cases;
    }
    return cases;
}

// Failure handling of the host-staged communicator, with a 1 s limit: a rank
// that never joins, a peer that posts nothing, two sides that disagree on a
// size.  Every call must come back with DFS_E_COMM, none may hang.
static int host_comm_failures() {
    setenv("DFS_HOST_COMM_TIMEOUT_S", "1", 1);
    uint8_t id[DFS_COMM_ID_BYTES];
    // 1. two of three ranks show up: the rendezvous gives up
    if (dfs::host_comm_make_id(id) != DFS_OK) return -1;
    {
        std::atomic<int> comm_err{0};
        std::vector<std::thread> th;
        for (uint32_t me = 0; me < 2; ++me)
            th.emplace_back([&, me] {
                dfs::HostComm* h = nullptr;
                if (dfs::host_comm_open(id, 3, me, &h) == DFS_E_COMM && !h) ++comm_err;
            });
        for (auto& t : th) t.join();
        if (comm_err.load() != 2) return -1;
    }
    // 2. rank 1 posts nothing: rank 0's receive gives up; 3. sizes differ: the receiver refuses
    for (int scenario = 0; scenario < 2; ++scenario) {
        if (dfs::host_comm_make_id(id) != DFS_OK) return -1;
        std::atomic<int> good{0};
        std::vector<std::thread> th;
        for (uint32_t me = 0; me < 2; ++me)
            th.emplace_back([&, me] {
                dfs::HostComm* h = nullptr;
                if (dfs::host_comm_open(id, 2, me, &h) != DFS_OK) return;
                std::vector<uint8_t> buf(1000, 7);
                std::vector<dfs::HostOp> ops;
                if (scenario == 0) {
                    if (me == 0) ops.push_back(dfs::HostOp{false, buf.data(), 100, 1, false});
                    const int rc = dfs::host_comm_exchange(h, ops);
                    if (rc == (me == 0 ? DFS_E_COMM : DFS_OK)) ++good;
                } else {
                    if (me == 0) ops.push_back(dfs::HostOp{true, buf.data(), 200, 1, false});
                    else ops.push_back(dfs::HostOp{false, buf.data(), 100, 0, false});
                    const int rc = dfs::host_comm_exchange(h, ops);
                    if (rc == (me == 0 ? DFS_OK : DFS_E_COMM)) ++good;  // the sender's chunk fitted its mailbox
                }
                dfs::host_comm_close(h);
            });
        for (auto& t : th) t.join();
        if (good.load() != 2) return -1;
    }
    unsetenv("DFS_HOST_COMM_TIMEOUT_S");
    return 3;
}

int main() {
    std::mt19937_64 rng(20261113);
    int cases = 0;
    const int hf = host_comm_failures();
    if (hf < 0) {
        std::printf("FAIL host-staged communicator failure handling\n");
        return 1;
    }
    cases += hf;
    const int hc = host_comm_cases();
    if (hc < 0) {
        std::printf("FAIL host-staged communicator\n");
        return 1;
    }
    cases += hc;
    for (uint32_t W : {1u, 2u, 3u, 4u, 5u, 7u, 8u, 16u, 64u})
        for (uint32_t N : {1u, 2u, 3u, 5u, 8u, 10u, 64u}) {
            std::vector<uint64_t> table(static_cast<size_t>(W) * N);
            for (auto& t : table) t = rng() % 5 == 0 ? 0 : rng() % 300;
            std::vector<std::vector<uint8_t>> src(W), held(W);
            std::vector<const uint8_t*> sp(W);
            std::vector<uint8_t*> dp(W);
            for (uint32_t mode : {DFS_PLACE_RING, DFS_PLACE_STAR}) {
                for (uint32_t r = 0; r < W; ++r) {
                    uint64_t n = 0;
                    for (uint32_t f = 0; f < N; ++f) n += table[static_cast<size_t>(r) * N + f];
                    src[r].assign(n + 1, 0);
                    for (auto& b : src[r]) b = static_cast<uint8_t>(rng());
                    std::vector<uint64_t> off(N + 1);
                    uint32_t nops = 0;
                    if (dfs_place_plan(W, r, N, table.data(), mode, 0, nullptr, &nops, off.data(), nullptr)) return fail("plan", W, N);
                    std::vector<dfs_xfer> ops(nops + 1);
                    if (dfs_place_plan(W, r, N, table.data(), mode, 0, ops.data(), &nops, nullptr, nullptr)) return fail("plan ops", W, N);
                    held[r].assign(off[N] + 1, 0);
                    sp[r] = src[r].data();
                    dp[r] = held[r].data();
                }
                if (dfs_place_simulate(W, N, table.data(), mode, 0, sp.data(), dp.data(), nullptr)) return fail("simulate", W, N);
                ++cases;
            }
            // degraded fetch out of the star's held buffers, one or two ranks offline
            for (uint64_t mask : {0ull, 1ull, 1ull << (W - 1), W > 2 ? 3ull : 0ull}) {
                std::vector<std::vector<uint8_t>> out(W);
                std::vector<const uint8_t*> hp(W);
                std::vector<uint8_t*> op(W);
                std::vector<int32_t> st(static_cast<size_t>(W) * N);
                for (uint32_t r = 0; r < W; ++r) {
                    out[r].assign(src[r].size() + 1, 0);
                    hp[r] = held[r].data();
                    op[r] = out[r].data();
                }
                if (dfs_place_simulate(W, N, table.data(), DFS_PLACE_FETCH, mask, hp.data(), op.data(), st.data()))
                    return fail("fetch", W, N);
                if (!mask)
                    for (uint32_t r = 0; r < W; ++r)
                        if (std::memcmp(out[r].data(), src[r].data(), src[r].size() - 1)) return fail("fetch bytes", W, N);
                ++cases;
            }
            // replica layout: ragged file counts and lengths, both alignments
            std::vector<uint32_t> nfiles(W);
            std::vector<uint64_t> lens;
            for (uint32_t r = 0; r < W; ++r) {
                nfiles[r] = static_cast<uint32_t>(rng() % 5);
                for (uint32_t j = 0; j < nfiles[r]; ++j) lens.push_back(rng() % 3 == 0 ? rng() % (N + 2) : rng() % 70000);
            }
            for (uint32_t flags : {0u, static_cast<uint32_t>(DFS_LAYOUT_ALIGN128)})
                for (uint32_t me = 0; me < W; me += (W > 8 ? 7 : 1)) {
                    uint64_t n = 0, heldb = 0, rawb = 0;
                    std::vector<uint64_t> t2(static_cast<size_t>(W) * N);
                    if (dfs_replica_layout(W, me, N, nfiles.data(), lens.empty() ? nullptr : lens.data(), flags, nullptr, &n,
                                           t2.data(), &heldb, &rawb) != DFS_OK && !lens.empty())
                        return fail("layout count", W, N);
                    std::vector<dfs_held_frag> fr(n + 1);
                    uint64_t cap = n;
                    if (!lens.empty() && dfs_replica_layout(W, me, N, nfiles.data(), lens.data(), flags, fr.data(), &cap, nullptr,
                                                            nullptr, nullptr))
                        return fail("layout frags", W, N);
                    for (uint64_t k = 0; k < n; ++k)
                        if (fr[k].b64_off + fr[k].b64_len > heldb || fr[k].raw_off + fr[k].raw_len > rawb) return fail("layout bounds", W, N);
                    ++cases;
                }
        }
    std::printf("placement sanitize driver OK (%d cases)\n", cases);
    return 0;
}
