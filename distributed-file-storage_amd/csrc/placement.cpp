// placement.cpp — replica placement and degraded fetch across GPUs over RCCL
// (include/dfs_gpu.h, dfs_comm_* / dfs_place_*).
//
// Reference (StorageNode.java, SN:line): node k (0-based) stores fragments
// {k, (k+1) mod N} (:143-145, :199-200); the uploader sends every peer its
// pair (star fan-out, :195-224; the receiver checks the hashes, :248-257);
// a download takes fragment i locally, else from node i, else from node i-1
// (:422-440), and fails with "Could not retrieve fragment i" (:443-446).
//
// MI355X mapping: one rank per GPU, node k hosted by rank
// k mod W.  A rank's Base64 is fragment-major: group f = the Base64 of
// fragment f of every file the rank uploaded, groups back to back.  After a
// placement every rank holds, for each fragment f it hosts, "held group f" =
// group f of rank 0, rank 1, ... concatenated in rank order.
//
//   RING  primary scatter (group f -> the rank of node f) then the replica
//         step (that rank forwards held group f to the rank of node f-1):
//         with W == N the ring g -> g-1 of north_star, one xGMI link per GPU
//         (BASELINE "GPU g sends to g+1" under the relabel node k <-> GPU k+1).
//   STAR  the reference's own fan-out as one all-to-all: group f goes
//         straight from its uploader to both holders, every link busy.
//   FETCH degraded read: every live rank gets its own groups back from the
//         first live holder in SN:427-428 order.
//
// The transfer schedule is a pure host function (dfs_place_plan), so it is
// checked on the CPU by simulating every rank in one process
// (tests/test_placement_plan.py); the runner only issues its ops:
// ncclSend / ncclRecv inside ncclGroupStart / End per phase, local copies as
// device-to-device hipMemcpyAsync, all on the ctx stream.  Between a pair of
// ranks sends and receives are issued in the same order on both sides, which
// is how RCCL matches them.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include <map>
#include <utility>

#include "../../include/dfs_gpu.h"
#include "dfs_internal.h"
#include "placement_internal.h"

static_assert(DFS_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "unique id size");

struct dfs_comm {
    dfs_ctx* ctx = nullptr;
    ncclComm_t nc = nullptr;       // RCCL communicator, or
    dfs::HostComm* host = nullptr; // shared-memory mailboxes (hostcomm.cpp): exactly one of the two
    uint32_t nranks = 0, rank = 0;
    uint64_t* d_gather = nullptr; // allgather_u64 scratch
    uint64_t gather_cap = 0;      // words
    // DFS_COMM_LOOPBACK=1 when the comm was made: a rank's local copies go
    // through ncclSend / ncclRecv to itself inside the phase's group instead of
    // hipMemcpyAsync, so a one-rank run drives the same RCCL calls, group
    // bracketing and stream ordering as a many-rank one.  For tests.
    bool loopback = false;
    uint64_t issued[3] = {0, 0, 0};  // sends, receives, local copies (dfs_comm_counters)
};

namespace {
bool env_loopback() {
    const char* e = std::getenv("DFS_COMM_LOOPBACK");
    return e && e[0] == '1';
}
}  // namespace

using dfs::holder_a;
using dfs::holder_b;
using dfs::holds;
using dfs::kMaxFrag;
using dfs::kMaxRanks;
using dfs::Plan;

namespace {

thread_local char g_last_comm[160];

int comm_fail(ncclResult_t r, const char* what) {
    std::snprintf(g_last_comm, sizeof g_last_comm, "%s: %s", what, ncclGetErrorString(r));
    return DFS_E_COMM;
}

#define NCCLC(x)                                        \
    do {                                                \
        ncclResult_t r_ = (x);                          \
        if (r_ != ncclSuccess) return comm_fail(r_, #x); \
    } while (0)
#define HIPCHK(x)                                       \
    do {                                                \
        if ((x) != hipSuccess) return DFS_E_HIP;        \
    } while (0)

// Bytes of rank r's group f.
inline uint64_t T(const uint64_t* table, uint32_t N, uint32_t r, uint32_t f) { return table[static_cast<uint64_t>(r) * N + f]; }

void add(Plan& p, uint32_t phase, uint32_t kind, int32_t peer, uint32_t f, uint32_t from_dst, uint64_t src, uint64_t dst,
         uint64_t len) {
    if (!len) return;  // both sides skip empty transfers (they see the same table)
    dfs_xfer x{};
    x.phase = phase;
    x.kind = kind;
    x.peer = peer;
    x.frag = f;
    x.from_dst = from_dst;
    x.src_off = src;
    x.dst_off = dst;
    x.len = len;
    p.ops.push_back(x);
}

}  // namespace

int dfs::build_plan(uint32_t W, uint32_t me, uint32_t N, const uint64_t* table, uint32_t mode, uint64_t offline, Plan& p) {
    if (!W || W > kMaxRanks || me >= W || !N || N > kMaxFrag || !table) return DFS_E_ARG;
    if (mode > DFS_PLACE_FETCH) return DFS_E_ARG;
    p.ops.clear();
    p.dst_off.assign(N + 1, 0);
    p.status.assign(N, DFS_OK);
    // own group offsets in the fragment-major source (groups back to back)
    std::vector<uint64_t> goff(N + 1, 0);
    for (uint32_t f = 0; f < N; ++f) goff[f + 1] = goff[f] + T(table, N, me, f);
    // position of rank r's piece inside held group f
    auto piece = [&](uint32_t f, uint32_t r) {
        uint64_t o = 0;
        for (uint32_t q = 0; q < r; ++q) o += T(table, N, q, f);
        return o;
    };
    auto total = [&](uint32_t f) { return piece(f, W); };
    if (mode == DFS_PLACE_FETCH) {
        for (uint32_t f = 0; f <= N; ++f) p.dst_off[f] = goff[f];  // same layout as the source groups
    } else {
        uint64_t o = 0;
        for (uint32_t f = 0; f < N; ++f) {
            if (holds(me, f, N, W)) {
                p.dst_off[f] = o;
                o += total(f);
            } else {
                p.dst_off[f] = UINT64_MAX;
            }
        }
        p.dst_off[N] = o;
    }
    const uint64_t* H = p.dst_off.data();
    if (mode == DFS_PLACE_RING) {
        p.phases = 2;
        // phase 0: primary scatter, group f -> rank of node f
        for (uint32_t f = 0; f < N; ++f) {
            const uint32_t a = holder_a(f, N, W);
            if (a == me) {
                for (uint32_t r = 0; r < W; ++r) {
                    if (r == me) add(p, 0, DFS_XFER_COPY, -1, f, 0, goff[f], H[f] + piece(f, r), T(table, N, r, f));
                    else add(p, 0, DFS_XFER_RECV, static_cast<int32_t>(r), f, 0, 0, H[f] + piece(f, r), T(table, N, r, f));
                }
            } else {
                add(p, 0, DFS_XFER_SEND, static_cast<int32_t>(a), f, 0, goff[f], 0, T(table, N, me, f));
            }
        }
        // phase 1: replica step, rank of node f -> rank of node f-1
        for (uint32_t f = 0; f < N; ++f) {
            const uint32_t a = holder_a(f, N, W), b = holder_b(f, N, W);
            if (a == b) continue;
            if (me == a) add(p, 1, DFS_XFER_SEND, static_cast<int32_t>(b), f, 1, H[f], 0, total(f));
            else if (me == b) add(p, 1, DFS_XFER_RECV, static_cast<int32_t>(a), f, 0, 0, H[f], total(f));
        }
    } else if (mode == DFS_PLACE_STAR) {
        p.phases = 1;
        for (uint32_t g = 0; g < W; ++g)
            for (uint32_t f = 0; f < N; ++f) {
                if (!holds(g, f, N, W)) continue;
                if (g == me) add(p, 0, DFS_XFER_COPY, -1, f, 0, goff[f], H[f] + piece(f, me), T(table, N, me, f));
                else add(p, 0, DFS_XFER_SEND, static_cast<int32_t>(g), f, 0, goff[f], 0, T(table, N, me, f));
            }
        for (uint32_t f = 0; f < N; ++f) {
            if (!holds(me, f, N, W)) continue;
            for (uint32_t r = 0; r < W; ++r)
                if (r != me) add(p, 0, DFS_XFER_RECV, static_cast<int32_t>(r), f, 0, 0, H[f] + piece(f, r), T(table, N, r, f));
        }
    } else {  // FETCH
        p.phases = 1;
        auto off = [&](uint32_t g) { return (offline >> g) & 1u; };
        // every rank walks every requester's plan so both sides of each
        // transfer are issued in the same order
        for (uint32_t q = 0; q < W; ++q) {
            if (off(q)) continue;
            for (uint32_t f = 0; f < N; ++f) {
                int32_t s = -1;
                if (holds(q, f, N, W)) s = static_cast<int32_t>(q);  // tryLoadFragmentLocal, SN:423
                else if (!off(holder_a(f, N, W))) s = static_cast<int32_t>(holder_a(f, N, W));  // nodeA, SN:427
                else if (!off(holder_b(f, N, W))) s = static_cast<int32_t>(holder_b(f, N, W));  // nodeB, SN:428
                if (s < 0) {
                    if (q == me) p.status[f] = DFS_E_MISSING;  // SN:443-446
                    continue;
                }
                const uint64_t len = T(table, N, q, f);
                if (static_cast<uint32_t>(s) == me) {
                    // serve q's piece of my held group f (dst_off of the server's layout)
                    uint64_t ho = 0;
                    for (uint32_t h = 0; h < f; ++h)
                        if (holds(me, h, N, W)) ho += total(h);
                    if (q == me) add(p, 0, DFS_XFER_COPY, -1, f, 0, ho + piece(f, q), H[f], len);
                    else add(p, 0, DFS_XFER_SEND, static_cast<int32_t>(q), f, 0, ho + piece(f, q), 0, len);
                } else if (q == me) {
                    add(p, 0, DFS_XFER_RECV, s, f, 0, 0, H[f], len);
                }
            }
        }
        if (offline >> me & 1u)  // an offline rank neither serves nor requests
            for (uint32_t f = 0; f < N; ++f) p.status[f] = DFS_E_MISSING;
    }
    return DFS_OK;
}

namespace dfs {

int run_plans(Transport& t, const std::vector<Plan>& plans, const void* const* src, void* const* dst) {
    const uint32_t n = static_cast<uint32_t>(plans.size());
    uint32_t phases = 0;
    for (const Plan& p : plans) phases = p.phases > phases ? p.phases : phases;
    for (uint32_t ph = 0; ph < phases; ++ph) {
        // local copies first (same stream as the group: ordered before it)
        for (uint32_t i = 0; i < n; ++i)
            for (const dfs_xfer& x : plans[i].ops) {
                if (x.phase != ph || x.kind != DFS_XFER_COPY || t.self_peer(i) >= 0) continue;
                const char* from = x.from_dst ? static_cast<const char*>(dst[i]) : static_cast<const char*>(src[i]);
                if (int rc = t.copy(i, static_cast<char*>(dst[i]) + x.dst_off, from + x.src_off, x.len)) return rc;
            }
        bool any = false;
        for (uint32_t i = 0; i < n && !any; ++i)
            for (const dfs_xfer& x : plans[i].ops)
                if (x.phase == ph && (x.kind != DFS_XFER_COPY || t.self_peer(i) >= 0)) {
                    any = true;
                    break;
                }
        if (!any) continue;
        if (int rc = t.group_start()) return rc;
        for (uint32_t i = 0; i < n; ++i)
            for (const dfs_xfer& x : plans[i].ops) {
                if (x.phase != ph || (x.kind == DFS_XFER_COPY && t.self_peer(i) < 0)) continue;
                int rc;
                if (x.kind == DFS_XFER_COPY) {
                    const char* from = x.from_dst ? static_cast<const char*>(dst[i]) : static_cast<const char*>(src[i]);
                    rc = t.send(i, from + x.src_off, x.len, t.self_peer(i));
                    if (!rc) rc = t.recv(i, static_cast<char*>(dst[i]) + x.dst_off, x.len, t.self_peer(i));
                } else if (x.kind == DFS_XFER_SEND) {
                    const char* from = x.from_dst ? static_cast<const char*>(dst[i]) : static_cast<const char*>(src[i]);
                    rc = t.send(i, from + x.src_off, x.len, x.peer);
                } else {
                    rc = t.recv(i, static_cast<char*>(dst[i]) + x.dst_off, x.len, x.peer);
                }
                if (rc) {
                    (void)t.group_end();
                    return rc;
                }
            }
        if (int rc = t.group_end()) return rc;
    }
    return DFS_OK;
}

// RCCL: every op on its comm's ctx stream, sends and receives of a phase
// inside one ncclGroupStart / End.
struct RcclTransport : Transport {
    dfs_comm* const* comms;
    uint32_t ncomms;
    RcclTransport(dfs_comm* const* c, uint32_t n) : comms(c), ncomms(n) {}
    int use(uint32_t i) {
        HIPCHK(hipSetDevice(dfs::ctx_device(comms[i]->ctx)));
        return DFS_OK;
    }
    int copy(uint32_t i, void* dst, const void* src, uint64_t n) override {
        if (int rc = use(i)) return rc;
        HIPCHK(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, dfs::ctx_stream(comms[i]->ctx)));
        ++comms[i]->issued[2];
        return DFS_OK;
    }
    int group_start() override {
        NCCLC(ncclGroupStart());
        return DFS_OK;
    }
    // One transfer goes out as pieces of at most piece_bytes(), the same split
    // on the sending and the receiving side (both know the length), so the
    // pieces pair in posting order like whole transfers do.  RCCL 2.26 was seen
    // to leave parts of a 1.4 GB send-to-self unwritten (358 MB and below were
    // complete); bounded pieces keep every count inside what was checked on
    // hardware, for peers as well.
    static uint64_t piece_bytes() {
        static const uint64_t v = [] {
            const char* e = std::getenv("DFS_COMM_PIECE_MB");
            const long mb = e ? std::atol(e) : 0;
            return (mb > 0 ? static_cast<uint64_t>(mb) : 256ull) << 20;
        }();
        return v;
    }
    int send(uint32_t i, const void* p, uint64_t n, int32_t peer) override {
        if (int rc = use(i)) return rc;
        const char* b = static_cast<const char*>(p);
        for (uint64_t o = 0; o < n; o += piece_bytes()) {  // plans hold no empty transfers
            const uint64_t len = n - o < piece_bytes() ? n - o : piece_bytes();
            const ncclResult_t r = ncclSend(b + o, len, ncclUint8, peer, comms[i]->nc, dfs::ctx_stream(comms[i]->ctx));
            ++comms[i]->issued[0];
            if (r != ncclSuccess) return comm_fail(r, "ncclSend");
        }
        return DFS_OK;
    }
    int recv(uint32_t i, void* p, uint64_t n, int32_t peer) override {
        if (int rc = use(i)) return rc;
        char* b = static_cast<char*>(p);
        for (uint64_t o = 0; o < n; o += piece_bytes()) {  // plans hold no empty transfers
            const uint64_t len = n - o < piece_bytes() ? n - o : piece_bytes();
            const ncclResult_t r = ncclRecv(b + o, len, ncclUint8, peer, comms[i]->nc, dfs::ctx_stream(comms[i]->ctx));
            ++comms[i]->issued[1];
            if (r != ncclSuccess) return comm_fail(r, "ncclRecv");
        }
        return DFS_OK;
    }
    int group_end() override {
        NCCLC(ncclGroupEnd());
        return DFS_OK;
    }
    int32_t self_peer(uint32_t i) const override { return comms[i]->loopback ? static_cast<int32_t>(comms[i]->rank) : -1; }
};

// Host-staged transport (one comm per process): the group's ops are collected
// and run to completion at group_end, after everything queued on the ctx
// stream before them has finished; what the caller queues next sees the data.
struct HostTransport : Transport {
    dfs_comm* c;
    std::vector<HostOp> ops;
    explicit HostTransport(dfs_comm* comm) : c(comm) {}
    int copy(uint32_t, void* dst, const void* src, uint64_t n) override {
        HIPCHK(hipSetDevice(dfs::ctx_device(c->ctx)));
        HIPCHK(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, dfs::ctx_stream(c->ctx)));
        ++c->issued[2];
        return DFS_OK;
    }
    int group_start() override {
        ops.clear();
        return DFS_OK;
    }
    int send(uint32_t, const void* p, uint64_t n, int32_t peer) override {
        ops.push_back(HostOp{true, const_cast<void*>(p), n, static_cast<uint32_t>(peer), true});
        ++c->issued[0];
        return DFS_OK;
    }
    int recv(uint32_t, void* p, uint64_t n, int32_t peer) override {
        ops.push_back(HostOp{false, p, n, static_cast<uint32_t>(peer), true});
        ++c->issued[1];
        return DFS_OK;
    }
    int group_end() override {
        HIPCHK(hipSetDevice(dfs::ctx_device(c->ctx)));
        HIPCHK(hipStreamSynchronize(dfs::ctx_stream(c->ctx)));
        const int rc = host_comm_exchange(c->host, ops);
        if (rc == DFS_E_COMM) std::snprintf(g_last_comm, sizeof g_last_comm, "host transport: a peer stopped answering or sizes differ");
        return rc;
    }
};

int run_plans_rccl(dfs_comm* const* comms, uint32_t ncomms, const std::vector<Plan>& plans, const void* const* src,
                   void* const* dst) {
    if (comms[0]->host) {
        HostTransport t(comms[0]);
        return run_plans(t, plans, src, dst);
    }
    RcclTransport t(comms, ncomms);
    return run_plans(t, plans, src, dst);
}

// Either RCCL communicators (any number per process) or one host-staged one.
int check_comms(dfs_comm* const* comms, uint32_t ncomms) {
    if (!comms || !ncomms) return DFS_E_ARG;
    for (uint32_t i = 0; i < ncomms; ++i) {
        if (!comms[i] || (!comms[i]->nc && !comms[i]->host) || comms[i]->nranks != comms[0]->nranks) return DFS_E_ARG;
        if (comms[i]->host && ncomms != 1) return DFS_E_ARG;
    }
    return DFS_OK;
}

// All-gather of host words over a host-staged comm.
int host_allgather(dfs_comm* c, const void* mine, uint64_t bytes, void* all) {
    std::vector<HostOp> ops;
    uint8_t* out = static_cast<uint8_t*>(all);
    std::memcpy(out + bytes * c->rank, mine, bytes);
    for (uint32_t r = 0; r < c->nranks; ++r) {
        if (r == c->rank) continue;
        ops.push_back(HostOp{true, const_cast<void*>(mine), bytes, r, false});
        ops.push_back(HostOp{false, out + bytes * r, bytes, r, false});
    }
    return host_comm_exchange(c->host, ops);
}

dfs_ctx* comm_ctx(const dfs_comm* c) { return c->ctx; }

int allreduce_u32(dfs_comm* const* comms, uint32_t ncomms, uint32_t* const* d_buf, uint32_t count) {
    if (comms[0]->host) {  // gather every rank's words on the host, add, put the sums back
        dfs_comm* c = comms[0];
        hipStream_t s = dfs::ctx_stream(c->ctx);
        HIPCHK(hipSetDevice(dfs::ctx_device(c->ctx)));
        std::vector<uint32_t> mine(count), all(static_cast<size_t>(count) * c->nranks);
        HIPCHK(hipMemcpyAsync(mine.data(), d_buf[0], 4ull * count, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        if (int rc = host_allgather(c, mine.data(), 4ull * count, all.data())) return rc;
        for (uint32_t k = 0; k < count; ++k) {
            uint32_t sum = 0;
            for (uint32_t r = 0; r < c->nranks; ++r) sum += all[static_cast<size_t>(r) * count + k];
            mine[k] = sum;
        }
        HIPCHK(hipMemcpyAsync(d_buf[0], mine.data(), 4ull * count, hipMemcpyHostToDevice, s));
        HIPCHK(hipStreamSynchronize(s));
        return DFS_OK;
    }
    NCCLC(ncclGroupStart());
    for (uint32_t i = 0; i < ncomms; ++i) {
        dfs_comm* c = comms[i];
        ncclResult_t r = ncclSuccess;
        if (hipSetDevice(dfs::ctx_device(c->ctx)) != hipSuccess) r = ncclUnhandledCudaError;
        if (r == ncclSuccess) r = ncclAllReduce(d_buf[i], d_buf[i], count, ncclUint32, ncclSum, c->nc, dfs::ctx_stream(c->ctx));
        if (r != ncclSuccess) {
            (void)ncclGroupEnd();
            return comm_fail(r, "ncclAllReduce");
        }
    }
    NCCLC(ncclGroupEnd());
    return DFS_OK;
}

int allgather_u64(dfs_comm* const* comms, uint32_t ncomms, const uint64_t* const* mine, uint64_t count,
                  uint64_t* const* all) {
    if (!count) return DFS_OK;
    if (comms[0]->host) return host_allgather(comms[0], mine[0], 8 * count, all[0]);
    const uint32_t W = comms[0]->nranks;
    for (uint32_t i = 0; i < ncomms; ++i) {
        dfs_comm* c = comms[i];
        HIPCHK(hipSetDevice(dfs::ctx_device(c->ctx)));
        const uint64_t need = (static_cast<uint64_t>(W) + 1) * count;
        if (c->gather_cap < need) {
            if (c->d_gather) (void)hipFree(c->d_gather);
            c->d_gather = nullptr;
            c->gather_cap = 0;
            HIPCHK(hipMalloc(&c->d_gather, 8 * need));
            c->gather_cap = need;
        }
        HIPCHK(hipMemcpyAsync(c->d_gather + static_cast<uint64_t>(W) * count, mine[i], 8 * count, hipMemcpyHostToDevice,
                              dfs::ctx_stream(c->ctx)));
    }
    NCCLC(ncclGroupStart());
    for (uint32_t i = 0; i < ncomms; ++i) {
        dfs_comm* c = comms[i];
        ncclResult_t r = ncclSuccess;
        if (hipSetDevice(dfs::ctx_device(c->ctx)) != hipSuccess) r = ncclUnhandledCudaError;
        if (r == ncclSuccess)
            r = ncclAllGather(c->d_gather + static_cast<uint64_t>(W) * count, c->d_gather, count, ncclUint64, c->nc,
                              dfs::ctx_stream(c->ctx));
        if (r != ncclSuccess) {
            (void)ncclGroupEnd();
            return comm_fail(r, "ncclAllGather");
        }
    }
    NCCLC(ncclGroupEnd());
    for (uint32_t i = 0; i < ncomms; ++i) {
        dfs_comm* c = comms[i];
        HIPCHK(hipSetDevice(dfs::ctx_device(c->ctx)));
        HIPCHK(hipMemcpyAsync(all[i], c->d_gather, 8ull * W * count, hipMemcpyDeviceToHost, dfs::ctx_stream(c->ctx)));
    }
    for (uint32_t i = 0; i < ncomms; ++i) {
        HIPCHK(hipSetDevice(dfs::ctx_device(comms[i]->ctx)));
        HIPCHK(hipStreamSynchronize(dfs::ctx_stream(comms[i]->ctx)));
    }
    return DFS_OK;
}

}  // namespace dfs

namespace {

using dfs::check_comms;

// In-process stand-in for RCCL's group semantics over host memory, one
// endpoint per rank: what a group posts is held until group_end, which pairs
// rank a's sends to b with b's receives from a in posting order, requires
// equal counts and equal sizes (RCCL would hang or corrupt otherwise), rejects
// a group in which a send reads bytes that a receive or another send's peer
// writes in the same group (their order is undefined on the wire), and only
// then moves the bytes.
struct SimTransport : dfs::Transport {
    struct Op {
        const char* src = nullptr;
        char* dst = nullptr;
        uint64_t n = 0;
    };
    uint32_t W;
    bool open = false;
    bool loop = env_loopback();  // copies as self send / receive pairs, as on an RCCL comm made with the same setting
    std::map<std::pair<uint32_t, uint32_t>, std::vector<Op>> sends, recvs;  // key = (from, to)
    std::string err;
    explicit SimTransport(uint32_t w) : W(w) {}
    int32_t self_peer(uint32_t i) const override { return loop ? static_cast<int32_t>(i) : -1; }
    int fail(const std::string& m) {
        err = m;
        std::snprintf(g_last_comm, sizeof g_last_comm, "simulated exchange: %s", m.c_str());
        return DFS_E_COMM;
    }
    int copy(uint32_t, void* dst, const void* src, uint64_t n) override {
        if (open) return fail("copy inside a group");
        std::memmove(dst, src, n);
        return DFS_OK;
    }
    int group_start() override {
        if (open) return fail("nested group");
        open = true;
        sends.clear();
        recvs.clear();
        return DFS_OK;
    }
    int send(uint32_t i, const void* p, uint64_t n, int32_t peer) override {
        if (!open || peer < 0 || static_cast<uint32_t>(peer) >= W || (static_cast<uint32_t>(peer) == i && !loop))
            return fail("bad send");
        Op o;
        o.src = static_cast<const char*>(p);
        o.n = n;
        sends[{i, static_cast<uint32_t>(peer)}].push_back(o);
        return DFS_OK;
    }
    int recv(uint32_t i, void* p, uint64_t n, int32_t peer) override {
        if (!open || peer < 0 || static_cast<uint32_t>(peer) >= W || (static_cast<uint32_t>(peer) == i && !loop))
            return fail("bad recv");
        Op o;
        o.dst = static_cast<char*>(p);
        o.n = n;
        recvs[{static_cast<uint32_t>(peer), i}].push_back(o);
        return DFS_OK;
    }
    int group_end() override {
        if (!open) return fail("group_end without group_start");
        open = false;
        char buf[128];
        for (const auto& kv : recvs)
            if (!sends.count(kv.first)) {
                std::snprintf(buf, sizeof buf, "%u receives from rank %u on rank %u without a send", static_cast<unsigned>(kv.second.size()),
                              kv.first.first, kv.first.second);
                return fail(buf);
            }
        std::vector<Op> moves;
        for (const auto& kv : sends) {
            const auto it = recvs.find(kv.first);
            const size_t nr = it == recvs.end() ? 0 : it->second.size();
            if (nr != kv.second.size()) {
                std::snprintf(buf, sizeof buf, "rank %u -> %u: %u sends vs %u receives", kv.first.first, kv.first.second,
                              static_cast<unsigned>(kv.second.size()), static_cast<unsigned>(nr));
                return fail(buf);
            }
            for (size_t k = 0; k < nr; ++k) {
                if (kv.second[k].n != it->second[k].n) {
                    std::snprintf(buf, sizeof buf, "rank %u -> %u op %u: send %llu bytes vs receive %llu", kv.first.first,
                                  kv.first.second, static_cast<unsigned>(k), static_cast<unsigned long long>(kv.second[k].n),
                                  static_cast<unsigned long long>(it->second[k].n));
                    return fail(buf);
                }
                Op m;
                m.src = kv.second[k].src;
                m.dst = it->second[k].dst;
                m.n = kv.second[k].n;
                moves.push_back(m);
            }
        }
        // no read of bytes written in the same group, no two writes to the same bytes
        for (size_t a = 0; a < moves.size(); ++a)
            for (size_t b = 0; b < moves.size(); ++b) {
                const Op &x = moves[a], &y = moves[b];
                if (!x.n || !y.n) continue;
                if (x.src < y.dst + y.n && y.dst < x.src + x.n) return fail("a send reads bytes a receive of the same group writes");
                if (a < b && x.dst < y.dst + y.n && y.dst < x.dst + x.n) return fail("two receives of one group overlap");
            }
        for (const Op& m : moves) std::memcpy(m.dst, m.src, m.n);
        return DFS_OK;
    }
};

int place(dfs_comm* const* comms, uint32_t ncomms, uint32_t nfrag, const uint64_t* table, uint32_t mode,
          uint64_t offline, const void* const* src, void* const* dst, int32_t* frag_status) {
    if (int rc = check_comms(comms, ncomms)) return rc;
    if (!src || !dst) return DFS_E_ARG;
    std::vector<Plan> plans(ncomms);
    for (uint32_t i = 0; i < ncomms; ++i) {
        if (int rc = dfs::build_plan(comms[i]->nranks, comms[i]->rank, nfrag, table, mode, offline, plans[i])) return rc;
        if (plans[i].dst_off[nfrag] && !dst[i]) return DFS_E_ARG;
        for (const dfs_xfer& x : plans[i].ops)
            if (x.kind != DFS_XFER_RECV && !x.from_dst && !src[i]) return DFS_E_ARG;
        if (frag_status) std::memcpy(frag_status + static_cast<uint64_t>(i) * nfrag, plans[i].status.data(), 4ull * nfrag);
    }
    return dfs::run_plans_rccl(comms, ncomms, plans, src, dst);
}

}  // namespace

extern "C" {

const char* dfs_comm_last_error(void) { return g_last_comm[0] ? g_last_comm : "RCCL error"; }

int dfs_place_plan(uint32_t nranks, uint32_t rank, uint32_t nfrag, const uint64_t* table, uint32_t mode,
                   uint64_t offline_mask, dfs_xfer* ops, uint32_t* nops, uint64_t* dst_off, int32_t* frag_status) {
    if (!nops) return DFS_E_ARG;
    Plan p;
    if (int rc = dfs::build_plan(nranks, rank, nfrag, table, mode, offline_mask, p)) return rc;
    const uint32_t cap = *nops;
    *nops = static_cast<uint32_t>(p.ops.size());
    if (dst_off) std::memcpy(dst_off, p.dst_off.data(), 8ull * (nfrag + 1));
    if (frag_status) std::memcpy(frag_status, p.status.data(), 4ull * nfrag);
    if (ops) {
        if (cap < p.ops.size()) return DFS_E_ARG;
        if (!p.ops.empty()) std::memcpy(ops, p.ops.data(), sizeof(dfs_xfer) * p.ops.size());
    }
    return DFS_OK;
}

int dfs_place_simulate(uint32_t nranks, uint32_t nfrag, const uint64_t* table, uint32_t mode, uint64_t offline_mask,
                       const uint8_t* const* src, uint8_t* const* dst, int32_t* frag_status) {
    if (!nranks || nranks > kMaxRanks || !src || !dst) return DFS_E_ARG;
    std::vector<Plan> plans(nranks);
    for (uint32_t r = 0; r < nranks; ++r) {
        if (int rc = dfs::build_plan(nranks, r, nfrag, table, mode, offline_mask, plans[r])) return rc;
        if (plans[r].dst_off[nfrag] && !dst[r]) return DFS_E_ARG;
        for (const dfs_xfer& x : plans[r].ops)
            if (x.kind != DFS_XFER_RECV && !x.from_dst && !src[r]) return DFS_E_ARG;
        if (frag_status) std::memcpy(frag_status + static_cast<uint64_t>(r) * nfrag, plans[r].status.data(), 4ull * nfrag);
    }
    SimTransport t(nranks);
    return dfs::run_plans(t, plans, reinterpret_cast<const void* const*>(src), reinterpret_cast<void* const*>(dst));
}

int dfs_comm_unique_id(uint8_t* id) {
    if (!id) return DFS_E_ARG;
    if (const char* t = std::getenv("DFS_COMM_TRANSPORT"))
        if (!std::strcmp(t, "host")) return dfs::host_comm_make_id(id);
    ncclUniqueId u;
    NCCLC(ncclGetUniqueId(&u));
    std::memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
    return DFS_OK;
}

int dfs_comm_init_rank(dfs_ctx* ctx, const uint8_t* id, uint32_t nranks, uint32_t rank, dfs_comm** out) {
    if (!ctx || !id || !out || !nranks || nranks > kMaxRanks || rank >= nranks) return DFS_E_ARG;
    *out = nullptr;
    HIPCHK(hipSetDevice(dfs::ctx_device(ctx)));
    auto* c = new (std::nothrow) dfs_comm;
    if (!c) return DFS_E_NOMEM;
    c->ctx = ctx;
    c->nranks = nranks;
    c->rank = rank;
    if (dfs::host_comm_is_id(id)) {
        const int rc = dfs::host_comm_open(id, nranks, rank, &c->host);
        if (rc != DFS_OK) {
            delete c;
            if (rc == DFS_E_COMM) std::snprintf(g_last_comm, sizeof g_last_comm, "host transport: shared memory rendezvous failed");
            return rc;
        }
        *out = c;
        return DFS_OK;
    }
    ncclUniqueId u;
    std::memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
    ncclResult_t r = ncclCommInitRank(&c->nc, static_cast<int>(nranks), u, static_cast<int>(rank));
    if (r != ncclSuccess) {
        delete c;
        return comm_fail(r, "ncclCommInitRank");
    }
    c->loopback = env_loopback();
    *out = c;
    return DFS_OK;
}

int dfs_comm_init_all(dfs_ctx* const* ctxs, uint32_t n, dfs_comm** out) {
    if (!ctxs || !out || !n || n > kMaxRanks) return DFS_E_ARG;
    std::vector<int> dev(n);
    for (uint32_t i = 0; i < n; ++i) {
        if (!ctxs[i]) return DFS_E_ARG;
        dev[i] = dfs::ctx_device(ctxs[i]);
        out[i] = nullptr;
    }
    std::vector<ncclComm_t> nc(n);
    NCCLC(ncclCommInitAll(nc.data(), static_cast<int>(n), dev.data()));
    for (uint32_t i = 0; i < n; ++i) {
        auto* c = new (std::nothrow) dfs_comm;
        if (!c) {
            for (uint32_t j = 0; j < n; ++j) {
                if (j < i) dfs_comm_destroy(out[j]);
                else (void)ncclCommDestroy(nc[j]);
                out[j] = nullptr;
            }
            return DFS_E_NOMEM;
        }
        c->ctx = ctxs[i];
        c->nc = nc[i];
        c->nranks = n;
        c->rank = i;
        c->loopback = env_loopback();
        out[i] = c;
    }
    return DFS_OK;
}

int dfs_comm_destroy(dfs_comm* c) {
    if (!c) return DFS_E_ARG;
    (void)hipSetDevice(dfs::ctx_device(c->ctx));
    (void)hipStreamSynchronize(dfs::ctx_stream(c->ctx));
    if (c->nc) (void)ncclCommDestroy(c->nc);
    if (c->host) dfs::host_comm_close(c->host);
    if (c->d_gather) (void)hipFree(c->d_gather);
    delete c;
    return DFS_OK;
}

int dfs_comm_info(const dfs_comm* c, uint32_t* nranks, uint32_t* rank) {
    if (!c) return DFS_E_ARG;
    if (nranks) *nranks = c->nranks;
    if (rank) *rank = c->rank;
    return DFS_OK;
}

int dfs_comm_counters(const dfs_comm* c, uint64_t* counters) {
    if (!c || !counters) return DFS_E_ARG;
    std::memcpy(counters, c->issued, sizeof c->issued);
    return DFS_OK;
}

int dfs_place_sizes(dfs_comm* const* comms, uint32_t ncomms, const uint64_t* grp_len, uint32_t nfrag,
                    uint64_t* table) {
    if (int rc = check_comms(comms, ncomms)) return rc;
    if (!grp_len || !table || !nfrag || nfrag > kMaxFrag) return DFS_E_ARG;
    const uint32_t W = comms[0]->nranks;
    // every comm gathers the same table: keep the first
    std::vector<std::vector<uint64_t>> all(ncomms, std::vector<uint64_t>(static_cast<size_t>(W) * nfrag));
    std::vector<const uint64_t*> in(ncomms);
    std::vector<uint64_t*> out(ncomms);
    for (uint32_t i = 0; i < ncomms; ++i) {
        in[i] = grp_len + static_cast<uint64_t>(i) * nfrag;
        out[i] = all[i].data();
    }
    if (int rc = dfs::allgather_u64(comms, ncomms, in.data(), nfrag, out.data())) return rc;
    std::memcpy(table, all[0].data(), 8ull * W * nfrag);
    return DFS_OK;
}

int dfs_place_ring(dfs_comm* const* comms, uint32_t ncomms, uint32_t nfrag, const uint64_t* table,
                   const char* const* d_b64, char* const* d_held) {
    return place(comms, ncomms, nfrag, table, DFS_PLACE_RING, 0, reinterpret_cast<const void* const*>(d_b64),
                 reinterpret_cast<void* const*>(d_held), nullptr);
}

int dfs_place_star(dfs_comm* const* comms, uint32_t ncomms, uint32_t nfrag, const uint64_t* table,
                   const char* const* d_b64, char* const* d_held) {
    return place(comms, ncomms, nfrag, table, DFS_PLACE_STAR, 0, reinterpret_cast<const void* const*>(d_b64),
                 reinterpret_cast<void* const*>(d_held), nullptr);
}

int dfs_fetch_degraded(dfs_comm* const* comms, uint32_t ncomms, uint32_t nfrag, const uint64_t* table,
                       uint64_t offline_mask, const char* const* d_held, char* const* d_out, int32_t* frag_status) {
    return place(comms, ncomms, nfrag, table, DFS_PLACE_FETCH, offline_mask,
                 reinterpret_cast<const void* const*>(d_held), reinterpret_cast<void* const*>(d_out), frag_status);
}

}  // extern "C"
