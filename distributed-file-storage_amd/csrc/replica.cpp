// replica.cpp — the replica receiver's verify over placed groups
// (include/dfs_gpu.h, dfs_replica_*).
//
// Reference (StorageNode.java, SN:line): a peer that receives its pair of
// fragments Base64-decodes each one (:281), hashes the decoded bytes (:282),
// writes them as <index>.frag (:284-285) and replies with the hashes
// (:290-292); the uploader compares them with its own (:248-257) and fails the
// upload with "Replication failed" if any peer's differ (:218-221).
//
// Here a rank holds, after dfs_place_ring / dfs_place_star, group f (the
// Base64 of fragment f of every file) of every rank for each fragment f it
// hosts.  dfs_replica_verify sends every rank's fragment digests to the
// holders with the placement's own schedule (32 bytes per fragment in place
// of its Base64, so the table a holder receives is in held-fragment order),
// decodes and hashes every held fragment on the device and compares.  The
// descriptor tables depend only on the batch shape (file lengths, N, W) and
// are built once (dfs_replica_plan).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/dfs_gpu.h"
#include "dfs_internal.h"
#include "placement_internal.h"

using dfs::holds;
using dfs::kMaxFrag;
using dfs::kMaxRanks;
using dfs::ShaDesc;
using dfs::StreamJob;

struct dfs_replica_plan {
    int device = 0;
    uint32_t W = 0, me = 0, N = 0, my_files = 0;
    std::vector<uint64_t> table;      // W*N Base64 group bytes
    std::vector<dfs_held_frag> frags; // held order
    uint64_t held_bytes = 0, raw_bytes = 0;
    dfs::Plan dig_plan;               // the placement schedule over 32-byte digests
    // The check can run in slices of the held order (DFS_REPLICA_SLICES; one
    // by default): slice i is hashed while slice i + 1 is decoded beside it
    // on the ctx's second stream.  Each slice has its own decode job table (with its
    // tile prefix and sentinel) inside d_jobs and its own length-sorted lanes
    // inside d_desc; status and digest slots stay indexed by held fragment.
    struct Slice {
        uint64_t k0 = 0, k1 = 0;   // held fragments [k0, k1)
        uint64_t job0 = 0;         // first entry of its job table in d_jobs
        uint64_t ntiles = 0;
        uint32_t prio = 0;         // lanes of its long items (sort_sha_lanes)
    };
    std::vector<Slice> slices;
    std::vector<hipEvent_t> ev;       // [0]: the call's start on its stream; [i]: slice i decoded
    // device tables
    StreamJob* d_jobs = nullptr;
    ShaDesc* d_desc = nullptr;
    uint32_t* d_queue = nullptr;
    int32_t* d_status = nullptr;      // decode status per held fragment
    uint8_t* d_got = nullptr;         // digests of the decoded fragments
    uint8_t* d_expected = nullptr;    // the uploaders' digests, held order
    uint8_t* d_dig_t = nullptr;       // this rank's digests, fragment-major
    uint64_t* d_piece_start = nullptr;
    uint32_t* d_piece_rank = nullptr;
    uint32_t npieces = 0;
    // One-pass check (sha256_b64dec_lanes): every held fragment's chars are
    // decoded, written and hashed by one lane; the decoded bytes cross HBM once
    // instead of twice.  The default from a mean fragment of 128 bytes up
    // (DFS_REPLICA_FUSED=0 / 1 when the plan is made forces it off / on; one
    // slice only): 14.6 against 7.5 + 10.2 ms on the 65,536 x 256 KiB / N = 8
    // chunk, and ahead at every size tried from 128-byte to 210 KB fragments.
    // The two-kernel check above stays for everything else.
    dfs::DecLane* d_lanes = nullptr;  // longest first
    bool fused = false;
};

namespace {

#define HIPR(x)                                  \
    do {                                         \
        if ((x) != hipSuccess) return DFS_E_HIP; \
    } while (0)

uint64_t enc_len(uint64_t n) { return 4 * ((n + 2) / 3); }

// Mean fragment length from which the one-pass check is taken by default.
constexpr uint64_t kOnePassMinMean = 128;  // faster from 128-byte fragments up (measured); below: untried

// Fragment f of a file of S bytes split into N (SN:138-141, 155).
uint64_t frag_len(uint64_t S, uint32_t N, uint32_t f) { return S / N + (f < S % N ? 1 : 0); }

struct Layout {
    std::vector<uint64_t> table;  // W*N
    std::vector<dfs_held_frag> frags;
    std::vector<uint64_t> piece_start;  // held-fragment index where piece p begins (+ end)
    std::vector<uint32_t> piece_rank;
    uint64_t held_bytes = 0, raw_bytes = 0;
};

// The fragment-major Base64 layout of an upload plan (build_host_plan in
// dfs_gpu.cpp): fragments in [fragment][file] order, each start rounded up to
// `align`; group f begins where its first fragment does.
int build_layout(uint32_t W, uint32_t me, uint32_t N, const uint32_t* nfiles, const uint64_t* file_len, uint32_t flags,
                 bool want_frags, Layout& L) {
    if (!W || W > kMaxRanks || me >= W || !N || N > kMaxFrag || !nfiles) return DFS_E_ARG;
    if (flags & ~static_cast<uint32_t>(DFS_LAYOUT_ALIGN128 | DFS_LAYOUT_FRAG_MAJOR)) return DFS_E_ARG;
    const uint64_t align = (flags & DFS_LAYOUT_ALIGN128) ? 128 : 1;
    std::vector<uint64_t> first(W + 1, 0);
    for (uint32_t r = 0; r < W; ++r) first[r + 1] = first[r] + nfiles[r];
    if (first[W] && !file_len) return DFS_E_ARG;
    L.table.assign(static_cast<size_t>(W) * N, 0);
    // group sizes: walk every rank's fragments in plan order; group f runs
    // from its first fragment's (aligned) start to the next group's, the last
    // group to the end of the buffer
    std::vector<uint64_t> gstart(N + 1);
    for (uint32_t r = 0; r < W; ++r) {
        uint64_t total = 0;
        for (uint32_t f = 0; f < N; ++f) {
            gstart[f] = total;
            for (uint32_t j = 0; j < nfiles[r]; ++j) {
                total = (total + align - 1) / align * align;
                if (j == 0) gstart[f] = total;
                total += enc_len(frag_len(file_len[first[r] + j], N, f));
            }
        }
        gstart[N] = total;
        for (uint32_t f = 0; f < N; ++f) L.table[static_cast<size_t>(r) * N + f] = gstart[f + 1] - gstart[f];
    }
    // held order: hosted fragment f ascending, uploader r, file j
    uint64_t held = 0, raw = 0;
    L.frags.clear();
    L.piece_start.clear();
    L.piece_rank.clear();
    uint64_t count = 0;
    for (uint32_t f = 0; f < N; ++f) {
        if (!holds(me, f, N, W)) continue;
        for (uint32_t r = 0; r < W; ++r) {
            L.piece_start.push_back(count);
            L.piece_rank.push_back(r);
            uint64_t rel = 0;
            for (uint32_t j = 0; j < nfiles[r]; ++j) {
                const uint64_t n = frag_len(file_len[first[r] + j], N, f);
                rel = (rel + align - 1) / align * align;
                if (want_frags) {
                    dfs_held_frag h{};
                    h.rank = r;
                    h.file = j;
                    h.frag = f;
                    h.b64_off = held + rel;
                    h.b64_len = enc_len(n);
                    h.raw_off = raw;
                    h.raw_len = n;
                    L.frags.push_back(h);
                }
                rel += enc_len(n);
                raw += (n + 15) & ~15ull;
                ++count;
            }
            held += L.table[static_cast<size_t>(r) * N + f];
        }
    }
    L.piece_start.push_back(count);
    L.held_bytes = held;
    L.raw_bytes = raw;
    return DFS_OK;
}

void free_plan(dfs_replica_plan* p) {
    if (!p) return;
    (void)hipSetDevice(p->device);
    for (hipEvent_t e : p->ev)
        if (e) (void)hipEventDestroy(e);
    for (void* q : {static_cast<void*>(p->d_jobs), static_cast<void*>(p->d_desc), static_cast<void*>(p->d_queue),
                    static_cast<void*>(p->d_lanes),
                    static_cast<void*>(p->d_status), static_cast<void*>(p->d_got), static_cast<void*>(p->d_expected),
                    static_cast<void*>(p->d_dig_t), static_cast<void*>(p->d_piece_start),
                    static_cast<void*>(p->d_piece_rank)})
        if (q) (void)hipFree(q);
    delete p;
}

template <class T>
hipError_t dev_copy(T** d, const std::vector<T>& h) {
    hipError_t e = hipMalloc(reinterpret_cast<void**>(d), std::max<size_t>(h.size(), 1) * sizeof(T));
    if (e == hipSuccess && !h.empty()) e = hipMemcpy(*d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice);
    return e;
}

}  // namespace

extern "C" {

int dfs_replica_layout(uint32_t nranks, uint32_t rank, uint32_t nfrag, const uint32_t* nfiles,
                       const uint64_t* file_len, uint32_t layout_flags, dfs_held_frag* frags, uint64_t* nfrags,
                       uint64_t* table, uint64_t* held_bytes, uint64_t* raw_bytes) {
    if (!nfrags) return DFS_E_ARG;
    Layout L;
    if (int rc = build_layout(nranks, rank, nfrag, nfiles, file_len, layout_flags, true, L)) return rc;
    const uint64_t cap = *nfrags;
    *nfrags = L.frags.size();
    if (table) std::memcpy(table, L.table.data(), 8 * L.table.size());
    if (held_bytes) *held_bytes = L.held_bytes;
    if (raw_bytes) *raw_bytes = L.raw_bytes;
    if (frags) {
        if (cap < L.frags.size()) return DFS_E_ARG;
        if (!L.frags.empty()) std::memcpy(frags, L.frags.data(), sizeof(dfs_held_frag) * L.frags.size());
    }
    return DFS_OK;
}

int dfs_replica_plan_create(dfs_comm* const* comms, uint32_t ncomms, uint32_t nfrag, const uint32_t* nfiles,
                            const uint64_t* const* file_len, uint32_t layout_flags, dfs_replica_plan** plans) {
    if (int rc = dfs::check_comms(comms, ncomms)) return rc;
    if (!nfiles || !file_len || !plans || !nfrag || nfrag > kMaxFrag) return DFS_E_ARG;
    for (uint32_t i = 0; i < ncomms; ++i) {
        plans[i] = nullptr;
        if (nfiles[i] && !file_len[i]) return DFS_E_ARG;
    }
    uint32_t W = 0;
    (void)dfs_comm_info(comms[0], &W, nullptr);
    // every rank's file count, then every rank's lengths padded to the largest count
    std::vector<std::vector<uint64_t>> cnt_all(ncomms, std::vector<uint64_t>(W)), mine(ncomms);
    std::vector<uint64_t> cnt_mine(ncomms);
    std::vector<const uint64_t*> in(ncomms);
    std::vector<uint64_t*> out(ncomms);
    for (uint32_t i = 0; i < ncomms; ++i) {
        cnt_mine[i] = nfiles[i];
        in[i] = &cnt_mine[i];
        out[i] = cnt_all[i].data();
    }
    if (int rc = dfs::allgather_u64(comms, ncomms, in.data(), 1, out.data())) return rc;
    uint64_t maxf = 0;
    for (uint64_t c : cnt_all[0]) maxf = std::max(maxf, c);
    std::vector<std::vector<uint64_t>> len_all(ncomms, std::vector<uint64_t>(static_cast<size_t>(W) * maxf));
    for (uint32_t i = 0; i < ncomms; ++i) {
        mine[i].assign(maxf, 0);
        if (nfiles[i]) std::memcpy(mine[i].data(), file_len[i], 8ull * nfiles[i]);
        in[i] = mine[i].data();
        out[i] = len_all[i].data();
    }
    if (int rc = dfs::allgather_u64(comms, ncomms, in.data(), maxf, out.data())) return rc;
    for (uint32_t i = 0; i < ncomms; ++i) {
        uint32_t me = 0;
        (void)dfs_comm_info(comms[i], nullptr, &me);
        std::vector<uint32_t> nf(W);
        std::vector<uint64_t> lens;
        for (uint32_t r = 0; r < W; ++r) {
            nf[r] = static_cast<uint32_t>(cnt_all[i][r]);
            lens.insert(lens.end(), len_all[i].begin() + static_cast<size_t>(r) * maxf,
                        len_all[i].begin() + static_cast<size_t>(r) * maxf + nf[r]);
        }
        Layout L;
        int rc = build_layout(W, me, nfrag, nf.data(), lens.data(), layout_flags, true, L);
        auto* p = rc ? nullptr : new (std::nothrow) dfs_replica_plan;
        if (!rc && !p) rc = DFS_E_NOMEM;
        if (!rc) {
            p->device = dfs::ctx_device(dfs::comm_ctx(comms[i]));
            p->W = W;
            p->me = me;
            p->N = nfrag;
            p->my_files = nfiles[i];
            p->table = L.table;
            p->held_bytes = L.held_bytes;
            p->raw_bytes = L.raw_bytes;
            p->npieces = static_cast<uint32_t>(L.piece_rank.size());
            const uint64_t K = L.frags.size();
            if (K > 0xffffffffull) rc = DFS_E_ARG;
            // digest exchange: the star schedule over 32 bytes per fragment
            std::vector<uint64_t> dig_table(static_cast<size_t>(W) * nfrag);
            for (uint32_t r = 0; r < W; ++r)
                for (uint32_t f = 0; f < nfrag; ++f) dig_table[static_cast<size_t>(r) * nfrag + f] = 32ull * nf[r];
            if (!rc) rc = dfs::build_plan(W, me, nfrag, dig_table.data(), DFS_PLACE_STAR, 0, p->dig_plan);
            if (!rc && p->dig_plan.dst_off[nfrag] != 32 * K) rc = DFS_E_ARG;  // held order == schedule order
            // decode jobs into the raw buffer (raw_off is 16-byte aligned: no
            // head bytes as long as d_raw is) and SHA lanes over the raw bytes
            // One slice unless DFS_REPLICA_SLICES asks for more: measured on the
            // 131,072 x 256 KiB / N = 8 shard (524,288 held fragments per call),
            // two slices make the check slower (38.9 against 36.0 ms) — the
            // narrow decode beside the SHA waves costs the SHA kernel more
            // clock than the overlap saves.
            uint64_t nslices = 1;
            if (const char* e = std::getenv("DFS_REPLICA_SLICES"))
                nslices = std::min<uint64_t>(std::max<uint64_t>(1, std::strtoull(e, nullptr, 10)), std::max<uint64_t>(K, 1));
            nslices = std::min<uint64_t>(nslices, 16);
            std::vector<StreamJob> jobs;   // the slices' job tables, back to back
            std::vector<ShaDesc> desc(K);
            for (uint64_t i = 0; i < nslices && !rc; ++i) {
                dfs_replica_plan::Slice sl;
                sl.k0 = K * i / nslices;
                sl.k1 = K * (i + 1) / nslices;
                std::vector<StreamJob> js(sl.k1 - sl.k0);
                std::vector<uint64_t> items(js.size());
                for (uint64_t k = sl.k0; k < sl.k1 && !rc; ++k) {
                    const dfs_held_frag& h = L.frags[k];
                    StreamJob& j = js[k - sl.k0];
                    j = StreamJob{};
                    j.src_off = h.b64_off;
                    j.len = h.b64_len;
                    j.dst_off = h.raw_off;
                    j.expect = h.raw_len + 1;
                    j.id = static_cast<uint32_t>(k);
                    items[k - sl.k0] = dfs::decode_items(h.b64_len, static_cast<uintptr_t>(h.raw_off));
                    desc[k] = ShaDesc{h.raw_off, h.raw_len, h.raw_len, static_cast<uint32_t>(k), 0, 0};
                    if (h.raw_len >= (1ull << 37)) rc = DFS_E_ARG;
                }
                sl.ntiles = dfs::finish_stream_jobs(js, items, static_cast<uint64_t>(dfs::kDecGpl) * dfs::kStreamBlock);
                std::vector<ShaDesc> lanes(desc.begin() + sl.k0, desc.begin() + sl.k1);
                sl.prio = dfs::sort_sha_lanes(lanes);
                std::copy(lanes.begin(), lanes.end(), desc.begin() + sl.k0);
                sl.job0 = jobs.size();
                jobs.insert(jobs.end(), js.begin(), js.end());  // with its sentinel
                p->slices.push_back(sl);
            }
            std::vector<dfs::DecLane> lanes;
            if (!rc) {
                uint64_t raw_total = 0;
                for (const dfs_held_frag& h : L.frags) raw_total += h.raw_len;
                p->fused = nslices == 1 && K && raw_total / K >= kOnePassMinMean;
                if (const char* e = std::getenv("DFS_REPLICA_FUSED")) p->fused = nslices == 1 && K && e[0] == '1';
                for (uint64_t k = 0; k < K && p->fused; ++k) {
                    const dfs_held_frag& h = L.frags[k];
                    // what the lanes assume: dword-aligned chars, 16-byte aligned bytes, the encoder's length
                    if ((h.b64_off & 3u) || (h.raw_off & 15u) || h.b64_len != enc_len(h.raw_len)) p->fused = false;
                }
                if (p->fused) {
                    lanes.resize(K);
                    for (uint64_t k = 0; k < K; ++k) {
                        const dfs_held_frag& h = L.frags[k];
                        lanes[k] = dfs::DecLane{h.b64_off, h.raw_off, h.raw_len, h.b64_len, static_cast<uint32_t>(k), 0};
                    }
                    std::stable_sort(lanes.begin(), lanes.end(),
                                     [](const dfs::DecLane& a, const dfs::DecLane& b) { return a.n > b.n; });
                }
            }
            if (!rc) {
                p->frags = std::move(L.frags);
                hipError_t e = hipSetDevice(p->device);
                p->ev.assign(p->slices.size(), nullptr);
                for (size_t i = 0; i < p->ev.size() && e == hipSuccess && p->ev.size() > 1; ++i)
                    e = hipEventCreateWithFlags(&p->ev[i], hipEventDisableTiming);
                if (e == hipSuccess) e = dev_copy(&p->d_jobs, jobs);
                if (e == hipSuccess) e = dev_copy(&p->d_desc, desc);
                if (e == hipSuccess && p->fused) e = dev_copy(&p->d_lanes, lanes);
                if (e == hipSuccess) e = dev_copy(&p->d_piece_start, L.piece_start);
                if (e == hipSuccess) e = dev_copy(&p->d_piece_rank, L.piece_rank);
                if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&p->d_queue), dfs::kShaQueueBytes);
                if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&p->d_status), std::max<uint64_t>(K, 1) * 4);
                if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&p->d_got), std::max<uint64_t>(K, 1) * 32);
                if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&p->d_expected), std::max<uint64_t>(K, 1) * 32);
                if (e == hipSuccess)
                    e = hipMalloc(reinterpret_cast<void**>(&p->d_dig_t),
                                  std::max<uint64_t>(static_cast<uint64_t>(nfiles[i]) * nfrag, 1) * 32);
                if (e != hipSuccess) rc = e == hipErrorOutOfMemory ? DFS_E_NOMEM : DFS_E_HIP;
            }
        }
        if (rc) {
            free_plan(p);
            for (uint32_t q = 0; q < i; ++q) {
                free_plan(plans[q]);
                plans[q] = nullptr;
            }
            return rc;
        }
        plans[i] = p;
    }
    return DFS_OK;
}

int dfs_replica_plan_info(const dfs_replica_plan* p, uint64_t* nheld, uint64_t* held_bytes, uint64_t* raw_bytes,
                          uint64_t* table) {
    if (!p) return DFS_E_ARG;
    if (nheld) *nheld = p->frags.size();
    if (held_bytes) *held_bytes = p->held_bytes;
    if (raw_bytes) *raw_bytes = p->raw_bytes;
    if (table) std::memcpy(table, p->table.data(), 8 * p->table.size());
    return DFS_OK;
}

int dfs_replica_plan_one_pass(const dfs_replica_plan* p) {
    if (!p) return DFS_E_ARG;
    return p->fused ? 1 : 0;
}

int dfs_replica_plan_frags(const dfs_replica_plan* p, dfs_held_frag* frags) {
    if (!p || (!frags && !p->frags.empty())) return DFS_E_ARG;
    if (!p->frags.empty()) std::memcpy(frags, p->frags.data(), sizeof(dfs_held_frag) * p->frags.size());
    return DFS_OK;
}

int dfs_replica_plan_destroy(dfs_replica_plan* p) {
    if (!p) return DFS_E_ARG;
    free_plan(p);
    return DFS_OK;
}

// Stage 1 (comm streams): every rank's fragment digests, fragment-major, to
// the holders with the placement's schedule.
int dfs_replica_exchange(dfs_comm* const* comms, uint32_t ncomms, dfs_replica_plan* const* plans,
                         const uint8_t* const* d_frag_digest) {
    if (int rc = dfs::check_comms(comms, ncomms)) return rc;
    if (!plans || !d_frag_digest) return DFS_E_ARG;
    std::vector<dfs::Plan> dig(ncomms);
    std::vector<const void*> src(ncomms);
    std::vector<void*> dst(ncomms);
    for (uint32_t i = 0; i < ncomms; ++i) {
        dfs_replica_plan* p = plans[i];
        uint32_t W = 0, me = 0;
        (void)dfs_comm_info(comms[i], &W, &me);
        if (!p || p->W != W || p->me != me || p->device != dfs::ctx_device(dfs::comm_ctx(comms[i]))) return DFS_E_ARG;
        if (p->my_files && !d_frag_digest[i]) return DFS_E_ARG;
        hipStream_t s = dfs::ctx_stream(dfs::comm_ctx(comms[i]));
        HIPR(hipSetDevice(p->device));
        HIPR(dfs::launch_digest_transpose(d_frag_digest[i], p->d_dig_t, p->my_files, p->N, s));
        dig[i] = p->dig_plan;
        src[i] = p->d_dig_t;
        dst[i] = p->d_expected;
    }
    return dfs::run_plans_rccl(comms, ncomms, dig, src.data(), dst.data());
}

// Stage 2 (any ctx of the plan's device; no communication): decode, hash,
// compare.  d_failed gets this holder's own counts.
int dfs_replica_check(dfs_ctx* ctx, dfs_replica_plan* p, const char* d_held, uint8_t* d_raw, int32_t* d_verdict,
                      uint32_t* d_failed) {
    if (!ctx || !p || !d_failed || p->device != dfs::ctx_device(ctx)) return DFS_E_ARG;
    if ((p->held_bytes && !d_held) || (p->raw_bytes && !d_raw) || (reinterpret_cast<uintptr_t>(d_raw) & 15u))
        return DFS_E_ARG;
    hipStream_t s = dfs::ctx_stream(ctx);
    HIPR(hipSetDevice(p->device));
    const uint64_t K = p->frags.size();
    HIPR(dfs::launch_fill_u32(d_failed, p->W, 0u, s));
    if (!K) return DFS_OK;
    if (p->fused && !(reinterpret_cast<uintptr_t>(d_held) & 3u)) {
        // one pass: each lane decodes, stores and hashes its fragment and sets its status word
        HIPR(dfs::launch_sha256_b64dec(d_held, p->d_lanes, static_cast<uint32_t>(K), d_raw, p->d_got, p->d_status,
                                       p->d_queue, 4, s));
        HIPR(dfs::launch_replica_verdict(p->d_status, p->d_got, p->d_expected, K, p->d_piece_start, p->d_piece_rank,
                                         p->npieces, DFS_E_DECODE, DFS_E_FRAG_MISMATCH, d_verdict, d_failed, s));
        return DFS_OK;
    }
    HIPR(dfs::launch_fill_u32(reinterpret_cast<uint32_t*>(p->d_status), K, 0u, s));
    // Slice 0 is decoded at full width on the call's stream; slices 1.. on the
    // ctx's second stream with a narrow, prioritised grid, each beside the
    // hashing of the slice before it.  Nothing waits inside a kernel: a decode
    // that finds no room beside the SHA waves simply runs after them.
    const size_t ns = p->slices.size();
    hipStream_t a = s;
    if (ns > 1) {
        HIPR(dfs::ctx_aux_stream(ctx, &a));
        HIPR(hipEventRecord(p->ev[0], s));
        HIPR(hipStreamWaitEvent(a, p->ev[0], 0));
    }
    for (size_t i = 0; i < ns; ++i) {
        const dfs_replica_plan::Slice& sl = p->slices[i];
        const uint32_t n = static_cast<uint32_t>(sl.k1 - sl.k0);
        if (!n) continue;
        if (i == 0)
            HIPR(dfs::launch_b64_decode(d_held, p->d_jobs + sl.job0, n, sl.ntiles, d_raw, p->d_status, nullptr, s));
        else {
            HIPR(dfs::launch_b64_decode(d_held, p->d_jobs + sl.job0, n, sl.ntiles, d_raw, p->d_status, nullptr, a, 1u, 2u));
            HIPR(hipEventRecord(p->ev[i], a));
        }
    }
    for (size_t i = 0; i < ns; ++i) {
        const dfs_replica_plan::Slice& sl = p->slices[i];
        const uint32_t n = static_cast<uint32_t>(sl.k1 - sl.k0);
        if (!n) continue;
        if (i) HIPR(hipStreamWaitEvent(s, p->ev[i], 0));
        HIPR(dfs::launch_sha256(d_raw, p->d_desc + sl.k0, n, static_cast<uint32_t>(K), sl.prio, p->d_got, p->d_got,
                                p->d_queue, ns > 1 ? 3 : 4, s));
    }
    HIPR(dfs::launch_replica_verdict(p->d_status, p->d_got, p->d_expected, K, p->d_piece_start, p->d_piece_rank,
                                     p->npieces, DFS_E_DECODE, DFS_E_FRAG_MISMATCH, d_verdict, d_failed, s));
    return DFS_OK;
}

// Stage 3 (comm streams): failures per uploader summed over the holders.
int dfs_replica_report(dfs_comm* const* comms, uint32_t ncomms, uint32_t* const* d_failed) {
    if (int rc = dfs::check_comms(comms, ncomms)) return rc;
    if (!d_failed) return DFS_E_ARG;
    for (uint32_t i = 0; i < ncomms; ++i)
        if (!d_failed[i]) return DFS_E_ARG;
    uint32_t W = 0;
    (void)dfs_comm_info(comms[0], &W, nullptr);
    return dfs::allreduce_u32(comms, ncomms, d_failed, W);
}

int dfs_replica_verify(dfs_comm* const* comms, uint32_t ncomms, dfs_replica_plan* const* plans,
                       const uint8_t* const* d_frag_digest, const char* const* d_held, uint8_t* const* d_raw,
                       int32_t* const* d_verdict, uint32_t* const* d_failed) {
    if (!plans || !d_held || !d_raw || !d_failed) return DFS_E_ARG;
    if (int rc = dfs_replica_exchange(comms, ncomms, plans, d_frag_digest)) return rc;
    for (uint32_t i = 0; i < ncomms; ++i)
        if (int rc = dfs_replica_check(dfs::comm_ctx(comms[i]), plans[i], d_held[i], d_raw[i],
                                       d_verdict ? d_verdict[i] : nullptr, d_failed[i]))
            return rc;
    return dfs_replica_report(comms, ncomms, d_failed);
}

}  // extern "C"
