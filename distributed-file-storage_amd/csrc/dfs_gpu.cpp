// dfs_gpu.cpp — C ABI of libdfsgpu.so (include/dfs_gpu.h).
//
// Owns the HIP context state (streams, events, device scratch), builds the
// per-batch descriptor tables on the host (split plan, Base64 offsets,
// length-sorted SHA lanes) and launches the gfx950 kernels.  There is no CPU
// implementation of any data-path step here: without a gfx950 device
// dfs_open fails and nothing runs.
//
// Reference sites replaced (StorageNode.java, SN:line): sha256Hex :603-613
// (called at :127, :159, :282, :454); split loop :138-171; Base64 encode
// :636; Base64 decode :281; ordered gather :422-451; verify :454-458.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <functional>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/dfs_gpu.h"
#include "dfs_internal.h"

using dfs::ShaDesc;
using dfs::StreamJob;

namespace {

constexpr uint64_t kMaxMsg = 1ull << 37;  // nfull (len/64) must fit 32 bits

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = n < 256 ? 256 : n;
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T> T* as() const { return static_cast<T*>(p); }
};

enum BufId { B_DATA_IN, B_DATA_OUT, B_DIG0, B_DIG1, B_DESC, B_JOBS, B_JOBS2, B_JOBS3, B_STATUS, B_OUTLEN, B_QUEUE, B_COPY, B_COUNT };

}  // namespace

struct dfs_ctx {
    int device = 0;
    hipStream_t own = nullptr;   // default stream of this ctx
    hipStream_t aux = nullptr;   // second stream (Base64 beside SHA), created on first use: a
                                 // process has few hardware queues (GPU_MAX_HW_QUEUES=4 on the
                                 // box) and every stream takes one until they are shared
    hipStream_t user = nullptr;  // borrowed (dfs_set_stream)
    bool profiling = false;
    int sha_wps = 4;             // SHA waves per SIMD (DFS_SHA_WPS overrides)
    int sha_wps_beside = 3;      // ... when the Base64 kernel runs beside it (4 x 116 VGPRs leave no room)
    int upload_mode = 1;         // 0 fused Base64 in the SHA lanes, 1 SHA || Base64 kernels, 2 hybrid: the fragment
                                 // lanes write their own Base64 and the encode kernel only the twins' (DFS_UPLOAD_MODE)
    int download_mode = 2;       // 2 decode-ahead (one SHA launch waits per fragment group), 0 pipelined passes,
                                 // 1 decode then SHA (DFS_DOWNLOAD_MODE=overlap|pipelined|serial)
    int ovl_sha_wps = 3;         // overlap: SHA waves per SIMD (DFS_OVL_SHA_WPS) ...
    uint32_t ovl_dec_wgs = 1;    // ... and decode workgroups per CU beside them (DFS_OVL_DEC_WGS); both
                                 // clamped at open so the two grids are resident together (ovl_fit)
    uint32_t ovl_gather_wgs = 2; // gather workgroups per CU beside them (reassembly overlap; fitted too)
    int b64_wgs = 2;             // encode workgroups per CU beside SHA (DFS_B64_WGS)
    uint32_t b64_prio = 1;       // s_setprio of the encode waves beside SHA (DFS_B64_PRIO; profiles/r02c_knobs)
    uint32_t dec_prio = 1;       // decode waves at s_setprio 3 beside SHA (DFS_DEC_PRIO=0: 0)
    uint32_t dec_wgs = 1;        // decode workgroups per CU beside SHA (DFS_DEC_WGS)
    bool recv_one_pass = true;   // dfs_receive_fragments_batch: one-pass kernel for big aligned batches (DFS_RECV_FUSED=0: never)
    uint64_t ovl_redo = 0;       // overlap downloads whose SHA launch was redone (a wait timed out)
    uint64_t recv_one_pass_calls = 0;  // dfs_receive_fragments_batch calls that took the one-pass kernel
    uint64_t wait_ticks = dfs::kShaWaitTicks;  // bound of an in-kernel group wait (DFS_SHA_WAIT_TICKS)
    uint32_t wait_never = 0;     // test hook (DFS_SHA_WAIT_FORCE_TIMEOUT=1): the SHA lanes wait for one more
                                 // workgroup than the decode / gather grid has and give up after 10 us, so
                                 // every overlapped call takes the timeout + redo path; all kernels still exit
    hipEvent_t ev[2 * DFS_T_COUNT] = {};
    bool ev_used[DFS_T_COUNT] = {};
    hipEvent_t fork = nullptr, join = nullptr;  // SHA || Base64 on two streams
    std::vector<hipEvent_t> pass_ev;             // download passes (decode of fragment i done)
    // The scratch buffers (buf[]) are reused by the next call.  An async call
    // leaves them in use on its stream: a call on another stream (after
    // dfs_set_stream) first waits for scratch_ev (recorded after the last
    // launch that used them) so it cannot overwrite descriptors in flight.
    hipEvent_t scratch_ev = nullptr;
    hipEvent_t sync_ev = nullptr;  // quiet_sync (calls run under mu, so one per ctx)
    hipStream_t scratch_stream = nullptr;
    // Pinned staging for the host -> device descriptor copies of one call
    // (two arenas, alternating per call): an async copy from pageable memory
    // is staged by the runtime and blocks, so tables go through here.  An
    // arena is reused once the copies of the call before last completed.
    struct Arena {
        uint8_t* p = nullptr;
        size_t cap = 0, used = 0;
        hipEvent_t ev = nullptr;
        bool pending = false;
    } arena[2];
    int cur_arena = 0;
    DevBuf buf[B_COUNT];
    dfs::StoreStaging* store = nullptr;  // pinned staging ring of the fragment store
    std::mutex mu;
    std::mutex store_mu;         // the fragment store's staging ring (fragstore.cpp)
    hipStream_t stream() const { return user ? user : own; }
};

namespace dfs {
hipStream_t ctx_stream(dfs_ctx* c) { return c->stream(); }

// hipStreamSynchronize / hipEventSynchronize busy-wait on this runtime, even
// for hipEventBlockingSync events: a 29 ms wait costs 29 ms of host CPU
// (tools/host_probe, profiles/r02c_host_probe.txt).  StorageNode runs one
// thread per connection (SN:30), and a handler blocked in a call must not
// spend a core of the node's share on nothing, so the synchronous calls poll
// an event with sleeps growing from 8 to 256 us (at most ~0.25 ms late on a
// call that runs milliseconds; 0.35 ms of CPU per 29 ms wait).
hipError_t quiet_wait(hipEvent_t ev) {
    unsigned us = 8;
    for (;;) {
        const hipError_t e = hipEventQuery(ev);
        if (e != hipErrorNotReady) {
            (void)hipGetLastError();  // the not-ready answers are not errors of this thread
            return e;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(us));
        if (us < 256) us *= 2;
    }
}

hipError_t quiet_sync(dfs_ctx* c, hipStream_t s) {
    const hipError_t e = hipEventRecord(c->sync_ev, s);
    return e == hipSuccess ? quiet_wait(c->sync_ev) : e;
}

// Device -> host copy into caller (usually pageable) memory.  Such a copy
// returns only when done and, issued behind running kernels, spins a core
// until they finish; so the stream is drained quietly first.
hipError_t d2h(dfs_ctx* c, void* dst, const void* src, size_t n, hipStream_t s) {
    hipError_t e = quiet_sync(c, s);
    if (e == hipSuccess) e = hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, s);
    return e;
}
int ctx_device(dfs_ctx* c) { return c->device; }
// The ctx's second stream (created on first use), for a stream kernel that
// runs beside the SHA kernel of the same call.
hipError_t ctx_aux_stream(dfs_ctx* c, hipStream_t* aux) {
    std::lock_guard<std::mutex> lk(c->mu);
    hipError_t e = hipSetDevice(c->device);
    if (e == hipSuccess && !c->aux) e = hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking);
    *aux = c->aux;
    return e;
}
std::mutex& ctx_store_mutex(dfs_ctx* c) { return c->store_mu; }
StoreStaging*& ctx_store(dfs_ctx* c) { return c->store; }
}  // namespace dfs

struct dfs_upload_plan {
    int device = 0;
    uint32_t* d_queue = nullptr;  // SHA work-queue word
    uint32_t nfiles = 0, nfrag = 0;
    uint32_t n_all = 0, n_frag_only = 0;  // SHA lanes with / without fileIds
    bool twins = false;                   // d_all holds twins behind its n_all lanes (kShaTwin)
    uint32_t prio_all = 0, prio_frag = 0;
    ShaDesc* d_all = nullptr;
    ShaDesc* d_frag = nullptr;
    StreamJob* d_enc = nullptr;
    uint32_t n_enc = 0;
    uint64_t enc_tiles = 0;
    StreamJob* d_enc_twin = nullptr;  // the encode jobs of the fragments that ride as twins (hybrid mode)
    uint32_t n_enc_twin = 0;
    uint64_t enc_twin_tiles = 0;
    std::vector<uint64_t> b64_off;
    uint64_t b64_total = 0;
};

namespace {

thread_local char g_last_hip[160];

int hip_fail(hipError_t e, const char* what) {
    std::snprintf(g_last_hip, sizeof g_last_hip, "%s: %s", what, hipGetErrorString(e));
    return e == hipErrorOutOfMemory ? DFS_E_NOMEM : DFS_E_HIP;
}

#define HIPC(x)                                   \
    do {                                          \
        hipError_t e_ = (x);                      \
        if (e_ != hipSuccess) return hip_fail(e_, #x); \
    } while (0)

void split(uint64_t S, uint32_t N, uint64_t* off, uint64_t* len) {
    const uint64_t base = S / N, rem = S % N;  // SN:140-141
    uint64_t o = 0;
    for (uint32_t i = 0; i < N; ++i) {
        const uint64_t part = base + (i < rem ? 1 : 0);  // SN:155
        off[i] = o;
        len[i] = part;
        o += part;  // SN:170
    }
}

uint64_t enc_len(uint64_t n) { return 4 * ((n + 2) / 3); }

// A whole message (not resumed): len bytes at off, digest slot out.
ShaDesc msg(uint64_t off, uint64_t len, uint64_t out) { return ShaDesc{off, len, len, static_cast<uint32_t>(out), 0, 0}; }

// Sort SHA lanes longest-first (uniform waves) and count the lanes that
// carry the long chains: those waves get issue priority in the kernel.
uint32_t sort_lanes(std::vector<ShaDesc>& d) {
    // Longest first, stable.  Batches hold few distinct lengths (N fragment
    // sizes + file sizes), so a counting sort over the distinct lengths is
    // O(n); many distinct lengths fall back to a comparison sort.
    std::vector<uint64_t> lens;
    for (const ShaDesc& x : d) {
        if (std::find(lens.begin(), lens.end(), x.len) == lens.end()) {
            lens.push_back(x.len);
            if (lens.size() > 32) break;
        }
    }
    if (lens.size() <= 32) {
        std::sort(lens.begin(), lens.end(), std::greater<uint64_t>());
        std::vector<size_t> start(lens.size() + 1, 0);
        std::vector<uint32_t> bucket(d.size());
        for (size_t i = 0; i < d.size(); ++i) {
            bucket[i] = static_cast<uint32_t>(std::find(lens.begin(), lens.end(), d[i].len) - lens.begin());
            ++start[bucket[i] + 1];
        }
        for (size_t b = 0; b < lens.size(); ++b) start[b + 1] += start[b];
        std::vector<ShaDesc> out(d.size());
        for (size_t i = 0; i < d.size(); ++i) out[start[bucket[i]]++] = d[i];
        d.swap(out);
    } else {
        std::stable_sort(d.begin(), d.end(), [](const ShaDesc& a, const ShaDesc& b) { return a.len > b.len; });
    }
    if (d.size() < 2) return 0;
    const uint64_t med = d[d.size() / 2].len;
    uint32_t n = 0;
    while (n < d.size() && d[n].len >= 2 * med + 64) ++n;
    return (n + 63) & ~63u;
}

// Twins (kShaTwin, sha256.hip): a fragment that starts on the 64-byte block
// grid of its file's fileId lane (or fileId part), is at least one block long
// and is a whole message rides in that lane: its blocks are loaded and their
// message schedule expanded once for both digests.  That is fragment 0 of
// every file (offset 0, SN:153) and, when the fragment size is a multiple of
// 64 (256 KiB files, N = 8: BASELINE configs[2]), every fragment.  Appends
// `primary` (with its twin list) and the fragments that are not twins to
// `lanes`, the twins to `tw` (launched as descs[n_lanes + ...]).  Twins need
// the persistent kernel: callers keep them only for launches of at least
// dfs::kTwinMinLanes lanes (> kChainMaxLanes) that run without the fused Base64.
void add_lane_with_twins(std::vector<ShaDesc>& lanes, std::vector<ShaDesc>& tw, ShaDesc primary,
                         const ShaDesc* frags, uint32_t nfr, bool enable) {
    const uint64_t first = tw.size();
    uint64_t cnt = 0, next = 0;  // first block of the primary a twin may start at
    const uint64_t pfull = primary.len >> 6;
    for (uint32_t i = 0; i < nfr; ++i) {
        const ShaDesc& f = frags[i];
        const uint64_t rel = f.off - primary.off;
        const bool ok = enable && f.flags == 0 && f.off >= primary.off && (rel & 63u) == 0 && f.len >= 64 &&
                        (rel >> 6) >= next && (rel >> 6) + (f.len >> 6) <= pfull;
        if (ok) {
            tw.push_back(f);
            ++cnt;
            next = (rel >> 6) + (f.len >> 6);
        } else {
            lanes.push_back(f);
        }
    }
    if (cnt) {
        primary.flags |= dfs::kShaTwin;
        primary.b64 = (cnt << 32) | first;
    }
    lanes.push_back(primary);
}

// Fill tile_start prefix for `items` work items per job; append sentinel.
uint64_t finish_jobs(std::vector<StreamJob>& jobs, const std::vector<uint64_t>& items, uint64_t per_tile) {
    uint64_t t = 0;
    for (size_t i = 0; i < jobs.size(); ++i) {
        jobs[i].tile_start = t;
        t += (items[i] + per_tile - 1) / per_tile;
    }
    StreamJob s{};
    s.tile_start = t;
    jobs.push_back(s);
    return t;
}

// Decode work of one message in 4-unit groups (dfs::dec_geom); at least one
// tile, whose last one also runs the tail step.
uint64_t dec_items(uint64_t L, uintptr_t dst) {
    const uint64_t ng = dfs::dec_geom(L, dst).ng;
    return ng ? ng : 1;
}

// Gather items of one fragment (must match gather_kernel): 16-byte chunks
// from the first 16-aligned destination address + one head/tail item.
uint64_t copy_items(uint64_t len, uintptr_t dst) {
    if (!len) return 0;
    const uint32_t h = static_cast<uint32_t>((16u - (dst & 15u)) & 15u);
    const uint64_t nc = len > h ? (len - h) / 16 : 0;
    return nc + 1;
}

struct Timer {
    dfs_ctx* c;
    explicit Timer(dfs_ctx* ctx) : c(ctx) {
        for (bool& u : c->ev_used) u = false;
    }
    void begin(int k, hipStream_t s) {
        if (!c->profiling) return;
        (void)hipEventRecord(c->ev[2 * k], s);
    }
    void end(int k, hipStream_t s) {
        if (!c->profiling) return;
        (void)hipEventRecord(c->ev[2 * k + 1], s);
        c->ev_used[k] = true;
    }
};

// Scope of one call's use of the ctx scratch on stream s (see dfs_ctx).
struct Scratch {
    dfs_ctx* c;
    hipStream_t s;
    Scratch(dfs_ctx* ctx, hipStream_t st) : c(ctx), s(st) {
        if (c->scratch_stream && c->scratch_stream != s) (void)hipStreamWaitEvent(s, c->scratch_ev, 0);
        c->cur_arena ^= 1;
        auto& a = c->arena[c->cur_arena];
        if (a.pending) (void)dfs::quiet_wait(a.ev);
        a.pending = false;
        a.used = 0;
    }
    ~Scratch() {
        if (hipEventRecord(c->scratch_ev, s) == hipSuccess) c->scratch_stream = s;
        auto& a = c->arena[c->cur_arena];
        if (a.used && hipEventRecord(a.ev, s) == hipSuccess) a.pending = true;
    }
};

constexpr size_t kArenaMax = 64ull << 20;  // larger host buffers (file data) are copied directly

int put(dfs_ctx* c, int id, const void* src, size_t n, hipStream_t s) {
    HIPC(c->buf[id].ensure(n));
    if (!n) return DFS_OK;
    auto& a = c->arena[c->cur_arena];
    if (n <= kArenaMax) {
        if (a.used + n > a.cap) {
            if (a.used) HIPC(dfs::quiet_sync(c, s));  // this call's earlier copies still read the arena
            const size_t want = std::max<size_t>({a.used + n, 2 * a.cap, size_t(1) << 20});
            if (a.p) (void)hipHostFree(a.p);
            a.p = nullptr;
            a.cap = a.used = 0;
            HIPC(hipHostMalloc(reinterpret_cast<void**>(&a.p), want, hipHostMallocDefault));
            a.cap = want;
        }
        std::memcpy(a.p + a.used, src, n);
        HIPC(hipMemcpyAsync(c->buf[id].p, a.p + a.used, n, hipMemcpyHostToDevice, s));
        a.used += (n + 255) & ~size_t(255);
        return DFS_OK;
    }
    HIPC(hipMemcpyAsync(c->buf[id].p, src, n, hipMemcpyHostToDevice, s));
    return DFS_OK;
}

bool is_device_ptr(const void* p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();  // plain host memory: clear the sticky error
        return false;
    }
    return a.type == hipMemoryTypeDevice;
}

int enter(dfs_ctx* c) {
    if (!c) return DFS_E_ARG;
    HIPC(hipSetDevice(c->device));
    return DFS_OK;
}

}  // namespace

namespace dfs {
uint32_t sort_sha_lanes(std::vector<ShaDesc>& d) { return sort_lanes(d); }
uint64_t finish_stream_jobs(std::vector<StreamJob>& jobs, const std::vector<uint64_t>& items, uint64_t per_tile) {
    return finish_jobs(jobs, items, per_tile);
}
uint64_t decode_items(uint64_t L, uintptr_t dst) { return dec_items(L, dst); }

int copy_spans(dfs_ctx* c, const CopySpan* spans, size_t n) {
    if (!c || (n && !spans)) return DFS_E_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    if (int rc = enter(c)) return rc;
    hipStream_t s = c->stream();
    Scratch scratch(c, s);
    std::vector<StreamJob> jobs;
    std::vector<uint64_t> items;
    jobs.reserve(n + 1);
    items.reserve(n);
    for (size_t i = 0; i < n; ++i) {
        if (!spans[i].len) continue;
        StreamJob j{};
        j.src_off = spans[i].src;
        j.len = spans[i].len;
        j.dst_off = spans[i].dst;  // absolute: gather_kernel's output base is 0
        jobs.push_back(j);
        items.push_back(copy_items(spans[i].len, static_cast<uintptr_t>(spans[i].dst)));
    }
    if (jobs.empty()) return DFS_OK;
    const uint64_t ntiles = finish_jobs(jobs, items, static_cast<uint64_t>(kGatherPer) * kStreamBlock);
    if (int rc = put(c, B_COPY, jobs.data(), jobs.size() * sizeof(StreamJob), s)) return rc;
    HIPC(launch_gather(c->buf[B_COPY].as<StreamJob>(), static_cast<uint32_t>(jobs.size() - 1), ntiles, nullptr, s));
    return DFS_OK;
}
}  // namespace dfs

extern "C" {

int dfs_abi_version(void) { return DFS_ABI_VERSION; }

const char* dfs_strerror(int code) {
    switch (code) {
        case DFS_OK: return "ok";
        case DFS_E_ARG: return "invalid argument";
        case DFS_E_HIP: return g_last_hip[0] ? g_last_hip : "HIP runtime error";
        case DFS_E_NOMEM: return "out of device memory";
        case DFS_E_DECODE: return "Illegal base64 input (IllegalArgumentException)";
        case DFS_E_MISSING: return "Could not retrieve fragment";
        case DFS_E_CORRUPT: return "File corrupted";
        case DFS_E_FRAG_MISMATCH: return "Hash mismatch on fragment";
        case DFS_E_NODEV: return "no gfx950 (MI355X) device available";
        case DFS_E_WIRE: return "storeFragments body not in buildFragmentsJson form (parse it with parseJson)";
        case DFS_E_IO: return "fragment store I/O error (IOException)";
        case DFS_E_COMM: return dfs_comm_last_error();
        case DFS_E_TOOBIG: return "batch exceeds the static scratch (dfs_sha256_batch_static: at most 65,536 messages)";
        default: return "unknown error";
    }
}

// Decode-ahead download: every SHA wave may wait on every decode workgroup,
// so both grids must be resident at once.  Per SIMD, wps SHA waves plus
// dec_wgs decode waves (a 256-thread workgroup puts one wave on each SIMD of
// its CU) must fit the 512-entry VGPR file (allocation granularity 8); LDS
// (one ~25 KB decode workgroup per wave slot) and the 32 waves per CU are far
// from their limits.  Fewer decode workgroups first, then fewer SHA waves.
static void ovl_fit(dfs_ctx* c) {
    const int sv = dfs::sha_wait_vgprs(), dv = dfs::dec_ahead_vgprs(), gv = dfs::gather_ahead_vgprs();
    if (sv <= 0 || dv <= 0 || gv <= 0) {  // attributes unavailable: the smallest grids
        c->ovl_sha_wps = 1;
        c->ovl_dec_wgs = c->ovl_gather_wgs = 1;
        return;
    }
    const int sa = (sv + 7) / 8 * 8, da = (dv + 7) / 8 * 8, ga = (gv + 7) / 8 * 8;
    while (c->ovl_sha_wps * sa + static_cast<int>(c->ovl_dec_wgs) * da > 512) {
        if (c->ovl_dec_wgs > 1) --c->ovl_dec_wgs;
        else if (c->ovl_sha_wps > 1) --c->ovl_sha_wps;
        else break;
    }
    while (c->ovl_gather_wgs > 1 && c->ovl_sha_wps * sa + static_cast<int>(c->ovl_gather_wgs) * ga > 512)
        --c->ovl_gather_wgs;
}

int dfs_open(dfs_ctx** out, int device) {
    if (!out) return DFS_E_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return DFS_E_NODEV;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return DFS_E_NODEV;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return DFS_E_NODEV;
    dfs_ctx* c = new (std::nothrow) dfs_ctx;
    if (!c) return DFS_E_NOMEM;
    c->device = device;
    if (const char* w = std::getenv("DFS_SHA_WPS")) c->sha_wps = c->sha_wps_beside = std::max(1, std::min(8, std::atoi(w)));
    if (const char* w = std::getenv("DFS_UPLOAD_MODE"))
        c->upload_mode = std::strcmp(w, "fused") == 0 ? 0 : (std::strcmp(w, "hybrid") == 0 ? 2 : 1);
    if (const char* w = std::getenv("DFS_DOWNLOAD_MODE"))
        c->download_mode = std::strcmp(w, "serial") == 0 ? 1 : (std::strcmp(w, "pipelined") == 0 ? 0 : 2);
    if (const char* w = std::getenv("DFS_OVL_SHA_WPS")) c->ovl_sha_wps = std::max(1, std::min(3, std::atoi(w)));
    if (const char* w = std::getenv("DFS_OVL_DEC_WGS"))
        c->ovl_dec_wgs = static_cast<uint32_t>(std::max(1, std::min(4, std::atoi(w))));
    ovl_fit(c);
    if (const char* w = std::getenv("DFS_SHA_WAIT_TICKS")) c->wait_ticks = std::max<uint64_t>(1, std::strtoull(w, nullptr, 10));
    if (const char* w = std::getenv("DFS_SHA_WAIT_FORCE_TIMEOUT"))
        if (std::atoi(w)) {
            c->wait_never = 1;
            c->wait_ticks = 1000;
        }
    if (const char* w = std::getenv("DFS_B64_WGS")) c->b64_wgs = std::max(1, std::min(8, std::atoi(w)));
    if (const char* w = std::getenv("DFS_B64_PRIO")) c->b64_prio = static_cast<uint32_t>(std::atoi(w) & 3);
    if (const char* w = std::getenv("DFS_DEC_PRIO")) c->dec_prio = std::atoi(w) ? 1u : 0u;
    if (const char* w = std::getenv("DFS_RECV_FUSED")) c->recv_one_pass = w[0] != '0';
    if (const char* w = std::getenv("DFS_DEC_WGS")) c->dec_wgs = static_cast<uint32_t>(std::max(1, std::min(8, std::atoi(w))));
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = dfs::static_scratch_init(device);  // dfs_sha256_batch_static's device array
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking);
    for (int i = 0; e == hipSuccess && i < 2 * DFS_T_COUNT; ++i) e = hipEventCreate(&c->ev[i]);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->fork, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->join, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->scratch_ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->sync_ev, hipEventDisableTiming);
    for (auto& a : c->arena)
        if (e == hipSuccess) e = hipEventCreateWithFlags(&a.ev, hipEventDisableTiming);
    if (e != hipSuccess) {
        dfs_close(c);
        return hip_fail(e, "dfs_open");
    }
    *out = c;
    return DFS_OK;
}

int dfs_close(dfs_ctx* c) {
    if (!c) return DFS_E_ARG;
    (void)hipSetDevice(c->device);
    if (c->own) (void)hipStreamSynchronize(c->own);
    if (c->aux) (void)hipStreamSynchronize(c->aux);
    for (auto& b : c->buf) b.release();
    dfs::store_staging_free(c->store);
    for (auto& ev : c->ev)
        if (ev) (void)hipEventDestroy(ev);
    for (hipEvent_t ev : {c->fork, c->join, c->scratch_ev, c->sync_ev})
        if (ev) (void)hipEventDestroy(ev);
    for (hipEvent_t ev : c->pass_ev) (void)hipEventDestroy(ev);
    for (auto& a : c->arena) {
        if (a.ev) (void)hipEventDestroy(a.ev);
        if (a.p) (void)hipHostFree(a.p);
    }
    if (c->own) (void)hipStreamDestroy(c->own);
    if (c->aux) (void)hipStreamDestroy(c->aux);
    delete c;
    return DFS_OK;
}

int dfs_set_stream(dfs_ctx* c, void* s) {
    if (!c) return DFS_E_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    c->user = static_cast<hipStream_t>(s);
    return DFS_OK;
}

int dfs_set_profiling(dfs_ctx* c, int on) {
    if (!c) return DFS_E_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    c->profiling = on != 0;
    return DFS_OK;
}

int dfs_get_timings(dfs_ctx* c, float* ms, int n) {
    if (!c || !ms) return DFS_E_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    if (int rc = enter(c)) return rc;
    for (int k = 0; k < n && k < DFS_T_COUNT; ++k) {
        ms[k] = -1.0f;
        if (!c->ev_used[k]) continue;
        HIPC(dfs::quiet_wait(c->ev[2 * k + 1]));
        HIPC(hipEventElapsedTime(&ms[k], c->ev[2 * k], c->ev[2 * k + 1]));
    }
    return DFS_OK;
}

int dfs_get_stats(dfs_ctx* c, uint64_t* out, int n) {
    if (!c || !out) return DFS_E_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    for (int k = 0; k < n; ++k)
        out[k] = k == DFS_S_OVL_REDO ? c->ovl_redo : k == DFS_S_RECV_ONE_PASS ? c->recv_one_pass_calls : 0;
    return DFS_OK;
}

int dfs_split_plan(uint64_t file_len, uint32_t nfrag, dfs_span* frags) {
    if (!nfrag || !frags) return DFS_E_ARG;
    for (uint32_t i = 0; i < nfrag; ++i) {
        const uint64_t base = file_len / nfrag, rem = file_len % nfrag;
        frags[i].len = base + (i < rem ? 1 : 0);
        frags[i].off = i * base + (i < rem ? i : rem);
    }
    return DFS_OK;
}

uint64_t dfs_b64_encoded_len(uint64_t n) { return enc_len(n); }
uint64_t dfs_b64_decoded_cap(uint64_t n) { return 3 * ((n + 3) / 4); }

int dfs_fragment_holders(uint32_t f, uint32_t n, uint32_t holders[2]) {
    if (!n || f >= n || !holders) return DFS_E_ARG;
    holders[0] = f;                // nodeA = i+1 (1-based), SN:427
    holders[1] = (f + n - 1) % n;  // nodeB = ((i-1+N)%N)+1, SN:428
    return DFS_OK;
}

// ---------------------------------------------------------------------------
int dfs_sha256_batch(dfs_ctx* c, const uint8_t* base, const dfs_span* msgs, uint32_t n, uint8_t* digests,
                     uint32_t flags) {
    if (!c || (n && (!msgs || !digests))) return DFS_E_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    if (int rc = enter(c)) return rc;
    Timer tm(c);
    if (!n) return DFS_OK;
    const bool dev = flags & DFS_DEVICE_PTRS;
    hipStream_t s = c->stream();
    Scratch scratch(c, s);
    std::vector<ShaDesc> d(n);
    uint64_t end = 0;
    for (uint32_t i = 0; i < n; ++i) {
        if (msgs[i].len >= kMaxMsg) return DFS_E_ARG;
        d[i] = msg(msgs[i].off, msgs[i].len, i);
        end = std::max(end, msgs[i].off + msgs[i].len);
    }
    if (end && !base) return DFS_E_ARG;
    const uint32_t prio = sort_lanes(d);
    const uint8_t* d_base = base;
    uint8_t* d_dig = digests;
    if (!dev) {
        if (int rc = put(c, B_DATA_IN, base, end, s)) return rc;
        d_base = c->buf[B_DATA_IN].as<uint8_t>();
        HIPC(c->buf[B_DIG0].ensure(32ull * n));
        d_dig = c->buf[B_DIG0].as<uint8_t>();
    }
    if (int rc = put(c, B_DESC, d.data(), d.size() * sizeof(ShaDesc), s)) return rc;
    tm.begin(DFS_T_TOTAL, s);
    tm.begin(DFS_T_SHA, s);
    HIPC(c->buf[B_QUEUE].ensure(dfs::kShaQueueBytes));
    HIPC(dfs::launch_sha256(d_base, c->buf[B_DESC].as<ShaDesc>(), n, n, prio, d_dig, d_dig,
                            c->buf[B_QUEUE].as<uint32_t>(), c->sha_wps, s));
    tm.end(DFS_T_SHA, s);
    tm.end(DFS_T_TOTAL, s);
    if (!dev) {
        HIPC(dfs::d2h(c, digests, d_dig, 32ull * n, s));
        HIPC(dfs::quiet_sync(c, s));
    }
    return DFS_OK;
}

// ---------------------------------------------------------------------------
// dfs_sha256_batch for callers that cannot allocate: every buffer is the
// caller's device memory and the kernels' scratch is the library's static
// device array (sha256.hip).  No hipMalloc / hipFree, no host staging.
static_assert(DFS_STATIC_MAX_MSGS == dfs::kStaticMaxMsgs, "header and kernel limits agree");
int dfs_sha256_batch_static(dfs_ctx* c, const uint8_t* d_base, const dfs_span* d_msgs, uint32_t n, uint8_t* d_digests,
                            int32_t* d_status) {
    if (!c || (n && (!d_msgs || !d_digests))) return DFS_E_ARG;
    if (n > DFS_STATIC_MAX_MSGS) return DFS_E_TOOBIG;
    std::lock_guard<std::mutex> lk(c->mu);
    if (int rc = enter(c)) return rc;
    Timer tm(c);
    if (!n) return DFS_OK;
    hipStream_t s = c->stream();
    tm.begin(DFS_T_TOTAL, s);
    tm.begin(DFS_T_SHA, s);
    HIPC(dfs::launch_sha256_static(c->device, d_base, reinterpret_cast<const uint64_t*>(d_msgs), n, d_digests, d_status,
                                   c->sha_wps, s));
    tm.end(DFS_T_SHA, s);
    tm.end(DFS_T_TOTAL, s);
    return DFS_OK;
}

// ---------------------------------------------------------------------------
int dfs_sha256_update_batch(dfs_ctx* c, const uint8_t* base, const dfs_span* parts, uint32_t n, uint32_t* state,
                            const uint64_t* total_len, uint8_t* digests, uint32_t flags) {
    const bool begin = flags & DFS_SHA_BEGIN, fin = flags & DFS_SHA_FINAL;
    if (!c || (n && (!parts || !state || (fin && (!total_len || !digests))))) return DFS_E_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    if (int rc = enter(c)) return rc;
    Timer tm(c);
    if (!n) return DFS_OK;
    const bool dev = flags & DFS_DEVICE_PTRS;
    hipStream_t s = c->stream();
    Scratch scratch(c, s);
    std::vector<ShaDesc> d(n);
    uint64_t end = 0;
    for (uint32_t i = 0; i < n; ++i) {
        if (parts[i].len >= kMaxMsg || (!fin && (parts[i].len & 63u))) return DFS_E_ARG;
        if (fin && total_len[i] < parts[i].len) return DFS_E_ARG;
        d[i] = ShaDesc{parts[i].off, parts[i].len, fin ? total_len[i] : parts[i].len, i,
                       (begin ? 0u : dfs::kShaResume) | (fin ? 0u : dfs::kShaPartial)};
        end = std::max(end, parts[i].off + parts[i].len);
    }
    if (end && !base) return DFS_E_ARG;
    const uint32_t prio = sort_lanes(d);
    const uint8_t* d_base = base;
    uint32_t* d_state = state;
    uint8_t* d_dig = digests;
    if (!dev) {
        if (int rc = put(c, B_DATA_IN, base, end, s)) return rc;
        d_base = c->buf[B_DATA_IN].as<uint8_t>();
        if (int rc = put(c, B_STATUS, state, begin ? 0 : 32ull * n, s)) return rc;
        HIPC(c->buf[B_STATUS].ensure(32ull * n));
        d_state = c->buf[B_STATUS].as<uint32_t>();
        HIPC(c->buf[B_DIG0].ensure(32ull * n));
        d_dig = c->buf[B_DIG0].as<uint8_t>();
    }
    if (int rc = put(c, B_DESC, d.data(), d.size() * sizeof(ShaDesc), s)) return rc;
    HIPC(c->buf[B_QUEUE].ensure(dfs::kShaQueueBytes));
    tm.begin(DFS_T_TOTAL, s);
    tm.begin(DFS_T_SHA, s);
    HIPC(dfs::launch_sha256(d_base, c->buf[B_DESC].as<ShaDesc>(), n, n, prio, d_dig, d_dig,
                            c->buf[B_QUEUE].as<uint32_t>(), c->sha_wps, s, d_state));
    tm.end(DFS_T_SHA, s);
    tm.end(DFS_T_TOTAL, s);
    if (!dev) {
        if (fin) HIPC(dfs::d2h(c, digests, d_dig, 32ull * n, s));
        else HIPC(dfs::d2h(c, state, d_state, 32ull * n, s));
        HIPC(dfs::quiet_sync(c, s));
    }
    return DFS_OK;
}

// ---------------------------------------------------------------------------
}  // extern "C"

namespace {

// dfs_receive_fragments_batch in one pass (sha256_b64dec_any_lanes: a lane
// decodes, stores and hashes its message) for batches big enough for the
// persistent kernel whose messages start on dword boundaries and decode to
// 16-byte aligned places.  Returns 1 if the batch is not of that kind (the
// caller then decodes and hashes with the two kernels), else the call's code.
int receive_one_pass(dfs_ctx* c, const char* in, const dfs_span* msgs, uint32_t n, uint8_t* out,
                     const uint64_t* out_off, uint64_t* out_len, uint8_t* digests, int32_t* status, uint32_t flags) {
    if (n <= dfs::kChainMaxLanes || !c->recv_one_pass) return 1;
    const bool dev = flags & DFS_DEVICE_PTRS;
    uint64_t in_end = 0, out_end = 0;
    for (uint32_t i = 0; i < n; ++i) {
        if ((msgs[i].off & 3u) || (out_off[i] & 15u) || msgs[i].len >= (kMaxMsg / 3) * 4) return 1;
        in_end = std::max(in_end, msgs[i].off + msgs[i].len);
        out_end = std::max(out_end, out_off[i] + dfs_b64_decoded_cap(msgs[i].len));
    }
    if ((in_end && !in) || (out_end && !out)) return DFS_E_ARG;
    if (dev && ((reinterpret_cast<uintptr_t>(in) & 3u) || (reinterpret_cast<uintptr_t>(out) & 15u))) return 1;
    std::lock_guard<std::mutex> lk(c->mu);
    if (int rc = enter(c)) return rc;
    Timer tm(c);
    hipStream_t s = c->stream();
    Scratch scratch(c, s);
    const char* d_in = in;
    uint8_t* d_out = out;
    if (!dev) {
        if (int rc = put(c, B_DATA_IN, in, in_end, s)) return rc;
        d_in = c->buf[B_DATA_IN].as<char>();
        HIPC(c->buf[B_DATA_OUT].ensure(out_end));
        d_out = c->buf[B_DATA_OUT].as<uint8_t>();
    }
    std::vector<dfs::DecLane> lanes(n);
    for (uint32_t i = 0; i < n; ++i) lanes[i] = dfs::DecLane{msgs[i].off, out_off[i], ~0ull, msgs[i].len, i, 0};
    std::stable_sort(lanes.begin(), lanes.end(), [](const dfs::DecLane& a, const dfs::DecLane& b) { return a.len > b.len; });
    if (int rc = put(c, B_DESC, lanes.data(), lanes.size() * sizeof(dfs::DecLane), s)) return rc;
    HIPC(c->buf[B_STATUS].ensure(4ull * n));
    HIPC(c->buf[B_OUTLEN].ensure(8ull * n));
    HIPC(c->buf[B_DIG1].ensure(32ull * n));
    HIPC(c->buf[B_QUEUE].ensure(dfs::kShaQueueBytes));
    ++c->recv_one_pass_calls;
    tm.begin(DFS_T_TOTAL, s);
    tm.begin(DFS_T_SHA, s);
    HIPC(dfs::launch_sha256_b64dec(d_in, c->buf[B_DESC].as<dfs::DecLane>(), n, d_out, c->buf[B_DIG1].as<uint8_t>(),
                                   c->buf[B_STATUS].as<int32_t>(), c->buf[B_QUEUE].as<uint32_t>(), c->sha_wps, s,
                                   c->buf[B_OUTLEN].as<uint64_t>()));
    tm.end(DFS_T_SHA, s);
    tm.end(DFS_T_TOTAL, s);
    std::vector<int32_t> st(n);
    std::vector<uint8_t> dig(32ull * n);
    HIPC(dfs::d2h(c, st.data(), c->buf[B_STATUS].p, 4ull * n, s));
    HIPC(dfs::d2h(c, out_len, c->buf[B_OUTLEN].p, 8ull * n, s));
    HIPC(dfs::d2h(c, dig.data(), c->buf[B_DIG1].p, 32ull * n, s));
    if (!dev && out_end) HIPC(dfs::d2h(c, out, d_out, out_end, s));
    HIPC(dfs::quiet_sync(c, s));
    int rc = DFS_OK;
    for (uint32_t i = 0; i < n; ++i) {
        status[i] = st[i] ? DFS_E_DECODE : DFS_OK;
        if (st[i]) {
            out_len[i] = 0;
            rc = DFS_E_DECODE;
        } else {
            std::memcpy(digests + 32ull * i, dig.data() + 32ull * i, 32);  // a failed message's digest stays untouched
        }
    }
    return rc;
}

}  // namespace

extern "C" {

int dfs_receive_fragments_batch(dfs_ctx* c, const char* in, const dfs_span* msgs, uint32_t n, uint8_t* out,
                                const uint64_t* out_off, uint64_t* out_len, uint8_t* digests, int32_t* status,
                                uint32_t flags) {
    if (!c || (n && (!msgs || !out_off || !digests || !out_len || !status))) return DFS_E_ARG;
    {
        const int one = receive_one_pass(c, in, msgs, n, out, out_off, out_len, digests, status, flags);
        if (one != 1) return one;
    }
    // Decode (SN:281); the decode call synchronises and fills out_len / status.
    int rc = dfs_b64_decode_batch(c, in, msgs, n, out, out_off, out_len, status, flags);
    if (rc != DFS_OK && rc != DFS_E_DECODE) return rc;
    std::vector<dfs_span> ok;
    std::vector<uint32_t> idx;
    for (uint32_t i = 0; i < n; ++i)
        if (status[i] == DFS_OK) {
            ok.push_back(dfs_span{out_off[i], out_len[i]});
            idx.push_back(i);
        }
    if (ok.empty()) return rc;
    // Hash the decoded bytes where they landed (SN:282).
    const bool dev = flags & DFS_DEVICE_PTRS;
    std::vector<uint8_t> dig(32ull * ok.size());
    if (dev) {
        std::lock_guard<std::mutex> lk(c->mu);
        if (int e = enter(c)) return e;
        hipStream_t s = c->stream();
        Scratch scratch(c, s);
        std::vector<ShaDesc> d(ok.size());
        for (size_t k = 0; k < ok.size(); ++k) d[k] = msg(ok[k].off, ok[k].len, k);
        const uint32_t prio = sort_lanes(d);
        HIPC(c->buf[B_DIG1].ensure(dig.size()));
        if (int e = put(c, B_DESC, d.data(), d.size() * sizeof(ShaDesc), s)) return e;
        HIPC(c->buf[B_QUEUE].ensure(dfs::kShaQueueBytes));
        HIPC(dfs::launch_sha256(out, c->buf[B_DESC].as<ShaDesc>(), static_cast<uint32_t>(d.size()),
                                static_cast<uint32_t>(d.size()), prio, c->buf[B_DIG1].as<uint8_t>(),
                                c->buf[B_DIG1].as<uint8_t>(), c->buf[B_QUEUE].as<uint32_t>(), c->sha_wps, s));
        HIPC(dfs::d2h(c, dig.data(), c->buf[B_DIG1].p, dig.size(), s));
        HIPC(dfs::quiet_sync(c, s));
    } else {
        if (int e = dfs_sha256_batch(c, out, ok.data(), static_cast<uint32_t>(ok.size()), dig.data(), 0)) return e;
    }
    for (size_t k = 0; k < idx.size(); ++k) std::memcpy(digests + 32ull * idx[k], dig.data() + 32 * k, 32);
    return rc;
}

// ---------------------------------------------------------------------------
int dfs_sha256_update_parts(dfs_ctx* c, const uint8_t* base, const dfs_part* parts, uint32_t n, uint32_t* state,
                            uint8_t* digests, uint32_t flags) {
    if (!c || !(flags & DFS_DEVICE_PTRS) || (n && (!parts || !state || !digests))) return DFS_E_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    if (int rc = enter(c)) return rc;
    Timer tm(c);
    if (!n) return DFS_OK;
    hipStream_t s = c->stream();
    Scratch scratch(c, s);
    std::vector<ShaDesc> d(n);
    uint64_t end = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const dfs_part& q = parts[i];
        const bool fin = q.flags & DFS_SHA_FINAL;
        if (q.len >= kMaxMsg || (!fin && (q.len & 63u)) || (fin && q.total < q.len)) return DFS_E_ARG;
        d[i] = ShaDesc{q.off, q.len, fin ? q.total : q.len, q.slot,
                       ((q.flags & DFS_SHA_BEGIN) ? 0u : dfs::kShaResume) | (fin ? 0u : dfs::kShaPartial), 0};
        end = std::max(end, q.off + q.len);
    }
    if (end && !base) return DFS_E_ARG;
    const uint32_t prio = sort_lanes(d);
    if (int rc = put(c, B_DESC, d.data(), d.size() * sizeof(ShaDesc), s)) return rc;
    HIPC(c->buf[B_QUEUE].ensure(dfs::kShaQueueBytes));
    tm.begin(DFS_T_TOTAL, s);
    tm.begin(DFS_T_SHA, s);
    // digests indexed by slot: split = UINT32_MAX keeps every slot in out0
    HIPC(dfs::launch_sha256(base, c->buf[B_DESC].as<ShaDesc>(), n, UINT32_MAX, prio, digests, digests,
                            c->buf[B_QUEUE].as<uint32_t>(), c->sha_wps, s, state));
    tm.end(DFS_T_SHA, s);
    tm.end(DFS_T_TOTAL, s);
    return DFS_OK;
}

// ---------------------------------------------------------------------------
int dfs_b64_encode_batch(dfs_ctx* c, const uint8_t* base, const dfs_span* msgs, uint32_t n, char* out,
                         uint64_t out_cap, uint64_t* out_off, uint32_t flags) {
    if (!c || !out_off || (n && !msgs)) return DFS_E_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    if (int rc = enter(c)) return rc;
    Timer tm(c);
    const bool dev = flags & DFS_DEVICE_PTRS;
    hipStream_t s = c->stream();
    Scratch scratch(c, s);
    uint64_t total = 0, end = 0;
    std::vector<StreamJob> jobs;
    std::vector<uint64_t> items;
    for (uint32_t i = 0; i < n; ++i) {
        out_off[i] = total;
        if (msgs[i].len) {
            StreamJob j{};
            j.src_off = msgs[i].off;
            j.len = msgs[i].len;
            j.dst_off = total;
            j.id = i;
            jobs.push_back(j);
            items.push_back((msgs[i].len + 11) / 12);
        }
        total += enc_len(msgs[i].len);
        end = std::max(end, msgs[i].off + msgs[i].len);
    }
    out_off[n] = total;
    if (total > out_cap || (total && !out) || (end && !base)) return DFS_E_ARG;
    const uint32_t njobs = static_cast<uint32_t>(jobs.size());
    const uint64_t ntiles = finish_jobs(jobs, items, static_cast<uint64_t>(dfs::kEncPer) * dfs::kStreamBlock);
    const uint8_t* d_base = base;
    char* d_out = out;
    if (!dev) {
        if (int rc = put(c, B_DATA_IN, base, end, s)) return rc;
        d_base = c->buf[B_DATA_IN].as<uint8_t>();
        HIPC(c->buf[B_DATA_OUT].ensure(total));
        d_out = c->buf[B_DATA_OUT].as<char>();
    } else if (reinterpret_cast<uintptr_t>(out) & 3u) {
        return DFS_E_ARG;
    }
    if (int rc = put(c, B_JOBS, jobs.data(), jobs.size() * sizeof(StreamJob), s)) return rc;
    tm.begin(DFS_T_TOTAL, s);
    tm.begin(DFS_T_B64ENC, s);
    HIPC(dfs::launch_b64_encode(d_base, c->buf[B_JOBS].as<StreamJob>(), njobs, ntiles, d_out, 8u, s));
    tm.end(DFS_T_B64ENC, s);
    tm.end(DFS_T_TOTAL, s);
    if (!dev) {
        if (total) HIPC(dfs::d2h(c, out, d_out, total, s));
        HIPC(dfs::quiet_sync(c, s));
    }
    return DFS_OK;
}

// ---------------------------------------------------------------------------
int dfs_b64_decode_batch(dfs_ctx* c, const char* in, const dfs_span* msgs, uint32_t n, uint8_t* out,
                         const uint64_t* out_off, uint64_t* out_len, int32_t* status, uint32_t flags) {
    if (!c || (n && (!msgs || !out_off || !out_len || !status))) return DFS_E_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    if (int rc = enter(c)) return rc;
    Timer tm(c);
    if (!n) return DFS_OK;
    const bool dev = flags & DFS_DEVICE_PTRS;
    hipStream_t s = c->stream();
    Scratch scratch(c, s);
    uint64_t in_end = 0, out_end = 0;
    for (uint32_t i = 0; i < n; ++i) {
        in_end = std::max(in_end, msgs[i].off + msgs[i].len);
        out_end = std::max(out_end, out_off[i] + dfs_b64_decoded_cap(msgs[i].len));
    }
    if ((in_end && !in) || (out_end && !out)) return DFS_E_ARG;
    const char* d_in = in;
    uint8_t* d_out = out;
    if (!dev) {
        if (int rc = put(c, B_DATA_IN, in, in_end, s)) return rc;
        d_in = c->buf[B_DATA_IN].as<char>();
        HIPC(c->buf[B_DATA_OUT].ensure(out_end));
        d_out = c->buf[B_DATA_OUT].as<uint8_t>();
    }
    std::vector<StreamJob> jobs(n);
    std::vector<uint64_t> items(n);
    for (uint32_t i = 0; i < n; ++i) {
        StreamJob& j = jobs[i];
        j = StreamJob{};
        j.src_off = msgs[i].off;
        j.len = msgs[i].len;
        j.dst_off = out_off[i];
        j.id = i;
        items[i] = dec_items(msgs[i].len, reinterpret_cast<uintptr_t>(d_out + out_off[i]));
    }
    const uint64_t ntiles = finish_jobs(jobs, items, static_cast<uint64_t>(dfs::kDecGpl) * dfs::kStreamBlock);
    if (int rc = put(c, B_JOBS, jobs.data(), jobs.size() * sizeof(StreamJob), s)) return rc;
    HIPC(c->buf[B_STATUS].ensure(4ull * n));
    HIPC(c->buf[B_OUTLEN].ensure(8ull * n));
    HIPC(hipMemsetAsync(c->buf[B_STATUS].p, 0, 4ull * n, s));
    tm.begin(DFS_T_TOTAL, s);
    tm.begin(DFS_T_B64DEC, s);
    HIPC(dfs::launch_b64_decode(d_in, c->buf[B_JOBS].as<StreamJob>(), n, ntiles, d_out,
                                c->buf[B_STATUS].as<int32_t>(), c->buf[B_OUTLEN].as<uint64_t>(), s));
    tm.end(DFS_T_B64DEC, s);
    tm.end(DFS_T_TOTAL, s);
    std::vector<int32_t> st(n);
    HIPC(dfs::d2h(c, st.data(), c->buf[B_STATUS].p, 4ull * n, s));
    HIPC(dfs::d2h(c, out_len, c->buf[B_OUTLEN].p, 8ull * n, s));
    if (!dev && out_end) HIPC(dfs::d2h(c, out, d_out, out_end, s));
    HIPC(dfs::quiet_sync(c, s));
    int rc = DFS_OK;
    for (uint32_t i = 0; i < n; ++i) {
        status[i] = st[i] ? DFS_E_DECODE : DFS_OK;
        if (st[i]) {
            out_len[i] = 0;
            rc = DFS_E_DECODE;
        }
    }
    return rc;
}

// ---------------------------------------------------------------------------
// Upload plan: descriptors built once on the host, uploaded once.
}  // extern "C"

namespace {

// The host half of an upload plan: SHA lanes (fileIds + fragments, and the
// fragments alone), encode jobs, Base64 layout.
struct HostPlan {
    std::vector<ShaDesc> all, frag;  // all = n_all lanes (fileIds + fragments) then their twins
    std::vector<StreamJob> enc, enc_twin;  // every fragment's encode job; those of the twins alone
    std::vector<uint64_t> b64_off;
    uint32_t prio_all = 0, prio_frag = 0, n_all = 0;
    uint64_t enc_tiles = 0, enc_twin_tiles = 0, total = 0;
    bool twins = false;
};

// The fileId + fragment lanes of one upload, fragments that can ride in
// their fileId lane as twins when `twins` (and the launch stays large).
void build_all_lanes(const dfs_span* files, uint32_t nfiles, uint32_t nfrag, const std::vector<ShaDesc>& frag,
                     bool twins, HostPlan& h) {
    std::vector<ShaDesc> tw;
    h.all.clear();
    h.all.reserve(nfiles + frag.size());
    for (uint32_t f = 0; f < nfiles; ++f)  // fileId, SN:127; fragments, SN:159
        add_lane_with_twins(h.all, tw, msg(files[f].off, files[f].len, f), frag.data() + static_cast<uint64_t>(f) * nfrag,
                            nfrag, twins);
    h.twins = !tw.empty();
    h.n_all = static_cast<uint32_t>(h.all.size());
    h.all.insert(h.all.end(), tw.begin(), tw.end());
}

int build_host_plan(const dfs_span* files, uint32_t nfiles, uint32_t nfrag, uint32_t flags, HostPlan& h,
                    bool twins = true) {
    const bool frag_major = flags & DFS_LAYOUT_FRAG_MAJOR;
    const uint64_t align = (flags & DFS_LAYOUT_ALIGN128) ? 128 : 1;
    const uint64_t nf = static_cast<uint64_t>(nfiles) * nfrag;
    if (nfiles + nf > 0xffffffffull) return DFS_E_ARG;
    h.frag.clear();
    h.enc.clear();
    h.frag.reserve(nf);
    std::vector<uint64_t> items;
    h.enc.reserve(nf + 1);
    items.reserve(nf);
    h.b64_off.assign(nf + 1, 0);
    std::vector<uint64_t> off(nfrag), len(nfrag);
    for (uint32_t f = 0; f < nfiles; ++f) {
        if (files[f].len >= kMaxMsg) return DFS_E_ARG;
        split(files[f].len, nfrag, off.data(), len.data());  // SN:138-157
        for (uint32_t i = 0; i < nfrag; ++i) {
            const uint64_t k = static_cast<uint64_t>(f) * nfrag + i;
            h.frag.push_back(msg(files[f].off + off[i], len[i], nfiles + k));  // SN:159
        }
    }
    build_all_lanes(files, nfiles, nfrag, h.frag, twins, h);
    if (h.twins && h.n_all < dfs::kTwinMinLanes) build_all_lanes(files, nfiles, nfrag, h.frag, false, h);
    // Base64 layout: [file][fragment] (default) or [fragment][file].
    uint64_t total = 0;
    auto place = [&](uint32_t f, uint32_t i) {
        const uint64_t k = static_cast<uint64_t>(f) * nfrag + i;
        const ShaDesc& d = h.frag[k];
        total = (total + align - 1) / align * align;
        h.b64_off[k] = total;
        if (d.len) {
            StreamJob j{};
            j.src_off = d.off;
            j.len = d.len;
            j.dst_off = total;
            j.id = static_cast<uint32_t>(k);
            h.enc.push_back(j);
            items.push_back((d.len + 11) / 12);
        }
        total += enc_len(d.len);  // SN:636
    };
    if (frag_major) {
        for (uint32_t i = 0; i < nfrag; ++i)
            for (uint32_t f = 0; f < nfiles; ++f) place(f, i);
    } else {
        for (uint32_t f = 0; f < nfiles; ++f)
            for (uint32_t i = 0; i < nfrag; ++i) place(f, i);
    }
    h.b64_off[nf] = total;
    h.total = total;
    // Fragment lanes carry their Base64 offset: the fused upload encodes in
    // the SHA pass (kShaB64 is ignored when the kernel gets no output).  A
    // plan with twins never runs fused (run_plan_locked).
    for (ShaDesc& d : h.frag) {
        d.b64 = h.b64_off[d.out - nfiles];
        d.flags |= dfs::kShaB64;
    }
    for (uint32_t i = 0; i < h.n_all; ++i) {
        ShaDesc& d = h.all[i];
        if (d.out >= nfiles) {
            d.b64 = h.b64_off[d.out - nfiles];
            d.flags |= dfs::kShaB64;
        }
    }
    std::vector<ShaDesc> lanes(h.all.begin(), h.all.begin() + h.n_all);
    h.prio_all = sort_lanes(lanes);  // twins stay behind the lanes, unsorted
    std::copy(lanes.begin(), lanes.end(), h.all.begin());
    h.prio_frag = sort_lanes(h.frag);
    // Hybrid upload: the fragment lanes write their own Base64 in the SHA pass
    // (kShaB64) and the encode kernel covers only the fragments hashed as
    // twins inside their fileId lane (the lane holds their blocks in registers
    // once, for two states; encoding there as well would put the Base64 on
    // the critical chain).
    h.enc_twin.clear();
    std::vector<uint64_t> titems;
    if (h.twins) {
        std::vector<uint8_t> is_twin(nf, 0);
        for (size_t i = h.n_all; i < h.all.size(); ++i) is_twin[h.all[i].out - nfiles] = 1;
        for (size_t q = 0; q + 0 < h.enc.size(); ++q)
            if (is_twin[h.enc[q].id]) {
                h.enc_twin.push_back(h.enc[q]);
                titems.push_back(items[q]);
            }
    }
    h.enc_twin_tiles = finish_jobs(h.enc_twin, titems, static_cast<uint64_t>(dfs::kEncPer) * dfs::kStreamBlock);
    h.enc_tiles = finish_jobs(h.enc, items, static_cast<uint64_t>(dfs::kEncPer) * dfs::kStreamBlock);
    return DFS_OK;
}

void fill_plan_header(dfs_upload_plan* p, const HostPlan& h, int device, uint32_t nfiles, uint32_t nfrag) {
    p->device = device;
    p->nfiles = nfiles;
    p->nfrag = nfrag;
    p->prio_all = h.prio_all;
    p->prio_frag = h.prio_frag;
    p->n_all = h.n_all;
    p->twins = h.twins;
    p->n_frag_only = static_cast<uint32_t>(h.frag.size());
    p->n_enc = static_cast<uint32_t>(h.enc.size() - 1);  // minus the sentinel
    p->enc_tiles = h.enc_tiles;
    p->n_enc_twin = static_cast<uint32_t>(h.enc_twin.size() - 1);
    p->enc_twin_tiles = h.enc_twin_tiles;
    p->b64_total = h.total;
}

// A plan whose device tables live in the ctx scratch (valid until the next
// call on the ctx): one-shot batches (dfs_upload_batch, the batcher) pay no
// hipMalloc / hipFree per call.  Asynchronous on the ctx stream.
int scratch_plan(dfs_ctx* c, const HostPlan& h, uint32_t nfiles, uint32_t nfrag, hipStream_t s, dfs_upload_plan& p) {
    fill_plan_header(&p, h, c->device, nfiles, nfrag);
    if (int rc = put(c, B_DESC, h.all.data(), h.all.size() * sizeof(ShaDesc), s)) return rc;
    if (int rc = put(c, B_JOBS2, h.frag.data(), h.frag.size() * sizeof(ShaDesc), s)) return rc;
    if (int rc = put(c, B_JOBS, h.enc.data(), h.enc.size() * sizeof(StreamJob), s)) return rc;
    if (int rc = put(c, B_JOBS3, h.enc_twin.data(), h.enc_twin.size() * sizeof(StreamJob), s)) return rc;
    HIPC(c->buf[B_QUEUE].ensure(dfs::kShaQueueBytes));
    p.d_enc_twin = c->buf[B_JOBS3].as<StreamJob>();
    p.d_all = c->buf[B_DESC].as<ShaDesc>();
    p.d_frag = c->buf[B_JOBS2].as<ShaDesc>();
    p.d_enc = c->buf[B_JOBS].as<StreamJob>();
    p.d_queue = c->buf[B_QUEUE].as<uint32_t>();
    return DFS_OK;
}

}  // namespace

extern "C" {

int dfs_upload_plan_create(dfs_ctx* c, const dfs_span* files, uint32_t nfiles, uint32_t nfrag, uint32_t flags,
                           dfs_upload_plan** out, uint64_t* b64_total) {
    if (!c || !out || !nfrag || (nfiles && !files)) return DFS_E_ARG;
    if (flags & ~(DFS_LAYOUT_FRAG_MAJOR | DFS_LAYOUT_ALIGN128)) return DFS_E_ARG;
    *out = nullptr;
    HostPlan h;
    if (int rc = build_host_plan(files, nfiles, nfrag, flags, h, c->upload_mode != 0)) return rc;
    std::lock_guard<std::mutex> lk(c->mu);
    if (int rc = enter(c)) return rc;
    auto* p = new (std::nothrow) dfs_upload_plan;
    if (!p) return DFS_E_NOMEM;
    fill_plan_header(p, h, c->device, nfiles, nfrag);
    p->b64_off = std::move(h.b64_off);
    hipError_t e = hipMalloc(&p->d_queue, dfs::kShaQueueBytes);
    if (e == hipSuccess) e = hipMalloc(&p->d_all, std::max<size_t>(h.all.size(), 1) * sizeof(ShaDesc));
    if (e == hipSuccess) e = hipMalloc(&p->d_frag, std::max<size_t>(h.frag.size(), 1) * sizeof(ShaDesc));
    if (e == hipSuccess) e = hipMalloc(&p->d_enc, h.enc.size() * sizeof(StreamJob));
    if (e == hipSuccess) e = hipMalloc(&p->d_enc_twin, h.enc_twin.size() * sizeof(StreamJob));
    if (e == hipSuccess)
        e = hipMemcpy(p->d_enc_twin, h.enc_twin.data(), h.enc_twin.size() * sizeof(StreamJob), hipMemcpyHostToDevice);
    if (e == hipSuccess && !h.all.empty())
        e = hipMemcpy(p->d_all, h.all.data(), h.all.size() * sizeof(ShaDesc), hipMemcpyHostToDevice);
    if (e == hipSuccess && !h.frag.empty())
        e = hipMemcpy(p->d_frag, h.frag.data(), h.frag.size() * sizeof(ShaDesc), hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = hipMemcpy(p->d_enc, h.enc.data(), h.enc.size() * sizeof(StreamJob), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        dfs_upload_plan_destroy(p);
        return hip_fail(e, "dfs_upload_plan_create");
    }
    if (b64_total) *b64_total = p->b64_total;
    *out = p;
    return DFS_OK;
}

int dfs_upload_plan_b64_offsets(const dfs_upload_plan* p, uint64_t* b64_off) {
    if (!p || !b64_off) return DFS_E_ARG;
    std::memcpy(b64_off, p->b64_off.data(), p->b64_off.size() * sizeof(uint64_t));
    return DFS_OK;
}

int dfs_upload_plan_destroy(dfs_upload_plan* p) {
    if (!p) return DFS_E_ARG;
    (void)hipSetDevice(p->device);
    if (p->d_queue) (void)hipFree(p->d_queue);
    if (p->d_all) (void)hipFree(p->d_all);
    if (p->d_frag) (void)hipFree(p->d_frag);
    if (p->d_enc) (void)hipFree(p->d_enc);
    if (p->d_enc_twin) (void)hipFree(p->d_enc_twin);
    delete p;
    return DFS_OK;
}

namespace {
int run_plan_locked(dfs_ctx* c, dfs_upload_plan* p, const uint8_t* d_files, uint8_t* d_fd, uint8_t* d_frd, char* d_b64,
                    uint32_t flags) {
    const bool do_fileid = !(flags & DFS_NO_FILEID);
    const bool do_b64 = !(flags & DFS_NO_B64) && p->n_enc;
    const bool serial = flags & DFS_SERIAL;
    // Fused (DFS_UPLOAD_MODE=fused, plans without twins): the fragment lanes
    // write every fragment's Base64.  Hybrid (DFS_UPLOAD_MODE=hybrid): the same
    // kernel on a plan with twins; the fragments that ride in their fileId
    // lane are encoded by the encode kernel beside it (a fifth of the bytes
    // for 1 MiB / N = 5; every fragment when all of them are twins).
    const bool hybrid = do_b64 && c->upload_mode == 2 && !serial;
    const bool fused = do_b64 && !serial && (hybrid || (c->upload_mode == 0 && !p->twins));
    if (!d_frd || (do_fileid && !d_fd) || (do_b64 && !d_b64)) return DFS_E_ARG;
    if (do_b64 && (reinterpret_cast<uintptr_t>(d_b64) & 3u)) return DFS_E_ARG;
    hipStream_t s = c->stream();
    
    if (flags & DFS_B64_ONLY) {  // the HBM-bound encode pass alone
        if (!do_b64) return DFS_OK;
        Timer tb(c);
        tb.begin(DFS_T_TOTAL, s);
        tb.begin(DFS_T_B64ENC, s);
        HIPC(dfs::launch_b64_encode(d_files, p->d_enc, p->n_enc, p->enc_tiles, d_b64, 8u, s, c->b64_prio));
        tb.end(DFS_T_B64ENC, s);
        tb.end(DFS_T_TOTAL, s);
        return DFS_OK;
    }
    if (!serial && !c->aux) HIPC(hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking));
    hipStream_t sb = serial ? s : c->aux;
    Timer tm(c);
    // separate Base64 encode kernel: every fragment, or (hybrid) the twins'
    const bool twin_enc = fused && hybrid && do_fileid && p->twins && p->n_enc_twin;
    const bool two = do_b64 && (!fused || twin_enc);
    const StreamJob* enc_jobs = twin_enc ? p->d_enc_twin : p->d_enc;
    const uint32_t enc_n = twin_enc ? p->n_enc_twin : p->n_enc;
    const uint64_t enc_tiles = twin_enc ? p->enc_twin_tiles : p->enc_tiles;
    const int wps = two && !serial ? c->sha_wps_beside : c->sha_wps;
    tm.begin(DFS_T_TOTAL, s);
    if (two && !serial) {  // fork: Base64 on the aux stream beside SHA
        HIPC(hipEventRecord(c->fork, s));
        HIPC(hipStreamWaitEvent(sb, c->fork, 0));
    }
    // Fused: the fragment lanes write the Base64 too (kShaB64, sha256.hip).
    char* fb64 = fused ? d_b64 : nullptr;
    tm.begin(DFS_T_SHA, s);
    if (do_fileid) {
        HIPC(dfs::launch_sha256(d_files, p->d_all, p->n_all, p->nfiles, p->prio_all, d_fd, d_frd, p->d_queue,
                                wps, s, nullptr, fb64));
    } else {
        HIPC(dfs::launch_sha256(d_files, p->d_frag, p->n_frag_only, p->nfiles, p->prio_frag, d_fd, d_frd,
                                p->d_queue, wps, s, nullptr, fb64));
    }
    tm.end(DFS_T_SHA, s);
    if (two) {
        tm.begin(DFS_T_B64ENC, sb);
        HIPC(dfs::launch_b64_encode(d_files, enc_jobs, enc_n, enc_tiles, d_b64,
                                    serial ? 8u : static_cast<uint32_t>(c->b64_wgs), sb, c->b64_prio));
        tm.end(DFS_T_B64ENC, sb);
        if (!serial) {  // join
            HIPC(hipEventRecord(c->join, sb));
            HIPC(hipStreamWaitEvent(s, c->join, 0));
        }
    }
    tm.end(DFS_T_TOTAL, s);
    return DFS_OK;
}
}  // namespace

int dfs_upload_plan_run(dfs_ctx* c, dfs_upload_plan* p, const uint8_t* d_files, uint8_t* d_fd, uint8_t* d_frd,
                        char* d_b64, uint32_t flags) {
    if (!c || !p || p->device != c->device) return DFS_E_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    if (int rc = enter(c)) return rc;
    Scratch scratch(c, c->stream());
    return run_plan_locked(c, p, d_files, d_fd, d_frd, d_b64, flags);
}

int dfs_upload_batch(dfs_ctx* c, const uint8_t* files, const dfs_span* spans, uint32_t nfiles, uint32_t nfrag,
                     uint8_t* fd, uint8_t* frd, char* b64, uint64_t b64_cap, uint64_t* b64_off, uint32_t flags) {
    if (!c || !nfrag || (nfiles && (!spans || !frd))) return DFS_E_ARG;
    if (!(flags & DFS_NO_FILEID) && nfiles && !fd) return DFS_E_ARG;
    HostPlan h;
    if (int rc = build_host_plan(spans, nfiles, nfrag, flags & DFS_LAYOUT_FRAG_MAJOR, h, c->upload_mode != 0))
        return rc;
    const bool do_b64 = !(flags & DFS_NO_B64);
    if (b64_off) std::memcpy(b64_off, h.b64_off.data(), h.b64_off.size() * sizeof(uint64_t));
    if (do_b64 && (h.total > b64_cap || (h.total && !b64))) return DFS_E_ARG;
    if (!nfiles) return DFS_OK;
    std::lock_guard<std::mutex> lk(c->mu);
    if (int rc = enter(c)) return rc;
    hipStream_t s = c->stream();
    Scratch scratch(c, s);
    const bool dev = flags & DFS_DEVICE_PTRS;
    uint64_t end = 0;
    for (uint32_t f = 0; f < nfiles; ++f) end = std::max(end, spans[f].off + spans[f].len);
    if (end && !files) return DFS_E_ARG;
    const uint64_t nf = static_cast<uint64_t>(nfiles) * nfrag;
    const uint8_t* d_files = files;
    uint8_t* d_fd = fd;
    uint8_t* d_frd = frd;
    char* d_b64 = b64;
    if (!dev) {
        if (int rc = put(c, B_DATA_IN, files, end, s)) return rc;
        d_files = c->buf[B_DATA_IN].as<uint8_t>();
        HIPC(c->buf[B_DIG0].ensure(32ull * nfiles));
        HIPC(c->buf[B_DIG1].ensure(32ull * nf));
        d_fd = c->buf[B_DIG0].as<uint8_t>();
        d_frd = c->buf[B_DIG1].as<uint8_t>();
        if (do_b64) {
            HIPC(c->buf[B_DATA_OUT].ensure(h.total));
            d_b64 = c->buf[B_DATA_OUT].as<char>();
        }
    }
    dfs_upload_plan p;
    if (int rc = scratch_plan(c, h, nfiles, nfrag, s, p)) return rc;
    if (int rc = run_plan_locked(c, &p, d_files, d_fd, d_frd, d_b64, flags)) return rc;
    if (!dev) {
        if (!(flags & DFS_NO_FILEID)) HIPC(dfs::d2h(c, fd, d_fd, 32ull * nfiles, s));
        HIPC(dfs::d2h(c, frd, d_frd, 32ull * nf, s));
        if (do_b64 && h.total) HIPC(dfs::d2h(c, b64, d_b64, h.total, s));
        HIPC(dfs::quiet_sync(c, s));
    }
    return DFS_OK;
}

// ---------------------------------------------------------------------------
int dfs_reassemble_verify(dfs_ctx* c, const uint8_t* const* src, const uint64_t* frag_len, uint32_t nfiles,
                          uint32_t nfrag, uint8_t* out, const uint64_t* file_off, const uint8_t* expected,
                          uint8_t* digest_out, int32_t* status, uint32_t flags) {
    if (!c || !nfrag || (nfiles && (!src || !frag_len || !out || !file_off || !status))) return DFS_E_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    if (int rc = enter(c)) return rc;
    Timer tm(c);
    if (!nfiles) return DFS_OK;
    const bool dev = flags & DFS_DEVICE_PTRS;
    hipStream_t s = c->stream();
    Scratch scratch(c, s);
    const uint64_t nf = static_cast<uint64_t>(nfiles) * nfrag;
    std::vector<uint64_t> flen(nfiles, 0);
    uint64_t out_end = 0, stage = 0;
    for (uint32_t f = 0; f < nfiles; ++f) {
        status[f] = DFS_OK;
        for (uint32_t i = 0; i < nfrag; ++i) {
            const uint64_t k = static_cast<uint64_t>(f) * nfrag + i;
            if (!src[k] && frag_len[k]) status[f] = DFS_E_MISSING;  // SN:443-446
            flen[f] += frag_len[k];
            stage += frag_len[k];
        }
        out_end = std::max(out_end, file_off[f] + flen[f]);
    }
    uint8_t* d_out = out;
    std::vector<uint64_t> src_addr(nf, 0);
    if (!dev) {
        // Stage every host fragment contiguously on the device.
        HIPC(c->buf[B_DATA_IN].ensure(stage));
        HIPC(c->buf[B_DATA_OUT].ensure(out_end));
        d_out = c->buf[B_DATA_OUT].as<uint8_t>();
        uint64_t o = 0;
        for (uint64_t k = 0; k < nf; ++k) {
            if (!src[k] || !frag_len[k]) continue;
            HIPC(hipMemcpyAsync(c->buf[B_DATA_IN].as<uint8_t>() + o, src[k], frag_len[k], hipMemcpyHostToDevice, s));
            src_addr[k] = reinterpret_cast<uint64_t>(c->buf[B_DATA_IN].as<uint8_t>() + o);
            o += frag_len[k];
        }
    } else {
        for (uint64_t k = 0; k < nf; ++k) src_addr[k] = reinterpret_cast<uint64_t>(src[k]);
    }
    // Large batches whose fragments have the split lengths (the normal case)
    // overlap the gather with the fileId SHA-256 as the download does: the
    // gather runs fragment by fragment (group g = fragment g of every file),
    // group 0 alone at full width, groups 1.. beside one SHA launch whose
    // lanes wait for each group (ShaWait with nf = 0: every lane a fileId).
    uint64_t nok = 0;
    bool split_lens = true;
    std::vector<uint64_t> soff(nfrag), slen(nfrag);
    for (uint32_t f = 0; f < nfiles && split_lens; ++f) {
        if (status[f] != DFS_OK) continue;
        ++nok;
        split(flen[f], nfrag, soff.data(), slen.data());
        for (uint32_t i = 0; i < nfrag; ++i) split_lens = split_lens && frag_len[static_cast<uint64_t>(f) * nfrag + i] == slen[i];
    }
    const bool ovl = c->download_mode == 2 && split_lens && nfrag > 1 && nfrag <= dfs::kShaWaitMaxGroups &&
                     nok > dfs::kChainMaxLanes;
    std::vector<StreamJob> jobs, gj;
    std::vector<uint64_t> items, gitems, gtile;
    std::vector<ShaDesc> sha;
    std::vector<uint64_t> frag_dst(nf, 0);
    for (uint32_t f = 0; f < nfiles; ++f) {
        if (status[f] != DFS_OK) continue;
        uint64_t o = file_off[f];
        for (uint32_t i = 0; i < nfrag; ++i) {
            const uint64_t k = static_cast<uint64_t>(f) * nfrag + i;
            frag_dst[k] = o;  // ordered append, SN:448
            o += frag_len[k];
        }
        sha.push_back(msg(file_off[f], flen[f], f));  // SN:454
    }
    // Jobs: file-major (serial), or fragment-major with group 0 in its own
    // table and groups 1.. in a second one with continuous tile numbers.
    uint64_t ntiles = 0, job2 = 0;
    const uint64_t per = static_cast<uint64_t>(dfs::kGatherPer) * dfs::kStreamBlock;
    auto add_job = [&](std::vector<StreamJob>& v, std::vector<uint64_t>& it, uint64_t k) {
        if (!frag_len[k]) return;
        StreamJob j{};
        j.src_off = src_addr[k];
        j.len = frag_len[k];
        j.dst_off = frag_dst[k];
        j.id = static_cast<uint32_t>(k);
        v.push_back(j);
        it.push_back(copy_items(frag_len[k], reinterpret_cast<uintptr_t>(d_out + frag_dst[k])));
    };
    if (!ovl) {
        for (uint32_t f = 0; f < nfiles; ++f)
            if (status[f] == DFS_OK)
                for (uint32_t i = 0; i < nfrag; ++i) add_job(jobs, items, static_cast<uint64_t>(f) * nfrag + i);
        ntiles = finish_jobs(jobs, items, per);
    } else {
        for (uint32_t f = 0; f < nfiles; ++f)
            if (status[f] == DFS_OK) add_job(jobs, items, static_cast<uint64_t>(f) * nfrag);
        ntiles = finish_jobs(jobs, items, per);
        job2 = jobs.size();
        uint64_t t = 0;
        for (uint32_t i = 1; i < nfrag; ++i) {
            gj.clear();
            gitems.clear();
            for (uint32_t f = 0; f < nfiles; ++f)
                if (status[f] == DFS_OK) add_job(gj, gitems, static_cast<uint64_t>(f) * nfrag + i);
            gtile.push_back(t);
            const uint64_t gt = finish_jobs(gj, gitems, per);
            for (size_t q = 0; q + 1 < gj.size(); ++q) {  // without the group's sentinel
                gj[q].tile_start += t;
                jobs.push_back(gj[q]);
            }
            t += gt;
        }
        gtile.push_back(t);
        StreamJob sent{};
        sent.tile_start = t;
        jobs.push_back(sent);
    }
    const uint32_t njobs = static_cast<uint32_t>(ovl ? job2 - 1 : jobs.size() - 1);
    const uint32_t prio = sort_lanes(sha);
    if (int rc = put(c, B_JOBS, jobs.data(), jobs.size() * sizeof(StreamJob), s)) return rc;
    if (int rc = put(c, B_DESC, sha.data(), sha.size() * sizeof(ShaDesc), s)) return rc;
    if (ovl)
        if (int rc = put(c, B_JOBS2, gtile.data(), gtile.size() * sizeof(uint64_t), s)) return rc;
    HIPC(c->buf[B_DIG0].ensure(32ull * nfiles));
    HIPC(c->buf[B_QUEUE].ensure(dfs::kShaQueueBytes));
    uint8_t* d_dig = c->buf[B_DIG0].as<uint8_t>();
    uint32_t* d_queue = c->buf[B_QUEUE].as<uint32_t>();
    const StreamJob* d_jobs = c->buf[B_JOBS].as<StreamJob>();
    tm.begin(DFS_T_TOTAL, s);
    if (!ovl) {
        tm.begin(DFS_T_GATHER, s);
        HIPC(dfs::launch_gather(d_jobs, njobs, ntiles, d_out, s));
        tm.end(DFS_T_GATHER, s);
        tm.begin(DFS_T_SHA, s);
        HIPC(dfs::launch_sha256(d_out, c->buf[B_DESC].as<ShaDesc>(), static_cast<uint32_t>(sha.size()), nfiles, prio,
                                d_dig, d_dig, d_queue, c->sha_wps, s));
        tm.end(DFS_T_SHA, s);
    } else {
        if (!c->aux) HIPC(hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking));
        if (c->pass_ev.empty()) {
            hipEvent_t ev = nullptr;
            HIPC(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            c->pass_ev.push_back(ev);
        }
        HIPC(hipMemsetAsync(d_queue, 0, dfs::kShaQueueBytes, s));  // the group counters (see dfs_download_batch)
        tm.begin(DFS_T_GATHER, s);
        HIPC(dfs::launch_gather(d_jobs, njobs, ntiles, d_out, s));
        HIPC(hipEventRecord(c->pass_ev[0], s));
        dfs::StreamAhead ah{c->buf[B_JOBS2].as<uint64_t>(), nfrag - 1, 256u * c->ovl_gather_wgs,
                            d_queue + dfs::kShaWaitSlot + 1};
        HIPC(dfs::launch_gather(d_jobs + job2, static_cast<uint32_t>(jobs.size() - job2 - 1), gtile.back(), d_out, s,
                                &ah));
        tm.end(DFS_T_GATHER, s);
        HIPC(hipStreamWaitEvent(c->aux, c->pass_ev[0], 0));
        tm.begin(DFS_T_SHA, c->aux);
        const dfs::ShaWait wt{d_queue + dfs::kShaWaitSlot, ah.grid + c->wait_never, 1u, nfrag, 0u, c->wait_ticks};
        HIPC(dfs::launch_sha256(d_out, c->buf[B_DESC].as<ShaDesc>(), static_cast<uint32_t>(sha.size()), nfiles, prio,
                                d_dig, d_dig, d_queue, c->ovl_sha_wps, c->aux, nullptr, nullptr, &wt));
        tm.end(DFS_T_SHA, c->aux);
        HIPC(hipEventRecord(c->join, c->aux));
        HIPC(hipStreamWaitEvent(s, c->join, 0));
    }
    tm.end(DFS_T_TOTAL, s);
    std::vector<uint8_t> dig(32ull * nfiles);
    uint32_t timed_out = 0;
    if (ovl) HIPC(dfs::d2h(c, &timed_out, d_queue + 2, 4, s));
    HIPC(dfs::d2h(c, dig.data(), d_dig, dig.size(), s));
    if (!dev && out_end) HIPC(dfs::d2h(c, out, d_out, out_end, s));
    HIPC(dfs::quiet_sync(c, s));
    if (timed_out) {  // an in-kernel wait gave up: hash again now that the gather is complete
        ++c->ovl_redo;
        HIPC(dfs::launch_sha256(d_out, c->buf[B_DESC].as<ShaDesc>(), static_cast<uint32_t>(sha.size()), nfiles, prio,
                                d_dig, d_dig, d_queue, c->sha_wps, s));
        HIPC(dfs::d2h(c, dig.data(), d_dig, dig.size(), s));
        HIPC(dfs::quiet_sync(c, s));
    }
    int rc = DFS_OK;
    for (uint32_t f = 0; f < nfiles; ++f) {
        if (status[f] == DFS_OK && expected && std::memcmp(dig.data() + 32ull * f, expected + 32ull * f, 32) != 0)
            status[f] = DFS_E_CORRUPT;  // SN:455-458
        if (digest_out) std::memcpy(digest_out + 32ull * f, dig.data() + 32ull * f, 32);
        if (status[f] != DFS_OK && rc == DFS_OK) rc = status[f];
    }
    return rc;
}

// ---------------------------------------------------------------------------
// Download (Base64 transport): host tables of one batch shape, and the launch
// sequence over device tables.  dfs_download_batch builds the tables per call
// into the ctx scratch; a dfs_download_plan builds them once and keeps them in
// HBM (dfs_download_plan_create / _run).
}  // extern "C"

struct DlTables {
    uint32_t nfiles = 0, nfrag = 0;
    uint64_t nf = 0;          // nfiles * nfrag
    uint32_t nout = 0;        // digest slots: nf fragments + nfiles fileIds
    uint64_t in_end = 0, out_end = 0;
    uintptr_t out_align = 0;  // d_out mod 16 the decode tiling was built for
    bool ovl = false, pipe = false;
    uint32_t npass = 0, nsha = 0;
    std::vector<int32_t> status0;  // per file: DFS_OK or DFS_E_MISSING (SN:443-446)
    std::vector<StreamJob> jobs;   // per-pass tables, then (ovl) groups 1.. with continuous tiles
    std::vector<ShaDesc> sha;      // per SHA launch: its lanes, then their twins
    std::vector<uint64_t> gtile;   // ovl: group bounds of the ahead decode
    std::vector<uint64_t> job0, desc0, tiles;
    std::vector<uint32_t> prio, nlanes;
    uint64_t job2 = 0;
    uint64_t njobs = 0;  // entries of `jobs` (kept when a plan drops the host copy)
};

// Device side of a download: the tables and the per-run result buffers.
struct DlDev {
    const StreamJob* jobs = nullptr;
    const ShaDesc* desc = nullptr;
    const uint64_t* gtile = nullptr;
    int32_t* st = nullptr;       // decode status per fragment
    int32_t* verdict = nullptr;  // per file (device-resident expected digests)
    uint8_t* dig = nullptr;      // 32 * (nf + nfiles)
    uint32_t* queue = nullptr;
    uint32_t* state = nullptr;   // pipelined passes: running fileId states (32 * nout)
};

struct dfs_download_plan {
    int device = 0;
    DlTables t;
    DlDev d;
    void* mem[8] = {};
};

namespace {

// Decode jobs write straight into the file at the split offsets (fused gather).
// Large batches, default (overlap): the decode runs fragment by fragment
// (group g = fragment g of every file): group 0 alone at full width, then
// groups 1.. beside ONE SHA launch over every lane (fileIds whole, twins),
// which waits in-kernel for each group's completion count (ShaWait,
// dfs_internal.h; bounded, the SHA launch is redone after the decode if a
// wait ever times out).  Pipelined (DFS_DOWNLOAD_MODE=pipelined): passes
// over fragment groups {0}, {1, 2}, {3..6}, ...:
// pass p decodes its group of every file on s while the aux stream hashes
// pass p - 1's fragments and advances every fileId over them (state in
// HBM between launches, kShaResume / kShaPartial), so the SHA starts after
// one fragment's decode instead of the whole batch's, and each decode pass
// runs beside a SHA launch about as long as itself.  A fileId part ends on
// the last 64-byte boundary inside its group, so it reads decoded bytes only.
int build_dl_tables(const dfs_ctx* c, const dfs_span* msgs, uint32_t nfiles, uint32_t nfrag, const uint64_t* file_len,
                    const uint64_t* file_off, uintptr_t out_base, DlTables& t) {
    t.nfiles = nfiles;
    t.nfrag = nfrag;
    const uint64_t nf = static_cast<uint64_t>(nfiles) * nfrag;
    if (nf + nfiles > 0xffffffffull) return DFS_E_ARG;
    t.nf = nf;
    t.nout = static_cast<uint32_t>(nf + nfiles);
    t.out_align = out_base & 15u;
    t.status0.assign(nfiles, DFS_OK);
    std::vector<int32_t>& status = t.status0;
    t.in_end = t.out_end = 0;
    for (uint32_t f = 0; f < nfiles; ++f) {
        if (file_len[f] >= kMaxMsg) return DFS_E_ARG;
        t.out_end = std::max(t.out_end, file_off[f] + file_len[f]);
        for (uint32_t i = 0; i < nfrag; ++i) {
            const dfs_span& m = msgs[static_cast<uint64_t>(f) * nfrag + i];
            if (m.len == DFS_SPAN_MISSING) status[f] = DFS_E_MISSING;  // SN:443-446
            else t.in_end = std::max(t.in_end, m.off + m.len);
        }
    }
    uint64_t nok = 0;
    for (uint32_t f = 0; f < nfiles; ++f) nok += status[f] == DFS_OK;
    const bool big = nfrag > 1 && nok * (nfrag + 1) > dfs::kChainMaxLanes;
    const bool ovl = big && c->download_mode == 2 && nfrag <= dfs::kShaWaitMaxGroups;
    const bool pipe = big && c->download_mode == 0;
    t.ovl = ovl;
    t.pipe = pipe;
    std::vector<uint32_t> gb{0};  // decode group p = fragments [gb[p], gb[p + 1])
    for (uint32_t w = 1; gb.back() < nfrag; w *= 2)
        gb.push_back(ovl ? gb.back() + 1 : (pipe ? std::min(nfrag, gb.back() + w) : nfrag));
    const uint32_t npass = static_cast<uint32_t>(gb.size() - 1);
    const uint32_t nsha = ovl ? 1 : npass;  // SHA launches (overlap: one over every lane)
    t.npass = npass;
    t.nsha = nsha;
    std::vector<StreamJob>& jobs = t.jobs;
    std::vector<StreamJob> pjobs;
    std::vector<uint64_t> items;
    std::vector<ShaDesc>& sha = t.sha;
    std::vector<ShaDesc> psha, ptw, gfr;  // per pass: fragments (out = k), files (out = nf + f); twins
    jobs.clear();
    sha.clear();
    t.job0.assign(npass + 1, 0);
    t.desc0.assign(nsha + 1, 0);
    t.tiles.assign(npass, 0);
    t.prio.assign(nsha, 0);
    t.nlanes.assign(nsha, 0);
    std::vector<uint64_t> off(nfrag), len(nfrag);
    // SHA lanes of launch p (fragments [i0, i1)): each file's fileId part,
    // with the fragments that sit on its block grid as twins (twins only if
    // the launch stays above kChainMaxLanes lanes).
    auto pass_lanes = [&](uint32_t p, bool twins) {
        const uint32_t i0 = ovl ? 0 : gb[p], i1 = ovl ? nfrag : gb[p + 1];
        psha.clear();
        ptw.clear();
        for (uint32_t f = 0; f < nfiles; ++f) {
            if (status[f] != DFS_OK) continue;
            split(file_len[f], nfrag, off.data(), len.data());
            gfr.clear();
            for (uint32_t i = i0; i < i1; ++i)
                gfr.push_back(msg(file_off[f] + off[i], len[i], static_cast<uint64_t>(f) * nfrag + i));
            const bool first = p == 0, last = p + 1 == nsha;
            const uint64_t a = first ? 0 : off[i0] & ~63ull, e = last ? file_len[f] : off[i1] & ~63ull;
            ShaDesc d = msg(file_off[f] + a, e - a, nf + f);
            d.total = file_len[f];
            d.flags = (first ? 0u : dfs::kShaResume) | (last ? 0u : dfs::kShaPartial);
            add_lane_with_twins(psha, ptw, d, gfr.data(), static_cast<uint32_t>(gfr.size()), twins);
        }
    };
    for (uint32_t p = 0; p < npass; ++p) {
        pjobs.clear();
        items.clear();
        for (uint32_t f = 0; f < nfiles; ++f) {
            if (status[f] != DFS_OK) continue;
            split(file_len[f], nfrag, off.data(), len.data());
            for (uint32_t i = gb[p]; i < gb[p + 1]; ++i) {
                const uint64_t k = static_cast<uint64_t>(f) * nfrag + i;
                StreamJob j{};
                j.src_off = msgs[k].off;
                j.len = msgs[k].len;
                j.dst_off = file_off[f] + off[i];
                j.expect = len[i] + 1;
                j.id = static_cast<uint32_t>(k);
                pjobs.push_back(j);
                items.push_back(dec_items(msgs[k].len, out_base + j.dst_off));
            }
        }
        t.tiles[p] = finish_jobs(pjobs, items, static_cast<uint64_t>(dfs::kDecGpl) * dfs::kStreamBlock);
        jobs.insert(jobs.end(), pjobs.begin(), pjobs.end());
        t.job0[p + 1] = jobs.size();
        if (p >= nsha) continue;
        pass_lanes(p, true);
        if (!ptw.empty() && psha.size() < dfs::kTwinMinLanes) pass_lanes(p, false);
        // Overlap: fragment lanes group-major (fragment 1 of every file, then
        // fragment 2, ...; fileIds first) before the stable longest-first
        // sort, so each 64-lane item waits for one group and the queue hands
        // out items in decode order.  File-major items would hold fragments
        // 1..N-1 of 16 files and wait for the last group.
        if (ovl) {  // stable bucket pass by (fileId | fragment index), O(n)
            auto key = [&](const ShaDesc& x) { return x.out >= nf ? 0u : 1u + static_cast<uint32_t>(x.out % nfrag); };
            std::vector<size_t> start(nfrag + 2, 0);
            for (const ShaDesc& x : psha) ++start[key(x) + 1];
            for (uint32_t b = 0; b <= nfrag; ++b) start[b + 1] += start[b];
            gfr.resize(psha.size());
            for (const ShaDesc& x : psha) gfr[start[key(x)]++] = x;
            psha.swap(gfr);
        }
        t.prio[p] = sort_lanes(psha);  // one message per lane, longest first
        // Long items (balanced per SIMD, sha256_body): the fileId parts, which
        // are |group| fragments long; in a one-fragment pass every lane is
        // about one fragment long, so every item counts as long.
        if (pipe) t.prio[p] = static_cast<uint32_t>(gb[p + 1] - gb[p] == 1 ? psha.size() : nok);
        t.nlanes[p] = static_cast<uint32_t>(psha.size());
        sha.insert(sha.end(), psha.begin(), psha.end());
        sha.insert(sha.end(), ptw.begin(), ptw.end());
        t.desc0[p + 1] = sha.size();
    }
    // Overlap: groups 1.. as one job table with continuous tile numbers
    // (jobs2, after the per-group tables) and group bounds gtile.
    t.gtile.clear();
    t.job2 = 0;
    if (ovl) {
        t.job2 = jobs.size();
        uint64_t tt = 0;
        for (uint32_t p = 1; p < npass; ++p) {
            t.gtile.push_back(tt);
            for (uint64_t j = t.job0[p]; j + 1 < t.job0[p + 1]; ++j) {  // without the group's sentinel
                StreamJob x = jobs[j];
                x.tile_start += tt;
                jobs.push_back(x);
            }
            tt += t.tiles[p];
        }
        t.gtile.push_back(tt);
        StreamJob sent{};
        sent.tile_start = tt;
        jobs.push_back(sent);
    }
    t.njobs = jobs.size();
    return DFS_OK;
}

// Launch sequence + result fetch of one download over device tables.  status
// must hold the caller's view of t.status0 on entry (DFS_OK / DFS_E_MISSING).
int run_dl(dfs_ctx* c, const DlTables& t, const DlDev& D, const char* d_in, uint8_t* d_out, const uint8_t* exp_frag,
           const uint8_t* exp_file, bool dev, uint8_t* host_out, int32_t* status, hipStream_t s, Timer& tm) {
    const uint32_t nfiles = t.nfiles, nfrag = t.nfrag, npass = t.npass;
    const uint64_t nf = t.nf;
    const uint32_t nout = t.nout;
    const bool ovl = t.ovl, pipe = t.pipe;
    HIPC(dfs::launch_fill_u32(reinterpret_cast<uint32_t*>(D.st), nf, 0u, s));
    uint8_t* d_dig = D.dig;
    const StreamJob* d_jobs = D.jobs;
    const ShaDesc* d_desc = D.desc;
    int32_t* d_st = D.st;
    uint32_t* d_queue = D.queue;
    tm.begin(DFS_T_TOTAL, s);
    if (ovl) {
        if (!c->aux) HIPC(hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking));
        if (c->pass_ev.empty()) {
            hipEvent_t ev = nullptr;
            HIPC(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            c->pass_ev.push_back(ev);
        }
        // The counters live in the SHA queue words, zeroed here (before the
        // decode that publishes them; the SHA launch does not re-zero them).
        HIPC(dfs::launch_fill_u32(d_queue, dfs::kShaQueueBytes / 4, 0u, s));
        tm.begin(DFS_T_B64DEC, s);
        HIPC(dfs::launch_b64_decode(d_in, d_jobs, static_cast<uint32_t>(t.job0[1]), t.tiles[0], d_out, d_st, nullptr, s));
        HIPC(hipEventRecord(c->pass_ev[0], s));
        dfs::StreamAhead ah{D.gtile, npass - 1, 256u * c->ovl_dec_wgs, d_queue + dfs::kShaWaitSlot + 1};
        HIPC(dfs::launch_b64_decode(d_in, d_jobs + t.job2, static_cast<uint32_t>(t.njobs - t.job2), t.gtile.back(),
                                    d_out, d_st, nullptr, s, c->dec_prio, 0, &ah));
        tm.end(DFS_T_B64DEC, s);
        // The SHA launch waits for group 0 by stream order and for groups
        // 1.. in-kernel.  Launched after the decode it waits on, and sized to
        // leave room for the decode waves, so the decode always progresses.
        HIPC(hipStreamWaitEvent(c->aux, c->pass_ev[0], 0));
        tm.begin(DFS_T_SHA, c->aux);
        const dfs::ShaWait wt{d_queue + dfs::kShaWaitSlot, ah.grid + c->wait_never, 1u, nfrag, static_cast<uint32_t>(nf),
                                c->wait_ticks};
        HIPC(dfs::launch_sha256(d_out, d_desc, t.nlanes[0], nout, t.prio[0], d_dig, d_dig, d_queue, c->ovl_sha_wps,
                                c->aux, nullptr, nullptr, &wt));
        tm.end(DFS_T_SHA, c->aux);
        HIPC(hipEventRecord(c->join, c->aux));
        HIPC(hipStreamWaitEvent(s, c->join, 0));
    } else if (!pipe) {
        tm.begin(DFS_T_B64DEC, s);
        HIPC(dfs::launch_b64_decode(d_in, d_jobs, static_cast<uint32_t>(t.njobs), t.tiles[0], d_out, d_st, nullptr,
                                    s));
        tm.end(DFS_T_B64DEC, s);
        tm.begin(DFS_T_SHA, s);
        HIPC(dfs::launch_sha256(d_out, d_desc, t.nlanes[0], nout, t.prio[0], d_dig, d_dig, d_queue, c->sha_wps, s));
        tm.end(DFS_T_SHA, s);
    } else {
        uint32_t* d_state = D.state;  // running fileId states
        if (!c->aux) HIPC(hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking));
        while (c->pass_ev.size() < npass) {
            hipEvent_t ev = nullptr;
            HIPC(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            c->pass_ev.push_back(ev);
        }
        tm.begin(DFS_T_B64DEC, s);
        for (uint32_t p = 0; p < npass; ++p) {
            HIPC(dfs::launch_b64_decode(d_in, d_jobs + t.job0[p], static_cast<uint32_t>(t.job0[p + 1] - t.job0[p]),
                                        t.tiles[p], d_out, d_st, nullptr, s, c->dec_prio, p ? c->dec_wgs : 8u));
            HIPC(hipEventRecord(c->pass_ev[p], s));
        }
        tm.end(DFS_T_B64DEC, s);
        for (uint32_t p = 0; p < npass; ++p) {
            HIPC(hipStreamWaitEvent(c->aux, c->pass_ev[p], 0));
            if (p == 0) tm.begin(DFS_T_SHA, c->aux);
            HIPC(dfs::launch_sha256(d_out, d_desc + t.desc0[p], t.nlanes[p], nout, t.prio[p], d_dig, d_dig, d_queue,
                                    c->sha_wps_beside, c->aux, d_state));
        }
        tm.end(DFS_T_SHA, c->aux);
        HIPC(hipEventRecord(c->join, c->aux));
        HIPC(hipStreamWaitEvent(s, c->join, 0));
    }
    tm.end(DFS_T_TOTAL, s);
    // Expected digests already on the device (or none): the verdict is
    // computed there and only one status word per file comes back.
    const bool dev_verdict = dev && (!exp_frag || is_device_ptr(exp_frag)) && (!exp_file || is_device_ptr(exp_file));
    std::vector<int32_t> st(dev_verdict ? nfiles : nf);
    std::vector<uint8_t> dig(dev_verdict ? 0 : 32ull * (nf + nfiles));
    auto fetch = [&]() -> int {
        if (dev_verdict) {
            HIPC(dfs::launch_download_verdict(d_st, d_dig, d_dig + 32ull * nf, exp_frag, exp_file, nfiles, nfrag,
                                              D.verdict, s));
            HIPC(dfs::d2h(c, st.data(), D.verdict, 4ull * nfiles, s));
        } else {
            HIPC(dfs::d2h(c, st.data(), D.st, 4ull * nf, s));
            HIPC(dfs::d2h(c, dig.data(), d_dig, dig.size(), s));
        }
        return DFS_OK;
    };
    uint32_t timed_out = 0;
    if (ovl) HIPC(dfs::d2h(c, &timed_out, d_queue + 2, 4, s));
    if (int e = fetch()) return e;
    if (!dev && t.out_end) HIPC(dfs::d2h(c, host_out, d_out, t.out_end, s));
    HIPC(dfs::quiet_sync(c, s));
    if (timed_out) {  // a decode-ahead wait gave up: hash again now that the decode is complete
        ++c->ovl_redo;
        HIPC(dfs::launch_sha256(d_out, d_desc, t.nlanes[0], nout, t.prio[0], d_dig, d_dig, d_queue, c->sha_wps, s));
        if (int e = fetch()) return e;
        HIPC(dfs::quiet_sync(c, s));
    }
    if (dev_verdict) {
        int rc = DFS_OK;
        for (uint32_t f = 0; f < nfiles; ++f) {
            if (status[f] == DFS_OK && st[f])
                status[f] = st[f] == 1 ? DFS_E_DECODE : (st[f] == 2 ? DFS_E_FRAG_MISMATCH : DFS_E_CORRUPT);
            if (status[f] != DFS_OK && rc == DFS_OK) rc = status[f];
        }
        return rc;
    }
    std::vector<uint8_t> expf, expd;
    if (dev && exp_frag && is_device_ptr(exp_frag)) {  // expected digests may live on the device in device mode
        expf.resize(32ull * nf);
        HIPC(hipMemcpy(expf.data(), exp_frag, expf.size(), hipMemcpyDeviceToHost));
        exp_frag = expf.data();
    }
    if (dev && exp_file && is_device_ptr(exp_file)) {
        expd.resize(32ull * nfiles);
        HIPC(hipMemcpy(expd.data(), exp_file, expd.size(), hipMemcpyDeviceToHost));
        exp_file = expd.data();
    }
    int rc = DFS_OK;
    for (uint32_t f = 0; f < nfiles; ++f) {
        if (status[f] == DFS_OK) {
            for (uint32_t i = 0; i < nfrag && status[f] == DFS_OK; ++i)
                if (st[static_cast<uint64_t>(f) * nfrag + i]) status[f] = DFS_E_DECODE;  // SN:281 IAE
            for (uint32_t i = 0; i < nfrag && status[f] == DFS_OK && exp_frag; ++i) {
                const uint64_t k = static_cast<uint64_t>(f) * nfrag + i;
                if (std::memcmp(dig.data() + 32 * k, exp_frag + 32 * k, 32) != 0)
                    status[f] = DFS_E_FRAG_MISMATCH;  // SN:250-257
            }
            if (status[f] == DFS_OK && exp_file &&
                std::memcmp(dig.data() + 32 * (nf + f), exp_file + 32ull * f, 32) != 0)
                status[f] = DFS_E_CORRUPT;  // SN:454-458
        }
        if (status[f] != DFS_OK && rc == DFS_OK) rc = status[f];
    }
    return rc;
}

}  // namespace

extern "C" {

int dfs_download_batch(dfs_ctx* c, const char* b64, const dfs_span* msgs, uint32_t nfiles, uint32_t nfrag,
                       const uint64_t* file_len, const uint8_t* exp_frag, const uint8_t* exp_file, uint8_t* out,
                       const uint64_t* file_off, int32_t* status, uint32_t flags) {
    if (!c || !nfrag || (nfiles && (!msgs || !file_len || !out || !file_off || !status))) return DFS_E_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    if (int rc = enter(c)) return rc;
    Timer tm(c);
    if (!nfiles) return DFS_OK;
    const bool dev = flags & DFS_DEVICE_PTRS;
    hipStream_t s = c->stream();
    Scratch scratch(c, s);
    // Host-mode output lands in ctx scratch, whose address the tiling needs:
    // size it first (a download's output never exceeds the sum of its files).
    uint64_t out_end = 0;
    for (uint32_t f = 0; f < nfiles; ++f) out_end = std::max(out_end, file_off[f] + file_len[f]);
    uint8_t* d_out = out;
    if (!dev) {
        HIPC(c->buf[B_DATA_OUT].ensure(out_end));
        d_out = c->buf[B_DATA_OUT].as<uint8_t>();
    }
    DlTables t;
    if (int rc = build_dl_tables(c, msgs, nfiles, nfrag, file_len, file_off, reinterpret_cast<uintptr_t>(d_out), t))
        return rc;
    std::memcpy(status, t.status0.data(), 4ull * nfiles);
    if ((t.in_end && !b64) || (t.out_end && !out)) return DFS_E_ARG;
    const char* d_in = b64;
    if (!dev) {
        if (int rc = put(c, B_DATA_IN, b64, t.in_end, s)) return rc;
        d_in = c->buf[B_DATA_IN].as<char>();
    }
    if (int rc = put(c, B_JOBS, t.jobs.data(), t.jobs.size() * sizeof(StreamJob), s)) return rc;
    if (int rc = put(c, B_DESC, t.sha.data(), t.sha.size() * sizeof(ShaDesc), s)) return rc;
    if (t.ovl)
        if (int rc = put(c, B_JOBS2, t.gtile.data(), t.gtile.size() * sizeof(uint64_t), s)) return rc;
    HIPC(c->buf[B_STATUS].ensure(4ull * t.nf));
    HIPC(c->buf[B_OUTLEN].ensure(4ull * nfiles));  // per-file verdicts (device-resident expected digests)
    HIPC(c->buf[B_DIG0].ensure(32ull * (t.nf + nfiles)));
    HIPC(c->buf[B_QUEUE].ensure(dfs::kShaQueueBytes));
    if (t.pipe) HIPC(c->buf[B_DIG1].ensure(32ull * t.nout));
    DlDev D;
    D.jobs = c->buf[B_JOBS].as<StreamJob>();
    D.desc = c->buf[B_DESC].as<ShaDesc>();
    D.gtile = c->buf[B_JOBS2].as<uint64_t>();
    D.st = c->buf[B_STATUS].as<int32_t>();
    D.verdict = c->buf[B_OUTLEN].as<int32_t>();
    D.dig = c->buf[B_DIG0].as<uint8_t>();
    D.queue = c->buf[B_QUEUE].as<uint32_t>();
    D.state = c->buf[B_DIG1].as<uint32_t>();
    return run_dl(c, t, D, d_in, d_out, exp_frag, exp_file, dev, out, status, s, tm);
}

// Prepared download: the descriptor tables of one batch shape (spans, file
// lengths and offsets, N) built once and kept in HBM; run many times on
// device buffers.  The mode (overlap / pipelined / serial) is the ctx's at
// creation.
int dfs_download_plan_create(dfs_ctx* c, const dfs_span* msgs, uint32_t nfiles, uint32_t nfrag,
                             const uint64_t* file_len, const uint64_t* file_off, dfs_download_plan** out) {
    if (!c || !out || !nfrag || !nfiles || !msgs || !file_len || !file_off) return DFS_E_ARG;
    *out = nullptr;
    auto* p = new (std::nothrow) dfs_download_plan;
    if (!p) return DFS_E_NOMEM;
    p->device = c->device;
    int rc = build_dl_tables(c, msgs, nfiles, nfrag, file_len, file_off, 0, p->t);  // for a 16-byte aligned output
    std::lock_guard<std::mutex> lk(c->mu);
    if (!rc) rc = enter(c);
    if (!rc) {
        const DlTables& t = p->t;
        const size_t sizes[8] = {std::max<size_t>(t.jobs.size(), 1) * sizeof(StreamJob),
                                 std::max<size_t>(t.sha.size(), 1) * sizeof(ShaDesc),
                                 std::max<size_t>(t.gtile.size(), 1) * sizeof(uint64_t),
                                 std::max<uint64_t>(t.nf, 1) * 4,
                                 static_cast<size_t>(nfiles) * 4,
                                 32ull * (t.nf + nfiles),
                                 dfs::kShaQueueBytes,
                                 t.pipe ? 32ull * t.nout : 256};
        hipError_t e = hipSuccess;
        for (int i = 0; i < 8 && e == hipSuccess; ++i) e = hipMalloc(&p->mem[i], sizes[i]);
        if (e == hipSuccess && !t.jobs.empty())
            e = hipMemcpy(p->mem[0], t.jobs.data(), t.jobs.size() * sizeof(StreamJob), hipMemcpyHostToDevice);
        if (e == hipSuccess && !t.sha.empty())
            e = hipMemcpy(p->mem[1], t.sha.data(), t.sha.size() * sizeof(ShaDesc), hipMemcpyHostToDevice);
        if (e == hipSuccess && !t.gtile.empty())
            e = hipMemcpy(p->mem[2], t.gtile.data(), t.gtile.size() * sizeof(uint64_t), hipMemcpyHostToDevice);
        if (e != hipSuccess) rc = hip_fail(e, "dfs_download_plan_create");
        p->d.jobs = static_cast<const StreamJob*>(p->mem[0]);
        p->d.desc = static_cast<const ShaDesc*>(p->mem[1]);
        p->d.gtile = static_cast<const uint64_t*>(p->mem[2]);
        p->d.st = static_cast<int32_t*>(p->mem[3]);
        p->d.verdict = static_cast<int32_t*>(p->mem[4]);
        p->d.dig = static_cast<uint8_t*>(p->mem[5]);
        p->d.queue = static_cast<uint32_t*>(p->mem[6]);
        p->d.state = static_cast<uint32_t*>(p->mem[7]);
    }
    if (rc) {
        dfs_download_plan_destroy(p);
        return rc;
    }
    // the host copies of the big tables are not needed again
    std::vector<ShaDesc>().swap(p->t.sha);
    std::vector<StreamJob>().swap(p->t.jobs);
    *out = p;
    return DFS_OK;
}

int dfs_download_plan_destroy(dfs_download_plan* p) {
    if (!p) return DFS_E_ARG;
    (void)hipSetDevice(p->device);
    for (void* m : p->mem)
        if (m) (void)hipFree(m);
    delete p;
    return DFS_OK;
}

int dfs_download_plan_run(dfs_ctx* c, dfs_download_plan* p, const char* d_b64, const uint8_t* exp_frag,
                          const uint8_t* exp_file, uint8_t* d_out, int32_t* status) {
    if (!c || !p || p->device != c->device || !status || !d_out) return DFS_E_ARG;
    if ((reinterpret_cast<uintptr_t>(d_out) & 15u) != p->t.out_align || (p->t.in_end && !d_b64)) return DFS_E_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    if (int rc = enter(c)) return rc;
    Timer tm(c);
    hipStream_t s = c->stream();
    Scratch scratch(c, s);
    std::memcpy(status, p->t.status0.data(), 4ull * p->t.nfiles);
    return run_dl(c, p->t, p->d, d_b64, d_out, exp_frag, exp_file, true, nullptr, status, s, tm);
}

// ---------------------------------------------------------------------------
int dfs_synth_fill(dfs_ctx* c, uint8_t* d_dst, const dfs_span* files, uint32_t nfiles, uint64_t first, uint64_t seed) {
    return dfs_synth_fill_at(c, d_dst, files, nfiles, first, seed, 0);
}

int dfs_synth_fill_at(dfs_ctx* c, uint8_t* d_dst, const dfs_span* files, uint32_t nfiles, uint64_t first,
                      uint64_t seed, uint64_t file_off) {
    if (!c || (nfiles && (!files || !d_dst)) || (file_off & 7u)) return DFS_E_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    if (int rc = enter(c)) return rc;
    if (!nfiles) return DFS_OK;
    hipStream_t s = c->stream();
    Scratch scratch(c, s);
    std::vector<StreamJob> jobs;
    std::vector<uint64_t> items;
    for (uint32_t f = 0; f < nfiles; ++f) {
        if (!files[f].len) continue;
        StreamJob j{};
        j.src_off = first + f;
        j.len = files[f].len;
        j.dst_off = files[f].off;
        jobs.push_back(j);
        items.push_back((files[f].len + 63) / 64);
    }
    const uint32_t njobs = static_cast<uint32_t>(jobs.size());
    const uint64_t ntiles = finish_jobs(jobs, items, dfs::kStreamBlock);
    if (int rc = put(c, B_JOBS2, jobs.data(), jobs.size() * sizeof(StreamJob), s)) return rc;
    HIPC(dfs::launch_synth(d_dst, c->buf[B_JOBS2].as<StreamJob>(), njobs, ntiles, seed, s, file_off));
    HIPC(dfs::quiet_sync(c, s));  // the job table lives in reusable scratch
    return DFS_OK;
}


// ---------------------------------------------------------------------------
// storeFragments wire codec, sender side: sendFragmentsToPeers (SN:195-205)
// + buildFragmentsJson (SN:629-642) for a whole batch on the device.
uint64_t dfs_store_body_len(uint64_t file_len, uint32_t nfrag, uint32_t a, uint32_t b) {
    if (!nfrag || a >= nfrag || b >= nfrag) return 0;
    std::vector<uint64_t> off(nfrag), len(nfrag);
    split(file_len, nfrag, off.data(), len.data());
    return dfs::kBodyFrameBytes + enc_len(len[a]) + enc_len(len[b]);
}

int dfs_store_bodies_build(dfs_ctx* c, const uint8_t* files, const dfs_span* file_spans, uint32_t nfiles,
                           uint32_t nfrag, uint32_t uploader, const uint8_t* file_digest, char* bodies,
                           uint64_t* body_off, uint32_t flags) {
    if (!c || !body_off || nfrag < 2 || nfrag > 10 || uploader >= nfrag || (nfiles && !file_spans))
        return DFS_E_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    if (int rc = enter(c)) return rc;
    Timer tm(c);
    const bool dev = flags & DFS_DEVICE_PTRS;
    const uint32_t peers = nfrag - 1;
    std::vector<dfs::StoreBody> desc;
    std::vector<StreamJob> jobs;
    std::vector<uint64_t> items, off(nfrag), len(nfrag);
    desc.reserve(static_cast<size_t>(nfiles) * peers);
    uint64_t total = 0, end = 0;
    for (uint32_t f = 0; f < nfiles; ++f) {
        split(file_spans[f].len, nfrag, off.data(), len.data());  // SN:138-157
        end = std::max(end, file_spans[f].off + file_spans[f].len);
        for (uint32_t k = 0, j = 0; k < nfrag; ++k) {
            if (k == uploader) continue;  // SN:197
            const uint32_t a = k, b = (k + 1) % nfrag;  // SN:199-200
            dfs::StoreBody B{};
            B.dst = total + dfs::kBodyStartPhase;
            B.len_a = enc_len(len[a]);
            B.len_b = enc_len(len[b]);
            B.file = f;
            B.a = static_cast<uint16_t>(a);
            B.b = static_cast<uint16_t>(b);
            desc.push_back(B);
            const uint64_t dst2[2] = {B.dst + dfs::kBodyDataA, B.dst + dfs::kBodyDataA + dfs::kBodyMidBytes + B.len_a};
            const uint32_t fr[2] = {a, b};
            for (int q = 0; q < 2; ++q) {
                if (!len[fr[q]]) continue;
                StreamJob jb{};
                jb.src_off = file_spans[f].off + off[fr[q]];
                jb.len = len[fr[q]];
                jb.dst_off = dst2[q];
                jb.id = static_cast<uint32_t>(jobs.size());
                jobs.push_back(jb);
                items.push_back((len[fr[q]] + 11) / 12);
            }
            body_off[static_cast<uint64_t>(f) * peers + j++] = B.dst;
            total += (dfs::kBodyStartPhase + dfs::kBodyFrameBytes + B.len_a + B.len_b + 15) & ~15ull;
        }
    }
    body_off[static_cast<uint64_t>(nfiles) * peers] = total;
    if (!bodies) return DFS_OK;  // layout query
    if (!nfiles) return DFS_OK;
    if ((end && !files) || !file_digest) return DFS_E_ARG;
    hipStream_t s = c->stream();
    Scratch scratch(c, s);
    const uint8_t* d_files = files;
    const uint8_t* d_dig = file_digest;
    char* d_out = bodies;
    if (!dev) {
        if (int rc = put(c, B_DATA_IN, files, end, s)) return rc;
        d_files = c->buf[B_DATA_IN].as<uint8_t>();
        if (int rc = put(c, B_DIG0, file_digest, 32ull * nfiles, s)) return rc;
        d_dig = c->buf[B_DIG0].as<uint8_t>();
        HIPC(c->buf[B_DATA_OUT].ensure(total));
        d_out = c->buf[B_DATA_OUT].as<char>();
    } else if (reinterpret_cast<uintptr_t>(bodies) & 15u) {
        return DFS_E_ARG;
    }
    const uint32_t njobs = static_cast<uint32_t>(jobs.size());
    const uint64_t ntiles = finish_jobs(jobs, items, static_cast<uint64_t>(dfs::kEncPer) * dfs::kStreamBlock);
    if (int rc = put(c, B_JOBS, jobs.data(), jobs.size() * sizeof(StreamJob), s)) return rc;
    if (int rc = put(c, B_DESC, desc.data(), desc.size() * sizeof(dfs::StoreBody), s)) return rc;
    tm.begin(DFS_T_TOTAL, s);
    HIPC(dfs::launch_store_body_frame(c->buf[B_DESC].as<dfs::StoreBody>(), static_cast<uint32_t>(desc.size()), d_dig,
                                      d_out, s));
    tm.begin(DFS_T_B64ENC, s);
    HIPC(dfs::launch_b64_encode(d_files, c->buf[B_JOBS].as<StreamJob>(), njobs, ntiles, d_out, 8u, s, 0u));
    tm.end(DFS_T_B64ENC, s);
    tm.end(DFS_T_TOTAL, s);
    if (!dev) {
        HIPC(dfs::d2h(c, bodies, d_out, total, s));
        HIPC(dfs::quiet_sync(c, s));
    }
    return DFS_OK;
}

// storeFragments wire codec, receiver side: handleInternalStoreFragments
// (SN:265-293) for bodies in buildFragmentsJson form.
int dfs_store_bodies_receive(dfs_ctx* c, const char* bodies, const dfs_span* body_spans, uint32_t n, uint8_t* out,
                             uint64_t* out_off, uint32_t* frag_index, uint64_t* frag_off, uint64_t* frag_len,
                             uint8_t* digests, char* file_ids, int32_t* status, uint32_t flags) {
    if (!c || !out_off ||
        (n && (!body_spans || !frag_index || !frag_off || !frag_len || !digests || !file_ids || !status)))
        return DFS_E_ARG;
    const bool dev = flags & DFS_DEVICE_PTRS;
    uint64_t end = 0, total = 0;
    for (uint32_t i = 0; i < n; ++i) {
        out_off[i] = total;
        // >= both decoded payloads, the second one's start and the next slot's rounded up to 16 bytes
        total += (3 * ((body_spans[i].len + 3) / 4) + 16 + 15) & ~15ull;
        end = std::max(end, body_spans[i].off + body_spans[i].len);
    }
    out_off[n] = total;
    if (!n) return DFS_OK;
    if ((end && !bodies) || (total && !out)) return DFS_E_ARG;
    std::vector<dfs::BodyParse> parsed(n);
    {
        std::lock_guard<std::mutex> lk(c->mu);
        if (int rc = enter(c)) return rc;
        hipStream_t s = c->stream();
        Scratch scratch(c, s);
        const char* d_in = bodies;
        if (!dev) {
            if (int rc = put(c, B_DATA_IN, bodies, end, s)) return rc;
            d_in = c->buf[B_DATA_IN].as<char>();
        }
        if (int rc = put(c, B_JOBS, body_spans, sizeof(dfs_span) * n, s)) return rc;
        HIPC(c->buf[B_DESC].ensure(sizeof(dfs::BodyParse) * n));
        HIPC(c->buf[B_DIG1].ensure(64ull * n));
        HIPC(dfs::launch_store_body_parse(d_in, c->buf[B_JOBS].as<uint64_t>(), n, c->buf[B_DESC].as<dfs::BodyParse>(),
                                          c->buf[B_DIG1].as<char>(), s));
        HIPC(dfs::d2h(c, parsed.data(), c->buf[B_DESC].p, sizeof(dfs::BodyParse) * n, s));
        HIPC(dfs::d2h(c, file_ids, c->buf[B_DIG1].p, 64ull * n, s));
        HIPC(dfs::quiet_sync(c, s));
    }
    // Decode each payload into the body's output slot and hash it (SN:280-282).
    std::vector<dfs_span> msgs;
    std::vector<uint64_t> dst, len;
    std::vector<int32_t> st;
    std::vector<uint32_t> who;
    for (uint32_t i = 0; i < n; ++i) {
        status[i] = parsed[i].status ? DFS_E_WIRE : DFS_OK;
        frag_len[2 * i] = frag_len[2 * i + 1] = 0;
        frag_off[2 * i] = frag_off[2 * i + 1] = out_off[i];
        if (parsed[i].status) {
            frag_index[2 * i] = frag_index[2 * i + 1] = UINT32_MAX;
            continue;
        }
        const dfs::BodyParse& p = parsed[i];
        frag_index[2 * i] = p.a;
        frag_index[2 * i + 1] = p.b;
        msgs.push_back(dfs_span{body_spans[i].off + p.off_a, p.len_a});
        dst.push_back(out_off[i]);
        msgs.push_back(dfs_span{body_spans[i].off + p.off_b, p.len_b});
        dst.push_back((out_off[i] + dfs_b64_decoded_cap(p.len_a) + 15) & ~15ull);
        frag_off[2 * i + 1] = dst.back();
        who.push_back(i);
    }
    if (msgs.empty()) return DFS_OK;
    len.resize(msgs.size());
    st.resize(msgs.size());
    std::vector<uint8_t> dig(32 * msgs.size());
    int rc = dfs_receive_fragments_batch(c, bodies, msgs.data(), static_cast<uint32_t>(msgs.size()), out, dst.data(),
                                         len.data(), dig.data(), st.data(), flags);
    if (rc != DFS_OK && rc != DFS_E_DECODE) return rc;
    for (size_t k = 0; k < who.size(); ++k) {
        const uint32_t i = who[k];
        for (int q = 0; q < 2; ++q) {
            frag_len[2 * i + q] = len[2 * k + q];
            std::memcpy(digests + 64ull * i + 32 * q, dig.data() + 64 * k + 32 * q, 32);
            if (st[2 * k + q] != DFS_OK) status[i] = DFS_E_DECODE;  // SN:281 IllegalArgumentException
        }
    }
    return DFS_OK;
}

}  // extern "C"
