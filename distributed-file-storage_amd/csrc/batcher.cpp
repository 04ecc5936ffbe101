// batcher.cpp — request batcher in front of the fragment pipeline
// (include/dfs_gpu.h, dfs_batcher_* / dfs_submit_*).
//
// Reference: StorageNode runs one thread per connection (StorageNode.java
// :28-31) and every handler processes one file: handleUpload (:118-189) and
// handleDownload (:399-461).  A GPU launch per file would be floored by that
// file's fileId chain and leave the chip almost empty, so concurrent handler
// calls are coalesced: a handler thread submits its one file and blocks; a
// worker takes every request queued within a short window (or until a batch
// is full) and runs them as one launch.
//
// Workers: `depth` threads, each with its own dfs_ctx (stream + scratch),
// pinned host staging and device buffers, so batch k+1's copies and launch
// overlap batch k's kernels.  The handler threads copy their own bytes into
// and out of the pinned staging, so those copies run in parallel instead of
// on the worker.  Host-resident data crosses PCIe twice (file in, Base64
// out for uploads; Base64 in, file out for downloads): that, not the
// kernels, bounds a host-buffer caller at high concurrency (an upload is
// capped near 42 GB/s of file bytes on a 56 GB/s link).
//
// A request's output goes back one of three ways: copied by its handler out
// of the batch's pinned result buffer (pageable callers), written by a DMA
// of its own into its pinned buffer (direct), or left in the result buffer
// and handed out as a pointer (dfs_submit_*_view: one DMA per batch, no host
// copy; the buffer is reused only after every view of it was released).
//
// Hand-off per request:
//   0 queued -> 1 worker assigned its staging slot (in_dst) -> 2 handler
//   copied its input in (BatchSync::copied_in) -> 3 results ready (out_src,
//   status) -> 4 handler copied its output out (BatchSync::copied_out); the
//   worker reuses the staging only after every request of its batch did.
// Locks: the batcher mutex guards only the queue and the stats (held for a
// few instructions); a request's phase has its own mutex, shared by its
// handler and the worker alone; a batch's counters have the BatchSync's.
// Whoever publishes a phase notifies while holding that lock, so the other
// side cannot see the phase, finish and free the object first.
#include <hip/hip_runtime.h>
#include <pthread.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <shared_mutex>
#include <thread>
#include <vector>

#include "../../include/dfs_gpu.h"
#include "dfs_internal.h"

namespace {

using Clock = std::chrono::steady_clock;

uint64_t enc_len(uint64_t n) { return 4 * ((n + 2) / 3); }
constexpr uint64_t kMaxFile = 1ull << 37;  // the SHA lanes count 64-byte blocks in 32 bits

// dfs_host_alloc buffers (base -> bytes, device-mapped base): a request is
// direct only if each of its buffers lies inside one of them, so the copy
// kernel never touches pageable memory.
struct Pinned {
    uint64_t bytes;
    uintptr_t dev;  // hipHostGetDevicePointer of the base
};
std::shared_mutex g_pin_mu;
std::map<uintptr_t, Pinned> g_pinned;

// Device-visible address of host bytes [p, p+n) if they lie in one
// dfs_host_alloc buffer, else 0 (n == 0: 1, nothing to move).
uint64_t pinned_dev(const void* p, uint64_t n) {
    if (!n) return 1;
    if (!p) return 0;
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    std::shared_lock<std::shared_mutex> lk(g_pin_mu);
    auto it = g_pinned.upper_bound(a);
    if (it == g_pinned.begin()) return 0;
    --it;
    const uint64_t o = a - it->first;
    return o <= it->second.bytes && n <= it->second.bytes - o ? it->second.dev + o : 0;
}
bool in_pinned(const void* p, uint64_t n) { return pinned_dev(p, n) != 0; }


struct Req;

// Lives on the worker's stack for one batch.  Handlers only touch it (under
// its mutex) before their submit returns; the worker leaves the batch only
// after `copied_out` reached the batch size, so it outlives every use.
// Requests themselves live on the handlers' stacks: the worker never reads
// a request once its handler may have returned.
struct BatchSync {
    std::mutex mu;
    std::condition_variable cv;  // a handler advanced its request
    size_t copied_in = 0, copied_out = 0;
    double return_s = 0;         // handlers' results-ready -> return time
};

// download kinds: 1 + (exp_frag ? 2 : 0) + (exp_file ? 1 : 0); raw-fragment download: kReassemble
enum Kind { kUpload = 0, kDownload = 1, kReassemble = 8 };

struct Req {
    int kind = kUpload;
    uint64_t len = 0;        // file bytes
    uint64_t need = 0;       // input bytes staged (upload: len; download: Base64 chars)
    uint64_t out_bytes = 0;  // output bytes copied back (upload: Base64; download: len)
    // upload
    const uint8_t* file = nullptr;
    uint8_t* fd = nullptr;
    uint8_t* frd = nullptr;
    char* b64 = nullptr;
    uint64_t* b64_off = nullptr;
    // download
    const char* text = nullptr;
    const dfs_span* frags = nullptr;
    const uint8_t* exp_frag = nullptr;
    const uint8_t* exp_file = nullptr;
    uint8_t* out = nullptr;
    // raw-fragment download (handleDownload as the reference has it)
    const uint8_t* const* raw = nullptr;  // the fragments, in index order
    const uint64_t* raw_len = nullptr;
    uint8_t* digest_out = nullptr;
    // hand-off
    Clock::time_point arrive;
    int phase = 0;
    BatchSync* sync = nullptr;
    uint8_t* in_dst = nullptr;         // staging slot of the input
    const uint8_t* out_src = nullptr;  // staging of the output
    int status = DFS_OK;
    bool direct = false;  // input (and, unless a view is asked for, output) in dfs_host_alloc buffers: DMA'd, no staging
    // output as a view of the batch's result buffer (dfs_submit_*_view)
    bool want_view = false;
    const void** view_ptr = nullptr;
    dfs_view** view_handle = nullptr;
    dfs_view* view = nullptr;  // set by the worker when the batch succeeded (one reference is this request's)
    std::mutex mu;  // guards phase (and the fields the phase publishes)
    std::condition_variable cv;
};

// Publish phase `p` of request r (the worker side).
void publish(Req* r, int p) {
    std::lock_guard<std::mutex> lk(r->mu);
    r->phase = p;
    r->cv.notify_one();
}

struct Buf {
    void* p = nullptr;
    size_t cap = 0;
    bool pinned = false;
    int grow(size_t n) {
        if (n <= cap) return DFS_OK;
        // doubling from 64 MiB: a pinned allocation and the free of the old
        // one are expensive (page pinning; frees synchronise the device)
        size_t want = std::max<size_t>(cap, size_t(64) << 20);
        while (want < n) want *= 2;
        void* q = nullptr;
        if ((pinned ? hipHostMalloc(&q, want, hipHostMallocDefault) : hipMalloc(&q, want)) != hipSuccess)
            return DFS_E_NOMEM;
        release();
        p = q;
        cap = want;
        return DFS_OK;
    }
    void release() {
        if (p) (void)(pinned ? hipHostFree(p) : hipFree(p));
        p = nullptr;
        cap = 0;
    }
    template <class T> T* as() const { return static_cast<T*>(p); }
};

}  // namespace

// A batch's results in pinned memory.  `refs` counts the views handed out of
// it; the worker that owns it takes it for a new batch only at zero.
struct dfs_view {
    std::mutex mu;
    std::condition_variable cv;
    int refs = 0;
    Buf pin;
    dfs_view() { pin.pinned = true; }
};

namespace {

struct Worker {
    dfs_ctx* ctx = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;  // polled with sleeps (dfs::quiet_wait): the worker does not spin on the CPU share
    Buf pin_in, d_in, d_out, d_dig;
    // Result buffers, taken in turn: batch k's views may outlive batch k + 1.
    // Two in the steady state.  Handlers that keep views while they wait for
    // a later request of their own could otherwise stop the worker for good
    // (it would wait for their views, they for its next batch), so a buffer
    // that stays referenced for kViewPatience makes the worker add another,
    // up to kMaxOuts; only there does it wait without a limit.
    static constexpr size_t kMaxOuts = 8;
    static constexpr std::chrono::milliseconds kViewPatience{20};
    std::vector<std::unique_ptr<dfs_view>> outs;
    size_t out_i = 0;
    std::thread th;
    Worker() {
        pin_in.pinned = true;
        for (int i = 0; i < 2; ++i) outs.emplace_back(new dfs_view);
    }
    // The result buffer of the next batch: one without views.
    dfs_view* next_out() {
        for (size_t k = 1; k <= outs.size(); ++k) {
            dfs_view* v = outs[(out_i + k) % outs.size()].get();
            std::lock_guard<std::mutex> lk(v->mu);
            if (v->refs == 0) {
                out_i = (out_i + k) % outs.size();
                return v;
            }
        }
        dfs_view* v = outs[out_i = (out_i + 1) % outs.size()].get();  // the oldest
        std::unique_lock<std::mutex> lk(v->mu);
        if (outs.size() >= kMaxOuts) {
            v->cv.wait(lk, [&] { return v->refs == 0; });
            return v;
        }
        if (v->cv.wait_for(lk, kViewPatience, [&] { return v->refs == 0; })) return v;
        lk.unlock();
        outs.emplace_back(new dfs_view);
        out_i = outs.size() - 1;
        return outs.back().get();
    }
};

}  // namespace

struct dfs_batcher {
    int device = 0;
    uint32_t nfrag = 5;
    dfs_batcher_opts o{};
    std::mutex mu;
    std::condition_variable cv_work;
    std::deque<Req*> q;
    uint64_t q_bytes = 0;
    bool stop = false;
    std::vector<Worker*> workers;
    dfs_batcher_stats_t st{};
    bool dl_in_kernel = true;  // direct downloads: Base64 in by one copy kernel (else one DMA per request); DFS_BATCH_DL_IN=dma
};

namespace {

// Direct requests' bytes: one DMA per request and direction, except a
// download's Base64 into HBM, which one copy kernel reads from the handlers'
// pinned buffers (dfs::copy_spans).  Measured at 4,096 clients
// (profiles/r02c_batcher/copy_modes.txt): uploads 26.8 GB/s with DMA both
// ways, 18.8-20.9 with the kernel for either direction (its launch competes
// with the other workers' kernels); downloads 16.5 with DMA, 17.7-18.9 with
// the kernel reading the Base64 in.
int move_in(Worker& w, const std::vector<dfs::CopySpan>& cp, bool kernel) {
    if (kernel) return dfs::copy_spans(w.ctx, cp.data(), cp.size());
    for (const auto& c : cp)
        if (hipMemcpyAsync(reinterpret_cast<void*>(c.dst), reinterpret_cast<const void*>(c.src), c.len, hipMemcpyDefault,
                           w.stream) != hipSuccess)
            return DFS_E_HIP;
    return DFS_OK;
}
int move_out(Worker& w, const std::vector<dfs::CopySpan>& cp) {
    for (const auto& c : cp)
        if (hipMemcpyAsync(reinterpret_cast<void*>(c.dst), reinterpret_cast<const void*>(c.src), c.len, hipMemcpyDefault,
                           w.stream) != hipSuccess)
            return DFS_E_HIP;
    return DFS_OK;
}

bool wait_stream(Worker& w) {
    // not hipEventSynchronize: it spins a core for the whole batch (dfs::quiet_wait)
    return hipEventRecord(w.done, w.stream) == hipSuccess && dfs::quiet_wait(w.done) == hipSuccess;
}

struct Timing {
    double stage_in = 0, device = 0;
};

double since(Clock::time_point t) { return std::chrono::duration<double>(Clock::now() - t).count(); }

// Give the first `staged` requests their staging slots and wait until they
// copied their input (direct requests have nothing to copy).
void stage_in(dfs_batcher* B, std::vector<Req*>& batch, size_t staged, BatchSync& bs, uint8_t* base,
              const std::vector<uint64_t>& off, Timing& tm) {
    const auto t0 = Clock::now();
    for (size_t i = 0; i < staged; ++i) {
        batch[i]->in_dst = base + off[i];
        publish(batch[i], 1);
    }
    std::unique_lock<std::mutex> lk(bs.mu);
    bs.cv.wait(lk, [&] { return bs.copied_in == staged; });
    tm.stage_in = since(t0);
}

// Order a batch so that the requests whose input is staged form a prefix
// (one DMA in) and so do those whose output leaves through the result buffer
// (staged or view: one DMA out): staged, staged + view, direct + view,
// direct.  Returns the two prefix lengths.
struct Prefix {
    size_t in = 0, out = 0;
};
Prefix order_batch(std::vector<Req*>& batch) {
    auto cls = [](const Req* r) { return r->direct ? (r->want_view ? 2 : 3) : (r->want_view ? 1 : 0); };
    std::stable_sort(batch.begin(), batch.end(), [&](const Req* a, const Req* b) { return cls(a) < cls(b); });
    Prefix p;
    for (const Req* r : batch) {
        p.in += !r->direct;
        p.out += !r->direct || r->want_view;
    }
    return p;
}

// Hand the batch's views out (the batch succeeded): one reference each.
void grant_views(std::vector<Req*>& batch, dfs_view* v) {
    int n = 0;
    for (Req* r : batch)
        if (r->want_view) {
            r->view = v;
            ++n;
        }
    if (n) {
        std::lock_guard<std::mutex> lk(v->mu);
        v->refs += n;
    }
}

int run_uploads(dfs_batcher* B, Worker& w, std::vector<Req*>& batch, BatchSync& bs, Timing& tm) {
    const uint32_t n = static_cast<uint32_t>(batch.size()), N = B->nfrag;
    const Prefix pre = order_batch(batch);
    const size_t staged = pre.in;
    std::vector<dfs_span> spans(n);
    std::vector<uint64_t> in_off(n);
    uint64_t total = 0, b64_total = 0, staged_in = 0, staged_b64 = 0;
    for (uint32_t i = 0; i < n; ++i) {
        in_off[i] = total;
        spans[i] = dfs_span{total, batch[i]->len};
        total += (batch[i]->len + 15) & ~15ull;  // 16-byte aligned file starts
        b64_total += batch[i]->b64_off[N];       // filled at submit: the request's Base64 bytes
        if (i + 1 == pre.in) staged_in = total;
        if (i + 1 == pre.out) staged_b64 = b64_total;
    }
    const uint64_t dig_bytes = 32ull * n * (N + 1);
    dfs_view* res = w.next_out();
    int rc = w.pin_in.grow(staged_in + 16);
    if (!rc) rc = res->pin.grow(dig_bytes + staged_b64 + 16);
    if (!rc) rc = w.d_in.grow(total + 16);
    if (!rc) rc = w.d_out.grow(b64_total + 16);
    if (!rc) rc = w.d_dig.grow(dig_bytes);
    if (rc) return rc;
    stage_in(B, batch, staged, bs, w.pin_in.as<uint8_t>(), in_off, tm);
    const auto t_dev = Clock::now();
    std::vector<uint64_t> b64_off(static_cast<uint64_t>(n) * N + 1);
    uint8_t* d_fd = w.d_dig.as<uint8_t>();
    uint8_t* d_frd = d_fd + 32ull * n;
    if (staged_in && hipMemcpyAsync(w.d_in.p, w.pin_in.p, staged_in, hipMemcpyHostToDevice, w.stream) != hipSuccess)
        return DFS_E_HIP;
    std::vector<dfs::CopySpan> cp;  // direct: read from the handlers' pinned buffers
    for (uint32_t i = static_cast<uint32_t>(staged); i < n; ++i)
        if (batch[i]->len)
            cp.push_back({pinned_dev(batch[i]->file, batch[i]->len),
                          reinterpret_cast<uint64_t>(w.d_in.as<uint8_t>() + in_off[i]), batch[i]->len});
    if (int e = move_in(w, cp, false)) return e;
    // one stream per worker (DFS_SERIAL: the Base64 kernel follows the SHA
    // kernel on it): a box exposes few hardware queues (GPU_MAX_HW_QUEUES=4),
    // and streams sharing one would serialise the workers' batches
    rc = dfs_upload_batch(w.ctx, w.d_in.as<uint8_t>(), spans.data(), n, N, d_fd, d_frd, w.d_out.as<char>(),
                          b64_total, b64_off.data(), DFS_DEVICE_PTRS | DFS_SERIAL);
    if (rc) return rc;
    uint8_t* h = res->pin.as<uint8_t>();
    if (hipMemcpyAsync(h, d_fd, dig_bytes, hipMemcpyDeviceToHost, w.stream) != hipSuccess ||
        (staged_b64 && hipMemcpyAsync(h + dig_bytes, w.d_out.p, staged_b64, hipMemcpyDeviceToHost, w.stream) != hipSuccess))
        return DFS_E_HIP;
    cp.clear();  // direct: into the handlers' pinned buffers
    for (uint32_t i = static_cast<uint32_t>(pre.out); i < n; ++i) {
        const Req* r = batch[i];
        if (r->out_bytes)
            cp.push_back({reinterpret_cast<uint64_t>(w.d_out.as<char>() + b64_off[static_cast<uint64_t>(i) * N]),
                          pinned_dev(r->b64, r->out_bytes), r->out_bytes});
    }
    if (int e = move_out(w, cp)) return e;
    if (!wait_stream(w)) return DFS_E_HIP;
    tm.device = since(t_dev);
    for (uint32_t i = 0; i < n; ++i) {
        Req* r = batch[i];
        std::memcpy(r->fd, h + 32ull * i, 32);
        std::memcpy(r->frd, h + 32ull * n + 32ull * N * i, 32ull * N);
        // its Base64, [fragment] order (direct: already in place)
        r->out_src = i < pre.out ? h + dig_bytes + b64_off[static_cast<uint64_t>(i) * N] : nullptr;
    }
    grant_views(batch, res);
    return DFS_OK;
}

int run_downloads(dfs_batcher* B, Worker& w, std::vector<Req*>& batch, BatchSync& bs, Timing& tm) {
    const uint32_t n = static_cast<uint32_t>(batch.size()), N = B->nfrag;
    const Prefix pre = order_batch(batch);
    const size_t staged = pre.in;
    uint64_t staged_in = 0, staged_out = 0;
    const bool have_f = batch.front()->exp_frag != nullptr, have_i = batch.front()->exp_file != nullptr;
    std::vector<uint64_t> in_off(n), file_len(n), file_off(n);
    std::vector<dfs_span> spans(static_cast<uint64_t>(n) * N);
    std::vector<uint8_t> ef(have_f ? 32ull * n * N : 0), ei(have_i ? 32ull * n : 0);
    uint64_t total = 0, out_total = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const Req* r = batch[i];
        in_off[i] = total;
        uint64_t o = total;  // the handler packs its fragments back to back
        for (uint32_t k = 0; k < N; ++k) {
            const dfs_span& s = r->frags[k];
            dfs_span& d = spans[static_cast<uint64_t>(i) * N + k];
            if (s.len == DFS_SPAN_MISSING) {
                d = s;
            } else {
                d = dfs_span{o, s.len};
                o += s.len;
            }
        }
        total += (r->need + 15) & ~15ull;
        file_len[i] = r->len;
        file_off[i] = out_total;
        out_total += (r->len + 15) & ~15ull;
        if (i + 1 == pre.in) staged_in = total;
        if (i + 1 == pre.out) staged_out = out_total;
        if (have_f) std::memcpy(ef.data() + 32ull * N * i, r->exp_frag, 32ull * N);
        if (have_i) std::memcpy(ei.data() + 32ull * i, r->exp_file, 32);
    }
    dfs_view* res = w.next_out();
    int rc = w.pin_in.grow(staged_in + 16);
    if (!rc) rc = res->pin.grow(staged_out + 16);
    if (!rc) rc = w.d_in.grow(total + 16);
    if (!rc) rc = w.d_out.grow(out_total + 16);
    if (rc) return rc;
    stage_in(B, batch, staged, bs, w.pin_in.as<uint8_t>(), in_off, tm);
    const auto t_dev = Clock::now();
    if (staged_in && hipMemcpyAsync(w.d_in.p, w.pin_in.p, staged_in, hipMemcpyHostToDevice, w.stream) != hipSuccess)
        return DFS_E_HIP;
    std::vector<dfs::CopySpan> cp;  // direct: the fragments' Base64, packed, by one copy kernel
    for (uint32_t i = static_cast<uint32_t>(staged); i < n; ++i) {
        const Req* r = batch[i];
        uint64_t d = reinterpret_cast<uint64_t>(w.d_in.as<uint8_t>() + in_off[i]);
        for (uint32_t k = 0; k < N; ++k) {
            const dfs_span& sp = r->frags[k];
            if (sp.len == DFS_SPAN_MISSING || !sp.len) continue;
            const uint64_t src = pinned_dev(r->text + sp.off, sp.len);
            if (!cp.empty() && cp.back().src + cp.back().len == src && cp.back().dst + cp.back().len == d)
                cp.back().len += sp.len;  // back to back in the handler's buffer
            else
                cp.push_back({src, d, sp.len});
            d += sp.len;
        }
    }
    if (int e = move_in(w, cp, B->dl_in_kernel)) return e;
    std::vector<int32_t> st(n);
    rc = dfs_download_batch(w.ctx, w.d_in.as<char>(), spans.data(), n, N, file_len.data(), have_f ? ef.data() : nullptr,
                            have_i ? ei.data() : nullptr, w.d_out.as<uint8_t>(), file_off.data(), st.data(),
                            DFS_DEVICE_PTRS);
    if (rc != DFS_OK && rc != DFS_E_MISSING && rc != DFS_E_DECODE && rc != DFS_E_FRAG_MISMATCH && rc != DFS_E_CORRUPT)
        return rc;
    if (staged_out && hipMemcpyAsync(res->pin.p, w.d_out.p, staged_out, hipMemcpyDeviceToHost, w.stream) != hipSuccess)
        return DFS_E_HIP;
    cp.clear();  // direct, good files only (as the staged copy-out)
    for (uint32_t i = static_cast<uint32_t>(pre.out); i < n; ++i)
        if (st[i] == DFS_OK && batch[i]->len)
            cp.push_back({reinterpret_cast<uint64_t>(w.d_out.as<uint8_t>() + file_off[i]),
                          pinned_dev(batch[i]->out, batch[i]->len), batch[i]->len});
    if (int e = move_out(w, cp)) return e;
    if (!wait_stream(w)) return DFS_E_HIP;
    tm.device = since(t_dev);
    for (uint32_t i = 0; i < n; ++i) {
        batch[i]->status = st[i];
        batch[i]->out_src = i < pre.out ? res->pin.as<uint8_t>() + file_off[i] : nullptr;
    }
    grant_views(batch, res);
    return DFS_OK;
}

// Raw-fragment downloads (handleDownload as the reference has it, SN:419-458:
// getFragment returns raw bytes, SN:513-514).  The ordered append (SN:448) is
// the handler's copy of its fragments, back to back, into the staging: the
// staged bytes are the rebuilt file.  The device hashes every file of the
// batch (SN:454); the handler compares with its fileId and takes the file
// from the staging.  All requests are staged.
int run_reassembles(dfs_batcher* B, Worker& w, std::vector<Req*>& batch, BatchSync& bs, Timing& tm) {
    (void)B;
    const uint32_t n = static_cast<uint32_t>(batch.size());
    std::vector<dfs_span> spans(n);
    std::vector<uint64_t> in_off(n);
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; ++i) {
        in_off[i] = total;
        spans[i] = dfs_span{total, batch[i]->len};
        total += (batch[i]->len + 15) & ~15ull;
    }
    dfs_view* res = w.next_out();
    int rc = w.pin_in.grow(total + 16);
    if (!rc) rc = res->pin.grow(32ull * n);
    if (!rc) rc = w.d_in.grow(total + 16);
    if (!rc) rc = w.d_dig.grow(32ull * n);
    if (rc) return rc;
    stage_in(B, batch, n, bs, w.pin_in.as<uint8_t>(), in_off, tm);
    const auto t_dev = Clock::now();
    if (total && hipMemcpyAsync(w.d_in.p, w.pin_in.p, total, hipMemcpyHostToDevice, w.stream) != hipSuccess)
        return DFS_E_HIP;
    rc = dfs_sha256_batch(w.ctx, w.d_in.as<uint8_t>(), spans.data(), n, w.d_dig.as<uint8_t>(), DFS_DEVICE_PTRS);
    if (rc) return rc;
    if (hipMemcpyAsync(res->pin.p, w.d_dig.p, 32ull * n, hipMemcpyDeviceToHost, w.stream) != hipSuccess)
        return DFS_E_HIP;
    if (!wait_stream(w)) return DFS_E_HIP;
    tm.device = since(t_dev);
    for (uint32_t i = 0; i < n; ++i) {
        Req* r = batch[i];
        const uint8_t* d = res->pin.as<uint8_t>() + 32ull * i;
        if (r->digest_out) std::memcpy(r->digest_out, d, 32);
        r->status = r->exp_file && std::memcmp(d, r->exp_file, 32) != 0 ? DFS_E_CORRUPT : DFS_OK;  // SN:455-458
        r->out_src = w.pin_in.as<uint8_t>() + in_off[i];  // the rebuilt file, where the handler assembled it
    }
    return DFS_OK;
}

void worker_main(dfs_batcher* B, Worker* w) {
    (void)pthread_setname_np(pthread_self(), "dfs-batch");  // per-thread CPU accounting (tools/batcher_load)
    (void)hipSetDevice(B->device);
    const auto window = std::chrono::microseconds(B->o.max_wait_us);
    for (;;) {
        std::vector<Req*> batch;
        BatchSync bs;
        {
            std::unique_lock<std::mutex> lk(B->mu);
            B->cv_work.wait(lk, [&] { return B->stop || !B->q.empty(); });
            if (B->q.empty()) return;  // stopping and drained
            // the window opens with the oldest request; a full queue goes at once
            while (!B->stop && !B->q.empty() && B->q.size() < B->o.max_files && B->q_bytes < B->o.max_bytes &&
                   Clock::now() < B->q.front()->arrive + window)
                B->cv_work.wait_until(lk, B->q.front()->arrive + window);
            if (B->q.empty()) continue;  // another worker took them
            const int kind = B->q.front()->kind;
            uint64_t bytes = 0;
            for (auto it = B->q.begin(); it != B->q.end() && batch.size() < B->o.max_files;) {
                Req* r = *it;
                if (r->kind != kind || (!batch.empty() && bytes + r->need > B->o.max_bytes)) {
                    ++it;
                    continue;
                }
                r->sync = &bs;
                batch.push_back(r);
                bytes += r->need;
                B->q_bytes -= r->need;
                it = B->q.erase(it);
            }
            const auto now = Clock::now();
            ++B->st.batches;
            B->st.requests += batch.size();
            B->st.max_batch = std::max<uint64_t>(B->st.max_batch, batch.size());
            for (const Req* r : batch) B->st.direct += r->direct, B->st.views += r->want_view;
            for (Req* r : batch) B->st.queue_s += std::chrono::duration<double>(now - r->arrive).count();
            if (!B->q.empty()) B->cv_work.notify_one();
        }
        Timing tm;
        const int kind0 = batch.front()->kind;
        const int rc = kind0 == kUpload ? run_uploads(B, *w, batch, bs, tm)
                       : kind0 == kReassemble ? run_reassembles(B, *w, batch, bs, tm)
                                              : run_downloads(B, *w, batch, bs, tm);
        // A batch that failed part-way may have DMAs or kernels queued on the
        // handlers' pinned buffers and on the staging: let them finish before
        // any handler is told (it may free or reuse its buffers on return).
        if (rc != DFS_OK) (void)wait_stream(*w);
        const auto t_done = Clock::now();
        // Results ready (or the batch failed); reuse the staging only after
        // every handler copied its output out.
        for (Req* r : batch) {
            if (rc != DFS_OK) {
                r->status = rc;
                r->out_src = nullptr;
            }
            publish(r, 3);
        }
        const size_t n = batch.size();
        {
            std::unique_lock<std::mutex> lk(bs.mu);
            bs.cv.wait(lk, [&] { return bs.copied_out == n; });
        }
        std::lock_guard<std::mutex> lk(B->mu);
        B->st.stage_in_s += tm.stage_in;
        B->st.device_s += tm.device;
        B->st.stage_out_s += std::chrono::duration<double>(Clock::now() - t_done).count();
        B->st.return_s += bs.return_s;
    }
}

// The handler side of one request: enqueue, copy the input into the
// staging slot when the worker hands it out, wait for the results, copy the
// output out of the staging.
int submit(dfs_batcher* B, Req& r) {
    const auto t_call = Clock::now();
    {
        std::lock_guard<std::mutex> lk(B->mu);
        if (B->stop) return DFS_E_ARG;
        r.arrive = Clock::now();
        B->st.enqueue_s += std::chrono::duration<double>(r.arrive - t_call).count();
        B->q.push_back(&r);
        B->q_bytes += r.need;
        B->cv_work.notify_one();
    }
    std::unique_lock<std::mutex> lk(r.mu);
    r.cv.wait(lk, [&] { return r.phase >= 1; });
    if (r.phase == 1) {
        lk.unlock();
        if (r.kind == kUpload) {
            if (r.len) std::memcpy(r.in_dst, r.file, r.len);
        } else if (r.kind == kReassemble) {  // full.write(fragData) in index order, SN:448
            uint8_t* d = r.in_dst;
            for (uint32_t k = 0; k < B->nfrag; ++k) {
                if (r.raw_len[k]) std::memcpy(d, r.raw[k], r.raw_len[k]);
                d += r.raw_len[k];
            }
        } else {  // the fragments' Base64 back to back (run_downloads rebases the spans)
            uint8_t* d = r.in_dst;
            for (uint32_t k = 0; k < B->nfrag; ++k) {
                const dfs_span& s = r.frags[k];
                if (s.len == DFS_SPAN_MISSING || !s.len) continue;
                std::memcpy(d, r.text + s.off, s.len);
                d += s.len;
            }
        }
        {
            std::lock_guard<std::mutex> bl(r.sync->mu);
            ++r.sync->copied_in;
            r.sync->cv.notify_one();
        }
        lk.lock();
    }
    r.cv.wait(lk, [&] { return r.phase >= 3; });
    lk.unlock();
    const auto t_ready = Clock::now();
    if (r.want_view) {
        // the view (and its reference) is the caller's only with a good result
        const bool take = r.view && r.out_src && (r.kind == kUpload || r.status == DFS_OK);
        *r.view_ptr = take ? r.out_src : nullptr;
        *r.view_handle = take ? r.view : nullptr;
        if (r.view && !take) (void)dfs_view_release(r.view);
    } else if (r.out_src && r.out_bytes && (r.kind == kUpload || r.status == DFS_OK)) {
        std::memcpy(r.kind == kUpload ? static_cast<void*>(r.b64) : static_cast<void*>(r.out), r.out_src, r.out_bytes);
    }
    const int status = r.status;
    std::lock_guard<std::mutex> bl(r.sync->mu);  // the last touch of the batch (the worker waits for it)
    r.sync->return_s += std::chrono::duration<double>(Clock::now() - t_ready).count();
    ++r.sync->copied_out;
    r.sync->cv.notify_one();
    return status;
}

}  // namespace

extern "C" {

int dfs_batcher_create(int device, uint32_t nfrag, const dfs_batcher_opts* opts, dfs_batcher** out) {
    if (!out || !nfrag || nfrag > 64) return DFS_E_ARG;
    *out = nullptr;
    auto* B = new (std::nothrow) dfs_batcher;
    if (!B) return DFS_E_NOMEM;
    B->device = device;
    B->nfrag = nfrag;
    B->o = dfs_batcher_opts{200, 1024, 1ull << 30, 2};
    if (const char* e = std::getenv("DFS_BATCH_DL_IN")) B->dl_in_kernel = std::strcmp(e, "dma") != 0;
    if (opts) {
        if (opts->max_wait_us) B->o.max_wait_us = opts->max_wait_us;
        if (opts->max_files) B->o.max_files = opts->max_files;
        if (opts->max_bytes) B->o.max_bytes = opts->max_bytes;
        if (opts->depth) B->o.depth = std::min<uint32_t>(opts->depth, 8);
    }
    int rc = DFS_OK;
    for (uint32_t i = 0; i < B->o.depth && rc == DFS_OK; ++i) {
        auto* w = new (std::nothrow) Worker;
        if (!w) {
            rc = DFS_E_NOMEM;
            break;
        }
        B->workers.push_back(w);
        rc = dfs_open(&w->ctx, device);
        if (rc == DFS_OK) w->stream = dfs::ctx_stream(w->ctx);  // the ctx's own stream: one hardware queue per worker
        if (rc == DFS_OK && hipEventCreateWithFlags(&w->done, hipEventDisableTiming) != hipSuccess)
            rc = DFS_E_HIP;
    }
    if (rc == DFS_OK)
        for (Worker* w : B->workers) w->th = std::thread(worker_main, B, w);
    if (rc != DFS_OK) {
        dfs_batcher_destroy(B);
        return rc;
    }
    *out = B;
    return DFS_OK;
}

int dfs_batcher_destroy(dfs_batcher* B) {
    if (!B) return DFS_E_ARG;
    {
        std::lock_guard<std::mutex> lk(B->mu);
        B->stop = true;
    }
    B->cv_work.notify_all();
    for (Worker* w : B->workers) {
        if (w->th.joinable()) w->th.join();
        (void)hipSetDevice(B->device);
        for (auto& v : w->outs) {  // views still out: their holders read this memory
            std::unique_lock<std::mutex> lk(v->mu);
            v->cv.wait(lk, [&] { return v->refs == 0; });
            v->pin.release();
        }
        for (Buf* b : {&w->pin_in, &w->d_in, &w->d_out, &w->d_dig}) b->release();
        if (w->ctx) dfs_close(w->ctx);  // destroys its stream
        if (w->done) (void)hipEventDestroy(w->done);
        delete w;
    }
    delete B;
    return DFS_OK;
}

int dfs_host_alloc(uint64_t bytes, void** p) {
    if (!p) return DFS_E_ARG;
    *p = nullptr;
    void* q = nullptr;
    // mapped + coherent (fine-grained): the batcher's copy kernel reads and writes it in place, and
    // the host sees the kernel's writes once the batch's event completes
    if (hipHostMalloc(&q, bytes ? bytes : 1, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
        (void)hipGetLastError();
        return DFS_E_NOMEM;
    }
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, q, 0) != hipSuccess || !d) {
        (void)hipGetLastError();
        (void)hipHostFree(q);
        return DFS_E_HIP;
    }
    std::unique_lock<std::shared_mutex> lk(g_pin_mu);
    g_pinned[reinterpret_cast<uintptr_t>(q)] = Pinned{bytes, reinterpret_cast<uintptr_t>(d)};
    *p = q;
    return DFS_OK;
}

int dfs_host_free(void* p) {
    if (!p) return DFS_E_ARG;
    {
        std::unique_lock<std::shared_mutex> lk(g_pin_mu);
        auto it = g_pinned.find(reinterpret_cast<uintptr_t>(p));
        if (it == g_pinned.end()) return DFS_E_ARG;
        g_pinned.erase(it);
    }
    return hipHostFree(p) == hipSuccess ? DFS_OK : DFS_E_HIP;
}

int dfs_batcher_stats(dfs_batcher* B, dfs_batcher_stats_t* out) {
    if (!B || !out) return DFS_E_ARG;
    std::lock_guard<std::mutex> lk(B->mu);
    *out = B->st;
    return DFS_OK;
}

}  // extern "C"

namespace {

// b64 != NULL: the Base64 is copied (or DMA'd) into the caller's buffer;
// view_ptr != NULL: it is handed out as a view of the batch's result buffer.
int submit_upload(dfs_batcher* B, const uint8_t* file, uint64_t len, uint8_t* file_digest, uint8_t* frag_digest,
                  char* b64, uint64_t b64_cap, uint64_t* b64_off, const char** view_ptr, dfs_view** view) {
    if (view_ptr) *view_ptr = nullptr;
    if (view) *view = nullptr;
    if (!B || (len && !file) || !file_digest || !frag_digest || !b64_off) return DFS_E_ARG;
    if (len >= kMaxFile) return DFS_E_ARG;  // refused here, to this caller only: a batch fails as a whole
    const uint32_t N = B->nfrag;
    dfs_span fr[64];
    if (dfs_split_plan(len, N, fr) != DFS_OK) return DFS_E_ARG;
    b64_off[0] = 0;
    for (uint32_t i = 0; i < N; ++i) b64_off[i + 1] = b64_off[i] + enc_len(fr[i].len);  // SN:636
    if (!view_ptr && (b64_off[N] > b64_cap || (b64_off[N] && !b64))) return DFS_E_ARG;
    Req r;
    r.kind = kUpload;
    r.file = file;
    r.len = r.need = len;
    r.out_bytes = b64_off[N];
    r.fd = file_digest;
    r.frd = frag_digest;
    r.b64 = b64;
    r.b64_off = b64_off;
    r.want_view = view_ptr != nullptr;
    r.view_ptr = reinterpret_cast<const void**>(view_ptr);
    r.view_handle = view;
    r.direct = in_pinned(file, len) && (r.want_view || in_pinned(b64, r.out_bytes));
    return submit(B, r);
}

}  // namespace

extern "C" {

int dfs_submit_upload(dfs_batcher* B, const uint8_t* file, uint64_t len, uint8_t* file_digest, uint8_t* frag_digest,
                      char* b64, uint64_t b64_cap, uint64_t* b64_off) {
    return submit_upload(B, file, len, file_digest, frag_digest, b64, b64_cap, b64_off, nullptr, nullptr);
}

int dfs_submit_upload_view(dfs_batcher* B, const uint8_t* file, uint64_t len, uint8_t* file_digest, uint8_t* frag_digest,
                           const char** b64, uint64_t* b64_off, dfs_view** view) {
    if (!b64 || !view) return DFS_E_ARG;
    return submit_upload(B, file, len, file_digest, frag_digest, nullptr, 0, b64_off, b64, view);
}

int dfs_view_release(dfs_view* v) {
    if (!v) return DFS_E_ARG;
    std::lock_guard<std::mutex> lk(v->mu);
    if (v->refs <= 0) return DFS_E_ARG;
    if (--v->refs == 0) v->cv.notify_all();
    return DFS_OK;
}

int dfs_submit_reassemble(dfs_batcher* B, const uint8_t* const* frags, const uint64_t* frag_len,
                          const uint8_t* expected_file_digest, uint8_t* out, uint8_t* file_digest_out) {
    if (!B || !frags || !frag_len) return DFS_E_ARG;
    uint64_t len = 0;
    for (uint32_t k = 0; k < B->nfrag; ++k) {
        if (!frags[k] && frag_len[k]) return DFS_E_MISSING;  // "Could not retrieve fragment i", SN:443-446: nothing is hashed
        if (frag_len[k] >= kMaxFile) return DFS_E_ARG;
        len += frag_len[k];
    }
    if (len >= kMaxFile || (len && !out)) return DFS_E_ARG;
    Req r;
    r.kind = kReassemble;
    r.raw = frags;
    r.raw_len = frag_len;
    r.len = r.need = r.out_bytes = len;
    r.exp_file = expected_file_digest;
    r.out = out;
    r.digest_out = file_digest_out;
    return submit(B, r);
}

}  // extern "C"

namespace {

int submit_download(dfs_batcher* B, const char* b64, const dfs_span* frags, uint64_t file_len,
                    const uint8_t* expected_frag_digest, const uint8_t* expected_file_digest, uint8_t* out,
                    const uint8_t** view_ptr, dfs_view** view) {
    if (view_ptr) *view_ptr = nullptr;
    if (view) *view = nullptr;
    if (!B || !frags || (file_len && !out && !view_ptr)) return DFS_E_ARG;
    Req r;
    r.kind = kDownload + (expected_frag_digest ? 2 : 0) + (expected_file_digest ? 1 : 0);
    // A request that could not run is refused here, to its caller only: inside
    // a batch it would fail its neighbours' requests too.  The file cannot be
    // longer than what its fragments' Base64 can decode to.
    uint64_t need = 0, cap = 0;
    for (uint32_t k = 0; k < B->nfrag; ++k)
        if (frags[k].len != DFS_SPAN_MISSING) {
            if (frags[k].len >= 2 * kMaxFile || frags[k].off >= (1ull << 62)) return DFS_E_ARG;
            need += frags[k].len;
            cap += dfs_b64_decoded_cap(frags[k].len);
        }
    if (need && !b64) return DFS_E_ARG;
    bool any_missing = false;
    for (uint32_t k = 0; k < B->nfrag; ++k) any_missing = any_missing || frags[k].len == DFS_SPAN_MISSING;
    if (file_len >= kMaxFile || (!any_missing && file_len > cap)) return DFS_E_ARG;
    r.text = b64;
    r.frags = frags;
    r.len = file_len;
    r.need = need;
    r.out_bytes = file_len;
    r.exp_frag = expected_frag_digest;
    r.exp_file = expected_file_digest;
    r.out = out;
    r.want_view = view_ptr != nullptr;
    r.view_ptr = reinterpret_cast<const void**>(view_ptr);
    r.view_handle = view;
    r.direct = r.want_view || in_pinned(out, file_len);
    for (uint32_t k = 0; k < B->nfrag && r.direct; ++k)
        if (frags[k].len != DFS_SPAN_MISSING) r.direct = in_pinned(b64 + frags[k].off, frags[k].len);
    return submit(B, r);
}

}  // namespace

extern "C" {

int dfs_submit_download(dfs_batcher* B, const char* b64, const dfs_span* frags, uint64_t file_len,
                        const uint8_t* expected_frag_digest, const uint8_t* expected_file_digest, uint8_t* out) {
    return submit_download(B, b64, frags, file_len, expected_frag_digest, expected_file_digest, out, nullptr, nullptr);
}

int dfs_submit_download_view(dfs_batcher* B, const char* b64, const dfs_span* frags, uint64_t file_len,
                             const uint8_t* expected_frag_digest, const uint8_t* expected_file_digest,
                             const uint8_t** out, dfs_view** view) {
    if (!out || !view) return DFS_E_ARG;
    return submit_download(B, b64, frags, file_len, expected_frag_digest, expected_file_digest, nullptr, out, view);
}

}  // extern "C"
