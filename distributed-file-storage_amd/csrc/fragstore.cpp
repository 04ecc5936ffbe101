// fragstore.cpp — the node's on-disk fragment store (include/dfs_gpu.h,
// dfs_store_write_fragments / dfs_store_read_fragments).
//
// Reference sites replaced (StorageNode.java, SN:line): the fragment
// directory <dataRoot>/<fileId>/fragments made by Files.createDirectories
// (:147-149 upload, :273-275 replica receiver), Files.write(<i>.frag) of the
// raw fragment bytes (:165-166, :284-285) and tryLoadFragmentLocal's
// Files.readAllBytes (:463-469).  The file format is unchanged: one file per
// fragment, raw bytes, so a reference node and this library read each
// other's data directories.
//
// Device buffers move through a ring of pinned host slots on the ctx stream:
// while a thread pool writes slot b to disk, the DMA engine fills slot b+1
// from HBM (upload); on download the pool reads slot b+1 from disk while
// slot b is copied into HBM.  Fragments longer than a slot are split into
// slot-sized chunks written / read at their file offsets; a multi-chunk
// fragment is written to <i>.frag.tmp and renamed into place once every chunk
// succeeded, so a concurrent reader never sees it half written.
//
// Locking: host-buffer calls touch no ctx state and take no lock (ctx may be
// NULL).  Device calls hold only the staging ring's own mutex, never the ctx
// mutex, so a long store does not block uploads / downloads on the same ctx.
// The file I/O runs on one process-wide pool of I/O threads.
#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/dfs_gpu.h"
#include "dfs_internal.h"

namespace dfs {

constexpr int kSlots = 4;

struct StoreStaging {
    int device = 0;
    size_t slot_bytes = 0;
    uint8_t* host[kSlots] = {};
    hipEvent_t ev[kSlots] = {};
};

void store_staging_free(StoreStaging* s) {
    if (!s) return;
    (void)hipSetDevice(s->device);
    for (int i = 0; i < kSlots; ++i) {
        if (s->host[i]) (void)hipHostFree(s->host[i]);
        if (s->ev[i]) (void)hipEventDestroy(s->ev[i]);
    }
    delete s;
}

}  // namespace dfs

namespace {

using dfs::kSlots;
using dfs::StoreStaging;

size_t env_size(const char* name, size_t def, size_t lo, size_t hi) {
    const char* v = std::getenv(name);
    if (!v) return def;
    long long x = std::atoll(v);
    if (x < static_cast<long long>(lo)) return lo;
    if (x > static_cast<long long>(hi)) return hi;
    return static_cast<size_t>(x);
}

// Process-wide pool of I/O threads (shared by every call; a call waits on
// its own latches, tasks never wait on each other).
class Pool {
   public:
    explicit Pool(unsigned n) {
        for (unsigned i = 0; i < n; ++i) th_.emplace_back([this] { run(); });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    void submit(std::function<void()> f) {
        {
            std::lock_guard<std::mutex> lk(m_);
            q_.push_back(std::move(f));
        }
        cv_.notify_one();
    }

   private:
    void run() {
        for (;;) {
            std::function<void()> f;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [this] { return stop_ || !q_.empty(); });
                if (q_.empty()) return;
                f = std::move(q_.front());
                q_.pop_front();
            }
            f();
        }
    }
    std::vector<std::thread> th_;
    std::deque<std::function<void()>> q_;
    std::mutex m_;
    std::condition_variable cv_;
    bool stop_ = false;
};

// Counts outstanding jobs of one group (a slot's batch, a phase).
class Latch {
   public:
    void add(int n) {
        std::lock_guard<std::mutex> lk(m_);
        left_ += n;
    }
    void done() {
        std::lock_guard<std::mutex> lk(m_);
        if (--left_ == 0) cv_.notify_all();
    }
    void wait() {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [this] { return left_ == 0; });
    }

   private:
    std::mutex m_;
    std::condition_variable cv_;
    int left_ = 0;
};

unsigned pool_threads() {
    unsigned hw = std::thread::hardware_concurrency();
    if (hw == 0) hw = 4;
    return static_cast<unsigned>(env_size("DFS_STORE_THREADS", std::min(16u, hw), 1, 64));
}

Pool& io_pool() {
    static Pool* p = new Pool(pool_threads());  // lives until exit (threads are detached at exit by the OS)
    return *p;
}

std::string hex32(const uint8_t* d) {
    static const char* k = "0123456789abcdef";
    std::string s(64, '0');
    for (int i = 0; i < 32; ++i) {
        s[2 * i] = k[d[i] >> 4];
        s[2 * i + 1] = k[d[i] & 15];
    }
    return s;
}

// Files.createDirectories: every missing component is created; an existing
// non-directory is an error.
bool mkdirs(const std::string& path) {
    struct stat st;
    if (::stat(path.c_str(), &st) == 0) return S_ISDIR(st.st_mode);
    size_t cut = path.find_last_of('/');
    if (cut != std::string::npos && cut > 0 && !mkdirs(path.substr(0, cut))) return false;
    if (::mkdir(path.c_str(), 0755) == 0) return true;
    return errno == EEXIST && ::stat(path.c_str(), &st) == 0 && S_ISDIR(st.st_mode);
}

bool pwrite_all(int fd, const uint8_t* p, size_t n, off_t at) {
    while (n) {
        ssize_t w = ::pwrite(fd, p, n, at);
        if (w < 0) {
            if (errno == EINTR) continue;
            return false;
        }
        p += w;
        n -= static_cast<size_t>(w);
        at += w;
    }
    return true;
}

bool pread_all(int fd, uint8_t* p, size_t n, off_t at) {
    while (n) {
        ssize_t r = ::pread(fd, p, n, at);
        if (r < 0) {
            if (errno == EINTR) continue;
            return false;
        }
        if (r == 0) return false;  // file shrank under us
        p += r;
        n -= static_cast<size_t>(r);
        at += r;
    }
    return true;
}

// One slot-sized piece of one fragment.
struct Chunk {
    uint32_t ref;
    uint64_t at;   // offset inside the fragment (and its file)
    uint64_t len;
};

struct Call {
    const char* root;
    const uint8_t* digests;
    const dfs_frag_ref* refs;
    uint32_t n;
    std::vector<std::string> dir;      // per ref: <root>/<hex>/fragments
    std::vector<std::atomic<int32_t>> st;
    explicit Call(uint32_t n_) : n(n_), dir(n_), st(n_) {
        for (auto& s : st) s.store(DFS_OK, std::memory_order_relaxed);
    }
    std::string path(uint32_t i) const { return dir[i] + "/" + std::to_string(refs[i].index) + ".frag"; }
    std::string tmp(uint32_t i) const { return path(i) + ".tmp"; }
    void fail(uint32_t i, int32_t code) {
        int32_t ok = DFS_OK;
        st[i].compare_exchange_strong(ok, code);
    }
};

// Directory names per ref, deduplicated per file index.
void plan_dirs(Call& c) {
    std::unordered_map<uint32_t, std::string> seen;
    std::string root(c.root);
    while (root.size() > 1 && root.back() == '/') root.pop_back();
    for (uint32_t i = 0; i < c.n; ++i) {
        auto it = seen.find(c.refs[i].file);
        if (it == seen.end())
            it = seen.emplace(c.refs[i].file, root + "/" + hex32(c.digests + 32ull * c.refs[i].file) + "/fragments")
                     .first;
        c.dir[i] = it->second;
    }
}

// Split refs (those still OK, sizes in len[]) into chunks of <= slot bytes,
// then pack consecutive chunks into batches of <= slot bytes.
void plan_batches(const Call& c, const std::vector<uint64_t>& len, size_t slot, std::vector<std::vector<Chunk>>& batches) {
    std::vector<Chunk> cur;
    uint64_t fill = 0;
    for (uint32_t i = 0; i < c.n; ++i) {
        if (c.st[i].load(std::memory_order_relaxed) != DFS_OK || len[i] == 0) continue;
        for (uint64_t at = 0; at < len[i]; at += slot) {
            const uint64_t l = std::min<uint64_t>(slot, len[i] - at);
            if (fill + l > slot) {
                batches.push_back(std::move(cur));
                cur.clear();
                fill = 0;
            }
            cur.push_back({i, at, l});
            fill += l;
        }
    }
    if (!cur.empty()) batches.push_back(std::move(cur));
}

int acquire_staging(dfs_ctx* ctx, StoreStaging** out) {
    StoreStaging*& s = dfs::ctx_store(ctx);
    const size_t want = env_size("DFS_STORE_SLOT_MB", 64, 1, 1024) << 20;
    if (s && s->slot_bytes == want) {
        *out = s;
        return DFS_OK;
    }
    dfs::store_staging_free(s);
    s = new (std::nothrow) StoreStaging;
    if (!s) return DFS_E_NOMEM;
    s->device = dfs::ctx_device(ctx);
    s->slot_bytes = want;
    for (int i = 0; i < kSlots; ++i) {
        if (hipHostMalloc(reinterpret_cast<void**>(&s->host[i]), want, hipHostMallocDefault) != hipSuccess ||
            hipEventCreateWithFlags(&s->ev[i], hipEventDisableTiming) != hipSuccess) {
            dfs::store_staging_free(s);
            s = nullptr;
            return DFS_E_NOMEM;
        }
    }
    *out = s;
    return DFS_OK;
}

int finish(Call& c, int32_t* status, int rc) {
    int first = DFS_OK;
    for (uint32_t i = 0; i < c.n; ++i) {
        const int32_t s = c.st[i].load();
        if (status) status[i] = s;
        if (s != DFS_OK && first == DFS_OK) first = s;
    }
    return rc != DFS_OK ? rc : first;
}

int check_args(dfs_ctx* ctx, const char* root, const uint8_t* dig, uint32_t nfiles, const void* data,
               const dfs_frag_ref* refs, uint32_t n, uint32_t flags) {
    if (!root || !*root || (n && (!dig || !refs))) return DFS_E_ARG;
    if ((flags & DFS_DEVICE_PTRS) && !ctx) return DFS_E_ARG;
    for (uint32_t i = 0; i < n; ++i)
        if ((refs[i].len && !data) || refs[i].file >= nfiles) return DFS_E_ARG;
    return DFS_OK;
}

}  // namespace

extern "C" {

int dfs_store_write_fragments(dfs_ctx* ctx, const char* node_root, const uint8_t* file_digest, uint32_t nfiles,
                              const uint8_t* data, const dfs_frag_ref* refs, uint32_t n, int32_t* status,
                              uint32_t flags) {
    if (int rc = check_args(ctx, node_root, file_digest, nfiles, data, refs, n, flags)) return rc;
    const bool dev = flags & DFS_DEVICE_PTRS;
    std::unique_lock<std::mutex> lk;
    if (dev) lk = std::unique_lock<std::mutex>(dfs::ctx_store_mutex(ctx));
    StoreStaging* stg = nullptr;
    if (dev) {
        if (hipSetDevice(dfs::ctx_device(ctx)) != hipSuccess) return DFS_E_HIP;
        if (int rc = acquire_staging(ctx, &stg)) return rc;
    }
    const size_t slot = dev ? stg->slot_bytes : env_size("DFS_STORE_SLOT_MB", 64, 1, 1024) << 20;

    Call c(n);
    c.root = node_root;
    c.digests = file_digest;
    c.refs = refs;
    plan_dirs(c);
    std::vector<uint64_t> len(n);
    for (uint32_t i = 0; i < n; ++i) len[i] = refs[i].len;

    Pool& pool = io_pool();
    // Chunks still to write per multi-chunk fragment (its .tmp is renamed
    // into place by the writer of the last one).
    std::vector<std::atomic<uint32_t>> chunks_left(n);
    for (uint32_t i = 0; i < n; ++i)
        chunks_left[i].store(len[i] > slot ? static_cast<uint32_t>((len[i] + slot - 1) / slot) : 0u,
                             std::memory_order_relaxed);
    // Phase 1: directories (Files.createDirectories, SN:149 / 275), empty
    // fragments, and the .tmp of fragments written in several chunks.
    {
        std::unordered_map<std::string, std::vector<uint32_t>> by_dir;
        for (uint32_t i = 0; i < n; ++i) by_dir[c.dir[i]].push_back(i);
        Latch l;
        l.add(static_cast<int>(by_dir.size()));
        for (auto& kv : by_dir) {
            pool.submit([&c, &l, &len, &kv, slot] {
                const bool ok = mkdirs(kv.first);
                for (uint32_t i : kv.second) {
                    if (!ok) {
                        c.fail(i, DFS_E_IO);
                        continue;
                    }
                    if (len[i] == 0 || len[i] > slot) {
                        const std::string p = len[i] ? c.tmp(i) : c.path(i);
                        int fd = ::open(p.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
                        if (fd < 0) c.fail(i, DFS_E_IO);
                        else ::close(fd);
                    }
                }
                l.done();
            });
        }
        l.wait();
    }

    std::vector<std::vector<Chunk>> batches;
    plan_batches(c, len, slot, batches);
    auto write_chunk = [&c, &len, &chunks_left, slot](const Chunk& k, const uint8_t* src) {
        const bool whole = len[k.ref] <= slot;
        const std::string p = whole ? c.path(k.ref) : c.tmp(k.ref);
        int fd = ::open(p.c_str(), O_WRONLY | O_CREAT | O_CLOEXEC | (whole ? O_TRUNC : 0), 0644);
        if (fd < 0) {
            c.fail(k.ref, DFS_E_IO);
        } else {
            if (!pwrite_all(fd, src, k.len, static_cast<off_t>(k.at))) c.fail(k.ref, DFS_E_IO);
            if (::close(fd) != 0) c.fail(k.ref, DFS_E_IO);
        }
        if (!whole && chunks_left[k.ref].fetch_sub(1, std::memory_order_acq_rel) == 1) {
            if (c.st[k.ref].load() == DFS_OK) {
                if (::rename(p.c_str(), c.path(k.ref).c_str()) != 0) c.fail(k.ref, DFS_E_IO);
            } else {
                ::unlink(p.c_str());
            }
        }
    };

    int rc = DFS_OK;
    if (!dev) {
        Latch l;
        for (auto& b : batches) {
            l.add(static_cast<int>(b.size()));
            for (const Chunk& k : b)
                pool.submit([&, k] {
                    write_chunk(k, data + refs[k.ref].off + k.at);
                    l.done();
                });
        }
        l.wait();
        return finish(c, status, rc);
    }

    // Device: D2H of batch b into slot b % kSlots overlaps the writes of the
    // batches before it; a slot is reused once its writers are done.
    hipStream_t s = dfs::ctx_stream(ctx);
    Latch slot_latch[kSlots];
    for (size_t b = 0; b < batches.size() && rc == DFS_OK; ++b) {
        const int k = static_cast<int>(b % kSlots);
        slot_latch[k].wait();
        uint8_t* host = stg->host[k];
        // One copy per run of chunks contiguous in HBM.
        uint64_t pos = 0;
        size_t i = 0;
        auto& batch = batches[b];
        while (i < batch.size() && rc == DFS_OK) {
            const uint64_t src0 = refs[batch[i].ref].off + batch[i].at;
            uint64_t run = batch[i].len;
            size_t j = i + 1;
            while (j < batch.size() && refs[batch[j].ref].off + batch[j].at == src0 + run) run += batch[j++].len;
            if (hipMemcpyAsync(host + pos, data + src0, run, hipMemcpyDeviceToHost, s) != hipSuccess) rc = DFS_E_HIP;
            pos += run;
            i = j;
        }
        if (rc == DFS_OK && (hipEventRecord(stg->ev[k], s) != hipSuccess || dfs::quiet_wait(stg->ev[k]) != hipSuccess))
            rc = DFS_E_HIP;
        if (rc != DFS_OK) break;
        slot_latch[k].add(static_cast<int>(batch.size()));
        pos = 0;
        for (const Chunk& ch : batch) {
            const uint8_t* src = host + pos;
            pos += ch.len;
            pool.submit([&, ch, src, k] {
                write_chunk(ch, src);
                slot_latch[k].done();
            });
        }
    }
    for (auto& l : slot_latch) l.wait();
    return finish(c, status, rc);
}

int dfs_store_read_fragments(dfs_ctx* ctx, const char* node_root, const uint8_t* file_digest, uint32_t nfiles,
                             uint8_t* data, const dfs_frag_ref* refs, uint32_t n, uint64_t* out_len, int32_t* status,
                             uint32_t flags) {
    if (int rc = check_args(ctx, node_root, file_digest, nfiles, data, refs, n, flags)) return rc;
    const bool dev = flags & DFS_DEVICE_PTRS;
    std::unique_lock<std::mutex> lk;
    if (dev) lk = std::unique_lock<std::mutex>(dfs::ctx_store_mutex(ctx));
    StoreStaging* stg = nullptr;
    if (dev) {
        if (hipSetDevice(dfs::ctx_device(ctx)) != hipSuccess) return DFS_E_HIP;
        if (int rc = acquire_staging(ctx, &stg)) return rc;
    }
    const size_t slot = dev ? stg->slot_bytes : env_size("DFS_STORE_SLOT_MB", 64, 1, 1024) << 20;

    Call c(n);
    c.root = node_root;
    c.digests = file_digest;
    c.refs = refs;
    plan_dirs(c);
    std::vector<uint64_t> len(n, 0);

    Pool& pool = io_pool();
    const unsigned nt = pool_threads();
    // Phase 1: sizes (Files.exists + readAllBytes length, SN:465-466).
    {
        Latch l;
        const uint32_t per = std::max<uint32_t>(1, (n + nt * 4 - 1) / (nt * 4));
        for (uint32_t a = 0; a < n; a += per) {
            const uint32_t e = std::min<uint32_t>(n, a + per);
            l.add(1);
            pool.submit([&c, &l, &len, refs, a, e] {
                for (uint32_t i = a; i < e; ++i) {
                    struct stat st;
                    if (::stat(c.path(i).c_str(), &st) != 0) {
                        c.fail(i, errno == ENOENT || errno == ENOTDIR ? DFS_E_MISSING : DFS_E_IO);
                    } else if (!S_ISREG(st.st_mode)) {
                        c.fail(i, DFS_E_IO);
                    } else if (static_cast<uint64_t>(st.st_size) > refs[i].len) {
                        c.fail(i, DFS_E_ARG);
                    } else {
                        len[i] = static_cast<uint64_t>(st.st_size);
                    }
                }
                l.done();
            });
        }
        l.wait();
    }
    if (out_len)
        for (uint32_t i = 0; i < n; ++i) out_len[i] = len[i];

    std::vector<std::vector<Chunk>> batches;
    plan_batches(c, len, slot, batches);
    auto read_chunk = [&c](const Chunk& k, uint8_t* dst) {
        int fd = ::open(c.path(k.ref).c_str(), O_RDONLY | O_CLOEXEC);
        if (fd < 0) {
            c.fail(k.ref, DFS_E_IO);
            return;
        }
        if (!pread_all(fd, dst, k.len, static_cast<off_t>(k.at))) c.fail(k.ref, DFS_E_IO);
        ::close(fd);
    };

    int rc = DFS_OK;
    if (!dev) {
        Latch l;
        for (auto& b : batches) {
            l.add(static_cast<int>(b.size()));
            for (const Chunk& k : b)
                pool.submit([&, k] {
                    read_chunk(k, data + refs[k.ref].off + k.at);
                    l.done();
                });
        }
        l.wait();
        return finish(c, status, rc);
    }

    // Device: the pool fills slot b+1 from disk while slot b goes to HBM.
    hipStream_t s = dfs::ctx_stream(ctx);
    Latch slot_latch[kSlots];
    bool pending[kSlots] = {};  // an H2D copy out of the slot may still run
    auto fill = [&](size_t b) -> int {
        const int k = static_cast<int>(b % kSlots);
        if (pending[k]) {
            if (dfs::quiet_wait(stg->ev[k]) != hipSuccess) return DFS_E_HIP;
            pending[k] = false;
        }
        slot_latch[k].add(static_cast<int>(batches[b].size()));
        uint64_t pos = 0;
        for (const Chunk& ch : batches[b]) {
            uint8_t* dst = stg->host[k] + pos;
            pos += ch.len;
            pool.submit([&, ch, dst, k] {
                read_chunk(ch, dst);
                slot_latch[k].done();
            });
        }
        return DFS_OK;
    };
    const size_t ahead = kSlots - 1;
    for (size_t b = 0; b < std::min(ahead, batches.size()) && rc == DFS_OK; ++b) rc = fill(b);
    for (size_t b = 0; b < batches.size() && rc == DFS_OK; ++b) {
        const int k = static_cast<int>(b % kSlots);
        slot_latch[k].wait();
        uint64_t pos = 0;
        size_t i = 0;
        auto& batch = batches[b];
        while (i < batch.size() && rc == DFS_OK) {
            const uint64_t dst0 = refs[batch[i].ref].off + batch[i].at;
            uint64_t run = batch[i].len;
            size_t j = i + 1;
            while (j < batch.size() && refs[batch[j].ref].off + batch[j].at == dst0 + run) run += batch[j++].len;
            if (hipMemcpyAsync(data + dst0, stg->host[k] + pos, run, hipMemcpyHostToDevice, s) != hipSuccess)
                rc = DFS_E_HIP;
            pos += run;
            i = j;
        }
        if (rc == DFS_OK && hipEventRecord(stg->ev[k], s) != hipSuccess) rc = DFS_E_HIP;
        pending[k] = true;
        if (rc == DFS_OK && b + ahead < batches.size()) rc = fill(b + ahead);
    }
    for (auto& l : slot_latch) l.wait();
    for (int k = 0; k < kSlots; ++k)  // the last copy out of every slot (recorded after it)
        if (pending[k] && dfs::quiet_wait(stg->ev[k]) != hipSuccess && rc == DFS_OK) rc = DFS_E_HIP;
    return finish(c, status, rc);
}

}  // extern "C"
