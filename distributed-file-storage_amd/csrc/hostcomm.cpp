// hostcomm.cpp — a communicator that moves bytes through host shared memory
// instead of RCCL: the ranks are processes of one host, each with its own
// dfs_ctx, on any GPUs — also several ranks on ONE GPU, which RCCL refuses.
//
// Why it exists: the multi-rank paths (placement, degraded fetch, the digest
// exchange and the failure report of the holders' verify; StorageNode.java
// :195-259, :265-293, :422-446) must be exercisable with every kernel and
// every buffer layout on a box with one GPU.  Only the wire differs: a send
// is device -> mailbox, a receive mailbox -> device, both synchronous, so the
// calls keep RCCL's meaning (ops of a group progress together; between two
// ranks they pair in posting order) without its asynchrony.  It is chosen by
// the unique id: dfs_comm_unique_id makes a host id when
// DFS_COMM_TRANSPORT=host is set, and dfs_comm_init_rank recognises it, so
// every rank of a communicator agrees.  Slow by construction (pageable
// staging, 4 MiB chunks): for tests and rehearsals, not for measurements.
//
// Shared region (POSIX shm, unlinked by rank 0 once every rank is attached):
// a header and one mailbox per ordered pair of ranks.  A mailbox has one
// producer and one consumer: chunk counters `wr` / `rd` (the slot is empty
// when equal), the chunk's length, the bytes.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <thread>
#include <vector>

#include "../../include/dfs_gpu.h"
#include "placement_internal.h"

namespace dfs {

namespace {

constexpr char kMagic[16] = "DFS-HOST-COMM-1";  // 15 chars + NUL
constexpr uint64_t kSlot = 4ull << 20;
// Seconds without progress after which a rendezvous or an exchange gives up
// (a peer died or never came): 120, or DFS_HOST_COMM_TIMEOUT_S.
double timeout_s() {
    if (const char* e = std::getenv("DFS_HOST_COMM_TIMEOUT_S")) {
        const double v = std::atof(e);
        if (v > 0) return v;
    }
    return 120.0;
}

struct Header {
    std::atomic<uint32_t> attached;
    std::atomic<uint32_t> nranks;  // set by the first rank to attach; the others must agree
    uint8_t pad[56];
};

struct Box {
    std::atomic<uint64_t> wr, rd;
    uint64_t len;
    uint8_t pad[40];
    uint8_t data[kSlot];
};

static_assert(std::atomic<uint64_t>::is_always_lock_free, "mailbox counters live in shared memory");

using Clock = std::chrono::steady_clock;
double since(Clock::time_point t) { return std::chrono::duration<double>(Clock::now() - t).count(); }

}  // namespace

struct HostComm {
    uint32_t W = 0, me = 0;
    void* map = nullptr;
    size_t bytes = 0;
    char name[64] = {0};
    Header* hdr() const { return static_cast<Header*>(map); }
    Box* box(uint32_t from, uint32_t to) const {
        return reinterpret_cast<Box*>(static_cast<uint8_t*>(map) + sizeof(Header)) + (static_cast<size_t>(from) * W + to);
    }
};

bool host_comm_is_id(const uint8_t* id) { return std::memcmp(id, kMagic, sizeof kMagic) == 0; }

int host_comm_make_id(uint8_t* id) {
    std::memset(id, 0, DFS_COMM_ID_BYTES);
    std::memcpy(id, kMagic, sizeof kMagic);
    int fd = open("/dev/urandom", O_RDONLY);
    if (fd < 0) return DFS_E_COMM;
    const ssize_t n = read(fd, id + sizeof kMagic, 12);
    close(fd);
    return n == 12 ? DFS_OK : DFS_E_COMM;
}

int host_comm_open(const uint8_t* id, uint32_t nranks, uint32_t rank, HostComm** out) {
    *out = nullptr;
    if (nranks > 16) return DFS_E_ARG;  // W * W mailboxes of 4 MiB
    auto* h = new (std::nothrow) HostComm;
    if (!h) return DFS_E_NOMEM;
    h->W = nranks;
    h->me = rank;
    char* p = h->name + std::snprintf(h->name, sizeof h->name, "/dfs-comm-");
    for (int i = 0; i < 12; ++i) p += std::snprintf(p, 3, "%02x", id[sizeof kMagic + i]);
    h->bytes = sizeof(Header) + sizeof(Box) * static_cast<size_t>(nranks) * nranks;
    const int fd = shm_open(h->name, O_CREAT | O_RDWR, 0600);
    struct stat sb;
    // grow only: a rank that disagrees on the world size must not shrink what others have mapped
    if (fd < 0 || fstat(fd, &sb) != 0 ||
        (static_cast<size_t>(sb.st_size) < h->bytes && ftruncate(fd, static_cast<off_t>(h->bytes)) != 0)) {
        if (fd >= 0) close(fd);
        delete h;
        return DFS_E_COMM;
    }
    h->map = mmap(nullptr, h->bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (h->map == MAP_FAILED) {
        delete h;
        return DFS_E_COMM;
    }
    // a fresh object is zero-filled: counters start at 0.  Wait for every rank.
    uint32_t seen = 0;
    bool ok = h->hdr()->nranks.compare_exchange_strong(seen, nranks) || seen == nranks;  // same world size everywhere
    h->hdr()->attached.fetch_add(1, std::memory_order_acq_rel);
    const auto t0 = Clock::now();
    const double limit = timeout_s();
    while (ok && h->hdr()->attached.load(std::memory_order_acquire) < nranks) {
        if (since(t0) > limit) {
            ok = false;
            break;
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    if (rank == 0 || !ok) (void)shm_unlink(h->name);  // the mapping stays; the name goes
    if (!ok) {
        munmap(h->map, h->bytes);
        delete h;
        return DFS_E_COMM;
    }
    *out = h;
    return DFS_OK;
}

void host_comm_close(HostComm* h) {
    if (!h) return;
    if (h->map) munmap(h->map, h->bytes);
    delete h;
}

// Progress every op of this rank until all are done.  Ops to / from one peer
// advance in posting order (only the first unfinished one of each direction
// moves); a chunk goes out when the mailbox is empty and comes in when it is
// full, so no rank ever blocks on one peer while another waits for it.
int host_comm_exchange(HostComm* h, std::vector<HostOp>& ops) {
    std::vector<uint64_t> done(ops.size(), 0);
    size_t left = 0;
    for (const HostOp& o : ops) {
        if (o.peer >= h->W || o.peer == h->me) return DFS_E_ARG;
        left += o.len != 0;
    }
    auto t_last = Clock::now();
    const double limit = timeout_s();
    while (left) {
        bool moved = false;
        // first unfinished op per (peer, direction)
        std::vector<uint8_t> busy(2 * static_cast<size_t>(h->W), 0);
        for (size_t i = 0; i < ops.size(); ++i) {
            HostOp& o = ops[i];
            if (done[i] == o.len) continue;
            uint8_t& b = busy[2 * o.peer + (o.send ? 1 : 0)];
            if (b) continue;
            b = 1;
            Box* bx = o.send ? h->box(h->me, o.peer) : h->box(o.peer, h->me);
            if (o.send) {
                const uint64_t wr = bx->wr.load(std::memory_order_relaxed);
                if (wr != bx->rd.load(std::memory_order_acquire)) continue;  // not consumed yet
                const uint64_t n = std::min(kSlot, o.len - done[i]);
                const uint8_t* src = static_cast<const uint8_t*>(o.p) + done[i];
                if (o.device) {
                    if (hipMemcpy(bx->data, src, n, hipMemcpyDeviceToHost) != hipSuccess) return DFS_E_HIP;
                } else {
                    std::memcpy(bx->data, src, n);
                }
                bx->len = n;
                bx->wr.store(wr + 1, std::memory_order_release);
                done[i] += n;
            } else {
                const uint64_t rd = bx->rd.load(std::memory_order_relaxed);
                if (bx->wr.load(std::memory_order_acquire) == rd) continue;  // nothing there yet
                const uint64_t n = bx->len;
                if (n > o.len - done[i]) return DFS_E_COMM;  // the two sides disagree on a size
                uint8_t* dst = static_cast<uint8_t*>(o.p) + done[i];
                if (o.device) {
                    if (hipMemcpy(dst, bx->data, n, hipMemcpyHostToDevice) != hipSuccess) return DFS_E_HIP;
                } else {
                    std::memcpy(dst, bx->data, n);
                }
                bx->rd.store(rd + 1, std::memory_order_release);
                done[i] += n;
            }
            moved = true;
            if (done[i] == o.len) --left;
        }
        if (moved) {
            t_last = Clock::now();
        } else {
            if (since(t_last) > limit) return DFS_E_COMM;  // a peer is gone
            std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
    }
    return DFS_OK;
}

}  // namespace dfs
