// placement_internal.h — the transfer schedule and its runner, shared by
// placement.cpp (RCCL placement / degraded fetch) and replica.cpp (the
// digest-table exchange of the replica receiver's verify).  Not part of the
// public boundary.
#pragma once
#include <stdint.h>

#include <vector>

#include "../../include/dfs_gpu.h"

namespace dfs {

constexpr uint32_t kMaxFrag = 64;
constexpr uint32_t kMaxRanks = 64;  // offline masks are 64-bit

// Node k is hosted by rank k mod W; fragment f lives on node f and node f-1
// (SN:143-145, 427-428).
inline uint32_t holder_a(uint32_t f, uint32_t, uint32_t W) { return f % W; }
inline uint32_t holder_b(uint32_t f, uint32_t N, uint32_t W) { return ((f + N - 1) % N) % W; }
inline bool holds(uint32_t g, uint32_t f, uint32_t N, uint32_t W) {
    return holder_a(f, N, W) == g || holder_b(f, N, W) == g;
}

struct Plan {
    std::vector<dfs_xfer> ops;
    std::vector<uint64_t> dst_off;  // nfrag + 1
    std::vector<int32_t> status;    // nfrag
    uint32_t phases = 0;
};

int build_plan(uint32_t W, uint32_t me, uint32_t N, const uint64_t* table, uint32_t mode, uint64_t offline, Plan& p);

// What the runner needs from the wire.  `i` is the local endpoint (index
// into the plans run together: the comms of one process, or every rank in
// the in-process simulator).  Sends and receives are posted between
// group_start and group_end and complete after group_end; between two
// endpoints they pair in posting order (RCCL's rule).
struct Transport {
    virtual ~Transport() {}
    virtual int copy(uint32_t i, void* dst, const void* src, uint64_t n) = 0;
    virtual int group_start() = 0;
    virtual int send(uint32_t i, const void* p, uint64_t n, int32_t peer) = 0;
    virtual int recv(uint32_t i, void* p, uint64_t n, int32_t peer) = 0;
    virtual int group_end() = 0;
    // Rank of endpoint i if its local copies are to travel as a send to itself
    // paired with a receive from itself inside the phase's group, else -1.
    virtual int32_t self_peer(uint32_t) const { return -1; }
};

// Issue every plan's ops phase by phase: local copies, then one group with
// the phase's sends and receives of every endpoint, in plan order.  On an
// endpoint with a self_peer the copies are posted in the group as well, as
// send + receive pairs to itself.
int run_plans(Transport& t, const std::vector<Plan>& plans, const void* const* src, void* const* dst);

// RCCL transport over `comms` (every op on its comm's ctx stream).
struct RcclTransport;
int run_plans_rccl(dfs_comm* const* comms, uint32_t ncomms, const std::vector<Plan>& plans, const void* const* src,
                   void* const* dst);
int check_comms(dfs_comm* const* comms, uint32_t ncomms);
// uint32 sum all-reduce in place over the comms (count words each).
int allreduce_u32(dfs_comm* const* comms, uint32_t ncomms, uint32_t* const* d_buf, uint32_t count);
// All-gather `count` uint64 words per rank (host in, host out: nranks*count), synchronous.
int allgather_u64(dfs_comm* const* comms, uint32_t ncomms, const uint64_t* const* mine, uint64_t count,
                  uint64_t* const* all);
dfs_ctx* comm_ctx(const dfs_comm* c);

// Host-staged communicator (hostcomm.cpp): the ranks are processes of one
// host and bytes cross through shared-memory mailboxes, so several ranks can
// share one GPU.  Chosen by the unique id (host_comm_is_id).
struct HostComm;
struct HostOp {
    bool send;
    void* p;        // device (hipMemcpy) or host memory
    uint64_t len;
    uint32_t peer;
    bool device;
};
bool host_comm_is_id(const uint8_t* id);
int host_comm_make_id(uint8_t* id);
int host_comm_open(const uint8_t* id, uint32_t nranks, uint32_t rank, HostComm** out);
void host_comm_close(HostComm* h);
// Run this rank's sends and receives to completion (synchronous).
int host_comm_exchange(HostComm* h, std::vector<HostOp>& ops);

}  // namespace dfs
