// stream_common.h — tile walker shared by the HBM-bound stream kernels
// (Base64 encode/decode, gather, synth).
//
// Work is cut into tiles; each job (message) owns a contiguous tile range
// [tile_start, next.tile_start).  Workgroup b walks the contiguous tile
// range [b*T/G, (b+1)*T/G), finding its first job by a binary search over
// the (host-built) job table and then stepping forward, so neighbouring
// tiles of one message stay on one workgroup (and one XCD's L2).
#pragma once
#include "dfs_internal.h"

namespace dfs {

// Index of the job owning tile t: largest j with jobs[j].tile_start <= t.
// `jobs` has njobs entries plus a sentinel.  Wave-uniform inputs, so the
// compiler keeps it on the scalar unit.
__device__ __forceinline__ uint32_t find_job(const StreamJob* __restrict__ jobs, uint32_t njobs, uint64_t t) {
    uint32_t lo = 0, hi = njobs;  // invariant: jobs[lo].tile_start <= t < jobs[hi].tile_start
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (jobs[mid].tile_start <= t) lo = mid; else hi = mid;
    }
    return lo;
}

__device__ __forceinline__ void tile_range(uint64_t ntiles, uint64_t& t0, uint64_t& t1) {
    const uint64_t g = gridDim.x, b = blockIdx.x;
    t0 = ntiles * b / g;
    t1 = ntiles * (b + 1) / g;
}

// Grid size for a tile count: wgs_per_cu workgroups (4 waves each) on each of
// the 256 CUs, never more than the tiles.  The encode kernel that runs beside
// the SHA kernel leaves 2 waves/SIMD free for it (wgs_per_cu = 6).
inline uint32_t stream_grid(uint64_t ntiles, uint32_t wgs_per_cu = 8) {
    const uint64_t cap = 256ull * wgs_per_cu;
    return static_cast<uint32_t>(ntiles < cap ? (ntiles ? ntiles : 1) : cap);
}

}  // namespace dfs
