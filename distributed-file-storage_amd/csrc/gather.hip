// gather.hip — reassembly gather and synthetic data.
//
// gather_kernel replaces handleDownload's ordered reassembly
// (ByteArrayOutputStream.write at StorageNode.java:448, toByteArray at :451):
// fragment i of file f is copied to file_off[f] + off_i (the split offsets
// of :138-157).  HBM-bound: every destination byte is written once, by
// 16-byte aligned stores; misaligned sources are funnel-shifted in registers.
#include "stream_common.h"

namespace dfs {
namespace {

// Tile = P x 256 16-byte output chunks (P = 4): chunk c of a fragment
// covers dst bytes [h + 16c, h + 16c + 16), a 16-byte aligned span (h = bytes
// up to the first 16-aligned address, copy_items in dfs_gpu.cpp).  Every lane
// issues the loads of all its chunks (dwordx4 + one dword when the source is
// not dword-aligned relative to the destination) before any store; a wave
// reads and writes 1 KiB contiguous per instruction.  One lane per fragment
// copies the head and tail bytes.  Loads and stores are non-temporal: every
// byte is touched once.
typedef uint32_t g32x4 __attribute__((ext_vector_type(4)));

constexpr int P = kGatherPer;  // 16-byte chunks per thread per tile

// Tiles [t0, t1) of the job table.
__device__ __forceinline__ void gather_range(const StreamJob* __restrict__ jobs, uint32_t njobs,
                                             uint8_t* __restrict__ out, uint64_t t0, uint64_t t1) {
    if (t0 >= t1) return;
    uint32_t j = find_job(jobs, njobs, t0);
    for (uint64_t t = t0; t < t1; ++t) {
        while (jobs[j + 1].tile_start <= t) ++j;
        const uint64_t len = jobs[j].len;
        const uint8_t* __restrict__ src = reinterpret_cast<const uint8_t*>(jobs[j].src_off);
        uint8_t* __restrict__ dst = out + jobs[j].dst_off;
        const uint32_t h = static_cast<uint32_t>((16u - (reinterpret_cast<uintptr_t>(dst) & 15u)) & 15u);
        const uint64_t nc = len > h ? (len - h) / 16 : 0;
        const uint32_t sa = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(src + h)) & 3u;
        const uint32_t* w0 = reinterpret_cast<const uint32_t*>(src + h - sa);
        const uint64_t c0 = (t - jobs[j].tile_start) * (P * kStreamBlock) + threadIdx.x;
        g32x4 v[P];
        uint32_t x[P];
#pragma unroll
        for (int i = 0; i < P; ++i) {
            const uint64_t c = c0 + static_cast<uint64_t>(i) * kStreamBlock;
            v[i] = g32x4{0u, 0u, 0u, 0u};
            x[i] = 0u;
            if (c < nc) {
                v[i] = __builtin_nontemporal_load(reinterpret_cast<const g32x4*>(w0 + 4 * c));
                if (sa) x[i] = __builtin_nontemporal_load(w0 + 4 * c + 4);
            }
        }
#pragma unroll
        for (int i = 0; i < P; ++i) {
            const uint64_t c = c0 + static_cast<uint64_t>(i) * kStreamBlock;
            if (c < nc) {
                g32x4 o = v[i];
                if (sa) {
                    o.x = __builtin_amdgcn_alignbyte(v[i].y, v[i].x, sa);
                    o.y = __builtin_amdgcn_alignbyte(v[i].z, v[i].y, sa);
                    o.z = __builtin_amdgcn_alignbyte(v[i].w, v[i].z, sa);
                    o.w = __builtin_amdgcn_alignbyte(x[i], v[i].w, sa);
                }
                __builtin_nontemporal_store(o, reinterpret_cast<g32x4*>(dst + h + 16 * c));
            } else if (c == nc) {
                const uint64_t head_end = h < len ? h : len;
                for (uint64_t b = 0; b < head_end; ++b) dst[b] = src[b];
                for (uint64_t b = h + 16 * nc; b < len; ++b) dst[b] = src[b];
            }
        }
    }
}

// AHEAD (dfs_reassemble_verify, overlap mode): fragment groups in order, each
// published to the SHA kernel beside it (StreamAhead, dfs_internal.h).
template <bool AHEAD>
__global__ __launch_bounds__(kStreamBlock) void gather_kernel(const StreamJob* __restrict__ jobs, uint32_t njobs,
                                                              uint64_t ntiles, uint8_t* __restrict__ out,
                                                              const uint64_t* __restrict__ gtile, uint32_t ngroups,
                                                              uint32_t* __restrict__ gdone) {
    if (!AHEAD) {
        uint64_t t0, t1;
        tile_range(ntiles, t0, t1);
        gather_range(jobs, njobs, out, t0, t1);
        return;
    }
    const uint64_t G = gridDim.x, b = blockIdx.x;
    for (uint32_t g = 0; g < ngroups; ++g) {
        const uint64_t a = gtile[g], n = gtile[g + 1] - a;
        gather_range(jobs, njobs, out, a + n * b / G, a + n * (b + 1) / G);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_fetch_add(gdone + g, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Per-file verdict of a download whose expected digests live on the device:
// 1 = a fragment's Base64 was rejected (SN:281), 2 = a fragment digest differs
// from the sender's (SN:250-257), 3 = the rebuilt file's digest differs from
// its fileId (SN:454-458), 0 = good.  One thread per file; the host maps the
// codes and keeps its own statuses (missing fragments) first.
__global__ __launch_bounds__(256) void verdict_kernel(const int32_t* __restrict__ dec_status,
                                                      const uint8_t* __restrict__ frag_dig,
                                                      const uint8_t* __restrict__ file_dig,
                                                      const uint8_t* __restrict__ exp_frag,
                                                      const uint8_t* __restrict__ exp_file, uint32_t nfiles,
                                                      uint32_t nfrag, int32_t* __restrict__ verdict) {
    const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= nfiles) return;
    int32_t v = 0;
    for (uint32_t i = 0; i < nfrag && !v; ++i)
        if (dec_status[static_cast<uint64_t>(f) * nfrag + i]) v = 1;
    for (uint32_t i = 0; i < nfrag && !v && exp_frag; ++i) {
        const uint64_t k = static_cast<uint64_t>(f) * nfrag + i;
        for (uint32_t b = 0; b < 32; ++b)
            if (frag_dig[32 * k + b] != exp_frag[32 * k + b]) v = 2;
    }
    if (!v && exp_file)
        for (uint32_t b = 0; b < 32; ++b)
            if (file_dig[32ull * f + b] != exp_file[32ull * f + b]) v = 3;
    verdict[f] = v;
}

__global__ __launch_bounds__(256) void fill_u32_kernel(uint32_t* __restrict__ p, uint64_t n, uint32_t v) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256u + threadIdx.x;
    if (i < n) p[i] = v;
}

// Fragment digests [file][frag] -> [frag][file] (32 bytes each, as two
// dwordx4): the order in which a rank's digests travel to the holders, group
// f = fragment f of every file, like its Base64.
__global__ __launch_bounds__(256) void digest_transpose_kernel(const uint4* __restrict__ in, uint4* __restrict__ out,
                                                               uint32_t nfiles, uint32_t nfrag) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256u + threadIdx.x;  // half-digest index in `out`
    if (i >= 2ull * nfiles * nfrag) return;
    const uint64_t k = i >> 1;
    const uint32_t f = static_cast<uint32_t>(k / nfiles), j = static_cast<uint32_t>(k % nfiles);
    out[i] = in[2ull * (static_cast<uint64_t>(j) * nfrag + f) + (i & 1u)];
}

// The sender's check of a replica receiver's hashes (SN:248-257), held
// fragment by held fragment, plus the failures per uploader.
__global__ __launch_bounds__(256) void replica_verdict_kernel(const int32_t* __restrict__ status,
                                                              const uint4* __restrict__ got,
                                                              const uint4* __restrict__ expected, uint64_t n,
                                                              const uint64_t* __restrict__ piece_start,
                                                              const uint32_t* __restrict__ piece_rank, uint32_t npieces,
                                                              int32_t code_decode, int32_t code_mismatch,
                                                              int32_t* __restrict__ verdict,
                                                              uint32_t* __restrict__ failed) {
    const uint64_t k = static_cast<uint64_t>(blockIdx.x) * 256u + threadIdx.x;
    if (k >= n) return;
    const int32_t st = status[k];
    int32_t v = 0;
    if (st & 1) {
        v = code_decode;
    } else {
        const uint4 a0 = got[2 * k], a1 = got[2 * k + 1], b0 = expected[2 * k], b1 = expected[2 * k + 1];
        const bool same = a0.x == b0.x && a0.y == b0.y && a0.z == b0.z && a0.w == b0.w && a1.x == b1.x &&
                          a1.y == b1.y && a1.z == b1.z && a1.w == b1.w;
        if ((st & 2) || !same) v = code_mismatch;
    }
    if (verdict) verdict[k] = v;
    if (v) {
        uint32_t lo = 0, hi = npieces;  // piece_start[lo] <= k < piece_start[hi]
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (piece_start[mid] <= k) lo = mid;
            else hi = mid;
        }
        atomicAdd(failed + piece_rank[lo], 1u);
    }
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// Synthetic files: job.src_off = file index, job.len = bytes, job.dst_off.
// Item c covers file bytes [64c, 64c+64).
__global__ __launch_bounds__(kStreamBlock) void synth_kernel(uint8_t* __restrict__ dst_base,
                                                             const StreamJob* __restrict__ jobs, uint32_t njobs,
                                                             uint64_t ntiles, uint64_t seed, uint64_t file_off) {
    uint64_t t0, t1;
    tile_range(ntiles, t0, t1);
    if (t0 >= t1) return;
    uint32_t j = find_job(jobs, njobs, t0);
    for (uint64_t t = t0; t < t1; ++t) {
        while (jobs[j + 1].tile_start <= t) ++j;
        const uint64_t f = jobs[j].src_off, len = jobs[j].len;
        uint8_t* __restrict__ dst = dst_base + jobs[j].dst_off;
        const bool aligned = (reinterpret_cast<uintptr_t>(dst) & 7u) == 0;
        const uint64_t c = (t - jobs[j].tile_start) * kStreamBlock + threadIdx.x;
        const uint64_t b0 = 64 * c;
        if (b0 >= len) continue;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint64_t o = b0 + 8 * k;
            if (o >= len) break;
            const uint64_t v = splitmix64(seed ^ ((f << 40) | ((file_off + o) >> 3)));  // file_off % 8 == 0
            if (aligned && o + 8 <= len) {
                *reinterpret_cast<uint64_t*>(dst + o) = v;
            } else {
                for (uint64_t b = o; b < o + 8 && b < len; ++b) dst[b] = static_cast<uint8_t>(v >> (8 * (b & 7)));
            }
        }
    }
}

}  // namespace

hipError_t launch_download_verdict(const int32_t* dec_status, const uint8_t* frag_dig, const uint8_t* file_dig,
                                   const uint8_t* exp_frag, const uint8_t* exp_file, uint32_t nfiles, uint32_t nfrag,
                                   int32_t* verdict, hipStream_t s) {
    if (nfiles == 0) return hipSuccess;
    hipLaunchKernelGGL(verdict_kernel, dim3((nfiles + 255) / 256), dim3(256), 0, s, dec_status, frag_dig, file_dig,
                       exp_frag, exp_file, nfiles, nfrag, verdict);
    return hipGetLastError();
}

hipError_t launch_fill_u32(uint32_t* p, uint64_t n, uint32_t v, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(fill_u32_kernel, dim3(static_cast<uint32_t>((n + 255) / 256)), dim3(256), 0, s, p, n, v);
    return hipGetLastError();
}

hipError_t launch_digest_transpose(const uint8_t* in, uint8_t* out, uint32_t nfiles, uint32_t nfrag, hipStream_t s) {
    const uint64_t n = 2ull * nfiles * nfrag;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(digest_transpose_kernel, dim3(static_cast<uint32_t>((n + 255) / 256)), dim3(256), 0, s,
                       reinterpret_cast<const uint4*>(in), reinterpret_cast<uint4*>(out), nfiles, nfrag);
    return hipGetLastError();
}

hipError_t launch_replica_verdict(const int32_t* status, const uint8_t* got, const uint8_t* expected, uint64_t n,
                                  const uint64_t* piece_start, const uint32_t* piece_rank, uint32_t npieces,
                                  int32_t code_decode, int32_t code_mismatch, int32_t* verdict, uint32_t* failed,
                                  hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(replica_verdict_kernel, dim3(static_cast<uint32_t>((n + 255) / 256)), dim3(256), 0, s, status,
                       reinterpret_cast<const uint4*>(got), reinterpret_cast<const uint4*>(expected), n, piece_start,
                       piece_rank, npieces, code_decode, code_mismatch, verdict, failed);
    return hipGetLastError();
}

int gather_ahead_vgprs() {
    hipFuncAttributes a{};
    return hipFuncGetAttributes(&a, reinterpret_cast<const void*>(gather_kernel<true>)) == hipSuccess ? a.numRegs : -1;
}

hipError_t launch_gather(const StreamJob* jobs, uint32_t njobs, uint64_t ntiles, uint8_t* out, hipStream_t s,
                         const StreamAhead* ahead) {
    if (ahead) {
        hipLaunchKernelGGL(gather_kernel<true>, dim3(ahead->grid), dim3(kStreamBlock), 0, s, jobs, njobs, ntiles, out,
                           ahead->gtile, ahead->ngroups, ahead->gdone);
        return hipGetLastError();
    }
    if (ntiles == 0) return hipSuccess;
    hipLaunchKernelGGL(gather_kernel<false>, dim3(stream_grid(ntiles)), dim3(kStreamBlock), 0, s, jobs, njobs, ntiles,
                       out, nullptr, 0u, nullptr);
    return hipGetLastError();
}

hipError_t launch_synth(uint8_t* dst, const StreamJob* jobs, uint32_t njobs, uint64_t ntiles, uint64_t seed,
                        hipStream_t s, uint64_t file_off) {
    if (ntiles == 0) return hipSuccess;
    hipLaunchKernelGGL(synth_kernel, dim3(stream_grid(ntiles)), dim3(kStreamBlock), 0, s, dst, jobs, njobs, ntiles,
                       seed, file_off);
    return hipGetLastError();
}

}  // namespace dfs
