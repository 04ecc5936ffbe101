// sha256.hip — multi-message SHA-256 for gfx950 (MI355X).
//
// Replaces MessageDigest.getInstance("SHA-256").digest(...) at every
// sha256Hex call site of StorageNode.java (SN:127 fileId, SN:159 fragment,
// SN:282 received fragment, SN:454 download verify).  FIPS 180-4.
//
// Design:
//  * One message per lane.  SHA-256 is a strict chain within a message, so
//    the parallelism is across messages (files' fragments and fileIds).
//  * Lanes are pre-sorted by length (longest first) on the host so waves are
//    uniform; the waves that carry the longest chains (fileIds) raise their
//    issue priority (s_setprio) because they are the critical path.
//  * Int-VALU bound: 64 rounds are fully unrolled; rotations are
//    v_alignbit_b32, the three-input XORs / Ch / Maj are single
//    v_bitop3_b32 ops (gfx950), additions fold into v_add3_u32.
//  * Arbitrary byte offsets (fragment starts are not aligned): each lane
//    loads 16 aligned dwords + 1 look-ahead dword per block and one
//    v_perm_b32 per word does the funnel shift and the big-endian swap.
//  * The next block is prefetched into a second register set while the
//    current one is compressed (two register buffers, loop unrolled x2).
#include "dfs_internal.h"

namespace dfs {
namespace {

__device__ __forceinline__ uint32_t rotr(uint32_t x, uint32_t n) { return __builtin_amdgcn_alignbit(x, x, n); }
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t bsig0(uint32_t a) { return xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22)); }
__device__ __forceinline__ uint32_t bsig1(uint32_t e) { return xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25)); }
__device__ __forceinline__ uint32_t ssig0(uint32_t x) { return xor3(rotr(x, 7), rotr(x, 18), x >> 3); }
__device__ __forceinline__ uint32_t ssig1(uint32_t x) { return xor3(rotr(x, 17), rotr(x, 19), x >> 10); }
// Ch(e,f,g) = e ? f : g  (truth table 0xCA);  Maj(a,b,c) (0xE8).
__device__ __forceinline__ uint32_t ch(uint32_t e, uint32_t f, uint32_t g) {
    return __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);
}
__device__ __forceinline__ uint32_t maj(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
}

constexpr uint32_t kK[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

// FIPS 180-4 §6.2.2 compression of one 64-byte block W (big-endian words).
// The empty volatile asm statements are ordering points (they emit nothing):
// each schedule word W[t] (t >= 16) is pinned to round t, so the compiler
// cannot hoist the whole 48-word message expansion ahead of the rounds
// (which costs ~30 VGPRs and drops occupancy from 6 to 4 waves/SIMD).
__device__ __forceinline__ void compress(uint32_t (&st)[8], uint32_t (&W)[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
    for (int t = 0; t < 64; ++t) {
        if (t >= 16) {
            W[t & 15] += ssig1(W[(t - 2) & 15]) + W[(t - 7) & 15] + ssig0(W[(t - 15) & 15]);
            asm volatile("" : "+v"(W[t & 15]));
        }
        const uint32_t t1 = h + bsig1(e) + ch(e, f, g) + kK[t] + W[t & 15];
        const uint32_t t2 = bsig0(a) + maj(a, b, c);
        h = g; g = f; f = e; e = d + t1;
        d = c; c = b; b = a; a = t1 + t2;
        asm volatile("" : "+v"(a), "+v"(e));
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
    st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// 16 words of block k plus the look-ahead word (first word of block k+1),
// which the unaligned funnel needs for the block's last word.
__device__ __forceinline__ void load_block(const uint32_t* __restrict__ p, uint32_t sh, uint32_t (&r)[16],
                                           uint32_t& x) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint4 v = q[i];
        r[4 * i + 0] = v.x; r[4 * i + 1] = v.y; r[4 * i + 2] = v.z; r[4 * i + 3] = v.w;
    }
    // Always 5 loads, no branch (a conditional load makes hipcc's counted
    // s_waitcnt wait for the fresh prefetch).  For sh == 0 the look-ahead
    // word is not needed and p[16] may lie past the message: re-read p[15].
    x = p[sh ? 16 : 15];
}

// In place: r[j] <- big-endian word at byte offset sh of {r[j], r[j+1]}.
__device__ __forceinline__ void to_be(uint32_t (&r)[16], uint32_t x, uint32_t sel) {
#pragma unroll
    for (int j = 0; j < 15; ++j) r[j] = __builtin_amdgcn_perm(r[j + 1], r[j], sel);
    r[15] = __builtin_amdgcn_perm(x, r[15], sel);
}

// Per-lane message geometry.
struct Msg {
    const uint32_t* p;  // dword-aligned pointer at or below the first byte
    uint64_t len;       // bytes of this part
    uint64_t total;     // whole-message length (padding bit count)
    uint32_t sh, sel, nfull, ntb, out, flags;
};

__device__ __forceinline__ Msg msg_setup(const uint8_t* __restrict__ base, const ShaDesc& d) {
    Msg m;
    m.sh = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(base + d.off)) & 3u;
    m.p = reinterpret_cast<const uint32_t*>(base + d.off - m.sh);
    m.sel = (m.sh + 3u) | ((m.sh + 2u) << 8) | ((m.sh + 1u) << 16) | (m.sh << 24);
    m.len = d.len;
    m.total = d.total;
    m.nfull = static_cast<uint32_t>(d.len >> 6);
    m.ntb = (static_cast<uint32_t>(d.len) & 63u) < 56u ? 1u : 2u;
    m.out = d.out;
    m.flags = d.flags;
    return m;
}

// Tail block tb (0 or 1) of a message: the last len mod 64 bytes, the 0x80
// pad byte, zeros and (in the final block) the 64-bit big-endian bit length
// (FIPS 180-4 §5.1.1).  Loads are guarded: a dword is read only if it holds
// at least one message byte.
__device__ __forceinline__ void tail_block(const Msg& m, uint32_t tb, uint32_t (&W)[16]) {
    const uint32_t r = static_cast<uint32_t>(m.len) & 63u;
    const uint32_t lim = m.len ? m.sh + r : 0u;  // tail word i holds message bytes iff 4i < lim
    const uint32_t* __restrict__ q = m.p + 16u * m.nfull;
    uint32_t T[17];
#pragma unroll
    for (int i = 0; i < 17; ++i) {
        const uint32_t wi = 16u * tb + static_cast<uint32_t>(i);
        T[i] = (4u * wi < lim) ? q[wi] : 0u;
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int rem = static_cast<int>(r) - 64 * static_cast<int>(tb) - 4 * j;  // message bytes in word j
        const uint32_t w = __builtin_amdgcn_perm(T[j + 1], T[j], m.sel);
        const uint32_t mask = rem >= 4 ? 0xffffffffu : (rem <= 0 ? 0u : (0xffffffffu << (32 - 8 * rem)));
        const uint32_t pad = (rem >= 0 && rem < 4) ? (0x80000000u >> (8 * rem)) : 0u;
        W[j] = (w & mask) | pad;
    }
    if (tb + 1u == m.ntb) {
        const uint64_t bits = m.total << 3;
        W[14] = static_cast<uint32_t>(bits >> 32);
        W[15] = static_cast<uint32_t>(bits);
    }
}

__device__ __forceinline__ void store_digest(const uint32_t (&st)[8], uint32_t out, uint32_t split,
                                             uint8_t* __restrict__ out0, uint8_t* __restrict__ out1) {
    uint8_t* dst = out < split ? out0 + 32ull * out : out1 + 32ull * (out - split);
    uint4* o = reinterpret_cast<uint4*>(dst);
    o[0] = make_uint4(__builtin_bswap32(st[0]), __builtin_bswap32(st[1]), __builtin_bswap32(st[2]),
                      __builtin_bswap32(st[3]));
    o[1] = make_uint4(__builtin_bswap32(st[4]), __builtin_bswap32(st[5]), __builtin_bswap32(st[6]),
                      __builtin_bswap32(st[7]));
}

__device__ __forceinline__ void init_state(uint32_t (&st)[8]) {
    st[0] = 0x6a09e667u; st[1] = 0xbb67ae85u; st[2] = 0x3c6ef372u; st[3] = 0xa54ff53au;
    st[4] = 0x510e527fu; st[5] = 0x9b05688cu; st[6] = 0x1f83d9abu; st[7] = 0x5be0cd19u;
}

__device__ __forceinline__ uint32_t hw_id() {
    uint32_t v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(v));
    return v;
}
__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return v;
}

// 13-bit id of the SIMD this wave runs on: XCC, SE, SH, CU, SIMD fields of
// HW_REG_XCC_ID / HW_REG_HW_ID (gfx9 layout).  Used only to balance work
// (speed), never for correctness.
__device__ __forceinline__ uint32_t simd_key() {
    const uint32_t hw = hw_id();
    return ((xcc_id() & 7u) << 10) | (((hw >> 13) & 7u) << 7) | (((hw >> 12) & 1u) << 6) |
           (((hw >> 8) & 15u) << 2) | ((hw >> 4) & 3u);
}

// Persistent: each wave pulls 64-message items (item i = sorted lanes
// [64i, 64i+64)) from two atomic queues.  Items [0, n_long) carry the long
// chains (fileIds): a wave may take one only while its SIMD holds fewer than
// `cap` of them (per-SIMD token counters), so every SIMD runs one long chain
// at full single-wave issue rate and the short items (fragments) fill the
// remaining issue slots dynamically.  The grid holds a fixed number of waves
// per SIMD, leaving the other wave slots to the Base64 kernel beside it.
// queue[0] = long counter, queue[1] = short counter, queue[64 + key] = SIMD
// token counters; all zeroed by the launcher before each launch.
__global__ __launch_bounds__(kShaBlock) void sha256_lanes(const uint8_t* __restrict__ base,
                                                          const ShaDesc* __restrict__ descs, uint32_t n,
                                                          uint32_t split, uint32_t n_long, uint32_t cap,
                                                          uint8_t* __restrict__ out0, uint8_t* __restrict__ out1,
                                                          uint32_t* __restrict__ queue,
                                                          uint32_t* __restrict__ census,
                                                          uint32_t* __restrict__ state, uint32_t rot) {
    const uint32_t nitems = (n + 63u) >> 6;
    const uint32_t n_short = nitems - n_long;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t key = simd_key();
    for (;;) {
        uint32_t item = 0xffffffffu;
        if (lane == 0) {
            if (n_long && __hip_atomic_load(queue, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < n_long &&
                atomicAdd(queue + 64 + key, 1u) < cap) {
                const uint32_t it = atomicAdd(queue, 1u);
                if (it < n_long) item = it;
            }
            if (item == 0xffffffffu) {
                const uint32_t it = atomicAdd(queue + 1, 1u);
                if (it < n_short) {
                    item = n_long + it;
                } else if (n_long) {  // long items a starved SIMD left behind
                    const uint32_t it2 = atomicAdd(queue, 1u);
                    if (it2 < n_long) item = it2;
                }
            }
        }
        item = __builtin_amdgcn_readfirstlane(item);
        if (item == 0xffffffffu) break;
        if (item < n_long) __builtin_amdgcn_s_setprio(2);
        else __builtin_amdgcn_s_setprio(0);
        uint64_t t_start = 0;
        if (census) t_start = __builtin_amdgcn_s_memrealtime();
        const uint32_t gid = item * 64u + lane;
        if (gid < n) {
            const Msg m = msg_setup(base, descs[gid]);
            uint32_t st[8];
            if (m.flags & kShaResume) {
                const uint4* s4 = reinterpret_cast<const uint4*>(state + 8ull * m.out);
                const uint4 s0 = s4[0], s1 = s4[1];
                st[0] = s0.x; st[1] = s0.y; st[2] = s0.z; st[3] = s0.w;
                st[4] = s1.x; st[5] = s1.y; st[6] = s1.z; st[7] = s1.w;
            } else {
                init_state(st);
            }
            // Short items rotate their issue priority (0/1, flipped every
            // two blocks): the SIMD arbiter breaks priority ties by wave
            // age, so without this the oldest short wave of a SIMD runs
            // ~2x faster than the youngest and the SIMD ends the kernel
            // with one wave left (tools/census.py).  Flipping on progress
            // is self-balancing: a wave that ran ahead spends less time at
            // the higher priority.
            const bool flip = rot && item >= n_long;
            if (m.nfull) {
                uint32_t A[16], B[16], xa, xb;
                load_block(m.p, m.sh, A, xa);
                uint32_t k = 0;
                for (;;) {
                    // A holds block k; prefetch block k+1 (clamped) into B.
                    load_block(m.p + 16u * min(k + 1u, m.nfull - 1u), m.sh, B, xb);
                    to_be(A, xa, m.sel);
                    compress(st, A);
                    if (++k >= m.nfull) break;
                    load_block(m.p + 16u * min(k + 1u, m.nfull - 1u), m.sh, A, xa);
                    to_be(B, xb, m.sel);
                    compress(st, B);
                    if (++k >= m.nfull) break;
                    if (flip) {
                        if (k & 2u) __builtin_amdgcn_s_setprio(1);
                        else __builtin_amdgcn_s_setprio(0);
                    }
                }
            }
            if (m.flags & kShaPartial) {  // message continues in a later launch
                uint4* s4 = reinterpret_cast<uint4*>(state + 8ull * m.out);
                s4[0] = make_uint4(st[0], st[1], st[2], st[3]);
                s4[1] = make_uint4(st[4], st[5], st[6], st[7]);
            } else {
                for (uint32_t tb = 0; tb < m.ntb; ++tb) {
                    uint32_t W[16];
                    tail_block(m, tb, W);
                    compress(st, W);
                }
                store_digest(st, m.out, split, out0, out1);
            }
        }
        if (census && lane == 0u) {
            const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
            uint32_t* c = census + 4ull * item;
            c[0] = hw_id();
            c[1] = xcc_id();
            c[2] = static_cast<uint32_t>(t_start);
            c[3] = static_cast<uint32_t>(t_end);
        }
    }
}

// Lane sequences: lane l hashes messages seq[l] .. seq[l+1]-1 one after the
// other, one 64-byte block per loop iteration, with a single compress body.
// The upload plan pairs, in one wave, the fileId lane of file f (lanes
// 0..31) with a lane that hashes f's N fragments in order (lanes 32..63):
// at every iteration both lanes read within 64 bytes of each other in the
// file, so the second read hits the line the first one brought in (the file
// crosses HBM once for both chains), and every wave runs the same
// ceil((S+9)/64)-ish iterations.  Messages switch at per-lane tail blocks
// (rare, exec-masked branches).
__device__ __forceinline__ void sha256_seq_lane(const uint8_t* __restrict__ base, const ShaDesc* __restrict__ descs,
                                                const uint32_t* __restrict__ seq, uint32_t l, uint32_t split,
                                                uint8_t* __restrict__ out0, uint8_t* __restrict__ out1);

__global__ __launch_bounds__(kShaBlock) void sha256_seq(const uint8_t* __restrict__ base,
                                                        const ShaDesc* __restrict__ descs,
                                                        const uint32_t* __restrict__ seq, uint32_t nlanes,
                                                        uint32_t split, uint8_t* __restrict__ out0,
                                                        uint8_t* __restrict__ out1, uint32_t* __restrict__ census) {
    const uint32_t l = blockIdx.x * kShaBlock + threadIdx.x;
    const uint64_t t_start = census ? __builtin_amdgcn_s_memrealtime() : 0;
    if (l < nlanes) sha256_seq_lane(base, descs, seq, l, split, out0, out1);
    if (census && (threadIdx.x & 63u) == 0u) {
        const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
        uint32_t* c = census + 4ull * (l >> 6);
        c[0] = hw_id();
        c[1] = xcc_id();
        c[2] = static_cast<uint32_t>(t_start);
        c[3] = static_cast<uint32_t>(t_end);
    }
}

__device__ __forceinline__ void sha256_seq_lane(const uint8_t* __restrict__ base, const ShaDesc* __restrict__ descs,
                                                const uint32_t* __restrict__ seq, uint32_t l, uint32_t split,
                                                uint8_t* __restrict__ out0, uint8_t* __restrict__ out1) {
    uint32_t mi = seq[l];
    const uint32_t mend = seq[l + 1];
    if (mi >= mend) return;
    Msg m = msg_setup(base, descs[mi]);
    uint32_t st[8];
    init_state(st);
    uint32_t A[16], B[16], xa = 0, xb = 0;
    if (m.nfull) load_block(m.p, m.sh, A, xa);
    uint32_t k = 0;
    // Two register buffers in ping-pong (the loop body is written twice so no
    // register copy ever waits on the prefetch): CUR holds block k, NXT
    // receives block k+1 (or block 0 of the lane's next message).
#define DFS_SHA_SEQ_STEP(CUR, XC, NXT, XN)                                              \
    {                                                                                   \
        uint32_t W[16];                                                                 \
        if (k < m.nfull) {                                                              \
            load_block(m.p + 16u * min(k + 1u, m.nfull - 1u), m.sh, NXT, XN);           \
            _Pragma("unroll") for (int i = 0; i < 16; ++i) W[i] = CUR[i];               \
            to_be(W, XC, m.sel);                                                        \
        } else {                                                                        \
            tail_block(m, k - m.nfull, W);                                              \
        }                                                                               \
        compress(st, W);                                                                \
        if (++k == m.nfull + m.ntb) { /* message done: publish, start the next one */  \
            store_digest(st, m.out, split, out0, out1);                                 \
            if (++mi >= mend) break;                                                    \
            m = msg_setup(base, descs[mi]);                                             \
            init_state(st);                                                             \
            k = 0;                                                                      \
            if (m.nfull) load_block(m.p, m.sh, NXT, XN);                                \
        }                                                                               \
    }
    for (;;) {
        DFS_SHA_SEQ_STEP(A, xa, B, xb)
        DFS_SHA_SEQ_STEP(B, xb, A, xa)
    }
#undef DFS_SHA_SEQ_STEP
}

}  // namespace

hipError_t launch_sha256_seq(const uint8_t* base, const ShaDesc* descs, const uint32_t* seq, uint32_t nlanes,
                             uint32_t split, uint8_t* out0, uint8_t* out1, uint32_t* census, hipStream_t s) {
    if (nlanes == 0) return hipSuccess;
    const uint32_t grid = (nlanes + kShaBlock - 1) / kShaBlock;
    hipLaunchKernelGGL(sha256_seq, dim3(grid), dim3(kShaBlock), 0, s, base, descs, seq, nlanes, split, out0, out1,
                       census);
    return hipGetLastError();
}

hipError_t launch_sha256(const uint8_t* base, const ShaDesc* descs, uint32_t n, uint32_t split,
                         uint32_t prio_lanes, uint8_t* out0, uint8_t* out1, uint32_t* queue, int waves_per_simd,
                         uint32_t* census, hipStream_t s, uint32_t* state, uint32_t rot) {
    if (n == 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(queue, 0, kShaQueueBytes, s);
    if (e != hipSuccess) return e;
    const uint32_t n_long = (prio_lanes + 63u) / 64u;
    const uint32_t cap = (n_long + 1023u) / 1024u;
    const uint64_t items = (n + 63u) / 64u;
    uint64_t waves = 1024ull * static_cast<uint64_t>(waves_per_simd < 1 ? 1 : waves_per_simd);
    if (waves > items) waves = items;
    const uint32_t grid = static_cast<uint32_t>((waves + 3) / 4);
    hipLaunchKernelGGL(sha256_lanes, dim3(grid), dim3(kShaBlock), 0, s, base, descs, n, split, n_long, cap, out0,
                       out1, queue, census, state, rot);
    return hipGetLastError();
}

}  // namespace dfs
