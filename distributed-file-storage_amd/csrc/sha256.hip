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
//  * Blocks are fetched in pairs (one 128-byte line for line-aligned
//    messages) and the next pair is in flight while the current pair is
//    compressed (four register buffers, loop unrolled x4).
#include <cstdlib>

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

// The same block W compressed into two independent states (a lane and its
// twin, kShaTwin): the message schedule W[16..63] and K[t] + W[t] are
// computed once, the two round chains interleave (2 x 14 ops per round +
// 10 per schedule word + 1: ~2,290 VALU ops for two blocks instead of 2,810).
__device__ __forceinline__ void compress2(uint32_t (&s1)[8], uint32_t (&s2)[8], uint32_t (&W)[16]) {
    uint32_t a = s1[0], b = s1[1], c = s1[2], d = s1[3], e = s1[4], f = s1[5], g = s1[6], h = s1[7];
    uint32_t a2 = s2[0], b2 = s2[1], c2 = s2[2], d2 = s2[3], e2 = s2[4], f2 = s2[5], g2 = s2[6], h2 = s2[7];
#pragma unroll
    for (int t = 0; t < 64; ++t) {
        if (t >= 16) {
            W[t & 15] += ssig1(W[(t - 2) & 15]) + W[(t - 7) & 15] + ssig0(W[(t - 15) & 15]);
            asm volatile("" : "+v"(W[t & 15]));
        }
        const uint32_t kw = kK[t] + W[t & 15];
        const uint32_t t1 = h + bsig1(e) + ch(e, f, g) + kw;
        const uint32_t t2 = bsig0(a) + maj(a, b, c);
        const uint32_t u1 = h2 + bsig1(e2) + ch(e2, f2, g2) + kw;
        const uint32_t u2 = bsig0(a2) + maj(a2, b2, c2);
        h = g; g = f; f = e; e = d + t1;
        d = c; c = b; b = a; a = t1 + t2;
        h2 = g2; g2 = f2; f2 = e2; e2 = d2 + u1;
        d2 = c2; c2 = b2; b2 = a2; a2 = u1 + u2;
        asm volatile("" : "+v"(a), "+v"(e), "+v"(a2), "+v"(e2));
    }
    s1[0] += a; s1[1] += b; s1[2] += c; s1[3] += d;
    s1[4] += e; s1[5] += f; s1[6] += g; s1[7] += h;
    s2[0] += a2; s2[1] += b2; s2[2] += c2; s2[3] += d2;
    s2[4] += e2; s2[5] += f2; s2[6] += g2; s2[7] += h2;
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

// Block k of the message at p.  The offset is formed in 64 bits: 16 * k dwords
// no longer fit 32 bits from a 16 GiB message on (k >= 2^28).
__device__ __forceinline__ const uint32_t* blk(const uint32_t* __restrict__ p, uint32_t k) {
    return p + (static_cast<uint64_t>(k) << 4);
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
    const uint32_t* __restrict__ q = blk(m.p, m.nfull);
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

// Full blocks [kb, ke) of m (kb < ke) into st.  Blocks are fetched in pairs
// (2j, 2j+1) requested back to back — one 128-byte line for line-aligned
// messages, so L2 never has to keep a half-read line across a compression —
// and the next pair is in flight while the current pair is compressed (two
// pairs of register buffers, loop unrolled x4).  Beside the Base64 stream
// this cut the SHA kernel's re-reads and its stalls on loaded HBM
// (154 GB read per config-2 launch against 198 GB with one-block-ahead fetch).
__device__ __forceinline__ void plain_range(uint32_t (&st)[8], const Msg& m, uint32_t kb, uint32_t ke) {
    uint32_t A[16], B[16], C[16], D[16], xa, xb, xc, xd;
    const uint32_t last = ke - 1u;
    load_block(blk(m.p, kb), m.sh, A, xa);
    load_block(blk(m.p, min(kb + 1u, last)), m.sh, B, xb);
    uint32_t k = kb;
    for (;;) {
        load_block(blk(m.p, min(k + 2u, last)), m.sh, C, xc);
        load_block(blk(m.p, min(k + 3u, last)), m.sh, D, xd);
        to_be(A, xa, m.sel);
        compress(st, A);
        if (++k >= ke) break;
        to_be(B, xb, m.sel);
        compress(st, B);
        if (++k >= ke) break;
        load_block(blk(m.p, min(k + 2u, last)), m.sh, A, xa);
        load_block(blk(m.p, min(k + 3u, last)), m.sh, B, xb);
        to_be(C, xc, m.sel);
        compress(st, C);
        if (++k >= ke) break;
        to_be(D, xd, m.sel);
        compress(st, D);
        if (++k >= ke) break;
    }
}

// Full blocks [kb, ke) of m into st and, from the same loads and schedule,
// into the twin state s2 (kShaTwin).  One block in flight while one is
// compressed (two buffers): a twin step is ~2,290 ops (~4 us), long enough to
// cover the load, and two buffers instead of plain_range's four keep the
// kernel at a VGPR count that leaves room for the Base64 / decode waves.
__device__ __forceinline__ void twin_range(uint32_t (&st)[8], uint32_t (&s2)[8], const Msg& m, uint32_t kb,
                                           uint32_t ke) {
    uint32_t A[16], B[16], xa, xb;
    const uint32_t last = ke - 1u;
    load_block(blk(m.p, kb), m.sh, A, xa);
    uint32_t k = kb;
    for (;;) {
        load_block(blk(m.p, min(k + 1u, last)), m.sh, B, xb);
        to_be(A, xa, m.sel);
        compress2(st, s2, A);
        if (++k >= ke) break;
        load_block(blk(m.p, min(k + 1u, last)), m.sh, A, xa);
        to_be(B, xb, m.sel);
        compress2(st, s2, B);
        if (++k >= ke) break;
    }
}

// ---------------------------------------------------------------------------
// Fused Base64 (upload plan, fragment lanes flagged kShaB64): the lane that
// hashes a fragment already holds each 64-byte block in registers as
// big-endian words, so it also emits the block's Base64 (StorageNode.java:636)
// instead of a second pass re-reading the fragment from HBM.  Groups of 3
// bytes straddle blocks with period 3: block k (phase k mod 3, uniform in the
// wave) encodes 21/21/22 groups = 84/84/88 chars and carries 1/2/0 bytes.
// Chars come from the 4,096-entry character-pair table in LDS (two reads per
// group).  The last < 66 bytes (carry + message tail) and the '=' padding are
// encoded after the block loop by enc_tail.

// x + x on the full-rate adder (hipcc would emit v_lshlrev_b32, half rate).
__device__ __forceinline__ uint32_t dbl(uint32_t x) {
    uint32_t r;
    asm("v_add_u32_e32 %0, %1, %1" : "=v"(r) : "v"(x));
    return r;
}
__device__ __forceinline__ uint32_t pair_rd(const uint16_t* __restrict__ pair, uint32_t byte_addr) {
    return *reinterpret_cast<const uint16_t*>(reinterpret_cast<const char*>(pair) + byte_addr);
}
// Chars of the group at byte q of X = {prev, W[0..15]} (68 bytes, big-endian
// words): byte addresses 2*hi12 and 2*lo12 straight from the word bits.
template <int Q>
__device__ __forceinline__ uint32_t enc_grp(const uint16_t* __restrict__ pair, const uint32_t (&W)[16], uint32_t prev) {
    constexpr int j = Q / 4, o = Q % 4;
    const uint32_t x = j == 0 ? prev : W[j == 0 ? 0 : j - 1];
    const uint32_t y = W[j < 16 ? j : 15];  // X[j+1] (only used for o >= 2, where j < 16)
    uint32_t ah, al;
    if (o == 0) {
        ah = (x >> 19) & 0x1ffeu; al = (x >> 7) & 0x1ffeu;
    } else if (o == 1) {
        ah = (x >> 11) & 0x1ffeu; al = dbl(x) & 0x1ffeu;
    } else if (o == 2) {
        ah = (x >> 3) & 0x1ffeu; al = __builtin_amdgcn_alignbit(x, y, 23) & 0x1ffeu;
    } else {
        ah = __builtin_amdgcn_alignbit(x, y, 27) & 0x1ffeu; al = (y >> 15) & 0x1ffeu;
    }
    return __builtin_amdgcn_perm(pair_rd(pair, al), pair_rd(pair, ah), 0x05040100u);
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// Four groups (8 LDS reads); the scheduling barrier bounds the reads in
// flight, otherwise hipcc issues all 42 of a block at once (+~60 VGPRs).
template <int F, int G0>
__device__ __forceinline__ u32x4 enc_quad(const uint16_t* __restrict__ pair, const uint32_t (&W)[16], uint32_t prev) {
    const u32x4 r{enc_grp<F + 3 * G0>(pair, W, prev), enc_grp<F + 3 * (G0 + 1)>(pair, W, prev),
                  enc_grp<F + 3 * (G0 + 2)>(pair, W, prev), enc_grp<F + 3 * (G0 + 3)>(pair, W, prev)};
    __builtin_amdgcn_sched_barrier(0);
    return r;
}

// A wave's staging tile for 64-byte runs its lanes produce (decoded blocks,
// halves of Base64 lines): lane l parks its 64 bytes in v[l] (80-byte rows keep
// the 16-byte accesses off each other's banks), then lanes 4i .. 4i+3 together
// write row i's 64 bytes to base[i] + the run's offset, so one store
// instruction carries 16 whole 64-byte runs instead of 64 separate 16-byte
// pieces (a lane's own 16-byte stores to its own cache line cost the one-pass
// replica check a third of its time).  Wave-private: ordered by wavefront
// fences, no barrier.
struct DecTile {
    uint4 v[64][5];
    uint64_t base[64];
};

// Every lane of the wave calls this together (coop = the whole wave is here);
// rows = ballot of the lanes whose q0..q3 are to be written at base[lane] + off.
__device__ __forceinline__ void stage_store(DecTile& tile, bool coop, uint64_t rows, bool act, const uint4& q0,
                                            const uint4& q1, const uint4& q2, const uint4& q3, uint64_t off) {
    const uint32_t lane = threadIdx.x & 63u;
    if (coop) {
        if (act) {
            tile.v[lane][0] = q0; tile.v[lane][1] = q1; tile.v[lane][2] = q2; tile.v[lane][3] = q3;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const uint32_t row = 16u * t + (lane >> 2), part = lane & 3u;
            if ((rows >> row) & 1ull) {
                const uint4 q = tile.v[row][part];
                *reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(tile.base[row]) + off + 16u * part) = q;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else if (act) {
        uint4* o = reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(tile.base[lane]) + off);
        o[0] = q0; o[1] = q1; o[2] = q2; o[3] = q3;
    }
}

// Block of phase PH (first group at X byte F = 4 - carry_in).  Output is
// written in whole 128-byte lines of the 256-char super-block sb (3 blocks):
// phase 0's 21 dwords wait in P, phase 1 writes line 0 (P[0..20] + its first
// 11 dwords) and keeps its last 10 in P, phase 2 writes line 1 (P[0..9] + its
// 22).  Each line is stored by 8 back-to-back dwordx4 of the lane, so L2
// never holds a partly written line across blocks (written block by block,
// the 64 lanes' interleaved partial lines were evicted half-written:
// WRITE_SIZE 1.8x and extra fills, 116 vs 82 ms).  With 128-byte aligned
// fragment starts (DFS_LAYOUT_ALIGN128) every store is a full-line piece.
template <int PH>
__device__ __forceinline__ void enc_block(const uint16_t* __restrict__ pair, const uint32_t (&W)[16], uint32_t prev,
                                          uint32_t (&P)[21], bool act, DecTile& tile, uint64_t off) {
    constexpr int F = PH == 0 ? 4 : (PH == 1 ? 3 : 2);
    auto u4 = [](uint32_t a, uint32_t b, uint32_t c, uint32_t d) { return make_uint4(a, b, c, d); };
    if (PH == 0) {
        if (act) {
#pragma unroll
            for (int q = 0; q < 5; ++q) {
                const u32x4 v = q == 0 ? enc_quad<F, 0>(pair, W, prev)
                              : q == 1 ? enc_quad<F, 4>(pair, W, prev)
                              : q == 2 ? enc_quad<F, 8>(pair, W, prev)
                              : q == 3 ? enc_quad<F, 12>(pair, W, prev)
                                       : enc_quad<F, 16>(pair, W, prev);
                P[4 * q] = v.x; P[4 * q + 1] = v.y; P[4 * q + 2] = v.z; P[4 * q + 3] = v.w;
            }
            P[20] = enc_grp<F + 60>(pair, W, prev);
        }
        return;
    }
    // Every lane of the wave's encode loop is here together (uniform trip
    // count); act = this lane still has a block of its own to encode.
    const bool coop = __ballot(1) == ~0ull;
    const uint64_t rows = __ballot(act);
    uint4 q0 = make_uint4(0, 0, 0, 0), q1 = q0, q2 = q0, q3 = q0;
    if (PH == 1) {  // line 0 of the super-block: P[0..20] + this block's first 11 dwords
        if (act) {
            q0 = u4(P[0], P[1], P[2], P[3]); q1 = u4(P[4], P[5], P[6], P[7]);
            q2 = u4(P[8], P[9], P[10], P[11]); q3 = u4(P[12], P[13], P[14], P[15]);
        }
        stage_store(tile, coop, rows, act, q0, q1, q2, q3, off);
        if (act) {
            const u32x4 n0 = enc_quad<F, 0>(pair, W, prev);
            const u32x4 n1 = enc_quad<F, 4>(pair, W, prev);
            const u32x4 n2 = enc_quad<F, 8>(pair, W, prev);
            q0 = u4(P[16], P[17], P[18], P[19]); q1 = u4(P[20], n0.x, n0.y, n0.z);
            q2 = u4(n0.w, n1.x, n1.y, n1.z); q3 = u4(n1.w, n2.x, n2.y, n2.z);
            const u32x4 n3 = enc_quad<F, 12>(pair, W, prev);
            const u32x4 n4 = enc_quad<F, 16>(pair, W, prev);
            P[0] = n2.w;
            P[1] = n3.x; P[2] = n3.y; P[3] = n3.z; P[4] = n3.w;
            P[5] = n4.x; P[6] = n4.y; P[7] = n4.z; P[8] = n4.w;
            P[9] = enc_grp<F + 60>(pair, W, prev);
        }
        stage_store(tile, coop, rows, act, q0, q1, q2, q3, off + 64);
    } else {  // line 1: P[0..9] + this block's 22 dwords
        uint32_t c0 = 0, c1 = 0;  // n1.z, n1.w: the second half's first two dwords
        if (act) {
            const u32x4 n0 = enc_quad<F, 0>(pair, W, prev);
            const u32x4 n1 = enc_quad<F, 4>(pair, W, prev);
            q0 = u4(P[0], P[1], P[2], P[3]); q1 = u4(P[4], P[5], P[6], P[7]);
            q2 = u4(P[8], P[9], n0.x, n0.y); q3 = u4(n0.z, n0.w, n1.x, n1.y);
            c0 = n1.z; c1 = n1.w;
        }
        stage_store(tile, coop, rows, act, q0, q1, q2, q3, off + 128);
        if (act) {
            const u32x4 n2 = enc_quad<F, 8>(pair, W, prev);
            const u32x4 n3 = enc_quad<F, 12>(pair, W, prev);
            const u32x4 n4 = enc_quad<F, 16>(pair, W, prev);
            const uint32_t n20 = enc_grp<F + 60>(pair, W, prev), n21 = enc_grp<F + 63>(pair, W, prev);
            q0 = u4(c0, c1, n2.x, n2.y); q1 = u4(n2.z, n2.w, n3.x, n3.y);
            q2 = u4(n3.z, n3.w, n4.x, n4.y); q3 = u4(n4.z, n4.w, n20, n21);
        }
        stage_store(tile, coop, rows, act, q0, q1, q2, q3, off + 192);
    }
}

// After the block loop: write what enc_block still holds (ph = phase of the
// next block: 1 -> phase 0's 21 dwords at sb, 2 -> phase 1's last 10 at sb+128).
__device__ __forceinline__ void enc_flush(uint32_t ph, char* __restrict__ sb, const uint32_t (&P)[21]) {
    u32x4* d4 = reinterpret_cast<u32x4*>(sb);
    if (ph == 1) {
        d4[0] = u32x4{P[0], P[1], P[2], P[3]};
        d4[1] = u32x4{P[4], P[5], P[6], P[7]};
        d4[2] = u32x4{P[8], P[9], P[10], P[11]};
        d4[3] = u32x4{P[12], P[13], P[14], P[15]};
        d4[4] = u32x4{P[16], P[17], P[18], P[19]};
        reinterpret_cast<uint32_t*>(sb)[20] = P[20];
    } else if (ph == 2) {
        d4[8] = u32x4{P[0], P[1], P[2], P[3]};
        d4[9] = u32x4{P[4], P[5], P[6], P[7]};
        *reinterpret_cast<u32x2*>(sb + 160) = u32x2{P[8], P[9]};
    }
}

// Bytes [start, len) of the fragment at src, start = 64*nfull - nfull%3 (a
// multiple of 3): full groups, then the RFC 4648 padded final group.
__device__ __forceinline__ void enc_tail(const uint16_t* __restrict__ pair, const uint8_t* __restrict__ src,
                                         uint64_t start, uint64_t len, char* __restrict__ out) {
    for (uint64_t pos = start; pos < len; pos += 3) {
        const uint64_t n = len - pos < 3 ? len - pos : 3;
        uint32_t v = static_cast<uint32_t>(src[pos]) << 16;
        if (n > 1) v |= static_cast<uint32_t>(src[pos + 1]) << 8;
        if (n > 2) v |= src[pos + 2];
        uint32_t w = pair_rd(pair, 2u * (v >> 12)) | (pair_rd(pair, 2u * (v & 0xfffu)) << 16);
        if (n == 1) w = (w & 0x0000ffffu) | 0x3d3d0000u;       // "xx=="
        else if (n == 2) w = (w & 0x00ffffffu) | 0x3d000000u;  // "xxx="
        *reinterpret_cast<uint32_t*>(out + 4 * (pos / 3)) = w;
    }
}

__constant__ uint32_t kB64Alpha[16] = {
    0x44434241u, 0x48474645u, 0x4c4b4a49u, 0x504f4e4du, 0x54535251u, 0x58575655u, 0x62615a59u, 0x66656463u,
    0x6a696867u, 0x6e6d6c6bu, 0x7271706fu, 0x76757473u, 0x7a797877u, 0x33323130u, 0x37363534u, 0x2f2b3938u};

// Max over the 64 lanes (all active).
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = max(v, static_cast<uint32_t>(__shfl_xor(static_cast<int>(v), d, 64)));
    return v;
}

// Read by lanes with no full block while their wave still runs the block loop.
__device__ uint32_t g_dummy_block[32];

// Park / restore a lane's 8-word state in LDS (word-major: conflict-free).
__device__ __forceinline__ void park(uint32_t* stash, const uint32_t (&st)[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) stash[i * kShaBlock + threadIdx.x] = st[i];
}
__device__ __forceinline__ void unpark(const uint32_t* stash, uint32_t (&st)[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) st[i] = stash[i * kShaBlock + threadIdx.x];
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
// ENC = the fused-Base64 instantiation (launched when the caller passes a
// Base64 output): lanes flagged kShaB64 also write their message's Base64;
// every other lane of the launch (fileId lanes, twins included) hashes as in
// the plain instantiation.
constexpr uint32_t kStealSpins = 16;  // x s_sleep 127 (8,128 clocks each)

// Decode-ahead (ShaWait, dfs_internal.h): the active lanes of the wave wait
// until fragment group `need` (per lane; ~0u = nothing to wait for) has been
// published by every decode workgroup, then acquire at agent scope so the
// loads that follow see the decoded bytes (the decode ran on other CUs / XCDs).
// Bounded (ShaWait::ticks of s_memrealtime): on timeout queue[2] is set (the host re-runs the SHA launch after
// the decode) and the lane goes on, so the grid always drains.
__device__ __forceinline__ void wait_group(const ShaWait& w, uint32_t need, uint32_t* __restrict__ queue) {
    const bool want = need != ~0u && need >= w.first;
    bool ok = !want || __hip_atomic_load(w.done + need, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= w.target;
    // Once any wave of the launch has timed out (queue[2]) the host will redo
    // the whole launch after the decode: nobody waits again, so a launch that
    // cannot run beside its decode stalls once, not once per item and group.
    if (__ballot(!ok) && !__hip_atomic_load(queue + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        for (;;) {
            __builtin_amdgcn_s_sleep(32);
            if (!ok) ok = __hip_atomic_load(w.done + need, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= w.target;
            if (!__ballot(!ok)) break;
            if (__hip_atomic_load(queue + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
            if (__builtin_amdgcn_s_memrealtime() - t0 > w.ticks) {
                atomicOr(queue + 2, 1u);
                break;
            }
        }
    }
    if (__ballot(want)) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

// First block of fragment g of a file of S bytes split into N (SN:138-157).
__device__ __forceinline__ uint32_t frag_block(uint64_t S, uint32_t N, uint32_t g) {
    const uint64_t base = S / N, rem = S % N;
    return static_cast<uint32_t>((g * base + (g < rem ? g : rem)) >> 6);
}

template <bool ENC, bool WAIT>
__device__ __forceinline__ void sha256_body(const uint8_t* __restrict__ base, const ShaDesc* __restrict__ descs,
                                            uint32_t n, uint32_t split, uint32_t n_long, uint32_t cap,
                                            uint8_t* __restrict__ out0, uint8_t* __restrict__ out1,
                                            uint32_t* __restrict__ queue, uint32_t* __restrict__ state,
                                            char* __restrict__ b64, const ShaWait& W) {
    const uint32_t nitems = (n + 63u) >> 6;
    const uint32_t n_short = nitems - n_long;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t key = simd_key();
    __shared__ uint16_t pair[ENC ? 4096 : 2];           // Base64 character pairs
    __shared__ uint32_t stash[ENC ? 8 * kShaBlock : 1];  // states parked by finished lanes
    __shared__ __align__(16) uint8_t tile_mem[ENC ? sizeof(DecTile) * (kShaBlock / 64) : 16];
    DecTile& tile = reinterpret_cast<DecTile*>(tile_mem)[ENC ? threadIdx.x >> 6 : 0];
    if (ENC) {
        const uint8_t* a = reinterpret_cast<const uint8_t*>(kB64Alpha);
        for (uint32_t k = threadIdx.x; k < 4096u; k += kShaBlock)
            pair[k] = static_cast<uint16_t>(a[k >> 6] | (static_cast<uint32_t>(a[k & 63u]) << 8));
        __syncthreads();
    }
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
                } else if (n_long) {
                    // Long items a starved SIMD left behind (one that got fewer
                    // than `cap` waves).  Taken only after the SIMDs that have
                    // waves claimed theirs (~50 us), so a launch whose items
                    // are all long keeps exactly `cap` per SIMD.
                    for (uint32_t spin = 0;; ++spin) {
                        if (__hip_atomic_load(queue, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= n_long) break;
                        if (spin == kStealSpins) {
                            const uint32_t it2 = atomicAdd(queue, 1u);
                            if (it2 < n_long) item = it2;
                            break;
                        }
                        __builtin_amdgcn_s_sleep(127);
                    }
                }
            }
        }
        item = __builtin_amdgcn_readfirstlane(item);
        if (item == 0xffffffffu) break;
        if (item < n_long) __builtin_amdgcn_s_setprio(2);
        else __builtin_amdgcn_s_setprio(0);
        const uint32_t gid = item * 64u + lane;
        // ENC: uniform trip count (the wave's longest message, in an SGPR).
        // A divergent loop exit inside the three-phase body made hipcc copy
        // the loop state on every exit edge (192 VGPRs, 2 waves/SIMD); lanes
        // past their own length run the body on a clamped block and park
        // their state in LDS.
        // Only the lanes that encode (kShaB64) run that loop; the others
        // (fileId lanes, with or without twins) take the plain path below.
        const uint32_t kmax =
            ENC ? __builtin_amdgcn_readfirstlane(wave_max(
                      gid < n && (descs[gid].flags & kShaB64) ? static_cast<uint32_t>(descs[gid].len >> 6) : 0u))
                : 0u;
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
            if (ENC && (m.flags & kShaB64) != 0u) {
                const bool enc = true;
                char* bdst = b64 + descs[gid].b64;
                tile.base[lane] = reinterpret_cast<uint64_t>(bdst);  // the wave's other lanes read it in stage_store
                uint64_t boff = 0;                                   // the super-block's offset in every lane's output
                if (kmax) {
                    // C holds block k, N receives block k+1 (clamped) while C
                    // is compressed; the body is unrolled over the three
                    // Base64 phases (k mod 3) so the pending-line registers P
                    // have static indices; C = N is a register copy.
                    const uint32_t* bp = m.nfull ? m.p : g_dummy_block;
                    const uint32_t last = m.nfull ? m.nfull - 1u : 0u;
                    const bool early = m.nfull < kmax;
                    if (early) park(stash, st);
                    uint32_t C[16], N[16], xc, xn;
                    uint32_t prev = 0;  // last word of the previous block
                    uint32_t P[21];     // Base64 dwords waiting for their line
                    load_block(bp, m.sh, C, xc);
                    uint32_t k = 0;
#define DFS_SHA_STEP(PH)                                                          \
    {                                                                             \
        load_block(blk(bp, min(k + 1u, last)), m.sh, N, xn);                    \
        to_be(C, xc, m.sel);                                                      \
        {                                                                         \
            const bool act = k < m.nfull;                                         \
            enc_block<PH>(pair, C, prev, P, act, tile, boff);                     \
            if (act) prev = C[15];                                                \
        }                                                                         \
        __builtin_amdgcn_sched_barrier(0); /* keep the encode out of the rounds */ \
        compress(st, C);                                                          \
        __builtin_amdgcn_sched_barrier(0);                                        \
        if (early && k + 1u == m.nfull) park(stash, st);                          \
        if (++k >= kmax) break;                                                   \
        _Pragma("unroll") for (int i = 0; i < 16; ++i) C[i] = N[i];               \
        xc = xn;                                                                  \
    }
                    for (;;) {
                        DFS_SHA_STEP(0)
                        DFS_SHA_STEP(1)
                        DFS_SHA_STEP(2)
                        boff += 256;
                    }
#undef DFS_SHA_STEP
                    if (early) unpark(stash, st);
                    if (enc && m.nfull)
                        enc_flush(m.nfull % 3u, b64 + descs[gid].b64 + 256ull * (m.nfull / 3u), P);
                }
                if (enc) {
                    const uint64_t start = 64ull * m.nfull - m.nfull % 3u;
                    enc_tail(pair, base + descs[gid].off, start, m.len, b64 + descs[gid].b64);
                }
            } else {
                // Segments of the lane's full blocks: plain blocks up to the
                // next twin's first block, then the twin's blocks with both
                // states, the twin's own tail block(s) and digest, and so on.
                // A lane without twins runs plain_range(0, nfull) once.
                // With ShaWait (decode-ahead download) a segment also ends
                // where the lane next has to wait for a fragment group: a
                // fragment lane waits for its own group before its first
                // block, a fileId lane for group g before the block holding
                // fragment g's first byte (twins never straddle those).
                uint32_t tw = 0, tw_end = 0;
                const uint64_t off0 = descs[gid].off;
                if (m.flags & kShaTwin) {
                    const uint64_t t = descs[gid].b64;
                    tw = n + static_cast<uint32_t>(t);
                    tw_end = tw + static_cast<uint32_t>(t >> 32);
                }
                uint32_t wg = 0, wn = 0, wb = ~0u;  // next group to wait for, groups end, its first block
                if (WAIT) {
                    if (m.out < W.nf) {
                        wg = m.out % W.nfrag;
                        wn = wg + 1;
                    } else {
                        wn = W.nfrag;
                    }
                    wb = 0;
                }
                uint32_t k = 0;
                for (;;) {
                    if (WAIT) {
                        uint32_t need = ~0u;
                        while (wg < wn && wb <= k) {
                            need = wg++;
                            wb = wg < wn ? (m.out < W.nf ? 0u : frag_block(m.total, W.nfrag, wg)) : ~0u;
                        }
                        wait_group(W, need, queue);
                    }
                    const bool has = tw < tw_end;
                    uint32_t k0 = m.nfull;
                    ShaDesc td{};
                    if (has) {
                        td = descs[tw];
                        k0 = static_cast<uint32_t>((td.off - off0) >> 6);
                    }
                    const uint32_t ke = min(k0, wb);
                    if (k < ke) {
                        plain_range(st, m, k, ke);
                        k = ke;
                        continue;
                    }
                    if (!has) break;
                    const Msg t = msg_setup(base, td);
                    uint32_t s2[8];
                    init_state(s2);
                    twin_range(st, s2, m, k0, k0 + t.nfull);
                    for (uint32_t tb = 0; tb < t.ntb; ++tb) {
                        uint32_t W[16];
                        tail_block(t, tb, W);
                        compress(s2, W);
                    }
                    store_digest(s2, t.out, split, out0, out1);
                    k = k0 + t.nfull;
                    ++tw;
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
    }
}

// ---------------------------------------------------------------------------
// Latency kernel for launches too small to fill the chip (a batcher batch,
// the long-fragment skew config, small host calls): each message's chain is
// the critical path, and one wave issues every instruction of its lanes'
// blocks.  Two waves share the 64 messages of a workgroup: the helper wave
// (wave 1) loads each block, byte-swaps it, expands the message schedule and
// writes K[t] + W[t] for all 64 rounds to LDS one block ahead; the owner
// wave (wave 0) runs only the rounds (14 VALU ops each, K and W folded into
// one LDS operand) — about 0.65 of the single-wave instruction stream of
// sha256_lanes per block.  One workgroup barrier per block hands the two
// LDS slots over (double buffering).  Lanes past their own block count keep
// their state (predicated update); partial / resumed messages as in
// sha256_lanes (kShaPartial stores the state, kShaResume loads it).
constexpr int kChainBlock = 128;  // owner + helper wave

__device__ __forceinline__ void owner_block(uint32_t (&st)[8], const uint4* __restrict__ kw, bool act) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    uint4 q = kw[0];
#pragma unroll
    for (int t4 = 0; t4 < 16; ++t4) {
        const uint4 cur = q;
        if (t4 + 1 < 16) q = kw[(t4 + 1) * 64];  // next quad of K+W in flight
        const uint32_t v[4] = {cur.x, cur.y, cur.z, cur.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t tmp = h + ch(e, f, g) + v[j];
            const uint32_t t1 = tmp + bsig1(e);
            const uint32_t na = t1 + bsig0(a) + maj(a, b, c);
            h = g; g = f; f = e; e = d + t1;
            d = c; c = b; b = a; a = na;
            asm volatile("" : "+v"(a), "+v"(e));
        }
    }
    if (act) {
        st[0] += a; st[1] += b; st[2] += c; st[3] += d;
        st[4] += e; st[5] += f; st[6] += g; st[7] += h;
    }
}

// K[t] + W[t] of block k of m (raw words r + look-ahead x for full blocks,
// the padded tail for k < nb, zeros past the lane's own blocks) into
// kw[t/4 * STRIDE][t%4].
template <int STRIDE = 64>
__device__ __forceinline__ void helper_block(const Msg& m, uint32_t nb, uint32_t k, uint32_t (&r)[16], uint32_t x,
                                             uint4* __restrict__ kw) {
    uint32_t W[16];
    if (k < m.nfull) {
        to_be(r, x, m.sel);
#pragma unroll
        for (int i = 0; i < 16; ++i) W[i] = r[i];
    } else if (k < nb) {
        tail_block(m, k - m.nfull, W);
    } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) W[i] = 0u;
    }
    uint32_t o[4];
#pragma unroll
    for (int t = 0; t < 64; ++t) {
        if (t >= 16) {
            W[t & 15] += ssig1(W[(t - 2) & 15]) + W[(t - 7) & 15] + ssig0(W[(t - 15) & 15]);
            asm volatile("" : "+v"(W[t & 15]));
        }
        o[t & 3] = kK[t] + W[t & 15];
        if ((t & 3) == 3) kw[(t >> 2) * STRIDE] = make_uint4(o[0], o[1], o[2], o[3]);
    }
}

// Helper wave of the chain kernels: K + W of every block of message m (nb
// blocks in all, kmax = the workgroup's longest) into kw[(k & 1)][..][lane],
// one block ahead of the owner wave; raw blocks k+1 (R) and k+2 (Q) in flight
// while block k+1 is expanded.
__device__ __forceinline__ void helper_run(const Msg& m, bool live, uint32_t nb, uint32_t kmax, uint4 (*kw)[16 * 64],
                                           uint32_t lane) {
    const uint32_t* bp = (live && m.nfull) ? m.p : g_dummy_block;
    const uint32_t last = (live && m.nfull) ? m.nfull - 1u : 0u;
    const uint32_t sh = live ? m.sh : 0u;
    uint32_t R[16], Q[16], xr, xq;
    load_block(bp, sh, R, xr);
    if (kmax) helper_block(m, nb, 0, R, xr, kw[0] + lane);
    load_block(blk(bp, min(1u, last)), sh, R, xr);
    __syncthreads();
    for (uint32_t k = 0; k < kmax; ++k) {
        if (k + 1 < kmax) {
            load_block(blk(bp, min(k + 2u, last)), sh, Q, xq);
            helper_block(m, nb, k + 1, R, xr, kw[(k + 1) & 1u] + lane);
#pragma unroll
            for (int i = 0; i < 16; ++i) R[i] = Q[i];
            xr = xq;
        }
        __syncthreads();
    }
}

// The pair-lane kernel's helper: TWO blocks ahead of the owner wave into three
// slots of 16 x 32 quads (kw3[(k % 3)][t/4 * 32 + idx], idx = the message's
// index in the wave; both lanes of a pair expand the same message and write
// the same words), so the owner can fetch the next block's first quads before
// the barrier that ends the current one.  Slot (k + 2) % 3 was last read by
// the owner during block k - 1, i.e. before the barrier this write follows.
__device__ __forceinline__ void helper_run3(const Msg& m, bool live, uint32_t nb, uint32_t kmax, uint4 (*kw3)[16 * 32],
                                            uint32_t idx) {
    const uint32_t* bp = (live && m.nfull) ? m.p : g_dummy_block;
    const uint32_t last = (live && m.nfull) ? m.nfull - 1u : 0u;
    const uint32_t sh = live ? m.sh : 0u;
    uint32_t R[16], Q[16], xr, xq;
    load_block(bp, sh, R, xr);
    load_block(blk(bp, min(1u, last)), sh, Q, xq);
    if (kmax) helper_block<32>(m, nb, 0, R, xr, kw3[0] + idx);
    load_block(blk(bp, min(2u, last)), sh, R, xr);
    if (kmax > 1) helper_block<32>(m, nb, 1, Q, xq, kw3[1] + idx);
    __syncthreads();  // blocks 0 and 1 staged
    uint32_t slot = 2;  // (k + 2) % 3
    for (uint32_t k = 0; k < kmax; ++k) {
        if (k + 2 < kmax) {
            load_block(blk(bp, min(k + 3u, last)), sh, Q, xq);
            helper_block<32>(m, nb, k + 2, R, xr, kw3[slot] + idx);
#pragma unroll
            for (int i = 0; i < 16; ++i) R[i] = Q[i];
            xr = xq;
        }
        slot = slot == 2u ? 0u : slot + 1u;
        __syncthreads();
    }
}

// Blocks the chain kernels run for message gid (0 past the launch's end).
__device__ __forceinline__ uint32_t chain_blocks(const ShaDesc* __restrict__ descs, uint32_t n, uint32_t gid) {
    if (gid >= n) return 0u;
    const uint64_t len = descs[gid].len;
    const uint32_t ntb = (static_cast<uint32_t>(len) & 63u) < 56u ? 1u : 2u;
    return static_cast<uint32_t>(len >> 6) + ((descs[gid].flags & kShaPartial) ? 0u : ntb);
}

// PAIRS owner/helper wave pairs per workgroup (waves [0, PAIRS) own, waves
// [PAIRS, 2 PAIRS) help): with two pairs a CU's four SIMDs each hold one wave
// of ONE workgroup.  Two workgroups of one pair on a CU put two of their four
// waves on one SIMD and leave another SIMD idle (tools/wave_place_probe), and
// two waves on a SIMD run these chains at nearly half the speed (a 1 MiB
// chain: 45.4 instead of 29.4 ms at 32,768 messages).  Every wave passes the
// same number of barriers: kmax is the workgroup's longest message.
template <int PAIRS>
__global__ __launch_bounds__(kChainBlock * PAIRS) void sha256_chain(const uint8_t* __restrict__ base,
                                                                    const ShaDesc* __restrict__ descs, uint32_t n,
                                                                    uint32_t split, uint8_t* __restrict__ out0,
                                                                    uint8_t* __restrict__ out1,
                                                                    uint32_t* __restrict__ state) {
    __shared__ uint4 kws[PAIRS][2][16 * 64];  // [pair][slot][t/4][lane]: 32 KiB per pair
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const bool owner = wave < static_cast<uint32_t>(PAIRS);
    const uint32_t pair = owner ? wave : wave - PAIRS;
    uint4 (*kw)[16 * 64] = kws[pair];
    const uint32_t gid = (blockIdx.x * PAIRS + pair) * 64u + lane;
    const bool live = gid < n;
    Msg m{};
    uint32_t nb = 0;
    if (live) {
        m = msg_setup(base, descs[gid]);
        nb = m.nfull + ((m.flags & kShaPartial) ? 0u : m.ntb);
    }
    uint32_t nbw = 0;
#pragma unroll
    for (int p = 0; p < PAIRS; ++p) nbw = max(nbw, chain_blocks(descs, n, (blockIdx.x * PAIRS + p) * 64u + lane));
    const uint32_t kmax = __builtin_amdgcn_readfirstlane(wave_max(nbw));
    if (owner) {
        uint32_t st[8];
        if (live && (m.flags & kShaResume)) {
            const uint4* s4 = reinterpret_cast<const uint4*>(state + 8ull * m.out);
            const uint4 s0 = s4[0], s1 = s4[1];
            st[0] = s0.x; st[1] = s0.y; st[2] = s0.z; st[3] = s0.w;
            st[4] = s1.x; st[5] = s1.y; st[6] = s1.z; st[7] = s1.w;
        } else {
            init_state(st);
        }
        __syncthreads();  // block 0 staged
        for (uint32_t k = 0; k < kmax; ++k) {
            owner_block(st, kw[k & 1u] + lane, k < nb);
            __syncthreads();
        }
        if (live) {
            if (m.flags & kShaPartial) {
                uint4* s4 = reinterpret_cast<uint4*>(state + 8ull * m.out);
                s4[0] = make_uint4(st[0], st[1], st[2], st[3]);
                s4[1] = make_uint4(st[4], st[5], st[6], st[7]);
            } else {
                store_digest(st, m.out, split, out0, out1);
            }
        }
    } else {
        helper_run(m, live, nb, kmax, kw, lane);
    }
}

// ---------------------------------------------------------------------------
// Pair-lane latency kernel: the owner wave's 14 ops per round are the critical
// path of a chain, and half of them (Sigma0 + Maj on a, b, c) do not depend on
// the other half (Sigma1 + Ch on e, f, g) within a round.  Here TWO lanes of
// the owner wave share one message: the E lane keeps (e, f, g, h), the A lane
// (a, b, c, d), both run the SAME instruction stream with per-lane rotate
// counts (6, 11, 25 / 2, 13, 22) and one select bit turns Ch into Maj
// (Maj(a, b, c) = Ch(a ^ c, b, c)), then three DPP adds exchange the round's
// results between the partners: 10 VALU ops per round instead of 14, 32
// messages per owner wave instead of 64 (the launches this kernel serves
// leave most of the chip idle anyway).
//
// Lane layout: DPP bank masks enable whole banks of 4 lanes, so E lanes are
// banks 0 and 2 of each row of 16 (lane & 4 == 0), A lanes banks 1 and 3, and
// a lane's partner is lane ^ 4 (row_shl:4 / row_shr:4).  Message p of the
// wave = lanes with ((lane >> 3) << 2 | (lane & 3)) == p; the helper wave
// expands the schedule on both lanes of a pair (same loads, same values,
// written to the message's one place in LDS).
//
// Hazards (VALU write -> DPP read of the same VGPR needs 2 wait states; the
// compiler does not see inside asm): every DPP source here is written at
// least one round earlier, or two instructions earlier inside the same asm
// statement, or by the s_nop statement that opens a block.
constexpr uint32_t kChain2Msgs = 32;  // messages per owner wave

__device__ __forceinline__ uint32_t pair_index(uint32_t lane) { return ((lane >> 3) << 2) | (lane & 3u); }

// One round of the pair-lane owner wave as asm text (operands: %0..%3 the
// four state registers, X0..X3 = the ones playing x0..x3 in this round; %4 = Z;
// %5..%7 temporaries; %8..%10 rotate counts; %11 the Maj select mask; KN = K + W
// of the round after this one):
//   S = rotr(x0, s0) ^ rotr(x0, s1) ^ rotr(x0, s2)   E: Sigma1(e)     A: Sigma0(a)
//   F = Ch(x0 ^ (x2 & m), x1, x2)                    E: Ch(e, f, g)   A: Maj(a, b, c)
//   Y = S + F + Z                                    E: T1            A: T2
//   E lanes: x3 = x3[partner] + Y       (e' = d + T1)
//   E lanes: Z  = x2 + KN               (the next round's h is this round's g)
//   A lanes: x3 = Y[partner] + Y        (a' = T1 + T2)
// The Z update sits between the two exchanges: it gives Y its two wait states
// before the DPP read.  Whole quads of rounds go into one asm statement: the
// compiler pads every asm result it cannot see into with a wait state.
#define DFS_PAIR_ROUND(X0, X1, X2, X3, KN)                                               \
    "v_alignbit_b32 %5, " X0 ", " X0 ", %8\n\t"                                          \
    "v_alignbit_b32 %6, " X0 ", " X0 ", %9\n\t"                                          \
    "v_alignbit_b32 %7, " X0 ", " X0 ", %10\n\t"                                         \
    "v_bitop3_b32 %5, %5, %6, %7 bitop3:0x96\n\t"                                        \
    "v_bitop3_b32 %6, " X0 ", " X2 ", %11 bitop3:0x78\n\t"                               \
    "v_bitop3_b32 %6, %6, " X1 ", " X2 " bitop3:0xca\n\t"                                \
    "v_add3_u32 %5, %5, %6, %4\n\t"                                                      \
    "v_add_u32_dpp " X3 ", " X3 ", %5 row_shl:4 row_mask:0xf bank_mask:0x5\n\t"          \
    "v_add_u32_dpp %4, " X2 ", " KN " quad_perm:[0,1,2,3] row_mask:0xf bank_mask:0x5\n\t" \
    "v_add_u32_dpp " X3 ", %5, %5 row_shr:4 row_mask:0xf bank_mask:0xa\n\t"

// kw: this block's K + W quads (kw[t/4 * 32]); nxt: the next block's (staged
// two blocks ahead by the helper, so readable throughout this block).  q / qn
// arrive holding this block's quads 0 and 1 and leave holding the next
// block's: no LDS read waits behind the block's barrier.
__device__ __forceinline__ void owner_block2(uint32_t (&st)[4], const uint4* __restrict__ kw,
                                             const uint4* __restrict__ nxt, uint4& q, uint4& qn, bool act, uint32_t s0,
                                             uint32_t s1, uint32_t s2, uint32_t m) {
    uint32_t x0 = st[0], x1 = st[1], x2 = st[2], x3 = st[3];
    // x2 / x3 are DPP sources below and were just written by the previous
    // block's state update: two wait states, and everything after depends on it.
    asm volatile("s_nop 1" : "+v"(x2), "+v"(x3));
    uint32_t Z = 0;  // E lanes: h + K + W of the coming round; A lanes: 0
    asm volatile("v_add_u32_dpp %0, %1, %2 quad_perm:[0,1,2,3] row_mask:0xf bank_mask:0x5"
                 : "+v"(Z)
                 : "v"(x3), "v"(q.x));
    // K + W quads are fetched two ahead: a quad's asm statement takes the next
    // quad's first word, so that quad must have landed by then as well (one
    // ahead, every statement waited out a fresh LDS read: 29.0 vs 22.5 ms per
    // 1 MiB chain).
#pragma unroll
    for (int t4 = 0; t4 < 16; ++t4) {
        const uint4 cur = q;
        q = qn;
        qn = t4 + 2 < 16 ? kw[(t4 + 2) * 32] : nxt[(t4 - 14) * 32];
        // Four rounds; the registers' roles rotate and are back in place after
        // the fourth.  The last operand is the next quad's first K + W (after
        // the block's last round: any register, Z is not used again).
        uint32_t r0, r1, r2;
        asm volatile(DFS_PAIR_ROUND("%0", "%1", "%2", "%3", "%12")
                     DFS_PAIR_ROUND("%3", "%0", "%1", "%2", "%13")
                     DFS_PAIR_ROUND("%2", "%3", "%0", "%1", "%14")
                     DFS_PAIR_ROUND("%1", "%2", "%3", "%0", "%15")
                     : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(Z), "=&v"(r0), "=&v"(r1), "=&v"(r2)
                     : "v"(s0), "v"(s1), "v"(s2), "v"(m), "v"(cur.y), "v"(cur.z), "v"(cur.w), "v"(q.x));
    }
    if (act) {
        st[0] += x0; st[1] += x1; st[2] += x2; st[3] += x3;
    }
}
#undef DFS_PAIR_ROUND

template <int PAIRS>
__global__ __launch_bounds__(kChainBlock * PAIRS) void sha256_chain2(const uint8_t* __restrict__ base,
                                                                     const ShaDesc* __restrict__ descs, uint32_t n,
                                                                     uint32_t split, uint8_t* __restrict__ out0,
                                                                     uint8_t* __restrict__ out1,
                                                                     uint32_t* __restrict__ state) {
    __shared__ uint4 kws[PAIRS][3][16 * 32];  // [pair][slot][t/4][message]: 24 KiB per pair
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const bool owner = wave < static_cast<uint32_t>(PAIRS);
    const uint32_t pair = owner ? wave : wave - PAIRS;
    uint4 (*kw)[16 * 32] = kws[pair];
    const uint32_t idx = pair_index(lane);
    const uint32_t gid = (blockIdx.x * PAIRS + pair) * kChain2Msgs + idx;
    const bool live = gid < n;
    Msg m{};
    uint32_t nb = 0;
    if (live) {
        m = msg_setup(base, descs[gid]);
        nb = m.nfull + ((m.flags & kShaPartial) ? 0u : m.ntb);
    }
    uint32_t nbw = 0;
#pragma unroll
    for (int p = 0; p < PAIRS; ++p)
        nbw = max(nbw, chain_blocks(descs, n, (blockIdx.x * PAIRS + p) * kChain2Msgs + pair_index(lane)));
    const uint32_t kmax = __builtin_amdgcn_readfirstlane(wave_max(nbw));  // same in every wave of the workgroup
    if (owner) {
        const bool A = (lane & 4u) != 0u;  // (a, b, c, d) lane; else (e, f, g, h)
        uint32_t st[4];
        if (live && (m.flags & kShaResume)) {
            const uint4 s = reinterpret_cast<const uint4*>(state + 8ull * m.out)[A ? 0 : 1];
            st[0] = s.x; st[1] = s.y; st[2] = s.z; st[3] = s.w;
        } else if (A) {
            st[0] = 0x6a09e667u; st[1] = 0xbb67ae85u; st[2] = 0x3c6ef372u; st[3] = 0xa54ff53au;
        } else {
            st[0] = 0x510e527fu; st[1] = 0x9b05688cu; st[2] = 0x1f83d9abu; st[3] = 0x5be0cd19u;
        }
        const uint32_t s0 = A ? 2u : 6u, s1 = A ? 13u : 11u, s2 = A ? 22u : 25u, sel = A ? ~0u : 0u;
        __syncthreads();  // blocks 0 and 1 staged
        uint4 q = kw[0][idx], qn = kw[0][32 + idx];
        uint32_t slot = 0;  // k % 3
        for (uint32_t k = 0; k < kmax; ++k) {
            const uint32_t ns = slot == 2u ? 0u : slot + 1u;
            owner_block2(st, kw[slot] + idx, kw[ns] + idx, q, qn, k < nb, s0, s1, s2, sel);
            slot = ns;
            __syncthreads();
        }
        if (live) {
            if (m.flags & kShaPartial) {
                reinterpret_cast<uint4*>(state + 8ull * m.out)[A ? 0 : 1] = make_uint4(st[0], st[1], st[2], st[3]);
            } else {
                uint8_t* dst = m.out < split ? out0 + 32ull * m.out : out1 + 32ull * (m.out - split);
                reinterpret_cast<uint4*>(dst)[A ? 0 : 1] =
                    make_uint4(__builtin_bswap32(st[0]), __builtin_bswap32(st[1]), __builtin_bswap32(st[2]),
                               __builtin_bswap32(st[3]));
            }
        }
    } else {
        helper_run3(m, live, nb, kmax, kw, idx);
    }
}

// ---------------------------------------------------------------------------
// Held replicas (dfs_replica_check): Base64 decode, the decoded bytes written
// out, and their SHA-256 in ONE pass, one fragment per lane (SN:281-282).  The
// separate decode kernel writes the raw bytes and the SHA lanes read them back;
// here a lane reads its fragment's chars, decodes them in registers, hands the
// 64 decoded bytes of each block to the wave's staged store (DecTile: a lane's
// own 16-byte stores to its own cache line cost the kernel a third of its time)
// and compresses them, so the raw bytes cross HBM once (written) instead of
// twice.  Only canonical encodings of a known
// length are taken (chars = 4 * ceil(n / 3), as the uploader's encoder writes
// them, SN:636); a lane whose chars are not that reports it in `status` exactly
// as the decode kernel does (bit 0: IllegalArgumentException case, bit 1:
// decoded length differs from n).
//
// Block k of the decoded stream is bytes [64k, 64k + 64) = the 22 units (4
// chars -> 3 bytes) from unit floor(64k / 3) on, starting ph = k mod 3 bytes
// into the first.  Units are decoded through four 256-entry LDS tables (one
// per char position, values pre-shifted, bit 31 = outside the alphabet), the
// 17 big-endian words at unit-aligned byte offsets 0, 4, ... 64 are put
// together with constant shifts, and one v_perm per word applies the phase
// (and a second one gives the dword in memory order for the store).  Blocks
// that reach into the final unit (the padded one) and the message tail go the
// slow way: units decoded one at a time into the raw buffer, then hashed from
// there like any message.
__device__ __forceinline__ void dec_load(const uint32_t* __restrict__ p, uint32_t (&d)[22]) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const uint4 v = q[i];
        d[4 * i + 0] = v.x; d[4 * i + 1] = v.y; d[4 * i + 2] = v.z; d[4 * i + 3] = v.w;
    }
    const uint2 w = *reinterpret_cast<const uint2*>(p + 20);
    d[20] = w.x; d[21] = w.y;
}

__device__ __forceinline__ uint32_t dec_unit4(const uint32_t* __restrict__ lut, uint32_t w) {
    return lut[w & 255u] | lut[256u + ((w >> 8) & 255u)] | lut[512u + ((w >> 16) & 255u)] | lut[768u + (w >> 24)];
}

// One block: chars d (22 units), phase ph -> schedule words W, stored to dst.
__device__ __forceinline__ void dec_block(const uint32_t* __restrict__ lut, uint32_t (&d)[22], uint32_t ph,
                                          uint32_t (&W)[16], uint8_t* __restrict__ dst, uint64_t koff,
                                          DecTile& tile, uint32_t& bad) {
#pragma unroll
    for (int j = 0; j < 22; ++j) {
        d[j] = dec_unit4(lut, d[j]);
        bad |= d[j];
    }
    uint32_t w0[17];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int a = (4 * i) / 3, r = (4 * i) % 3;
        w0[i] = r == 0 ? (d[a] << 8) | (d[a + 1] >> 16) : r == 1 ? (d[a] << 16) | (d[a + 1] >> 8) : (d[a] << 24) | d[a + 1];
    }
    w0[16] = d[21] << 16;  // stream bytes 64, 65 (only a phase > 0 reaches them)
    const uint32_t be = 0x07060504u - ph * 0x01010101u, le = 0x04050607u - ph * 0x01010101u;
    uint32_t m[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        W[i] = __builtin_amdgcn_perm(w0[i], w0[i + 1], be);
        m[i] = __builtin_amdgcn_perm(w0[i], w0[i + 1], le);
    }
    const uint32_t lane = threadIdx.x & 63u;
    if (__ballot(1) == ~0ull) {  // the whole wave is in this block together
#pragma unroll
        for (int i = 0; i < 4; ++i) tile.v[lane][i] = make_uint4(m[4 * i], m[4 * i + 1], m[4 * i + 2], m[4 * i + 3]);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const uint32_t row = 16u * t + (lane >> 2), part = lane & 3u;
            const uint4 q = tile.v[row][part];
            *reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(tile.base[row]) + koff + 16u * part) = q;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        return;
    }
    uint4* o = reinterpret_cast<uint4*>(dst + koff);
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = make_uint4(m[4 * i], m[4 * i + 1], m[4 * i + 2], m[4 * i + 3]);
}

// KNOWN: the lane's decoded length n is given and its chars are the encoder's
// 4 * ceil(n / 3) (held replicas; status bit 1 reports a decoded length that
// is not n).  Otherwise (a received request body, SN:281) the length follows
// from the chars: len chars = whole units plus a final unit of 2 or 3 chars,
// or of 4 with padding; one dangling char is the decoder's error; out_len gets
// the decoded length (0 on error) and a failed message's digest is not written.
template <bool KNOWN>
__device__ __forceinline__ void b64dec_body(const char* __restrict__ in, const DecLane* __restrict__ lanes, uint32_t n,
                                            uint8_t* __restrict__ raw, uint8_t* __restrict__ digests,
                                            int32_t* __restrict__ status, uint64_t* __restrict__ out_len,
                                            uint32_t* __restrict__ queue) {
    __shared__ uint32_t lut[4 * 256];
    __shared__ DecTile tiles[kShaBlock / 64];
    DecTile& tile = tiles[threadIdx.x >> 6];
    for (uint32_t c = threadIdx.x; c < 256u; c += kShaBlock) {
        uint32_t v = 0x80000000u;
        if (c >= 'A' && c <= 'Z') v = c - 'A';
        else if (c >= 'a' && c <= 'z') v = c - 'a' + 26u;
        else if (c >= '0' && c <= '9') v = c - '0' + 52u;
        else if (c == '+') v = 62u;
        else if (c == '/') v = 63u;
        const bool ok = v < 64u;
        lut[c] = ok ? v << 18 : v;
        lut[256u + c] = ok ? v << 12 : v;
        lut[512u + c] = ok ? v << 6 : v;
        lut[768u + c] = v;
    }
    __syncthreads();
    const uint32_t nitems = (n + 63u) >> 6;
    const uint32_t lane = threadIdx.x & 63u;
    for (;;) {
        uint32_t item = 0;
        if (lane == 0) item = atomicAdd(queue + 1, 1u);
        item = __builtin_amdgcn_readfirstlane(item);
        if (item >= nitems) break;
        const uint32_t gid = item * 64u + lane;
        if (gid >= n) continue;
        const DecLane L = lanes[gid];
        const uint32_t* __restrict__ src = reinterpret_cast<const uint32_t*>(in + L.src);
        const uint8_t* __restrict__ ch8 = reinterpret_cast<const uint8_t*>(src);
        uint8_t* __restrict__ dst = raw + L.dst;
        tile.base[lane] = reinterpret_cast<uint64_t>(dst);  // read by the wave's other lanes in dec_block, after its fences
        // Units of 4 chars -> 3 bytes; the last one is the final unit: 4 chars
        // "xxxx" | "xxx=" | "xx==", or (unknown length only) 2 or 3 chars.
        const uint32_t r = KNOWN ? 0u : static_cast<uint32_t>(L.len & 3u);
        const uint64_t q = KNOWN ? (L.n + 2) / 3 : (L.len >> 2) + (r ? 1u : 0u);
        const uint64_t body = q ? 3 * (q - 1) : 0;  // bytes of the units before the final one
        bool err = !KNOWN && r == 1u;               // a dangling char
        uint32_t fin = 0, val = 0;
        if (q && !err) {
            const uint64_t f = 4 * (q - 1);
            const uint32_t d0 = lut[768u + ch8[f]], d1 = lut[768u + ch8[f + 1]];
            if (r == 0u) {
                const uint32_t c2 = ch8[f + 2], c3 = ch8[f + 3];
                const uint32_t d2 = lut[768u + c2], d3 = lut[768u + c3];
                if ((d0 | d1) >> 31) err = true;
                else if (c2 == '=' && c3 == '=') { fin = 1; val = (d0 << 18) | (d1 << 12); }
                else if (!(d2 >> 31) && c3 == '=') { fin = 2; val = (d0 << 18) | (d1 << 12) | (d2 << 6); }
                else if (!((d2 | d3) >> 31)) { fin = 3; val = (d0 << 18) | (d1 << 12) | (d2 << 6) | d3; }
                else err = true;
            } else {
                const uint32_t d2 = r == 3u ? lut[768u + ch8[f + 2]] : 0u;
                if ((d0 | d1 | d2) >> 31) err = true;
                fin = r - 1u;
                val = (d0 << 18) | (d1 << 12) | (d2 << 6);
            }
        }
        const uint64_t total = err ? 0 : body + fin;    // what the decoder returns
        const uint64_t len = KNOWN ? L.n : total;       // bytes written and hashed
        const bool skip = !KNOWN && err;                // nothing to decode: the request fails (SN:281)
        const uint64_t nfull = len >> 6;
        const uint32_t kb = static_cast<uint32_t>(nfull < (body >> 6) ? nfull : (body >> 6));  // blocks of body units only
        uint32_t st[8];
        init_state(st);
        uint32_t bad = 0;
        if (kb) {
            uint32_t A[22], B[22], W[16];
            const uint32_t last = kb - 1u;
            // unit index of block k's first unit: floor(64k / 3) = 21k + floor(k / 3)
            dec_load(src, A);
            uint32_t k = 0, ph = 0;
            const uint32_t* p = src;  // block k's first unit
            for (;;) {
                const uint32_t* pn = p + 21 + (ph == 2u ? 1 : 0);
                dec_load(k < last ? pn : p, B);
                dec_block(lut, A, ph, W, dst, 64ull * k, tile, bad);
                compress(st, W);
                if (++k >= kb) break;
                p = pn;
                ph = ph == 2u ? 0u : ph + 1u;
                pn = p + 21 + (ph == 2u ? 1 : 0);
                dec_load(k < last ? pn : p, A);
                dec_block(lut, B, ph, W, dst, 64ull * k, tile, bad);
                compress(st, W);
                if (++k >= kb) break;
                p = pn;
                ph = ph == 2u ? 0u : ph + 1u;
            }
        }
        // The rest, unit by unit into the raw buffer: body units from the one
        // holding byte 64 kb, then the final unit's bytes.
        const uint64_t pos = 64ull * kb;
        if (q && !skip) {
            for (uint64_t u = pos / 3; u + 1 < q; ++u) {
                const uint32_t v = dec_unit4(lut, src[u]);
                bad |= v;
#pragma unroll
                for (uint32_t t = 0; t < 3; ++t) {
                    const uint64_t i = 3 * u + t;
                    if (i >= pos) dst[i] = static_cast<uint8_t>(v >> (16 - 8 * t));
                }
            }
            for (uint32_t t = 0; t < fin; ++t) {
                const uint64_t i = body + t;
                if (i >= pos && i < len) dst[i] = static_cast<uint8_t>(val >> (16 - 8 * t));
            }
        }
        if (bad >> 31) err = true;
        // what this lane wrote, read back by its own loads below
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        ShaDesc sd{};
        sd.off = L.dst;
        sd.len = sd.total = len;
        const Msg m = msg_setup(raw, sd);
        if (kb < m.nfull) plain_range(st, m, kb, m.nfull);
        for (uint32_t tb = 0; tb < m.ntb; ++tb) {
            uint32_t W[16];
            tail_block(m, tb, W);
            compress(st, W);
        }
        if (KNOWN) {
            store_digest(st, L.out, ~0u, digests, digests);
            status[L.out] = (err ? 1 : 0) | (!err && total != L.n ? 2 : 0);
        } else {
            if (!err) store_digest(st, L.out, ~0u, digests, digests);
            status[L.out] = err ? 1 : 0;
            out_len[L.out] = err ? 0 : total;
        }
    }
}

__global__ __launch_bounds__(kShaBlock) void sha256_b64dec_lanes(const char* __restrict__ in,
                                                                  const DecLane* __restrict__ lanes, uint32_t n,
                                                                  uint8_t* __restrict__ raw,
                                                                  uint8_t* __restrict__ digests,
                                                                  int32_t* __restrict__ status,
                                                                  uint32_t* __restrict__ queue) {
    b64dec_body<true>(in, lanes, n, raw, digests, status, nullptr, queue);
}
__global__ __launch_bounds__(kShaBlock) void sha256_b64dec_any_lanes(const char* __restrict__ in,
                                                                      const DecLane* __restrict__ lanes, uint32_t n,
                                                                      uint8_t* __restrict__ raw,
                                                                      uint8_t* __restrict__ digests,
                                                                      int32_t* __restrict__ status,
                                                                      uint64_t* __restrict__ out_len,
                                                                      uint32_t* __restrict__ queue) {
    b64dec_body<false>(in, lanes, n, raw, digests, status, out_len, queue);
}

#define DFS_SHA_ARGS                                                                                     \
    const uint8_t *__restrict__ base, const ShaDesc *__restrict__ descs, uint32_t n, uint32_t split,       \
        uint32_t n_long, uint32_t cap, uint8_t *__restrict__ out0, uint8_t *__restrict__ out1,             \
        uint32_t *__restrict__ queue, uint32_t *__restrict__ state, char *__restrict__ b64, ShaWait wait
// Plain (hash only).  The pair-fetch block loop measured 76.6 ms alone on
// config 2 (78.8 ms with two register buffers, 79.4 ms with one compression
// per iteration); beside Base64 91.3 / 93.1 / 93.9 ms.
__global__ __launch_bounds__(kShaBlock) void sha256_lanes(DFS_SHA_ARGS) {
    sha256_body<false, false>(base, descs, n, split, n_long, cap, out0, out1, queue, state, b64, wait);
}
// Decode-ahead download (ShaWait): lanes wait in-kernel for fragment groups.
// Its own instantiation: the wait state costs VGPRs (157 vs 149), and the
// upload's SHA waves must leave room for the Base64 waves beside them.
__global__ __launch_bounds__(kShaBlock) void sha256_lanes_wait(DFS_SHA_ARGS) {
    sha256_body<false, true>(base, descs, n, split, n_long, cap, out0, out1, queue, state, b64, wait);
}
// Fused: fragment lanes flagged kShaB64 also write their Base64.
__global__ __launch_bounds__(kShaBlock) void sha256_lanes_b64(DFS_SHA_ARGS) {
    sha256_body<true, false>(base, descs, n, split, n_long, cap, out0, out1, queue, state, b64, wait);
}
#undef DFS_SHA_ARGS

// Latency-bound launch (n <= kChainMaxLanes).  Up to kChain2MaxLanes messages
// the pair-lane kernel (two owner lanes per message, 32 messages per owner
// wave), above that the one-lane kernel (64 per owner wave): either way at
// most one wave per SIMD.  DFS_SHA_CHAIN=1 forces the one-lane kernel (A/B
// measurements).
constexpr uint32_t kChain2MaxLanes = kChainMaxLanes / 2;

hipError_t launch_chain(const uint8_t* base, const ShaDesc* descs, uint32_t n, uint32_t split, uint8_t* out0,
                        uint8_t* out1, uint32_t* state, hipStream_t s) {
    static const bool one_lane = [] {
        const char* e = std::getenv("DFS_SHA_CHAIN");
        return e && e[0] == '1';
    }();
    // One wave pair per workgroup while that leaves at most one workgroup per
    // CU (256 CUs), two pairs above.
    if (n <= kChain2MaxLanes && !one_lane) {
        if (n <= 256u * kChain2Msgs)
            hipLaunchKernelGGL(sha256_chain2<1>, dim3((n + kChain2Msgs - 1u) / kChain2Msgs), dim3(kChainBlock), 0, s,
                               base, descs, n, split, out0, out1, state);
        else
            hipLaunchKernelGGL(sha256_chain2<2>, dim3((n + 2u * kChain2Msgs - 1u) / (2u * kChain2Msgs)),
                               dim3(2 * kChainBlock), 0, s, base, descs, n, split, out0, out1, state);
    } else if (n <= 256u * 64u) {
        hipLaunchKernelGGL(sha256_chain<1>, dim3((n + 63u) / 64u), dim3(kChainBlock), 0, s, base, descs, n, split,
                           out0, out1, state);
    } else {
        hipLaunchKernelGGL(sha256_chain<2>, dim3((n + 127u) / 128u), dim3(2 * kChainBlock), 0, s, base, descs, n,
                           split, out0, out1, state);
    }
    return hipGetLastError();
}

}  // namespace

int sha_wait_vgprs() {
    hipFuncAttributes a{};
    return hipFuncGetAttributes(&a, reinterpret_cast<const void*>(sha256_lanes_wait)) == hipSuccess ? a.numRegs : -1;
}

hipError_t launch_sha256(const uint8_t* base, const ShaDesc* descs, uint32_t n, uint32_t split,
                         uint32_t prio_lanes, uint8_t* out0, uint8_t* out1, uint32_t* queue, int waves_per_simd,
                         hipStream_t s, uint32_t* state, char* b64, const ShaWait* wait) {
    if (n == 0) return hipSuccess;
    if (!b64 && !wait && n <= kChainMaxLanes)  // latency-bound launch: owner + helper waves
        return launch_chain(base, descs, n, split, out0, out1, state, s);
    const ShaWait wt = wait && !b64 ? *wait : ShaWait{};
    if (!wait) {  // with a wait the caller zeroed the queue before the decode it waits on
        hipError_t e = hipMemsetAsync(queue, 0, kShaQueueBytes, s);
        if (e != hipSuccess) return e;
    }
    const uint32_t n_long = (prio_lanes + 63u) / 64u;
    const uint32_t cap = (n_long + 1023u) / 1024u;
    const uint64_t items = (n + 63u) / 64u;
    uint64_t waves = 1024ull * static_cast<uint64_t>(waves_per_simd < 1 ? 1 : waves_per_simd);
    if (waves > items && !n_long) waves = items;  // with long items the spare waves keep SIMDs balanced
    const uint32_t grid = static_cast<uint32_t>((waves + 3) / 4);
    if (b64) {
        hipLaunchKernelGGL(sha256_lanes_b64, dim3(grid), dim3(kShaBlock), 0, s, base, descs, n, split, n_long, cap,
                           out0, out1, queue, state, b64, ShaWait{});
    } else if (wt.done) {
        hipLaunchKernelGGL(sha256_lanes_wait, dim3(grid), dim3(kShaBlock), 0, s, base, descs, n, split, n_long, cap,
                           out0, out1, queue, state, nullptr, wt);
    } else {
        hipLaunchKernelGGL(sha256_lanes, dim3(grid), dim3(kShaBlock), 0, s, base, descs, n, split, n_long, cap, out0,
                           out1, queue, state, nullptr, wt);
    }
    return hipGetLastError();
}

hipError_t launch_sha256_b64dec(const char* in, const DecLane* lanes, uint32_t n, uint8_t* raw, uint8_t* digests,
                                int32_t* status, uint32_t* queue, int waves_per_simd, hipStream_t s, uint64_t* out_len) {
    if (n == 0) return hipSuccess;
    hipError_t e = launch_fill_u32(queue, 64, 0u, s);
    if (e != hipSuccess) return e;
    const uint64_t items = (n + 63u) / 64u;
    uint64_t waves = 1024ull * static_cast<uint64_t>(waves_per_simd < 1 ? 1 : waves_per_simd);
    if (waves > items) waves = items;
    const dim3 grid(static_cast<uint32_t>((waves + 3) / 4));
    if (out_len)
        hipLaunchKernelGGL(sha256_b64dec_any_lanes, grid, dim3(kShaBlock), 0, s, in, lanes, n, raw, digests, status, out_len,
                           queue);
    else
        hipLaunchKernelGGL(sha256_b64dec_lanes, grid, dim3(kShaBlock), 0, s, in, lanes, n, raw, digests, status, queue);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Allocation-free SHA-256 batch (dfs_sha256_batch_static): the lane
// descriptors and the persistent kernel's queue words live in a file-scope
// device array instead of the ctx's hipMalloc'ed scratch.  Every GPU holds
// its own copy of the array until the process ends; its address on a device
// is resolved once (static_scratch_init, with that device current) and host
// code uses only that address, never the array's name.  All calls on one GPU
// share the array: calls that overlap on a GPU race.
namespace {

constexpr size_t kStaticDescBytes = static_cast<size_t>(kStaticMaxMsgs) * sizeof(ShaDesc);
static_assert(kStaticDescBytes % 256 == 0, "queue words start 256-byte aligned");
constexpr size_t kStaticBytes = kStaticDescBytes + kShaQueueBytes;

static __device__ __align__(256) uint8_t scratch[kStaticBytes];

constexpr int kStaticMaxDevices = 64;
std::mutex g_static_mu;
void* g_static_ptr[kStaticMaxDevices] = {};

// Span i ({off, len} pairs in device memory) -> lane descriptor i; clears
// the queue words (a fill kernel, so the sequence may sit in a captured graph).
__global__ __launch_bounds__(256) void static_prep_kernel(const uint64_t* __restrict__ msgs, uint32_t n,
                                                         ShaDesc* __restrict__ descs, uint32_t* __restrict__ queue,
                                                         int32_t* __restrict__ status) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i < kShaQueueBytes / 4) queue[i] = 0u;
    if (i >= n) return;
    const uint64_t off = msgs[2ull * i], len = msgs[2ull * i + 1];
    const bool bad = len >= (1ull << 37);  // nfull = len / 64 must fit 32 bits
    ShaDesc d;
    d.off = off;
    d.len = d.total = bad ? 0ull : len;
    d.out = i;
    d.flags = 0u;
    d.b64 = 0ull;
    descs[i] = d;
    if (status) status[i] = bad ? -1 : 0;
}

}  // namespace

hipError_t static_scratch_init(int device) {
    if (device < 0 || device >= kStaticMaxDevices) return hipErrorInvalidDevice;
    std::lock_guard<std::mutex> lk(g_static_mu);
    if (g_static_ptr[device]) return hipSuccess;
    void* p = nullptr;
    const hipError_t e = hipGetSymbolAddress(&p, HIP_SYMBOL(scratch));  // the current device's copy
    if (e != hipSuccess) return e;
    if (!p) return hipErrorInvalidSymbol;
    g_static_ptr[device] = p;
    return hipSuccess;
}

hipError_t launch_sha256_static(int device, const uint8_t* base, const uint64_t* d_msgs, uint32_t n, uint8_t* out,
                                int32_t* status, int waves_per_simd, hipStream_t s) {
    if (n == 0) return hipSuccess;
    if (n > kStaticMaxMsgs || device < 0 || device >= kStaticMaxDevices) return hipErrorInvalidValue;
    uint8_t* ptr;
    {
        std::lock_guard<std::mutex> lk(g_static_mu);
        ptr = static_cast<uint8_t*>(g_static_ptr[device]);
    }
    if (!ptr) return hipErrorNotInitialized;
    ShaDesc* descs = reinterpret_cast<ShaDesc*>(ptr);
    uint32_t* queue = reinterpret_cast<uint32_t*>(ptr + kStaticDescBytes);
    const uint32_t work = n > kShaQueueBytes / 4 ? n : static_cast<uint32_t>(kShaQueueBytes / 4);
    hipLaunchKernelGGL(static_prep_kernel, dim3((work + 255u) / 256u), dim3(256), 0, s, d_msgs, n, descs, queue,
                       status);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (n <= kChainMaxLanes) {
        return launch_chain(base, descs, n, n, out, out, nullptr, s);
    } else {  // unsorted lanes, no long items: every wave pulls from the short queue
        const uint64_t items = (n + 63u) / 64u;
        uint64_t waves = 1024ull * static_cast<uint64_t>(waves_per_simd < 1 ? 1 : waves_per_simd);
        if (waves > items) waves = items;
        hipLaunchKernelGGL(sha256_lanes, dim3(static_cast<uint32_t>((waves + 3) / 4)), dim3(kShaBlock), 0, s, base,
                           descs, n, n, 0u, 0u, out, out, queue, nullptr, nullptr, ShaWait{});
    }
    return hipGetLastError();
}

}  // namespace dfs
