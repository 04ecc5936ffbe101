// base64.hip — RFC 4648 Base64 encode / decode for gfx950 (MI355X).
//
// Encode replaces Base64.getEncoder().encodeToString(f.data) inside
// buildFragmentsJson (StorageNode.java:636); decode replaces
// Base64.getDecoder().decode(fragInfo.get("data")) in
// handleInternalStoreFragments (StorageNode.java:281), including the JDK
// basic decoder's IllegalArgumentException cases.
//
// Both kernels are HBM-bound byte streams: 12 input bytes
// -> 16 chars per lane-step, 64 lanes of a wave touch 768 contiguous input
// bytes and 1 KiB of contiguous output, the 6-bit -> ASCII map (and its
// inverse) is a table in LDS, and misaligned starts are fixed in registers
// with v_alignbyte / v_perm so every global access is dword aligned.
#include "stream_common.h"

namespace dfs {
namespace {

__constant__ uint32_t kAlphaWords[16] = {
    // "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/" as LE words
    0x44434241u, 0x48474645u, 0x4c4b4a49u, 0x504f4e4du, 0x54535251u, 0x58575655u, 0x62615a59u, 0x66656463u,
    0x6a696867u, 0x6e6d6c6bu, 0x7271706fu, 0x76757473u, 0x7a797877u, 0x33323130u, 0x37363534u, 0x2f2b3938u};

__device__ __forceinline__ uint32_t align_bytes(uint32_t hi, uint32_t lo, uint32_t s) {
    return __builtin_amdgcn_alignbyte(hi, lo, s);
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// 64-entry alphabet as LE words (kAlphaWords) expanded to a 4,096-entry
// table of character PAIRS: pair[k] = alpha[k >> 6] | alpha[k & 63] << 8, so
// one 24-bit group is two LDS reads (its high and low 12 bits) and no
// per-character shifts/masks.  8 KiB per workgroup, built once per
// (persistent) workgroup.
__device__ __forceinline__ void build_pair_lut(uint16_t* pair) {
    const uint8_t* a = reinterpret_cast<const uint8_t*>(kAlphaWords);
    for (uint32_t k = threadIdx.x; k < 4096u; k += blockDim.x)
        pair[k] = static_cast<uint16_t>(a[k >> 6] | (static_cast<uint32_t>(a[k & 63u]) << 8));
}

// x + x on the full-rate adder (the compiler would emit v_lshlrev_b32, a
// half-rate op on gfx950: tools/valu_peak).
__device__ __forceinline__ uint32_t dbl(uint32_t x) {
    uint32_t r;
    asm("v_add_u32_e32 %0, %1, %1" : "=v"(r) : "v"(x));
    return r;
}

// Four ASCII chars (first char in the low byte) of the 24-bit group v:
// byte addresses 2*(v>>12) and 2*(v&0xfff) into the pair table.
__device__ __forceinline__ uint32_t enc4_pair(const uint16_t* __restrict__ pair, uint32_t v) {
    const char* p = reinterpret_cast<const char*>(pair);
    const uint32_t hi = *reinterpret_cast<const uint16_t*>(p + ((v >> 11) & 0x1ffeu));
    const uint32_t lo = *reinterpret_cast<const uint16_t*>(p + dbl(v & 0xfffu));
    return __builtin_amdgcn_perm(lo, hi, 0x05040100u);
}

// perm selector that yields the big-endian 24-bit group at byte position p
// of the 16 raw bytes {raw[d], raw[d+1]} (d = p / 4).
constexpr uint32_t grp_sel(int p) {
    return static_cast<uint32_t>((p + 2) - 4 * (p / 4)) | (static_cast<uint32_t>((p + 1) - 4 * (p / 4)) << 8) |
           (static_cast<uint32_t>(p - 4 * (p / 4)) << 16) | (0x0cu << 24);
}
template <int P>
__device__ __forceinline__ uint32_t grp(const uint32_t (&raw)[4]) {
    constexpr int d = P / 4;
    return __builtin_amdgcn_perm(d + 1 < 4 ? raw[d + 1 < 4 ? d + 1 : 3] : 0u, raw[d], grp_sel(P));
}

// One tile of full 12-byte groups whose source starts SA bytes past a dword
// boundary.  tsrc (dword aligned, = first group - SA) and tdst are uniform;
// every per-lane address is a constant 32-bit offset from them.
template <int SA>
__device__ __forceinline__ void enc_tile(const uint32_t* __restrict__ tsrc, uint8_t* __restrict__ tdst,
                                         int64_t left, const uint16_t* __restrict__ pair) {
    constexpr int PER = kEncPer;
    uint32_t raw[PER][4];
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const uint32_t lg = threadIdx.x + static_cast<uint32_t>(i) * kStreamBlock;
        raw[i][0] = raw[i][1] = raw[i][2] = raw[i][3] = 0u;
        if (static_cast<int64_t>(lg) < left) {
            const uint32_t* w = tsrc + 3u * lg;
            if (SA) {
                const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(w));
                raw[i][0] = v.x; raw[i][1] = v.y; raw[i][2] = v.z; raw[i][3] = v.w;
            } else {
                raw[i][0] = __builtin_nontemporal_load(w);
                raw[i][1] = __builtin_nontemporal_load(w + 1);
                raw[i][2] = __builtin_nontemporal_load(w + 2);
            }
        }
    }
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const uint32_t lg = threadIdx.x + static_cast<uint32_t>(i) * kStreamBlock;
        if (static_cast<int64_t>(lg) < left) {
            uint32_t g[4] = {grp<SA>(raw[i]), grp<SA + 3>(raw[i]), grp<SA + 6>(raw[i]), grp<SA + 9>(raw[i])};
            const u32x4 o{enc4_pair(pair, g[0]), enc4_pair(pair, g[1]), enc4_pair(pair, g[2]), enc4_pair(pair, g[3])};
            __builtin_nontemporal_store(o, reinterpret_cast<u32x4*>(tdst + 16u * lg));
        }
    }
}

// kEncPer groups per thread per tile (tile = 4 x 256 groups); loads and
// stores are non-temporal (streaming): this pass touches every byte once.
// The 12-bit pair table costs 2 LDS reads + 5 VALU per group (a 6-bit
// alphabet would be 4 LDS reads + ~10 VALU).
__global__ __launch_bounds__(kStreamBlock) void b64_encode_kernel(const uint8_t* __restrict__ base,
                                                                  const StreamJob* __restrict__ jobs,
                                                                  uint32_t njobs, uint64_t ntiles,
                                                                  char* __restrict__ out, uint32_t prio) {
    // Memory-bound waves issue first: beside the VALU-bound SHA kernel they
    // need few issue slots but must keep their loads in flight.
    switch (prio) {  // s_setprio takes an immediate
        case 0: break;
        case 1: __builtin_amdgcn_s_setprio(1); break;
        case 2: __builtin_amdgcn_s_setprio(2); break;
        default: __builtin_amdgcn_s_setprio(3); break;
    }
    __shared__ uint16_t pair[4096];
    build_pair_lut(pair);
    __syncthreads();

    uint64_t t0, t1;
    tile_range(ntiles, t0, t1);
    if (t0 >= t1) return;
    uint32_t j = find_job(jobs, njobs, t0);
    for (uint64_t t = t0; t < t1; ++t) {
        while (jobs[j + 1].tile_start <= t) ++j;
        const uint64_t len = jobs[j].len;
        const uint64_t nfg = len / 12;  // full 12-byte groups
        const uint32_t rem = static_cast<uint32_t>(len - 12 * nfg);
        const uint8_t* __restrict__ src = base + jobs[j].src_off;
        uint8_t* __restrict__ dst = reinterpret_cast<uint8_t*>(out) + jobs[j].dst_off;
        const uint32_t sa = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(src)) & 3u;
        const uint64_t tg = (t - jobs[j].tile_start) * (kEncPer * kStreamBlock);  // first group of the tile
        const int64_t left = static_cast<int64_t>(nfg) - static_cast<int64_t>(tg);
        const uint32_t* tsrc = reinterpret_cast<const uint32_t*>(src + 12 * tg - sa);
        uint8_t* tdst = dst + 16 * tg;
        switch (sa) {  // wave-uniform
            case 0: enc_tile<0>(tsrc, tdst, left, pair); break;
            case 1: enc_tile<1>(tsrc, tdst, left, pair); break;
            case 2: enc_tile<2>(tsrc, tdst, left, pair); break;
            default: enc_tile<3>(tsrc, tdst, left, pair); break;
        }
        // Last partial group: full triples then "==" / "=" padding (RFC 4648 §4).
        if (rem && left >= 0 && left < kEncPer * kStreamBlock && threadIdx.x == static_cast<uint32_t>(left) % kStreamBlock) {
            uint32_t* o = reinterpret_cast<uint32_t*>(dst + 16 * nfg);
            const uint8_t* s = src + 12 * nfg;
            for (uint32_t k = 0; k < rem; k += 3) {
                const uint32_t n = rem - k < 3 ? rem - k : 3;
                uint32_t v = static_cast<uint32_t>(s[k]) << 16;
                if (n > 1) v |= static_cast<uint32_t>(s[k + 1]) << 8;
                if (n > 2) v |= s[k + 2];
                uint32_t wv = enc4_pair(pair, v);
                if (n == 1) wv = (wv & 0x0000ffffu) | 0x3d3d0000u;  // "xx=="
                else if (n == 2) wv = (wv & 0x00ffffffu) | 0x3d000000u;  // "xxx="
                o[k / 3] = wv;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Decode (geometry: dec_geom in dfs_internal.h).
// Message of L chars: q = L/4 full units, r = L%4.
//   r == 1           -> IllegalArgumentException (dangling char / bad ending)
//   r == 2, 3        -> q body units + a final unit of r alphabet chars
//   r == 0, q >= 1   -> q-1 body units + a final unit "xxxx" | "xxx=" | "xx=="
// Body units must be 4 alphabet chars.  Output byte i goes to dst + i.
// ---------------------------------------------------------------------------
// 6-bit value of each char; 0xFF for anything outside the alphabet ('=' too).
__device__ __forceinline__ void build_dec_lut(uint8_t* lut) {
    for (uint32_t c = threadIdx.x; c < 256; c += blockDim.x) {
        uint32_t v = 0xFFu;
        if (c >= 'A' && c <= 'Z') v = c - 'A';
        else if (c >= 'a' && c <= 'z') v = c - 'a' + 26;
        else if (c >= '0' && c <= '9') v = c - '0' + 52;
        else if (c == '+') v = 62;
        else if (c == '/') v = 63;
        lut[c] = static_cast<uint8_t>(v);
    }
}

// Decode the 4 chars (LE word) of one unit: returns 24-bit value, ORs the raw
// lookups into `bad` (bit 7+ set iff a char is outside the alphabet).
__device__ __forceinline__ uint32_t dec_unit(const uint8_t* __restrict__ lut, uint32_t w, uint32_t& bad) {
    const uint32_t d0 = lut[w & 255u], d1 = lut[(w >> 8) & 255u], d2 = lut[(w >> 16) & 255u], d3 = lut[w >> 24];
    bad |= d0 | d1 | d2 | d3;
    return (d0 << 18) | (d1 << 12) | (d2 << 6) | d3;
}

// Value of char at index i of a message (tail path, byte loads).
__device__ __forceinline__ uint32_t dec_char(const uint8_t* __restrict__ lut, const uint8_t* s, uint64_t i) {
    return lut[s[i]];
}

__device__ __forceinline__ uint32_t dec_unit_bytes(const uint8_t* __restrict__ lut, const uint8_t* s, uint64_t u,
                                                   uint32_t& bad) {
    const uint32_t d0 = lut[s[4 * u]], d1 = lut[s[4 * u + 1]], d2 = lut[s[4 * u + 2]], d3 = lut[s[4 * u + 3]];
    bad |= d0 | d1 | d2 | d3;
    return (d0 << 18) | (d1 << 12) | (d2 << 6) | d3;
}

// Tail step of one message, run by the 64 lanes of one wave: validates the
// body units no tile owns (at most 8: before u_first and after the last whole
// group), decodes the final unit (every lane, same address: a broadcast
// load), writes the head bytes [0, h) and tail bytes [h + 16 nchunks, total)
// — at most 15 + 28, one byte per lane, all loads in flight at once — and
// sets status / out_len (SN:281's IllegalArgumentException cases: a char
// outside the alphabet, a 1-char final unit, wrong padding).
__device__ __forceinline__ void dec_tail(const uint8_t* __restrict__ lut, const StreamJob& job, const DecGeom& G,
                                      const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                      int32_t* __restrict__ status, uint64_t* __restrict__ out_len) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t L = job.len;
    const uint32_t r = static_cast<uint32_t>(L & 3u);
    bool err = (r == 1u);
    // Units outside the tiles: [0, u_first) and [covered_end, body_units).
    const uint64_t covered_end = G.u_first + 4 * G.ng;
    const uint64_t head_units = G.u_first < G.body_units ? G.u_first : G.body_units;
    const uint64_t u = lane < head_units ? lane : covered_end + (lane - head_units);
    uint32_t bad = 0;
    if (u < G.body_units && (lane < head_units || u >= covered_end)) dec_unit_bytes(lut, src, u, bad);
    if (__ballot((bad & 0x80u) != 0)) err = true;
    uint32_t fin_bytes = 0, fin_val = 0;
    if (!err && L) {
        const uint64_t f = 4 * G.body_units;  // first char of the final unit
        if (r == 0) {
            const uint32_t c2 = src[f + 2], c3 = src[f + 3];
            const uint32_t d0 = dec_char(lut, src, f), d1 = dec_char(lut, src, f + 1);
            const uint32_t d2 = lut[c2], d3 = lut[c3];
            if ((d0 | d1) & 0x80u) err = true;
            else if (c2 == '=' && c3 == '=') { fin_bytes = 1; fin_val = (d0 << 18) | (d1 << 12); }
            else if (!(d2 & 0x80u) && c3 == '=') { fin_bytes = 2; fin_val = (d0 << 18) | (d1 << 12) | (d2 << 6); }
            else if (!((d2 | d3) & 0x80u)) { fin_bytes = 3; fin_val = (d0 << 18) | (d1 << 12) | (d2 << 6) | d3; }
            else err = true;
        } else {  // r == 2 or 3: unpadded final unit
            const uint32_t d0 = dec_char(lut, src, f), d1 = dec_char(lut, src, f + 1);
            const uint32_t d2 = r == 3 ? dec_char(lut, src, f + 2) : 0u;
            if ((d0 | d1 | d2) & 0x80u) err = true;
            fin_bytes = r - 1;
            fin_val = (d0 << 18) | (d1 << 12) | (d2 << 6);
        }
    }
    const uint64_t total = err ? 0 : G.nb + fin_bytes;
    if (!err) {
        // Lane i < 16: head byte i; lane i >= 16: tail byte tail_start + i - 16.
        const uint64_t head_end = G.h < total ? G.h : total;
        const uint64_t tail_start = G.h + 16 * G.nchunks > head_end ? G.h + 16 * G.nchunks : head_end;
        const uint64_t i = lane < 16 ? lane : tail_start + (lane - 16);
        if (lane < 16 ? i < head_end : i < total) {
            const uint64_t q = i / 3;
            uint32_t b2 = 0;
            const uint32_t v = (q < G.body_units) ? dec_unit_bytes(lut, src, q, b2) : fin_val;
            dst[i] = static_cast<uint8_t>(v >> (16 - 8 * static_cast<uint32_t>(i % 3)));
        }
    }
    if (lane == 0) {
        int32_t flags = err ? 1 : 0;
        if (job.expect && !err && total + 1 != job.expect) flags |= 2;
        if (flags) atomicOr(status + job.id, flags);
        if (out_len) out_len[job.id] = total;
    }
}

// One tile = GPL x 256 4-unit groups (GPL = 8: 32 KiB of chars -> 24 KiB of
// output).  Phase 1: lane l loads groups 256i + l (i < GPL) with one dwordx4
// each (a wave reads 1 KiB contiguous per instruction, all eight loads in
// flight), decodes them through the LDS alphabet and parks the 12 bytes of
// each at LDS offset 12 * group.  Phase 2: lane l cuts 16-byte output chunks
// 256i + l (i < 3) out of the decoded stream at byte offset e and writes
// each with one dwordx4 store at a 16-byte aligned address (a wave writes
// 1 KiB contiguous per instruction).  Head, tail and final unit: dec_tail,
// on wave 0 of the message's last tile.  Loads and stores are non-temporal.
// dec_range decodes tiles [t0, t1) of the job table.
__device__ __forceinline__ void dec_range(const uint8_t* __restrict__ lut, uint32_t* __restrict__ stream,
                                          const char* __restrict__ in, const StreamJob* __restrict__ jobs,
                                          uint32_t njobs, uint8_t* __restrict__ out, int32_t* __restrict__ status,
                                          uint64_t* __restrict__ out_len, uint64_t t0, uint64_t t1) {
    constexpr int GPL = kDecGpl;
    constexpr uint32_t kGroups = GPL * kStreamBlock;  // 4-unit groups per tile
    constexpr uint32_t kChunks = 3 * GPL * 64;        // 16-byte output chunks per tile (12 kGroups / 16)
    if (t0 >= t1) return;
    uint32_t j = find_job(jobs, njobs, t0);
    for (uint64_t t = t0; t < t1; ++t) {
        while (jobs[j + 1].tile_start <= t) ++j;
        const uint8_t* __restrict__ src = reinterpret_cast<const uint8_t*>(in) + jobs[j].src_off;
        uint8_t* __restrict__ dst = out + jobs[j].dst_off;
        const DecGeom G = dec_geom(jobs[j].len, reinterpret_cast<uintptr_t>(dst));
        const uint32_t sa = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(src)) & 3u;
        const uint64_t k = t - jobs[j].tile_start;
        const uint64_t g0 = k * kGroups;  // first group of the tile
        // Group g's chars start at unit u_first + 4g, i.e. dword w0 + 4g.
        const uint32_t* w0 = reinterpret_cast<const uint32_t*>(src + 4 * G.u_first - sa);
        uint32_t raw[GPL][5];
#pragma unroll
        for (int i = 0; i < GPL; ++i) {
            const uint64_t g = g0 + threadIdx.x + static_cast<uint64_t>(i) * kStreamBlock;
            raw[i][0] = raw[i][1] = raw[i][2] = raw[i][3] = raw[i][4] = 0u;
            if (g < G.ng) {
                const uint32_t* w = w0 + 4 * g;
                const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(w));
                raw[i][0] = v.x; raw[i][1] = v.y; raw[i][2] = v.z; raw[i][3] = v.w;
                if (sa) raw[i][4] = __builtin_nontemporal_load(w + 4);
            }
        }
        uint32_t bad = 0;
#pragma unroll
        for (int i = 0; i < GPL; ++i) {
            const uint32_t gl = threadIdx.x + static_cast<uint32_t>(i) * kStreamBlock;  // group in the tile
            if (g0 + gl < G.ng) {
                uint32_t v[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) v[q] = dec_unit(lut, align_bytes(raw[i][q + 1], raw[i][q], sa), bad);
                stream[3 * gl] = __builtin_amdgcn_perm(v[1], v[0], 0x06000102u);
                stream[3 * gl + 1] = __builtin_amdgcn_perm(v[2], v[1], 0x05060001u);
                stream[3 * gl + 2] = __builtin_amdgcn_perm(v[3], v[2], 0x04050600u);
            }
        }
        // The tile's last chunk reaches e bytes into the next group's first
        // unit (a body unit whenever that chunk exists); its chars are
        // validated by the tile that owns it.
        const uint64_t c0 = k * kChunks;  // first chunk of the tile
        if (threadIdx.x == 0 && G.e && c0 + kChunks <= G.nchunks) {
            uint32_t b2 = 0;
            const uint32_t v = dec_unit_bytes(lut, src, G.u_first + 4 * (g0 + kGroups), b2);
            stream[3 * kGroups] = __builtin_amdgcn_perm(0u, v, 0x0c000102u);
        }
        if (bad & 0x80u) atomicOr(status + jobs[j].id, 1);
        __syncthreads();
#pragma unroll
        for (int i = 0; i < (kChunks + kStreamBlock - 1) / kStreamBlock; ++i) {
            const uint32_t m = threadIdx.x + static_cast<uint32_t>(i) * kStreamBlock;  // chunk in the tile
            if ((kChunks % kStreamBlock == 0 || m < kChunks) && c0 + m < G.nchunks) {
                const u32x4 a = *reinterpret_cast<const u32x4*>(stream + 4 * m);
                const uint32_t n4 = G.e ? stream[4 * m + 4] : 0u;
                const u32x4 o = u32x4{align_bytes(a.y, a.x, G.e), align_bytes(a.z, a.y, G.e),
                                      align_bytes(a.w, a.z, G.e), align_bytes(n4, a.w, G.e)};
                __builtin_nontemporal_store(o, reinterpret_cast<u32x4*>(dst + G.h + 16 * (c0 + m)));
            }
        }
        if (threadIdx.x < 64 && t + 1 == jobs[j + 1].tile_start)  // wave 0 of the message's last tile
            dec_tail(lut, jobs[j], G, src, dst, status, out_len);
        __syncthreads();  // stream[] is rewritten by the next tile
    }
}

template <bool AHEAD>
__global__ __launch_bounds__(kStreamBlock) void b64_decode_kernel(const char* __restrict__ in,
                                                                  const StreamJob* __restrict__ jobs,
                                                                  uint32_t njobs, uint64_t ntiles,
                                                                  uint8_t* __restrict__ out,
                                                                  int32_t* __restrict__ status,
                                                                  uint64_t* __restrict__ out_len, uint32_t prio,
                                                                  const uint64_t* __restrict__ gtile, uint32_t ngroups,
                                                                  uint32_t* __restrict__ gdone) {
    if (prio) __builtin_amdgcn_s_setprio(3);  // beside the SHA kernel (pipelined / overlapped download)
    constexpr uint32_t kGroups = kDecGpl * kStreamBlock;
    __shared__ uint8_t lut[256];
    __shared__ uint32_t stream[kGroups * 3 + 4];  // decoded bytes of the tile (+1 unit)
    build_dec_lut(lut);
    __syncthreads();

    if (!AHEAD) {
        uint64_t t0, t1;
        tile_range(ntiles, t0, t1);
        dec_range(lut, stream, in, jobs, njobs, out, status, out_len, t0, t1);
        return;
    }
    // Decode-ahead (dfs_download_batch, overlap mode): fragment groups in
    // order — every workgroup decodes its share of group g's tiles
    // [gtile[g], gtile[g+1]), then publishes it: its stores drained and
    // written back to memory at agent scope (release) before one lane adds 1
    // to gdone[g].  The SHA kernel beside it reads group g once gdone[g]
    // equals the grid size (then acquires).  This kernel never waits.
    const uint64_t G = gridDim.x, b = blockIdx.x;
    for (uint32_t g = 0; g < ngroups; ++g) {
        const uint64_t a = gtile[g], n = gtile[g + 1] - a;
        dec_range(lut, stream, in, jobs, njobs, out, status, out_len, a + n * b / G, a + n * (b + 1) / G);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_fetch_add(gdone + g, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
}

}  // namespace

int dec_ahead_vgprs() {
    hipFuncAttributes a{};
    return hipFuncGetAttributes(&a, reinterpret_cast<const void*>(b64_decode_kernel<true>)) == hipSuccess ? a.numRegs
                                                                                                        : -1;
}

hipError_t launch_b64_encode(const uint8_t* base, const StreamJob* jobs, uint32_t njobs, uint64_t ntiles, char* out,
                             uint32_t wgs_per_cu, hipStream_t s, uint32_t prio) {
    if (ntiles == 0) return hipSuccess;
    hipLaunchKernelGGL(b64_encode_kernel, dim3(stream_grid(ntiles, wgs_per_cu)), dim3(kStreamBlock), 0, s, base, jobs,
                       njobs, ntiles, out, prio);
    return hipGetLastError();
}

hipError_t launch_b64_decode(const char* in, const StreamJob* jobs, uint32_t njobs, uint64_t ntiles, uint8_t* out,
                             int32_t* status, uint64_t* out_len, hipStream_t s, uint32_t prio, uint32_t wgs_per_cu,
                             const StreamAhead* ahead) {
    if (ahead) {  // every workgroup takes part in every group (gdone counts workgroups)
        hipLaunchKernelGGL(b64_decode_kernel<true>, dim3(ahead->grid), dim3(kStreamBlock), 0, s, in, jobs, njobs, ntiles,
                           out, status, out_len, prio, ahead->gtile, ahead->ngroups, ahead->gdone);
        return hipGetLastError();
    }
    if (ntiles == 0) return hipSuccess;
    hipLaunchKernelGGL(b64_decode_kernel<false>, dim3(stream_grid(ntiles, wgs_per_cu)), dim3(kStreamBlock), 0, s, in,
                       jobs, njobs, ntiles, out, status, out_len, prio, nullptr, 0u, nullptr);
    return hipGetLastError();
}

}  // namespace dfs

// ---------------------------------------------------------------------------
// storeFragments body framing (buildFragmentsJson, StorageNode.java:629-642):
//   {"fileId":"<64 hex>","fragments":[{"index":"a","data":"<B1 chars>"},
//    {"index":"b","data":"<B2 chars>"}]}
// 139 framing bytes around two Base64 payloads (written by the encode
// kernel at body + 111 and body + 135 + B1).  One thread per framing byte.
// ---------------------------------------------------------------------------
namespace dfs {
namespace {

__constant__ char kBodyPrefix[] = "{\"fileId\":\"0123456789012345678901234567890123456789012345678901234567890123"
                                  "\",\"fragments\":[{\"index\":\"0\",\"data\":\"";
__constant__ char kBodyMid[] = "\"},{\"index\":\"0\",\"data\":\"";
__constant__ char kBodySuffix[] = "\"}]}";

__global__ __launch_bounds__(256) void store_body_frame_kernel(const StoreBody* __restrict__ bodies, uint32_t n,
                                                               const uint8_t* __restrict__ digests,
                                                               char* __restrict__ out) {
    const uint64_t g = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    const uint64_t k = g / kBodyFrameBytes;
    if (k >= n) return;
    const uint32_t p = static_cast<uint32_t>(g - k * kBodyFrameBytes);
    const StoreBody B = bodies[k];
    char c;
    uint64_t at;
    if (p < kBodyDataA) {
        at = p;
        if (p >= 11 && p < 75) {  // fileId hex, lowercase %02x (SN:607-609)
            const uint32_t byte = digests[32ull * B.file + (p - 11) / 2];
            const uint32_t nib = (p & 1u) ? (byte >> 4) : (byte & 15u);  // p = 11 -> high nibble
            c = static_cast<char>(nib < 10 ? '0' + nib : 'a' + nib - 10);
        } else if (p == kBodyDataA - 11) {
            c = static_cast<char>('0' + B.a);
        } else {
            c = kBodyPrefix[p];
        }
    } else if (p < kBodyDataA + kBodyMidBytes) {
        const uint32_t q = p - kBodyDataA;
        at = kBodyDataA + B.len_a + q;
        c = (q == kBodyMidBytes - 11) ? static_cast<char>('0' + B.b) : kBodyMid[q];
    } else {
        const uint32_t q = p - kBodyDataA - kBodyMidBytes;
        at = kBodyDataA + kBodyMidBytes + B.len_a + B.len_b + q;
        c = kBodySuffix[q];
    }
    out[B.dst + at] = c;
}

}  // namespace

hipError_t launch_store_body_frame(const StoreBody* bodies, uint32_t n, const uint8_t* digests, char* out,
                                   hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint64_t threads = static_cast<uint64_t>(n) * kBodyFrameBytes;
    hipLaunchKernelGGL(store_body_frame_kernel, dim3(static_cast<uint32_t>((threads + 255) / 256)), dim3(256), 0, s,
                       bodies, n, digests, out);
    return hipGetLastError();
}

}  // namespace dfs

// ---------------------------------------------------------------------------
// storeFragments body parse (receiver, handleInternalStoreFragments
// SN:265-279 / parseJson SN:704-753) for bodies in buildFragmentsJson's exact
// form: two entries with one-digit indices.  One wave per body checks the
// framing bytes and finds each payload's closing quote with a wave-wide scan
// (16 bytes per lane per step, dword compares, first hit by ballot).  A body
// in any other form gets status 1 and is left to the host's parseJson.
// ---------------------------------------------------------------------------
namespace dfs {
namespace {

// First '"' at or after body position `from` (< L), or L if none.  Loads are
// 16-byte aligned blocks that start inside [body, body + L), so they never
// cross a page the body does not touch.
__device__ uint64_t scan_quote(const char* __restrict__ body, uint64_t from, uint64_t L) {
    const uint32_t lane = threadIdx.x & 63u;
    const uintptr_t b = reinterpret_cast<uintptr_t>(body);
    uintptr_t blk = (b + from) & ~static_cast<uintptr_t>(15);
    for (; blk < b + L; blk += 1024) {
        const uintptr_t my = blk + 16u * lane;
        uint32_t hit = 16;  // byte index of the first quote in my block
        if (my < b + L) {
            const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(my));
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int q = 3; q >= 0; --q) {
                uint32_t y = w[q] ^ 0x22222222u;
                // bytes before `from` never match
                const intptr_t lo = static_cast<intptr_t>(b + from) - static_cast<intptr_t>(my + 4 * q);
                if (lo >= 4) y = 0xffffffffu;
                else if (lo > 0) y |= (1u << (8 * lo)) - 1u;
                const uint32_t z = (y - 0x01010101u) & ~y & 0x80808080u;
                if (z) hit = 4 * q + (__builtin_ctz(z) >> 3);
            }
        }
        const uint64_t m = __ballot(hit < 16);
        if (m) {
            const uint32_t first = __builtin_ctzll(m);
            const uint32_t h = __shfl(hit, first, 64);
            const uint64_t pos = (blk + 16u * first + h) - b;
            return pos < L ? pos : L;
        }
    }
    return L;
}

// Wave-parallel compare of n framing bytes at body + at with text (digit
// placeholders '0' at index dpos match any decimal digit).
__device__ bool frame_ok(const char* __restrict__ body, uint64_t at, const char* text, uint32_t n, uint32_t dpos) {
    const uint32_t lane = threadIdx.x & 63u;
    bool ok = true;
    for (uint32_t i = lane; i < n; i += 64) {
        const char c = body[at + i];
        ok &= (i == dpos) ? (c >= '0' && c <= '9') : (c == text[i]);
    }
    return __ballot(!ok) == 0;
}

__global__ __launch_bounds__(256) void store_body_parse_kernel(const char* __restrict__ in,
                                                               const uint64_t* __restrict__ spans, uint32_t n,
                                                               BodyParse* __restrict__ out,
                                                               char* __restrict__ file_ids) {
    const uint32_t k = blockIdx.x * 4u + (threadIdx.x >> 6);
    if (k >= n) return;
    const uint32_t lane = threadIdx.x & 63u;
    const char* body = in + spans[2 * k];
    const uint64_t L = spans[2 * k + 1];
    BodyParse r{};
    r.status = 1;
    bool ok = L >= kBodyFrameBytes;
    // {"fileId":"<64 chars>","fragments":[{"index":"d","data":"
    if (ok) ok = frame_ok(body, 0, kBodyPrefix, 11, ~0u) &&
                 frame_ok(body, 75, kBodyPrefix + 75, kBodyDataA - 75, kBodyDataA - 11 - 75);
    if (ok) ok = __ballot(body[11 + lane] == '"') == 0;  // the fileId holds no quote
    if (ok) {
        const uint64_t qa = scan_quote(body, kBodyDataA, L);
        ok = qa + kBodyMidBytes + 4 <= L && frame_ok(body, qa, kBodyMid, kBodyMidBytes, kBodyMidBytes - 11);
        if (ok) {
            const uint64_t sb = qa + kBodyMidBytes;
            const uint64_t qb = scan_quote(body, sb, L);
            ok = qb + 4 == L && frame_ok(body, qb, kBodySuffix, 4, ~0u);
            if (ok) {
                r.off_a = kBodyDataA;
                r.len_a = qa - kBodyDataA;
                r.off_b = sb;
                r.len_b = qb - sb;
                r.a = static_cast<uint16_t>(body[kBodyDataA - 11] - '0');
                r.b = static_cast<uint16_t>(body[qa + kBodyMidBytes - 11] - '0');
                r.status = 0;
            }
        }
    }
    if (r.status == 0) file_ids[64ull * k + lane] = body[11 + lane];
    if (lane == 0) out[k] = r;
}

}  // namespace

hipError_t launch_store_body_parse(const char* in, const uint64_t* spans, uint32_t n, BodyParse* out,
                                   char* file_ids, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(store_body_parse_kernel, dim3((n + 3) / 4), dim3(256), 0, s, in, spans, n, out, file_ids);
    return hipGetLastError();
}

}  // namespace dfs
