// valu_peak.hip — on-box int32 VALU issue-rate microbenchmark (gfx950).
//
// For each instruction the SHA-256 / Base64 kernels can be built from, runs 8
// independent dependency chains per lane (a = op(a, b, c), b and c loop
// invariant), 8 waves per SIMD on every CU, and reports wave64 lane-ops/s.
// The survey's roofline denominator (256 CU x 4 SIMD x 32 lanes x 2.4 GHz)
// is printed beside it as clock_peak_ops.
//   build: hipcc -O3 --offload-arch=gfx950 tools/valu_peak.hip -o tools/valu_peak
//   run:   tools/valu_peak  -> one JSON line
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kIters = 2048;
constexpr int kChains = 8;
constexpr int kUnroll = 8;

#define DEFOP(NAME, ASM)                                                           \
    struct NAME {                                                                  \
        static constexpr const char* name = #NAME;                                 \
        static __device__ __forceinline__ void f(uint32_t& a, uint32_t b, uint32_t c) { \
            asm volatile(ASM : "+v"(a) : "v"(b), "v"(c));                          \
        }                                                                          \
    };

DEFOP(add3, "v_add3_u32 %0, %0, %1, %2")
DEFOP(alignbit, "v_alignbit_b32 %0, %0, %1, 7")
DEFOP(alignbit_rot, "v_alignbit_b32 %0, %0, %0, 7")
DEFOP(bitop3, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96")
DEFOP(add, "v_add_u32_e32 %0, %0, %1")
DEFOP(xor2, "v_xor_b32_e32 %0, %0, %1")
DEFOP(lshr, "v_lshrrev_b32_e32 %0, 7, %0")
DEFOP(lshl_or, "v_lshl_or_b32 %0, %0, 7, %1")
DEFOP(lshl_add, "v_lshl_add_u32 %0, %0, 3, %1")
DEFOP(xad, "v_xad_u32 %0, %0, %1, %2")
DEFOP(perm, "v_perm_b32 %0, %0, %1, %2")
DEFOP(alignbyte, "v_alignbyte_b32 %0, %0, %1, 1")
DEFOP(bfi, "v_bfi_b32 %0, %0, %1, %2")
DEFOP(or3, "v_or3_b32 %0, %0, %1, %2")
DEFOP(and_or, "v_and_or_b32 %0, %0, %1, %2")
DEFOP(pk_add_u16, "v_pk_add_u16 %0, %0, %1")
DEFOP(bfe, "v_bfe_u32 %0, %0, 6, 6")
DEFOP(mad_u24, "v_mad_u32_u24 %0, %0, %1, %2")
DEFOP(lshl, "v_lshlrev_b32_e32 %0, 7, %0")
DEFOP(and2, "v_and_b32_e32 %0, %0, %1")
DEFOP(mov, "v_mov_b32_e32 %0, %1")

// 64-bit ops on a register pair (a:a'): one op counts once.
#define DEFOP64(NAME, ASM)                                                         \
    struct NAME {                                                                  \
        static constexpr const char* name = #NAME;                                 \
        static __device__ __forceinline__ void f(uint32_t& a, uint32_t b, uint32_t c) { \
            uint64_t x = (static_cast<uint64_t>(b) << 32) | a;                     \
            asm volatile(ASM : "+v"(x) : "v"(b), "v"(c));                          \
            a = static_cast<uint32_t>(x);                                          \
        }                                                                          \
    };
DEFOP64(lshr64, "v_lshrrev_b64 %0, 7, %0")
DEFOP64(lshl64, "v_lshlrev_b64 %0, 7, %0")
DEFOP64(pk_mov_dup, "v_pk_mov_b32 %0, %0, %0 op_sel:[0,0]")
DEFOP64(lshl_add64, "v_lshl_add_u64 %0, %0, 2, %0")
// rotate through a pair: dup (v_pk_mov_b32 low->both) + 64-bit shift = 2
// instructions per rotate (counted as one op); chain state stays in a pair.
struct rot64 {
    static constexpr const char* name = "rot64_dup_shift";
    static __device__ __forceinline__ void f(uint32_t& a, uint32_t b, uint32_t) {
        uint64_t x = (static_cast<uint64_t>(b) << 32) | a;
        asm volatile("v_pk_mov_b32 %0, %0, %0 op_sel:[0,0]\n\tv_lshrrev_b64 %0, 7, %0" : "+v"(x));
        a = static_cast<uint32_t>(x);
    }
};

// SHA-256 compression on register data only (no memory): the compute floor
// of the multi-message kernel.  Same round code as csrc/sha256.hip (kept in
// sync by hand; bitop3 / alignbit / add3 and the per-round ordering points).
__device__ __forceinline__ uint32_t rotr(uint32_t x, uint32_t n) { return __builtin_amdgcn_alignbit(x, x, n); }
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }
__constant__ uint32_t kKc[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
constexpr uint32_t kKs[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
__device__ __forceinline__ void sha_compress(uint32_t (&st)[8], uint32_t (&W)[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
    for (int t = 0; t < 64; ++t) {
        if (t >= 16) {
            const uint32_t x = W[(t - 2) & 15], y = W[(t - 15) & 15];
            W[t & 15] += xor3(rotr(x, 17), rotr(x, 19), x >> 10) + W[(t - 7) & 15] + xor3(rotr(y, 7), rotr(y, 18), y >> 3);
            asm volatile("" : "+v"(W[t & 15]));
        }
        const uint32_t t1 = h + xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25)) + __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA) + kKs[t] + W[t & 15];
        const uint32_t t2 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22)) + __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
        h = g; g = f; f = e; e = d + t1;
        d = c; c = b; b = a; a = t1 + t2;
        asm volatile("" : "+v"(a), "+v"(e));
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
    st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}
constexpr int kShaIters = 256;
__global__ __launch_bounds__(256) void sha_floor(uint32_t* out, uint32_t seed) {
    uint32_t st[8], W[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) st[i] = seed * (threadIdx.x + 1) + i;
#pragma unroll
    for (int i = 0; i < 16; ++i) W[i] = seed ^ (threadIdx.x * 16 + i);
    for (int k = 0; k < kShaIters; ++k) {
        uint32_t w[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = W[i] ^ st[i & 7];
        sha_compress(st, w);
    }
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) r ^= st[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

// blocks/s at `wps` waves per SIMD (grid = CUs * wps workgroups of 4 waves).
double sha_rate(uint32_t* d, int cus, int wps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int blocks = cus * wps;
    hipLaunchKernelGGL(sha_floor, dim3(blocks), dim3(256), 0, 0, d, 1u);
    (void)hipEventRecord(a);
    const int reps = 5;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(sha_floor, dim3(blocks), dim3(256), 0, 0, d, 2u + r);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return 1.0 * reps * blocks * 256.0 * kShaIters / (ms * 1e-3);
}

template <class OP>
__global__ __launch_bounds__(256) void chains(uint32_t* out, uint32_t seed) {
    uint32_t v[kChains];
#pragma unroll
    for (int c = 0; c < kChains; ++c) v[c] = seed * (threadIdx.x + 1) + c * 0x9e3779b9u + blockIdx.x;
    const uint32_t b = seed ^ threadIdx.x, cc = seed + 0x01020304u;
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
#pragma unroll
            for (int c = 0; c < kChains; ++c) OP::f(v[c], b, cc);
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int c = 0; c < kChains; ++c) r ^= v[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <class OP>
void run(uint32_t* d, int blocks, bool comma) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(chains<OP>, dim3(blocks), dim3(256), 0, 0, d, 1u);  // warm
    (void)hipEventRecord(a);
    const int reps = 5;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(chains<OP>, dim3(blocks), dim3(256), 0, 0, d, 2u + r);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    const double ops = 1.0 * reps * blocks * 256.0 * kIters * kUnroll * kChains;
    std::printf("%s\"%s\": %.4g", comma ? ", " : "", OP::name, ops / (ms * 1e-3));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
}

int main() {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 1;
    const int blocks = p.multiProcessorCount * 8;  // 8 waves per SIMD
    uint32_t* d;
    if (hipMalloc(&d, sizeof(uint32_t) * blocks * 256) != hipSuccess) return 1;
    std::printf("{\"cus\": %d, \"clock_mhz\": %d, \"clock_peak_ops\": %.4g, \"ops\": {", p.multiProcessorCount,
                p.clockRate / 1000, p.multiProcessorCount * 4.0 * 32.0 * p.clockRate * 1e3);
    run<add3>(d, blocks, false);
    run<alignbit>(d, blocks, true);
    run<alignbit_rot>(d, blocks, true);
    run<bitop3>(d, blocks, true);
    run<add>(d, blocks, true);
    run<xor2>(d, blocks, true);
    run<lshr>(d, blocks, true);
    run<lshl_or>(d, blocks, true);
    run<lshl_add>(d, blocks, true);
    run<xad>(d, blocks, true);
    run<perm>(d, blocks, true);
    run<alignbyte>(d, blocks, true);
    run<bfi>(d, blocks, true);
    run<or3>(d, blocks, true);
    run<and_or>(d, blocks, true);
    run<pk_add_u16>(d, blocks, true);
    run<bfe>(d, blocks, true);
    run<mad_u24>(d, blocks, true);
    run<lshl>(d, blocks, true);
    run<and2>(d, blocks, true);
    run<mov>(d, blocks, true);
    run<lshr64>(d, blocks, true);
    run<lshl64>(d, blocks, true);
    run<pk_mov_dup>(d, blocks, true);
    run<lshl_add64>(d, blocks, true);
    run<rot64>(d, blocks, true);
    std::printf("}, \"sha_compress_blocks_per_s\": {");
    for (int w = 1; w <= 8; w *= 2) std::printf("%s\"wps%d\": %.4g", w > 1 ? ", " : "", w, sha_rate(d, p.multiProcessorCount, w));
    std::printf("}}\n");
    (void)hipFree(d);
    return 0;
}
