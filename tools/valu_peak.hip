// valu_peak.hip — on-box int32 VALU peak microbenchmark (gfx950).
//
// Measures sustained wave64 issue rate of the instructions the SHA-256 kernel
// is made of (v_add3_u32, v_alignbit_b32, v_bitop3_b32, v_add_u32), as
// 8 independent dependency chains per lane, 8 waves per SIMD, every CU busy.
// Reported as int32 lane-ops/s; the roofline peak in bench.py is the larger
// of this and the clock-derived 256 CU x 4 SIMD x 32 lanes x 2.4 GHz.
//   build: hipcc -O3 --offload-arch=gfx950 tools/valu_peak.hip -o tools/valu_peak
//   run:   tools/valu_peak  -> one JSON line
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHAINS 8
constexpr int kIters = 4096;

template <int OP>
__global__ __launch_bounds__(256) void chains(uint32_t* out, uint32_t seed) {
    uint32_t v[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) v[c] = seed * (threadIdx.x + 1) + c * 0x9e3779b9u + blockIdx.x;
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
#pragma unroll
            for (int c = 0; c < CHAINS; ++c) {
                if (OP == 0) v[c] = v[c] + v[(c + 1) % CHAINS] + 0x1234567u;  // folds to v_add3
                if (OP == 1) v[c] = __builtin_amdgcn_alignbit(v[c], v[(c + 1) % CHAINS], 7 + u);
                if (OP == 2) v[c] = __builtin_amdgcn_bitop3_b32(v[c], v[(c + 1) % CHAINS], v[(c + 3) % CHAINS], 0x96);
                if (OP == 3) v[c] = v[c] + v[(c + 5) % CHAINS];
            }
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) r ^= v[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int OP>
double run(uint32_t* d, int blocks) {
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
    const double ops = 1.0 * reps * blocks * 256.0 * kIters * 8 * CHAINS;
    return ops / (ms * 1e-3);
}

int main() {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 1;
    const int blocks = p.multiProcessorCount * 8;  // 8 waves/SIMD
    uint32_t* d;
    (void)hipMalloc(&d, sizeof(uint32_t) * blocks * 256);
    const double add3 = run<0>(d, blocks), align = run<1>(d, blocks), bop = run<2>(d, blocks), add = run<3>(d, blocks);
    std::printf("{\"cus\": %d, \"clock_mhz\": %d, \"add3_ops\": %.4g, \"alignbit_ops\": %.4g, \"bitop3_ops\": %.4g, "
                "\"add_ops\": %.4g, \"clock_peak_ops\": %.4g}\n",
                p.multiProcessorCount, p.clockRate / 1000, add3, align, bop, add,
                p.multiProcessorCount * 4.0 * 32.0 * p.clockRate * 1e3);
    (void)hipFree(d);
    return 0;
}
