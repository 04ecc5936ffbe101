// wave_place_probe.hip — where do the waves of small workgroups land?  Launches
// G workgroups of T threads that all stay resident (each wave spins until every
// wave has checked in), records the SIMD of every wave (XCC / SE / SH / CU / SIMD
// fields of HW_REG_XCC_ID and HW_REG_HW_ID, gfx9 layout) and prints how many
// SIMDs hold 0, 1, 2, ... waves.  Used to explain the latency kernels' timings
// with one and two workgroups per CU.
//   build: hipcc -O3 --offload-arch=gfx950 -Xclang -target-feature -Xclang -packed-fp32-ops \
//          tools/wave_place_probe.hip -o tools/wave_place_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <vector>

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

// lds: bytes of LDS per workgroup (as the latency kernels hold), so that the
// occupancy limits are the same.
template <int LDS>
__global__ void place(uint32_t* keys, uint32_t* arrived, uint32_t total, uint64_t max_ticks) {
    __shared__ uint8_t pad[LDS];
    if (threadIdx.x == 0) pad[0] = 1;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if ((threadIdx.x & 63u) == 0) {
        const uint32_t hw = hw_id();
        keys[wave] = ((xcc_id() & 7u) << 10) | (((hw >> 13) & 7u) << 7) | (((hw >> 12) & 1u) << 6) |
                     (((hw >> 8) & 15u) << 2) | ((hw >> 4) & 3u);
        atomicAdd(arrived, 1u);
        // stay resident until every wave is (bounded: the grid always drains)
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(arrived, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < total &&
               __builtin_amdgcn_s_memrealtime() - t0 < max_ticks)
            __builtin_amdgcn_s_sleep(32);
    }
    __syncthreads();
    if (threadIdx.x == 0 && pad[0] == 7) keys[0] = 0;
}

template <int LDS>
void run(int groups, int threads) {
    const uint32_t waves = static_cast<uint32_t>(groups) * (threads / 64);
    uint32_t *d_keys, *d_arr;
    (void)hipMalloc(&d_keys, 4ull * waves);
    (void)hipMalloc(&d_arr, 4);
    (void)hipMemset(d_arr, 0, 4);
    hipLaunchKernelGGL(place<LDS>, dim3(groups), dim3(threads), 0, 0, d_keys, d_arr, waves, 20000000ull /* 0.2 s */);
    (void)hipDeviceSynchronize();
    std::vector<uint32_t> keys(waves);
    (void)hipMemcpy(keys.data(), d_keys, 4ull * waves, hipMemcpyDeviceToHost);
    std::map<uint32_t, int> per_simd, per_cu;
    for (uint32_t k : keys) ++per_simd[k], ++per_cu[k >> 2];
    std::map<int, int> hist, hist_cu;
    for (auto& kv : per_simd) ++hist[kv.second];
    for (auto& kv : per_cu) ++hist_cu[kv.second];
    std::printf("{\"groups\": %d, \"threads\": %d, \"lds\": %d, \"simds_used\": %zu, \"cus_used\": %zu, \"waves_per_simd\": {", groups,
                threads, LDS, per_simd.size(), per_cu.size());
    const char* sep = "";
    for (auto& kv : hist) std::printf("%s\"%d\": %d", sep, kv.first, kv.second), sep = ", ";
    std::printf("}, \"waves_per_cu\": {");
    sep = "";
    for (auto& kv : hist_cu) std::printf("%s\"%d\": %d", sep, kv.first, kv.second), sep = ", ";
    std::printf("}}\n");
    (void)hipFree(d_keys);
    (void)hipFree(d_arr);
}

int main() {
    run<24576>(256, 128);  // pair-lane kernel, one pair per workgroup, 8,192 messages
    run<24576>(512, 128);  // ... 16,384 messages as one-pair workgroups (not used)
    run<49152>(256, 256);  // ... as two-pair workgroups (used)
    run<32768>(512, 128);  // one-lane kernel, 32,768 messages as one-pair workgroups (not used)
    run<65536>(256, 256);  // ... as two-pair workgroups (used)
    return 0;
}
