// hbm_stream.hip — on-box HBM ceiling for the Base64 traffic shapes (gfx950).
//
// The encode kernel reads n bytes and writes 4n/3; decode the reverse.  This
// measures what plain streaming kernels with the SAME byte counts and access
// shapes (no compute) reach, so the Base64 kernels' roofline fraction can be
// read against both the 8 TB/s spec and the achievable ceiling.
//   read      : dwordx4 loads, n bytes (reduced so nothing is optimised away)
//   write     : dwordx4 stores, n bytes
//   copy      : dwordx4 load + store, n bytes each way
//   expand    : 12 B loaded / 16 B stored per lane (the encode shape)
//   contract  : 16 B loaded / 12 B stored per lane (the decode shape)
// Grid: 8 workgroups x 256 threads per CU, grid-stride loop, 4 items per
// thread in flight.  Bytes in GB/s count read + write.
//   build: hipcc -O3 --offload-arch=gfx950 tools/hbm_stream.hip -o tools/hbm_stream
//   run:   tools/hbm_stream [GiB of input, default 16]  -> one JSON line
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            std::exit(1);                                                          \
        }                                                                          \
    } while (0)

constexpr int kU = 4;

__global__ __launch_bounds__(256) void k_read(const u32x4* __restrict__ in, size_t n16, uint32_t* __restrict__ sink) {
    uint32_t acc = 0;
    const size_t stride = static_cast<size_t>(gridDim.x) * 256 * kU;
    for (size_t b = static_cast<size_t>(blockIdx.x) * 256 * kU + threadIdx.x; b < n16; b += stride) {
        u32x4 v[kU];
#pragma unroll
        for (int i = 0; i < kU; ++i) v[i] = b + i * 256 < n16 ? __builtin_nontemporal_load(in + b + i * 256) : u32x4{0, 0, 0, 0};
#pragma unroll
        for (int i = 0; i < kU; ++i) acc ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void k_write(u32x4* __restrict__ out, size_t n16) {
    const size_t stride = static_cast<size_t>(gridDim.x) * 256 * kU;
    for (size_t b = static_cast<size_t>(blockIdx.x) * 256 * kU + threadIdx.x; b < n16; b += stride) {
#pragma unroll
        for (int i = 0; i < kU; ++i)
            if (b + i * 256 < n16) __builtin_nontemporal_store(u32x4{uint32_t(b), 1u, 2u, 3u}, out + b + i * 256);
    }
}

__global__ __launch_bounds__(256) void k_copy(const u32x4* __restrict__ in, u32x4* __restrict__ out, size_t n16) {
    const size_t stride = static_cast<size_t>(gridDim.x) * 256 * kU;
    for (size_t b = static_cast<size_t>(blockIdx.x) * 256 * kU + threadIdx.x; b < n16; b += stride) {
        u32x4 v[kU];
#pragma unroll
        for (int i = 0; i < kU; ++i) v[i] = b + i * 256 < n16 ? in[b + i * 256] : u32x4{0, 0, 0, 0};
#pragma unroll
        for (int i = 0; i < kU; ++i)
            if (b + i * 256 < n16) __builtin_nontemporal_store(v[i], out + b + i * 256);
    }
}

// ng groups: group g reads 12 bytes at 12g, writes 16 at 16g.
__global__ __launch_bounds__(256) void k_expand(const uint32_t* __restrict__ in, u32x4* __restrict__ out, size_t ng) {
    const size_t stride = static_cast<size_t>(gridDim.x) * 256 * kU;
    for (size_t b = static_cast<size_t>(blockIdx.x) * 256 * kU + threadIdx.x; b < ng; b += stride) {
        u32x3 v[kU];
#pragma unroll
        for (int i = 0; i < kU; ++i)
            v[i] = b + i * 256 < ng ? *reinterpret_cast<const u32x3*>(in + 3 * (b + i * 256)) : u32x3{0, 0, 0};
#pragma unroll
        for (int i = 0; i < kU; ++i)
            if (b + i * 256 < ng)
                __builtin_nontemporal_store(u32x4{v[i].x, v[i].y, v[i].z, v[i].x ^ v[i].z}, out + b + i * 256);
    }
}

// ng groups: group g reads 16 bytes at 16g, writes 12 at 12g.
__global__ __launch_bounds__(256) void k_contract(const u32x4* __restrict__ in, uint32_t* __restrict__ out, size_t ng) {
    const size_t stride = static_cast<size_t>(gridDim.x) * 256 * kU;
    for (size_t b = static_cast<size_t>(blockIdx.x) * 256 * kU + threadIdx.x; b < ng; b += stride) {
        u32x4 v[kU];
#pragma unroll
        for (int i = 0; i < kU; ++i) v[i] = b + i * 256 < ng ? in[b + i * 256] : u32x4{0, 0, 0, 0};
#pragma unroll
        for (int i = 0; i < kU; ++i)
            if (b + i * 256 < ng)
                *reinterpret_cast<u32x3*>(out + 3 * (b + i * 256)) = u32x3{v[i].x ^ v[i].w, v[i].y, v[i].z};
    }
}

template <class F>
static double time_ms(F f, int reps) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    f();  // warm
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) f();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char** argv) {
    const double gib = argc > 1 ? std::atof(argv[1]) : 16.0;
    const size_t n = static_cast<size_t>(gib * (1ull << 30)) / 48 * 48;  // input bytes
    const size_t nout = n / 3 * 4;
    uint8_t *in = nullptr, *out = nullptr;
    uint32_t* sink = nullptr;
    CHECK(hipMalloc(&in, nout));
    CHECK(hipMalloc(&out, nout));
    CHECK(hipMalloc(&sink, 4));
    CHECK(hipMemset(in, 0x5a, nout));
    CHECK(hipMemset(out, 0, nout));
    const dim3 grid(256 * 8), blk(256);
    const int reps = 5;
    auto gbs = [](double bytes, double ms) { return bytes / (ms * 1e-3) / 1e9; };
    const double t_read = time_ms([&] { hipLaunchKernelGGL(k_read, grid, blk, 0, 0, (const u32x4*)in, n / 16, sink); }, reps);
    const double t_write = time_ms([&] { hipLaunchKernelGGL(k_write, grid, blk, 0, 0, (u32x4*)out, n / 16); }, reps);
    const double t_copy = time_ms([&] { hipLaunchKernelGGL(k_copy, grid, blk, 0, 0, (const u32x4*)in, (u32x4*)out, n / 16); }, reps);
    const double t_exp = time_ms([&] { hipLaunchKernelGGL(k_expand, grid, blk, 0, 0, (const uint32_t*)in, (u32x4*)out, n / 12); }, reps);
    const double t_con = time_ms([&] { hipLaunchKernelGGL(k_contract, grid, blk, 0, 0, (const u32x4*)in, (uint32_t*)out, n / 12); }, reps);
    CHECK(hipGetLastError());
    std::printf("{\"input_bytes\": %zu, \"read_gbs\": %.1f, \"write_gbs\": %.1f, \"copy_gbs\": %.1f, "
                "\"expand_12to16_gbs\": %.1f, \"contract_16to12_gbs\": %.1f, \"expand_ms\": %.3f, \"contract_ms\": %.3f}\n",
                n, gbs(n, t_read), gbs(n, t_write), gbs(2.0 * n, t_copy), gbs(n + nout, t_exp), gbs(n + nout, t_con),
                t_exp, t_con);
    CHECK(hipFree(in));
    CHECK(hipFree(out));
    CHECK(hipFree(sink));
    return 0;
}
