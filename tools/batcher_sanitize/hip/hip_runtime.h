// Host-only stand-in for the few HIP runtime calls csrc/batcher.cpp makes, so
// that the batcher's thread hand-off can run under ThreadSanitizer /
// AddressSanitizer on a machine without a GPU (tools/batcher_sanitize.sh).
// "Device" memory is host memory and every stream call completes at once:
// what is exercised is the host protocol (queue, staging slots, views), not
// the kernels.  Never part of the product build.
#pragma once
#include <cstdlib>
#include <cstring>

#define __host__
#define __device__
typedef int hipError_t;
typedef struct dfs_fake_stream* hipStream_t;
typedef struct dfs_fake_event* hipEvent_t;
enum { hipSuccess = 0, hipErrorOutOfMemory = 2 };
enum { hipMemcpyHostToDevice = 1, hipMemcpyDeviceToHost = 2, hipMemcpyDefault = 4 };
enum { hipHostMallocDefault = 0, hipHostMallocMapped = 2, hipHostMallocCoherent = 0x40000000 };
enum { hipEventDisableTiming = 2 };

inline hipError_t hipMalloc(void** p, size_t n) { return (*p = std::malloc(n ? n : 1)) ? hipSuccess : hipErrorOutOfMemory; }
inline hipError_t hipHostMalloc(void** p, size_t n, unsigned) { return hipMalloc(p, n); }
inline hipError_t hipFree(void* p) { std::free(p); return hipSuccess; }
inline hipError_t hipHostFree(void* p) { std::free(p); return hipSuccess; }
inline hipError_t hipHostGetDevicePointer(void** d, void* h, unsigned) { *d = h; return hipSuccess; }
inline hipError_t hipGetLastError() { return hipSuccess; }
inline hipError_t hipSetDevice(int) { return hipSuccess; }
inline hipError_t hipMemcpyAsync(void* dst, const void* src, size_t n, int, hipStream_t) {
    if (n) std::memcpy(dst, src, n);
    return hipSuccess;
}
inline hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned) { *e = reinterpret_cast<hipEvent_t>(std::malloc(1)); return hipSuccess; }
inline hipError_t hipEventDestroy(hipEvent_t e) { std::free(e); return hipSuccess; }
inline hipError_t hipEventRecord(hipEvent_t, hipStream_t) { return hipSuccess; }
