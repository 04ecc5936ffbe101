// host_probe.cpp — host-side costs behind the request batcher:
//  1. memcpy rate between pageable and pinned (hipHostMalloc) memory, 1 and
//     T threads (a handler's copy in / out of the staging);
//  2. thread CPU time a caller spends per dfs_upload_batch of one 1 MiB file
//     (device pointers) + a blocking-sync event wait, i.e. whether any wait
//     on the path spins;
//  3. DMA rate of 512 per-request 1 MiB copies vs one 512 MiB copy, each
//     way (the batcher's direct path before its copy kernel).
//   host_probe [threads]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <thread>
#include <vector>

#include "../include/dfs_gpu.h"

namespace {
double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
double thread_cpu_s() {
    timespec t;
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

void copy_rate(const char* name, int T, size_t n, int reps, bool pinned_src, bool pinned_dst) {
    std::vector<std::thread> th;
    std::vector<double> gbs(T);
    for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            void *s = nullptr, *d = nullptr;
            if (pinned_src) (void)hipHostMalloc(&s, n, hipHostMallocDefault); else s = std::malloc(n);
            if (pinned_dst) (void)hipHostMalloc(&d, n, hipHostMallocDefault); else d = std::malloc(n);
            std::memset(s, t + 1, n);
            std::memset(d, 0, n);
            const double t0 = now_s();
            for (int r = 0; r < reps; ++r) std::memcpy(d, s, n);
            gbs[t] = n * double(reps) / (now_s() - t0) / 1e9;
            if (pinned_src) (void)hipHostFree(s); else std::free(s);
            if (pinned_dst) (void)hipHostFree(d); else std::free(d);
        });
    for (auto& x : th) x.join();
    double sum = 0;
    for (double g : gbs) sum += g;
    std::printf("{\"probe\": \"memcpy\", \"case\": \"%s\", \"threads\": %d, \"bytes\": %zu, \"gbps_per_thread\": %.2f, \"gbps_total\": %.2f}\n",
                name, T, n, sum / T, sum);
}
}  // namespace

int main(int argc, char** argv) {
    const int T = argc > 1 ? std::atoi(argv[1]) : 16;
    const size_t n = size_t(1) << 20;
    for (int t : {1, T}) {
        copy_rate("pageable->pageable", t, n, 400, false, false);
        copy_rate("pageable->pinned", t, n, 400, false, true);
        copy_rate("pinned->pageable", t, n, 400, true, false);
    }
    dfs_ctx* c = nullptr;
    if (dfs_open(&c, 0) != DFS_OK) return 3;
    uint8_t *d_in = nullptr, *d_dig = nullptr;
    char* d_b64 = nullptr;
    (void)hipMalloc(&d_in, n);
    (void)hipMalloc(&d_dig, 32 * 6);
    (void)hipMalloc(&d_b64, 2 * n);
    (void)hipMemset(d_in, 7, n);
    hipStream_t s = nullptr;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    (void)dfs_set_stream(c, s);
    hipEvent_t ev;
    (void)hipEventCreateWithFlags(&ev, hipEventBlockingSync | hipEventDisableTiming);
    dfs_span sp{0, n};
    uint64_t off[6];
    for (int mode = 0; mode < 3; ++mode) {
        const int reps = 20;
        double wall = 0, cpu_call = 0, cpu_wait = 0;
        for (int r = 0; r < reps + 2; ++r) {
            const double w0 = now_s(), c0 = thread_cpu_s();
            int rc = dfs_upload_batch(c, d_in, &sp, 1, 5, d_dig, d_dig + 32, d_b64, 2 * n, off, DFS_DEVICE_PTRS | DFS_SERIAL);
            const double c1 = thread_cpu_s();
            if (rc) return 4;
            if (mode == 0) {
                (void)hipEventRecord(ev, s);
                (void)hipEventSynchronize(ev);
            } else if (mode == 1) {
                (void)hipStreamSynchronize(s);
            } else {
                (void)hipEventRecord(ev, s);
                while (hipEventQuery(ev) == hipErrorNotReady) std::this_thread::sleep_for(std::chrono::microseconds(200));
            }
            const double c2 = thread_cpu_s(), w1 = now_s();
            if (r >= 2) {
                wall += w1 - w0;
                cpu_call += c1 - c0;
                cpu_wait += c2 - c1;
            }
        }
        static const char* names[] = {"blocking-event", "stream-sync", "query-sleep"};
        std::printf("{\"probe\": \"upload_1MiB\", \"wait\": \"%s\", \"wall_ms\": %.3f, \"cpu_call_ms\": %.3f, \"cpu_wait_ms\": %.3f}\n",
                    names[mode], wall / reps * 1e3, cpu_call / reps * 1e3, cpu_wait / reps * 1e3);
    }
    // 3. DMA per request vs one DMA per batch: 512 x 1 MiB pinned -> device
    //    (and 512 x 1.33 MiB back), one stream, as the batcher's direct path.
    {
        const int R = 512;
        const size_t up = n, down = 4 * ((n / 5 + 3) / 3) * 5;
        void *h_in = nullptr, *h_out = nullptr, *d_a = nullptr, *d_b = nullptr;
        (void)hipHostMalloc(&h_in, R * up, hipHostMallocDefault);
        (void)hipHostMalloc(&h_out, R * down, hipHostMallocDefault);
        (void)hipMalloc(&d_a, R * up);
        (void)hipMalloc(&d_b, R * down);
        std::memset(h_in, 1, R * up);
        for (int mode = 0; mode < 2; ++mode) {
            double best_h2d = 1e9, best_d2h = 1e9, cpu = 0;
            for (int rep = 0; rep < 4; ++rep) {
                (void)hipStreamSynchronize(s);
                double t0 = now_s(), c0 = thread_cpu_s();
                if (mode == 0)
                    for (int r = 0; r < R; ++r)
                        (void)hipMemcpyAsync(static_cast<char*>(d_a) + r * up, static_cast<char*>(h_in) + r * up, up,
                                             hipMemcpyHostToDevice, s);
                else
                    (void)hipMemcpyAsync(d_a, h_in, R * up, hipMemcpyHostToDevice, s);
                const double c1 = thread_cpu_s();
                (void)hipStreamSynchronize(s);
                double t1 = now_s();
                if (mode == 0)
                    for (int r = 0; r < R; ++r)
                        (void)hipMemcpyAsync(static_cast<char*>(h_out) + r * down, static_cast<char*>(d_b) + r * down,
                                             down, hipMemcpyDeviceToHost, s);
                else
                    (void)hipMemcpyAsync(h_out, d_b, R * down, hipMemcpyDeviceToHost, s);
                (void)hipStreamSynchronize(s);
                double t2 = now_s();
                if (rep) {
                    best_h2d = std::min(best_h2d, t1 - t0);
                    best_d2h = std::min(best_d2h, t2 - t1);
                    cpu += c1 - c0;
                }
            }
            std::printf("{\"probe\": \"dma\", \"mode\": \"%s\", \"requests\": %d, \"h2d_ms\": %.3f, \"h2d_gbs\": %.1f, "
                        "\"d2h_ms\": %.3f, \"d2h_gbs\": %.1f, \"issue_cpu_ms\": %.3f}\n",
                        mode ? "one_copy" : "per_request", R, best_h2d * 1e3, R * up / best_h2d / 1e9, best_d2h * 1e3,
                        R * down / best_d2h / 1e9, cpu / 3 * 1e3);
        }
        (void)hipHostFree(h_in);
        (void)hipHostFree(h_out);
        (void)hipFree(d_a);
        (void)hipFree(d_b);
    }
    dfs_close(c);
    return 0;
}
