// batcher_load.cpp — closed-loop load generator for the request batcher.
//
// C native threads stand for StorageNode's connection handlers
// (StorageNode.java:28-31): each submits one file at a time through
// dfs_submit_upload or dfs_submit_download (host buffers) until the deadline
// and records every call's latency.  Native threads, so the measurement
// carries no interpreter lock.  Prints one JSON line; bench.py runs it per
// concurrency and checks the printed fileIds against its own checker.
//
//   batcher_load <clients> <seconds> <upload|download> <file_bytes> <nfrag> [max_wait_us] [depth] [pinned]
// pinned = 1: every client's buffers come from dfs_host_alloc (direct
// requests: DMA straight from / into them, no staging copies); pinned = 2:
// pinned inputs and the outputs as views (dfs_submit_*_view: the answer stays
// in the batch's result buffer, one DMA per batch, released after the check);
// pinned = 3: pageable inputs (staged by the handler) with view outputs.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <string>
#include <thread>
#include <vector>

#include <dirent.h>
#include <sys/syscall.h>
#include <unistd.h>

#include "../include/dfs_gpu.h"

namespace {

using Clock = std::chrono::steady_clock;
constexpr int kDistinct = 64;
constexpr uint64_t kSeed = 0x5EED5EEDull;

uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// The bench's synthetic file f (dfs_synth_fill's byte stream).
void synth(uint64_t f, uint64_t len, uint8_t* out) {
    for (uint64_t o = 0; o < len; o += 8) {
        const uint64_t v = splitmix64(kSeed ^ ((f << 40) | (o >> 3)));
        for (uint64_t b = 0; b < 8 && o + b < len; ++b) out[o + b] = static_cast<uint8_t>(v >> (8 * b));
    }
}

std::string hex(const uint8_t* d) {
    static const char* k = "0123456789abcdef";
    std::string s(64, '0');
    for (int i = 0; i < 32; ++i) {
        s[2 * i] = k[d[i] >> 4];
        s[2 * i + 1] = k[d[i] & 15];
    }
    return s;
}

uint64_t enc_len(uint64_t n) { return 4 * ((n + 2) / 3); }

// cgroup v2 CPU accounting of this process's share (a GPU box gives a
// process a CPU quota): usage and throttled microseconds.
void cpu_stat(unsigned long long& usage, unsigned long long& throttled) {
    usage = throttled = 0;
    if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.stat", "r")) {
        char key[64];
        unsigned long long v;
        while (std::fscanf(f, "%63s %llu", key, &v) == 2) {
            if (!std::strcmp(key, "usage_usec")) usage = v;
            if (!std::strcmp(key, "throttled_usec")) throttled = v;
        }
        std::fclose(f);
    }
}

double thread_cpu_now() {
    timespec ts;
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

// CPU seconds (utime + stime) of this process's threads, split into the
// client threads (tids), the batcher's workers (named "dfs-batch") and the
// rest (main thread, HIP / ROCr runtime threads).
void thread_cpu(const std::vector<long>& tids, double& clients, double& workers, double& other) {
    clients = workers = other = 0;
    const double hz = static_cast<double>(sysconf(_SC_CLK_TCK));
    DIR* d = opendir("/proc/self/task");
    if (!d) return;
    while (dirent* e = readdir(d)) {
        if (e->d_name[0] == '.') continue;
        const long tid = std::atol(e->d_name);
        char path[96], comm[64] = {0};
        std::snprintf(path, sizeof path, "/proc/self/task/%ld/comm", tid);
        if (FILE* f = std::fopen(path, "r")) {
            if (!std::fgets(comm, sizeof comm, f)) comm[0] = 0;
            std::fclose(f);
        }
        std::snprintf(path, sizeof path, "/proc/self/task/%ld/stat", tid);
        FILE* f = std::fopen(path, "r");
        if (!f) continue;
        char buf[1024];
        const size_t n = std::fread(buf, 1, sizeof buf - 1, f);
        std::fclose(f);
        buf[n] = 0;
        const char* p = std::strrchr(buf, ')');  // fields after the comm: state is field 3, utime 14, stime 15
        unsigned long long ut = 0, st = 0;
        if (!p || std::sscanf(p + 2, "%*c %*d %*d %*d %*d %*d %*u %*u %*u %*u %*u %llu %llu", &ut, &st) != 2) continue;
        const double s = (ut + st) / hz;
        if (std::find(tids.begin(), tids.end(), tid) != tids.end()) clients += s;
        else if (!std::strncmp(comm, "dfs-batch", 9)) workers += s;
        else other += s;
    }
    closedir(d);
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 6) {
        std::fprintf(stderr, "usage: %s clients seconds upload|download file_bytes nfrag [max_wait_us] [depth] [pinned]\n", argv[0]);
        return 2;
    }
    const int C = std::atoi(argv[1]);
    const double secs = std::atof(argv[2]);
    const bool up = std::strcmp(argv[3], "upload") == 0;
    const uint64_t S = std::strtoull(argv[4], nullptr, 10);
    const uint32_t N = static_cast<uint32_t>(std::atoi(argv[5]));
    dfs_batcher_opts o{};
    if (argc > 6) o.max_wait_us = static_cast<uint32_t>(std::atoi(argv[6]));
    if (argc > 7) o.depth = static_cast<uint32_t>(std::atoi(argv[7]));
    const int pin_mode = argc > 8 ? std::atoi(argv[8]) : 0;
    const bool pinned = pin_mode == 1 || pin_mode == 2, views = pin_mode >= 2;  // 3: pageable inputs, view outputs
    // A client buffer: pageable (std::vector) or a slice of one dfs_host_alloc
    // pool (a server would pin its connection buffers once, not per request;
    // one pool instead of 3 x C pinned allocations also keeps the setup of
    // 4,096 clients short).
    struct Pool {
        uint8_t* base = nullptr;
        uint64_t cap = 0;
        std::atomic<uint64_t> used{0};
        ~Pool() {
            if (base) dfs_host_free(base);
        }
        uint8_t* take(uint64_t n) {
            const uint64_t a = used.fetch_add((n + 255) & ~255ull);
            return base && a + n <= cap ? base + a : nullptr;
        }
    } pool;
    struct HostBuf {
        std::vector<uint8_t> v;
        uint8_t* p = nullptr;
        uint8_t* data() { return p ? p : v.data(); }
        void make(uint64_t n, Pool* pl) {
            if (pl && (p = pl->take(n ? n : 1))) return;
            p = nullptr;
            v.assign(n ? n : 1, 0);
        }
    };    if (C < 1 || N < 1 || N > 64) return 2;
    dfs_batcher* B = nullptr;
    if (int rc = dfs_batcher_create(0, N, &o, &B)) {
        std::fprintf(stderr, "dfs_batcher_create: %s\n", dfs_strerror(rc));
        return 3;
    }
    // distinct files, their upload results (Base64, digests) for the download clients
    std::vector<std::vector<uint8_t>> file(kDistinct, std::vector<uint8_t>(S));
    std::vector<std::vector<uint8_t>> fd(kDistinct, std::vector<uint8_t>(32)), frd(kDistinct, std::vector<uint8_t>(32 * N));
    std::vector<std::vector<char>> b64(kDistinct);
    std::vector<std::vector<uint64_t>> off(kDistinct, std::vector<uint64_t>(N + 1));
    const uint64_t cap = N * enc_len(S / N + 1) + 16;
    // the distinct files' reference results, uploaded concurrently (one batch)
    std::atomic<int> warm_rc{0};
    {
        std::vector<std::thread> w;
        for (int f = 0; f < kDistinct; ++f)
            w.emplace_back([&, f] {
                synth(f, S, file[f].data());
                b64[f].resize(cap);
                if (int rc = dfs_submit_upload(B, file[f].data(), S, fd[f].data(), frd[f].data(), b64[f].data(), cap,
                                               off[f].data()))
                    warm_rc = rc;
            });
        for (auto& x : w) x.join();
    }
    if (warm_rc.load()) {
        std::fprintf(stderr, "warm-up upload: %s\n", dfs_strerror(warm_rc.load()));
        return 3;
    }
    if (pinned) {
        const uint64_t per = up ? (S + 256) + (cap + 256) + 512 : 256 + 256 + (S + 256);
        pool.cap = static_cast<uint64_t>(C) * per + kDistinct * (cap + 256);
        void* q = nullptr;
        if (dfs_host_alloc(pool.cap, &q) != DFS_OK) {
            std::fprintf(stderr, "dfs_host_alloc(%llu): out of pinned memory\n", (unsigned long long)pool.cap);
            return 3;
        }
        pool.base = static_cast<uint8_t*>(q);
    }
    Pool* pl = pinned ? &pool : nullptr;
    std::vector<HostBuf> text(kDistinct);  // the Base64 download clients read (pinned if asked)
    for (int f = 0; f < kDistinct; ++f) {
        text[f].make(cap, pl);
        std::memcpy(text[f].data(), b64[f].data(), cap);
    }
    std::atomic<int> ready{0};
    std::atomic<bool> go{false}, bad{false};
    std::atomic<int> first_rc{0}, mismatches{0};
    std::vector<std::vector<double>> lat(C);
    std::vector<double> cpu_in(C, 0.0), cpu_out(C, 0.0);  // thread CPU inside / outside the submit calls (window)
    Clock::time_point deadline, measure_from;
    std::vector<std::thread> th;
    std::vector<long> tids(C, 0);
    th.reserve(C);
    for (int t = 0; t < C; ++t) {
        th.emplace_back([&, t] {
            const int f = t % kDistinct;
            tids[t] = static_cast<long>(syscall(SYS_gettid));
            std::vector<uint8_t> mfd(32), mfrd(32 * N);
            HostBuf in, mb, out;  // the handler's request body / Base64 answer / downloaded file
            in.make(up ? S : 1, pl);
            if (up) std::memcpy(in.data(), file[f].data(), S);
            mb.make(up ? cap : 1, pl);
            out.make(up ? 1 : S, pl);
            std::vector<uint64_t> moff(N + 1);
            std::vector<dfs_span> spans(N);
            for (uint32_t k = 0; k < N; ++k) spans[k] = dfs_span{off[f][k], off[f][k + 1] - off[f][k]};
            ++ready;
            while (!go.load()) std::this_thread::yield();
            for (uint64_t it = 0;; ++it) {
                const auto t0 = Clock::now();
                const double k0 = thread_cpu_now();
                int rc;
                const char* ans_b64 = reinterpret_cast<const char*>(mb.data());
                const uint8_t* ans_file = out.data();
                dfs_view* view = nullptr;
                if (up && views) {
                    rc = dfs_submit_upload_view(B, in.data(), S, mfd.data(), mfrd.data(), &ans_b64, moff.data(), &view);
                } else if (up) {
                    rc = dfs_submit_upload(B, in.data(), S, mfd.data(), mfrd.data(), reinterpret_cast<char*>(mb.data()), cap,
                                           moff.data());
                } else if (views) {
                    rc = dfs_submit_download_view(B, reinterpret_cast<const char*>(text[f].data()), spans.data(), S,
                                                  frd[f].data(), fd[f].data(), &ans_file, &view);
                } else {
                    rc = dfs_submit_download(B, reinterpret_cast<const char*>(text[f].data()), spans.data(), S, frd[f].data(),
                                             fd[f].data(), out.data());
                }
                const auto t1 = Clock::now();
                const double k1 = thread_cpu_now();
                if (t0 >= measure_from) lat[t].push_back(std::chrono::duration<double>(t1 - t0).count());
                if (t0 >= measure_from) cpu_in[t] += k1 - k0;
                if (rc != DFS_OK) {
                    bad = true;
                    int z = 0;
                    first_rc.compare_exchange_strong(z, rc);
                } else if (it % 8) {  // every 8th result is compared in full (the handler's own work stays small)
                } else if (up && (std::memcmp(mfd.data(), fd[f].data(), 32) || std::memcmp(mfrd.data(), frd[f].data(), 32 * N) ||
                                std::memcmp(ans_b64, b64[f].data(), off[f][N])))
                    bad = true, ++mismatches;
                else if (!up && std::memcmp(ans_file, file[f].data(), S))
                    bad = true, ++mismatches;
                if (view) dfs_view_release(view);
                if (t0 >= measure_from) cpu_out[t] += thread_cpu_now() - k1;
                if (t1 >= deadline) break;
            }
        });
    }
    while (ready.load() < C) std::this_thread::yield();
    // 0.5 s of warm-up at the same concurrency (staging buffers reach their
    // size), then the measured window: requests started inside it
    const auto dur = [](double x) { return std::chrono::duration_cast<Clock::duration>(std::chrono::duration<double>(x)); };
    measure_from = Clock::now() + dur(0.5);
    deadline = measure_from + dur(secs);
    go = true;
    std::this_thread::sleep_until(measure_from);
    // the batcher's counters are cumulative since its creation: snapshot them
    // where the measured window opens and report the differences, so that
    // batches / requests / direct cover the window the throughput covers
    dfs_batcher_stats_t st_warm{};
    dfs_batcher_stats(B, &st_warm);
    unsigned long long u0, th0, u1, th1;
    cpu_stat(u0, th0);
    const auto t0 = Clock::now();
    // client threads exit at the deadline: sample per-thread CPU just before
    std::this_thread::sleep_until(deadline - dur(0.02));
    double cpu_cl = 0, cpu_wk = 0, cpu_ot = 0;
    thread_cpu(tids, cpu_cl, cpu_wk, cpu_ot);
    for (auto& x : th) x.join();
    const double wall = std::chrono::duration<double>(deadline - t0).count();
    cpu_stat(u1, th1);
    double cin = 0, cout_ = 0;
    for (int t = 0; t < C; ++t) cin += cpu_in[t], cout_ += cpu_out[t];
    std::vector<double> all;
    for (auto& v : lat) all.insert(all.end(), v.begin(), v.end());
    std::sort(all.begin(), all.end());
    auto pct = [&](double p) { return all.empty() ? 0.0 : all[std::min(all.size() - 1, static_cast<size_t>(p * all.size()))]; };
    dfs_batcher_stats_t st{};
    dfs_batcher_stats(B, &st);
    st.batches -= st_warm.batches;
    st.requests -= st_warm.requests;
    st.direct -= st_warm.direct;
    st.views -= st_warm.views;
    st.queue_s -= st_warm.queue_s;
    st.stage_in_s -= st_warm.stage_in_s;
    st.device_s -= st_warm.device_s;
    st.stage_out_s -= st_warm.stage_out_s;
    st.enqueue_s -= st_warm.enqueue_s;
    st.return_s -= st_warm.return_s;
    dfs_batcher_destroy(B);
    std::printf("{\"clients\": %d, \"kind\": \"%s\", \"requests\": %zu, \"wall_s\": %.4f, \"gbps\": %.4f, "
                "\"p50_ms\": %.3f, \"p99_ms\": %.3f, \"cpu_s\": %.3f, \"throttled_s\": %.3f, \"cpu_threads_s\": {\"clients\": %.3f, \"workers\": %.3f, \"other\": %.3f}, \"client_cpu_us_per_req\": {\"in_submit\": %.1f, \"outside\": %.1f}, \"ok\": %s, \"file0_id\": \"%s\", \"file1_id\": \"%s\", "
                "\"pinned\": %d, \"stats\": {\"direct\": %llu, \"views\": %llu, \"batches\": %llu, \"requests\": %llu, \"max_batch\": %llu, \"queue_s\": %.4f, "
                "\"stage_in_s\": %.4f, \"device_s\": %.4f, \"stage_out_s\": %.4f, \"enqueue_s\": %.4f, \"return_s\": %.4f}}\n",
                C, up ? "upload" : "download", all.size(), wall, all.size() * static_cast<double>(S) / wall / 1e9,
                pct(0.5) * 1e3, pct(0.99) * 1e3, (u1 - u0) / 1e6, (th1 - th0) / 1e6, cpu_cl, cpu_wk, cpu_ot, cin / std::max<size_t>(all.size(), 1) * 1e6, cout_ / std::max<size_t>(all.size(), 1) * 1e6, bad ? "false" : "true", hex(fd[0].data()).c_str(),
                hex(fd[1].data()).c_str(), pin_mode, (unsigned long long)st.direct, (unsigned long long)st.views, (unsigned long long)st.batches, (unsigned long long)st.requests,
                (unsigned long long)st.max_batch, st.queue_s, st.stage_in_s, st.device_s, st.stage_out_s, st.enqueue_s,
                st.return_s);
    if (bad)
        std::fprintf(stderr, "batcher_load: %d mismatching results, first failing status %d (%s)\n", mismatches.load(),
                     first_rc.load(), first_rc.load() ? dfs_strerror(first_rc.load()) : "-");
    return bad ? 1 : 0;
}
