/*
 * dfs_oracle.c — CPU restatement of StorageNode's fragment pipeline.
 *
 * TEST INFRASTRUCTURE ONLY (see dfs_oracle.h).  Plain C, no GPU, used as
 * the checker in tests/, in __graft_entry__.smoke(), and as the
 * cpu_baseline leg of bench.py.  Never linked into libdfsgpu.so.
 *
 * Citations: SN = /root/reference/storage-node/src/StorageNode.java.
 */
#define _GNU_SOURCE
#include "dfs_oracle.h"

#include <dlfcn.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ------------------------------------------------------------------ */
/* SHA-256 (FIPS 180-4 §6.2), the algorithm behind                     */
/* MessageDigest.getInstance("SHA-256").digest(data) at SN:605-606.    */
/* ------------------------------------------------------------------ */
static const uint32_t K256[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

#define ROTR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

static void sha256_compress(uint32_t h[8], const uint8_t blk[64]) {
    uint32_t w[64];
    for (int t = 0; t < 16; t++)
        w[t] = (uint32_t)blk[4 * t] << 24 | (uint32_t)blk[4 * t + 1] << 16 |
               (uint32_t)blk[4 * t + 2] << 8 | (uint32_t)blk[4 * t + 3];
    for (int t = 16; t < 64; t++) {
        uint32_t s0 = ROTR(w[t - 15], 7) ^ ROTR(w[t - 15], 18) ^ (w[t - 15] >> 3);
        uint32_t s1 = ROTR(w[t - 2], 17) ^ ROTR(w[t - 2], 19) ^ (w[t - 2] >> 10);
        w[t] = w[t - 16] + s0 + w[t - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int t = 0; t < 64; t++) {
        uint32_t S1 = ROTR(e, 6) ^ ROTR(e, 11) ^ ROTR(e, 25);
        uint32_t ch = (e & f) ^ (~e & g);
        uint32_t t1 = hh + S1 + ch + K256[t] + w[t];
        uint32_t S0 = ROTR(a, 2) ^ ROTR(a, 13) ^ ROTR(a, 22);
        uint32_t maj = (a & b) ^ (a & c) ^ (b & c);
        uint32_t t2 = S0 + maj;
        hh = g; g = f; f = e; e = d + t1;
        d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d;
    h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

void oracle_sha256(const uint8_t* data, uint64_t len, uint8_t out[32]) {
    uint32_t h[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                     0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
    uint64_t nfull = len / 64;
    for (uint64_t i = 0; i < nfull; i++) sha256_compress(h, data + 64 * i);
    /* FIPS 180-4 §5.1.1 padding: 0x80, zeros, 64-bit big-endian bit length. */
    uint8_t tail[128];
    uint64_t r = len - 64 * nfull;
    memset(tail, 0, sizeof tail);
    if (r) memcpy(tail, data + 64 * nfull, r);
    tail[r] = 0x80;
    uint64_t tl = (r < 56) ? 64 : 128;
    uint64_t bits = len * 8;
    for (int i = 0; i < 8; i++) tail[tl - 1 - i] = (uint8_t)(bits >> (8 * i));
    sha256_compress(h, tail);
    if (tl == 128) sha256_compress(h, tail + 64);
    for (int i = 0; i < 8; i++) {
        out[4 * i] = (uint8_t)(h[i] >> 24);
        out[4 * i + 1] = (uint8_t)(h[i] >> 16);
        out[4 * i + 2] = (uint8_t)(h[i] >> 8);
        out[4 * i + 3] = (uint8_t)h[i];
    }
}

/* SN:607-609: StringBuilder of String.format("%02x", b) per digest byte. */
void oracle_hex(const uint8_t d[32], char out[65]) {
    static const char hx[] = "0123456789abcdef";
    for (int i = 0; i < 32; i++) {
        out[2 * i] = hx[d[i] >> 4];
        out[2 * i + 1] = hx[d[i] & 15];
    }
    out[64] = 0;
}

/* ------------------------------------------------------------------ */
/* Base64 (RFC 4648 §4) — java.util.Base64.getEncoder() at SN:636 and   */
/* getDecoder() at SN:281.                                              */
/* ------------------------------------------------------------------ */
static const char B64[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";

uint64_t oracle_b64_encode(const uint8_t* in, uint64_t len, char* out) {
    uint64_t o = 0, i = 0;
    for (; i + 3 <= len; i += 3) {
        uint32_t v = (uint32_t)in[i] << 16 | (uint32_t)in[i + 1] << 8 | in[i + 2];
        out[o++] = B64[v >> 18];
        out[o++] = B64[(v >> 12) & 63];
        out[o++] = B64[(v >> 6) & 63];
        out[o++] = B64[v & 63];
    }
    uint64_t r = len - i; /* encoder's padding branch: "==" for 1, "=" for 2 */
    if (r == 1) {
        uint32_t v = (uint32_t)in[i] << 16;
        out[o++] = B64[v >> 18];
        out[o++] = B64[(v >> 12) & 63];
        out[o++] = '=';
        out[o++] = '=';
    } else if (r == 2) {
        uint32_t v = (uint32_t)in[i] << 16 | (uint32_t)in[i + 1] << 8;
        out[o++] = B64[v >> 18];
        out[o++] = B64[(v >> 12) & 63];
        out[o++] = B64[(v >> 6) & 63];
        out[o++] = '=';
    }
    return o;
}

static int b64_val(unsigned char c) {
    if (c >= 'A' && c <= 'Z') return c - 'A';
    if (c >= 'a' && c <= 'z') return c - 'a' + 26;
    if (c >= '0' && c <= '9') return c - '0' + 52;
    if (c == '+') return 62;
    if (c == '/') return 63;
    if (c == '=') return -2;
    return -1;
}

/* Restates the JDK basic decoder's state machine (non-MIME): characters
 * are consumed into a 24-bit accumulator from bit 18 down; '=' ends the
 * data and is only legal as "xx==" or "xxx="; a dangling single char, any
 * character outside the alphabet, or anything after the padding is an
 * IllegalArgumentException.  Inputs shorter than 2 chars (except empty)
 * are rejected up front, as the JDK's decodedOutLength does.  Unused low
 * bits of the final unit are not checked (the JDK does not check them). */
int oracle_b64_decode(const char* in, uint64_t len, uint8_t* out, uint64_t* out_len) {
    const unsigned char* s = (const unsigned char*)in;
    uint64_t sp = 0, dp = 0;
    uint32_t bits = 0;
    int shiftto = 18;
    *out_len = 0;
    if (len == 0) return 0;
    if (len < 2) return -1;
    while (sp < len) {
        int b = b64_val(s[sp++]);
        if (b < 0) {
            if (b == -2) {
                if ((shiftto == 6 && (sp == len || s[sp++] != '=')) || shiftto == 18) return -1;
                break;
            }
            return -1;
        }
        bits |= (uint32_t)b << shiftto;
        shiftto -= 6;
        if (shiftto < 0) {
            out[dp++] = (uint8_t)(bits >> 16);
            out[dp++] = (uint8_t)(bits >> 8);
            out[dp++] = (uint8_t)bits;
            shiftto = 18;
            bits = 0;
        }
    }
    if (shiftto == 6) {
        out[dp++] = (uint8_t)(bits >> 16);
    } else if (shiftto == 0) {
        out[dp++] = (uint8_t)(bits >> 16);
        out[dp++] = (uint8_t)(bits >> 8);
    } else if (shiftto == 12) {
        return -1;
    }
    if (sp < len) return -1;
    *out_len = dp;
    return 0;
}

/* ------------------------------------------------------------------ */
/* Split and placement (SN:138-171, 143-145, 196-205, 427-428).         */
/* ------------------------------------------------------------------ */
void oracle_split(uint64_t total, uint32_t parts, uint64_t* off, uint64_t* len) {
    uint64_t base = total / parts, rem = total % parts, o = 0; /* SN:140-141 */
    for (uint32_t i = 0; i < parts; i++) {
        uint64_t part = base + (i < rem ? 1 : 0); /* SN:155 */
        off[i] = o;
        len[i] = part;
        o += part; /* SN:170 */
    }
}

void oracle_fragment_holders(uint32_t f, uint32_t n, uint32_t holders[2]) {
    holders[0] = f;                 /* nodeA = i+1 (1-based), SN:427 */
    holders[1] = (f + n - 1) % n;   /* nodeB = ((i-1+N)%N)+1, SN:428 */
}

/* ------------------------------------------------------------------ */
/* Upload batch (SN:118-189) and download verify (SN:419-458).          */
/* ------------------------------------------------------------------ */
typedef void (*sha_fn)(const uint8_t*, uint64_t, uint8_t*);

static void upload_one(const uint8_t* file, uint64_t flen, uint32_t nfrag, sha_fn sha,
                       uint8_t* fd, uint8_t* frd, char* b64, const uint64_t* b64_off) {
    sha(file, flen, fd); /* fileId, SN:127 */
    uint64_t off[256], len[256];
    uint64_t* po = nfrag <= 256 ? off : (uint64_t*)malloc(8 * nfrag);
    uint64_t* pl = nfrag <= 256 ? len : (uint64_t*)malloc(8 * nfrag);
    oracle_split(flen, nfrag, po, pl);
    for (uint32_t i = 0; i < nfrag; i++) {
        sha(file + po[i], pl[i], frd + 32 * i); /* SN:159 */
        if (b64) oracle_b64_encode(file + po[i], pl[i], b64 + b64_off[i]); /* SN:636 */
    }
    if (po != off) free(po);
    if (pl != len) free(pl);
}

typedef struct {
    const uint8_t* files; const uint64_t* file_off; const uint64_t* file_len;
    uint32_t nfiles, nfrag; uint8_t* fd; uint8_t* frd; char* b64; const uint64_t* b64_off;
    sha_fn sha; uint32_t next; pthread_mutex_t mu;
} batch_job;

static void* batch_worker(void* p) {
    batch_job* j = (batch_job*)p;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        uint32_t f = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (f >= j->nfiles) break;
        upload_one(j->files + j->file_off[f], j->file_len[f], j->nfrag, j->sha, j->fd + 32 * (uint64_t)f,
                   j->frd + 32 * (uint64_t)f * j->nfrag, j->b64, j->b64 ? j->b64_off + (uint64_t)f * j->nfrag : 0);
    }
    return 0;
}

uint64_t oracle_upload_batch(const uint8_t* files, const uint64_t* file_off, const uint64_t* file_len,
                             uint32_t nfiles, uint32_t nfrag, uint8_t* file_digest, uint8_t* frag_digest,
                             char* b64, uint64_t* b64_off, int threads) {
    uint64_t total = 0;
    for (uint32_t f = 0; f < nfiles; f++) {
        uint64_t base = file_len[f] / nfrag, rem = file_len[f] % nfrag;
        for (uint32_t i = 0; i < nfrag; i++) {
            uint64_t l = base + (i < rem ? 1 : 0);
            b64_off[(uint64_t)f * nfrag + i] = total;
            total += 4 * ((l + 2) / 3);
        }
    }
    b64_off[(uint64_t)nfiles * nfrag] = total;
    batch_job j = {files, file_off, file_len, nfiles, nfrag, file_digest, frag_digest, b64, b64_off,
                   oracle_sha256, 0, PTHREAD_MUTEX_INITIALIZER};
    if (threads <= 1) {
        batch_worker(&j);
    } else {
        pthread_t* t = (pthread_t*)malloc(sizeof(pthread_t) * threads);
        for (int i = 0; i < threads; i++) pthread_create(&t[i], 0, batch_worker, &j);
        for (int i = 0; i < threads; i++) pthread_join(t[i], 0);
        free(t);
    }
    return total;
}

int oracle_reassemble_verify(const uint8_t* const* src, const uint64_t* len, uint32_t nfrag,
                             const uint8_t expected[32], uint8_t* out) {
    uint64_t o = 0;
    for (uint32_t i = 0; i < nfrag; i++) { /* ordered append, SN:422-449 */
        if (len[i]) memcpy(out + o, src[i], len[i]);
        o += len[i];
    }
    uint8_t d[32];
    oracle_sha256(out, o, d); /* SN:454 */
    return memcmp(d, expected, 32) == 0 ? 0 : -6; /* SN:455-458 */
}

/* ------------------------------------------------------------------ */
/* Synthetic data: counter-based splitmix64.                            */
/* ------------------------------------------------------------------ */
static uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

void oracle_synth(uint64_t seed, uint64_t f, uint64_t start, uint64_t len, uint8_t* out) {
    uint64_t i = 0;
    while (i < len) {
        uint64_t o = start + i;
        uint64_t v = splitmix64(seed ^ ((f << 40) | (o >> 3)));
        for (uint64_t b = o & 7; b < 8 && i < len; b++, i++) out[i] = (uint8_t)(v >> (8 * b));
    }
}

/* ------------------------------------------------------------------ */
/* CPU baseline (bench.py cpu_baseline leg).                           */
/* ------------------------------------------------------------------ */
typedef unsigned char* (*openssl_sha256_t)(const unsigned char*, size_t, unsigned char*);
static openssl_sha256_t g_ossl_sha256;

static void sha_openssl(const uint8_t* d, uint64_t n, uint8_t* out) { g_ossl_sha256(d, (size_t)n, out); }

typedef struct {
    uint64_t seed; uint32_t nfiles; uint64_t flen; uint32_t nfrag; sha_fn sha;
    uint8_t* fd; uint8_t* frd; uint32_t next; pthread_mutex_t mu; double busy; int err;
} cpu_bench_job;

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void* cpu_bench_worker(void* p) {
    cpu_bench_job* j = (cpu_bench_job*)p;
    uint8_t* file = (uint8_t*)malloc(j->flen ? j->flen : 1);
    uint64_t b64cap = 4 * ((j->flen / j->nfrag + 3) / 3) + 16;
    char* b64 = (char*)malloc(b64cap * 1);
    uint64_t* b64_off = (uint64_t*)calloc(j->nfrag, 8); /* each fragment re-uses one buffer */
    double busy = 0;
    if (!file || !b64 || !b64_off) { j->err = 1; goto out; }
    for (;;) {
        pthread_mutex_lock(&j->mu);
        uint32_t f = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (f >= j->nfiles) break;
        oracle_synth(j->seed, f, 0, j->flen, file);
        double t0 = now_s();
        upload_one(file, j->flen, j->nfrag, j->sha, j->fd + 32 * (uint64_t)f,
                   j->frd + 32 * (uint64_t)f * j->nfrag, b64, b64_off);
        busy += now_s() - t0;
    }
out:
    pthread_mutex_lock(&j->mu);
    if (busy > j->busy) j->busy = busy; /* wall of the slowest worker */
    pthread_mutex_unlock(&j->mu);
    free(file); free(b64); free(b64_off);
    return 0;
}

double oracle_cpu_upload_bench(uint64_t seed, uint32_t nfiles, uint64_t flen, uint32_t nfrag, int threads,
                               int use_openssl, uint8_t* fd, uint8_t* frd) {
    sha_fn sha = oracle_sha256;
    if (use_openssl) {
        if (!g_ossl_sha256) {
            void* h = dlopen("libcrypto.so.3", RTLD_NOW);
            if (!h) h = dlopen("libcrypto.so", RTLD_NOW);
            if (h) g_ossl_sha256 = (openssl_sha256_t)dlsym(h, "SHA256");
        }
        if (!g_ossl_sha256) return -1.0;
        sha = sha_openssl;
    }
    cpu_bench_job j = {seed, nfiles, flen, nfrag, sha, fd, frd, 0, PTHREAD_MUTEX_INITIALIZER, 0.0, 0};
    if (threads < 1) threads = 1;
    pthread_t* t = (pthread_t*)malloc(sizeof(pthread_t) * threads);
    for (int i = 0; i < threads; i++) pthread_create(&t[i], 0, cpu_bench_worker, &j);
    for (int i = 0; i < threads; i++) pthread_join(t[i], 0);
    free(t);
    return j.err ? -2.0 : j.busy;
}

/* Checker for a whole synthetic batch (bench.py's verify leg and the GPU
 * tests): for files [first, first + nfiles) of flen bytes, the fileId
 * (SN:127), every fragment digest (SN:159) and the SHA-256 of every
 * fragment's Base64 text (SN:636: a 32-byte stand-in for the text itself),
 * one file per worker thread.  Returns 0, or < 0 on error. */
typedef struct {
    uint64_t seed, first; uint32_t nfiles; uint64_t flen; uint32_t nfrag; sha_fn sha;
    uint8_t* fd; uint8_t* frd; uint8_t* b64d; uint32_t next; pthread_mutex_t mu; int err;
} digest_job;

static void* digest_worker(void* p) {
    digest_job* j = (digest_job*)p;
    const uint32_t N = j->nfrag;
    uint8_t* file = (uint8_t*)malloc(j->flen ? j->flen : 1);
    char* b64 = (char*)malloc(4 * ((j->flen / N + 3) / 3) + 16);
    uint64_t* off = (uint64_t*)malloc(8 * N);
    uint64_t* len = (uint64_t*)malloc(8 * N);
    if (!file || !b64 || !off || !len) {
        pthread_mutex_lock(&j->mu);
        j->err = 1;
        pthread_mutex_unlock(&j->mu);
        goto out;
    }
    oracle_split(j->flen, N, off, len);
    for (;;) {
        pthread_mutex_lock(&j->mu);
        uint32_t f = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (f >= j->nfiles) break;
        oracle_synth(j->seed, j->first + f, 0, j->flen, file);
        j->sha(file, j->flen, j->fd + 32 * (uint64_t)f);
        for (uint32_t i = 0; i < N; i++) {
            const uint64_t k = (uint64_t)f * N + i;
            j->sha(file + off[i], len[i], j->frd + 32 * k);
            if (j->b64d) {
                const uint64_t n = oracle_b64_encode(file + off[i], len[i], b64);
                j->sha((const uint8_t*)b64, n, j->b64d + 32 * k);
            }
        }
    }
out:
    free(file); free(b64); free(off); free(len);
    return 0;
}

int oracle_synth_digests(uint64_t seed, uint64_t first, uint32_t nfiles, uint64_t flen, uint32_t nfrag, int threads,
                         int use_openssl, uint8_t* fd, uint8_t* frd, uint8_t* b64d) {
    sha_fn sha = oracle_sha256;
    if (use_openssl) {
        if (!g_ossl_sha256) {
            void* h = dlopen("libcrypto.so.3", RTLD_NOW);
            if (!h) h = dlopen("libcrypto.so", RTLD_NOW);
            if (h) g_ossl_sha256 = (openssl_sha256_t)dlsym(h, "SHA256");
        }
        if (!g_ossl_sha256) return -1;
        sha = sha_openssl;
    }
    if (!nfrag) return -3;
    digest_job j = {seed, first, nfiles, flen, nfrag, sha, fd, frd, b64d, 0, PTHREAD_MUTEX_INITIALIZER, 0};
    if (threads < 1) threads = 1;
    pthread_t* t = (pthread_t*)malloc(sizeof(pthread_t) * threads);
    for (int i = 0; i < threads; i++) pthread_create(&t[i], 0, digest_worker, &j);
    for (int i = 0; i < threads; i++) pthread_join(t[i], 0);
    free(t);
    return j.err ? -2 : 0;
}

/* Download-side CPU baseline (bench.py cpu_baseline leg, download object):
 * per file, what the GPU download path computes — Base64-decode every
 * fragment (SN:281), SHA-256 it against the upload-time digest (SN:282,
 * 248-257), ordered append into the file (SN:448-451), SHA-256 of the
 * rebuilt file against the fileId (SN:454-458).  The Base64 and the expected
 * digests are prepared per file outside the timed part (they stand for the
 * fetched fragments and the digest table).  Returns the slowest worker's
 * busy seconds, or < 0 on error / mismatch. */
/* Table-driven decode of the body units, 4 chars -> 3 bytes per step (the
 * shape of the JDK's non-intrinsic decodeBlock), falling back to the exact
 * state machine above for the final unit and for any invalid input. */
static int8_t g_dec[256];
static pthread_once_t g_dec_once = PTHREAD_ONCE_INIT;
static void dec_init(void) {
    for (int c = 0; c < 256; c++) g_dec[c] = (int8_t)(b64_val((unsigned char)c) >= 0 ? b64_val((unsigned char)c) : -1);
}
static int fast_b64_decode(const char* in, uint64_t len, uint8_t* out, uint64_t* out_len) {
    pthread_once(&g_dec_once, dec_init);
    const unsigned char* s = (const unsigned char*)in;
    if (len < 8 || (len & 3)) return oracle_b64_decode(in, len, out, out_len);
    uint64_t units = len / 4 - 1, dp = 0;
    for (uint64_t u = 0; u < units; u++) {
        const int a = g_dec[s[4 * u]], b = g_dec[s[4 * u + 1]], c = g_dec[s[4 * u + 2]], d = g_dec[s[4 * u + 3]];
        if ((a | b | c | d) < 0) return oracle_b64_decode(in, len, out, out_len);
        const uint32_t v = (uint32_t)a << 18 | (uint32_t)b << 12 | (uint32_t)c << 6 | (uint32_t)d;
        out[dp] = (uint8_t)(v >> 16); out[dp + 1] = (uint8_t)(v >> 8); out[dp + 2] = (uint8_t)v;
        dp += 3;
    }
    uint64_t tail = 0;
    if (oracle_b64_decode(in + 4 * units, 4, out + dp, &tail) != 0) return oracle_b64_decode(in, len, out, out_len);
    *out_len = dp + tail;
    return 0;
}

typedef struct {
    uint64_t seed; uint32_t nfiles; uint64_t flen; uint32_t nfrag; sha_fn sha;
    uint32_t next; pthread_mutex_t mu; double busy; int err;
} cpu_dl_job;

static void* cpu_dl_worker(void* p) {
    cpu_dl_job* j = (cpu_dl_job*)p;
    const uint32_t N = j->nfrag;
    uint8_t* file = (uint8_t*)malloc(j->flen ? j->flen : 1);
    uint8_t* out = (uint8_t*)malloc(j->flen ? j->flen : 1);
    uint64_t fcap = j->flen / N + 1;
    uint8_t* frag = (uint8_t*)malloc(fcap + 3);
    char* b64 = (char*)malloc(N * (4 * ((fcap + 2) / 3)) + 16);
    uint64_t* off = (uint64_t*)malloc(8 * N);
    uint64_t* len = (uint64_t*)malloc(8 * N);
    uint64_t* boff = (uint64_t*)malloc(8 * (N + 1));
    uint8_t* exp = (uint8_t*)malloc(32 * (N + 1));
    double busy = 0;
    int err = 0;
    if (!file || !out || !frag || !b64 || !off || !len || !boff || !exp) { err = 1; goto done; }
    oracle_split(j->flen, N, off, len);
    for (;;) {
        pthread_mutex_lock(&j->mu);
        uint32_t f = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (f >= j->nfiles) break;
        oracle_synth(j->seed, f, 0, j->flen, file);
        boff[0] = 0;
        for (uint32_t i = 0; i < N; i++) {
            boff[i + 1] = boff[i] + oracle_b64_encode(file + off[i], len[i], b64 + boff[i]);
            j->sha(file + off[i], len[i], exp + 32 * i);
        }
        j->sha(file, j->flen, exp + 32 * N);
        double t0 = now_s();
        uint64_t o = 0;
        for (uint32_t i = 0; i < N; i++) {
            uint64_t got = 0;
            uint8_t d[32];
            if (fast_b64_decode(b64 + boff[i], boff[i + 1] - boff[i], frag, &got) != 0) err = 1; /* SN:281 */
            j->sha(frag, got, d);                                                                  /* SN:282 */
            if (memcmp(d, exp + 32 * i, 32) != 0) err = 1;                                        /* SN:250-257 */
            memcpy(out + o, frag, got);                                                            /* SN:448 */
            o += got;
        }
        uint8_t d[32];
        j->sha(out, o, d);                                   /* SN:454 */
        if (memcmp(d, exp + 32 * N, 32) != 0) err = 1;       /* SN:455-458 */
        busy += now_s() - t0;
    }
done:
    pthread_mutex_lock(&j->mu);
    if (busy > j->busy) j->busy = busy;
    if (err) j->err = 1;
    pthread_mutex_unlock(&j->mu);
    free(file); free(out); free(frag); free(b64); free(off); free(len); free(boff); free(exp);
    return 0;
}

double oracle_cpu_download_bench(uint64_t seed, uint32_t nfiles, uint64_t flen, uint32_t nfrag, int threads,
                                 int use_openssl) {
    sha_fn sha = oracle_sha256;
    if (use_openssl) {
        if (!g_ossl_sha256) {
            void* h = dlopen("libcrypto.so.3", RTLD_NOW);
            if (!h) h = dlopen("libcrypto.so", RTLD_NOW);
            if (h) g_ossl_sha256 = (openssl_sha256_t)dlsym(h, "SHA256");
        }
        if (!g_ossl_sha256) return -1.0;
        sha = sha_openssl;
    }
    cpu_dl_job j = {seed, nfiles, flen, nfrag, sha, 0, PTHREAD_MUTEX_INITIALIZER, 0.0, 0};
    if (threads < 1) threads = 1;
    pthread_t* t = (pthread_t*)malloc(sizeof(pthread_t) * threads);
    for (int i = 0; i < threads; i++) pthread_create(&t[i], 0, cpu_dl_worker, &j);
    for (int i = 0; i < threads; i++) pthread_join(t[i], 0);
    free(t);
    return j.err ? -2.0 : j.busy;
}
