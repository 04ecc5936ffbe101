/*
 * dfs_oracle.h — CPU restatement of the StorageNode fragment pipeline.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the HIP
 * path.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load it.  The product library (libdfsgpu.so) never links or calls it.
 *
 * Reference: hiagoluansilva/distributed-file-storage,
 *            storage-node/src/StorageNode.java (cited as SN:line).
 * The reference's arithmetic lives in the JDK (java.security.MessageDigest
 * "SHA-256", java.util.Base64 basic encoder/decoder; JDK version unpinned,
 * >= 11 inferred).  Those are restated here from FIPS 180-4 and RFC 4648 plus
 * the JDK decoder's documented error behaviour.  Parity is pinned by the
 * golden vectors in tests/golden/ (FIPS/RFC known answers and the
 * reference's own examples/ files), not by running the reference: no JDK
 * exists in this image.
 */
#ifndef DFS_ORACLE_H
#define DFS_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* FIPS 180-4 SHA-256.  Replaces MessageDigest.digest (SN:603-613). */
void oracle_sha256(const uint8_t* data, uint64_t len, uint8_t out[32]);

/* Lowercase %02x hex of a 32-byte digest (SN:608).  out: 65 bytes. */
void oracle_hex(const uint8_t digest[32], char out[65]);

/* Base64.getEncoder().encodeToString (SN:636): RFC 4648 basic alphabet,
 * '=' padding, no line breaks.  Returns chars written = 4*ceil(len/3). */
uint64_t oracle_b64_encode(const uint8_t* in, uint64_t len, char* out);

/* Base64.getDecoder().decode (SN:281).  Returns 0 and sets *out_len on
 * success, -1 where the JDK throws IllegalArgumentException.  `out` must hold
 * 3*ceil(len/4) bytes. */
int oracle_b64_decode(const char* in, uint64_t len, uint8_t* out, uint64_t* out_len);

/* Split plan of handleUpload (SN:138-171): fragment i has length
 * floor(S/N) + (i < S mod N) and starts after fragments 0..i-1. */
void oracle_split(uint64_t file_len, uint32_t nfrag, uint64_t* off, uint64_t* len);

/* Placement (SN:143-145, 196-205): 0-based node k stores fragments
 * {k, (k+1) mod N}.  Writes the two holders of fragment f (0-based nodes):
 * holders[0] = f (download candidate nodeA, SN:427) and
 * holders[1] = (f-1+N) mod N (candidate nodeB, SN:428). */
void oracle_fragment_holders(uint32_t f, uint32_t nfrag, uint32_t holders[2]);

/* Upload half over a batch of files laid out in one buffer (SN:118-189):
 * file_digest[f] = SHA-256(file f) (SN:127), frag_digest[f*N+i] =
 * SHA-256(fragment i) (SN:159), b64 = concatenation of the Base64 of every
 * fragment in (file, fragment) order (SN:636); b64_off has nfiles*N+1
 * entries (prefix offsets).  Returns total Base64 chars.
 * threads<=1 runs serially; otherwise one file per worker thread, mirroring
 * the reference's thread-per-connection handler (SN:30). */
uint64_t oracle_upload_batch(const uint8_t* files, const uint64_t* file_off,
                             const uint64_t* file_len, uint32_t nfiles, uint32_t nfrag,
                             uint8_t* file_digest, uint8_t* frag_digest,
                             char* b64, uint64_t* b64_off, int threads);

/* Download verify (SN:419-458): concatenate fragments in index order into
 * out, SHA-256 the result and compare with expected_file_digest.
 * Returns 0 ok, -6 "File corrupted" (SN:455-458). */
int oracle_reassemble_verify(const uint8_t* const* frag_src, const uint64_t* frag_len,
                             uint32_t nfrag, const uint8_t expected[32], uint8_t* out);

/* Synthetic file bytes: byte o of file f is byte (o mod 8) of
 * splitmix64(seed ^ (f<<40 | o>>3)), little endian. */
void oracle_synth(uint64_t seed, uint64_t file_index, uint64_t start, uint64_t len, uint8_t* out);

/* CPU baseline driver (bench.py cpu_baseline leg only): runs the upload
 * half on `nfiles` synthetic files of `file_len` bytes, generating each
 * file on the worker thread into a private buffer.  use_openssl != 0 uses
 * libcrypto's SHA256 (SHA-NI when the CPU has it, approximating HotSpot's
 * SHA intrinsic); otherwise the scalar restatement.  Returns seconds spent
 * hashing + encoding (generation excluded), or < 0 on error. */
double oracle_cpu_upload_bench(uint64_t seed, uint32_t nfiles, uint64_t file_len,
                               uint32_t nfrag, int threads, int use_openssl,
                               uint8_t* file_digest_out, uint8_t* frag_digest_out);
/* Checker for a whole synthetic batch: files [first, first + nfiles) of
 * file_len bytes (oracle_synth): file_digest (nfiles x 32, SN:127),
 * frag_digest (nfiles x nfrag x 32, SN:159) and, if b64_digest is not NULL,
 * the SHA-256 of every fragment's Base64 text (SN:636), one file per worker
 * thread.  use_openssl as above (a second, independent SHA-256).  0 or < 0. */
int oracle_synth_digests(uint64_t seed, uint64_t first, uint32_t nfiles, uint64_t file_len, uint32_t nfrag,
                         int threads, int use_openssl, uint8_t* file_digest, uint8_t* frag_digest,
                         uint8_t* b64_digest);
/* Download-side CPU baseline: per file, Base64-decode each fragment (SN:281),
 * SHA-256 it against the upload digest (SN:282), ordered append (SN:448),
 * SHA-256 of the file against its fileId (SN:454).  Seconds of the slowest
 * worker (fragment Base64 and expected digests prepared untimed), < 0 on
 * error or mismatch. */
double oracle_cpu_download_bench(uint64_t seed, uint32_t nfiles, uint64_t file_len, uint32_t nfrag,
                                 int threads, int use_openssl);

#ifdef __cplusplus
}
#endif
#endif
