/*
 * dfs_gpu.h — C ABI of libdfsgpu.so, the MI355X (gfx950) fragment pipeline.
 *
 * This is the drop-in boundary for StorageNode's fragment pipeline
 * (hiagoluansilva/distributed-file-storage, storage-node/src/StorageNode.java,
 * cited as SN:line).  The reference has no plugin/FFI API: its hot path is
 * private methods and JDK calls.  Each entry point below replaces the listed
 * reference sites; a Java host binds them through FFM (java.lang.foreign) or
 * JNI.  HTTP routes, JSON bodies, manifest.json and
 * the on-disk layout are unchanged.
 *
 * Conventions
 *  - Plain C types only.  The caller owns every buffer; the library never
 *    returns memory.  The library owns device scratch and streams in a ctx.
 *  - Every function returns an int: DFS_OK (0) or a negative DFS_E_* code.
 *  - Data pointers are host memory unless `flags` has DFS_DEVICE_PTRS, in
 *    which case they are HIP device pointers and the call is asynchronous on
 *    the ctx's stream (see dfs_set_stream); descriptor arrays (spans, offsets,
 *    pointer tables) are always host memory.
 *  - Digests are the raw 32-byte SHA-256; the Java side formats lowercase hex
 *    exactly as sha256Hex does (SN:607-609).
 *  - A ctx serialises its own calls (one mutex), so StorageNode's
 *    thread-per-connection handlers (SN:30) may share one ctx.  The stream
 *    set by dfs_set_stream is ctx state (not per thread).  Asynchronous
 *    (DFS_DEVICE_PTRS) calls reuse the ctx's device scratch: a call issued on
 *    another stream than the previous one first waits (on the device) for
 *    the previous call's scratch use, so switching streams is always safe.
 *    An upload plan runs one launch at a time: two concurrent runs of the
 *    same plan must be on the same stream.
 *  - For many small concurrent requests use the batcher (dfs_batcher_*),
 *    which coalesces them into one launch.
 *  - No CPU fallback: without a usable gfx950 device dfs_open fails with
 *    DFS_E_NODEV and nothing else runs.
 */
#ifndef DFS_GPU_H
#define DFS_GPU_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DFS_ABI_VERSION 3

/* Return codes. */
#define DFS_OK 0
#define DFS_E_ARG (-1)          /* invalid argument / capacity too small          */
#define DFS_E_HIP (-2)          /* HIP runtime error (maps to RuntimeException,   */
                                /* the catch-all of sha256Hex, SN:610-611)        */
#define DFS_E_NOMEM (-3)        /* device or pinned allocation failed             */
#define DFS_E_DECODE (-4)       /* Base64 IllegalArgumentException (SN:281)       */
#define DFS_E_MISSING (-5)      /* "Could not retrieve fragment i" (SN:443-446)   */
#define DFS_E_CORRUPT (-6)      /* "File corrupted": SHA-256(file)!=fileId (SN:455)*/
#define DFS_E_FRAG_MISMATCH (-7) /* "Hash mismatch on fragment" (SN:250-257)      */
#define DFS_E_NODEV (-8)        /* no gfx950 device                               */
#define DFS_E_WIRE (-9)         /* storeFragments body not in buildFragmentsJson  */
                                /* form: the host parses it with parseJson        */
#define DFS_E_IO (-10)          /* fragment store: Files.write / readAllBytes      */
                                /* IOException (SN:166, 285, 466)                 */
#define DFS_E_COMM (-11)        /* RCCL error (the peer POST failed, SN:218-221)   */
#define DFS_E_TOOBIG (-12)      /* dfs_sha256_batch_static: more messages than     */
                                /* DFS_STATIC_MAX_MSGS                             */

/* Flags. */
#define DFS_DEVICE_PTRS 0x1u    /* data pointers are device pointers; async       */
#define DFS_NO_FILEID 0x2u      /* upload: skip the whole-file SHA-256            */
#define DFS_NO_B64 0x4u         /* upload: skip the Base64 encode                 */
#define DFS_SERIAL 0x8u         /* upload: separate SHA and Base64 kernels, one   */
                                /* stream (default: Base64 fused into the SHA     */
                                /* fragment lanes, or DFS_UPLOAD_MODE=kernels:    */
                                /* the two kernels on two streams)                */
#define DFS_B64_ONLY 0x80u      /* upload plan: only the Base64 encode kernel     */
                                /* (measurement of the HBM-bound pass alone)      */

typedef struct dfs_ctx dfs_ctx;
typedef struct dfs_upload_plan dfs_upload_plan;

/* One message: `len` bytes starting `off` bytes past a base pointer. */
typedef struct dfs_span {
    uint64_t off;
    uint64_t len;
} dfs_span;
#define DFS_SPAN_MISSING UINT64_MAX

/* ---- context ------------------------------------------------------------ */
int dfs_open(dfs_ctx** ctx, int device);
int dfs_close(dfs_ctx* ctx);
const char* dfs_strerror(int code);
int dfs_abi_version(void);
/* Run subsequent calls on `hip_stream` (a hipStream_t; NULL = the ctx's own).
 * The ctx's own stream is non-blocking: it does not wait for the legacy
 * default stream or for any other stream.  A DFS_DEVICE_PTRS caller whose own
 * work fills or reads the buffers on another stream must order the two
 * itself: hand that stream in here, or synchronise / use events around the
 * call.  (Seen without it: a zero fill queued on the default stream just
 * before an encode landed after it and wiped the encode's output.) */
int dfs_set_stream(dfs_ctx* ctx, void* hip_stream);
/* When on, every call records HIP events around each kernel on the stream it
 * is launched on; dfs_get_timings returns the last call's per-stage ms. */
int dfs_set_profiling(dfs_ctx* ctx, int on);
#define DFS_T_SHA 0      /* multi-message SHA-256 kernel          */
#define DFS_T_B64ENC 1   /* Base64 encode kernel                  */
#define DFS_T_B64DEC 2   /* Base64 decode (+ fused gather) kernel */
#define DFS_T_GATHER 3   /* reassembly gather kernel              */
#define DFS_T_TOTAL 4    /* whole call, first launch to last     */
#define DFS_T_COUNT 5
int dfs_get_timings(dfs_ctx* ctx, float* ms, int n);
/* Counters of the ctx since dfs_open (diagnostics, no reference equivalent):
 * DFS_S_OVL_REDO = decode-ahead downloads whose SHA launch was redone after
 * the decode because an in-kernel wait for a fragment group timed out (the
 * results are still exact; the call was slow). */
#define DFS_S_OVL_REDO 0
#define DFS_S_RECV_ONE_PASS 1 /* dfs_receive_fragments_batch calls that ran in one pass */
#define DFS_S_COUNT 2
int dfs_get_stats(dfs_ctx* ctx, uint64_t* out, int n);

/* ---- pure host helpers (no device) ---------------------------------------- */
/* handleUpload's split (SN:138-171): fragment i has floor(S/N) + (i < S mod N)
 * bytes, contiguous, in order.  frags: nfrag entries. */
int dfs_split_plan(uint64_t file_len, uint32_t nfrag, dfs_span* frags);
/* 4*ceil(n/3): length of Base64.getEncoder().encodeToString (SN:636). */
uint64_t dfs_b64_encoded_len(uint64_t n);
/* 3*ceil(n/4): capacity bound for decoding n Base64 chars (SN:281). */
uint64_t dfs_b64_decoded_cap(uint64_t n);
/* Placement (SN:143-145, 196-205, 427-428): the 0-based nodes holding
 * fragment f are holders[0] = f and holders[1] = (f-1+N) mod N; node k
 * stores {k, (k+1) mod N}. */
int dfs_fragment_holders(uint32_t frag, uint32_t nfrag, uint32_t holders[2]);

/* ---- batch entry points ----------------------------------------------------- */
/* sha256Hex at SN:127, 159, 282, 454 for `n` messages of one buffer:
 * digests[32*i] = SHA-256(base + msgs[i].off, msgs[i].len). */
int dfs_sha256_batch(dfs_ctx* ctx, const uint8_t* base, const dfs_span* msgs, uint32_t n,
                     uint8_t* digests, uint32_t flags);

/* dfs_sha256_batch for callers that cannot allocate device memory.  It has no
 * counterpart in the reference; it exists for code under HIP graph capture,
 * tight serving loops and harnesses that forbid hipMalloc.  Same digests as
 * dfs_sha256_batch (sha256Hex, SN:603-613) with DFS_DEVICE_PTRS, but:
 *  - every argument is device memory, the spans included: d_msgs[i] =
 *    {off, len} of message i in d_base; d_digests gets n*32 bytes;
 *  - d_status (n entries, may be NULL) gets 0, or DFS_E_ARG for a message of
 *    2^37 bytes or more (its digest is then that of the empty message);
 *  - the lane descriptors and work-queue words live in a static device array
 *    of the library (about 2.6 MB per GPU, held until the process ends), so
 *    the call makes no hipMalloc / hipFree and stages nothing on the host;
 *  - n > DFS_STATIC_MAX_MSGS returns DFS_E_TOOBIG before anything is launched;
 *  - asynchronous on the ctx stream.  Every call on one GPU (any ctx, any
 *    process thread) shares that GPU's array: calls that overlap on one GPU
 *    race, so order them on one stream or with events. */
#define DFS_STATIC_MAX_MSGS 65536u
int dfs_sha256_batch_static(dfs_ctx* ctx, const uint8_t* d_base, const dfs_span* d_msgs, uint32_t n,
                            uint8_t* d_digests, int32_t* d_status);

/* Streaming SHA-256 for messages too long to hold at once (the 256 MiB skew
 * config): each call hashes the next part of every message.
 *   parts[i]     the bytes of message i in this call (base + off, len)
 *   state        n*8 uint32 running states (device memory with
 *                DFS_DEVICE_PTRS, else host); read unless DFS_SHA_BEGIN,
 *                written unless DFS_SHA_FINAL
 *   DFS_SHA_FINAL  this is the last part: pad with total_len[i] (host array,
 *                whole-message length) and write digests[32*i]
 * Every non-final part must be a multiple of 64 bytes (DFS_E_ARG otherwise).
 * Concatenated calls give exactly MessageDigest.digest of the whole message. */
#define DFS_SHA_BEGIN 0x20u
#define DFS_SHA_FINAL 0x40u
int dfs_sha256_update_batch(dfs_ctx* ctx, const uint8_t* base, const dfs_span* parts, uint32_t n,
                            uint32_t* state, const uint64_t* total_len, uint8_t* digests, uint32_t flags);

/* Streaming SHA-256 with per-part state slots and flags: one call advances
 * any subset of a larger set of messages, each at its own stage (the chunked
 * upload of files larger than HBM, BASELINE config 4, where fragment i of a
 * file begins and ends in different chunks than the file's fileId message).
 *   parts[i].off/len  bytes of this part (base + off); len % 64 == 0 unless
 *                     DFS_SHA_FINAL is set in parts[i].flags
 *   parts[i].total    whole-message length (used with DFS_SHA_FINAL)
 *   parts[i].slot     message index: state + 8*slot, digests + 32*slot
 *   parts[i].flags    DFS_SHA_BEGIN (start from H0, state not read) and/or
 *                     DFS_SHA_FINAL (pad, write the digest, state not written)
 * A slot may appear at most once per call.  `base`, `state`, `digests` are
 * device pointers (DFS_DEVICE_PTRS is required); the call is asynchronous on
 * the ctx stream.  Same kernel as dfs_sha256_batch (sha256_lanes). */
typedef struct dfs_part {
    uint64_t off, len, total;
    uint32_t slot, flags;
} dfs_part;
int dfs_sha256_update_parts(dfs_ctx* ctx, const uint8_t* base, const dfs_part* parts, uint32_t n,
                            uint32_t* state, uint8_t* digests, uint32_t flags);

/* Base64.getEncoder().encodeToString at SN:636 for `n` messages.  Output i is
 * written at out + out_off[i]; out_off (n+1 entries) is computed by the
 * library as the prefix sum of dfs_b64_encoded_len and returned. */
int dfs_b64_encode_batch(dfs_ctx* ctx, const uint8_t* base, const dfs_span* msgs, uint32_t n,
                         char* out, uint64_t out_cap, uint64_t* out_off, uint32_t flags);

/* Base64.getDecoder().decode at SN:281 for `n` messages of `in`.  Message i
 * decodes to out + out_off[i] (caller layout, capacity dfs_b64_decoded_cap);
 * out_len[i] = bytes written; status[i] = 0 or DFS_E_DECODE where the JDK
 * throws IllegalArgumentException.  Returns DFS_E_DECODE if any message
 * failed (after every message was processed). */
int dfs_b64_decode_batch(dfs_ctx* ctx, const char* in, const dfs_span* msgs, uint32_t n,
                         uint8_t* out, const uint64_t* out_off, uint64_t* out_len, int32_t* status,
                         uint32_t flags);

/* The replica receiver, handleInternalStoreFragments (SN:265-293): for each
 * received fragment, Base64-decode it (SN:281) to out + out_off[i] and
 * SHA-256 the decoded bytes (SN:282); digests[32*i] is the hash the node
 * replies with (buildHashResponse, SN:644-655), which the sender compares
 * with its own (SN:248-257).  status[i] / out_len[i] as dfs_b64_decode_batch;
 * digests of failed messages are left untouched.  Synchronous. 
 * A batch of more than 32,768 messages whose chars start on 4-byte boundaries
 * of `in` and decode to 16-byte aligned places of `out` is decoded and hashed
 * in one pass, every message by one lane; other batches by the decode kernel
 * followed by the SHA-256 lanes.  Same results; DFS_RECV_FUSED=0 at dfs_open
 * keeps the two kernels. */
int dfs_receive_fragments_batch(dfs_ctx* ctx, const char* in, const dfs_span* msgs, uint32_t n,
                                uint8_t* out, const uint64_t* out_off, uint64_t* out_len, uint8_t* digests,
                                int32_t* status, uint32_t flags);

/* The upload half of handleUpload (SN:118-189) for a batch of files:
 * fileId (SN:127), N-way split (SN:138-157), fragment SHA-256 (SN:159) and
 * the Base64 of every fragment (SN:636), encoded once each.
 *   file_digest: nfiles*32            frag_digest: nfiles*nfrag*32
 *   b64: concatenation in (file, fragment) order; b64_off: nfiles*nfrag+1
 *   prefix offsets, computed and returned by the library.
 * b64 may be NULL with DFS_NO_B64. */
int dfs_upload_batch(dfs_ctx* ctx, const uint8_t* files, const dfs_span* file_spans, uint32_t nfiles,
                     uint32_t nfrag, uint8_t* file_digest, uint8_t* frag_digest, char* b64,
                     uint64_t b64_cap, uint64_t* b64_off, uint32_t flags);

/* handleDownload's gather + verify (SN:419-458): file f is rebuilt at
 * out + file_off[f] from fragments frag_src[f*nfrag+i] (frag_len bytes each,
 * in index order, SN:448); file_digest_out[f] = SHA-256(rebuilt file) (SN:454)
 * and status[f] = 0, DFS_E_MISSING (a NULL source, SN:443-446) or
 * DFS_E_CORRUPT (digest != expected_file_digest[f], SN:455-458).
 * expected_file_digest may be NULL (status then only reports MISSING);
 * expected_file_digest, file_digest_out and status are host memory in every
 * mode (DFS_DEVICE_PTRS covers frag_src and out). */
int dfs_reassemble_verify(dfs_ctx* ctx, const uint8_t* const* frag_src, const uint64_t* frag_len,
                          uint32_t nfiles, uint32_t nfrag, uint8_t* out, const uint64_t* file_off,
                          const uint8_t* expected_file_digest, uint8_t* file_digest_out,
                          int32_t* status, uint32_t flags);

/* Download with Base64 transport: per file, Base64-decode each fragment
 * (SN:281) straight into its place in the file (gather keyed on the split
 * offsets, SN:138-157/448), SHA-256 every fragment against the upload-time
 * digests (the receiver/sender check of SN:282 + 250-257), then SHA-256 the
 * whole file against its fileId (SN:454-458).
 *   b64_msgs: nfiles*nfrag spans into `b64`; a span with
 *             len == DFS_SPAN_MISSING marks a fragment no holder could
 *             supply -> DFS_E_MISSING
 *   file_len: original sizes (the split plan is recomputed from them)
 *   expected_frag_digest: nfiles*nfrag*32 (may be NULL)
 *   expected_file_digest: nfiles*32 (may be NULL)
 *   status[f]: 0 / DFS_E_MISSING / DFS_E_DECODE / DFS_E_FRAG_MISMATCH /
 *              DFS_E_CORRUPT (first failure in pipeline order).
 * status is host memory in every mode; the call synchronises. */
int dfs_download_batch(dfs_ctx* ctx, const char* b64, const dfs_span* b64_msgs, uint32_t nfiles,
                       uint32_t nfrag, const uint64_t* file_len, const uint8_t* expected_frag_digest,
                       const uint8_t* expected_file_digest, uint8_t* out, const uint64_t* file_off,
                       int32_t* status, uint32_t flags);

/* ---- prepared download (descriptor build once, run many; device pointers) -- */
/* dfs_download_batch rebuilds its descriptor tables (decode jobs, SHA lanes,
 * group order) on the host on every call; for a batch shape that repeats —
 * the same spans, file lengths and offsets, e.g. a node serving the same set
 * of files, or a fixed-shape degraded read — a plan builds them once and
 * keeps them in HBM.  Arguments as dfs_download_batch's; the mode (overlap /
 * pipelined / serial) is the ctx's at creation.  nfiles >= 1. */
typedef struct dfs_download_plan dfs_download_plan;
int dfs_download_plan_create(dfs_ctx* ctx, const dfs_span* b64_msgs, uint32_t nfiles, uint32_t nfrag,
                             const uint64_t* file_len, const uint64_t* file_off, dfs_download_plan** plan);
/* d_b64, d_out (16-byte aligned) and the expected digests (may be NULL) are
 * device memory; status (nfiles, host) as dfs_download_batch's.  The call
 * synchronises (the verdict comes back); one run of a plan at a time. */
int dfs_download_plan_run(dfs_ctx* ctx, dfs_download_plan* plan, const char* d_b64,
                          const uint8_t* d_expected_frag_digest, const uint8_t* d_expected_file_digest, uint8_t* d_out,
                          int32_t* status);
int dfs_download_plan_destroy(dfs_download_plan* plan);

/* ---- storeFragments wire codec, sender side (SN:195-205, 629-642) ------- */
/* Length of the storeFragments body carrying fragments a and b of a file of
 * file_len bytes split into nfrag (buildFragmentsJson with two entries and
 * one-digit indices): 139 framing bytes + both Base64 payloads. */
uint64_t dfs_store_body_len(uint64_t file_len, uint32_t nfrag, uint32_t a, uint32_t b);

/* sendFragmentsToPeers + buildFragmentsJson for a whole upload batch, built
 * on the device: for every file f and every peer node k != uploader (0-based,
 * ascending, SN:196-197) the request body
 *   {"fileId":"<hex>","fragments":[{"index":"k","data":"<Base64 of fragment k>"},
 *    {"index":"k+1 mod N","data":"<Base64 of fragment k+1 mod N>"}]}
 * (SN:199-200, 629-642), byte-identical to the reference's, is written at
 * bodies + body_off[f*(nfrag-1) + j], j = k's rank among the peers.  The
 * Base64 is encoded straight from the file bytes into the body (no
 * intermediate string, SN:636-637); the fileId hex comes from file_digest
 * (raw 32 B per file, e.g. dfs_upload_batch's output).
 *   body_off: nfiles*(nfrag-1)+1 entries, filled by the library (each
 *             body starts 1 byte past a 16-byte boundary so both payloads
 *             are dword aligned; last entry = bytes needed); a body's length
 *             is dfs_store_body_len (the gap to the next start is unwritten)
 *   bodies:   NULL = only fill body_off (layout query)
 *   nfrag:    2..10 (one-digit indices keep both payloads dword aligned)
 * With DFS_DEVICE_PTRS, files, file_digest and bodies are device memory
 * (bodies 16-byte aligned) and the call is asynchronous. */
int dfs_store_bodies_build(dfs_ctx* ctx, const uint8_t* files, const dfs_span* file_spans, uint32_t nfiles,
                           uint32_t nfrag, uint32_t uploader, const uint8_t* file_digest, char* bodies,
                           uint64_t* body_off, uint32_t flags);

/* Receiver side, handleInternalStoreFragments (SN:265-293) for a batch of
 * storeFragments request bodies in buildFragmentsJson form (what
 * dfs_store_bodies_build and the reference's senders write: two entries,
 * one-digit indices): the device parses every body (SN:268-272, parseJson
 * SN:704-753), Base64-decodes both payloads (SN:281) and SHA-256s the
 * decoded fragments (SN:282).  Per body i:
 *   file_ids[64i..]      the fileId string (64 chars, not NUL-terminated)
 *   frag_index[2i+q]     entry q's "index" (q = 0, 1), in body order
 *   out_off              n+1 entries filled by the library: body i's slot
 *                        in out (3*ceil(len/4) + 16 bytes rounded up to a
 *                        multiple of 16, so that both payloads decode to
 *                        16-byte aligned places; out_off[n] = bytes needed)
 *   out + frag_off[2i+q] entry q's decoded bytes (frag_len[2i+q] of them);
 *                        digests[64i + 32q] their SHA-256,
 *                        the hashes of the reply (buildHashResponse, SN:644-655)
 *   status[i]            0, DFS_E_DECODE (IllegalArgumentException, SN:281:
 *                        no reply) or DFS_E_WIRE (body in another form:
 *                        parse it on the host with the reference's parseJson
 *                        and use dfs_receive_fragments_batch)
 * bodies/out device memory with DFS_DEVICE_PTRS; synchronous. */
int dfs_store_bodies_receive(dfs_ctx* ctx, const char* bodies, const dfs_span* body_spans, uint32_t n,
                             uint8_t* out, uint64_t* out_off, uint32_t* frag_index, uint64_t* frag_off,
                             uint64_t* frag_len, uint8_t* digests, char* file_ids, int32_t* status,
                             uint32_t flags);

/* The reply half of the exchange, on the host (a reply is ~200 bytes).
 * Receiver: buildHashResponse (SN:644-655) over the HashMap filled by
 * response.put(index, hash) (SN:277-288), for the n bodies of one
 * dfs_store_bodies_receive call: file_ids (64 chars per body), frag_index
 * (2 per body), digests (2 x 32 raw bytes per body) and status are that
 * call's outputs; a body whose status is not 0 gets no reply (its handler
 * threw, SN:280-282: the sender sees a dropped connection).  Replies are
 * written back to back into out (NULL: lengths only), out_off[n + 1]; a
 * reply is at most dfs_store_hash_response_cap() bytes.
 * Sender: parseResponseHashes (SN:657-701) and the comparison of SN:248-257
 * for n replies (spans into `responses`; len 0 = no reply): frag_index and
 * expected (2 x 32 raw bytes per body) are what the sender put into body i.
 * status[i] = 0, DFS_E_FRAG_MISMATCH ("Hash mismatch on fragment", or no
 * entry for a fragment) or DFS_E_WIRE (where the Java parser throws); each
 * makes that attempt fail (SN:212-221).  Returns 0 or the first failure. */
uint64_t dfs_store_hash_response_cap(void);
int dfs_store_hash_responses_build(const char* file_ids, const uint32_t* frag_index, const uint8_t* digests,
                                   const int32_t* status, uint32_t n, char* out, uint64_t out_cap, uint64_t* out_off);
int dfs_store_hash_responses_check(const char* responses, const dfs_span* spans, uint32_t n,
                                   const uint32_t* frag_index, const uint8_t* expected, int32_t* status);

/* ---- on-disk fragment store (SN:147-149, 163-166, 273-285, 463-469) ------ */
/* A node's fragments live at
 *   <node_root>/<fileId hex>/fragments/<index>.frag
 * holding the raw fragment bytes (Files.write of the byte[] at SN:166 on
 * upload and SN:285 on the replica receiver; read back by
 * tryLoadFragmentLocal, SN:463-469).  node_root is the reference's dataRoot,
 * data/node-<id> (SN:20).  The manifest.json beside them is not written here.
 *   file_digest  host memory, 32 raw bytes per file; the directory name is
 *                its lowercase hex (sha256Hex, SN:607-609); nfiles entries
 *   refs[i]      fragment i: bytes data + off, len of them (read: capacity),
 *                of file refs[i].file (< nfiles, else DFS_E_ARG before any
 *                I/O), fragment number refs[i].index
 *   status[i]    0, DFS_E_IO (write / read failed), DFS_E_MISSING (read:
 *                no such file, tryLoadFragmentLocal returns null) or
 *                DFS_E_ARG (read: the file is longer than len)
 * Directories are created as Files.createDirectories does (SN:149, 275);
 * files are created or truncated (Files.write's default options); a
 * fragment larger than one staging slot (DFS_STORE_SLOT_MB, 64 MiB) is
 * written to <index>.frag.tmp and renamed into place when complete.  With
 * DFS_DEVICE_PTRS `data` is device memory: the bytes move through the ctx's
 * pinned staging ring (HBM <-> host on the ctx stream, overlapped with the
 * file I/O of a process-wide thread pool).  Ordering: the copies run on the
 * ctx stream only, so work that produces `data` (write) or reads it back
 * (read) on another stream must be ordered by the caller (dfs_set_stream to
 * that stream, or synchronise it first).  Device calls hold the staging
 * ring's own lock, not the ctx lock.  Without DFS_DEVICE_PTRS `data` is host
 * memory, no lock is taken and ctx may be NULL (pure file I/O).  Returns
 * DFS_OK or the first failing status; every ref is attempted.  Synchronous. */
typedef struct dfs_frag_ref {
    uint64_t off;
    uint64_t len;
    uint32_t file;
    uint32_t index;
} dfs_frag_ref;
int dfs_store_write_fragments(dfs_ctx* ctx, const char* node_root, const uint8_t* file_digest, uint32_t nfiles,
                              const uint8_t* data, const dfs_frag_ref* refs, uint32_t n, int32_t* status,
                              uint32_t flags);
/* out_len[i] = bytes of fragment i (the file's size) when status[i] is 0. */
int dfs_store_read_fragments(dfs_ctx* ctx, const char* node_root, const uint8_t* file_digest, uint32_t nfiles,
                             uint8_t* data, const dfs_frag_ref* refs, uint32_t n, uint64_t* out_len,
                             int32_t* status, uint32_t flags);

/* ---- prepared upload (descriptor build once, run many; device pointers) --- */
/* flags: DFS_LAYOUT_FRAG_MAJOR stores the Base64 of fragment i of every file
 * contiguously ([fragment][file] order) so the bytes bound for one node are
 * one span (multi-GPU placement exchange); default is [file][fragment]. */
#define DFS_LAYOUT_FRAG_MAJOR 0x10u
/* DFS_LAYOUT_ALIGN128 starts every fragment's Base64 on a 128-byte boundary
 * (gaps between fragments are left unwritten): the fused upload then stores
 * whole 128-byte lines.  Fragment ends are start + dfs_b64_encoded_len. */
#define DFS_LAYOUT_ALIGN128 0x100u
int dfs_upload_plan_create(dfs_ctx* ctx, const dfs_span* file_spans, uint32_t nfiles, uint32_t nfrag,
                           uint32_t flags, dfs_upload_plan** plan, uint64_t* b64_total);
/* Copy the plan's Base64 offsets to host memory: nfiles*nfrag+1 entries,
 * entry f*nfrag+i is where fragment i of file f starts (its length is
 * dfs_b64_encoded_len of the fragment); the last entry is the total. */
int dfs_upload_plan_b64_offsets(const dfs_upload_plan* plan, uint64_t* b64_off);
/* Run the plan on device buffers (always asynchronous on the ctx stream). */
int dfs_upload_plan_run(dfs_ctx* ctx, dfs_upload_plan* plan, const uint8_t* d_files,
                        uint8_t* d_file_digest, uint8_t* d_frag_digest, char* d_b64, uint32_t flags);
int dfs_upload_plan_destroy(dfs_upload_plan* plan);

/* ---- request batcher: thread-per-connection callers (SN:28-31) ---------- */
/* StorageNode's handlers each process ONE file (handleUpload SN:118-189,
 * handleDownload SN:399-461) on their own thread.  A batcher coalesces the
 * concurrent calls: dfs_submit_* blocks the calling thread, a worker runs
 * every request queued within max_wait_us of the oldest (or until max_files
 * / max_bytes) as one launch, and `depth` workers keep batches in flight
 * (each has its own ctx, stream, pinned staging and device buffers).  All
 * buffers are host memory.  A request whose input AND output each lie inside
 * one dfs_host_alloc buffer is "direct": the worker's DMA reads and writes
 * those buffers, nothing is copied on the host.  Any other request's bytes
 * are copied by its own (handler) thread into / out of the worker's pinned
 * staging.  Thread-safe; results are bit-identical to
 * dfs_upload_batch / dfs_download_batch on the same file.  Zero fields of
 * opts take the defaults (200 us, 1024 files, 1 GiB, depth 2). */
typedef struct dfs_batcher dfs_batcher;
typedef struct dfs_batcher_opts {
    uint32_t max_wait_us;
    uint32_t max_files;
    uint64_t max_bytes;
    uint32_t depth;
    uint32_t reserved;
} dfs_batcher_opts;
int dfs_batcher_create(int device, uint32_t nfrag, const dfs_batcher_opts* opts, dfs_batcher** batcher);
/* Pinned host memory for request buffers (a handler's upload body, its
 * Base64 answer, the file it returns): page-locked, so the batcher moves a
 * direct request over PCIe without a staging copy.  From Java: allocate the
 * per-connection buffers once (MemorySegment.ofAddress(p).reinterpret(n)).
 * dfs_host_free takes exactly the pointer dfs_host_alloc returned. */
int dfs_host_alloc(uint64_t bytes, void** p);
int dfs_host_free(void* p);
/* Stops accepting requests, finishes the queued ones, joins the workers. */
int dfs_batcher_destroy(dfs_batcher* batcher);
typedef struct dfs_batcher_stats_t {
    uint64_t batches, requests, max_batch;
    double queue_s;      /* requests' time from submit to a worker taking them (summed) */
    double stage_in_s;   /* workers waiting for handlers to copy inputs in       */
    double device_s;     /* H2D + kernels + D2H per batch                        */
    double stage_out_s;  /* workers waiting for handlers to copy outputs out     */
    double enqueue_s;    /* handlers' time from the call to holding a queue slot */
    double return_s;     /* handlers' time from results ready to returning       */
    uint64_t direct;     /* requests moved straight from / to dfs_host_alloc buffers */
    uint64_t views;      /* requests whose output was handed out as a view           */
} dfs_batcher_stats_t;
int dfs_batcher_stats(dfs_batcher* batcher, dfs_batcher_stats_t* stats);
/* One upload (SN:127, 138-159, 636): file_digest[32], frag_digest[nfrag*32],
 * the fragments' Base64 back to back in b64 (b64_off[nfrag+1], relative). */
int dfs_submit_upload(dfs_batcher* batcher, const uint8_t* file, uint64_t len, uint8_t* file_digest,
                      uint8_t* frag_digest, char* b64, uint64_t b64_cap, uint64_t* b64_off);
/* One download with Base64 transport (SN:281-282, 422-458): frags[nfrag]
 * spans into b64 (len DFS_SPAN_MISSING = no holder had it); out = file_len
 * bytes; returns 0 / DFS_E_MISSING / DFS_E_DECODE / DFS_E_FRAG_MISMATCH /
 * DFS_E_CORRUPT as dfs_download_batch's status.  Expected digests may be
 * NULL (not checked). */
int dfs_submit_download(dfs_batcher* batcher, const char* b64, const dfs_span* frags, uint64_t file_len,
                        const uint8_t* expected_frag_digest, const uint8_t* expected_file_digest, uint8_t* out);

/* One download as the reference has it (handleDownload, SN:419-458): the
 * fragments arrive as RAW bytes (tryLoadFragmentLocal SN:463-469 or a peer's
 * getFragment reply, SN:513-514), frags[i] / frag_len[i] in index order
 * (nfrag of them).  They are appended in order into `out` (SN:448) and the
 * rebuilt file is SHA-256ed (SN:454): file_digest_out (may be NULL) gets the
 * digest.  Returns 0, DFS_E_MISSING (a NULL fragment of non-zero length:
 * "Could not retrieve fragment i", SN:443-446, nothing is hashed) or
 * DFS_E_CORRUPT (digest != expected_file_digest, SN:455-458; `out` is left
 * untouched).  expected_file_digest may be NULL (not checked). */
int dfs_submit_reassemble(dfs_batcher* batcher, const uint8_t* const* frags, const uint64_t* frag_len,
                          const uint8_t* expected_file_digest, uint8_t* out, uint8_t* file_digest_out);

/* Outputs as views.  A handler does not need its own copy of the answer: it
 * forwards the Base64 to the peers (sendFragmentsBulk, SN:226-246) or the file
 * to the client (SN:460) and is done with it.  The *_view calls leave the
 * output where the batch's single device-to-host DMA put it, in pinned memory
 * the batcher owns, and return a pointer to it: no copy on the host and one
 * DMA per batch instead of one per request (a pinned caller's per-request
 * DMAs reach 36-40 GB/s on a link that moves 56 GB/s in one piece).  The
 * input is read in place if it lies in a dfs_host_alloc buffer, else staged
 * as for dfs_submit_upload.  *view is the handle to give back with
 * dfs_view_release once the bytes have been used (NULL when the call failed
 * or produced no view).  A worker reuses a result buffer only after every
 * view of it was released and dfs_batcher_destroy waits for all of them, so
 * release promptly, and before the same thread submits again: a worker that
 * finds its buffers still referenced adds more (up to 8), then waits.
 * Same results and return codes as the calls above. */
typedef struct dfs_view dfs_view;
int dfs_submit_upload_view(dfs_batcher* batcher, const uint8_t* file, uint64_t len, uint8_t* file_digest,
                           uint8_t* frag_digest, const char** b64, uint64_t* b64_off, dfs_view** view);
int dfs_submit_download_view(dfs_batcher* batcher, const char* b64, const dfs_span* frags, uint64_t file_len,
                             const uint8_t* expected_frag_digest, const uint8_t* expected_file_digest,
                             const uint8_t** out, dfs_view** view);
int dfs_view_release(dfs_view* view);

/* ---- multi-GPU placement over RCCL / xGMI (SN:143-145, 195-259, 422-446) -- */
/* One rank per GPU; node k (0-based) is hosted by rank k mod W (W = ranks).
 * Node k stores fragments {k, (k+1) mod N} (SN:143-145), so fragment f lives
 * on the ranks of node f and node f-1 (the download candidates nodeA / nodeB,
 * SN:427-428).
 *
 * Buffers (device memory of each rank's ctx):
 *   source "groups": a rank's Base64 in fragment-major order (an upload plan
 *     built with DFS_LAYOUT_FRAG_MAJOR): group f = fragment f of every file
 *     the rank uploaded, groups back to back, table[r*nfrag + f] bytes each.
 *   "held": for every fragment f the rank hosts (ascending f) the held group
 *     f = group f of rank 0, 1, ..., W-1 concatenated.  dfs_place_plan
 *     returns its layout (dst_off).
 * Comms: rank-per-process (dfs_comm_unique_id on one rank, shared out of
 * band, then dfs_comm_init_rank on every rank) or one process driving
 * several GPUs (dfs_comm_init_all, ncclCommInitAll).  The place / fetch
 * calls take an array of `ncomms` comms (1 in rank-per-process mode; all of
 * a process's comms otherwise, one source / destination pointer each) and
 * are asynchronous on each comm's ctx stream (dfs_set_stream).
 *
 * Host-staged transport: with DFS_COMM_TRANSPORT=host in the environment
 * dfs_comm_unique_id returns an id that makes dfs_comm_init_rank join a
 * communicator over host shared memory instead of RCCL (every rank a process
 * of one host, at most 16, one comm per process).  Ranks may then share a
 * GPU, which RCCL refuses, so every multi-rank call below runs on a box with
 * one GPU; the calls are synchronous and slow (device -> mailbox -> device in
 * 4 MiB chunks): for tests and rehearsals.
 *
 * Loopback: a comm made while DFS_COMM_LOOPBACK=1 is in the environment posts
 * a rank's local copies as ncclSend to itself paired with ncclRecv from itself
 * inside the phase's group instead of hipMemcpyAsync, so a one-rank run on one
 * GPU drives the same RCCL calls, group bracketing and stream ordering as a
 * many-rank one.  For tests; results are identical. */
#define DFS_COMM_ID_BYTES 128
typedef struct dfs_comm dfs_comm;
int dfs_comm_unique_id(uint8_t* id /* DFS_COMM_ID_BYTES */);
int dfs_comm_init_rank(dfs_ctx* ctx, const uint8_t* id, uint32_t nranks, uint32_t rank, dfs_comm** comm);
int dfs_comm_init_all(dfs_ctx* const* ctxs, uint32_t n, dfs_comm** comms);
int dfs_comm_destroy(dfs_comm* comm);
int dfs_comm_info(const dfs_comm* comm, uint32_t* nranks, uint32_t* rank);
/* Transfers the place / fetch / verify calls have issued on this comm since
 * it was made: counters[0] sends, [1] receives, [2] local copies. */
int dfs_comm_counters(const dfs_comm* comm, uint64_t* counters /* 3 */);
/* Text of the last RCCL failure on this thread (DFS_E_COMM). */
const char* dfs_comm_last_error(void);

/* table[r*nfrag + f] = bytes of rank r's group f, gathered from every rank's
 * grp_len (ncomms*nfrag entries, host); synchronous. */
int dfs_place_sizes(dfs_comm* const* comms, uint32_t ncomms, const uint64_t* grp_len, uint32_t nfrag,
                    uint64_t* table);

#define DFS_PLACE_RING 0   /* primary scatter + replica step g -> g-1 (north_star's ring) */
#define DFS_PLACE_STAR 1   /* the reference's fan-out: one all-to-all (SN:195-205)        */
#define DFS_PLACE_FETCH 2  /* degraded read: own groups back from live holders           */
#define DFS_XFER_SEND 0
#define DFS_XFER_RECV 1
#define DFS_XFER_COPY 2    /* local device-to-device copy */
/* One transfer of a rank's schedule.  Sends read src + src_off (or, with
 * from_dst, the rank's destination buffer: the ring's forward step);
 * receives and copies write dst + dst_off.  Transfers of one phase run as
 * one RCCL group; phases run in order. */
typedef struct dfs_xfer {
    uint32_t phase;
    uint32_t kind;
    int32_t peer;     /* rank, -1 for a copy */
    uint32_t frag;
    uint32_t from_dst;
    uint32_t reserved;
    uint64_t src_off;
    uint64_t dst_off;
    uint64_t len;
} dfs_xfer;
/* Pure host: the schedule rank `rank` of `nranks` runs for `mode`.
 *   ops / *nops   in: capacity (ops may be NULL: count only), out: count
 *   dst_off       nfrag+1: where group f lands in the destination
 *                 (UINT64_MAX: not on this rank); dst_off[nfrag] = bytes
 *   frag_status   FETCH: DFS_E_MISSING for a fragment no live holder has
 *                 ("Could not retrieve fragment i", SN:443-446), else 0
 * offline_mask: bit g = rank g is down (FETCH only; W <= 64). */
int dfs_place_plan(uint32_t nranks, uint32_t rank, uint32_t nfrag, const uint64_t* table, uint32_t mode,
                   uint64_t offline_mask, dfs_xfer* ops, uint32_t* nops, uint64_t* dst_off, int32_t* frag_status);
/* Upload placement (sendFragmentsToPeers, SN:195-224) of every rank's groups
 * into the hosts' held buffers: as a ring (primary scatter then the replica
 * step) or as the reference's star (one all-to-all over every xGMI link).
 * Both leave identical held buffers. */
int dfs_place_ring(dfs_comm* const* comms, uint32_t ncomms, uint32_t nfrag, const uint64_t* table,
                   const char* const* d_b64, char* const* d_held);
int dfs_place_star(dfs_comm* const* comms, uint32_t ncomms, uint32_t nfrag, const uint64_t* table,
                   const char* const* d_b64, char* const* d_held);
/* Degraded download fetch (SN:422-446): every rank not in offline_mask gets
 * its own groups back, in source layout, at d_out, each from the first live
 * holder in SN:427-428 order; frag_status (ncomms*nfrag, host) as
 * dfs_place_plan's.  Offline ranks neither serve nor request. */
int dfs_fetch_degraded(dfs_comm* const* comms, uint32_t ncomms, uint32_t nfrag, const uint64_t* table,
                       uint64_t offline_mask, const char* const* d_held, char* const* d_out, int32_t* frag_status);

/* The same runner as dfs_place_ring / dfs_place_star / dfs_fetch_degraded,
 * for all `nranks` ranks at once over HOST buffers and an in-process stand-in
 * for RCCL's group semantics (no GPU, no RCCL call): per phase every rank's
 * sends and receives are posted in the runner's order, then rank a's sends to
 * b are paired with b's receives from a in posting order.  Unequal counts or
 * sizes, a receive without a send, or a send that reads bytes written in the
 * same group return DFS_E_COMM (dfs_comm_last_error names the pair).  It is
 * how a schedule is checked before it meets hardware: src[r] / dst[r] are rank
 * r's source groups (FETCH: its held buffer) and destination buffer,
 * frag_status is nranks*nfrag (may be NULL). */
int dfs_place_simulate(uint32_t nranks, uint32_t nfrag, const uint64_t* table, uint32_t mode, uint64_t offline_mask,
                       const uint8_t* const* src, uint8_t* const* dst, int32_t* frag_status);

/* ---- replica receiver over placed groups (SN:226-259, 265-293) ------------- */
/* In the reference an upload succeeds only after every holder has
 * Base64-decoded and hashed the pair it received (handleInternalStoreFragments,
 * SN:281-282) and the uploader has compared those hashes with its own
 * (sendFragmentsToNode, SN:248-257); a mismatch is "Replication failed"
 * (SN:218-221).  After dfs_place_ring / dfs_place_star a rank holds, for every
 * fragment f it hosts, group f of every rank.  dfs_replica_verify does the
 * holders' half and the comparison for all of it:
 *   1. every rank's fragment digests (what its upload computed) go to the
 *      holders, fragment-major, 32 bytes per fragment, over the same comm and
 *      with the placement's own schedule (so entry k of the table a holder
 *      receives belongs to held fragment k);
 *   2. each holder Base64-decodes every held fragment into d_raw (the bytes it
 *      would store as <index>.frag, SN:284-285) and SHA-256s them;
 *   3. verdict[k] = 0, DFS_E_DECODE (the decoder's IllegalArgumentException) or
 *      DFS_E_FRAG_MISMATCH (digest or length differs from the uploader's);
 *   4. failed[r] = fragments of uploader r that failed on ANY holder (summed
 *      over the comm), so every uploader learns whether its upload replicated.
 * Held fragments are numbered in held-buffer order: hosted fragment f
 * ascending, then uploader rank, then that uploader's files in order
 * (dfs_held_frag). */
typedef struct dfs_held_frag {
    uint32_t rank;     /* uploader                                         */
    uint32_t file;     /* index among that uploader's files                */
    uint32_t frag;     /* fragment number                                  */
    uint32_t reserved;
    uint64_t b64_off;  /* its Base64 in the held buffer                    */
    uint64_t b64_len;
    uint64_t raw_off;  /* its decoded bytes in d_raw (16-byte aligned)     */
    uint64_t raw_len;
} dfs_held_frag;
/* Pure host: what rank `rank` of `nranks` holds after a placement of uploads
 * whose Base64 is fragment-major (DFS_LAYOUT_FRAG_MAJOR, optionally
 * DFS_LAYOUT_ALIGN128 in layout_flags).
 *   nfiles[r]   files uploaded by rank r
 *   file_len    every rank's file lengths, rank 0's first
 *   frags       out, capacity *nfrags entries (NULL: count only); *nfrags = count
 *   table       out (may be NULL): nranks*nfrag Base64 group bytes, what
 *               dfs_place_sizes gathers and dfs_place_* take
 *   held_bytes / raw_bytes  out (may be NULL): sizes of the held and raw buffers */
int dfs_replica_layout(uint32_t nranks, uint32_t rank, uint32_t nfrag, const uint32_t* nfiles,
                       const uint64_t* file_len, uint32_t layout_flags, dfs_held_frag* frags, uint64_t* nfrags,
                       uint64_t* table, uint64_t* held_bytes, uint64_t* raw_bytes);
typedef struct dfs_replica_plan dfs_replica_plan;
/* Descriptors of one batch shape, built once and kept in HBM.  Every rank
 * passes its own files' lengths; they are gathered over the comm (the call is
 * a collective and synchronises).  plans: ncomms out. */
int dfs_replica_plan_create(dfs_comm* const* comms, uint32_t ncomms, uint32_t nfrag, const uint32_t* nfiles,
                            const uint64_t* const* file_len, uint32_t layout_flags, dfs_replica_plan** plans);
/* nheld = held fragments; table (nranks*nfrag, may be NULL) as dfs_replica_layout's. */
int dfs_replica_plan_info(const dfs_replica_plan* plan, uint64_t* nheld, uint64_t* held_bytes, uint64_t* raw_bytes,
                          uint64_t* table);
/* 1 if dfs_replica_check runs this plan in one pass (every lane decodes,
 * stores and hashes its own fragment: the default for plans whose fragments
 * average 128 bytes or more; DFS_REPLICA_FUSED=0 / 1 in the environment when
 * the plan is made forces it off / on), 0 if it runs the decode kernel and
 * then the SHA-256 lanes.  Same results either way. */
int dfs_replica_plan_one_pass(const dfs_replica_plan* plan);
int dfs_replica_plan_frags(const dfs_replica_plan* plan, dfs_held_frag* frags);
/* Asynchronous on each comm's ctx stream; a plan runs one verify at a time.
 *   d_frag_digest  this rank's upload digests, [file][fragment] x 32 B
 *                  (dfs_upload_plan_run's frag_digest)
 *   d_held         the held buffer a placement filled
 *   d_raw          out: raw_bytes of decoded fragments
 *   d_verdict      out: nheld int32 (may be NULL)
 *   d_failed       out: nranks uint32, identical on every rank afterwards */
int dfs_replica_verify(dfs_comm* const* comms, uint32_t ncomms, dfs_replica_plan* const* plans,
                       const uint8_t* const* d_frag_digest, const char* const* d_held, uint8_t* const* d_raw,
                       int32_t* const* d_verdict, uint32_t* const* d_failed);
/* The three stages of dfs_replica_verify on their own, for a pipeline that
 * keeps the hashing off the communication stream (each asynchronous):
 *   dfs_replica_exchange  comm streams: the digest tables to the holders;
 *   dfs_replica_check     the stream of `ctx` (any ctx of the plan's device),
 *                         no communication: decode, hash, compare; d_failed
 *                         = this holder's own counts.  The caller orders it
 *                         after the placement and the exchange (events);
 *   dfs_replica_report    comm streams: d_failed summed over the holders
 *                         (order it after dfs_replica_check). */
int dfs_replica_exchange(dfs_comm* const* comms, uint32_t ncomms, dfs_replica_plan* const* plans,
                         const uint8_t* const* d_frag_digest);
int dfs_replica_check(dfs_ctx* ctx, dfs_replica_plan* plan, const char* d_held, uint8_t* d_raw, int32_t* d_verdict,
                      uint32_t* d_failed);
int dfs_replica_report(dfs_comm* const* comms, uint32_t ncomms, uint32_t* const* d_failed);
int dfs_replica_plan_destroy(dfs_replica_plan* plan);

/* ---- synthetic data (bench / tests) -------------------------------------- */
/* Byte o of file (first_file_index + f) is byte o mod 8 (little endian) of
 * splitmix64(seed ^ (file_index << 40 | o >> 3)); written at
 * d_dst + file_spans[f].off (device pointer). */
int dfs_synth_fill(dfs_ctx* ctx, uint8_t* d_dst, const dfs_span* file_spans, uint32_t nfiles,
                   uint64_t first_file_index, uint64_t seed);
/* As dfs_synth_fill, but the bytes written at d_dst + file_spans[f].off are
 * those of file offsets [file_off, file_off + len) (file_off % 8 == 0): one
 * chunk of files larger than HBM (BASELINE config 4). */
int dfs_synth_fill_at(dfs_ctx* ctx, uint8_t* d_dst, const dfs_span* file_spans, uint32_t nfiles,
                      uint64_t first_file_index, uint64_t seed, uint64_t file_off);

#ifdef __cplusplus
}
#endif
#endif /* DFS_GPU_H */
