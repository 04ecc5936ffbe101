// dfs_internal.h — device-side job descriptors and kernel launchers shared by
// the HIP kernels (sha256.hip, base64.hip, gather.hip) and the C ABI
// (dfs_gpu.cpp).  Not part of the public boundary (include/dfs_gpu.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>
#include <vector>

typedef struct dfs_ctx dfs_ctx;

namespace dfs {

// One SHA-256 lane: message bytes [off, off+len) of the batch buffer; the
// digest goes to out0 + 32*out (out < split) or out1 + 32*(out - split).
struct ShaDesc {
    uint64_t off;
    uint64_t len;    // bytes hashed by this lane in this launch
    uint64_t total;  // whole-message length (the padding's bit count); = len unless resumed
    uint32_t out;
    uint32_t flags;  // kShaResume / kShaPartial / kShaB64
    uint64_t b64;    // kShaB64: output offset of this fragment's Base64 (dword aligned)
};
// Streaming (SHA-256 update across launches, e.g. the 256 MiB skew config):
// kShaResume: start from the 8-word state in state[8*out] instead of H0;
// kShaPartial: len is a multiple of 64 and the message continues: store the
// running state to state[8*out] instead of padding and emitting a digest.
constexpr uint32_t kShaResume = 1u;
constexpr uint32_t kShaPartial = 2u;
// kShaB64: also write the RFC 4648 Base64 of the message at b64out + b64
// (fused upload encode; whole messages only, never with Resume/Partial).
constexpr uint32_t kShaB64 = 4u;
// kShaTwin (persistent kernel, plain instantiation only): the lane also
// hashes `count` whole "twin" messages that start on its own 64-byte block
// grid and lie inside its full blocks (a file's fragments that start at a
// multiple of 64 bytes, e.g. fragment 0, or every fragment of a 256 KiB / N=8
// file).  b64 = count << 32 | first: the twins are descs[n + first ...] (n =
// the launch's lane count), in block order.  A twin block is loaded and its
// message schedule expanded once for both states (sha256.hip compress2).
constexpr uint32_t kShaTwin = 8u;

// One byte-stream job for the tiled HBM-bound kernels (Base64 encode/decode,
// gather, synth).  Jobs are sorted by tile_start; a sentinel job with
// tile_start = total tiles ends the array.
struct StreamJob {
    uint64_t src_off;     // input byte offset (or absolute address for gather)
    uint64_t len;         // input length (bytes or chars)
    uint64_t dst_off;     // output byte offset
    uint64_t tile_start;  // first tile index of this job
    uint64_t expect;      // decode: expected decoded length + 1 (0 = any)
    uint32_t id;          // message index (status / out_len slot)
    uint32_t aux;         // kernel-specific (synth: unused)
};

constexpr int kShaBlock = 256;       // threads per SHA workgroup (4 waves)
constexpr size_t kShaQueueBytes = 4 * (64 + 8192);  // SHA queue words + per-SIMD tokens
// Launches of at most this many lanes (512 two-wave workgroups: all resident
// at once) run the latency kernel sha256_chain; larger ones the persistent
// throughput kernel sha256_lanes.
constexpr uint32_t kChainMaxLanes = 32768;
// Twin lanes (kShaTwin) are built only when the launch keeps at least one
// wave of lanes per SIMD (1,024 SIMDs x 64): each twin lane is a whole file's
// chain, so fewer lanes leave SIMDs idle and the plain split wins (e.g. a
// 32,768-file chunk of 256 KiB files: 17.6 ms with twins on half the SIMDs
// vs ~11.5 ms as 294,912 plain lanes).
constexpr uint32_t kTwinMinLanes = 65536;
constexpr int kStreamBlock = 256;    // threads per stream workgroup
constexpr int kEncPer = 4;           // encode: 12-byte groups per thread per tile
constexpr int kDecGpl = 8;           // decode: 4-unit groups per thread per tile
constexpr int kGatherPer = 4;        // gather: 16-byte chunks per thread per tile
// Base64 decode geometry of one message of L chars decoding to dst (shared
// by the host's tile count and b64_decode_kernel).  q = L/4 full units, r =
// L%4; the final unit (padded, or the r trailing chars) is decoded by the
// tail step, the body_units before it by tiles of gpl x 256 4-unit
// groups starting at unit u_first = h/3, where h = bytes up to the first
// 16-byte aligned output address.  Main output = 16-byte chunks
// [h + 16m, h + 16m + 16), m < nchunks, cut from the decoded stream of the
// ng whole groups at byte offset e = h % 3.
struct DecGeom {
    uint64_t body_units;
    uint64_t nb;       // body bytes
    uint32_t h;        // head bytes
    uint32_t u_first;  // first unit of group 0
    uint32_t e;        // h % 3
    uint64_t ng;       // whole 4-unit groups decoded by the tiles
    uint64_t nchunks;  // 16-byte output chunks written by the tiles
};
__host__ __device__ inline DecGeom dec_geom(uint64_t L, uintptr_t dst) {
    DecGeom g;
    const uint64_t q = L >> 2;
    const uint32_t r = static_cast<uint32_t>(L & 3u);
    g.body_units = (r == 0) ? (q ? q - 1 : 0) : q;
    g.nb = 3 * g.body_units;
    g.h = static_cast<uint32_t>((16u - (dst & 15u)) & 15u);
    g.u_first = g.h / 3u;
    g.e = g.h % 3u;
    g.ng = g.body_units > g.u_first ? (g.body_units - g.u_first) / 4 : 0;
    g.nchunks = 12 * g.ng > g.e ? (12 * g.ng - g.e) / 16 : 0;
    return g;
}

// One storeFragments request body (buildFragmentsJson, SN:629-642) carrying
// fragments a and b (one digit each) of file `file`: framing bytes around
// two Base64 payloads of len_a / len_b chars, at out + dst.
struct StoreBody {
    uint64_t dst;
    uint64_t len_a;
    uint64_t len_b;
    uint32_t file;  // index into the fileId digests
    uint16_t a, b;
};
constexpr uint32_t kBodyDataA = 111;     // first payload offset: {"fileId":"<64>","fragments":[{"index":"a","data":"
constexpr uint32_t kBodyMidBytes = 24;   // "},{"index":"b","data":"
constexpr uint32_t kBodyFrameBytes = 139;  // + the 4-byte "}]} suffix
// Bodies start 1 byte past a 16-byte boundary so both payloads (at +111 and
// +135 + len_a, len_a a multiple of 4) are dword aligned for the encoder.
constexpr uint32_t kBodyStartPhase = 1;

// Receiver-side parse of one storeFragments body (offsets relative to the
// body; status 0 = buildFragmentsJson form, 1 = any other form).
struct BodyParse {
    uint64_t off_a, len_a, off_b, len_b;
    int32_t status;
    uint16_t a, b;
};

// Launchers (return hipError_t of the launch).
// Multi-message SHA-256: up to kChainMaxLanes lanes (without fused Base64)
// the owner/helper latency kernel, else the persistent throughput kernel.
// `queue` is kShaQueueBytes of device memory, zeroed by the launcher on `s`
// before a persistent launch; its grid holds waves_per_simd waves on each of
// the 1024 SIMDs (fewer for small batches).
// Decode-ahead download (dfs_download_batch, overlap mode): the SHA kernel
// runs beside the decode and reads fragment group g (fragment g of every
// file) only after done[g] reached `target` (the decode grid size: every
// decode workgroup adds 1 after publishing its share of g with an agent-scope
// release; sha256.hip acquires).  Groups below `first` were decoded by an
// earlier launch on the stream the SHA launch waits for.  Fragment lanes
// (digest slot out < nf) read group out % nfrag; fileId lanes (out >= nf,
// whole files split SN:138-157 into nfrag fragments) wait at each fragment's
// first block.  A wait is bounded: past `ticks` the lane goes on, sets
// queue[2] (after which no lane of the launch waits again) and the host
// re-runs the SHA launch after the decode.
struct ShaWait {
    const uint32_t* done;
    uint32_t target, first, nfrag, nf;
    uint64_t ticks;  // bound of one wait in s_memrealtime ticks (100 MHz)
};
constexpr uint64_t kShaWaitTicks = 200000000ull;  // 2 s
constexpr uint32_t kShaWaitSlot = 8;  // done[g] = queue[kShaWaitSlot + g] (kShaQueueBytes)
constexpr uint32_t kShaWaitMaxGroups = 48;
// VGPRs per lane of the kernels that run in "ahead" mode beside the waiting
// SHA kernel (hipFuncGetAttributes): the host sizes the grids so that both
// are resident at once (the SHA waves wait on every stream workgroup).
int sha_wait_vgprs();
int dec_ahead_vgprs();
int gather_ahead_vgprs();
// A stream kernel (decode, gather) in ahead mode: groups in order, every
// workgroup takes its share of group g's tiles, publishes it (agent-scope
// release) and adds 1 to gdone[g]; `grid` workgroups, all of them in every
// group.
struct StreamAhead {
    const uint64_t* gtile;  // group g = tiles [gtile[g], gtile[g + 1])
    uint32_t ngroups, grid;
    uint32_t* gdone;
};

// Lanes flagged kShaTwin need the persistent plain kernel: the host builds
// twins only for launches of more than kChainMaxLanes lanes without b64
// (add_lane_with_twins in dfs_gpu.cpp); the descriptor array then holds the
// n lanes followed by their twins.
hipError_t launch_sha256(const uint8_t* base, const ShaDesc* descs, uint32_t n, uint32_t split,
                         uint32_t prio_lanes, uint8_t* out0, uint8_t* out1, uint32_t* queue,
                         int waves_per_simd, hipStream_t s, uint32_t* state = nullptr, char* b64 = nullptr,
                         const ShaWait* wait = nullptr);
// Base64 decode + SHA-256 in one pass, one message per lane (held replicas:
// dfs_replica_check; received request bodies: dfs_receive_fragments_batch).
// Lane i decodes the chars at in + src (dword aligned), writes the decoded
// bytes at raw + dst (16-byte aligned) and their SHA-256 at digests + 32 * out.
// out_len == nullptr: the decoded length n is known and the chars are the
// encoder's 4 * ceil(n / 3) (len is ignored); status[out] = bit 0 (a char
// outside the alphabet or a bad final unit) | bit 1 (the decoded length is not
// n), as the decode kernel reports them.  out_len != nullptr: len chars of
// unknown decoded length (n is ignored); status[out] = 0 / 1, out_len[out] =
// decoded bytes (0 on error), a failed message's digest is not written.
// Lanes sorted longest first keep the waves uniform.  `queue`: 64 words.
struct DecLane {
    uint64_t src, dst, n, len;
    uint32_t out, pad;
};
hipError_t launch_sha256_b64dec(const char* in, const DecLane* lanes, uint32_t n, uint8_t* raw, uint8_t* digests,
                                int32_t* status, uint32_t* queue, int waves_per_simd, hipStream_t s,
                                uint64_t* out_len = nullptr);
// Allocation-free variant (dfs_sha256_batch_static): descriptors and queue
// words live in a file-scope device array of sha256.hip, whose address on
// `device` static_scratch_init resolves once (that device current; called by
// dfs_open).  d_msgs = n {off, len} pairs in device memory; status (device,
// may be null) gets 0 or -1 (message of 2^37 bytes or more: hashed as empty).
constexpr uint32_t kStaticMaxMsgs = 65536;
hipError_t static_scratch_init(int device);
hipError_t launch_sha256_static(int device, const uint8_t* base, const uint64_t* d_msgs, uint32_t n, uint8_t* out,
                                int32_t* status, int waves_per_simd, hipStream_t s);
// Tiles hold kEncPer*256 12-byte groups (the job table's tile_start must be
// built with that tile size); prio = s_setprio of the encode waves.
hipError_t launch_b64_encode(const uint8_t* base, const StreamJob* jobs, uint32_t njobs, uint64_t ntiles,
                             char* out, uint32_t wgs_per_cu, hipStream_t s, uint32_t prio = 3);
// Decode: chars of job j at in + src_off decode to out + dst_off.
// status[id] |= 1 on an IllegalArgumentException case; out_len[id] = bytes.
// If job.expect != 0 it is the expected decoded length + 1 (download path):
// a different length sets status bit 2.  Tiles hold kDecGpl*256 4-unit groups.
// prio != 0: the waves run at s_setprio 3 (beside the SHA kernel); the grid
// holds at most wgs_per_cu persistent workgroups per CU.
// ahead: decode-ahead mode (group order, per-group completion counters,
// grid = ahead->grid workgroups); the tile count is then ahead->gtile's.
hipError_t launch_b64_decode(const char* in, const StreamJob* jobs, uint32_t njobs, uint64_t ntiles,
                             uint8_t* out, int32_t* status, uint64_t* out_len, hipStream_t s, uint32_t prio = 0,
                             uint32_t wgs_per_cu = 8, const StreamAhead* ahead = nullptr);
// Framing bytes of n storeFragments bodies (digests: raw 32 B per file).
hipError_t launch_store_body_frame(const StoreBody* bodies, uint32_t n, const uint8_t* digests, char* out,
                                   hipStream_t s);
// Parse n bodies (spans = n x {off, len} into `in`, device memory); the
// 64 fileId chars of body k go to file_ids + 64k.
hipError_t launch_store_body_parse(const char* in, const uint64_t* spans, uint32_t n, BodyParse* out,
                                   char* file_ids, hipStream_t s);
// Gather: job.src_off is an absolute device address of the fragment; tiles
// of kGatherPer x 256 16-byte chunks.
// ahead: ahead mode (as launch_b64_decode).
hipError_t launch_gather(const StreamJob* jobs, uint32_t njobs, uint64_t ntiles, uint8_t* out, hipStream_t s,
                         const StreamAhead* ahead = nullptr);
// Download verdict per file on the device (expected digests in device
// memory): verdict[f] = 0 good, 1 decode error, 2 fragment digest, 3 fileId.
hipError_t launch_download_verdict(const int32_t* dec_status, const uint8_t* frag_dig, const uint8_t* file_dig,
                                   const uint8_t* exp_frag, const uint8_t* exp_file, uint32_t nfiles, uint32_t nfrag,
                                   int32_t* verdict, hipStream_t s);
hipError_t launch_synth(uint8_t* dst, const StreamJob* jobs, uint32_t njobs, uint64_t ntiles, uint64_t seed,
                        hipStream_t s, uint64_t file_off);

// Host-side descriptor helpers shared by the entry points (dfs_gpu.cpp):
// longest-first lane order (returns the lanes of the long items, a multiple
// of 64), tile_start prefix + sentinel of a job table (returns the tiles),
// decode work items of one message.
uint32_t sort_sha_lanes(std::vector<ShaDesc>& d);
uint64_t finish_stream_jobs(std::vector<StreamJob>& jobs, const std::vector<uint64_t>& items, uint64_t per_tile);
uint64_t decode_items(uint64_t L, uintptr_t dst);

// Replica receiver (replica.cpp).  fill: n words = v.  transpose: digests
// [file][frag] -> [frag][file], 32 bytes each.  verdict: held fragment k gets
// 0 / code_decode (status bit 0) / code_mismatch (status bit 1: wrong length,
// or got != expected); failed[piece_rank[p]] counts the failures of piece p =
// held fragments [piece_start[p], piece_start[p + 1]).
hipError_t launch_fill_u32(uint32_t* p, uint64_t n, uint32_t v, hipStream_t s);
hipError_t launch_digest_transpose(const uint8_t* in, uint8_t* out, uint32_t nfiles, uint32_t nfrag, hipStream_t s);
hipError_t launch_replica_verdict(const int32_t* status, const uint8_t* got, const uint8_t* expected, uint64_t n,
                                  const uint64_t* piece_start, const uint32_t* piece_rank, uint32_t npieces,
                                  int32_t code_decode, int32_t code_mismatch, int32_t* verdict, uint32_t* failed,
                                  hipStream_t s);

// ctx internals for the on-disk fragment store (fragstore.cpp).  The store's
// pinned staging ring lives in the ctx and is freed by dfs_close.
struct StoreStaging;
void store_staging_free(StoreStaging* s);
hipStream_t ctx_stream(dfs_ctx* c);
// Wait for an event / for everything queued on a ctx stream without spinning
// a host core (dfs_gpu.cpp).
hipError_t quiet_wait(hipEvent_t ev);
hipError_t quiet_sync(dfs_ctx* c, hipStream_t s);
// Many copies between device memory and device-mapped pinned host memory
// (dfs_host_alloc) as ONE gather_kernel launch on the ctx stream: addresses
// are absolute and device-visible.  Replaces one DMA per request in the
// batcher (one 1 MiB DMA each: 36-40 GB/s; one launch: PCIe rate).
struct CopySpan {
    uint64_t src, dst, len;
};
int copy_spans(dfs_ctx* c, const CopySpan* spans, size_t n);
int ctx_device(dfs_ctx* c);
hipError_t ctx_aux_stream(dfs_ctx* c, hipStream_t* aux);  // the ctx's second stream, created on first use
std::mutex& ctx_store_mutex(dfs_ctx* c);  // guards the staging ring only
StoreStaging*& ctx_store(dfs_ctx* c);

}  // namespace dfs
