/*
 * cfsec.h -- C ABI of the MI355X-native erasure-coding engine for CubeFS blobstore.
 *
 * This is the drop-in boundary.  Two layers are exported, each replacing one Go
 * interface of the reference (paths relative to the CubeFS tree):
 *
 *  1. cfsec_rs_*  replaces the reedsolomon.Encoder engine that blobstore/common/ec
 *     constructs at blobstore/common/ec/encoder.go:86 (global) and :95 (local),
 *     i.e. vendor/github.com/klauspost/reedsolomon/reedsolomon.go:25-131 with the
 *     default (Vandermonde) matrix of reedsolomon.go:220-244.  Only the six methods
 *     CubeFS uses are exported (Encode, Verify, Reconstruct, ReconstructData, Split,
 *     Join), plus GPU batch entry points.
 *
 *  2. cfsec_ec_*  replaces ec.Encoder (blobstore/common/ec/encoder.go:41-62) as
 *     returned by ec.NewEncoder (encoder.go:78-112), for both the plain RS encoder
 *     (encoder.go:71-180) and the LRC encoder (lrcencoder.go:28-247).
 *
 * Shard vectors.  A Go [][]byte is passed as an array of cfsec_shard {data,len,cap}.
 * len == 0 marks a missing shard (KRS/reedsolomon.go:1416-1428).  Reconstruct
 * writes into a missing shard's buffer and sets its len to the shard size; the
 * caller must have given it cap >= shard size (the cgo shim does what
 * KRS/reedsolomon.go:1514-1518 does: reuse cap, else allocate 64-B aligned).
 *
 * Memory.  mem = CFSEC_MEM_HOST: plain host memory; the engine stages through HBM
 * and returns after the results are back in host memory.  mem = CFSEC_MEM_DEVICE:
 * pointers are HBM device pointers on the engine's device; the call is enqueued on
 * `stream` (hipStream_t) and returns after it completes.  stream = NULL: the call runs on an
 * engine-owned non-blocking stream that first waits for an event recorded on the legacy default
 * stream, i.e. it is ordered after everything already queued on the default stream and on every
 * blocking stream of the device, but not after work on other non-blocking streams (PyTorch's
 * side streams are non-blocking: pass the producer's stream explicitly).
 * *_batch entry points never synchronise: they enqueue on `stream`.
 *
 * Threading.  Every handle is safe for concurrent calls from many threads (the
 * reference shares one encoder across goroutines, encoder.go:90,115-116).
 * The library never retains a caller pointer after a call returns (cgo rule).
 *
 * Errors.  Return codes map 1:1 onto the Go sentinel errors named in each value.
 */
#ifndef CFSEC_H_
#define CFSEC_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  CFSEC_OK = 0,
  CFSEC_ERR_TOO_FEW_SHARDS = 1,        /* reedsolomon.ErrTooFewShards   KRS/reedsolomon.go:601  */
  CFSEC_ERR_SHARD_NO_DATA = 2,         /* reedsolomon.ErrShardNoData    KRS/reedsolomon.go:1305 */
  CFSEC_ERR_SHARD_SIZE = 3,            /* reedsolomon.ErrShardSize      KRS/reedsolomon.go:1309 */
  CFSEC_ERR_INV_SHARD_NUM = 4,         /* reedsolomon.ErrInvShardNum    KRS/reedsolomon.go:204  */
  CFSEC_ERR_MAX_SHARD_NUM = 5,         /* reedsolomon.ErrMaxShardNum    KRS/reedsolomon.go:209  */
  CFSEC_ERR_SHORT_DATA = 6,            /* reedsolomon.ErrShortData      KRS/reedsolomon.go:1556 (also ec.ErrShortData) */
  CFSEC_ERR_RECONSTRUCT_REQUIRED = 7,  /* reedsolomon.ErrReconstructRequired KRS/reedsolomon.go:1636 */
  CFSEC_ERR_SINGULAR = 8,              /* errSingular                   KRS/matrix.go:185       */
  CFSEC_ERR_INVALID_CODE_MODE = 9,     /* ec.ErrInvalidCodeMode         common/ec/encoder.go:35 */
  CFSEC_ERR_VERIFY = 10,               /* ec.ErrVerify                  common/ec/encoder.go:36 */
  CFSEC_ERR_INVALID_SHARDS = 11,       /* ec.ErrInvalidShards           common/ec/encoder.go:37 */
  CFSEC_ERR_INVALID_ARG = 12,          /* boundary misuse (NULL handle, cap < shard size, ...) */
  CFSEC_ERR_DEVICE = 13,               /* HIP runtime failure; see cfsec_last_error()         */
  CFSEC_ERR_NOT_SUPPORTED = 14,        /* reedsolomon.ErrNotSupported   KRS/reedsolomon.go:212  */
  CFSEC_ERR_INVALID_BLOCK = 15,        /* crc32block.ErrInvalidBlock    common/crc32block/util.go:29 */
  CFSEC_ERR_MISMATCHED_CRC = 16        /* crc32block.ErrMismatchedCrc   common/crc32block/util.go:30 */
} cfsec_status;

typedef enum { CFSEC_MEM_HOST = 0, CFSEC_MEM_DEVICE = 1 } cfsec_mem;

/* One Go []byte: pointer, length, capacity. */
typedef struct {
  uint8_t* data;
  size_t len;
  size_t cap;
} cfsec_shard;

/* codemode.Tactic (blobstore/common/codemode/codemode.go:129-163). */
typedef struct {
  int n, m, l, az_count, put_quorum, get_quorum, min_shard_size;
} cfsec_tactic;

typedef struct cfsec_rs cfsec_rs;
typedef struct cfsec_ec cfsec_ec;

/* ---------------- library ---------------- */
/* "cfsec MAJOR.MINOR.PATCH (gfx950)".  ABI history: 0.2.0 inserted src_len into
 * cfsec_crc32block_decode / cfsec_crc32block_decode_batch (callers built against 0.1.0 must be
 * rebuilt); 0.3.0 and 0.4.0 add entry points only. */
const char* cfsec_version(void);
/* Message for the last CFSEC_ERR_DEVICE on this thread ("" if none). */
const char* cfsec_last_error(void);
/* Name of a status code, e.g. "ErrTooFewShards". */
const char* cfsec_status_name(int status);
/* Number of visible HIP devices (0 if none; never an error). */
int cfsec_device_count(void);
/* How synchronous calls wait for their stream (no reference counterpart: a tuning knob):
 * 1 = poll a pinned marker word the stream writes after the call's work (default), 0 =
 * hipStreamSynchronize.  Process-wide; returns the previous mode.  Env: CFSEC_SYNC_POLL=0. */
int cfsec_set_sync_poll(int on);

/* ---------------- reedsolomon.Encoder seam ---------------- */
/* reedsolomon.New(dataShards, parityShards) -- KRS/reedsolomon.go:413-581.  The engine binds
 * to `device` (-1 = the calling thread's current HIP device). */
int cfsec_rs_new(int data_shards, int parity_shards, int device, cfsec_rs** out);
void cfsec_rs_free(cfsec_rs* h);
int cfsec_rs_data_shards(const cfsec_rs* h);
int cfsec_rs_parity_shards(const cfsec_rs* h);
/* Copy the (data+parity) x data encoding matrix (row-major) into out. */
int cfsec_rs_matrix(const cfsec_rs* h, uint8_t* out, size_t out_len);

/* Encode -- KRS/reedsolomon.go:609-625 */
int cfsec_rs_encode(cfsec_rs* h, cfsec_shard* shards, int n, int mem, void* stream);
/* Encode followed by crc32.ChecksumIEEE of every shard (access/stream_put.go:125-143 then
 * :249-253) in one fused pass: crcs is a host array of n words.  Host memory from
 * cfsec_host_alloc is coded in place over PCIe; other host memory is staged through HBM. */
int cfsec_rs_encode_crc(cfsec_rs* h, cfsec_shard* shards, int n, int mem, void* stream, uint32_t* crcs);
/* Verify -- KRS/reedsolomon.go:770-784; *ok = 1 when every parity shard matches. */
int cfsec_rs_verify(cfsec_rs* h, cfsec_shard* shards, int n, int mem, void* stream, int* ok);
/* Reconstruct / ReconstructData -- KRS/reedsolomon.go:1377-1552 */
int cfsec_rs_reconstruct(cfsec_rs* h, cfsec_shard* shards, int n, int mem, void* stream);
int cfsec_rs_reconstruct_data(cfsec_rs* h, cfsec_shard* shards, int n, int mem, void* stream);
/* Split -- KRS/reedsolomon.go:1574-1632 (host memory).  data has len/cap; the engine fills
 * out[0..total) with views into data and, when cap is short, into pad (caller-owned, at least
 * *pad_needed bytes; call once with pad == NULL to learn pad_needed), laid out as the reference's
 * AllocAligned (KRS/unsafe.go:17-41): from the first 64-byte aligned address of pad, shard j at
 * j * roundup(per, 64), len per, cap roundup(per, 64). */
int cfsec_rs_split(cfsec_rs* h, uint8_t* data, size_t len, size_t cap, cfsec_shard* out,
                   uint8_t* pad, size_t pad_len, size_t* pad_needed);
/* Join -- KRS/reedsolomon.go:1646-1684 (host memory): copies out_size bytes into dst. */
int cfsec_rs_join(cfsec_rs* h, uint8_t* dst, size_t dst_len, const cfsec_shard* shards, int n,
                  size_t out_size);

/* GPU batch entry points (device memory, asynchronous on `stream`).
 * ptrs holds nstripes * (data+parity) device pointers, stripe-major; every shard is
 * shard_size bytes. */
int cfsec_rs_encode_batch(cfsec_rs* h, uint8_t* const* ptrs, size_t shard_size, int nstripes,
                          void* stream);
/* flags: device array of nstripes uint32; flags[s] is OR-ed with 1 when stripe s mismatches
 * (caller zeroes it). */
int cfsec_rs_verify_batch(cfsec_rs* h, uint8_t* const* ptrs, size_t shard_size, int nstripes,
                          uint32_t* flags, void* stream);
/* Rebuild the shards listed in erased[] (same pattern for every stripe) from the first
 * data_shards surviving shards, in one fused pass (missing data rows = inv(sub), missing
 * parity rows = parity * inv(sub)).  data_only = 1 rebuilds only erased data shards. */
int cfsec_rs_reconstruct_batch(cfsec_rs* h, uint8_t* const* ptrs, size_t shard_size, int nstripes,
                               const int* erased, int nerased, int data_only, void* stream);

/* Encode / reconstruct with the shard checksums CubeFS computes right after coding
 * (crc32.ChecksumIEEE, access/stream_put.go:249-253; blobnode/work_shard_recover.go:335-342),
 * fused into the coding kernel where the shape allows (k in {6,8,12,16,18}, <= 6 outputs): no
 * extra pass over the shards.  crcs: device array of nstripes * (data+parity) uint32, indexed
 * [stripe][shard].  Encode fills every word; reconstruct fills the words of the shards it rebuilt
 * and zeroes the rest.  Asynchronous on `stream`. */
int cfsec_rs_encode_crc_batch(cfsec_rs* h, uint8_t* const* ptrs, size_t shard_size, int nstripes,
                              uint32_t* crcs, void* stream);
int cfsec_rs_reconstruct_crc_batch(cfsec_rs* h, uint8_t* const* ptrs, size_t shard_size, int nstripes,
                                   const int* erased, int nerased, int data_only, uint32_t* crcs,
                                   void* stream);

/* ---------------- stripe batches over one or more GPUs ----------------
 * The reference codes one stripe per call: access encodes blob by blob (access/stream_put.go:104-143,
 * up to 4 blobs in flight per request) and blobnode repairs a tasklet bid by bid, each bid with
 * its own shard size and missing set, Reconstruct then Verify (blobnode/work_shard_recover.go:
 * 708-771).  These entry points take a whole batch: `shards` holds nstripes consecutive shard
 * vectors of (data+parity) entries each (stripe-major), every stripe with its own shard size and
 * its own missing shards (len == 0); stripes with one erasure pattern share a decode plan and run
 * in the same launches.  mem = CFSEC_MEM_HOST: the stripes are split into contiguous runs over the
 * handle's devices (balanced by bytes), page-locked buffers (cfsec_host_alloc) are coded in place,
 * pageable ones through double-buffered staging, one host thread and stream pair per device.
 * mem = CFSEC_MEM_DEVICE: each stripe runs on the device its memory lives on (one of the handle's
 * devices), after the work queued on that device's legacy default stream; with a one-device handle
 * every stripe must live on that device (only the first stripe's memory is queried -- one pointer
 * query costs ~1 us -- so a stripe on another GPU is the caller's error, not detected).  Synchronous: returns
 * when every result is in place.  status[s] (nstripes words) receives stripe s's result as the
 * single-stripe call would return it; the return value reports failures of the call itself
 * (CFSEC_ERR_DEVICE, CFSEC_ERR_INVALID_ARG). */
/* Devices batches are spread over (default: the handle's own device).  Call before sharing the
 * handle between threads. */
int cfsec_rs_set_devices(cfsec_rs* h, const int* devices, int ndev);
/* The split a host-memory batch uses: stripe i (moving bytes[i] bytes) runs on device index dev[i]
 * of the handle's list -- contiguous runs, balanced by bytes.  Host only (no device needed); lets a
 * caller place its staging per device ahead of the call. */
int cfsec_batch_partition(const uint64_t* bytes, int n, int ndev, int* dev);
/* Encode each stripe (KRS/reedsolomon.go:609-625). */
int cfsec_rs_encode_stripes(cfsec_rs* h, cfsec_shard* shards, int nstripes, int mem, int* status);
/* Verify each stripe (KRS/reedsolomon.go:770-784): status CFSEC_OK when it holds, CFSEC_ERR_VERIFY
 * when Verify would return false (no error), another code for Verify's errors. */
int cfsec_rs_verify_stripes(cfsec_rs* h, cfsec_shard* shards, int nstripes, int mem, int* status);
/* Reconstruct each stripe (KRS/reedsolomon.go:1377-1552; missing shards need cap >= shard size and
 * get len = shard size) and, with verify != 0, Verify it afterwards, in one fused pass per stripe:
 * the kernel reads the first data_shards present shards and every other present parity shard once,
 * writes the missing ones and compares the rest (status CFSEC_ERR_VERIFY when Verify would return
 * false).  Bit-exact with the two calls on any input, consistent or not. */
int cfsec_rs_reconstruct_stripes(cfsec_rs* h, cfsec_shard* shards, int nstripes, int verify, int mem,
                                 int* status);

/* ---------------- ec.Encoder ---------------- */
/* Code-mode table (codemode.go:26-79): fill *t for a CodeMode value; CFSEC_ERR_INVALID_CODE_MODE
 * when unknown. */
int cfsec_codemode_tactic(int codemode, cfsec_tactic* t);
/* ec.NewEncoder(Config{CodeMode, EnableVerify, Concurrency}) -- encoder.go:78-112 */
int cfsec_ec_new(const cfsec_tactic* tactic, int enable_verify, int concurrency, int device,
                 cfsec_ec** out);
void cfsec_ec_free(cfsec_ec* h);
int cfsec_ec_encode(cfsec_ec* h, cfsec_shard* shards, int n, int mem, void* stream);
int cfsec_ec_reconstruct(cfsec_ec* h, cfsec_shard* shards, int n, const int* bad_idx, int nbad,
                         int mem, void* stream);
int cfsec_ec_reconstruct_data(cfsec_ec* h, cfsec_shard* shards, int n, const int* bad_idx,
                              int nbad, int mem, void* stream);
int cfsec_ec_verify(cfsec_ec* h, cfsec_shard* shards, int n, int mem, void* stream, int* ok);
/* blobnode's repair loop over a tasklet (blobnode/work_shard_recover.go:708-771) in one call: bid b
 * is the n shards at shards[b*n ..] and its bad indices bad_idx[bad_off[b] .. bad_off[b+1]) (global
 * stripe indices, or local ones for a local stripe: n = its size); per bid exactly
 * encoder.Reconstruct(shards_b, bad_b) then, with verify != 0, encoder.Verify(shards_b).  status[b]:
 * the Reconstruct error, CFSEC_ERR_VERIFY when Verify returns false, or CFSEC_OK.  RS modes run one
 * fused Reconstruct+Verify pass; LRC modes (lrcencoder.go:133-186, 89-131) one pass too for a bid
 * with no bad local shard (its local parities compared in the global pass as rows over the data),
 * else the global pass then every AZ's local pass.  Memory and devices as for cfsec_rs_*_stripes. */
int cfsec_ec_reconstruct_batch(cfsec_ec* h, cfsec_shard* shards, int n, int nbids, const int* bad_idx,
                               const int* bad_off, int verify, int mem, int* status);
int cfsec_ec_set_devices(cfsec_ec* h, const int* devices, int ndev);
/* access's Put over a batch of blobs (stream_put.go:104-143 encodes them one by one): for stripe s
 * (the n shards at shards[s*n ..]) exactly encoder.Encode(shards_s), EnableVerify included; LRC
 * modes as one fused (M+L) x N pass (lrcencoder.go:35-82).  status[s]: Encode's result (CFSEC_ERR_VERIFY
 * when the enabled Verify fails).  Memory and devices as for cfsec_rs_*_stripes. */
int cfsec_ec_encode_batch(cfsec_ec* h, cfsec_shard* shards, int n, int nstripes, int mem, int* status);
/* The two batch calls above returning the shard checksums CubeFS takes right after coding
 * (crc32.ChecksumIEEE): crcs is a host array of nstripes * n (nbids * n) words, indexed
 * [item][shard].  Encode: every shard of the stripe after the Encode (access/stream_put.go:249-253).
 * Reconstruct: the shards the call rebuilt -- global or local, data or parity -- (blobnode's
 * ShardCrc32 of each repaired shard, blobnode/work_shard_recover.go:335-342), 0 for the others.
 * Items whose status is not CFSEC_OK get all-zero words.  Computed on the GPU from the rows the
 * product wrote (device or staged copies), before they leave HBM.  CFSEC_ERR_NOT_SUPPORTED for
 * shapes with more than 32 inputs and Verify. */
int cfsec_ec_encode_batch_crc(cfsec_ec* h, cfsec_shard* shards, int n, int nstripes, int mem, int* status,
                              uint32_t* crcs);
int cfsec_ec_reconstruct_batch_crc(cfsec_ec* h, cfsec_shard* shards, int n, int nbids, const int* bad_idx,
                                   const int* bad_off, int verify, int mem, int* status, uint32_t* crcs);
/* Asynchronous forms of the two batch calls above, for device memory on the handle's (first) device:
 * the call plans the batch, enqueues its kernels on `stream` (hipStream_t; NULL = the legacy default
 * stream) and returns without waiting, so a caller overlaps the next tasklet's planning with this
 * one's kernels.  status[b] (host) receives at return what the synchronous call would report
 * except a false Verify: the shard checks and planning errors (the buffers of a failed bid are not
 * touched).  flags (device, one uint32 per bid, zeroed by the caller; may be NULL when no Verify is
 * asked for): once the stream has passed the call, flags[b] != 0 where Verify is false
 * (CFSEC_ERR_VERIFY of the synchronous call).  Missing shards' lengths are set at return, as in the
 * synchronous call; the bytes are there when the stream gets there.  The library keeps no caller
 * pointer after the call returns (the shard pointers are copied into the kernel arguments).  Shapes
 * the kernels cannot compare in one pass: more than 32 inputs with Verify (no code mode has them)
 * return CFSEC_ERR_NOT_SUPPORTED -- use the synchronous call; an LRC stripe whose local shard has
 * another length runs synchronously on `stream` and reports ErrVerify in status[b].
 * crcs (device, nbids * n / nstripes * n words, may be NULL): the checksums of the _crc forms,
 * written on the stream (zeroed by the call first); a flagged or failed item's words are
 * meaningless. */
int cfsec_ec_reconstruct_batch_async(cfsec_ec* h, cfsec_shard* shards, int n, int nbids, const int* bad_idx,
                                     const int* bad_off, int verify, int* status, uint32_t* flags, uint32_t* crcs,
                                     void* stream);
int cfsec_ec_encode_batch_async(cfsec_ec* h, cfsec_shard* shards, int n, int nstripes, int* status, uint32_t* flags,
                                uint32_t* crcs, void* stream);
/* Repair over survivors held elsewhere (the multi-GPU repair of chubaofs_amd/repair.py ships only
 * the shards a decode reads): with the shards in bad_idx[0..nbad) lost (global or LRC local
 * indices), in_idx[0..N) = the first N present global shards in index order -- the ones
 * Reconstruct decodes from (KRS/reedsolomon.go:1453-1465) -- and rows[w*N .. w*N+N) = shard
 * want[w] (a data, global parity or local parity index) as a GF(2^8) row over them (the local
 * parity through lrcencoder.go's local engine over the AZ's shards).  No reference counterpart:
 * the reference repairs one bid at a time on one host. */
int cfsec_ec_repair_rows(cfsec_ec* h, const int* bad_idx, int nbad, const int* want, int nwant,
                         int* in_idx, uint8_t* rows);
/* outputs = coef (rows x N) x inputs over device memory, asynchronously on `stream` (NULL: the
 * legacy default stream): stripe s has N input pointers then `rows` output pointers at
 * ptrs[s*(N+rows) ..], shard_size bytes each (the product kernel of cfsec_rs_encode_batch with
 * caller rows, e.g. cfsec_ec_repair_rows'). */
int cfsec_ec_matvec_batch(cfsec_ec* h, const uint8_t* coef, int rows, uint8_t* const* ptrs, size_t shard_size,
                          int nstripes, void* stream);
/* GetShardsInIdc index map (encoder.go:169-176 / lrcencoder.go:236-243): writes the global
 * shard indices of AZ idx into out (capacity out_cap) and their count into *count. */
int cfsec_ec_shards_in_idc(const cfsec_ec* h, int idx, int* out, int out_cap, int* count);

/* ---------------- contiguous stripes (ec.Buffer's layout) ----------------
 * ec.Buffer carves a stripe's N+M+L shards at one stride from one allocation (common/ec/buf.go:
 * 83-84) and encoder.Split hands out exactly those slices (KRS/reedsolomon.go:1574-1632).  These
 * entry points take such a stripe as (base, shard_size, stride): shard i is shard_size bytes at
 * base + i * stride (stride >= shard_size), every shard present -- the broken ones are named by
 * bad_idx (ec) or missing (reedsolomon: what a len-0 shard marks in the vector forms) and rebuilt in
 * place.  One pointer per call: a Go caller passes Go memory under cgo's pointer rules as they stand
 * since Go 1.6 (no runtime.Pinner, no C array holding Go pointers), which is what CubeFS's Go 1.17
 * toolchain (go.mod:3, docker/Dockerfile:1) can build.  Semantics otherwise those of the vector
 * calls. */
int cfsec_rs_encode_contig(cfsec_rs* h, uint8_t* base, size_t shard_size, size_t stride, int n, int mem,
                           void* stream);
int cfsec_rs_verify_contig(cfsec_rs* h, uint8_t* base, size_t shard_size, size_t stride, int n, int mem,
                           void* stream, int* ok);
int cfsec_rs_reconstruct_contig(cfsec_rs* h, uint8_t* base, size_t shard_size, size_t stride, int n,
                                const int* missing, int nmissing, int data_only, int mem, void* stream);
int cfsec_ec_encode_contig(cfsec_ec* h, uint8_t* base, size_t shard_size, size_t stride, int n, int mem,
                           void* stream);
int cfsec_ec_verify_contig(cfsec_ec* h, uint8_t* base, size_t shard_size, size_t stride, int n, int mem,
                           void* stream, int* ok);
int cfsec_ec_reconstruct_contig(cfsec_ec* h, uint8_t* base, size_t shard_size, size_t stride, int n,
                                const int* bad_idx, int nbad, int data_only, int mem, void* stream);
/* Batches in one allocation: stripe s at base + s * stripe_stride (encode); bid b at
 * base + bid_off[b] with its shards packed at its own shard size bid_shard_size[b] (repair tasklet;
 * a zero-size bid is all empty shards).  crcs (host, may be NULL): the _crc forms' checksums. */
int cfsec_ec_encode_batch_contig(cfsec_ec* h, uint8_t* base, size_t shard_size, size_t stride, size_t stripe_stride,
                                 int n, int nstripes, int mem, int* status, uint32_t* crcs);
int cfsec_ec_reconstruct_batch_contig(cfsec_ec* h, uint8_t* base, const uint64_t* bid_off,
                                      const uint64_t* bid_shard_size, int n, int nbids, const int* bad_idx,
                                      const int* bad_off, int verify, int mem, int* status, uint32_t* crcs);

/* ---------------- pinned host memory ---------------- */
/* Page-locked host memory for shard buffers (the hook is resourcepool.NewMemPoolWith,
 * common/resourcepool/mempool.go:60, which ec.Buffer draws from, common/ec/buf.go:93-117).
 * CFSEC_MEM_HOST calls on such buffers DMA straight to HBM instead of through the runtime's
 * staging copies.  C memory: safe to hand to cgo. */
int cfsec_host_alloc(size_t size, void** out);
int cfsec_host_free(void* p);

/* ---------------- shard CRC32 (access/stream_put.go:249-253) ---------------- */
/* crc32.ChecksumIEEE of each device shard; out: host array of n uint32. Synchronous. */
int cfsec_crc32_ieee_batch(uint8_t* const* ptrs, size_t shard_size, int n, uint32_t* out,
                           int device, void* stream);

/* Checksums of concatenations (host only, no device).  cfsec_crc32_combine: crc32.ChecksumIEEE(A || B)
 * from crc1 = ChecksumIEEE(A), crc2 = ChecksumIEEE(B) and len2 = |B| (zlib's crc32_combine).
 * cfsec_crc32_shift: words[i] <- words[i] * x^(8 nbytes) mod P, i.e. the term a byte range's checksum
 * contributes to the checksum of a longer run that continues for nbytes more bytes: the checksum of a
 * shard cut into column slices is the XOR of its slices' shifted checksums (the multi-GPU repair's
 * rebuilt shards, chubaofs_amd/repair.py; blobnode's ShardCrc32, blobnode/work_shard_recover.go:335-342). */
uint32_t cfsec_crc32_combine(uint32_t crc1, uint32_t crc2, int64_t len2);
int cfsec_crc32_shift(uint32_t* words, int n, int64_t nbytes);

/* Measurement helper (no reference counterpart): a flat grid-stride copy of `bytes` bytes (a
 * multiple of 16; both pointers device memory, 16-byte aligned) with non-temporal 16-byte loads and
 * stores, asynchronous on `stream` -- the device's streaming ceiling for a 1:1 read/write pattern,
 * which bench.py reports beside the HBM spec peak (tools/rot_probe.hip measured this form at 72-75 %
 * of 8 TB/s, above the HIP runtime's own copy). */
int cfsec_stream_copy(void* dst, const void* src, size_t bytes, void* stream);

/* ---------------- crc32block framing (blobstore/common/crc32block) ---------------- */
/* A framed object is a run of block_len-byte blocks (default 64 KiB; block_len a positive multiple
 * of 4096), each the little-endian crc32.ChecksumIEEE of its payload followed by the payload
 * (block_len - 4 bytes; fewer in the last block) -- block.go:34-49, encode.go:87-109.
 * Sizes: EncodeSize / DecodeSize (util.go:50-65); -1 when block_len is invalid (the Go functions
 * panic with ErrInvalidBlock) or the size is negative. */
int64_t cfsec_crc32block_encode_size(int64_t size, int64_t block_len);
int64_t cfsec_crc32block_decode_size(int64_t total, int64_t block_len);
/* Encoder.Encode (encode.go:48-58, blobnode core/storage/datafile.go:345-373): frame `size` payload
 * bytes of src into dst (cfsec_crc32block_encode_size bytes).  shard_crc (host, may be NULL)
 * receives crc32.ChecksumIEEE of the whole payload, which datafile.go:345-373 computes on the way
 * (shard.Crc).  One pass: every payload byte is read once and written once.  mem as for cfsec_rs_*:
 * CFSEC_MEM_DEVICE pointers run on `stream` (NULL = an internal stream) on `device` (-1 = current);
 * CFSEC_MEM_HOST buffers from cfsec_host_alloc are read and written in place, other host memory is
 * staged through HBM.  Returns after completion. */
int cfsec_crc32block_encode(const uint8_t* src, int64_t size, int64_t block_len, uint8_t* dst,
                            uint32_t* shard_crc, int mem, int device, void* stream);
/* Decoder.Reader(from, to) (decode.go:122-146; blobnode datafile.go:406-426): check the blocks of
 * the framed object src (src_len bytes readable; payload size `size`) that hold payload bytes
 * [from, to) -- and the block holding `from` when from == to is not block-aligned, as the
 * reference's skip does -- and copy those bytes to dst (to - from bytes; may be NULL when
 * from == to).  CFSEC_ERR_SHORT_DATA, before anything is read, when src_len ends before the last
 * touched block (the reference's SectionReader gives io.ErrUnexpectedEOF).
 * CFSEC_ERR_MISMATCHED_CRC when a checked block's checksum differs; *bad_block (may be NULL) =
 * index of the first such block, -1 otherwise. */
int cfsec_crc32block_decode(const uint8_t* src, int64_t src_len, int64_t size, int64_t block_len, int64_t from,
                            int64_t to, uint8_t* dst, int64_t* bad_block, int mem, int device, void* stream);
/* Batch forms on device memory, asynchronous on `stream` (NULL = the null stream): n objects of one
 * payload size -- the shards of a stripe batch (blobnode puts and repairs); decode: every source
 * object has at least src_len readable bytes (CFSEC_ERR_SHORT_DATA otherwise, as above).  encode: shard_crcs
 * (device, n words, may be NULL) receives each payload's crc32.ChecksumIEEE.  decode: checks and
 * unframes payload range [from, to) of each object; bad (device, n words) receives per object the
 * index of the first mismatching block counted from block from / (block_len - 4), or 0xFFFFFFFF. */
int cfsec_crc32block_encode_batch(const uint8_t* const* srcs, uint8_t* const* dsts, int n, int64_t size,
                                  int64_t block_len, uint32_t* shard_crcs, void* stream);
int cfsec_crc32block_decode_batch(const uint8_t* const* srcs, int64_t src_len, uint8_t* const* dsts, int n,
                                  int64_t size, int64_t block_len, int64_t from, int64_t to, uint32_t* bad,
                                  void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CFSEC_H_ */
