// kernels.hpp -- host-side interface of the gfx950 GF(2^8) shard kernels.
//
// One kernel family does all the byte arithmetic of the path: a GF(2^8)
// matrix x shard-vector product over a batch of stripes,
//
//     out[s][r][b] = XOR_c coef[r][c] * in[s][c][b]      (b over the shard bytes)
//
// which is what KRS/reedsolomon.go:807-1134 (codeSomeShards / ...P / ...AVXP) and the
// generated AVX2/GFNI kernels (KRS/galois_gen_amd64.s) compute for Encode, for both
// passes of reconstruct, and (with a compare instead of a store) for Verify.
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>

namespace cfsec {

enum class MatVecMode : uint32_t {
  kStore = 0,        // out = M * in
  kAccum = 1,        // out ^= M * in     (input chunking when k > kMaxK)
  kVerify = 2,       // flags[s] |= (out != M * in)
  kStoreVerify = 3,  // rows [0, nstore): out = M * in; rows [nstore, m): flags[s] |= (out != M * in)
};

struct MatVecJob {
  int k = 0;                           // inputs per stripe
  int m = 0;                           // outputs per stripe
  const uint8_t* coef = nullptr;       // host, m x k row-major
  size_t len = 0;                      // bytes per shard
  int nstripes = 0;
  const uint8_t* const* in = nullptr;  // host array [nstripes * k] of device pointers
  uint8_t* const* out = nullptr;       // host array [nstripes * m] of device pointers
  MatVecMode mode = MatVecMode::kStore;
  uint32_t* flags = nullptr;           // device [nstripes], kVerify / kStoreVerify
  int nstore = 0;                      // kStoreVerify: stored rows (the first nstore of m)
  const uint64_t* lens = nullptr;      // host [nstripes] per-stripe lengths (len = 0 then); NULL: all `len`
};

// Reconstruct (+ Verify) of stripes of the 16 + 20 code through the 16x16 dyadic block
// (gf_dyadic16.hpp repair_dy16): the nd <= 4 missing data rows from decode rows, then every parity
// row from the 16 data rows, stored (pstore bit r) or compared (pcmp bit r, mismatch -> flags).
struct Dy16RepairJob {
  int nd = 0;                          // missing data rows
  int e = 0;                           // extra rows over the data after the parity rows (0 or 2)
  const uint8_t* coef = nullptr;       // host: parity matrix (20 x 16), the e extra rows, the nd decode rows
  uint8_t src[16] = {};                // data row i: input slot, or 16 + j for missing data row j
  uint32_t pstore = 0, pcmp = 0;       // parity (then extra) rows stored / compared
  size_t len = 0;
  const uint64_t* lens = nullptr;      // host [nstripes] per-stripe lengths, or NULL
  int nstripes = 0;
  const uint8_t* const* in = nullptr;  // host [nstripes * 16]: the first 16 present rows
  uint8_t* const* out = nullptr;       // host [nstripes * (nd + 20 + e)]: missing data rows, parity 0..19, extras
  uint32_t* flags = nullptr;           // device [nstripes]
  uint32_t* zero_words = nullptr;      // device: nzero words the first launch zeroes (a batch's checksum
  uint32_t nzero = 0;                  // words, XOR-accumulated by the checksum pass that follows)
  bool syn = false;                    // the syndrome form below is set: the bit-sliced kernel may run
  uint8_t prow[4] = {};                // input 16 - nd + q is parity row prow[q]
  uint8_t ainv[16] = {};               // missing row j = sum_q ainv[j * 4 + q] * syndrome of prow[q]
  // the stored rows' checksums in the same pass (bit-sliced kernel only): stripe s's checksummed row
  // k (the missing data rows, then the stored parity rows in order) XOR-accumulates crc32.ChecksumIEEE
  // into crc_words[s * crc_stride + crc_slot[k]] (zeroed by the caller, zero_words must be NULL);
  // crc_done[s] is set to 1 for the stripes whose words the launches accumulated (host array)
  uint32_t* crc_words = nullptr;
  uint32_t crc_stride = 0;
  uint8_t crc_slot[4] = {};
  int crc_mode = 1;  // gf_launch.hpp BsCrcReq::mode
  char* crc_done = nullptr;
};
hipError_t launch_dy16_repair(const Dy16RepairJob& job, hipStream_t stream);
// what the bit-sliced repair (and its checksums) takes: whole 2 KiB column tiles, <= 2 missing data
// rows (gf_launch.hpp kBs16Tile / kBsRepairMaxNd)
constexpr uint64_t kBsRepairTileBytes = 2048;
constexpr int kBsRepairMaxMissing = 2;

// Verify flags of a batch call gathered per batch item (batch.cpp run_device): for every item o,
// out[o] = OR of the per-task words tmp[word[j]] of the pairs (o, word[j]) -- `accumulate`: out[o] |=
// (v != 0), else out[o] = (v != 0) -- and those tmp words are reset to 0, so a workspace's flag words
// stay zero between calls (no memset per call).  pairs: n (item, word) entries sorted by item; out
// may be host-mapped pinned memory (the synchronous calls read it after the sync, no D2H copy).
// cfsec_stream_copy: dst[0, bytes) <- src, 16-byte non-temporal grid-stride copy (bytes % 16 == 0).
hipError_t launch_stream_copy(void* dst, const void* src, size_t bytes, hipStream_t stream);
hipError_t launch_flag_gather(uint32_t* tmp, uint32_t* out, const int* item, const int* word, int n,
                              bool accumulate, hipStream_t stream);

// Rows one launch carries (dev::kMaxK / dev::kMaxM); kStoreVerify needs m <= kLaunchMaxRows.
constexpr int kLaunchMaxRows = 32;

// Enqueue the product on `stream`.  Splits into as many launches as the kernel
// argument block needs (inputs > 32, outputs > 32, or too many pointers).
hipError_t launch_matvec(const MatVecJob& job, hipStream_t stream);

// crc32.ChecksumIEEE of n device shards of `len` bytes into device out[n].
// Leaves the raw (pre-conditioning) word per shard in out; crc32_finalize turns it
// into crc32.ChecksumIEEE.
hipError_t launch_crc32(const uint8_t* const* ptrs, size_t len, int n, uint32_t* out,
                        hipStream_t stream);
uint32_t crc32_finalize(uint32_t raw, size_t len);
// Standalone form with scattered outputs: shard i's word is out[idx[i]] (idx NULL: out[i]),
// accumulated with atomicXor into words the caller has zeroed, `fin` XOR-ed in once per shard
// (crc32_shift_ones(len) gives crc32.ChecksumIEEE directly).
hipError_t launch_crc32_to(const uint8_t* const* ptrs, size_t len, int n, uint32_t* out, const uint32_t* idx,
                           uint32_t fin, hipStream_t stream);

// Encode / reconstruct (kStore) with crc32.ChecksumIEEE of the rows the product touches, fused
// into the product kernel (gf_crc.hpp): row i of the product (inputs 0..k-1, then outputs) has its
// checksum in device word crc[s * crc_stride + slot[i]] of stripe s.  slot[0] < 0 skips the inputs
// (checksum the outputs only).  Every word of crc[0 .. nstripes*crc_stride) is zeroed first, so
// words no row maps to read 0 (zero = false: the caller zeroed them; the kernel XORs into them).
// Only for matvec_crc_supported shapes (k in {6,8,12,16,18}, m <= 6; and k = 6, m = 12 when coef is
// EC6P10L2's fused LRC matrix: 10 rows of 2x2 dyadic blocks + 2 plain rows).
bool matvec_crc_supported(int k, int m, size_t len, const uint8_t* coef = nullptr);
// launch_matvec_crc takes exactly the jobs this accepts (a supported shape, kStore, checksum slots
// inside [0, crc_stride) with crc_stride <= 256, the inputs checksummed where the only instantiated
// form does so); callers route everything else to the product and the separate pass.
bool matvec_crc_accepts(const MatVecJob& job, int crc_stride, const int* slot);
hipError_t launch_matvec_crc(const MatVecJob& job, uint32_t* crc, int crc_stride, const int* slot,
                             hipStream_t stream, bool zero = true);
// shift(~0, len) ^ ~0: XOR it into a raw (zero-preset) CRC of len bytes to get crc32.ChecksumIEEE.
uint32_t crc32_shift_ones(size_t len);

// blobstore/common/crc32block framing (crc32block.hip): blocks of block_len bytes, each the
// little-endian crc32.ChecksumIEEE of its payload (block_len - 4 bytes, less in the last block)
// followed by the payload.  Device pointers.
struct Crc32BlockJob {
  bool encode = true;
  int n = 1;                           // objects, all of the same payload size
  const uint8_t* const* in = nullptr;  // host array [n]: encode: payloads; decode: framed objects
  uint8_t* const* out = nullptr;       // host array [n]: encode: framed objects (EncodeSize bytes);
                                       // decode: to - from bytes each
  int64_t size = 0;                    // payload bytes of each object
  int64_t block_len = 0;               // positive multiple of 4096
  int64_t from = 0, to = 0;            // decode: payload range (Decoder.Reader(from, to))
  uint32_t* bad = nullptr;    // decode: device words [n] preset to ~0; receive the smallest mismatching
                              // block index relative to block from / (block_len - 4)
  uint32_t* whole = nullptr;  // encode, optional: device words [n] preset to 0; receive
                              // crc32.ChecksumIEEE of each whole payload
};
bool crc32block_valid_len(int64_t block_len);  // util.go:34-36
hipError_t launch_crc32block(const Crc32BlockJob& job, hipStream_t stream);

}  // namespace cfsec
