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
  kStore = 0,   // out = M * in
  kAccum = 1,   // out ^= M * in     (input chunking when k > kMaxK)
  kVerify = 2,  // flags[s] |= (out != M * in)
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
  uint32_t* flags = nullptr;           // device [nstripes], kVerify only
};

// Enqueue the product on `stream`.  Splits into as many launches as the kernel
// argument block needs (inputs > 32, outputs > 32, or too many pointers).
hipError_t launch_matvec(const MatVecJob& job, hipStream_t stream);

// crc32.ChecksumIEEE of n device shards of `len` bytes into device out[n].
// Leaves the raw (pre-conditioning) word per shard in out; crc32_finalize turns it
// into crc32.ChecksumIEEE.
hipError_t launch_crc32(const uint8_t* const* ptrs, size_t len, int n, uint32_t* out,
                        hipStream_t stream);
uint32_t crc32_finalize(uint32_t raw, size_t len);

}  // namespace cfsec
