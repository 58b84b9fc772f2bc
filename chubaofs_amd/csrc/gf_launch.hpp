// gf_launch.hpp -- launcher internals shared by gf_kernels.hip and the fixed-K translation
// units gf_k<K>.hip (one TU per input count so the instantiations build in parallel).
#pragma once
#include <hip/hip_runtime.h>

#include "gf_device.hpp"
#include "kernels.hpp"

namespace cfsec {

// (M output rows per wave, OS waves sharing a column chunk) for mc outputs: small m keeps every
// output in one wave; larger m splits the outputs over 2 or 4 waves of the workgroup so each
// wave's accumulators + tables stay under ~64-90 VGPRs (a single wave holding 20 outputs
// needed 271 VGPRs = one wave per SIMD).
struct Shape {
  int M, OS;
};
inline Shape choose(int mc) {
  if (mc <= 6) return {mc, 1};
  if (mc <= 8) return {4, 2};
  if (mc <= 12) return {(mc + 1) / 2, 2};
  if (mc <= 24) return {(mc + 3) / 4, 4};
  return {8, 4};
}

// Fixed-K kernels for the input counts of the CubeFS code modes (codemode.go:40-120): k = 6
// (EC6P6, EC6P10, EC6P3), 8 (the EC6P10L2 local stripe), 12 (EC12P4, EC12P9), 16 (EC16P20,
// EC16P4), 18 (the EC16P20L2 local stripe), 15 (EC15P12), 10 (EC10P4), 3 (EC3P3, the EC6P3L3
// local stripe), 4 (EC4P4L2 and its local stripe, the EC6P6L9 local stripe), 7 (the EC6P8L10
// local stripe).
inline bool fixed_k(int k) {
  switch (k) {
    case 3: case 4: case 6: case 7: case 8: case 10: case 12: case 15: case 16: case 18: return true;
    default: return false;
  }
}

// Largest output count with a fixed-K kernel: EC6P10L2's 10 global + 2 local parities (6 x 12),
// up to 12 EC12P4 / EC12P9 / EC15P12 repair rows, EC16P20L2's 20 + 2 (16 x 22) and up to 24
// EC16P20 repair rows; 6 for the small stripes.
constexpr int fixed_max_m(int k) {
  return k == 6 || k == 12 || k == 15 ? 12 : k == 16 ? 24 : k == 8 ? 8 : k == 18 ? 4 : 6;
}

// Launch gf_matvec_k_kernel<K, m, MODE> on a (tiles of 4096 B, stripes) grid (defined in
// gf_fixed.hpp, instantiated for kStore and kVerify in gf_k<K>.hip).
template <int K, MatVecMode MODE, int M = fixed_max_m(K)>
hipError_t launch_k(int m, const dev::GfArgs& a, dim3 grid, hipStream_t st);

// Dyadic-block kernels (gf_dyadic.hpp) for an m x k matrix whose first m - E rows are made of
// B x B blocks with M[r0+i][c0+j] = M[r0][c0 + (i ^ j)] (E plain rows follow); specialised in
// gf_dy_k<K>.hip for the shapes dyadic_plan lists.
template <int K>
hipError_t launch_dy(int m, int B, int E, MatVecMode mode, const dev::GfArgs& a, unsigned ns, hipStream_t st);
template <>
hipError_t launch_dy<6>(int, int, int, MatVecMode, const dev::GfArgs&, unsigned, hipStream_t);
template <>
hipError_t launch_dy<12>(int, int, int, MatVecMode, const dev::GfArgs&, unsigned, hipStream_t);
template <>
hipError_t launch_dy<16>(int, int, int, MatVecMode, const dev::GfArgs&, unsigned, hipStream_t);

// The block size of the shipped dyadic kernel for an m x k matrix with e trailing plain rows, or 0:
// 4x4 blocks for k = 12 (m = 4, 8, 12) and k = 16 (m = 4 .. 20), 2x2 for k = 6 (m = 6 .. 12), and
// the fused LRC encodes with their 2 local rows (EC6P10L2: 6 x (10 + 2), EC16P20L2: 16 x (20 + 2)).
constexpr int dyadic_shape(int k, int m, int e = 0) {
  if (e == 2) return k == 16 && m == 22 ? 4 : k == 6 && m == 12 ? 2 : 0;
  if (e != 0) return 0;
  return ((k == 12 && m <= 12) || (k == 16 && m <= 20)) && m % 4 == 0 ? 4
         : k == 6 && m >= 6 && m <= 12 && m % 2 == 0                  ? 2
                                                                      : 0;
}

struct DyPlan {
  int B, E;  // B = 0: no dyadic kernel
};

// The dyadic kernel a matrix can take: all rows dyadic, else all but the last 2.
inline DyPlan dyadic_plan(const uint8_t* coef, int m, int k) {
  const auto blocks_hold = [&](int B, int md) {
    for (int r0 = 0; r0 < md; r0 += B)
      for (int c0 = 0; c0 < k; c0 += B)
        for (int i = 0; i < B; ++i)
          for (int j = 0; j < B; ++j)
            if (coef[(size_t)(r0 + i) * k + c0 + j] != coef[(size_t)r0 * k + c0 + (i ^ j)]) return false;
    return true;
  };
  for (int e : {0, 2}) {
    const int B = dyadic_shape(k, m, e);
    if (B && blocks_hold(B, m - e)) return {B, e};
  }
  return {0, 0};
}

// 16-input matrices whose first 16 rows form one 16x16 dyadic block, then one 4x4-dyadic row
// block (gf_dyadic16.hpp; m = 20: EC16P20), then for m = 22 two plain rows (the EC16P20L2 fused
// encode's local parity).
hipError_t launch_dy16(int m, MatVecMode mode, const dev::GfArgs& a, unsigned ns, hipStream_t st);

// The bit-sliced parity kernels (gf_bs16.hip) for the fixed matrices of EC16P20 (k 16, m 20) and
// EC16P20L2's fused encode (16, 22): coef (m x k, row stride k) must equal the network's constants
// (bs_matches); launch_bs covers columns [0, len) of every stripe, len a multiple of kBs16Tile,
// every row pointer (and sstride) 16-byte aligned.
constexpr uint64_t kBs16Tile = 2048;
bool bs_matches(const uint8_t* coef, int m, int k);
hipError_t launch_bs(int k, int m, const dev::GfArgs& a, unsigned ns, uint64_t len, hipStream_t st);
// The same network for a repair_dy16 argument block (ne = 0 / 2 extra rows) of an affine batch (tab
// == 1): missing[q] the data row of missing row q, prow[q] the parity row of input 16 - nd + q, ainv
// (nd x nd, row stride 4) the inverse of those parity rows at the missing columns; columns [0, len),
// len a multiple of kBs16Tile; nd <= kBsRepairMaxNd (3 and 4 missing data rows spill: dyadic kernel).
constexpr int kBsRepairMaxNd = 2;
// The rebuilt shards' checksums in the same pass (gf_bs16.hip, CRC launches): nrows (= nd + the stored
// parity rows, at most 4) rows per stripe, row k's crc32.ChecksumIEEE XOR-accumulated into
// words[s * stride + slot[k]] (the caller zeroes the words before the launch; a.nzw must be 0).
// Taken only when len == the launch's columns (no row tail) and the device tables can be had:
// *crc_done says whether this launch accumulated the words.
struct BsCrcReq {
  uint32_t stride = 0;
  uint8_t slot[4] = {};
  int nrows = 0;
  int mode = 1;  // 1: Horner inside the network (blocked tile order); 2: a pass over the wave's own tiles after them
};
hipError_t launch_bs16_repair(int nd, int ne, const uint8_t* missing, const uint8_t* prow, const uint8_t* ainv,
                              const dev::GfArgs& a, unsigned ns, uint64_t len, hipStream_t st,
                              const BsCrcReq* crc = nullptr, uint32_t* crc_words = nullptr, bool* crc_done = nullptr);
// The same for stripes at unrelated addresses (every shard its own buffer): rows[s * (16 + mo) + i]
// (the 16 inputs, then the mo = nd + 20 + ne outputs of stripe s) for ns stripes, every pointer
// 16-byte aligned; a's other fields (flags, zw, pstore / pcmp, src) as for launch_bs16_repair.  The
// rows go into the launch as 32-bit offsets from the lowest address, kBsTabStripes(mo) stripes per
// launch; false in *ok when the rows span 4 GiB or more (the caller keeps its route).
int bs_tab_stripes(int mo);
// launch_bs for stripes at unrelated addresses: rows[s * (k + m) + i] (inputs, then outputs), any
// number of stripes in one launch through a device copy of their 32-bit offsets; *ok false when the
// rows span 4 GiB or more or the table cannot be had (the caller keeps its route)
hipError_t launch_bs_tab(int k, int m, const dev::GfArgs& a, const uint8_t* const* rows, unsigned ns, uint64_t len,
                         hipStream_t st, bool* ok);
hipError_t launch_bs16_repair_tab(int nd, int ne, const uint8_t* missing, const uint8_t* prow, const uint8_t* ainv,
                                  const dev::GfArgs& a, const uint8_t* const* rows, unsigned ns, uint64_t len,
                                  hipStream_t st, bool* ok, const BsCrcReq* crc = nullptr,
                                  uint32_t* crc_words = nullptr, bool* crc_done = nullptr);

// Fused encode + crc32.ChecksumIEEE of every row on the bit-sliced networks (gf_bs_crc.hip, round 6):
// EC6P10L2's fused LRC encode (6 x 12) and EC12P4's encode (12 x 4), coef equal to the network's
// constants, the inputs checksummed too (slot[0] >= 0), any row alignment and length; words as
// launch_matvec_crc (zeroed by the caller).  CFSEC_BS_CRC (bit 0: 6 x 12, bit 1: 12 x 4) = 0 keeps
// the lookup-product kernels.
bool bs_crc_matches(int k, int m, const uint8_t* coef);
bool bs_crc_takes(const MatVecJob& job, int crc_stride, const int* slot);
hipError_t launch_bs_crc(const MatVecJob& job, uint32_t* crc, int crc_stride, const int* slot, hipStream_t st);
// The product alone on the same kernel (no checksums) for the wide LRC modes' fused encodes (EC6P6L9,
// EC6P8L10): a kStore job whose coef equals their networks, any alignment and length
bool bs_plain_matches(int k, int m, const uint8_t* coef);
hipError_t launch_bs_plain(const MatVecJob& job, hipStream_t st);

// repair_dy16 on a GfArgs block (gf_dy16.hip); launch_dy16_repair (gf_kernels.hip) fills it.
hipError_t launch_dy16_repair_args(int nd, int ne, const dev::GfArgs& a, unsigned ns, hipStream_t st);

inline bool dyadic16_plan(const uint8_t* coef, int m, int k) {
  if (k != 16 || (m != 20 && m != 22)) return false;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j)
      if (coef[(size_t)i * 16 + j] != coef[i ^ j]) return false;
  for (int c0 = 0; c0 < 16; c0 += 4)
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j)
        if (coef[(size_t)(16 + i) * 16 + c0 + j] != coef[(size_t)16 * 16 + c0 + (i ^ j)]) return false;
  return true;
}

#define CFSEC_EXTERN_K(K)                                                                         \
  extern template hipError_t launch_k<K, MatVecMode::kStore, fixed_max_m(K)>(int, const dev::GfArgs&, \
                                                                            dim3, hipStream_t);     \
  extern template hipError_t launch_k<K, MatVecMode::kVerify, fixed_max_m(K)>(int, const dev::GfArgs&, \
                                                                             dim3, hipStream_t);     \
  extern template hipError_t launch_k<K, MatVecMode::kStoreVerify, fixed_max_m(K)>(                   \
      int, const dev::GfArgs&, dim3, hipStream_t);
CFSEC_EXTERN_K(3)
CFSEC_EXTERN_K(4)
CFSEC_EXTERN_K(6)
CFSEC_EXTERN_K(7)
CFSEC_EXTERN_K(8)
CFSEC_EXTERN_K(10)
CFSEC_EXTERN_K(15)
CFSEC_EXTERN_K(12)
CFSEC_EXTERN_K(16)
CFSEC_EXTERN_K(18)
#undef CFSEC_EXTERN_K

}  // namespace cfsec
