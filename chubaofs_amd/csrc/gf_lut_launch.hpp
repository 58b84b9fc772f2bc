// gf_lut_launch.hpp -- the lookup-product kernels (gf_lut.hpp) behind launch_matvec: which (k, m)
// take them, and their launchers (instantiated per k in gf_lut_k<K>.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "gf_device.hpp"
#include "kernels.hpp"

namespace cfsec {

// Outputs the lookups carry for a k x m product (the rest take the v_perm product in the same
// kernel), or 0 when the shape keeps the v_perm / dyadic kernels.  Measured against them on the
// same stripes (tools/lut_probe.hip, profiles/r03/lut_probe*.txt): EC15P12 encode 116 -> 94 us,
// verify 118 -> 89; EC12P9 encode 73 -> 63 (8 lookups + 1 v_perm row).  EC12P4 stays on its 4x4-
// dyadic kernel: faster in the probe (135 vs 141 us) but slower in the bench's rotated batches
// (0.659 vs 0.685 of 8 TB/s, profiles/r03/bench_lut_ab.txt); EC16P20(L2) and EC6P10(L2) stay on
// their dyadic kernels, and so do the narrow shapes of other k.
// Round 3, later (8-byte lanes, profiles/r03/lut_probe5.txt): k = 16, m = 5..16 -- EC16P20(L2) repairs
// of 5-16 shards -- beat both the plain v_perm kernel (16x8 107 -> 80 us, 16x12 152 -> 109, 16x16
// 192 -> 116) and the dyadic ones (16x8 94 -> 81, 16x12 125 -> 111, 16x16 160 -> 117); k = 6,
// m = 5..12 beat the plain kernel (6x8 71 -> 62, 6x10 86 -> 75) -- `dyadic` tells the launcher a
// dyadic kernel applies, which keeps EC6P6 / EC6P10 encodes on it (faster there).
inline int lut_outputs(int k, int m, bool dyadic = false) {
  if (k == 12 && m >= 5 && m <= 9) return m <= 8 ? m : 8;
  if ((k == 15 && m >= 5 && m <= 12) || (k == 16 && m >= 5 && m <= 16)) return m == 9 ? 8 : m;
  if (k == 6 && m >= 5 && m <= 12 && !dyadic) return m == 9 ? 8 : m;
  return 0;
}

// Lane chunk of the lookup kernel for k inputs: 8 bytes (EC15P12: 64 instead of 107 VGPRs, 8 waves
// per SIMD instead of 4; encode 96 -> 81 us, verify unchanged: profiles/r03/lut_probe4.txt), 16 bytes
// for k = 12 (EC12P9: no difference).  The launch grid's tiles are 256 lanes of it.
#ifndef CFSEC_LUT_K12_LW
#define CFSEC_LUT_K12_LW 4
#endif
constexpr int lut_lane_dwords(int k) { return k == 12 ? CFSEC_LUT_K12_LW : 2; }
constexpr size_t lut_tile_bytes(int k) { return size_t(256) * 4 * lut_lane_dwords(k); }

template <int K>
hipError_t launch_lut_k(int m, MatVecMode mode, const dev::GfArgs& a, dim3 grid, hipStream_t st);
template <>
hipError_t launch_lut_k<12>(int, MatVecMode, const dev::GfArgs&, dim3, hipStream_t);
template <>
hipError_t launch_lut_k<15>(int, MatVecMode, const dev::GfArgs&, dim3, hipStream_t);
template <>
hipError_t launch_lut_k<16>(int, MatVecMode, const dev::GfArgs&, dim3, hipStream_t);
template <>
hipError_t launch_lut_k<6>(int, MatVecMode, const dev::GfArgs&, dim3, hipStream_t);

inline hipError_t launch_lut(int k, int m, MatVecMode mode, const dev::GfArgs& a, dim3 grid, hipStream_t st) {
  switch (k) {
    case 6: return launch_lut_k<6>(m, mode, a, grid, st);
    case 12: return launch_lut_k<12>(m, mode, a, grid, st);
    case 15: return launch_lut_k<15>(m, mode, a, grid, st);
    case 16: return launch_lut_k<16>(m, mode, a, grid, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace cfsec
