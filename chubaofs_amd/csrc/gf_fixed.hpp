// gf_fixed.hpp -- definition of the fixed-K kernels (included only by gf_k<K>.hip).
//
// Rows are prefetched fixed_d() ahead (tools/gf_pipe.hip, EC12P4 8 x 64 MiB on MI355X: D=2
// fastest; the runtime-k kernel waits for each row before multiplying it).  Every output row of a
// column chunk stays in one wave (OS = 1) up to fixed_max_m(K): splitting the rows over 2 or 4
// waves re-reads the inputs once per wave from L2/LDS and was 8-22 % slower for m in 10..22
// (profiles/r01/wide_output_probe.txt) even though the single wave runs at 1-2 waves per SIMD.
#pragma once
#include "gf_launch.hpp"

namespace cfsec {

#ifndef CFSEC_FIXED_D
#define CFSEC_FIXED_D 2
#endif
// Verify modes load the compared rows in the same sequence and take 4 rows ahead: round 3, same call
// (tools/fixed_d_ab.sh, profiles/r03/fixed_d_ab.txt): EC4P4 verify 26.5 -> 21.0 us, EC6P10L2 local
// (8,1) 65.0 -> 63.4, EC6P3 38.5 -> 37.1; encode (store) unchanged at D = 4 or 8.
#ifndef CFSEC_FIXED_DV
#define CFSEC_FIXED_DV 4
#endif
template <MatVecMode MODE>
constexpr int fixed_d() {
  return MODE == MatVecMode::kVerify || MODE == MatVecMode::kStoreVerify ? CFSEC_FIXED_DV : CFSEC_FIXED_D;
}

template <int K, int M, MatVecMode MODE>
__global__ __launch_bounds__(256) void gf_matvec_k_kernel(const dev::GfArgs a) {
  dev::matvec_k<K, M, MODE, fixed_d<MODE>(), 1, true, true, true, dev::fixed_lane_dwords(K, M),
                dev::fixed_tiles_per_wg(M)>(a);
}

template <int K, MatVecMode MODE, int M>
hipError_t launch_k(int m, const dev::GfArgs& a, dim3 grid, hipStream_t st) {
  if constexpr (M == 0) {
    return hipErrorInvalidValue;
  } else {
    if (m != M) return launch_k<K, MODE, M - 1>(m, a, grid, st);
    constexpr unsigned T = dev::fixed_tiles_per_wg(M);
    const dim3 g((grid.x + T - 1) / T, grid.y);
    hipLaunchKernelGGL((gf_matvec_k_kernel<K, M, MODE>), g, dim3(256), 0, st, a);
    return hipGetLastError();
  }
}

}  // namespace cfsec

#define CFSEC_INSTANTIATE_K(K)                                                                   \
  namespace cfsec {                                                                              \
  template hipError_t launch_k<K, MatVecMode::kStore, fixed_max_m(K)>(int, const dev::GfArgs&, dim3, \
                                                                     hipStream_t);                  \
  template hipError_t launch_k<K, MatVecMode::kVerify, fixed_max_m(K)>(int, const dev::GfArgs&, dim3, \
                                                                      hipStream_t);                 \
  template hipError_t launch_k<K, MatVecMode::kStoreVerify, fixed_max_m(K)>(int, const dev::GfArgs&,   \
                                                                           dim3, hipStream_t);      \
  }
