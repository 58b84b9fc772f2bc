// gf_lut_inst.hpp -- the launcher body of launch_lut_k<K> (included by gf_lut_k<K>.hip).
#pragma once
#include "gf_lut.hpp"
#include "gf_lut_launch.hpp"

namespace cfsec {
namespace lutinst {

template <int K, int M>
hipError_t go(MatVecMode mode, const dev::GfArgs& a, dim3 grid, hipStream_t st) {
  constexpr int ML = M <= 8 ? M : (M == 9 ? 8 : M);
  constexpr int LA = CFSEC_LUT_LOOKAHEAD, LW = lut_lane_dwords(K);
  switch (mode) {
    case MatVecMode::kStore:
      hipLaunchKernelGGL((lut::gf_lut_kernel<K, M, ML, MatVecMode::kStore, LA, LW>), grid, dim3(256), 0, st, a);
      break;
    case MatVecMode::kVerify:
      hipLaunchKernelGGL((lut::gf_lut_kernel<K, M, ML, MatVecMode::kVerify, LA, LW>), grid, dim3(256), 0, st, a);
      break;
    case MatVecMode::kStoreVerify:
      hipLaunchKernelGGL((lut::gf_lut_kernel<K, M, ML, MatVecMode::kStoreVerify, LA, LW>), grid, dim3(256), 0, st, a);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace lutinst
}  // namespace cfsec
