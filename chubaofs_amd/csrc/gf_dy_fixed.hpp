// gf_dy_fixed.hpp -- dyadic-block kernels (gf_dyadic.hpp) and their launch switch; included only
// by gf_dy_k<K>.hip, one translation unit per input count.
#pragma once
#include "gf_dyadic.hpp"
#include "gf_launch.hpp"

namespace cfsec {

template <int K, int M, int B, MatVecMode MODE>
__global__ __launch_bounds__((dev::DyShape<M, B>::kThreadsPerWg)) void gf_dy_kernel(const dev::GfArgs a) {
  dev::matvec_dy<K, M, B, MODE>(a);
}

template <int K, int M, int B, MatVecMode MODE>
hipError_t launch_dy_one(const dev::GfArgs& a, unsigned ns, hipStream_t st) {
  using Sh = dev::DyShape<M, B>;
  const unsigned tiles = (unsigned)((a.len + Sh::kTileBytes - 1) / Sh::kTileBytes);
  hipLaunchKernelGGL((gf_dy_kernel<K, M, B, MODE>), dim3(tiles, ns), dim3(Sh::kThreadsPerWg), 0, st, a);
  return hipGetLastError();
}

}  // namespace cfsec

// K with 4x4 blocks, 4 outputs (one wave per column chunk).  Wider outputs (EC16P20) and the 2x2
// kernels are slower than the plain tile on MI355X (shape sweep: the multi-wave split halves the
// occupancy at ~120 VGPRs), so only this shape ships.
#define CFSEC_DY_INSTANTIATE_B4(K)                                                                  \
  namespace cfsec {                                                                                 \
  template <>                                                                                       \
  hipError_t launch_dy<K>(int m, int B, MatVecMode mode, const dev::GfArgs& a, unsigned ns,         \
                          hipStream_t st) {                                                         \
    if (B != 4 || m != 4) return hipErrorInvalidValue;                                              \
    return mode == MatVecMode::kVerify ? launch_dy_one<K, 4, 4, MatVecMode::kVerify>(a, ns, st)     \
                                       : launch_dy_one<K, 4, 4, MatVecMode::kStore>(a, ns, st);     \
  }                                                                                                 \
  }
