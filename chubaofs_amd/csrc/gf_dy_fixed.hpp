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

// Launch the kernel for output count m, one of Ms.
template <int K, int B, MatVecMode MODE, int... Ms>
hipError_t launch_dy_m(int m, const dev::GfArgs& a, unsigned ns, hipStream_t st) {
  hipError_t e = hipErrorInvalidValue;
  (void)((m == Ms ? (e = launch_dy_one<K, Ms, B, MODE>(a, ns, st), true) : false) || ...);
  return e;
}

}  // namespace cfsec

// launch_dy<K> for block size BV and the output counts listed after it (dyadic_shape in
// gf_launch.hpp must list the same ones).
#define CFSEC_DY_INSTANTIATE(K, BV, ...)                                                            \
  namespace cfsec {                                                                                 \
  template <>                                                                                       \
  hipError_t launch_dy<K>(int m, int B, MatVecMode mode, const dev::GfArgs& a, unsigned ns,         \
                          hipStream_t st) {                                                         \
    if (B != BV || dyadic_shape(K, m) != BV) return hipErrorInvalidValue;                           \
    return mode == MatVecMode::kVerify                                                              \
               ? launch_dy_m<K, BV, MatVecMode::kVerify, __VA_ARGS__>(m, a, ns, st)                 \
               : launch_dy_m<K, BV, MatVecMode::kStore, __VA_ARGS__>(m, a, ns, st);                 \
  }                                                                                                 \
  }
