// gf_dy_fixed.hpp -- dyadic-block kernels (gf_dyadic.hpp) and their launch switch; included only
// by gf_dy_k<K>.hip, one translation unit per input count.
#pragma once
#include "gf_dyadic.hpp"
#include "gf_launch.hpp"

namespace cfsec {

#ifndef CFSEC_DY_WPE
#define CFSEC_DY_WPE 1  // amdgpu_waves_per_eu floor (1: the compiler's choice)
#endif
template <int K, int M, int B, MatVecMode MODE, int E>
__global__ __launch_bounds__((dev::DyShape<M - E, B>::kThreadsPerWg))
__attribute__((amdgpu_waves_per_eu(CFSEC_DY_WPE, 8))) void gf_dy_kernel(const dev::GfArgs a) {
  dev::matvec_dy<K, M, B, MODE, true, true, 64, E>(a);
}

template <int K, int M, int B, MatVecMode MODE, int E>
hipError_t launch_dy_one(const dev::GfArgs& a, unsigned ns, hipStream_t st) {
  using Sh = dev::DyShape<M - E, B>;
  const unsigned tiles = (unsigned)((a.len + Sh::kTileBytes - 1) / Sh::kTileBytes);
  hipLaunchKernelGGL((gf_dy_kernel<K, M, B, MODE, E>), dim3(tiles, ns), dim3(Sh::kThreadsPerWg), 0, st, a);
  return hipGetLastError();
}

// Launch the kernel for output count m, one of Ms.
template <int K, int B, MatVecMode MODE, int E, int... Ms>
hipError_t launch_dy_m(int m, const dev::GfArgs& a, unsigned ns, hipStream_t st) {
  hipError_t e = hipErrorInvalidValue;
  (void)((m == Ms ? (e = launch_dy_one<K, Ms, B, MODE, E>(a, ns, st), true) : false) || ...);
  return e;
}

template <int... M>
struct Ms {};

// launch_dy<K> body: block size BV, all-dyadic output counts M0, output counts M2 with 2 plain
// rows (dyadic_plan in gf_launch.hpp must list the same ones).
template <int K, int BV, int... M0, int... M2>
hipError_t dy_dispatch(Ms<M0...>, Ms<M2...>, int m, int B, int E, MatVecMode mode, const dev::GfArgs& a,
                       unsigned ns, hipStream_t st) {
  constexpr MatVecMode kV = MatVecMode::kVerify, kS = MatVecMode::kStore;
  if (B != BV) return hipErrorInvalidValue;
  const bool v = mode == kV;
  if (E == 0) return v ? launch_dy_m<K, BV, kV, 0, M0...>(m, a, ns, st) : launch_dy_m<K, BV, kS, 0, M0...>(m, a, ns, st);
  if (E == 2) return v ? launch_dy_m<K, BV, kV, 2, M2...>(m, a, ns, st) : launch_dy_m<K, BV, kS, 2, M2...>(m, a, ns, st);
  return hipErrorInvalidValue;
}

}  // namespace cfsec
