// gf_fixed.hpp -- definition of the fixed-K kernels (included only by gf_k<K>.hip).
//
// Rows are prefetched kFixedD ahead (tools/gf_pipe.hip, EC12P4 8 x 64 MiB on MI355X: D=2
// fastest; the runtime-k kernel waits for each row before multiplying it).
#pragma once
#include "gf_launch.hpp"

namespace cfsec {

constexpr int kFixedD = 2;

template <int K, int M, int OS, MatVecMode MODE>
__global__ __launch_bounds__(256) void gf_matvec_k_kernel(const dev::GfArgs a) {
  dev::matvec_k<K, M, MODE, kFixedD, OS>(a);
}

template <int K, MatVecMode MODE>
hipError_t launch_k(Shape sh, const dev::GfArgs& a, dim3 grid, hipStream_t st) {
#define CFSEC_KCASE(MV, OSV)                                                                  \
  case MV * 8 + OSV:                                                                          \
    hipLaunchKernelGGL((gf_matvec_k_kernel<K, MV, OSV, MODE>), grid, dim3(256), 0, st, a);    \
    break;
  switch (sh.M * 8 + sh.OS) {
    CFSEC_KCASE(1, 1) CFSEC_KCASE(2, 1) CFSEC_KCASE(3, 1) CFSEC_KCASE(4, 1) CFSEC_KCASE(5, 1)
    CFSEC_KCASE(6, 1) CFSEC_KCASE(4, 2) CFSEC_KCASE(5, 2) CFSEC_KCASE(6, 2) CFSEC_KCASE(4, 4)
    CFSEC_KCASE(5, 4) CFSEC_KCASE(6, 4) CFSEC_KCASE(8, 4)
    default: return hipErrorInvalidValue;
  }
#undef CFSEC_KCASE
  return hipGetLastError();
}

}  // namespace cfsec

#define CFSEC_INSTANTIATE_K(K)                                                                  \
  namespace cfsec {                                                                             \
  template hipError_t launch_k<K, MatVecMode::kStore>(Shape, const dev::GfArgs&, dim3, hipStream_t); \
  template hipError_t launch_k<K, MatVecMode::kVerify>(Shape, const dev::GfArgs&, dim3, hipStream_t); \
  }
