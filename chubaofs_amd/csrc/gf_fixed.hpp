// gf_fixed.hpp -- definition of the fixed-K kernels (included only by gf_k<K>.hip).
//
// Rows are prefetched fixed_d() ahead (tools/gf_pipe.hip, EC12P4 8 x 64 MiB on MI355X: D=2
// fastest; the runtime-k kernel waits for each row before multiplying it).  Every output row of a
// column chunk stays in one wave (OS = 1) up to fixed_max_m(K): splitting the rows over 2 or 4
// waves re-reads the inputs once per wave from L2/LDS and was 8-22 % slower for m in 10..22
// (profiles/r01/wide_output_probe.txt) even though the single wave runs at 1-2 waves per SIMD.
#pragma once
#include <cstring>

#include "gf256.hpp"
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

// Products of at most CFSEC_FIXED_REGTAB coefficients keep their tables in registers (5 words per
// coefficient, packed by the host into the argument block) instead of building them in LDS behind a
// barrier: a workgroup codes one 4 KiB tile, so for few coefficients the build and barrier were a
// large share of its life.  tools/c4l_pattern_probe.hip (C4's local repair, k = 8, m = 1, 48 x
// 699,051 B, 3 batches rotated): LDS tables 57.7 us (0.654 of 8 TB/s); register tables 51.2 us at
// D = 2, 50.9 at D = 4; with sc1 stores 49.5 / 49.0 us (0.770) -- the same 8-read / 1-write pattern
// with trivial arithmetic 47.1-49.7 us.  These kernels take 4 rows of lookahead and sc1 stores.
#ifndef CFSEC_FIXED_REGTAB
#define CFSEC_FIXED_REGTAB 12
#endif
#ifndef CFSEC_FIXED_DREG
#define CFSEC_FIXED_DREG 4
#endif
#ifndef CFSEC_FIXED_REG_STORE_POL
#define CFSEC_FIXED_REG_STORE_POL 2  // st16_pol: sc1
#endif
constexpr bool fixed_regtab(int K, int M) { return K * M <= CFSEC_FIXED_REGTAB; }

template <int K, int M, MatVecMode MODE>
__global__ __launch_bounds__(256) void gf_matvec_k_kernel(const dev::GfArgs a) {
  constexpr bool kReg = fixed_regtab(K, M);
  dev::matvec_k<K, M, MODE, kReg ? CFSEC_FIXED_DREG : fixed_d<MODE>(), 1, true, true, true,
                dev::fixed_lane_dwords(K, M), dev::fixed_tiles_per_wg(M), kReg,
                kReg ? CFSEC_FIXED_REG_STORE_POL : CFSEC_STORE_POL>(a);
}

// The register-table kernels' argument block: from dev::kRegTabOff in the coef area, coefficient
// (c, r)'s t01 words at 4 * (c * m + r), then its t2 word at 4 * k * m + (c * m + r)
// (gf_device.hpp coef_tables).
inline void pack_reg_tables(int k, int m, const uint8_t* coef, uint8_t* area) {
  const GF& gf = GF::get();
  uint32_t w[5 * dev::kMaxK];  // k * m <= dev::kMaxK coefficients (launch_k)
  for (int c = 0; c < k; ++c)
    for (int r = 0; r < m; ++r) {
      uint32_t p[8];
      p[0] = coef[r * k + c];
      for (int j = 1; j < 8; ++j) p[j] = gf.mul((uint8_t)p[j - 1], 2);
      uint32_t t[5] = {0u, 0u, 0u, 0u, 0u};  // T0 lo, T0 hi, T1 lo, T1 hi, T2
      for (int e = 0; e < 8; ++e) {
        const uint32_t v0 = ((e & 1) ? p[0] : 0u) ^ ((e & 2) ? p[1] : 0u) ^ ((e & 4) ? p[2] : 0u);
        const uint32_t v1 = ((e & 1) ? p[3] : 0u) ^ ((e & 2) ? p[4] : 0u) ^ ((e & 4) ? p[5] : 0u);
        t[e < 4 ? 0 : 1] |= v0 << (8 * (e & 3));
        t[e < 4 ? 2 : 3] |= v1 << (8 * (e & 3));
        if (e < 4) t[4] |= (((e & 1) ? p[6] : 0u) ^ ((e & 2) ? p[7] : 0u)) << (8 * e);
      }
      const int i = c * m + r;
      for (int q = 0; q < 4; ++q) w[4 * i + q] = t[q];
      w[4 * k * m + i] = t[4];
    }
  std::memcpy(area + dev::kRegTabOff, w, (size_t)20 * k * m);
}

template <int K, MatVecMode MODE, int M>
hipError_t launch_k(int m, const dev::GfArgs& a, dim3 grid, hipStream_t st) {
  if constexpr (M == 0) {
    return hipErrorInvalidValue;
  } else {
    if (m != M) return launch_k<K, MODE, M - 1>(m, a, grid, st);
    constexpr unsigned T = dev::fixed_tiles_per_wg(M);
    const dim3 g((grid.x + T - 1) / T, grid.y);
    if constexpr (fixed_regtab(K, M)) {
      static_assert(20 * K * M + dev::kRegTabOff <= sizeof(dev::GfArgs::coef) && K * M <= dev::kMaxK,
                    "packed tables fit the coef area");
      static thread_local dev::GfArgs t;
      std::memcpy(&t, &a, sizeof(dev::GfArgs));
      pack_reg_tables(K, M, a.coef, t.coef);
      hipLaunchKernelGGL((gf_matvec_k_kernel<K, M, MODE>), g, dim3(256), 0, st, t);
    } else {
      hipLaunchKernelGGL((gf_matvec_k_kernel<K, M, MODE>), g, dim3(256), 0, st, a);
    }
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
