// gf_dy16.hip -- kernels for 16-input matrices opening with a 16x16 dyadic block (EC16P20 encode
// and the EC16P20L2 fused encode, the same 20 rows + 2 local rows); see gf_dyadic16.hpp.  The local
// rows share the 4x4 row block's registers and take one input column at a time (pairs of columns
// needed 256 VGPRs + AGPRs: 1 wave/SIMD; this form 214-217, 2 waves/SIMD like EC16P20's 178-201).
#include <cstdlib>
#include <cstring>

#include "gf_dyadic16.hpp"
#include "gf_launch.hpp"

#ifndef CFSEC_DY16_W
#define CFSEC_DY16_W 2  // dwords per lane: 8-byte lane chunks (byte-form kernels)
#endif

namespace cfsec {

template <int M, int R4, int E, MatVecMode MODE, int W>
__global__ __launch_bounds__(256) void gf_dy16_kernel(const dev::GfArgs a) {
  dev::matvec_dy16<M, R4, E, MODE, true, W>(a);
}

namespace {
// The 16x16-dyadic repair (A/B): CFSEC_DY16F=0 the round-3 form (inputs in first-present order,
// data rows permuted with selects), default the inputs in data-row slots
int dy16_form() {
  static const int f = [] {
    const char* v = std::getenv("CFSEC_DY16F");
    return v && *v ? std::atoi(v) : 2;
  }();
  return f;
}

template <int M, int R4, int E, int W>
hipError_t launch_one(MatVecMode mode, const dev::GfArgs& a, unsigned ns, hipStream_t st) {
  constexpr uint64_t tile = 256 * 4 * W;
  const unsigned tiles = (unsigned)((a.len + tile - 1) / tile);
  if (mode == MatVecMode::kVerify)
    hipLaunchKernelGGL((gf_dy16_kernel<M, R4, E, MatVecMode::kVerify, W>), dim3(tiles, ns), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((gf_dy16_kernel<M, R4, E, MatVecMode::kStore, W>), dim3(tiles, ns), dim3(256), 0, st, a);
  return hipGetLastError();
}
}  // namespace

template <int ND, int E>
__global__ __launch_bounds__(256) void gf_dy16_repair_kernel(const dev::GfArgs a) {
  dev::repair_dy16<ND, E, true, CFSEC_DY16_W>(a);
}

// The slot-ordered repair's argument block from the first-present one: inputs in data-row slots
// (slot i = data row i when present, else the parity input standing in for missing row j), decode
// coefficients permuted to slot order, src[j] = the data row of missing row j.
static void to_slot_order(int nd, int ne, const dev::GfArgs& a, dev::GfArgs& f) {
  std::memcpy(&f, &a, sizeof(dev::GfArgs));
  int col[16];
  for (int i = 0; i < 16; ++i) {
    const int s = a.src[i];
    col[i] = s < 16 ? s : (16 - nd) + (s - 16);
    if (s >= 16) f.src[s - 16] = (uint8_t)i;
  }
  for (int j = 0; j < nd; ++j)
    for (int i = 0; i < 16; ++i) f.coef[(20 + ne + j) * 16 + i] = a.coef[(20 + ne + j) * 16 + col[i]];
  for (uint32_t s = 0; s < a.tab; ++s)
    for (int i = 0; i < 16; ++i) f.ptr[s * 16 + i] = a.ptr[s * 16 + col[i]];
}

#ifndef CFSEC_DY16_PF
// compared rows of the 16x16 block loaded before it (repair_dy16 PF): 152 VGPRs, 3 waves per SIMD,
// C5 201-203 vs 190 us per call without (profiles/r04/dy16_pf_ab.txt)
#define CFSEC_DY16_PF 0
#endif
#ifndef CFSEC_DY16_WPE
#define CFSEC_DY16_WPE 4  // waves per SIMD the repair kernel's registers aim at (probes: 5)
#endif
template <int ND, int E>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(CFSEC_DY16_WPE, 8))) void gf_dy16s_repair_kernel(
    const dev::GfArgs a) {
  dev::repair_dy16<ND, E, true, CFSEC_DY16_W, true, (bool)CFSEC_DY16_PF>(a);
}

template <int E>
hipError_t launch_repair_s(int nd, const dev::GfArgs& a, dim3 grid, hipStream_t st) {
  switch (nd) {
    case 0: hipLaunchKernelGGL((gf_dy16s_repair_kernel<0, E>), grid, dim3(256), 0, st, a); break;
    case 1: hipLaunchKernelGGL((gf_dy16s_repair_kernel<1, E>), grid, dim3(256), 0, st, a); break;
    case 2: hipLaunchKernelGGL((gf_dy16s_repair_kernel<2, E>), grid, dim3(256), 0, st, a); break;
    case 3: hipLaunchKernelGGL((gf_dy16s_repair_kernel<3, E>), grid, dim3(256), 0, st, a); break;
    case 4: hipLaunchKernelGGL((gf_dy16s_repair_kernel<4, E>), grid, dim3(256), 0, st, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <int E>
hipError_t launch_repair_e(int nd, const dev::GfArgs& a, dim3 grid, hipStream_t st) {
  switch (nd) {
    case 0: hipLaunchKernelGGL((gf_dy16_repair_kernel<0, E>), grid, dim3(256), 0, st, a); break;
    case 1: hipLaunchKernelGGL((gf_dy16_repair_kernel<1, E>), grid, dim3(256), 0, st, a); break;
    case 2: hipLaunchKernelGGL((gf_dy16_repair_kernel<2, E>), grid, dim3(256), 0, st, a); break;
    case 3: hipLaunchKernelGGL((gf_dy16_repair_kernel<3, E>), grid, dim3(256), 0, st, a); break;
    case 4: hipLaunchKernelGGL((gf_dy16_repair_kernel<4, E>), grid, dim3(256), 0, st, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ne extra rows: 0, or 2 (EC16P20L2's local parities checked in the global pass)
hipError_t launch_dy16_repair_args(int nd, int ne, const dev::GfArgs& a, unsigned ns, hipStream_t st) {
  constexpr uint64_t tile = 256 * 4 * CFSEC_DY16_W;
  const dim3 grid((unsigned)((a.len + tile - 1) / tile), ns);
  if (dy16_form() == 2) {
    static thread_local dev::GfArgs f;
    to_slot_order(nd, ne, a, f);
    switch (ne) {
      case 0: return launch_repair_s<0>(nd, f, grid, st);
      case 2: return launch_repair_s<2>(nd, f, grid, st);
      default: return hipErrorInvalidValue;
    }
  }
  switch (ne) {
    case 0: return launch_repair_e<0>(nd, a, grid, st);
    case 2: return launch_repair_e<2>(nd, a, grid, st);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_dy16(int m, MatVecMode mode, const dev::GfArgs& a, unsigned ns, hipStream_t st) {
  switch (m) {
    case 20: return launch_one<20, 1, 0, CFSEC_DY16_W>(mode, a, ns, st);  // EC16P20 global parity
    case 22: return launch_one<22, 1, 2, CFSEC_DY16_W>(mode, a, ns, st);  // EC16P20L2 fused: + 2 local rows
    default: return hipErrorInvalidValue;
  }
}

}  // namespace cfsec
