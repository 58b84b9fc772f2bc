// gf_kernels.hip -- gfx950 kernels for GF(2^8) Reed-Solomon shard coding (launcher).
//
// Replaces the CPU kernels of klauspost/reedsolomon v1.11.7 (the generated
// mulAvxTwo_RxC / mulGFNI_RxC_64 families in KRS/galois_gen_amd64.s and the
// galMulSlice[Xor] tails in KRS/galois_amd64.go:57-122) with one HBM-streaming
// kernel per output-row count.  Device code: gf_device.hpp.
//
// Arithmetic.  GF(2^8) multiplication by a constant is linear over GF(2), so a
// byte x is split into bit fields x = x[2:0] | x[5:3] | x[7:6] and
//     c*x = T0_c[x[2:0]] ^ T1_c[x[5:3]] ^ T2_c[x[7:6]]
// with 8-, 8- and 4-entry product tables.  An 8-entry byte table is exactly
// what one v_perm_b32 indexes: the two table dwords are the perm's data
// operands and the 3-bit fields (one per byte of the lane's dword) its
// selector, so one VALU op looks up 4 bytes at once.  Per (coefficient, dword)
// the cost is 3 v_perm_b32 + v_bitop3_b32 + v_xor; per input dword the 3
// selectors cost 5 ops, amortised over all outputs.  No MFMA: GF arithmetic is
// not an FP/int contraction.
//
// Data movement.  Each lane owns 16 consecutive bytes of the shard (one
// global_load_dwordx4 per input row, one global_store_dwordx4 per output row),
// so a workgroup streams whole 1 KiB-per-wave runs of every row and every byte
// of HBM is touched exactly once: read k*len, write m*len (verify: read
// (k+m)*len, write nothing).  Loads and stores are non-temporal (each byte is
// touched once).  The product tables are rebuilt per workgroup in LDS from the
// coefficient matrix carried in the kernel argument block, which keeps the
// launch free of device allocations and host->device copies (safe under
// concurrent callers and hipGraph capture).
//
// Policies (tools/gf_variants.hip, interleaved A/B on MI355X, EC12P4 8x64 MiB):
//   store/accum: 256-thread workgroups, 1 chunk per lane, loads one row at a time
//                (deeper per-lane load batches and persistent grids measured slower)
//   verify:      128-thread workgroups, 2 chunks per lane, rows loaded in pairs
#include <algorithm>

#include "gf_device.hpp"
#include "kernels.hpp"

namespace cfsec {
namespace {

using dev::GfArgs;
constexpr int kStoreThreads = 256;
constexpr int kStoreW = 1;
constexpr int kVerifyThreads = 128;
constexpr int kVerifyW = 2;

template <int M, MatVecMode MODE>
__global__ __launch_bounds__(256) void gf_matvec_kernel(const GfArgs a) {
  if constexpr (MODE == MatVecMode::kVerify)
    dev::matvec<M, MODE, kVerifyW, 2, false, true, true, false>(a);
  else
    dev::matvec<M, MODE, kStoreW, 1, false, true, true, false>(a);
}

template <MatVecMode MODE>
hipError_t launch_mode(int mpad, const GfArgs& a, dim3 grid, int threads, hipStream_t st) {
#define CFSEC_CASE(MV)                                                                   \
  case MV:                                                                               \
    hipLaunchKernelGGL((gf_matvec_kernel<MV, MODE>), grid, dim3(threads), 0, st, a);     \
    break;
  switch (mpad) {
    CFSEC_CASE(1) CFSEC_CASE(2) CFSEC_CASE(3) CFSEC_CASE(4) CFSEC_CASE(5) CFSEC_CASE(6)
    CFSEC_CASE(8) CFSEC_CASE(10) CFSEC_CASE(12) CFSEC_CASE(16) CFSEC_CASE(20)
    CFSEC_CASE(24) CFSEC_CASE(32)
    default: return hipErrorInvalidValue;
  }
#undef CFSEC_CASE
  return hipGetLastError();
}

int pad_outputs(int m) {
  static const int kSizes[] = {1, 2, 3, 4, 5, 6, 8, 10, 12, 16, 20, 24, 32};
  for (int s : kSizes)
    if (s >= m) return s;
  return -1;
}

}  // namespace

hipError_t launch_matvec(const MatVecJob& job, hipStream_t stream) {
  using dev::kMaxK;
  using dev::kMaxM;
  using dev::kPtrSlots;
  if (job.k <= 0 || job.m < 0 || job.nstripes < 0 || !job.coef || !job.in || !job.out)
    return hipErrorInvalidValue;
  if (job.m == 0 || job.nstripes == 0 || job.len == 0) return hipSuccess;
  if (job.mode == MatVecMode::kVerify && (job.k > kMaxK || !job.flags)) return hipErrorInvalidValue;

  GfArgs a;
  for (int r0 = 0; r0 < job.m; r0 += kMaxM) {
    const int mc = std::min(kMaxM, job.m - r0);
    for (int c0 = 0; c0 < job.k; c0 += kMaxK) {
      const int kc = std::min(kMaxK, job.k - c0);
      MatVecMode mode = job.mode;
      if (mode == MatVecMode::kStore && c0 > 0) mode = MatVecMode::kAccum;
      const bool verify = mode == MatVecMode::kVerify;
      const int threads = verify ? kVerifyThreads : kStoreThreads;
      const size_t tile = size_t(threads) * dev::kLaneBytes * (verify ? kVerifyW : kStoreW);
      const size_t tiles = (job.len + tile - 1) / tile;
      const int per_stripe = kc + mc;
      int stripes_per_launch = kPtrSlots / per_stripe;
      // one launch covers tiles * stripes workgroups: keep that in a 32-bit grid
      stripes_per_launch = (int)std::min<size_t>(stripes_per_launch, std::max<size_t>(1, 0x7fffffffu / tiles));
      if (tiles > 0x7fffffffu) return hipErrorInvalidValue;
      for (int s0 = 0; s0 < job.nstripes; s0 += stripes_per_launch) {
        const int ns = std::min(stripes_per_launch, job.nstripes - s0);
        a.len = job.len;
        a.k = (uint32_t)kc;
        a.m = (uint32_t)mc;
        a.nstripes = (uint32_t)ns;
        a.tiles_per_stripe = (uint32_t)tiles;
        a.flags = job.flags ? job.flags + s0 : nullptr;
        for (int r = 0; r < mc; ++r)
          for (int c = 0; c < kc; ++c)
            a.coef[r * kc + c] = job.coef[(size_t)(r0 + r) * job.k + (c0 + c)];
        for (int s = 0; s < ns; ++s) {
          for (int c = 0; c < kc; ++c)
            a.ptr[s * kc + c] = job.in[(size_t)(s0 + s) * job.k + c0 + c];
          for (int r = 0; r < mc; ++r)
            a.ptr[ns * kc + s * mc + r] = job.out[(size_t)(s0 + s) * job.m + r0 + r];
        }
        const dim3 grid((unsigned)(tiles * ns));
        const int mpad = pad_outputs(mc);
        hipError_t e;
        switch (mode) {
          case MatVecMode::kStore: e = launch_mode<MatVecMode::kStore>(mpad, a, grid, threads, stream); break;
          case MatVecMode::kAccum: e = launch_mode<MatVecMode::kAccum>(mpad, a, grid, threads, stream); break;
          default: e = launch_mode<MatVecMode::kVerify>(mpad, a, grid, threads, stream); break;
        }
        if (e != hipSuccess) return e;
      }
    }
  }
  return hipSuccess;
}

}  // namespace cfsec
