// gf_bs16.hip -- the EC16P20 / EC16P20L2 parity as a bit-sliced XOR network (gf_bitslice.hpp,
// bs_net_ec16p20l2.hpp): the encodes' whole 2 KiB column runs; the launcher (gf_kernels.hip) sends
// the rest of each row (and every other matrix) to the dyadic kernels.
//
// Persistent waves, 8 per CU (2 per SIMD at <= 256 VGPRs: the 128 input planes of a 32-byte column
// stay in registers).  While a wave runs the network on its tile, data rows 0-7 of its next tile
// are copied into its 16 KiB of LDS by global_load_lds (no VGPRs); rows 8-15 are loaded at the
// tile's top, where the other wave of the SIMD covers their latency.  EC16P20L2's fused encode,
// 64 x 262,144: 131.9 us against 148.6 us for the 16x16-dyadic v_perm kernel (profiles/r04/
// bs_probe.txt); it issues ~40 % fewer VALU instructions at 2 instead of 4 waves per SIMD.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "bs_net_ec16p20l2.hpp"
#include "gf_bitslice.hpp"
#include "gf_launch.hpp"

namespace cfsec {

namespace {
constexpr int kBsK = 16, kBsPrefetch = 8, kBsWaves = 8;

template <int M>
__global__ __launch_bounds__(64 * kBsWaves) __attribute__((amdgpu_waves_per_eu(2, 2))) void gf_bs16_kernel(
    const dev::GfArgs a, uint32_t tiles_per_stripe, uint32_t ntiles) {
  using namespace dev;
  __shared__ __attribute__((aligned(16))) uint8_t lds[kBsWaves][kBsPrefetch * kBsWaveBytes];
  // the wave index as a scalar: tiles, stripes and row pointers are then wave-uniform (scalar loads
  // of the pointer table, no vector memory operations besides the shard copies counted below)
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  uint8_t* pre = lds[wave];
  const uint32_t nw = gridDim.x * kBsWaves;
  // row i of stripe s (inputs 0..15, then outputs), at the lane's first byte of column tile c
  const auto row = [&](uint32_t s, int i, uint32_t c) -> uint8_t* {
    const uint8_t* base;
    if (i < kBsK) base = a.sstride ? a.ptr[i] + (int64_t)s * a.sstride : a.ptr[(size_t)s * kBsK + i];
    else base = a.sstride ? a.ptr[kBsK + (i - kBsK)] + (int64_t)s * a.sstride
                          : a.ptr[(size_t)a.tab * kBsK + (size_t)s * M + (i - kBsK)];
    return const_cast<uint8_t*>(base) + (size_t)c * kBsWaveBytes + lane * 16;
  };
  const auto prefetch = [&](uint32_t t) {
    const uint32_t s = t / tiles_per_stripe, c = t % tiles_per_stripe;
#pragma unroll
    for (int i = 0; i < kBsPrefetch; ++i) bs_glds_row(row(s, i, c), pre + i * kBsWaveBytes);
  };
  uint32_t t = blockIdx.x * kBsWaves + wave;
  if (t >= ntiles) return;  // no barrier in this kernel: idle waves leave at once
  prefetch(t);
  __builtin_amdgcn_s_waitcnt(bs_waitcnt_vm(0));
  for (; t < ntiles; t += nw) {
    const uint32_t s = t / tiles_per_stripe, c = t % tiles_per_stripe;
    uint32_t x[128];
#pragma unroll
    for (int i = kBsPrefetch; i < kBsK; ++i) bs_ld_row(row(s, i, c), &x[8 * i]);
    // the prefetched rows were issued before the previous tile's stores and these 16 loads, and
    // vector memory operations retire in issue order: at most 16 + 2 M may still be in flight
    __builtin_amdgcn_s_waitcnt(bs_waitcnt_vm(2 * (kBsK - kBsPrefetch) + 2 * M > 63 ? 63 : 2 * (kBsK - kBsPrefetch) + 2 * M));
#pragma unroll
    for (int i = 0; i < kBsPrefetch; ++i) bs_lds_row(pre + i * kBsWaveBytes, lane, &x[8 * i]);
    __builtin_amdgcn_s_waitcnt(kBsWaitLgkm0);
#pragma unroll
    for (int i = 0; i < kBsK; ++i) bs_transpose8(&x[8 * i]);
    __builtin_amdgcn_sched_barrier(0);
    prefetch(t + nw < ntiles ? t + nw : t);  // branch-free: nothing sinks below it (the last re-reads)
    __builtin_amdgcn_sched_barrier(0);
    bs_net_ec16p20l2<M>(x, [&](int r, uint32_t (&o)[8]) {
      bs_transpose8(o);
      bs_st_row(row(s, kBsK + r, c), o);
    });
  }
}

int cu_count() {
  static int n[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!n[dev]) {
    int v = 0;
    n[dev] = hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0 ? v : 256;
  }
  return n[dev];
}
}  // namespace

bool bs16_matches(const uint8_t* coef, int m, int k) {
  if (k != 16 || (m != 20 && m != 22)) return false;
  for (int r = 0; r < m; ++r)
    for (int c = 0; c < 16; ++c)
      if (coef[(size_t)r * 16 + c] != dev::kBsEc16p20l2Rows[r][c]) return false;
  return true;
}

hipError_t launch_bs16(int m, const dev::GfArgs& a, unsigned ns, uint64_t len, hipStream_t st) {
  const uint32_t tps = (uint32_t)(len / dev::kBsWaveBytes);
  const uint64_t ntiles = (uint64_t)tps * ns;
  if (tps == 0 || ntiles > 0xFFFFFFFFull || (len % dev::kBsWaveBytes)) return hipErrorInvalidValue;
  const unsigned grid = (unsigned)std::min<uint64_t>((uint64_t)cu_count(), (ntiles + kBsWaves - 1) / kBsWaves);
  switch (m) {
    case 20: hipLaunchKernelGGL(gf_bs16_kernel<20>, dim3(grid), dim3(64 * kBsWaves), 0, st, a, tps, (uint32_t)ntiles); break;
    case 22: hipLaunchKernelGGL(gf_bs16_kernel<22>, dim3(grid), dim3(64 * kBsWaves), 0, st, a, tps, (uint32_t)ntiles); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace cfsec
