// bs_probe.hip -- bit-sliced EC16P20L2 parity (dev probe, round 4).
//
// The 22 parity rows of EC16P20L2 (20 global + 2 AZ-local, over the 16 data rows) from the
// generated XOR network (chubaofs_amd/csrc/bs_net_ec16p20l2.hpp): each lane holds 32 bytes of
// every data row as 8 bit planes (an 8x8 bit transpose per byte lane: 3 swap stages), runs the
// network row by row and transposes each output row back.  Same tasklet shape as the library's
// EC16P20L2 fused encode in tools/gf_shapes (64 stripes x S = 262,144), three batches in rotation;
// stripe 0 and stripe 63 checked against a scalar GF product on the host.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../chubaofs_amd/csrc bs_probe.hip \
//         -L../chubaofs_amd -lcfsec -Wl,-rpath,'$ORIGIN/../chubaofs_amd' -o bs_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "bs_net_ec16p20l2.hpp"
#include "kernels.hpp"

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

constexpr int K = 16, M = 22, ROWS = K + M, NB = 64, NT = 3;
constexpr size_t S = 262144;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void swapmove(uint32_t& a, uint32_t& b, int s, uint32_t m) {
  const uint32_t t = ((a >> s) ^ b) & m;
  b ^= t;
  a ^= t << s;
}

// 8 dwords (32 bytes) <-> 8 bit planes; an involution
__device__ __forceinline__ void transpose8(uint32_t* w) {
#pragma unroll
  for (int i = 0; i < 8; i += 2) swapmove(w[i], w[i + 1], 1, 0x55555555u);
#pragma unroll
  for (int i = 0; i < 8; ++i)
    if (!(i & 2)) swapmove(w[i], w[i + 2], 2, 0x33333333u);
#pragma unroll
  for (int i = 0; i < 4; ++i) swapmove(w[i], w[i + 4], 4, 0x0F0F0F0Fu);
}

// the network header's input basis (tools/gen_bs_net.py --paired): even rows' planes hold the pair's XOR
__device__ __forceinline__ void pair_basis(uint32_t* x) {
  if constexpr (cfsec::dev::kBsEc16p20l2Paired)
    for (int c = 0; c < K; c += 2)
      for (int j = 0; j < 8; ++j) x[8 * c + j] ^= x[8 * (c + 1) + j];
}

__device__ __forceinline__ u32x4 ld16nt(const uint8_t* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
}
__device__ __forceinline__ void st16nt(uint8_t* p, u32x4 v) {
  __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
}

template <int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void bs_encode(uint8_t* base) {
  const uint32_t stripe = blockIdx.y;
  const size_t off = ((size_t)blockIdx.x * 256 + threadIdx.x) * 32;
  uint8_t* row0 = base + (size_t)stripe * ROWS * S;
  uint32_t x[128];
#pragma unroll
  for (int c = 0; c < K; ++c) {
    const u32x4 a = ld16nt(row0 + c * S + off), b = ld16nt(row0 + c * S + off + 16);
    x[8 * c + 0] = a.x; x[8 * c + 1] = a.y; x[8 * c + 2] = a.z; x[8 * c + 3] = a.w;
    x[8 * c + 4] = b.x; x[8 * c + 5] = b.y; x[8 * c + 6] = b.z; x[8 * c + 7] = b.w;
  }
#pragma unroll
  for (int c = 0; c < K; ++c) transpose8(&x[8 * c]);
  pair_basis(x);
  cfsec::dev::bs_net_ec16p20l2(x, [&](int r, uint32_t (&o)[8]) {
    transpose8(o);
    uint8_t* p = row0 + (size_t)(K + r) * S + off;
    st16nt(p, u32x4{o[0], o[1], o[2], o[3]});
    st16nt(p + 16, u32x4{o[4], o[5], o[6], o[7]});
  });
}

// Persistent form: one wave per SIMD (216 VGPRs), every wave prefetching its next tile's 16 input
// rows straight into its own 32 KiB of LDS (global_load_lds_dwordx4, no VGPRs) while the network
// runs on the current tile; the lane's 32 bytes of a row are bytes [16 lane, +16) and
// [1024 + 16 lane, +16) of the wave's 2 KiB (each load instruction a contiguous 1 KiB).
constexpr int kWaveTileBytes = 2048;
__device__ __forceinline__ void glds16(const uint8_t* g, uint8_t* l) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}
constexpr unsigned waitcnt_vm(unsigned n) { return (n & 0xFu) | (0x7u << 4) | (0xFu << 8) | ((n >> 4) << 14); }

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void bs_encode_glds(uint8_t* base, uint32_t ntiles) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[4][K * kWaveTileBytes];
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint8_t* my = lds[wave];
  const uint32_t tiles_per_stripe = (uint32_t)(S / kWaveTileBytes);
  const uint32_t gw = blockIdx.x * 4 + wave, nw = gridDim.x * 4;
  const auto prefetch = [&](uint32_t t) {
    const uint32_t stripe = t / tiles_per_stripe;
    const size_t off = (size_t)(t % tiles_per_stripe) * kWaveTileBytes + lane * 16;
    const uint8_t* row0 = base + (size_t)stripe * ROWS * S;
#pragma unroll
    for (int c = 0; c < K; ++c) {
      glds16(row0 + c * S + off, my + c * kWaveTileBytes);
      glds16(row0 + c * S + off + 1024, my + c * kWaveTileBytes + 1024);
    }
  };
  uint32_t t = gw;
  if (t < ntiles) prefetch(t);
  __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));  // the first tile: nothing else in flight
  for (; t < ntiles; t += nw) {
    // this tile's 32 loads, issued before the previous tile's 44 stores (vmcnt retires in order):
    // those stores may still fly
    __builtin_amdgcn_s_waitcnt(waitcnt_vm(44));
    uint32_t x[128];
#pragma unroll
    for (int c = 0; c < K; ++c) {
      const u32x4 a = *reinterpret_cast<const u32x4*>(my + c * kWaveTileBytes + lane * 16);
      const u32x4 b = *reinterpret_cast<const u32x4*>(my + c * kWaveTileBytes + 1024 + lane * 16);
      x[8 * c + 0] = a.x; x[8 * c + 1] = a.y; x[8 * c + 2] = a.z; x[8 * c + 3] = a.w;
      x[8 * c + 4] = b.x; x[8 * c + 5] = b.y; x[8 * c + 6] = b.z; x[8 * c + 7] = b.w;
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the tile is in registers before the buffer is refilled
    if (t + nw < ntiles) prefetch(t + nw);
    const uint32_t stripe = t / tiles_per_stripe;
    const size_t off = (size_t)(t % tiles_per_stripe) * kWaveTileBytes + lane * 16;
    uint8_t* row0 = base + (size_t)stripe * ROWS * S;
#pragma unroll
    for (int c = 0; c < K; ++c) transpose8(&x[8 * c]);
    pair_basis(x);
    cfsec::dev::bs_net_ec16p20l2(x, [&](int r, uint32_t (&o)[8]) {
      transpose8(o);
      uint8_t* p = row0 + (size_t)(K + r) * S + off;
      st16nt(p, u32x4{o[0], o[1], o[2], o[3]});
      st16nt(p + 1024, u32x4{o[4], o[5], o[6], o[7]});
    });
  }
}

// Two waves per SIMD: 8 waves per workgroup, 16 KiB of LDS each -- data rows 0-7 of the next tile
// are prefetched into LDS (global_load_lds) while the network runs, rows 8-15 are loaded into
// registers at the top of the tile (the other wave on the SIMD computes meanwhile).
constexpr int kHalfRows = 8;
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void bs_encode_glds2(uint8_t* base, uint32_t ntiles) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[8][kHalfRows * kWaveTileBytes];
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint8_t* my = lds[wave];
  const uint32_t tiles_per_stripe = (uint32_t)(S / kWaveTileBytes);
  const uint32_t gw = blockIdx.x * 8 + wave, nw = gridDim.x * 8;
  const auto where = [&](uint32_t t, const uint8_t*& row0, size_t& off) {
    row0 = base + (size_t)(t / tiles_per_stripe) * ROWS * S;
    off = (size_t)(t % tiles_per_stripe) * kWaveTileBytes + lane * 16;
  };
  const auto prefetch = [&](uint32_t t) {
    const uint8_t* row0;
    size_t off;
    where(t, row0, off);
#pragma unroll
    for (int c = 0; c < kHalfRows; ++c) {
      glds16(row0 + c * S + off, my + c * kWaveTileBytes);
      glds16(row0 + c * S + off + 1024, my + c * kWaveTileBytes + 1024);
    }
  };
  uint32_t t = gw;
  if (t < ntiles) prefetch(t);
  __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
  for (; t < ntiles; t += nw) {
    const uint8_t* row0c;
    size_t off;
    where(t, row0c, off);
    uint8_t* row0 = const_cast<uint8_t*>(row0c);
    uint32_t x[128];
#pragma unroll
    for (int c = kHalfRows; c < K; ++c) {
      const u32x4 a = ld16nt(row0 + c * S + off), b = ld16nt(row0 + c * S + off + 1024);
      x[8 * c + 0] = a.x; x[8 * c + 1] = a.y; x[8 * c + 2] = a.z; x[8 * c + 3] = a.w;
      x[8 * c + 4] = b.x; x[8 * c + 5] = b.y; x[8 * c + 6] = b.z; x[8 * c + 7] = b.w;
    }
    // the prefetched rows: issued before the previous tile's 44 stores and these 16 loads
    __builtin_amdgcn_s_waitcnt(waitcnt_vm(60));
#pragma unroll
    for (int c = 0; c < kHalfRows; ++c) {
      const u32x4 a = *reinterpret_cast<const u32x4*>(my + c * kWaveTileBytes + lane * 16);
      const u32x4 b = *reinterpret_cast<const u32x4*>(my + c * kWaveTileBytes + 1024 + lane * 16);
      x[8 * c + 0] = a.x; x[8 * c + 1] = a.y; x[8 * c + 2] = a.z; x[8 * c + 3] = a.w;
      x[8 * c + 4] = b.x; x[8 * c + 5] = b.y; x[8 * c + 6] = b.z; x[8 * c + 7] = b.w;
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
#pragma unroll
    for (int c = 0; c < kHalfRows; ++c) transpose8(&x[8 * c]);
#pragma unroll
    for (int c = kHalfRows; c < K; ++c) transpose8(&x[8 * c]);
    pair_basis(x);
    __builtin_amdgcn_sched_barrier(0);
    prefetch(t + nw < ntiles ? t + nw : t);  // branch-free (the last tile re-reads itself): no code sinks past it
    __builtin_amdgcn_sched_barrier(0);
    cfsec::dev::bs_net_ec16p20l2(x, [&](int r, uint32_t (&o)[8]) {
      transpose8(o);
      uint8_t* p = row0 + (size_t)(K + r) * S + off;
      st16nt(p, u32x4{o[0], o[1], o[2], o[3]});
      st16nt(p + 1024, u32x4{o[4], o[5], o[6], o[7]});
    });
  }
}

__global__ void fill(uint32_t* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t v = (uint32_t)i * 2654435761u ^ seed;
    v ^= v >> 15; v *= 0x2c1b3c6du; v ^= v >> 12;
    p[i] = v;
  }
}

static uint8_t gmul(uint8_t a, uint8_t b) {
  uint8_t p = 0;
  while (b) {
    if (b & 1) p ^= a;
    a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1D : 0));
    b >>= 1;
  }
  return p;
}

template <int WPE>
static double run(std::vector<uint8_t*>& bufs, int reps) {
  const dim3 grid((unsigned)(S / (256 * 32)), NB);
  for (int i = 0; i < 6; ++i) hipLaunchKernelGGL((bs_encode<WPE>), grid, dim3(256), 0, 0, bufs[i % NT]);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((bs_encode<WPE>), grid, dim3(256), 0, 0, bufs[i % NT]);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3 / reps;
}

static double run_glds(std::vector<uint8_t*>& bufs, int reps, int& grid_out) {
  int dev = 0, ncu = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const uint32_t ntiles = (uint32_t)(NB * (S / kWaveTileBytes));
  grid_out = ncu;
  for (int i = 0; i < 6; ++i) hipLaunchKernelGGL(bs_encode_glds, dim3(ncu), dim3(256), 0, 0, bufs[i % NT], ntiles);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(bs_encode_glds, dim3(ncu), dim3(256), 0, 0, bufs[i % NT], ntiles);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3 / reps;
}

static double run_glds2(std::vector<uint8_t*>& bufs, int reps) {
  int dev = 0, ncu = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const uint32_t ntiles = (uint32_t)(NB * (S / kWaveTileBytes));
  for (int i = 0; i < 6; ++i) hipLaunchKernelGGL(bs_encode_glds2, dim3(ncu), dim3(512), 0, 0, bufs[i % NT], ntiles);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(bs_encode_glds2, dim3(ncu), dim3(512), 0, 0, bufs[i % NT], ntiles);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3 / reps;
}

static long check(uint8_t* buf) {
  std::vector<uint8_t> h((size_t)ROWS * S);
  long bad = 0;
  for (int st : {0, NB / 2, NB - 1}) {
    CK(hipMemcpy(h.data(), buf + (size_t)st * ROWS * S, h.size(), hipMemcpyDeviceToHost));
    for (int r = 0; r < M; ++r)
      for (size_t i = 0; i < S; ++i) {
        uint8_t v = 0;
        for (int c = 0; c < K; ++c) v ^= gmul(cfsec::dev::kBsEc16p20l2Rows[r][c], h[(size_t)c * S + i]);
        if (v != h[(size_t)(K + r) * S + i] && bad++ < 5)
          printf("mismatch stripe %d row %d byte %zu: %02x vs %02x\n", st, r, i, h[(size_t)(K + r) * S + i], v);
      }
  }
  return bad;
}

int main() {
  std::vector<uint8_t*> bufs(NT);
  const size_t bytes = (size_t)NB * ROWS * S;
  for (int t = 0; t < NT; ++t) {
    CK(hipMalloc(&bufs[t], bytes));
    fill<<<4096, 256>>>((uint32_t*)bufs[t], bytes / 4, 0x9E3779B9u * (t + 1));
  }
  CK(hipDeviceSynchronize());
  // correctness: every parity byte of stripes 0, NB/2 and NB-1, both kernels
  const dim3 grid((unsigned)(S / (256 * 32)), NB);
  hipLaunchKernelGGL((bs_encode<2>), grid, dim3(256), 0, 0, bufs[0]);
  CK(hipDeviceSynchronize());
  long bad = check(bufs[0]);
  CK(hipMemset(bufs[1], 0, 0));
  int g = 0;
  run_glds(bufs, 1, g);
  for (int t = 0; t < NT; ++t) bad += check(bufs[t]);
  for (int t = 0; t < NT; ++t) CK(hipMemset(bufs[t] + (size_t)K * S, 0, (size_t)M * S));  // stripe 0's parity
  run_glds2(bufs, 1);
  for (int t = 0; t < NT; ++t) bad += check(bufs[t]);
  printf("parity check: %s (%ld bad bytes)\n", bad ? "FAIL" : "ok", bad);
  if (bad) return 1;
  const double algo = (double)NB * ROWS * S;
  // the shipped launcher on the same tasklets (CFSEC_BS16 chooses its route)
  std::vector<std::vector<const uint8_t*>> lin(NT);
  std::vector<std::vector<uint8_t*>> lout(NT);
  std::vector<cfsec::MatVecJob> jobs(NT);
  for (int t = 0; t < NT; ++t) {
    for (int b = 0; b < NB; ++b) {
      for (int c = 0; c < K; ++c) lin[t].push_back(bufs[t] + ((size_t)b * ROWS + c) * S);
      for (int r = 0; r < M; ++r) lout[t].push_back(bufs[t] + ((size_t)b * ROWS + K + r) * S);
    }
    cfsec::MatVecJob& j = jobs[t];
    j.k = K;
    j.m = M;
    j.coef = &cfsec::dev::kBsEc16p20l2Rows[0][0];
    j.len = S;
    j.nstripes = NB;
    j.in = lin[t].data();
    j.out = lout[t].data();
  }
  const auto run_lib = [&](int reps) {
    for (int i = 0; i < 6; ++i) CK(cfsec::launch_matvec(jobs[i % NT], 0));
    CK(hipDeviceSynchronize());
    hipEvent_t a0, a1;
    CK(hipEventCreate(&a0));
    CK(hipEventCreate(&a1));
    CK(hipEventRecord(a0, 0));
    for (int i = 0; i < reps; ++i) CK(cfsec::launch_matvec(jobs[i % NT], 0));
    CK(hipEventRecord(a1, 0));
    CK(hipEventSynchronize(a1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a0, a1));
    return ms * 1e3 / reps;
  };
  {
    for (int t = 0; t < NT; ++t) CK(hipMemset(bufs[t] + (size_t)K * S, 0, (size_t)M * S));
    run_lib(1);
    CK(hipDeviceSynchronize());
    long lb = 0;
    for (int t = 0; t < NT; ++t) lb += check(bufs[t]);
    printf("library launcher parity: %s (CFSEC_BS16=%s)\n", lb ? "FAIL" : "ok", getenv("CFSEC_BS16") ? getenv("CFSEC_BS16") : "default");
    if (lb) return 1;
  }
  for (int rep = 0; rep < 2; ++rep) {
    double us = run<2>(bufs, 30);
    printf("bs_encode 16->22 waves/EU 2: %8.1f us  %6.1f GB/s  %5.1f %% of 8 TB/s\n", us, algo / us / 1e3, algo / us / 8e4);
    us = run<1>(bufs, 30);
    printf("bs_encode 16->22 waves/EU 1: %8.1f us  %6.1f GB/s  %5.1f %% of 8 TB/s\n", us, algo / us / 1e3, algo / us / 8e4);
    us = run_glds(bufs, 30, g);
    printf("bs_encode_glds (%d x 256, LDS prefetch): %8.1f us  %6.1f GB/s  %5.1f %% of 8 TB/s\n", g, us, algo / us / 1e3, algo / us / 8e4);
    us = run_glds2(bufs, 30);
    printf("bs_encode_glds2 (8 waves, half LDS prefetch): %8.1f us  %6.1f GB/s  %5.1f %% of 8 TB/s\n", us, algo / us / 1e3, algo / us / 8e4);
    us = run_lib(30);
    printf("library launch_matvec (22 x 16, CFSEC_BS16=%s): %8.1f us  %6.1f GB/s  %5.1f %% of 8 TB/s\n",
           getenv("CFSEC_BS16") ? getenv("CFSEC_BS16") : "1", us, algo / us / 1e3, algo / us / 8e4);
  }
  return 0;
}
