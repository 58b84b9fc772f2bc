// rot_probe.hip -- HBM-honest A/B of the EC12P4 step kernel (dev tool, profiles/r02/rot_probe.txt).
//
// Every variant is timed over THREE 8-stripe batches in rotation (launch i codes batch i % 3), as
// bench.py's step does, so no launch finds its inputs in the 256 MB Infinity Cache.  Variants: the
// shipped launcher, the dyadic kernel with other store / load cache policies, and ceilings of the
// access pattern: the same 12-read / 4-write tiling with trivial arithmetic, a 16-row read-only
// pass, and a flat float4 copy.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../chubaofs_amd/csrc rot_probe.hip \
//         -L../chubaofs_amd -lcfsec -Wl,-rpath,'$ORIGIN/../chubaofs_amd' -o rot_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <functional>
#include <string>
#include <vector>

#include "gf256.hpp"
#include "gf_dyadic.hpp"
#include "kernels.hpp"

using namespace cfsec;
using dev::GfArgs;
using dev::u32x4;

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

constexpr int K = 12, M = 4, B = 4, NB = 3, NST = 8;
constexpr size_t S = 5592406;

template <int SP, int LP = -1, bool PIN = true>
__global__ __launch_bounds__(256) void kdy(const GfArgs a) {
  dev::matvec_dy<K, M, B, MatVecMode::kStore, true, true, 64, 0, PIN, SP, LP>(a);
}

// trivial arithmetic, same tiling: out r = in[3r] ^ in[3r+1] ^ in[3r+2]; all 12 loads issued first
template <int SP>
__global__ __launch_bounds__(256) void ktriv(const GfArgs a) {
  const uint32_t stripe = blockIdx.y, tile = blockIdx.x;
  const int64_t sbase = (int64_t)stripe * a.sstride;
  const uint32_t off = tile * 4096u + threadIdx.x * 16u;
  if ((uint64_t)off + 16 > a.len) return;
  u32x4 x[K];
#pragma unroll
  for (int c = 0; c < K; ++c) x[c] = dev::ld16<true>(a.ptr[c] + sbase + off);
#pragma unroll
  for (int r = 0; r < M; ++r) {
    u32x4 v = x[3 * r] ^ x[3 * r + 1] ^ x[3 * r + 2];
    uint8_t* p = const_cast<uint8_t*>(a.ptr[K + r]) + sbase + off;
    if constexpr (SP >= 0) dev::st16_pol<SP>(p, v);
    else dev::st16<true>(p, v);
  }
}

// trivial arithmetic with W 16-B chunks per lane per row (chunk w at w*1 KiB inside the wave's
// run: each wave streams W KiB of every row), ORD 0: grid (tiles, stripes); ORD 1: stripes fastest
template <int W, int ORD, int SP = 1>
__global__ __launch_bounds__(256) void ktrivw(const GfArgs a) {
  const uint32_t stripe = ORD ? blockIdx.x % a.nstripes : blockIdx.y;
  const uint32_t tile = ORD ? blockIdx.x / a.nstripes : blockIdx.x;
  const int64_t sbase = (int64_t)stripe * a.sstride;
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t off = tile * (4096u * W) + wave * (1024u * W) + lane * 16u;
  if ((uint64_t)off + 1024u * (W - 1) + 16 > a.len) return;
  u32x4 x[K][W];
#pragma unroll
  for (int c = 0; c < K; ++c)
#pragma unroll
    for (int w = 0; w < W; ++w) x[c][w] = dev::ld16<true>(a.ptr[c] + sbase + off + 1024u * w);
#pragma unroll
  for (int r = 0; r < M; ++r)
#pragma unroll
    for (int w = 0; w < W; ++w) {
      u32x4 v = x[3 * r][w] ^ x[3 * r + 1][w] ^ x[3 * r + 2][w];
      dev::st16_pol<SP>(const_cast<uint8_t*>(a.ptr[K + r]) + sbase + off + 1024u * w, v);
    }
}

// trivial arithmetic, W chunks per lane walked one after the other (one chunk's 12 loads in flight
// at a time): the W-KiB-per-wave footprint of ktrivw without its simultaneity
template <int W>
__global__ __launch_bounds__(256) void ktrivs(const GfArgs a) {
  const uint32_t stripe = blockIdx.y, tile = blockIdx.x;
  const int64_t sbase = (int64_t)stripe * a.sstride;
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t off0 = tile * (4096u * W) + wave * (1024u * W) + lane * 16u;
#pragma unroll 1
  for (int w = 0; w < W; ++w) {
    const uint32_t off = off0 + 1024u * w;
    if ((uint64_t)off + 16 > a.len) return;
    u32x4 x[K];
#pragma unroll
    for (int c = 0; c < K; ++c) x[c] = dev::ld16<true>(a.ptr[c] + sbase + off);
#pragma unroll
    for (int r = 0; r < M; ++r)
      dev::st16_pol<1>(const_cast<uint8_t*>(a.ptr[K + r]) + sbase + off, x[3 * r] ^ x[3 * r + 1] ^ x[3 * r + 2]);
  }
}

// persistent: gridDim.x workgroups walk (stripe, tile) pairs; XCD-contiguous runs (block b runs on
// XCD b % 8: XCD x takes the x-th eighth of the work)
__global__ __launch_bounds__(256) void ktrivp(const GfArgs a, uint32_t ntiles) {
  const uint32_t total = ntiles * a.nstripes;
  const uint32_t nb = gridDim.x, per = (total + 7) / 8;
  const uint32_t x = blockIdx.x % 8, q = blockIdx.x / 8, nq = nb / 8;
  for (uint32_t t = x * per + q; t < (x + 1) * per && t < total; t += nq) {
    const uint32_t stripe = t / ntiles, tile = t % ntiles;
    const int64_t sbase = (int64_t)stripe * a.sstride;
    const uint32_t off = tile * 4096u + threadIdx.x * 16u;
    if ((uint64_t)off + 16 > a.len) continue;
    u32x4 xv[K];
#pragma unroll
    for (int c = 0; c < K; ++c) xv[c] = dev::ld16<true>(a.ptr[c] + sbase + off);
#pragma unroll
    for (int r = 0; r < M; ++r)
      dev::st16_pol<1>(const_cast<uint8_t*>(a.ptr[K + r]) + sbase + off, xv[3 * r] ^ xv[3 * r + 1] ^ xv[3 * r + 2]);
  }
}

// read all 16 rows, fold into one flag (what verify's memory traffic is)
__global__ __launch_bounds__(256) void kread16(const GfArgs a) {
  const uint32_t stripe = blockIdx.y, tile = blockIdx.x;
  const int64_t sbase = (int64_t)stripe * a.sstride;
  const uint32_t off = tile * 4096u + threadIdx.x * 16u;
  if ((uint64_t)off + 16 > a.len) return;
  u32x4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int c = 0; c < K + M; ++c) acc ^= dev::ld16<true>(a.ptr[c] + sbase + off);
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) atomicOr(a.flags, 1u);
}

// flat copy: first 12 rows' bytes -> next region (same byte count as 12r4w is not the point; this
// is the device's 1:1 streaming ceiling)
__global__ __launch_bounds__(256) void kcopy(const u32x4* __restrict__ src, u32x4* __restrict__ dst, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

__global__ void fill(uint32_t* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t z = ((uint64_t)i + seed) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    p[i] = (uint32_t)(z ^ (z >> 31));
  }
}

int main() {
  const size_t pitch = (S + 255) / 256 * 256;
  const size_t per = pitch * (K + M) * NST;
  std::vector<uint8_t*> buf(NB);
  for (int b = 0; b < NB; ++b) {
    CK(hipMalloc(&buf[b], per));
    fill<<<4096, 256>>>((uint32_t*)buf[b], per / 4, 77u * b);
  }
  uint32_t* flag;
  CK(hipMalloc(&flag, 64));
  Matrix mat;
  build_matrix(K, K + M, mat);
  std::vector<uint8_t> coef((size_t)M * K);
  for (int r = 0; r < M; ++r)
    for (int c = 0; c < K; ++c) coef[(size_t)r * K + c] = mat.at(K + r, c);
  std::vector<GfArgs> args(NB);
  std::vector<MatVecJob> jobs(NB);
  std::vector<std::vector<const uint8_t*>> ins(NB);
  std::vector<std::vector<uint8_t*>> outs(NB);
  for (int b = 0; b < NB; ++b) {
    for (int s = 0; s < NST; ++s) {
      for (int c = 0; c < K; ++c) ins[b].push_back(buf[b] + ((size_t)s * (K + M) + c) * pitch);
      for (int r = 0; r < M; ++r) outs[b].push_back(buf[b] + ((size_t)s * (K + M) + K + r) * pitch);
    }
    MatVecJob& j = jobs[b];
    j.k = K;
    j.m = M;
    j.coef = coef.data();
    j.len = S;
    j.nstripes = NST;
    j.in = ins[b].data();
    j.out = outs[b].data();
    GfArgs& a = args[b];
    a = GfArgs{};
    a.len = S;
    a.k = K;
    a.m = M;
    a.nstripes = NST;
    a.tab = 1;
    a.sstride = (int64_t)(pitch * (K + M));
    a.flags = flag;
    for (size_t i = 0; i < coef.size(); ++i) a.coef[i] = coef[i];
    for (int c = 0; c < K; ++c) a.ptr[c] = ins[b][c];
    for (int r = 0; r < M; ++r) a.ptr[K + r] = outs[b][r];
  }
  const dim3 grid((unsigned)((S + 4095) / 4096), NST);
  const unsigned nt1 = (unsigned)((S + 4095) / 4096);
  struct Var {
    std::string name;
    std::function<void(int)> run;
    double bytes;  // per launch
  };
  const double step_bytes = double(K + M) * S * NST;
  std::vector<Var> vs;
  vs.push_back({"shipped launcher (dy, st sc1)", [&](int b) { CK(launch_matvec(jobs[b], 0)); }, step_bytes});
  vs.push_back({"dy st nt", [&](int b) { hipLaunchKernelGGL(kdy<1>, grid, dim3(256), 0, 0, args[b]); }, step_bytes});
  vs.push_back({"dy st sc1", [&](int b) { hipLaunchKernelGGL(kdy<2>, grid, dim3(256), 0, 0, args[b]); }, step_bytes});
  vs.push_back({"dy st nt sc1", [&](int b) { hipLaunchKernelGGL(kdy<4>, grid, dim3(256), 0, 0, args[b]); }, step_bytes});
  vs.push_back({"triv 12r4w st nt", [&](int b) { hipLaunchKernelGGL(ktriv<1>, grid, dim3(256), 0, 0, args[b]); }, step_bytes});
  vs.push_back({"triv 12r4w st sc1", [&](int b) { hipLaunchKernelGGL(ktriv<2>, grid, dim3(256), 0, 0, args[b]); }, step_bytes});
  vs.push_back({"triv W2 (8 KiB/row/wg)", [&](int b) { hipLaunchKernelGGL((ktrivw<2, 0>), dim3((nt1 + 1) / 2, NST), dim3(256), 0, 0, args[b]); }, step_bytes});
  vs.push_back({"triv W4 (16 KiB/row/wg)", [&](int b) { hipLaunchKernelGGL((ktrivw<4, 0>), dim3((nt1 + 3) / 4, NST), dim3(256), 0, 0, args[b]); }, step_bytes});
  vs.push_back({"triv seq W2", [&](int b) { hipLaunchKernelGGL((ktrivs<2>), dim3((nt1 + 1) / 2, NST), dim3(256), 0, 0, args[b]); }, step_bytes});
  vs.push_back({"triv seq W4", [&](int b) { hipLaunchKernelGGL((ktrivs<4>), dim3((nt1 + 3) / 4, NST), dim3(256), 0, 0, args[b]); }, step_bytes});
  vs.push_back({"triv seq W8", [&](int b) { hipLaunchKernelGGL((ktrivs<8>), dim3((nt1 + 7) / 8, NST), dim3(256), 0, 0, args[b]); }, step_bytes});
  vs.push_back({"triv W1 stripes fastest", [&](int b) { hipLaunchKernelGGL((ktrivw<1, 1>), dim3(nt1 * NST), dim3(256), 0, 0, args[b]); }, step_bytes});
  vs.push_back({"triv persistent 2048 wg xcd", [&](int b) { hipLaunchKernelGGL(ktrivp, dim3(2048), dim3(256), 0, 0, args[b], nt1); }, step_bytes});
  vs.push_back({"read 16 rows", [&](int b) { hipLaunchKernelGGL(kread16, grid, dim3(256), 0, 0, args[b]); }, step_bytes});
  const size_t half = per / 2 / 16;
  vs.push_back({"flat copy (nt) half->half",
                [&](int b) {
                  hipLaunchKernelGGL(kcopy, dim3(8192), dim3(256), 0, 0, (const u32x4*)buf[b], (u32x4*)(buf[b] + per / 2), half);
                },
                double(per)});
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int j = 0; j < 300; ++j) vs[0].run(j % NB);  // clocks up
  CK(hipDeviceSynchronize());
  std::vector<std::vector<float>> t(vs.size());
  for (int rnd = 0; rnd < 12; ++rnd)
    for (size_t i = 0; i < vs.size(); ++i) {
      for (int j = 0; j < 3; ++j) vs[i].run(j % NB);
      CK(hipEventRecord(e0, 0));
      for (int j = 0; j < 30; ++j) vs[i].run(j % NB);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[i].push_back(ms / 30);
    }
  printf("EC12P4 8 x 64 MiB-blob stripes per launch, 3 batches rotated (no Infinity-Cache reuse)\n");
  for (size_t i = 0; i < vs.size(); ++i) {
    std::sort(t[i].begin(), t[i].end());
    const double med = t[i][t[i].size() / 2];
    printf("%-34s median %8.1f us  %7.1f GB/s  %6.1f%% of 8 TB/s\n", vs[i].name.c_str(), med * 1e3,
           vs[i].bytes / (med * 1e-3) / 1e9, 100 * vs[i].bytes / (med * 1e-3) / 8e12);
  }
  return 0;
}
