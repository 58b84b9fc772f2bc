// c4l_pattern_probe.hip -- rot_probe.hip's method for C4's AZ-local repair shape (dev tool, round 5):
// k = 8 inputs, m = 1 output, 48 stripes of 699,051 B per launch, 3 batches rotated: the shipped
// launcher against the same 8-read / 1-write pattern with trivial arithmetic (XOR of the 8 rows) at
// 1 / 2 / 4 chunks per lane, walked at once or one after the other, and a flat copy.
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
#include <cstring>
#include <cstdio>
#include <functional>
#include <string>
#include <vector>

#include "gf256.hpp"
#include "gf_device.hpp"
#include "gf_fixed.hpp"
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

constexpr int K = 8, M = 1, NB = 3, NST = 48;
constexpr size_t S = 699051;

__device__ __forceinline__ u32x4 xor_all(const u32x4 (&x)[K]) {
  u32x4 v = x[0];
#pragma unroll
  for (int c = 1; c < K; ++c) v ^= x[c];
  return v;
}
template <int W>
__device__ __forceinline__ u32x4 xor_w(const u32x4 (&x)[K][W], int w) {
  u32x4 v = x[0][w];
#pragma unroll
  for (int c = 1; c < K; ++c) v ^= x[c][w];
  return v;
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
    u32x4 v = xor_all(x);
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
      u32x4 v = xor_w(x, w);
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
      dev::st16_pol<1>(const_cast<uint8_t*>(a.ptr[K + r]) + sbase + off, xor_all(x));
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
      dev::st16_pol<1>(const_cast<uint8_t*>(a.ptr[K + r]) + sbase + off, xor_all(xv));
  }
}

// the fixed-K tile with its product tables in registers: the host packs each coefficient's tables
// (t01 = 4 words, t2 = 1 word) into the argument block's coef area, no LDS build and no barrier
template <int D>
__global__ __launch_bounds__(256) void kregtab(const GfArgs a) {
  const uint32_t* kw = reinterpret_cast<const uint32_t*>(a.coef);
  u32x4 t01[K];
  uint32_t t2[K];
#pragma unroll
  for (int c = 0; c < K; ++c) {
    t01[c] = u32x4{kw[5 * c], kw[5 * c + 1], kw[5 * c + 2], kw[5 * c + 3]};
    t2[c] = kw[5 * c + 4];
  }
  const uint32_t stripe = blockIdx.y, tile = blockIdx.x;
  const int64_t sbase = (int64_t)stripe * a.sstride;
  const uint8_t* const* in = a.ptr;
  uint8_t* const* out = const_cast<uint8_t* const*>(a.ptr + K);
  const uint32_t off = tile * 4096u + threadIdx.x * 16u;
  uint32_t diff = 0;
  if ((uint64_t)off + 16 <= a.len)
    dev::lane_tile_k<K, 1, 1, MatVecMode::kStore, D, true, true, true, 4>(1, 1, t01, t2, in, out, 0, sbase, off, diff);
}

// kregtab with the library kernel's extras one at a time (F bits): 1 the tail branch (lane_tail_k over
// the argument block's tables), 2 the run-time m check and the one-round argument reads (varlen, tab,
// slen, len, sstride), 4 row pointers through tab / tstripe
template <int F>
__global__ __launch_bounds__(256) void kregx(const GfArgs a) {
  const uint32_t* kw = reinterpret_cast<const uint32_t*>(a.coef);
  u32x4 t01[K];
  uint32_t t2[K];
#pragma unroll
  for (int c = 0; c < K; ++c) {
    t01[c] = u32x4{kw[5 * c], kw[5 * c + 1], kw[5 * c + 2], kw[5 * c + 3]};
    t2[c] = kw[5 * c + 4];
  }
  const uint32_t stripe = blockIdx.y, tile = blockIdx.x;
  uint64_t len = a.len;
  int64_t sstride = a.sstride;
  uint32_t tab = 1, mrows = 1;
  if constexpr (F & 2) {
    uint32_t varlen = a.varlen, tb = a.tab;
    uint32_t slen = a.slen[stripe < (uint32_t)dev::kLenSlots ? stripe : (uint32_t)dev::kLenSlots - 1];
    uint64_t len0 = a.len;
    asm volatile("" : "+s"(varlen), "+s"(tb), "+s"(slen), "+s"(len0), "+s"(sstride));
    len = varlen ? (uint64_t)slen : len0;
    tab = tb;
    mrows = a.m;
  }
  const int64_t sbase = (int64_t)stripe * sstride;
  const uint8_t* const* in = a.ptr;
  uint8_t* const* out = const_cast<uint8_t* const*>(a.ptr + K);
  if constexpr (F & 4) {
    const size_t tstripe = sstride ? 0 : (size_t)stripe;
    in = a.ptr + tstripe * K;
    out = const_cast<uint8_t* const*>(a.ptr + (size_t)tab * K + tstripe * mrows);
  }
  const uint32_t off = tile * 4096u + threadIdx.x * 16u;
  uint32_t diff = 0;
  if ((F & 2) && (int)mrows < 1) return;
  if constexpr (F & 24) {
    // the ragged end: the last lane's piece clamped to end at len (overlapping its neighbour's bytes with
    // the same values); F 8: rows shorter than a piece take the byte path under a uniform branch
    if (off < len) {
      if (len >= 16) {
        const uint32_t loff = (uint64_t)off + 16 <= len ? off : (uint32_t)(len - 16);
        dev::lane_tile_k<K, 1, 1, MatVecMode::kStore, 4, true, true, true, 4>(1, 1, t01, t2, in, out, 0, sbase, loff,
                                                                            diff);
      } else if constexpr (F & 8) {
        const u32x4* k01 = reinterpret_cast<const u32x4*>(a.coef + 16);
        dev::lane_tail_k<K, 1, 1, MatVecMode::kStore>(a, k01, kw, in, out, 0, (size_t)sbase + off, len - off, diff);
      }
    }
    return;
  }
  if ((uint64_t)off + 16 <= len)
    dev::lane_tile_k<K, 1, 1, MatVecMode::kStore, 4, true, true, true, 4>((F & 2) ? (int)mrows : 1, 1, t01, t2, in, out, 0,
                                                                        sbase, off, diff);
  else if constexpr (F & 1) {
    if (off < len) {
      const u32x4* k01 = reinterpret_cast<const u32x4*>(a.coef + 16);  // any table (timing only)
      dev::lane_tail_k<K, 1, 1, MatVecMode::kStore>(a, k01, kw, in, out, 0, (size_t)sbase + off, len - off, diff);
    }
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
  std::vector<uint8_t> coef((size_t)M * K);  // a local repair row: arbitrary nonzero coefficients
  for (int c = 0; c < K; ++c) coef[c] = (uint8_t)(0x1d + 37 * c);
  // packed register tables (kregtab), same layout as gf_device.hpp coef_tables
  const GF& gf = GF::get();
  std::vector<uint32_t> packed(5 * K);
  for (int c = 0; c < K; ++c) {
    uint32_t pw[8];
    pw[0] = coef[c];
    for (int j = 1; j < 8; ++j) pw[j] = gf.mul((uint8_t)pw[j - 1], 2);
    uint32_t t0lo = 0, t0hi = 0, t1lo = 0, t1hi = 0, tt2 = 0;
    for (int e = 0; e < 8; ++e) {
      const uint32_t v0 = ((e & 1) ? pw[0] : 0u) ^ ((e & 2) ? pw[1] : 0u) ^ ((e & 4) ? pw[2] : 0u);
      const uint32_t v1 = ((e & 1) ? pw[3] : 0u) ^ ((e & 2) ? pw[4] : 0u) ^ ((e & 4) ? pw[5] : 0u);
      if (e < 4) {
        t0lo |= v0 << (8 * e);
        t1lo |= v1 << (8 * e);
        tt2 |= (((e & 1) ? pw[6] : 0u) ^ ((e & 2) ? pw[7] : 0u)) << (8 * e);
      } else {
        t0hi |= v0 << (8 * (e - 4));
        t1hi |= v1 << (8 * (e - 4));
      }
    }
    packed[5 * c] = t0lo, packed[5 * c + 1] = t0hi, packed[5 * c + 2] = t1lo, packed[5 * c + 3] = t1hi;
    packed[5 * c + 4] = tt2;
  }
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
    std::memcpy(a.coef, packed.data(), packed.size() * 4);
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
  vs.push_back({"shipped launcher (fixed-K k8 m1)", [&](int b) { CK(launch_matvec(jobs[b], 0)); }, step_bytes});
  std::vector<GfArgs> sargs(args);  // the library's fixed-K kernel, instantiated here, launched directly
  for (int b = 0; b < NB; ++b) {
    for (int c = 0; c < K; ++c) sargs[b].coef[c] = coef[c];
    cfsec::pack_reg_tables(K, M, coef.data(), sargs[b].coef);
  }
  vs.push_back({"fixed-K kernel, direct launch", [&](int b) { hipLaunchKernelGGL((cfsec::gf_matvec_k_kernel<K, M, MatVecMode::kStore>), grid, dim3(256), 0, 0, sargs[b]); }, step_bytes});
  vs.push_back({"regx F1 (+tail branch)", [&](int b) { hipLaunchKernelGGL(kregx<1>, grid, dim3(256), 0, 0, args[b]); }, step_bytes});
  vs.push_back({"regx F2 (+m check, arg round)", [&](int b) { hipLaunchKernelGGL(kregx<2>, grid, dim3(256), 0, 0, args[b]); }, step_bytes});
  vs.push_back({"regx F6 (+pointer base)", [&](int b) { hipLaunchKernelGGL(kregx<6>, grid, dim3(256), 0, 0, args[b]); }, step_bytes});
  vs.push_back({"regx F8 (clamped end + small-row branch)", [&](int b) { hipLaunchKernelGGL(kregx<8>, grid, dim3(256), 0, 0, args[b]); }, step_bytes});
  vs.push_back({"regx F16 (clamped end only)", [&](int b) { hipLaunchKernelGGL(kregx<16>, grid, dim3(256), 0, 0, args[b]); }, step_bytes});
  vs.push_back({"regx F7 (all)", [&](int b) { hipLaunchKernelGGL(kregx<7>, grid, dim3(256), 0, 0, args[b]); }, step_bytes});
  vs.push_back({"regtab D2", [&](int b) { hipLaunchKernelGGL(kregtab<2>, grid, dim3(256), 0, 0, args[b]); }, step_bytes});
  vs.push_back({"regtab D4", [&](int b) { hipLaunchKernelGGL(kregtab<4>, grid, dim3(256), 0, 0, args[b]); }, step_bytes});
  vs.push_back({"regtab D8", [&](int b) { hipLaunchKernelGGL(kregtab<8>, grid, dim3(256), 0, 0, args[b]); }, step_bytes});
  vs.push_back({"triv 8r1w st nt", [&](int b) { hipLaunchKernelGGL(ktriv<1>, grid, dim3(256), 0, 0, args[b]); }, step_bytes});
  vs.push_back({"triv 8r1w st sc1", [&](int b) { hipLaunchKernelGGL(ktriv<2>, grid, dim3(256), 0, 0, args[b]); }, step_bytes});
  vs.push_back({"triv W2 (8 KiB/row/wg)", [&](int b) { hipLaunchKernelGGL((ktrivw<2, 0>), dim3((nt1 + 1) / 2, NST), dim3(256), 0, 0, args[b]); }, step_bytes});
  vs.push_back({"triv W4 (16 KiB/row/wg)", [&](int b) { hipLaunchKernelGGL((ktrivw<4, 0>), dim3((nt1 + 3) / 4, NST), dim3(256), 0, 0, args[b]); }, step_bytes});
  vs.push_back({"triv seq W2", [&](int b) { hipLaunchKernelGGL((ktrivs<2>), dim3((nt1 + 1) / 2, NST), dim3(256), 0, 0, args[b]); }, step_bytes});
  vs.push_back({"triv W1 stripes fastest", [&](int b) { hipLaunchKernelGGL((ktrivw<1, 1>), dim3(nt1 * NST), dim3(256), 0, 0, args[b]); }, step_bytes});
  vs.push_back({"triv persistent 2048 wg xcd", [&](int b) { hipLaunchKernelGGL(ktrivp, dim3(2048), dim3(256), 0, 0, args[b], nt1); }, step_bytes});
  vs.push_back({"read 9 rows", [&](int b) { hipLaunchKernelGGL(kread16, grid, dim3(256), 0, 0, args[b]); }, step_bytes});
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
  {  // the register-table kernel's rows equal the shipped launcher's
    const size_t nbytes = S;
    std::vector<uint8_t> h1(nbytes), h2(nbytes);
    CK(launch_matvec(jobs[0], 0));
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h1.data(), outs[0][NST - 1], nbytes, hipMemcpyDeviceToHost));
    CK(hipMemset(outs[0][NST - 1], 0, nbytes));
    hipLaunchKernelGGL(kregtab<2>, grid, dim3(256), 0, 0, args[0]);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h2.data(), outs[0][NST - 1], nbytes - nbytes % 16, hipMemcpyDeviceToHost));
    printf("regtab rows equal the shipped launcher's (full 16-B pieces): %s\n",
           std::memcmp(h1.data(), h2.data(), nbytes - nbytes % 16) == 0 ? "yes" : "NO");
    CK(hipMemset(outs[0][NST - 1], 0, nbytes));
    hipLaunchKernelGGL(kregx<8>, grid, dim3(256), 0, 0, args[0]);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h2.data(), outs[0][NST - 1], nbytes, hipMemcpyDeviceToHost));
    printf("clamped-end rows equal the shipped launcher's (every byte): %s\n",
           std::memcmp(h1.data(), h2.data(), nbytes) == 0 ? "yes" : "NO");
  }
  printf("C4 local (8, 1): 48 x 699,051 B stripes per launch, 3 batches rotated (no Infinity-Cache reuse)\n");
  for (size_t i = 0; i < vs.size(); ++i) {
    std::sort(t[i].begin(), t[i].end());
    const double med = t[i][t[i].size() / 2];
    printf("%-34s median %8.1f us  %7.1f GB/s  %6.1f%% of 8 TB/s\n", vs[i].name.c_str(), med * 1e3,
           vs[i].bytes / (med * 1e-3) / 1e9, 100 * vs[i].bytes / (med * 1e-3) / 8e12);
  }
  return 0;
}
