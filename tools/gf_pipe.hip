// gf_pipe.hip -- memory-level-parallelism experiments for the GF matvec kernel (dev tool).
//
// Question: is the shipped EC12P4 kernel (load row -> wait -> compute, one 1 KiB load per wave
// in flight) bound by HBM, by VALU, or by the bytes it keeps in flight?  Variants:
//   ctl          shipped dev::matvec policy (runtime k, serial rows)
//   gfK D=d      compile-time K, rolling prefetch of d rows ahead (d = K: all loads up front)
//   xorK D=d     same data movement, trivial arithmetic (acc ^= x): the memory-pattern ceiling
//   copy         float4 device copy of the same byte count (calibration)
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../chubaofs_amd/csrc gf_pipe.hip -o gf_pipe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "gf256.hpp"
#include "gf_device.hpp"
#include "gf_dyadic.hpp"

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

__global__ __launch_bounds__(256) void kctl(const GfArgs a) {
  dev::matvec<4, MatVecMode::kStore, 1, 1, false, true, true, false>(a);
}

// Compile-time K inputs, M outputs, one 16-B chunk per lane, 256-thread workgroups (4 KiB tile),
// rows prefetched D ahead.  SB: sched_barrier after every row (keeps the issue order as written).
template <int K, int M, int D, bool TRIV, bool SB>
__global__ __launch_bounds__(256) void kpipe(const GfArgs a) {
  __shared__ u32x4 tab01[K * M];
  __shared__ uint32_t tab2[K * M];
  if constexpr (!TRIV) dev::build_tables<M>(a, tab01, tab2);
  __syncthreads();
  const uint32_t tps = a.tiles_per_stripe;
  const uint32_t t = blockIdx.x;
  const uint32_t stripe = t / tps;
  const size_t off = (size_t)(t - stripe * tps) * 4096 + threadIdx.x * 16;
  const size_t soff = (size_t)stripe * a.sstride;
  const uint8_t* in[K];
#pragma unroll
  for (int c = 0; c < K; ++c) in[c] = a.ptr[c] + soff;
  if (off + 16 <= a.len) {
    u32x4 acc[M];
#pragma unroll
    for (int r = 0; r < M; ++r) acc[r] = u32x4{0u, 0u, 0u, 0u};
    u32x4 x[K];
#pragma unroll
    for (int c = 0; c < D && c < K; ++c) x[c] = dev::ld16<true>(in[c] + off);
#pragma unroll
    for (int c = 0; c < K; ++c) {
      if (c + D < K) x[c + D] = dev::ld16<true>(in[c + D] + off);
      if constexpr (TRIV) {
#pragma unroll
        for (int r = 0; r < M; ++r) acc[r] ^= x[c] + (uint32_t)r;
      } else {
        dev::mac_row<M>(acc, x[c], tab01 + c * M, tab2 + c * M);
      }
      if constexpr (SB) __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int r = 0; r < M; ++r) dev::st16<true>(const_cast<uint8_t*>(a.ptr[K + r]) + soff + off, acc[r]);
  } else if (off < a.len) {
    uint8_t* const* out = const_cast<uint8_t* const*>(a.ptr + K);
    uint32_t diff = 0;
    const uint8_t* const* inb = a.ptr;
    if constexpr (!TRIV)
      dev::lane_tail<M, M, MatVecMode::kStore>(a, tab01, tab2, inb, out, 0, soff + off, a.len - off, diff);
  }
}


// Runtime k (the shipped kernel's interface) with a 3-deep rolling prefetch: a ring of three
// 16-B registers, the loop unrolled by 3 so every ring slot has a static name.
template <int M, bool SB>
__global__ __launch_bounds__(256) void kring3(const GfArgs a) {
  constexpr int MT = M;
  __shared__ u32x4 tab01[dev::kMaxK * MT];
  __shared__ uint32_t tab2[dev::kMaxK * MT];
  dev::build_tables<MT>(a, tab01, tab2);
  __syncthreads();
  const int k = (int)a.k;
  const uint32_t tps = a.tiles_per_stripe;
  const uint32_t t = blockIdx.x;
  const uint32_t stripe = t / tps;
  const size_t off = (size_t)(t - stripe * tps) * 4096 + threadIdx.x * 16;
  const size_t soff = (size_t)stripe * a.sstride + off;
  const uint8_t* const* in = a.ptr;
  if (off + 16 <= a.len) {
    u32x4 acc[M];
#pragma unroll
    for (int r = 0; r < M; ++r) acc[r] = u32x4{0u, 0u, 0u, 0u};
    u32x4 x0 = dev::ld16<true>(in[0] + soff), x1, x2;
    if (k > 1) x1 = dev::ld16<true>(in[1] + soff);
    if (k > 2) x2 = dev::ld16<true>(in[2] + soff);
    for (int c = 0; c < k; c += 3) {
      u32x4 cur = x0;
      if (c + 3 < k) x0 = dev::ld16<true>(in[c + 3] + soff);
      dev::mac_row<M>(acc, cur, tab01 + c * MT, tab2 + c * MT);
      if constexpr (SB) __builtin_amdgcn_sched_barrier(0);
      if (c + 1 >= k) break;
      cur = x1;
      if (c + 4 < k) x1 = dev::ld16<true>(in[c + 4] + soff);
      dev::mac_row<M>(acc, cur, tab01 + (c + 1) * MT, tab2 + (c + 1) * MT);
      if constexpr (SB) __builtin_amdgcn_sched_barrier(0);
      if (c + 2 >= k) break;
      cur = x2;
      if (c + 5 < k) x2 = dev::ld16<true>(in[c + 5] + soff);
      dev::mac_row<M>(acc, cur, tab01 + (c + 2) * MT, tab2 + (c + 2) * MT);
      if constexpr (SB) __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int r = 0; r < M; ++r) dev::st16<true>(const_cast<uint8_t*>(a.ptr[a.k + r]) + soff, acc[r]);
  } else if (off < a.len) {
    uint8_t* const* out = const_cast<uint8_t* const*>(a.ptr + a.k);
    uint32_t diff = 0;
    dev::lane_tail<M, MT, MatVecMode::kStore>(a, tab01, tab2, in, out, 0, (size_t)stripe * a.sstride + off,
                                              a.len - off, diff);
  }
}


// Compile-time K, W 16-B chunks per lane at 1 KiB stride (each wave covers W KiB contiguous of
// every row), rows prefetched D ahead.  NTS: non-temporal stores.
template <int K, int M, int D, int W, bool NTS = true>
__global__ __launch_bounds__(256) void kgfw(const GfArgs a) {
  __shared__ u32x4 tab01[K * M];
  __shared__ uint32_t tab2[K * M];
  dev::build_tables<M>(a, tab01, tab2);
  __syncthreads();
  const uint32_t tps = a.tiles_per_stripe;
  const uint32_t t = blockIdx.x;
  const uint32_t stripe = t / tps;
  const size_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t off = (size_t)(t - stripe * tps) * (4096 * W) + wave * (1024 * W) + lane * 16;
  const size_t soff = (size_t)stripe * a.sstride + off;
  if (off + (W - 1) * 1024 + 16 > a.len) return;  // probe: tails skipped (timing only)
  u32x4 acc[W][M];
#pragma unroll
  for (int w = 0; w < W; ++w)
#pragma unroll
    for (int r = 0; r < M; ++r) acc[w][r] = u32x4{0u, 0u, 0u, 0u};
  u32x4 x[K][W];
#pragma unroll
  for (int c = 0; c < D && c < K; ++c)
#pragma unroll
    for (int w = 0; w < W; ++w) x[c][w] = dev::ld16<true>(a.ptr[c] + soff + w * 1024);
#pragma unroll
  for (int c = 0; c < K; ++c) {
    if (c + D < K)
#pragma unroll
      for (int w = 0; w < W; ++w) x[c + D][w] = dev::ld16<true>(a.ptr[c + D] + soff + w * 1024);
#pragma unroll
    for (int w = 0; w < W; ++w) dev::mac_row<M>(acc[w], x[c][w], tab01 + c * M, tab2 + c * M);
  }
#pragma unroll
  for (int r = 0; r < M; ++r)
#pragma unroll
    for (int w = 0; w < W; ++w)
      dev::st16<NTS>(const_cast<uint8_t*>(a.ptr[K + r]) + soff + w * 1024, acc[w][r]);
}

// Pattern probe, sequential: a workgroup walks T consecutive 4 KiB tiles of the stripe (1 KiB
// per wave per row per tile), so its writes advance through each row.
template <int NIN, int NOUT, int T, bool NTS>
__global__ __launch_bounds__(256) void kpats(const GfArgs a) {
  const uint32_t tps = a.tiles_per_stripe;  // in units of T tiles
  const uint32_t t = blockIdx.x;
  const uint32_t stripe = t / tps;
  const size_t soff = (size_t)stripe * a.sstride;
  for (int i = 0; i < T; ++i) {
    const size_t base = ((size_t)(t - stripe * tps) * T + i) * 4096 + threadIdx.x * 16;
    if (base + 16 > a.len) return;
    u32x4 acc = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
    for (int c = 0; c < NIN; ++c) acc ^= dev::ld16<true>(a.ptr[c] + soff + base);
#pragma unroll
    for (int r = 0; r < NOUT; ++r)
      dev::st16<NTS>(const_cast<uint8_t*>(a.ptr[NIN + r]) + soff + base, acc + (uint32_t)r);
  }
}


// Store cache-policy probes: the pattern kernel (12 -> 4, trivial arithmetic) and the shipped
// fixed-K tile, with the output stores issued as inline asm carrying the given modifiers.
template <int SP>
__device__ __forceinline__ void st_pol(uint8_t* p, u32x4 v) {
  if constexpr (SP == 0) asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
  else if constexpr (SP == 1) asm volatile("global_store_dwordx4 %0, %1, off nt\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
  else if constexpr (SP == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
  else if constexpr (SP == 3) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
  else if constexpr (SP == 4) asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
  else if constexpr (SP == 5) asm volatile("global_store_dwordx4 %0, %1, off nt sc0 sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
  else asm volatile("global_store_dwordx4 %0, %1, off sc0\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

template <int SP>
__global__ __launch_bounds__(256) void kpatp(const GfArgs a) {
  const uint32_t stripe = blockIdx.y;
  const size_t base = (size_t)blockIdx.x * 4096 + threadIdx.x * 16;
  const size_t soff = (size_t)stripe * a.sstride;
  if (base + 16 > a.len) return;
  u32x4 acc = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
  for (int c = 0; c < 12; ++c) acc ^= dev::ld16<true>(a.ptr[c] + soff + base);
#pragma unroll
  for (int r = 0; r < 4; ++r) st_pol<SP>(const_cast<uint8_t*>(a.ptr[12 + r]) + soff + base, acc + (uint32_t)r);
}


template <int D, bool NTL, bool NTS, bool PAIR = true, int K = 12, int M = 4, int OS = 1>
__global__ __launch_bounds__(256) void kfix(const GfArgs a) {
  dev::matvec_k<K, M, MatVecMode::kStore, D, OS, NTL, NTS, PAIR>(a);
}


template <int K, int M, int B, bool NTS = true, bool NTL = true>
__global__ __launch_bounds__(256) void kdy(const GfArgs a) {
  dev::matvec_dy<K, M, B, MatVecMode::kStore, NTS, NTL>(a);
}

__global__ __launch_bounds__(256) void kcopy(const u32x4* __restrict__ src, u32x4* __restrict__ dst, size_t n) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < n) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}


// Memory-pattern probes, trivial arithmetic.  NIN input rows, NOUT output rows, each wave
// covers W KiB contiguous of every row (W 1-KiB chunks per lane at 1 KiB stride).
template <int NIN, int NOUT, int W>
__global__ __launch_bounds__(256) void kpat(const GfArgs a) {
  const uint32_t tps = a.tiles_per_stripe;
  const uint32_t t = blockIdx.x;
  const uint32_t stripe = t / tps;
  const size_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t base = (size_t)(t - stripe * tps) * (4096 * W) + wave * (1024 * W) + lane * 16;
  const size_t soff = (size_t)stripe * a.sstride;
  u32x4 acc[W];
#pragma unroll
  for (int w = 0; w < W; ++w) acc[w] = u32x4{0u, 0u, 0u, 0u};
  if (base + (W - 1) * 1024 + 16 > a.len) return;
#pragma unroll
  for (int c = 0; c < NIN; ++c)
#pragma unroll
    for (int w = 0; w < W; ++w) acc[w] ^= dev::ld16<true>(a.ptr[c] + soff + base + w * 1024);
  if constexpr (NOUT == 0) {
    uint32_t d = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) d |= acc[w].x & acc[w].y & acc[w].z & acc[w].w;
    if (d == 0x12345678u) a.flags[0] = d;
  }
#pragma unroll
  for (int r = 0; r < NOUT; ++r)
#pragma unroll
    for (int w = 0; w < W; ++w)
      dev::st16<true>(const_cast<uint8_t*>(a.ptr[NIN + r]) + soff + base + w * 1024, acc[w] + (uint32_t)r);
}

__global__ void fill_kernel(uint32_t* p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t z = (uint64_t)(i >> 1) * 0x9E3779B97F4A7C15ull + 0xCF5EC000ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    p[i] = (i & 1) ? (uint32_t)(z >> 32) : (uint32_t)z;
  }
}

struct Variant {
  std::string name;
  void (*kern)(GfArgs);
  bool gf;  // output must match ctl
  int tilekb = 4;
  double bytes_scale = 1.0;  // algorithmic bytes relative to 16 rows
};

template <int D, bool TRIV, bool SB = false>
Variant mk(const char* name) {
  return Variant{name, kpipe<12, 4, D, TRIV, SB>, !TRIV};
}

int main(int argc, char** argv) {
  const size_t S = argc > 1 ? strtoull(argv[1], 0, 10) : 5592406;
  const int nst = argc > 2 ? atoi(argv[2]) : 8;
  const int rounds = argc > 3 ? atoi(argv[3]) : 15;
  const int k = 12, m = 4, total = 16;
  const size_t pitch = (S + 255) / 256 * 256;
  const size_t bytes = pitch * total * nst;
  uint8_t* buf = nullptr;
  uint8_t* cbuf = nullptr;
  CK(hipMalloc(&buf, bytes));
  const size_t copy_bytes = (size_t(k + m) * S * nst / 2) / 16 * 16;  // read + write = algorithmic bytes
  CK(hipMalloc(&cbuf, 2 * copy_bytes));
  fill_kernel<<<4096, 256>>>((uint32_t*)buf, bytes / 4);
  fill_kernel<<<4096, 256>>>((uint32_t*)cbuf, 2 * copy_bytes / 4);
  CK(hipDeviceSynchronize());

  Matrix mat;
  build_matrix(k, total, mat);
  GfArgs a{};
  a.len = S;
  a.k = k;
  a.m = m;
  a.nstripes = nst;
  a.tab = 1;
  a.sstride = (int64_t)(pitch * total);
  a.tiles_per_stripe = (uint32_t)((S + 4095) / 4096);
  for (int r = 0; r < m; ++r)
    for (int c = 0; c < k; ++c) a.coef[r * k + c] = mat.at(k + r, c);
  for (int c = 0; c < k; ++c) a.ptr[c] = buf + c * pitch;
  for (int r = 0; r < m; ++r) a.ptr[k + r] = buf + (k + r) * pitch;

  std::vector<Variant> vs = {
      {"ctl (runtime k)", kctl, true},
      {"dyadic B4", kdy<12, 4, 4>, true, -4},
      {"dyadic B4 plainS", kdy<12, 4, 4, false>, true, -4},
      {"dyadic B4 plainL", kdy<12, 4, 4, true, false>, true, -4},
      {"dyadic B4 plain LS", kdy<12, 4, 4, false, false>, true, -4},
      {"dyadic B4 (2)", kdy<12, 4, 4>, true, -4},
      {"dyadic B4 plainS (2)", kdy<12, 4, 4, false>, true, -4},
      {"pat2d st plain", kpatp<0>, false, -4},
      {"pat2d st nt", kpatp<1>, false, -4},
  };
  uint32_t* flags = nullptr;
  CK(hipMalloc(&flags, 64));
  a.flags = flags;
  auto launch = [&](const Variant& v) {
    if (v.kern && v.tilekb < 0) {  // 2-D grid (tiles, stripes)
      GfArgs b = a;
      b.tiles_per_stripe = (uint32_t)((S - v.tilekb * 1024 - 1) / (-v.tilekb * 1024));
      hipLaunchKernelGGL(v.kern, dim3(b.tiles_per_stripe, nst), dim3(256), 0, 0, b);
    } else if (v.kern) {
      GfArgs b = a;
      b.tiles_per_stripe = (uint32_t)((S + v.tilekb * 1024 - 1) / (v.tilekb * 1024));
      hipLaunchKernelGGL(v.kern, dim3(b.tiles_per_stripe * nst), dim3(256), 0, 0, b);
    } else {
      const size_t n = copy_bytes / 16;
      hipLaunchKernelGGL(kcopy, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, (const u32x4*)cbuf,
                         (u32x4*)(cbuf + copy_bytes), n);
    }
  };
  auto snapshot = [&](std::vector<uint8_t>& out) {
    out.resize(size_t(nst) * m * S);
    for (int s = 0; s < nst; ++s)
      for (int r = 0; r < m; ++r)
        CK(hipMemcpy(out.data() + (size_t(s) * m + r) * S, buf + (s * total + k + r) * pitch, S,
                     hipMemcpyDeviceToHost));
  };
  std::vector<uint8_t> golden, cur;
  for (size_t i = 0; i < vs.size(); ++i) {
    if (!vs[i].gf) continue;
    for (int s = 0; s < nst; ++s) CK(hipMemset(buf + (s * total + k) * pitch, 0, m * pitch));
    launch(vs[i]);
    CK(hipDeviceSynchronize());
    snapshot(i == 0 ? golden : cur);
    if (i && cur != golden) {
      printf("MISMATCH in variant %s\n", vs[i].name.c_str());
      return 2;
    }
  }
  printf("all GF variants agree with the shipped kernel\n");

  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  // settle the clock (bench_env_clock_ramp.txt)
  for (int j = 0; j < 300; ++j) launch(vs[0]);
  CK(hipDeviceSynchronize());
  const int reps = 10;
  std::vector<std::vector<float>> t(vs.size());
  for (int rnd = 0; rnd < rounds; ++rnd)
    for (size_t i = 0; i < vs.size(); ++i) {
      launch(vs[i]);
      CK(hipEventRecord(e0, 0));
      for (int j = 0; j < reps; ++j) launch(vs[i]);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[i].push_back(ms / reps);
    }
  const double algo = double(k + m) * S * nst;
  printf("S=%zu stripes=%d  algorithmic bytes/launch=%.0f (copy: same bytes read+written)\n", S, nst, algo);
  for (size_t i = 0; i < vs.size(); ++i) {
    auto v = t[i];
    std::sort(v.begin(), v.end());
    const float med = v[v.size() / 2], mn = v[0];
    printf("%-18s median %8.1f us  min %8.1f us  -> %7.1f GB/s (%.1f%% of 8 TB/s)\n", vs[i].name.c_str(),
           med * 1e3, mn * 1e3, algo * vs[i].bytes_scale / (med * 1e-3) / 1e9, 100.0 * algo * vs[i].bytes_scale / (med * 1e-3) / 8e12);
  }
  return 0;
}
