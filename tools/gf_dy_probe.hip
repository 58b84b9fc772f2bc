// gf_dy_probe.hip -- A/B of the dyadic-block kernel against the shipped launcher for wide outputs
// (EC16P20 global encode, k=16 m=20; EC6P10, k=6 m=10), dev tool.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../chubaofs_amd/csrc gf_dy_probe.hip \
//         -L../chubaofs_amd -lcfsec -Wl,-rpath,'$ORIGIN/../chubaofs_amd' -o gf_dy_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <string>
#include <vector>

#include "gf256.hpp"
#include "gf_dyadic.hpp"
#include "gf_fixed.hpp"
#include "kernels.hpp"

using namespace cfsec;
using dev::GfArgs;

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

template <int K, int M, int B, int RBW>
__global__ __launch_bounds__((dev::DyShape<M, B, RBW>::kThreadsPerWg)) void kdy(const GfArgs a) {
  dev::matvec_dy<K, M, B, MatVecMode::kStore, true, true, RBW>(a);
}

// free scheduling: no accumulator pins / sched barriers (the compiler may hoist every load)
template <int K, int M, int B, int SP, int LP = -1>
__global__ __launch_bounds__((dev::DyShape<M, B>::kThreadsPerWg)) void kdysp(const GfArgs a) {
  dev::matvec_dy<K, M, B, MatVecMode::kStore, true, true, 64, 0, true, SP, LP>(a);
}

template <int K, int M, int B, bool NTS, bool NTL>
__global__ __launch_bounds__((dev::DyShape<M, B>::kThreadsPerWg)) void kdyf(const GfArgs a) {
  dev::matvec_dy<K, M, B, MatVecMode::kStore, NTS, NTL, 64, 0, false>(a);
}

__global__ void fill(uint32_t* p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    p[i] = (uint32_t)(z ^ (z >> 31));
  }
}

struct V {
  std::string name;
  void (*k)(GfArgs);
  int threads, tile;
};

template <int K, int M, int OS>
__global__ __launch_bounds__(256) void kplain(const GfArgs a) {
  dev::matvec_k<K, (M + OS - 1) / OS, MatVecMode::kStore, 2, OS>(a);
}

template <int K, int M, int OS>
V mkp(const char* n) {
  return V{n, kplain<K, M, OS>, 256, 4096 / OS};
}

template <int K, int M, int B, int RBW>
V mk(const char* n) {
  using Sh = dev::DyShape<M, B, RBW>;
  return V{n, kdy<K, M, B, RBW>, Sh::kThreadsPerWg, Sh::kTileBytes};
}

template <int K, int M, int B, int SP, int LP = -1>
V mksp(const char* n) {
  using Sh = dev::DyShape<M, B>;
  return V{n, kdysp<K, M, B, SP, LP>, Sh::kThreadsPerWg, Sh::kTileBytes};
}

template <int K, int M, int B, bool NTS = true, bool NTL = true>
V mkf(const char* n) {
  using Sh = dev::DyShape<M, B>;
  return V{n, kdyf<K, M, B, NTS, NTL>, Sh::kThreadsPerWg, Sh::kTileBytes};
}

template <int K, int M, int B>
void run(size_t S, int nst, std::vector<V> vs) {
  const size_t pitch = (S + 255) / 256 * 256;
  uint8_t* buf;
  CK(hipMalloc(&buf, pitch * (K + M) * nst));
  fill<<<2048, 256>>>((uint32_t*)buf, pitch * (K + M) * nst / 4);
  Matrix mat;
  build_matrix(K, K + M, mat);
  std::vector<uint8_t> coef((size_t)M * K);
  for (int r = 0; r < M; ++r)
    for (int c = 0; c < K; ++c) coef[(size_t)r * K + c] = mat.at(K + r, c);
  std::vector<const uint8_t*> in((size_t)nst * K);
  std::vector<uint8_t*> out((size_t)nst * M);
  for (int s = 0; s < nst; ++s) {
    for (int c = 0; c < K; ++c) in[(size_t)s * K + c] = buf + ((size_t)s * (K + M) + c) * pitch;
    for (int r = 0; r < M; ++r) out[(size_t)s * M + r] = buf + ((size_t)s * (K + M) + K + r) * pitch;
  }
  MatVecJob job;
  job.k = K;
  job.m = M;
  job.coef = coef.data();
  job.len = S;
  job.nstripes = nst;
  job.in = in.data();
  job.out = out.data();
  GfArgs a{};
  a.len = S;
  a.k = K;
  a.m = M;
  a.nstripes = nst;
  a.tab = 1;
  a.sstride = (int64_t)(pitch * (K + M));
  for (size_t i = 0; i < coef.size(); ++i) a.coef[i] = coef[i];
  for (int c = 0; c < K; ++c) a.ptr[c] = in[c];
  for (int r = 0; r < M; ++r) a.ptr[K + r] = out[r];
  std::vector<uint8_t> gold((size_t)M * S), cur((size_t)M * S);
  auto snap = [&](std::vector<uint8_t>& v) {
    for (int r = 0; r < M; ++r) CK(hipMemcpy(v.data() + (size_t)r * S, out[r], S, hipMemcpyDeviceToHost));
  };
  CK(launch_matvec(job, 0));
  CK(hipDeviceSynchronize());
  snap(gold);
  auto launch = [&](int i) {
    if (i < 0) {
      CK(launch_matvec(job, 0));
    } else {
      const V& v = vs[i];
      hipLaunchKernelGGL(v.k, dim3((unsigned)((S + v.tile - 1) / v.tile), nst), dim3(v.threads), 0, 0, a);
    }
  };
  for (size_t i = 0; i < vs.size(); ++i) {
    for (int r = 0; r < M; ++r) CK(hipMemset(out[r], 0, S));
    launch((int)i);
    CK(hipDeviceSynchronize());
    snap(cur);
    if (cur != gold) {
      printf("k=%2d m=%2d %-22s MISMATCH (matrix not dyadic?) -- skipped\n", K, M, vs[i].name.c_str());
      vs.erase(vs.begin() + (long)i--);
    }
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int j = 0; j < 200; ++j) launch(-1);
  const int n = (int)vs.size() + 1;
  std::vector<std::vector<float>> t(n);
  for (int rnd = 0; rnd < 15; ++rnd)
    for (int i = -1; i < (int)vs.size(); ++i) {
      launch(i);
      CK(hipEventRecord(e0, 0));
      for (int j = 0; j < 10; ++j) launch(i);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[i + 1].push_back(ms / 10);
    }
  const double bytes = double(K + M) * S * nst;
  for (int i = 0; i < n; ++i) {
    std::sort(t[i].begin(), t[i].end());
    const double med = t[i][t[i].size() / 2];
    printf("k=%2d m=%2d %-22s median %8.1f us  %6.1f%% of 8 TB/s\n", K, M, i ? vs[i - 1].name.c_str() : "shipped launcher",
           med * 1e3, 100 * bytes / (med * 1e-3) / 8e12);
  }
  CK(hipFree(buf));
}

int main() {
  // stores sc1 (SP 2) throughout; loads: builtin nt, then buffer loads with aux bits
  run<12, 4, 4>(5592406, 8, {mksp<12, 4, 4, 2>("ld nt (builtin)"), mksp<12, 4, 4, 2, 2>("ld buf nt"),
                             mksp<12, 4, 4, 2, 0>("ld buf plain"), mksp<12, 4, 4, 2, 16>("ld buf sc1"),
                             mksp<12, 4, 4, 2, 18>("ld buf nt sc1"), mksp<12, 4, 4, 2, 1>("ld buf sc0"),
                             mksp<12, 4, 4, 2, 17>("ld buf sc0 sc1"), mksp<12, 4, 4, 2, 19>("ld buf nt sc0 sc1")});
  run<12, 4, 4>(5592406, 8, {mksp<12, 4, 4, 2>("ld nt (builtin) (2)"), mksp<12, 4, 4, 2, 2>("ld buf nt (2)"),
                             mksp<12, 4, 4, 2, 16>("ld buf sc1 (2)"), mksp<12, 4, 4, 2, 18>("ld buf nt sc1 (2)")});
  return 0;
}
