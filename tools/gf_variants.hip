// gf_variants.hip -- A/B harness for the GF matvec kernel policies (dev tool, not shipped).
//
// Builds every policy variant of cfsec::dev::matvec for the EC12P4 bench shape, checks
// each against the first variant's output, then times them in interleaved rounds in one
// process (cdna_hip_programming.md §5.4 rule 24) and prints median/min per variant.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../chubaofs_amd/csrc gf_variants.hip -o gf_variants
//   ./gf_variants [S] [stripes] [rounds] [mode: 0 encode, 2 verify]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gf256.hpp"
#include "gf_device.hpp"

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

template <int M, MatVecMode MODE, int W, int G, bool PERSIST, bool NTL, bool NTS, bool XCD, int LB, bool WC>
__global__ __launch_bounds__(LB) void kvar(const GfArgs a) {
  dev::matvec<M, MODE, W, G, PERSIST, NTL, NTS, XCD, WC>(a);
}

__global__ void fill_kernel(uint32_t* p, size_t n, uint32_t seed) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
    if (seed == 0) {  // splitmix64 per 8-byte word (full-entropy bytes)
      uint64_t z = (uint64_t)(i >> 1) * 0x9E3779B97F4A7C15ull + 0xCF5EC000ull;
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
      z ^= z >> 31;
      p[i] = (i & 1) ? (uint32_t)(z >> 32) : (uint32_t)z;
    } else {
      uint32_t x = (uint32_t)i * 2654435761u ^ seed;
      x ^= x << 13; x ^= x >> 17; x ^= x << 5;
      p[i] = x;
    }
  }
}

struct Variant {
  std::string name;
  void (*kern)(GfArgs);
  int W;
  bool persist;
  int bt = 256;
  size_t lds = 0;
};

template <int W, int G, bool P, bool NTL, bool NTS = NTL, bool XCD = false, int LB = 256, bool WC = false>
Variant mk(const char* name, MatVecMode mode, int bt = 256, size_t lds = 0) {
  Variant v;
  v.bt = bt;
  v.lds = lds;
  v.name = name;
  v.W = W;
  v.persist = P;
  if (mode == MatVecMode::kVerify) v.kern = kvar<4, MatVecMode::kVerify, W, G, P, NTL, NTS, XCD, LB, WC>;
  else v.kern = kvar<4, MatVecMode::kStore, W, G, P, NTL, NTS, XCD, LB, WC>;
  return v;
}

int main(int argc, char** argv) {
  const size_t S = argc > 1 ? strtoull(argv[1], 0, 10) : 5592406;
  const int nst = argc > 2 ? atoi(argv[2]) : 8;
  const int rounds = argc > 3 ? atoi(argv[3]) : 15;
  const MatVecMode mode = (argc > 4 && atoi(argv[4]) == 2) ? MatVecMode::kVerify : MatVecMode::kStore;
  const int k = 12, m = 4, total = 16;
  const size_t pitch = (S + 255) / 256 * 256;
  uint8_t* buf = nullptr;
  const size_t bytes = pitch * total * nst;
  CK(hipMalloc(&buf, bytes));
  fill_kernel<<<4096, 256>>>((uint32_t*)buf, bytes / 4, argc > 6 ? (uint32_t)atoi(argv[6]) : 0xCF5EC000u);
  uint32_t* flags = nullptr;
  CK(hipMalloc(&flags, 4 * nst));
  CK(hipDeviceSynchronize());

  Matrix mat;
  build_matrix(k, total, mat);
  GfArgs a{};
  a.len = S;
  a.k = k;
  a.m = m;
  a.nstripes = nst;
  a.tab = nst;
  a.flags = flags;
  for (int r = 0; r < m; ++r)
    for (int c = 0; c < k; ++c) a.coef[r * k + c] = mat.at(k + r, c);
  for (int s = 0; s < nst; ++s) {
    for (int c = 0; c < k; ++c) a.ptr[s * k + c] = buf + (s * total + c) * pitch;
    for (int r = 0; r < m; ++r) a.ptr[nst * k + s * m + r] = buf + (s * total + k + r) * pitch;
  }

  std::vector<Variant> vs = {
      mk<1, 1, false, true>("b256 W1 nt (ctl)", mode),
      mk<2, 1, false, true, true, false, 256, true>("b256 W2 nt wavec", mode),
      mk<4, 1, false, true, true, false, 256, true>("b256 W4 nt wavec", mode),
      mk<2, 1, false, true, true, false, 256, true>("b128 W2 nt wavec", mode, 128),
      mk<4, 1, false, true, true, false, 256, true>("b128 W4 nt wavec", mode, 128),
      mk<2, 2, false, true, true, false, 256, true>("b128 W2 G2 nt wavec", mode, 128),
      mk<2, 2, false, true>("b128 W2 G2 nt", mode, 128),
      mk<1, 1, false, true>("b256 W1 nt (ctl2)", mode),
  };




  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));

  std::vector<uint8_t> golden, cur;
  auto launch = [&](const Variant& v) {
    const size_t tile = size_t(v.bt) * dev::kLaneBytes * v.W;
    GfArgs b = a;
    b.tiles_per_stripe = (uint32_t)((S + tile - 1) / tile);
    unsigned grid = b.tiles_per_stripe * nst;
    if (v.persist) {
      int per = 0;
      CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, v.kern, v.bt, v.lds));
      grid = std::min<unsigned>(grid, (unsigned)(per * ncu));
    }
    hipLaunchKernelGGL(v.kern, dim3(grid), dim3(v.bt), v.lds, 0, b);
  };
  auto snapshot = [&](std::vector<uint8_t>& out) {
    out.resize(size_t(nst) * m * S);
    for (int s = 0; s < nst; ++s)
      for (int r = 0; r < m; ++r)
        CK(hipMemcpy(out.data() + (size_t(s) * m + r) * S, buf + (s * total + k + r) * pitch, S, hipMemcpyDeviceToHost));
  };
  // correctness: every variant writes identical parity (verify mode: flags stay 0 after an encode)
  if (mode == MatVecMode::kStore) {
    for (size_t i = 0; i < vs.size(); ++i) {
      CK(hipMemset(buf + k * pitch, 0, 4 * pitch));  // clobber stripe 0 parity
      launch(vs[i]);
      CK(hipDeviceSynchronize());
      snapshot(i == 0 ? golden : cur);
      if (i && cur != golden) {
        printf("MISMATCH in variant %s\n", vs[i].name.c_str());
        return 2;
      }
    }
  } else {
    launch(mk<1, 12, false, false>("enc", MatVecMode::kStore));
    CK(hipDeviceSynchronize());
    for (auto& v : vs) {
      CK(hipMemset(flags, 0, 4 * nst));
      launch(v);
      uint32_t h[64];
      CK(hipMemcpy(h, flags, 4 * nst, hipMemcpyDeviceToHost));
      for (int s = 0; s < nst; ++s)
        if (h[s]) { printf("verify false positive in %s\n", v.name.c_str()); return 2; }
    }
  }
  printf("all %zu variants agree\n", vs.size());

  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
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
  printf("S=%zu stripes=%d mode=%d  algorithmic bytes/launch=%.0f\n", S, nst, (int)mode, algo);
  const int soak = argc > 5 ? atoi(argv[5]) : 0;
  if (soak > 0) {
    // Steady state: control variant, encode-only vs alternating encode / reconstruct({0,1,2,3}),
    // mean per launch over consecutive windows of 100 launches.
    GfArgs rec = a;
    Matrix sub(k, k), dec;
    for (int r = 0; r < k; ++r)
      for (int c = 0; c < k; ++c) sub.at(r, c) = mat.at(4 + r, c);
    mat_invert(sub, dec);
    for (int r = 0; r < m; ++r)
      for (int c = 0; c < k; ++c) rec.coef[r * k + c] = dec.at(r, c);
    for (int s = 0; s < nst; ++s) {
      for (int c = 0; c < k; ++c) rec.ptr[s * k + c] = buf + (s * total + 4 + c) * pitch;
      for (int r = 0; r < m; ++r) rec.ptr[nst * k + s * m + r] = buf + (s * total + r) * pitch;
    }
    const Variant& v = vs[0];
    for (int alt = 0; alt < 2; ++alt) {
      printf("soak %s:", alt ? "alternating enc/rec" : "encode only");
      for (int w = 0; w < soak / 100; ++w) {
        CK(hipEventRecord(e0, 0));
        for (int j = 0; j < 100; ++j) {
          GfArgs b = (alt && (j & 1)) ? rec : a;
          const size_t tile = size_t(v.bt) * dev::kLaneBytes * v.W;
          b.tiles_per_stripe = (uint32_t)((S + tile - 1) / tile);
          hipLaunchKernelGGL(v.kern, dim3(b.tiles_per_stripe * nst), dim3(v.bt), 0, 0, b);
        }
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf(" %.1f", ms * 10);  // us per launch
      }
      printf("\n");
    }
  }
  for (size_t i = 0; i < vs.size(); ++i) {
    auto v = t[i];
    std::sort(v.begin(), v.end());
    const float med = v[v.size() / 2], mn = v[0];
    printf("%-18s median %8.1f us  min %8.1f us  -> %7.1f GB/s (%.1f%% of 8 TB/s)\n", vs[i].name.c_str(),
           med * 1e3, mn * 1e3, algo / (med * 1e-3) / 1e9, 100.0 * algo / (med * 1e-3) / 8e12);
  }
  return 0;
}
