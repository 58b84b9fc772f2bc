// c5_pattern_probe.hip -- the access-pattern ceiling of C5's repair pass (dev tool, profiles/r04).
//
// C5's tasklet: 64 bids of EC16P20L2 at S = 262,144; the fused Reconstruct + Verify pass per bid
// reads 16 input rows, writes 4 rebuilt rows and reads 18 more rows to compare (38 rows).  These
// kernels keep that access pattern -- same grid (tiles, bids), 256-thread workgroups, W-dword lane
// chunks, non-temporal loads and stores -- with trivial arithmetic (XORs), over three tasklets in
// rotation (no Infinity-Cache reuse), so their time bounds what any arithmetic in the repair
// kernel can reach.  Variants: compared rows loaded after the outputs are stored (the repair
// kernel's order) or together with the inputs; W = 1, 2, 4.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../chubaofs_amd/csrc c5_pattern_probe.hip -o c5_pattern_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "gf_device.hpp"

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

constexpr int NIN = 16, NOUT = 4, NCMP = 18, ROWS = NIN + NOUT + NCMP, NB = 64, NT = 3;
constexpr size_t S = 262144;

struct Args {
  uint8_t* base;  // tasklet: bid b row r at base + (b * ROWS + r) * S
  uint32_t* flags;
};

template <int W, bool EARLY>
__global__ __launch_bounds__(256) void kpat(const Args a) {
  const uint32_t bid = blockIdx.y;
  const uint32_t off = blockIdx.x * (256u * 4 * W) + threadIdx.x * 4 * W;
  const uint8_t* row0 = a.base + (size_t)bid * ROWS * S;
  uint32_t x[NIN][W], y[NCMP][W];
#pragma unroll
  for (int c = 0; c < NIN; ++c) cfsec::dev::ld_chunk<W, true>(row0 + c * S + off, x[c]);
  if constexpr (EARLY)
#pragma unroll
    for (int j = 0; j < NCMP; ++j) cfsec::dev::ld_chunk<W, true>(row0 + (NIN + NOUT + j) * S + off, y[j]);
  uint32_t o[NOUT][W];
#pragma unroll
  for (int r = 0; r < NOUT; ++r)
#pragma unroll
    for (int w = 0; w < W; ++w) o[r][w] = x[4 * r][w] ^ x[4 * r + 1][w] ^ x[4 * r + 2][w] ^ x[4 * r + 3][w];
#pragma unroll
  for (int r = 0; r < NOUT; ++r) cfsec::dev::st_chunk<W, true>(const_cast<uint8_t*>(row0) + (NIN + r) * S + off, o[r]);
  if constexpr (!EARLY)
#pragma unroll
    for (int j = 0; j < NCMP; ++j) cfsec::dev::ld_chunk<W, true>(row0 + (NIN + NOUT + j) * S + off, y[j]);
  uint32_t diff = 0;
#pragma unroll
  for (int j = 0; j < NCMP; ++j)
#pragma unroll
    for (int w = 0; w < W; ++w) diff |= y[j][w] ^ x[j % NIN][w];
  if (diff == 0x12345678u) a.flags[bid] = 1;  // keeps the compares alive; never true for the fill
}

__global__ void fill(uint32_t* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = (uint32_t)(i * 2654435761u) ^ seed;
}

template <int W, bool EARLY>
void run(const char* name, std::vector<Args>& args) {
  const dim3 grid((unsigned)(S / (256 * 4 * W)), NB);
  for (int i = 0; i < 6; ++i) hipLaunchKernelGGL((kpat<W, EARLY>), grid, dim3(256), 0, 0, args[i % NT]);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int n = 60;
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < n; ++i) hipLaunchKernelGGL((kpat<W, EARLY>), grid, dim3(256), 0, 0, args[i % NT]);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / n, bytes = (double)ROWS * S * NB;
  printf("%-34s %8.1f us  %7.1f GB/s  %5.1f %% of 8 TB/s\n", name, us, bytes / (us * 1e-6) / 1e9,
         100.0 * bytes / (us * 1e-6) / 8e12);
}

int main() {
  std::vector<Args> args(NT);
  for (int t = 0; t < NT; ++t) {
    CK(hipMalloc(&args[t].base, (size_t)NB * ROWS * S));
    CK(hipMalloc(&args[t].flags, NB * 4));
    fill<<<4096, 256>>>((uint32_t*)args[t].base, (size_t)NB * ROWS * S / 4, 77u * t);
  }
  CK(hipDeviceSynchronize());
  for (int rep = 0; rep < 2; ++rep) {
    run<2, false>("W=2 compare rows after stores", args);
    run<2, true>("W=2 compare rows with inputs", args);
    run<1, false>("W=1 compare rows after stores", args);
    run<1, true>("W=1 compare rows with inputs", args);
    run<4, false>("W=4 compare rows after stores", args);
    run<4, true>("W=4 compare rows with inputs", args);
  }
  return 0;
}
