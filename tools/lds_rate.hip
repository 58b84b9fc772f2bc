// lds_rate.hip -- issue rate of nibble-table lookups on gfx950 (dev tool, round 3).
//
// The lookup kernels (gf_crc.hpp gf_crc_lds_kernel, gf_lut.hpp) read 16-entry tables of EW-word
// entries at a data-dependent nibble: conflict-free by the bank rule, 2 (b32, b64) or 4 (b128) LDS
// cycles per wave-instruction.  Measured in the kernels they reach ~50 % of that.  This loop does
// only the lookups: per step 8 reads at addresses from one data word (as the kernels do), the
// results XOR-accumulated; the data word is rotated per step so nothing is loop-invariant.
// Variants: EW, workgroups per CU (occupancy), and ADDR = 0 (addresses from one shift+mask per
// read) / 1 (the kernels' form: 2 masks per word, one byte extract per read).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 lds_rate.hip -o lds_rate
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kTables = 24;  // distinct 16-entry tables (positions x nibbles of the kernels)

template <int EW>
__device__ __forceinline__ void lookup(const char* T, uint32_t off, uint32_t (&acc)[EW]) {
  if constexpr (EW == 1) {
    acc[0] ^= *reinterpret_cast<const uint32_t*>(T + off);
  } else if constexpr (EW == 2) {
    const u32x2 v = *reinterpret_cast<const u32x2*>(T + off);
    acc[0] ^= v.x;
    acc[1] ^= v.y;
  } else {
    const u32x4 v = *reinterpret_cast<const u32x4*>(T + off);
    acc[0] ^= v.x;
    acc[1] ^= v.y;
    acc[2] ^= v.z;
    acc[3] ^= v.w;
  }
}

template <int EW, int DEP>
__global__ __launch_bounds__(256) void rate_kernel(uint32_t* out, int iters, uint32_t seed) {
  constexpr int EB = 4 * EW, SH = EW == 1 ? 2 : (EW == 2 ? 3 : 4);
  __shared__ __attribute__((aligned(16))) uint32_t T[kTables * 16 * EW];
  for (int i = threadIdx.x; i < kTables * 16 * EW; i += 256) T[i] = i * 0x9E3779B9u;
  __syncthreads();
  uint32_t d[4];
  uint32_t z = seed ^ (blockIdx.x * 256 + threadIdx.x) * 0x85EBCA6Bu;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    z ^= z << 13, z ^= z >> 17, z ^= z << 5;
    d[w] = z;
  }
  uint32_t acc[4][EW];
#pragma unroll
  for (int w = 0; w < 4; ++w)
#pragma unroll
    for (int q = 0; q < EW; ++q) acc[w][q] = 0u;
  const char* Tc = reinterpret_cast<const char*>(T);
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const uint32_t v = d[w];
      uint32_t lo = (v << SH) & (0x0F0F0F0Fu << SH), hi = (SH == 4 ? v : (v >> (4 - SH))) & (0x0F0F0F0Fu << SH);
      asm volatile("" : "+v"(lo), "+v"(hi));
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int t = (w * 8 + 2 * j) % kTables;
        lookup<EW>(Tc + t * 16 * EB, (lo >> (8 * j)) & 0xFFu, acc[w]);
        lookup<EW>(Tc + ((t + 1) % kTables) * 16 * EB, (hi >> (8 * j)) & 0xFFu, acc[w]);
      }
      // DEP: the next step's word depends on this one's reads (a latency chain); else independent
      d[w] = __builtin_amdgcn_alignbit(v, v, 7) ^ (DEP ? acc[w][0] : (uint32_t)it);
    }
  }
  uint32_t r = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w)
#pragma unroll
    for (int q = 0; q < EW; ++q) r ^= acc[w][q];
  if (r == 0x12345678u) out[blockIdx.x] = r;
}

template <int EW, int DEP>
void run(const char* name, int wg_per_cu) {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint32_t* out;
  CK(hipMalloc(&out, 4 << 20));
  const int blocks = cus * wg_per_cu, iters = 2048;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((rate_kernel<EW, DEP>), dim3(blocks), dim3(256), 0, 0, out, iters, 1u);
  CK(hipEventRecord(e0));
  const int reps = 10;
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((rate_kernel<EW, DEP>), dim3(blocks), dim3(256), 0, 0, out, iters, 1u);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double reads_per_cu = (double)wg_per_cu * 4 /*waves*/ * iters * 32.0;  // wave-instructions
  const double ns = ms * 1e6 / reps;
  const double cyc = ns * 2.4;  // peak clock
  const double lds_cyc = reads_per_cu * (EW == 4 ? 4 : 2);
  std::printf("%-6s dep %d wg/CU %2d (%2d waves/SIMD)  %8.1f us  %.3f wave-reads/cycle/CU at 2.4 GHz  = %5.1f %% of the LDS-array rate\n",
              name, DEP, wg_per_cu, wg_per_cu, ns / 1e3, reads_per_cu / cyc, 100 * lds_cyc / cyc);
  CK(hipFree(out));
}

int main() {
  for (int wg : {1, 2, 3, 4, 6, 8}) run<1, 0>("b32", wg);
  for (int wg : {1, 2, 3, 4, 6, 8}) run<2, 0>("b64", wg);
  for (int wg : {1, 2, 3, 4, 6, 8}) run<4, 0>("b128", wg);
  for (int wg : {1, 2, 3, 4, 8}) run<2, 1>("b64", wg);
  for (int wg : {1, 2, 3, 4, 8}) run<4, 1>("b128", wg);
  return 0;
}
