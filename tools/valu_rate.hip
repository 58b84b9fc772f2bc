// valu_rate.hip -- issue rate of the VALU instructions the GF and CRC kernels are made of (dev tool).
//
// Every lane runs 8 independent chains of one instruction kind for `iters` rounds; the grid fills the
// chip (4096 workgroups x 256 threads = 16 waves per CU).  Reports wave-instructions per cycle per
// SIMD from the kernel time and the clock, for v_perm_b32, v_bitop3_b32, v_xor_b32, v_and_b32 with
// SDWA-free operands, v_bfe_u32 and ds_read_b32 (conflict-free, as the CRC step issues them).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 valu_rate.hip -o valu_rate
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#ifndef NCH
#define NCH 8  // independent chains per lane
#endif
#ifndef NWG
#define NWG 4096  // workgroups of 256 threads
#endif

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                              \
    }                                                                            \
  } while (0)

template <int KIND>
__global__ __launch_bounds__(256) void rate_kernel(uint32_t* out, int iters, uint32_t seed) {
  __shared__ uint32_t tab[32 * 35];
  for (int i = threadIdx.x; i < 32 * 35; i += 256) tab[i] = i * 2654435761u;
  __syncthreads();
  uint32_t v[NCH], s = seed ^ (threadIdx.x * 0x9E3779B9u) ^ blockIdx.x;
#pragma unroll
  for (int j = 0; j < NCH; ++j) v[j] = s * (j + 1);
  const uint32_t a = seed * 3u, b = seed * 5u;
  uint32_t sel[NCH];
#pragma unroll
  for (int j = 0; j < NCH; ++j) sel[j] = (s >> (j % 24)) & 0x07070707u;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      if constexpr (KIND == 0) v[j] = __builtin_amdgcn_perm(a, v[j], sel[j]);          // v_perm_b32
      else if constexpr (KIND == 1) v[j] = __builtin_amdgcn_bitop3_b32(v[j], a, b, 0x96);  // v_bitop3_b32
      else if constexpr (KIND == 2) v[j] = (v[j] ^ a) + b;                            // v_xad_u32 or xor + add
      else if constexpr (KIND == 3) v[j] = __builtin_amdgcn_ubfe(v[j], 3, 29);         // v_bfe_u32
      else if constexpr (KIND == 4) {  // ds_read_b32 at a 5-bit index (conflict-free), chained
        v[j] = tab[(j % 35) * 32 + (v[j] & 31u)];
      } else if constexpr (KIND == 5) {  // v_xor_b32 (VOP2), one per chain step
        v[j] ^= sel[j];
        asm volatile("" : "+v"(v[j]));
      } else if constexpr (KIND == 6) {  // v_add3_u32 (VOP3, 3 VGPR sources)
        v[j] = __builtin_amdgcn_perm(0u, 0u, 0u) + v[j] + sel[j] + a;
        asm volatile("" : "+v"(v[j]));
      } else {  // v_and_b32 (VOP2)
        v[j] &= sel[j] | 0x80000000u;
        asm volatile("" : "+v"(v[j]));
      }
    }
  }
  uint32_t r = 0;
#pragma unroll
  for (int j = 0; j < NCH; ++j) r ^= v[j];
  if (r == 0x12345678u) out[blockIdx.x] = r;
}

template <int KIND>
float run(uint32_t* out, int iters) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(rate_kernel<KIND>, dim3(NWG), dim3(256), 0, 0, out, iters, 7u);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(rate_kernel<KIND>, dim3(NWG), dim3(256), 0, 0, out, iters, 7u + r);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / 5;
}

int main() {
  uint32_t* out;
  CK(hipMalloc(&out, 4096 * 4));
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const double clk = p.clockRate * 1e3;  // Hz (peak)
  const int iters = 4096;
  const double waves = NWG * 4.0, simds = p.multiProcessorCount * 4.0;
  const char* names[] = {"v_perm_b32", "v_bitop3_b32", "xor+add (2 VOP2)", "v_lshrrev (bfe 3,29)", "ds_read_b32 5-bit",
                         "v_xor_b32 (VOP2)", "v_add3_u32 (VOP3)", "v_and_b32 (VOP2)"};
  const float ms[] = {run<0>(out, iters), run<1>(out, iters), run<2>(out, iters), run<3>(out, iters), run<4>(out, iters),
                      run<5>(out, iters), run<6>(out, iters), run<7>(out, iters)};
  std::printf("CUs %d, peak clock %.0f MHz; %d waves x %d rounds x %d chains\n", p.multiProcessorCount, clk / 1e6,
              (int)waves, iters, NCH);
  for (int k = 0; k < 8; ++k) {
    const double ops = waves * iters * NCH;  // wave-instructions of the kind (plus a helper op for 0, 3)
    const double cyc = ms[k] * 1e-3 * clk;
    std::printf("%-22s %8.3f ms  %6.3f wave-ops / cycle / SIMD at peak clock\n", names[k], ms[k], ops / cyc / simds);
  }
  return 0;
}
