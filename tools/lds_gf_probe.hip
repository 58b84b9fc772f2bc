// lds_gf_probe.hip -- probe: part of a wide GF(2^8) product on the LDS pipe (dev tool, round-2 study).
//
// v_perm_b32 / v_bitop3_b32 issue at half rate on gfx950 (valu_rate.hip), so the many-output shapes
// (EC15P12: 15 x 12) are VALU-issue-bound.  Here G of the M/4 output groups take their products from
// LDS instead: per input byte x, T5[x & 31] ^ T3[x >> 5] where each table word holds the products of
// 4 outputs (one byte each) -- 32- and 8-word tables, conflict-free for ds_read_b32 -- XOR-accumulated
// byte-transposed (acc[k] = the 4 outputs' bytes at byte position k) and transposed once at the end.
// The other outputs take the shipped v_perm pair product.  Times the product against the library's
// fixed-K kernel (launch_matvec) on the same stripes and checks the bytes against it.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../chubaofs_amd/csrc lds_gf_probe.hip \
//         -L../chubaofs_amd -lcfsec -Wl,-rpath,'$ORIGIN/../chubaofs_amd' -o lds_gf_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "gf256.hpp"
#include "gf_device.hpp"
#include "kernels.hpp"

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

using namespace cfsec;
using dev::u32x4;

constexpr int kW = 2;  // dwords per lane per row (8 bytes), as the shipped fixed-K kernel for M >= 10

struct ProbeArgs {
  const uint8_t* in;   // stripe-major rows: stripe s, row c at in + (s*(K+M) + c) * pitch
  uint8_t* out;        // same buffer layout, rows K.. written
  size_t pitch, len;
  const uint32_t* lt;  // LDS tables: [K][G][40] words (T5[32], T3[8])
  const uint8_t* coef; // M x K
};

// K inputs, M outputs, G output groups of 4 (the first 4G outputs) from LDS tables, the rest v_perm.
template <int K, int M, int G>
__global__ __launch_bounds__(256) void hybrid_kernel(ProbeArgs a) {
  constexpr int MP = M - 4 * G;  // v_perm outputs
  __shared__ uint32_t lt[K * (G > 0 ? G : 1) * 40];
  __shared__ u32x4 tab01[K * (MP > 0 ? MP : 1)];
  __shared__ uint32_t tab2[K * (MP > 0 ? MP : 1)];
  for (int i = threadIdx.x; i < K * G * 40; i += 256) lt[i] = a.lt[i];
  for (int i = threadIdx.x; i < K * MP; i += 256) {
    const int c = i / (MP > 0 ? MP : 1), r = i % (MP > 0 ? MP : 1);  // slot c * MP + r
    dev::coef_tables(a.coef[(4 * G + r) * K + c], tab01[i], tab2[i]);
  }
  __syncthreads();
  const size_t s = blockIdx.y;
  const size_t off = ((size_t)blockIdx.x * 256 + threadIdx.x) * (4 * kW);
  if (off + 4 * kW > a.len) return;  // probe: lengths are multiples of the tile
  const uint8_t* base = a.in + s * (K + M) * a.pitch;
  uint32_t accT[G > 0 ? G : 1][kW][4];
  uint32_t accP[MP > 0 ? MP : 1][kW];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int w = 0; w < kW; ++w)
#pragma unroll
      for (int k = 0; k < 4; ++k) accT[g][w][k] = 0u;
#pragma unroll
  for (int r = 0; r < MP; ++r)
#pragma unroll
    for (int w = 0; w < kW; ++w) accP[r][w] = 0u;
  uint32_t x[K][kW];
  const auto load = [&](int c) {
    dev::ld_chunk<kW, true>(base + c * a.pitch + off, x[c]);
  };
  load(0);
  load(1);
#pragma unroll
  for (int c = 0; c < K; ++c) {
    if (c + 2 < K) load(c + 2);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (G > 0) {
#pragma unroll
      for (int w = 0; w < kW; ++w) {
        uint32_t lo = (x[c][w] << 2) & 0x7C7C7C7Cu, hi = (x[c][w] >> 3) & 0x1C1C1C1Cu;
        asm volatile("" : "+v"(lo), "+v"(hi));
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t a5 = (lo >> (8 * k)) & 0xFFu, a3 = (hi >> (8 * k)) & 0xFFu;
#pragma unroll
          for (int g = 0; g < G; ++g) {
            const uint32_t* t = lt + (c * G + g) * 40;
            const uint32_t v5 = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(t) + a5);
            const uint32_t v3 = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(t + 32) + a3);
            accT[g][w][k] ^= v5 ^ v3;
          }
        }
      }
    }
    if constexpr (MP > 0) {
      dev::mac_row_k<MP, kW>(accP, x[c], tab01 + c * MP, tab2 + c * MP);
#pragma unroll
      for (int r = 0; r < MP; ++r)
#pragma unroll
        for (int w = 0; w < kW; ++w) asm volatile("" : "+v"(accP[r][w]));
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  uint8_t* ob = a.out + s * (K + M) * a.pitch + K * a.pitch;
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      uint32_t o[kW];
#pragma unroll
      for (int w = 0; w < kW; ++w) {
        // output 4g+r, dword w: byte k = byte r of accT[g][w][k]
        o[w] = ((accT[g][w][0] >> (8 * r)) & 0xFFu) | (((accT[g][w][1] >> (8 * r)) & 0xFFu) << 8) |
               (((accT[g][w][2] >> (8 * r)) & 0xFFu) << 16) | (((accT[g][w][3] >> (8 * r)) & 0xFFu) << 24);
      }
      *reinterpret_cast<uint2*>(ob + (4 * g + r) * a.pitch + off) = uint2{o[0], o[1]};
    }
#pragma unroll
  for (int r = 0; r < MP; ++r)
    *reinterpret_cast<uint2*>(ob + (4 * G + r) * a.pitch + off) = uint2{accP[r][0], accP[r][1]};
}

template <int K, int M, int G>
void run_case(const char* name, size_t S, int nst) {
  const GF& gf = GF::get();
  Matrix mat;
  build_matrix(K, K + M, mat);
  std::vector<uint8_t> coef((size_t)M * K);
  for (int r = 0; r < M; ++r)
    for (int c = 0; c < K; ++c) coef[(size_t)r * K + c] = mat.at(K + r, c);
  std::vector<uint32_t> lt((size_t)K * (G > 0 ? G : 1) * 40, 0u);
  for (int c = 0; c < K; ++c)
    for (int g = 0; g < G; ++g)
      for (int e = 0; e < 40; ++e) {
        const uint32_t xv = e < 32 ? (uint32_t)e : (uint32_t)(e - 32) << 5;
        uint32_t w = 0;
        for (int r = 0; r < 4; ++r) w |= (uint32_t)gf.mul(coef[(size_t)(4 * g + r) * K + c], (uint8_t)xv) << (8 * r);
        lt[((size_t)c * G + g) * 40 + e] = w;
      }
  const size_t pitch = (S + 255) / 256 * 256, bytes = pitch * (K + M) * nst;
  uint8_t *buf, *ref;
  uint8_t* dcoef;
  uint32_t* dlt;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&ref, bytes));
  CK(hipMalloc(&dcoef, coef.size()));
  CK(hipMalloc(&dlt, lt.size() * 4));
  CK(hipMemcpy(dcoef, coef.data(), coef.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(dlt, lt.data(), lt.size() * 4, hipMemcpyHostToDevice));
  std::vector<uint8_t> h(bytes);
  uint64_t z = 0x9E3779B97F4A7C15ull;
  for (auto& b : h) {
    z ^= z << 13, z ^= z >> 7, z ^= z << 17;
    b = (uint8_t)z;
  }
  CK(hipMemcpy(buf, h.data(), bytes, hipMemcpyHostToDevice));
  CK(hipMemcpy(ref, h.data(), bytes, hipMemcpyHostToDevice));
  // the library's kernel on `ref`
  std::vector<const uint8_t*> in((size_t)nst * K);
  std::vector<uint8_t*> out((size_t)nst * M);
  for (int s = 0; s < nst; ++s) {
    for (int c = 0; c < K; ++c) in[(size_t)s * K + c] = ref + ((size_t)s * (K + M) + c) * pitch;
    for (int r = 0; r < M; ++r) out[(size_t)s * M + r] = ref + ((size_t)s * (K + M) + K + r) * pitch;
  }
  MatVecJob job;
  job.k = K;
  job.m = M;
  job.coef = coef.data();
  job.len = S;
  job.nstripes = nst;
  job.in = in.data();
  job.out = out.data();
  ProbeArgs pa{buf, buf, pitch, S, dlt, dcoef};
  const dim3 grid((unsigned)(S / (256 * 4 * kW)), (unsigned)nst);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 50;
  for (int i = 0; i < 20; ++i) CK(launch_matvec(job, 0));
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) CK(launch_matvec(job, 0));
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms_lib = 0;
  CK(hipEventElapsedTime(&ms_lib, e0, e1));
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL((hybrid_kernel<K, M, G>), grid, dim3(256), 0, 0, pa);
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((hybrid_kernel<K, M, G>), grid, dim3(256), 0, 0, pa);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms_h = 0;
  CK(hipEventElapsedTime(&ms_h, e0, e1));
  std::vector<uint8_t> a1(bytes), a2(bytes);
  CK(hipMemcpy(a1.data(), buf, bytes, hipMemcpyDeviceToHost));
  CK(hipMemcpy(a2.data(), ref, bytes, hipMemcpyDeviceToHost));
  bool same = true;
  for (int s = 0; s < nst && same; ++s)
    for (int r = 0; r < M && same; ++r)
      same = std::memcmp(a1.data() + ((size_t)s * (K + M) + K + r) * pitch,
                         a2.data() + ((size_t)s * (K + M) + K + r) * pitch, S) == 0;
  const double alg = (double)(K + M) * S * nst;
  std::printf("%-28s G=%d (%2d outputs on LDS)  library %8.1f us (%5.1f %%)  hybrid %8.1f us (%5.1f %%)  bytes %s\n", name,
              G, 4 * G, ms_lib * 1e3 / reps, alg / (ms_lib * 1e-3 / reps) / 8e12 * 100, ms_h * 1e3 / reps,
              alg / (ms_h * 1e-3 / reps) / 8e12 * 100, same ? "equal" : "DIFFER");
  CK(hipFree(buf));
  CK(hipFree(ref));
  CK(hipFree(dcoef));
  CK(hipFree(dlt));
}

int main() {
  const size_t S = 2048 * 170;  // ~4 MiB-blob shard, a multiple of the 2 KiB tile
  run_case<15, 12, 0>("EC15P12", S, 32);
  run_case<15, 12, 1>("EC15P12", S, 32);
  run_case<15, 12, 2>("EC15P12", S, 32);
  run_case<15, 12, 3>("EC15P12", S, 32);
  run_case<12, 8, 1>("EC12P9-like 12x8", S, 32);
  run_case<12, 8, 2>("EC12P9-like 12x8", S, 32);
  return 0;
}
