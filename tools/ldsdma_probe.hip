// ldsdma_probe.hip -- the access-pattern ceiling of the headline shape (EC12P4: 12 rows read, 4
// written, 8 stripes of ~5.6 MB rows, three batches rotated) with the rows streamed into LDS by
// global_load_lds (no registers held by loads in flight) by persistent waves, against the shipped
// launcher on the same buffers (dev probe, round 4).  The arithmetic is trivial (every output row
// the XOR of the 12 inputs and a constant): only the memory schedule is measured.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../chubaofs_amd/csrc ldsdma_probe.hip \
//         -L../chubaofs_amd -lcfsec -Wl,-rpath,'$ORIGIN/../chubaofs_amd' -o ldsdma_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "gf256.hpp"
#include "kernels.hpp"

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

constexpr int K = 12, M = 4, ROWS = K + M, NB = 8, NT = 3;
constexpr size_t S = 2731 * 2048;  // the headline's 5,592,406 B rounded up to whole 2 KiB tiles

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void glds16(const uint8_t* g, uint8_t* l) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}
__device__ __forceinline__ void glds16nt(const uint8_t* g, uint8_t* l) {
  // aux bit 1 = slc, 2 = nt on gfx950's LDS-DMA form (the same cache policy bits as the load)
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)l, 16, 0, 2);
}
constexpr unsigned waitcnt_vm(unsigned n) { return (n & 0xFu) | (0x7u << 4) | (0xFu << 8) | ((n >> 4) << 14); }

// W waves per workgroup (one workgroup per CU), RB bytes of each row per wave tile (16 B per lane
// per 1 KiB), NBUF tile buffers per wave in LDS (NBUF - 1 tiles prefetched ahead), NTL: LDS-DMA
// with the non-temporal bit.
template <int W, int RB, int NBUF, bool NTL>
__global__ __launch_bounds__(64 * W) void triv_glds(uint8_t* base, uint32_t tps, uint32_t ntiles) {
  constexpr int IPR = RB / 1024;
  constexpr unsigned AHEAD = (NBUF - 1) * (K + M) * IPR;  // vector memory ops issued after a tile's prefetch
  static_assert(AHEAD <= 63, "vmcnt");
  __shared__ __attribute__((aligned(16))) uint8_t lds[W][NBUF][K * RB];
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * W;
  const auto rowp = [&](uint32_t t, int i) -> uint8_t* {
    const uint32_t s = t / tps, c = t % tps;
    return base + ((size_t)s * ROWS + i) * S + (size_t)c * RB + lane * 16;
  };
  const auto pf = [&](uint32_t t, int b) {
#pragma unroll
    for (int i = 0; i < K; ++i)
#pragma unroll
      for (int h = 0; h < IPR; ++h) {
        if constexpr (NTL) glds16nt(rowp(t, i) + h * 1024, &lds[wave][b][i * RB + h * 1024]);
        else glds16(rowp(t, i) + h * 1024, &lds[wave][b][i * RB + h * 1024]);
      }
  };
  uint32_t t = blockIdx.x * W + wave;
  if (t >= ntiles) return;
#pragma unroll
  for (int j = 0; j < NBUF - 1; ++j) {
    const uint32_t tj = t + j * nw;
    pf(tj < ntiles ? tj : t, j);
  }
  int b = 0;
  for (uint32_t j = 0; t < ntiles; t += nw, ++j) {
    const uint32_t tn = t + (NBUF - 1) * nw;
    pf(tn < ntiles ? tn : t, (b + NBUF - 1) % NBUF);
    // the first NBUF - 1 tiles have fewer stores behind their prefetch
    if (NBUF == 1) __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
    else if (j == 0) __builtin_amdgcn_s_waitcnt(waitcnt_vm((NBUF - 1) * K * IPR));
    else if (NBUF > 2 && j == 1) __builtin_amdgcn_s_waitcnt(waitcnt_vm((NBUF - 1) * K * IPR + M * IPR));
    else __builtin_amdgcn_s_waitcnt(waitcnt_vm(AHEAD));
    uint32_t o[IPR][4];
#pragma unroll
    for (int h = 0; h < IPR; ++h) o[h][0] = o[h][1] = o[h][2] = o[h][3] = 0;
#pragma unroll
    for (int i = 0; i < K; ++i)
#pragma unroll
      for (int h = 0; h < IPR; ++h) {
        const u32x4 v = *reinterpret_cast<const u32x4*>(&lds[wave][b][i * RB + h * 1024 + lane * 16]);
        o[h][0] ^= v.x, o[h][1] ^= v.y, o[h][2] ^= v.z, o[h][3] ^= v.w;
      }
    __builtin_amdgcn_s_waitcnt(0xC07F);
#pragma unroll
    for (int r = 0; r < M; ++r)
#pragma unroll
      for (int h = 0; h < IPR; ++h)
        __builtin_nontemporal_store(u32x4{o[h][0] ^ r, o[h][1], o[h][2], o[h][3]},
                                    reinterpret_cast<u32x4*>(rowp(t, K + r) + h * 1024));
    b = (b + 1) % NBUF;
  }
}

// The register-load form at the same persistent grid (reference point): the wave loads its 12
// rows into registers, XORs and stores.
template <int W>
__global__ __launch_bounds__(64 * W) void triv_reg(uint8_t* base, uint32_t tps, uint32_t ntiles) {
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * W;
  for (uint32_t t = blockIdx.x * W + wave; t < ntiles; t += nw) {
    const uint32_t s = t / tps, c = t % tps;
    uint8_t* r0 = base + (size_t)s * ROWS * S + (size_t)c * 1024 + lane * 16;
    u32x4 x[K];
#pragma unroll
    for (int i = 0; i < K; ++i) x[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(r0 + i * S));
    u32x4 o = x[0];
#pragma unroll
    for (int i = 1; i < K; ++i) o ^= x[i];
#pragma unroll
    for (int r = 0; r < M; ++r)
      __builtin_nontemporal_store(u32x4{o.x ^ r, o.y, o.z, o.w}, reinterpret_cast<u32x4*>(r0 + (K + r) * S));
  }
}

__global__ void fill(uint32_t* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 0x9E3779B9u ^ seed;
    x ^= x >> 16; x *= 0x85EBCA6Bu; x ^= x >> 13;
    p[i] = x;
  }
}

static int ncu() {
  int dev = 0, n = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
  return n;
}

template <typename F>
static double timed(F launch, int reps) {
  for (int i = 0; i < 6; ++i) launch(i % NT);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < reps; ++i) launch(i % NT);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return ms * 1e3 / reps;
}

static std::vector<uint8_t*> g_bufs;

// row 0 of stripe NB-1 of batch 0 against the XOR of its inputs (the schedule's waits are right)
static bool check_triv() {
  std::vector<uint8_t> in(K * S), out(S);
  const uint8_t* s0 = g_bufs[0] + (size_t)(NB - 1) * ROWS * S;
  CK(hipMemcpy(in.data(), s0, K * S, hipMemcpyDeviceToHost));
  CK(hipMemcpy(out.data(), s0 + K * S, S, hipMemcpyDeviceToHost));
  for (size_t j = 0; j < S; ++j) {
    uint8_t v = 0;
    for (int i = 0; i < K; ++i) v ^= in[i * S + j];
    if (v != out[j]) return false;
  }
  return true;
}

template <int W, int RB, int NBUF, bool NTL>
static void run_glds(const char* name, double algo) {
  const uint32_t tps = (uint32_t)(S / RB), nt = tps * NB;
  const int g = ncu();
  for (int t = 0; t < NT; ++t) CK(hipMemset(g_bufs[t] + K * S, 0, M * S));
  auto launch = [&](int t) { hipLaunchKernelGGL((triv_glds<W, RB, NBUF, NTL>), dim3(g), dim3(64 * W), 0, 0, g_bufs[t], tps, nt); };
  launch(0);
  CK(hipDeviceSynchronize());
  const bool ok = check_triv();
  for (int rep = 0; rep < 3; ++rep) {
    const double us = timed(launch, 40);
    printf("%-40s %8.1f us  %7.1f GB/s  %5.1f %% of 8 TB/s  %s\n", name, us, algo / us / 1e3, algo / us / 8e4, ok ? "ok" : "WRONG");
  }
}

template <int W>
static void run_reg(const char* name, double algo, int per_cu) {
  const uint32_t tps = (uint32_t)(S / 1024), nt = tps * NB;
  const int g = ncu() * per_cu;
  for (int t = 0; t < NT; ++t) CK(hipMemset(g_bufs[t] + K * S, 0, M * S));
  auto launch = [&](int t) { hipLaunchKernelGGL((triv_reg<W>), dim3(g), dim3(64 * W), 0, 0, g_bufs[t], tps, nt); };
  launch(0);
  CK(hipDeviceSynchronize());
  const bool ok = check_triv();
  for (int rep = 0; rep < 3; ++rep) {
    const double us = timed(launch, 40);
    printf("%-40s %8.1f us  %7.1f GB/s  %5.1f %% of 8 TB/s  %s\n", name, us, algo / us / 1e3, algo / us / 8e4, ok ? "ok" : "WRONG");
  }
}

int main() {
  g_bufs.resize(NT);
  const size_t bytes = (size_t)NB * ROWS * S;
  for (int t = 0; t < NT; ++t) {
    CK(hipMalloc(&g_bufs[t], bytes));
    fill<<<4096, 256>>>((uint32_t*)g_bufs[t], bytes / 4, 0x9E3779B9u * (t + 1));
  }
  CK(hipDeviceSynchronize());
  const double algo = (double)NB * ROWS * S;
  printf("EC12P4 access pattern, %d stripes x %d rows x %zu B, %d batches rotated, %d CUs\n", NB, ROWS, S, NT, ncu());
  // the shipped launcher (EC12P4 parity of KRS buildMatrix) on the same rows
  cfsec::Matrix mat;
  if (!cfsec::build_matrix(K, ROWS, mat)) return 1;
  std::vector<std::vector<const uint8_t*>> lin(NT);
  std::vector<std::vector<uint8_t*>> lout(NT);
  std::vector<cfsec::MatVecJob> jobs(NT);
  for (int t = 0; t < NT; ++t) {
    for (int b = 0; b < NB; ++b) {
      for (int c = 0; c < K; ++c) lin[t].push_back(g_bufs[t] + ((size_t)b * ROWS + c) * S);
      for (int r = 0; r < M; ++r) lout[t].push_back(g_bufs[t] + ((size_t)b * ROWS + K + r) * S);
    }
    cfsec::MatVecJob& j = jobs[t];
    j.k = K;
    j.m = M;
    j.coef = mat.row(K);
    j.len = S;
    j.nstripes = NB;
    j.in = lin[t].data();
    j.out = lout[t].data();
  }
  for (int rep = 0; rep < 3; ++rep) {
    const double us = timed([&](int t) { CK(cfsec::launch_matvec(jobs[t], 0)); }, 40);
    printf("%-40s %8.1f us  %7.1f GB/s  %5.1f %% of 8 TB/s\n", "library launch_matvec (EC12P4)", us, algo / us / 1e3, algo / us / 8e4);
  }
  run_reg<4>("triv reg loads, 4 waves x 2/CU", algo, 2);
  run_reg<4>("triv reg loads, 4 waves x 4/CU", algo, 4);
  run_glds<4, 1024, 2, false>("glds W4 RB1K NBUF2", algo);
  run_glds<4, 1024, 3, false>("glds W4 RB1K NBUF3", algo);
  run_glds<6, 1024, 2, false>("glds W6 RB1K NBUF2", algo);
  run_glds<8, 1024, 1, false>("glds W8 RB1K NBUF1 (no overlap)", algo);
  run_glds<3, 2048, 2, false>("glds W3 RB2K NBUF2", algo);
  run_glds<6, 1024, 2, true>("glds W6 RB1K NBUF2 nt", algo);
  run_glds<4, 1024, 3, true>("glds W4 RB1K NBUF3 nt", algo);
  for (int t = 0; t < NT; ++t) CK(hipFree(g_bufs[t]));
  return 0;
}
