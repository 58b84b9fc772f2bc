// lut_probe.hip -- probe: the lookup-table product (csrc/gf_lut.hpp) against the library's launcher
// (launch_matvec: dyadic / fixed-K v_perm kernels) on the same stripes (dev tool, round 3).
// Encode bytes compared; Verify run on the encoded stripes (flags 0) and after a flipped byte (1).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../chubaofs_amd/csrc lut_probe.hip \
//         -L../chubaofs_amd -lcfsec -Wl,-rpath,'$ORIGIN/../chubaofs_amd' -o lut_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "gf256.hpp"
#include "gf_lut.hpp"
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

// PERM: the m rows are parity rows 7r mod 20 of the k + 20 code (no dyadic block structure left), as
// a repair's non-coset-aligned rows are; else parity rows 0..m-1.
template <int K, int M, int ML, int LA = 2, int LW = 4, bool PERM = false>
void run_case(const char* name, size_t S, int nst) {
  Matrix mat;
  build_matrix(K, K + (PERM ? 20 : M), mat);
  std::vector<uint8_t> coef((size_t)M * K);
  for (int r = 0; r < M; ++r)
    for (int c = 0; c < K; ++c) coef[(size_t)r * K + c] = mat.at(K + (PERM ? (7 * r) % 20 : r), c);
  const size_t pitch = (S + 255) / 256 * 256, per = pitch * (K + M), bytes = per * nst;
  uint8_t *buf, *ref;
  uint32_t* flags;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&ref, bytes));
  CK(hipMalloc(&flags, 4 * nst));
  std::vector<uint8_t> h(bytes);
  uint64_t z = 0x9E3779B97F4A7C15ull;
  for (auto& b : h) {
    z ^= z << 13, z ^= z >> 7, z ^= z << 17;
    b = (uint8_t)z;
  }
  CK(hipMemcpy(buf, h.data(), bytes, hipMemcpyHostToDevice));
  CK(hipMemcpy(ref, h.data(), bytes, hipMemcpyHostToDevice));
  std::vector<const uint8_t*> in((size_t)nst * K);
  std::vector<uint8_t*> out((size_t)nst * M);
  for (int s = 0; s < nst; ++s) {
    for (int c = 0; c < K; ++c) in[(size_t)s * K + c] = ref + s * per + c * pitch;
    for (int r = 0; r < M; ++r) out[(size_t)s * M + r] = ref + s * per + (K + r) * pitch;
  }
  MatVecJob job;
  job.k = K;
  job.m = M;
  job.coef = coef.data();
  job.len = S;
  job.nstripes = nst;
  job.in = in.data();
  job.out = out.data();
  dev::GfArgs a{};
  a.len = S;
  a.k = K;
  a.m = M;
  a.nstripes = nst;
  a.tiles_per_stripe = (uint32_t)((S + 4095) / 4096);
  a.flags = flags;
  a.sstride = (int64_t)per;
  a.tab = 1;
  for (int r = 0; r < M; ++r)
    for (int c = 0; c < K; ++c) a.coef[r * K + c] = coef[(size_t)r * K + c];
  for (int c = 0; c < K; ++c) a.ptr[c] = buf + c * pitch;
  for (int r = 0; r < M; ++r) a.ptr[K + r] = buf + (K + r) * pitch;
  const dim3 grid((unsigned)((S + 1024 * LW - 1) / (1024 * LW)), (unsigned)nst);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 50;
  const auto time = [&](auto&& f) {
    for (int i = 0; i < 10; ++i) f();
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e3 / reps;
  };
  const double us_lib = time([&] { CK(launch_matvec(job, 0)); });
  const double us_lut =
      time([&] { hipLaunchKernelGGL((lut::gf_lut_kernel<K, M, ML, MatVecMode::kStore, LA, LW>), grid, dim3(256), 0, 0, a); });
  CK(hipDeviceSynchronize());
  std::vector<uint8_t> a1(bytes), a2(bytes);
  CK(hipMemcpy(a1.data(), buf, bytes, hipMemcpyDeviceToHost));
  CK(hipMemcpy(a2.data(), ref, bytes, hipMemcpyDeviceToHost));
  bool same = std::memcmp(a1.data(), a2.data(), bytes) == 0;
  // verify: library vs lookup kernel on the encoded stripes
  MatVecJob vjob = job;
  vjob.mode = MatVecMode::kVerify;
  vjob.flags = flags;
  CK(hipMemset(flags, 0, 4 * nst));
  const double vus_lib = time([&] { CK(launch_matvec(vjob, 0)); });
  const double vus_lut =
      time([&] { hipLaunchKernelGGL((lut::gf_lut_kernel<K, M, ML, MatVecMode::kVerify, LA, LW>), grid, dim3(256), 0, 0, a); });
  std::vector<uint32_t> fl(nst);
  CK(hipMemcpy(fl.data(), flags, 4 * nst, hipMemcpyDeviceToHost));
  for (uint32_t f : fl) same = same && f == 0;
  // one flipped parity byte in the last stripe's last byte: only that flag
  const size_t at = (size_t)(nst - 1) * per + (K + M - 1) * pitch + S - 1;
  uint8_t byte;
  CK(hipMemcpy(&byte, buf + at, 1, hipMemcpyDeviceToHost));
  byte ^= 0x40;
  CK(hipMemcpy(buf + at, &byte, 1, hipMemcpyHostToDevice));
  CK(hipMemset(flags, 0, 4 * nst));
  hipLaunchKernelGGL((lut::gf_lut_kernel<K, M, ML, MatVecMode::kVerify, LA, LW>), grid, dim3(256), 0, 0, a);
  CK(hipMemcpy(fl.data(), flags, 4 * nst, hipMemcpyDeviceToHost));
  for (int s = 0; s < nst; ++s) same = same && fl[s] == (s == nst - 1 ? 1u : 0u);
  const double alg = (double)(K + M) * S * nst;
  const auto pct = [&](double us) { return alg / (us * 1e-6) / 8e12 * 100; };
  std::printf("%-22s k=%2d m=%2d ml=%2d la=%2d lw=%d  encode lib %7.1f us (%4.1f %%)  lut %7.1f us (%4.1f %%)   verify lib %7.1f (%4.1f %%)  lut %7.1f (%4.1f %%)  %s\n",
              name, K, M, ML, LA, LW, us_lib, pct(us_lib), us_lut, pct(us_lut), vus_lib, pct(vus_lib), vus_lut, pct(vus_lut),
              same ? "bytes+flags equal" : "DIFFER");
  CK(hipFree(buf));
  CK(hipFree(ref));
  CK(hipFree(flags));
}

int main(int argc, char** argv) {
  if (argc > 1 && std::strcmp(argv[1], "c5") == 0) {  // C5's row count: 16 inputs, 4 + 18 outputs
    run_case<16, 16, 16, 2, 2, true>("16x16 (perm rows)", 262144, 64);
    run_case<16, 22, 16, 2, 2, true>("16x22 hybrid 16+6", 262144, 64);
    run_case<16, 20, 16, 2, 2, true>("16x20 hybrid 16+4", 262144, 64);
    run_case<16, 18, 16, 2, 2, true>("16x18 hybrid 16+2", 262144, 64);
    return 0;
  }
  run_case<6, 6, 6, 2, 2>("EC6P6 (dyadic lib)", 174763, 256);
  run_case<6, 6, 6, 4, 2>("EC6P6 (dyadic lib)", 174763, 256);
  run_case<6, 10, 10, 2, 2>("EC6P10 (dyadic lib)", 699051, 32);
  run_case<6, 12, 12, 2, 2>("6x12 (EC6P10L2 fused)", 699051, 32);
  run_case<6, 12, 8, 2, 2>("6x12 (EC6P10L2 fused)", 699051, 32);
  run_case<16, 20, 16, 4, 2>("EC16P20 global", 262144, 64);
  run_case<12, 4, 4, 2, 2>("EC12P4 64MiB", 5592406, 8);
  run_case<6, 6, 6, 2, 2>("EC6P6 (dyadic lib)", 174763, 256);
  return 0;
}
