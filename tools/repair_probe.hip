// repair_probe.hip -- the C5 repair step of one EC16P20 bid batch, kernel by kernel (dev tool):
// 64 stripes of S = 262,144, erased {0, 1, 16, 17}, Reconstruct + Verify.  Times the plain fused
// product over the first 16 present rows (kStoreVerify, 20 rows), the 16x16-dyadic repair kernel
// (repair_dy16) with and without its compared rows, and the dyadic encode / verify of the same
// stripes; checks that the repair rebuilds the erased rows and flags nothing on a codeword.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../chubaofs_amd/csrc repair_probe.hip \
//         -L../chubaofs_amd -lcfsec -Wl,-rpath,'$ORIGIN/../chubaofs_amd' -o repair_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <vector>

#include "gf256.hpp"
#include "kernels.hpp"

using namespace cfsec;

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));  \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)

__global__ void fill(uint32_t* p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    p[i] = (uint32_t)(z ^ (z >> 31));
  }
}

int main() {
  const int K = 16, M = 20, T = 36, NS = 64;
  const size_t S = 262144, pitch = S;
  uint8_t* buf;
  CK(hipMalloc(&buf, pitch * T * NS));
  fill<<<4096, 256>>>((uint32_t*)buf, pitch * T * NS / 4);
  uint32_t* flags;
  CK(hipMalloc(&flags, 4 * NS));
  CK(hipMemset(flags, 0, 4 * NS));
  Matrix mat;
  build_matrix(K, T, mat);
  const auto row = [&](int s, int i) { return buf + ((size_t)s * T + i) * pitch; };
  // encode: a codeword in every stripe
  std::vector<uint8_t> P((size_t)M * K);
  for (int r = 0; r < M; ++r)
    for (int c = 0; c < K; ++c) P[(size_t)r * K + c] = mat.at(K + r, c);
  std::vector<const uint8_t*> ein((size_t)NS * K);
  std::vector<uint8_t*> eout((size_t)NS * M);
  for (int s = 0; s < NS; ++s) {
    for (int c = 0; c < K; ++c) ein[(size_t)s * K + c] = row(s, c);
    for (int r = 0; r < M; ++r) eout[(size_t)s * M + r] = row(s, K + r);
  }
  MatVecJob enc;
  enc.k = K, enc.m = M, enc.coef = P.data(), enc.len = S, enc.nstripes = NS, enc.in = ein.data(), enc.out = eout.data();
  CK(launch_matvec(enc, 0));
  MatVecJob ver = enc;
  ver.mode = MatVecMode::kVerify;
  ver.flags = flags;
  // the repair plan: inputs = first 16 present = data 2..15, parity 18, 19
  const int ins[16] = {2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 18, 19};
  Matrix sub(K, K), dec;
  for (int r = 0; r < K; ++r)
    for (int c = 0; c < K; ++c) sub.at(r, c) = mat.at(ins[r], c);
  if (!mat_invert(sub, dec)) return 1;
  const GF& gf = GF::get();
  std::vector<int> outs = {0, 1, 16, 17};
  for (int r = 20; r < 36; ++r) outs.push_back(r);
  std::vector<uint8_t> rows(outs.size() * K);
  for (size_t o = 0; o < outs.size(); ++o)
    for (int c = 0; c < K; ++c) {
      uint8_t v = 0;
      if (outs[o] < K) v = dec.at(outs[o], c);
      else
        for (int j = 0; j < K; ++j) v ^= gf.mul(mat.at(outs[o], j), dec.at(j, c));
      rows[o * K + c] = v;
    }
  std::vector<const uint8_t*> rin((size_t)NS * K);
  std::vector<uint8_t*> rout((size_t)NS * outs.size()), hout((size_t)NS * 22);
  for (int s = 0; s < NS; ++s) {
    for (int c = 0; c < K; ++c) rin[(size_t)s * K + c] = row(s, ins[c]);
    for (size_t o = 0; o < outs.size(); ++o) rout[s * outs.size() + o] = row(s, outs[o]);
    hout[(size_t)s * 22 + 0] = row(s, 0);
    hout[(size_t)s * 22 + 1] = row(s, 1);
    for (int r = 0; r < 20; ++r) hout[(size_t)s * 22 + 2 + r] = row(s, K + r);
  }
  MatVecJob gen;
  gen.k = K, gen.m = (int)outs.size(), gen.coef = rows.data(), gen.len = S, gen.nstripes = NS, gen.in = rin.data();
  gen.out = rout.data(), gen.mode = MatVecMode::kStoreVerify, gen.nstore = 4, gen.flags = flags;
  std::vector<uint8_t> hc((size_t)22 * K);
  memcpy(hc.data(), P.data(), 20 * K);
  for (int q = 0; q < 2; ++q) memcpy(hc.data() + (20 + q) * K, dec.row(q), K);
  Dy16RepairJob rep;
  rep.nd = 2, rep.coef = hc.data(), rep.len = S, rep.nstripes = NS, rep.in = rin.data(), rep.out = hout.data();
  rep.flags = flags;
  rep.src[0] = 16, rep.src[1] = 17;
  for (int i = 2; i < 16; ++i) rep.src[i] = (uint8_t)(i - 2);
  rep.pstore = 0x3;
  rep.pcmp = 0xFFFF0u;
  Dy16RepairJob rep_nc = rep;
  rep_nc.pcmp = 0;
  // correctness: zero the erased rows of every stripe, repair, compare with the codeword
  std::vector<uint8_t> want(4 * S), got(4 * S);
  for (int i = 0; i < 4; ++i) CK(hipMemcpy(want.data() + i * S, row(NS - 1, outs[i]), S, hipMemcpyDeviceToHost));
  for (int s = 0; s < NS; ++s)
    for (int i = 0; i < 4; ++i) CK(hipMemset(row(s, outs[i]), 0, S));
  CK(launch_dy16_repair(rep, 0));
  for (int i = 0; i < 4; ++i) CK(hipMemcpy(got.data() + i * S, row(NS - 1, outs[i]), S, hipMemcpyDeviceToHost));
  std::vector<uint32_t> hf(NS);
  CK(hipMemcpy(hf.data(), flags, 4 * NS, hipMemcpyDeviceToHost));
  int nflag = 0;
  for (uint32_t f : hf) nflag += f != 0;
  printf("repair_dy16 rebuilds the erased rows: %s, stripes flagged: %d\n", want == got ? "yes" : "NO", nflag);

  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct V {
    const char* name;
    std::function<void()> f;
    double rows;  // rows moved per stripe
  };
  std::vector<V> vs = {
      {"fused kStoreVerify 16x20", [&] { CK(launch_matvec(gen, 0)); }, 36},
      {"repair_dy16 (store 4, cmp 16)", [&] { CK(launch_dy16_repair(rep, 0)); }, 36},
      {"repair_dy16, no compares", [&] { CK(launch_dy16_repair(rep_nc, 0)); }, 20},
      {"dy16 verify 16x20", [&] { CK(launch_matvec(ver, 0)); }, 36},
      {"dy16 encode 16x20", [&] { CK(launch_matvec(enc, 0)); }, 36},
  };
  for (int i = 0; i < 200; ++i) vs[0].f();
  for (auto& v : vs) {
    for (int i = 0; i < 5; ++i) v.f();
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < 50; ++i) v.f();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / 50;
    printf("%-32s %8.1f us  %5.1f%% of 8 TB/s\n", v.name, us, v.rows * S * NS / (us * 1e-6) / 8e12 * 100);
  }
  return 0;
}
