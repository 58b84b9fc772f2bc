// gf_shapes.hip -- times the shipped kernel policy over every code-mode shape (dev tool).
//
// For each (k, m, S, stripes): one launch = m outputs from k inputs over `stripes` stripes;
// reports us/launch, algorithmic GB/s ((k+m)*S*stripes per launch) and % of 8 TB/s, plus the
// VALU lane-op estimate of the v_perm arithmetic.  Correctness of the same kernels is covered
// by tests/test_gpu_parity.py; this tool only times.
//
// Encode (kStore) and Verify (kVerify) per shape.  Links the shipped library:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../chubaofs_amd/csrc gf_shapes.hip \
//         -L../chubaofs_amd -lcfsec -Wl,-rpath,'$ORIGIN/../chubaofs_amd' -o gf_shapes
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "gf256.hpp"
#include "bs_net_ec16p20l2.hpp"
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
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    p[i] = (uint32_t)(z ^ (z >> 31));
  }
}

struct Shape {
  const char* name;
  int k, m;
  size_t S;
  int stripes;
};

int main() {
  const Shape shapes[] = {
      {"EC12P4 encode 64MiB blob", 12, 4, 5592406, 8},
      {"EC12P4 encode 4MiB blob", 12, 4, 349526, 128},
      {"EC6P6 encode 1MiB blob", 6, 6, 174763, 256},
      {"EC6P10 global encode", 6, 10, 699051, 32},
      {"EC6P10L2 fused encode", 6, 12, 699051, 32},
      {"EC6P10L2 local repair (8,1)", 8, 1, 699051, 64},
      {"EC16P20 global encode", 16, 20, 262144, 64},
      {"EC16P20L2 fused encode", 16, 22, 262144, 64},
      {"EC16P20L2 repair 4 erased", 16, 4, 262144, 64},
      {"EC16P20 repair 8 rows", 16, 8, 262144, 64},
      {"EC16P20 repair 16 rows", 16, 16, 262144, 64},
      {"EC15P12 encode", 15, 12, 349526, 32},
      {"EC16P4 encode", 16, 4, 262144, 64},
      {"EC12P9 encode", 12, 9, 349526, 32},
      {"EC10P4 encode", 10, 4, 419431, 32},
      {"EC6P3 encode", 6, 3, 699051, 32},
      {"EC6P8 encode", 6, 8, 699051, 32},
      {"EC4P4 encode", 4, 4, 1048576, 16},
      {"EC3P3 encode", 3, 3, 1398102, 16},
  };
  size_t maxbytes = 0;
  for (auto& s : shapes) maxbytes = std::max(maxbytes, ((s.S + 255) / 256 * 256) * (s.k + s.m) * s.stripes);
  uint8_t* buf;
  CK(hipMalloc(&buf, maxbytes));
  fill<<<4096, 256>>>((uint32_t*)buf, maxbytes / 4);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  uint32_t* flags;
  CK(hipMalloc(&flags, 4096));
  uint32_t* crcs;
  CK(hipMalloc(&crcs, 4 * 64 * 1024));
  printf("%-30s %3s %3s %9s %4s %9s %8s %6s %9s %9s %6s %9s %6s %11s\n", "shape", "k", "m", "S", "nst", "us/launch", "GB/s",
         "%8TB", "Tlaneop/s", "verify us", "%8TB", "+crc us", "%8TB", "crc-only us");  // + the +crc route
  for (auto& sh : shapes) {
    const size_t pitch = (sh.S + 255) / 256 * 256;
    Matrix mat;
    build_matrix(sh.k, sh.k + sh.m, mat);
    const int per = sh.k + sh.m;
    std::vector<const uint8_t*> in((size_t)sh.stripes * sh.k);
    std::vector<uint8_t*> out((size_t)sh.stripes * sh.m);
    for (int s = 0; s < sh.stripes; ++s) {
      uint8_t* base = buf + size_t(s) * per * pitch;
      for (int c = 0; c < sh.k; ++c) in[(size_t)s * sh.k + c] = base + c * pitch;
      for (int r = 0; r < sh.m; ++r) out[(size_t)s * sh.m + r] = base + (sh.k + r) * pitch;
    }
    std::vector<uint8_t> coef((size_t)sh.m * sh.k);
    for (int r = 0; r < sh.m; ++r)
      for (int c = 0; c < sh.k; ++c) coef[(size_t)r * sh.k + c] = mat.at(sh.k + r, c);
    if (sh.k == 16 && sh.m == 22)  // EC16P20L2's fused encode: the 2 AZ-local rows over the data, as the engine builds them
      for (int r = 20; r < 22; ++r)
        for (int c = 0; c < 16; ++c) coef[(size_t)r * 16 + c] = dev::kBsEc16p20l2Rows[r][c];
    if (sh.k == 6 && sh.m == 12) {  // EC6P10L2's fused encode: the 2 AZ-local rows over the data (lrcencoder.go)
      // AZ a's local stripe = data [3a, 3a+3) + global parities [5a, 5a+5) (N/AZ, M/AZ per AZ), one
      // local parity from RS(8, 1); over the data: l[c] = sum over the stripe's members of their row
      Matrix lm;
      build_matrix(8, 9, lm);
      const GF& gf = GF::get();
      for (int a = 0; a < 2; ++a)
        for (int c = 0; c < 6; ++c) {
          uint8_t v = 0;
          for (int j = 0; j < 3; ++j)
            if (c == 3 * a + j) v ^= lm.at(8, j);
          for (int j = 0; j < 5; ++j) v ^= gf.mul(lm.at(8, 3 + j), mat.at(6 + 5 * a + j, c));
          coef[(size_t)(10 + a) * 6 + c] = v;
        }
    }
    MatVecJob job;
    job.k = sh.k;
    job.m = sh.m;
    job.coef = coef.data();
    job.len = sh.S;
    job.nstripes = sh.stripes;
    job.in = in.data();
    job.out = out.data();
    auto launch_all = [&]() { CK(launch_matvec(job, 0)); };  // the shipped launcher
    MatVecJob vjob = job;
    vjob.mode = MatVecMode::kVerify;
    vjob.flags = flags;
    static float settled = getenv("GF_SHAPES_NOSETTLE") ? 1e9f : 0.f;  // ~300 ms of load once (clock ramp)
    while (settled < 300) {
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < 20; ++i) launch_all();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      settled += ms;
    }
    for (int i = 0; i < 5; ++i) launch_all();
    const int reps = getenv("GF_SHAPES_REPS") ? atoi(getenv("GF_SHAPES_REPS")) : 100;
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) launch_all();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / reps;
    for (int i = 0; i < 3; ++i) CK(launch_matvec(vjob, 0));  // warm (first launch of a kernel loads its code)
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) CK(launch_matvec(vjob, 0));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float vms;
    CK(hipEventElapsedTime(&vms, e0, e1));
    const double vus = vms * 1e3 / reps;
    // encode + crc32.ChecksumIEEE of every shard: the fused kernel where it takes the job (same
    // algorithmic bytes as the encode), else what the engine runs then -- the product and the
    // standalone checksum pass (route 's')
    double cus = 0;
    std::vector<const uint8_t*> all;
    for (int s = 0; s < sh.stripes; ++s) {
      for (int c = 0; c < sh.k; ++c) all.push_back(in[(size_t)s * sh.k + c]);
      for (int r = 0; r < sh.m; ++r) all.push_back(out[(size_t)s * sh.m + r]);
    }
    std::vector<int> slot(sh.k + sh.m);
    for (int i = 0; i < sh.k + sh.m; ++i) slot[i] = i;
    const bool fused = matvec_crc_accepts(job, sh.k + sh.m, slot.data());
    const auto with_crc = [&]() {
      if (fused) {
        CK(launch_matvec_crc(job, crcs, sh.k + sh.m, slot.data(), 0));
      } else {
        CK(launch_matvec(job, 0));
        CK(launch_crc32(all.data(), sh.S, (int)all.size(), crcs, 0));
      }
    };
    {
      for (int i = 0; i < 5; ++i) with_crc();
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < reps; ++i) with_crc();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float cms;
      CK(hipEventElapsedTime(&cms, e0, e1));
      cus = cms * 1e3 / reps;
    }
    // the standalone checksum pass over the same shards (what the fused kernel saves)
    double ous = 0;
    {
      for (int i = 0; i < 3; ++i) CK(launch_crc32(all.data(), sh.S, (int)all.size(), crcs, 0));
      const int creps = std::max(5, reps / 4);
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < creps; ++i) CK(launch_crc32(all.data(), sh.S, (int)all.size(), crcs, 0));
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float oms;
      CK(hipEventElapsedTime(&oms, e0, e1));
      ous = oms * 1e3 / creps;
    }
    const double bytes = double(sh.k + sh.m) * sh.S * sh.stripes;
    // lane-ops: per 16-B lane chunk, k inputs x (20 selector ops + m x 20 perm/xor ops)
    const double laneops = double(sh.S) / 16 * sh.stripes * sh.k * (20.0 + 20.0 * sh.m);
    printf("%-30s %3d %3d %9zu %4d %9.1f %8.1f %6.1f %9.1f %9.1f %6.1f %9.1f %6.1f %11.1f %s\n", sh.name, sh.k, sh.m, sh.S,
           sh.stripes, us, bytes / (us * 1e-6) / 1e9, 100 * bytes / (us * 1e-6) / 8e12, laneops / (us * 1e-6) / 1e12,
           vus, 100 * bytes / (vus * 1e-6) / 8e12, cus, cus > 0 ? 100 * bytes / (cus * 1e-6) / 8e12 : 0.0, ous,
           fused ? "fused" : "sep");
  }
  return 0;
}
