// crc_pass_probe.hip -- the standalone shard CRC pass (launch_crc32_to, csrc/crc32.hip) timed with HIP
// events over a repair tasklet's rebuilt rows (256 x 262,144 B at non-uniform addresses, as the ec
// batch calls hand them over) and over 128 rows of 5,592,406 B, vs the workgroup count
// (CFSEC_CRC32_GROUPS_PROBE, re-read per launch) (dev tool, round 3).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../chubaofs_amd/csrc crc_pass_probe.hip \
//         -L../chubaofs_amd -lcfsec -Wl,-rpath,'$ORIGIN/../chubaofs_amd' -o crc_pass_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "kernels.hpp"

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

using namespace cfsec;

void run(const char* name, int n, size_t S, int spread) {
  const size_t pitch = (S + 255) / 256 * 256;
  uint8_t* buf;
  CK(hipMalloc(&buf, pitch * n * spread));
  CK(hipMemset(buf, 0x5A, pitch * n * spread));
  std::vector<const uint8_t*> ptrs(n);
  std::vector<uint32_t> idx(n);
  for (int i = 0; i < n; ++i) ptrs[i] = buf + (size_t)i * spread * pitch + (i % 7) * 256, idx[i] = i;
  uint32_t* out;
  CK(hipMalloc(&out, 4 * n));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  uint32_t ref = 0;
  for (int g : {512, 1024, 2048, 4096, 8192}) {
    setenv("CFSEC_CRC32_GROUPS_PROBE", std::to_string(g).c_str(), 1);
    for (int i = 0; i < 5; ++i) CK(launch_crc32_to(ptrs.data(), S, n, out, idx.data(), 0u, 0));
    const int reps = 50;
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) {
      CK(hipMemsetAsync(out, 0, 4 * n, 0));
      CK(launch_crc32_to(ptrs.data(), S, n, out, idx.data(), crc32_shift_ones(S), 0));
    }
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    uint32_t w;
    CK(hipMemcpy(&w, out + n - 1, 4, hipMemcpyDeviceToHost));
    if (g == 512) ref = w;
    std::printf("%-34s groups %5d  %8.1f us (memset + pass)  %7.1f GB/s  %s\n", name, g, ms * 1e3 / reps,
                (double)n * S / (ms * 1e-3 / reps) / 1e9, w == ref ? "same word" : "DIFFER");
  }
  CK(hipFree(buf));
  CK(hipFree(out));
}

int main() {
  run("C5 rebuilt rows 256 x 262144", 256, 262144, 2);
  run("EC12P4 8 stripes 128 x 5592406", 128, 5592406, 1);
  return 0;
}
