// fg_probe.hip -- can the host write fine-grained device memory directly (large BAR), and what does
// a kernel reading a 9.7 KiB table from it / from mapped host memory cost (dev probe, round 5)
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)
__global__ void sum_kernel(const unsigned* t, int n, unsigned* out) {
  unsigned s = 0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += t[i];
  atomicAdd(out, s);
}
int main() {
  const int n = 2432;
  unsigned* fg = nullptr;
  hipError_t e = hipExtMallocWithFlags(reinterpret_cast<void**>(&fg), n * 4, hipDeviceMallocFinegrained);
  std::printf("hipExtMallocWithFlags(fine-grained): %s\n", hipGetErrorString(e));
  if (e != hipSuccess) return 0;
  hipPointerAttribute_t at;
  CK(hipPointerGetAttributes(&at, fg));
  std::printf("type %d hostPointer %p devicePointer %p\n", (int)at.type, at.hostPointer, at.devicePointer);
  unsigned* out;
  CK(hipMalloc(&out, 4));
  CK(hipMemset(out, 0, 4));
  // host write: only if the runtime hands out a host pointer
  if (at.hostPointer) {
    unsigned* h = static_cast<unsigned*>(at.hostPointer);
    for (int i = 0; i < n; ++i) h[i] = i;
    __builtin_ia32_sfence();
    hipLaunchKernelGGL(sum_kernel, dim3(1), dim3(256), 0, 0, fg, n, out);
    unsigned r = 0;
    CK(hipMemcpy(&r, out, 4, hipMemcpyDeviceToHost));
    std::printf("host-written fine-grained sum %u (want %u)\n", r, (unsigned)(n * (n - 1) / 2));
  }
  return 0;
}
