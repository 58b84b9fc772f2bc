// null_query_probe.hip -- does hipStreamQuery(NULL) report work pending on a *blocking* stream?
// (engine.cpp order_after_default skips its event wait when the legacy null stream is idle; the
// C ABI promises ordering after blocking streams too.)  A ~2 ms spin kernel on a blocking stream,
// then hipStreamQuery(NULL) at once; the same with a non-blocking stream as the control.
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void spin_kernel(long long cycles, int* out) {
  const long long t0 = clock64();
  while (clock64() - t0 < cycles) __builtin_amdgcn_s_sleep(10);
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = 1;
}

int main() {
  int* out = nullptr;
  if (hipMalloc(&out, 4) != hipSuccess) return 1;
  for (int nonblocking = 0; nonblocking < 2; ++nonblocking) {
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, nonblocking ? hipStreamNonBlocking : hipStreamDefault) != hipSuccess) return 2;
    hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, s, 200000000LL, out);
    const hipError_t q0 = hipStreamQuery(nullptr);
    const hipError_t qs = hipStreamQuery(s);
    std::printf("{\"stream\": \"%s\", \"query_null\": \"%s\", \"query_stream\": \"%s\"}\n",
                nonblocking ? "non-blocking" : "blocking", hipGetErrorName(q0), hipGetErrorName(qs));
    if (hipStreamSynchronize(s) != hipSuccess) return 3;
    (void)hipStreamDestroy(s);
  }
  return 0;
}
