// seg_latency.hip -- per-call latency of the single-stripe C ABI on device memory (access's degraded
// range read: ReconstructData of one segment per shard, access/stream_get.go:420-427), without
// Python: cfsec_ec_reconstruct_data on HBM shards, median over repeated calls, beside the floor a
// synchronous call cannot go under (one trivial kernel launched and waited for, by
// hipStreamSynchronize and by a polled marker word); round 6: the same segments in page-locked and in
// pageable host memory with a NULL stream (the Go shim's CFSEC_MEM_HOST call).  Build: make -C tools seg_latency (links
// ../chubaofs_amd/libcfsec.so).  CFSEC_HOST_TIMING=1 adds the engine's phase times on stderr.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../include/cfsec.h"

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

__global__ void nop_kernel(int* p) {
  if (p && threadIdx.x == 0 && blockIdx.x == 0) p[0] = 1;
}

// the same with a kernel argument block the size of dev::GfArgs (3.5 KiB)
struct BigArgs {
  int* p;
  uint8_t pad[3584 - 8];
};
__global__ void nop_big_kernel(const BigArgs a) {
  if (a.p && threadIdx.x == 0 && blockIdx.x == 0) a.p[0] = a.pad[5];
}

// the same, ending with its own completion word in host memory (system-scope release store)
__global__ void nop_mark_kernel(int* p, uint32_t* mark, uint32_t seq) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    p[0] = 1;
    __hip_atomic_store(mark, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <class F>
static double median_us(F f, int reps) {
  for (int i = 0; i < 5; ++i) f();
  std::vector<double> t(reps);
  for (int i = 0; i < reps; ++i) {
    const double t0 = now_us();
    f();
    t[i] = now_us() - t0;
  }
  std::sort(t.begin(), t.end());
  return t[reps / 2];
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 200;
  const bool null_stream = argc > 2 && std::strcmp(argv[2], "null") == 0;  // the calls on NULL (Go's nil)
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipStream_t call_st = null_stream ? nullptr : st;
  int* flag = nullptr;
  CK(hipMalloc(&flag, 4));
  // floors
  const double f_sync = median_us([&] {
    hipLaunchKernelGGL(nop_kernel, dim3(1), dim3(64), 0, st, flag);
    CK(hipStreamSynchronize(st));
  }, reps);
  uint32_t* hm = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void**>(&hm), 64, hipHostMallocMapped | hipHostMallocCoherent));
  uint32_t* dm = nullptr;
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dm), hm, 0));
  uint32_t seq = 0;
  const double f_poll = median_us([&] {
    hipLaunchKernelGGL(nop_kernel, dim3(1), dim3(64), 0, st, flag);
    ++seq;
    CK(hipStreamWriteValue32(st, dm, seq, 0));
    while (__atomic_load_n(hm, __ATOMIC_ACQUIRE) != seq) __builtin_ia32_pause();
  }, reps);
  const double f_kmark = median_us([&] {
    ++seq;
    hipLaunchKernelGGL(nop_mark_kernel, dim3(1), dim3(64), 0, st, flag, dm, seq);
    while (__atomic_load_n(hm, __ATOMIC_ACQUIRE) != seq) __builtin_ia32_pause();
  }, reps);
  BigArgs big{};
  big.p = flag;
  const double f_big = median_us([&] {
    hipLaunchKernelGGL(nop_big_kernel, dim3(1), dim3(64), 0, st, big);
    ++seq;
    CK(hipStreamWriteValue32(st, dm, seq, 0));
    while (__atomic_load_n(hm, __ATOMIC_ACQUIRE) != seq) __builtin_ia32_pause();
  }, reps);
  // host cost of the launch calls alone (no wait): 64 B vs 3.5 KiB of arguments
  const auto launch_cost = [&](bool large) {
    CK(hipStreamSynchronize(st));
    const double t0 = now_us();
    for (int i = 0; i < 64; ++i) {
      if (large) hipLaunchKernelGGL(nop_big_kernel, dim3(1), dim3(64), 0, st, big);
      else hipLaunchKernelGGL(nop_kernel, dim3(1), dim3(64), 0, st, flag);
    }
    const double t = (now_us() - t0) / 64;
    CK(hipStreamSynchronize(st));
    return t;
  };
  double l_small = 1e9, l_big = 1e9;
  for (int r = 0; r < 20; ++r) {
    l_small = std::min(l_small, launch_cost(false));
    l_big = std::min(l_big, launch_cost(true));
  }
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  const double f_event = median_us([&] {
    hipLaunchKernelGGL(nop_kernel, dim3(1), dim3(64), 0, st, flag);
    CK(hipEventRecord(ev, st));
    while (hipEventQuery(ev) == hipErrorNotReady) __builtin_ia32_pause();
  }, reps);
  std::printf("{\"stream\": \"%s\", \"sync_floor_us\": %.1f, \"poll_floor_us\": %.1f, \"kernel_mark_floor_us\": %.1f, "
              "\"event_query_floor_us\": %.1f, \"poll_floor_3.5KiB_args_us\": %.1f, \"launch_call_us\": %.2f, "
              "\"launch_call_3.5KiB_args_us\": %.2f", null_stream ? "null" : "own", f_sync, f_poll, f_kmark, f_event, f_big,
              l_small, l_big);
  const int modes[2] = {2, 9};  // codemode.EC6P6, codemode.EC12P4 (codemode.go:30-60)
  const char* names[2] = {"EC6P6", "EC12P4"};
  for (int mi = 0; mi < 2; ++mi) {
    cfsec_tactic t;
    if (cfsec_codemode_tactic(modes[mi], &t)) return 2;
    cfsec_ec* h = nullptr;
    if (cfsec_ec_new(&t, 0, 0, 0, &h)) return 3;
    const int n = t.n + t.m;
    for (size_t seg : {(size_t)4096, (size_t)65536, (size_t)1 << 20}) {
      std::vector<uint8_t*> d(n);
      std::vector<uint8_t> host(seg);
      for (int i = 0; i < n; ++i) {
        CK(hipMalloc(&d[i], seg));
        for (size_t b = 0; b < seg; ++b) host[b] = (uint8_t)(b * 7 + i * 13 + (b >> 8));
        CK(hipMemcpy(d[i], host.data(), seg, hipMemcpyHostToDevice));
      }
      std::vector<cfsec_shard> sh(n);
      for (int i = 0; i < n; ++i) sh[i] = cfsec_shard{d[i], seg, seg};
      if (cfsec_ec_encode(h, sh.data(), n, CFSEC_MEM_DEVICE, st)) return 4;
      std::vector<uint8_t> want(seg), got(seg);
      CK(hipMemcpy(want.data(), d[0], seg, hipMemcpyDeviceToHost));
      const int bad[2] = {0, 1};
      const double us = median_us([&] {
        for (int i = 0; i < n; ++i) sh[i] = cfsec_shard{d[i], seg, seg};
        const int e = cfsec_ec_reconstruct_data(h, sh.data(), n, bad, 2, CFSEC_MEM_DEVICE, call_st);
        if (e) std::exit(5);
      }, reps);
      CK(hipMemcpy(got.data(), d[0], seg, hipMemcpyDeviceToHost));
      if (got != want) {
        std::fprintf(stderr, "rebuilt segment differs\n");
        return 6;
      }
      std::printf(", \"%s_%zu_us\": %.1f", names[mi], seg, us);
      // the same call on host memory with a NULL stream, as the Go shim makes it: page-locked rows
      // (cfsec_host_alloc: the kernel reads and writes them over PCIe) and pageable rows (staged)
      for (int pinned = 1; pinned >= 0; --pinned) {
        std::vector<uint8_t*> hrow(n);
        uint8_t* block = nullptr;
        std::vector<uint8_t> pageable;
        if (pinned) {
          if (cfsec_host_alloc((size_t)n * seg, reinterpret_cast<void**>(&block))) return 7;
        } else {
          pageable.resize((size_t)n * seg);
          block = pageable.data();
        }
        for (int i = 0; i < n; ++i) {
          hrow[i] = block + (size_t)i * seg;
          CK(hipMemcpy(hrow[i], d[i], seg, hipMemcpyDeviceToHost));
        }
        const double hus = median_us([&] {
          for (int i = 0; i < n; ++i) sh[i] = cfsec_shard{hrow[i], seg, seg};
          const int e = cfsec_ec_reconstruct_data(h, sh.data(), n, bad, 2, CFSEC_MEM_HOST, nullptr);
          if (e) std::exit(8);
        }, reps);
        if (std::memcmp(hrow[0], want.data(), seg) != 0) {
          std::fprintf(stderr, "rebuilt host segment differs\n");
          return 9;
        }
        std::printf(", \"%s_%zu_%s_us\": %.1f", names[mi], seg, pinned ? "pinned" : "pageable", hus);
        if (pinned) cfsec_host_free(block);
      }
      for (int i = 0; i < n; ++i) CK(hipFree(d[i]));
    }
    cfsec_ec_free(h);
  }
  std::printf("}\n");
  return 0;
}
