// crc32.hip -- shard CRC32-IEEE on gfx950 (the checksum access computes per shard after
// encode, blobstore/access/stream_put.go:249-253, and blobnode recomputes on repair,
// blobnode/work_shard_recover.go:336-342).  Go's crc32.ChecksumIEEE: reflected polynomial
// 0xEDB88320, register preset ~0 and final inversion.
//
// Parallel form.  Write f(r, B) for the register after feeding bytes B from register r
// (no pre/post inversion).  f is affine: f(r, B) = shift(r, |B|) ^ f(0, B), where
// shift(v, n) multiplies v by x^(8n) mod P.  For a shard split into chunks C_i ending at
// byte e_i:  crc = ~( shift(~0, S) ^ XOR_i shift(f(0, C_i), S - e_i) ).
// Each lane folds one 1 KiB chunk with slice-by-4 tables in LDS, shifts its remainder to
// the end of the shard, and XORs it into the shard's word; the host applies the ~0 terms.
#include "kernels.hpp"

#include <algorithm>

namespace cfsec {
namespace {

constexpr uint32_t kPoly = 0xEDB88320u;
constexpr int kThreads = 256;
constexpr size_t kChunk = 1024;
constexpr int kSlots = 280;

struct __attribute__((aligned(16))) CrcArgs {
  uint64_t len;
  uint32_t* out;
  uint32_t fin, pad;            // XOR-ed in once per shard (0: leave the raw word)
  const uint8_t* ptr[kSlots];
  uint32_t idx[kSlots];         // output word of shard i
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_ua __attribute__((aligned(1)));

// a * b mod P, reflected bit order (bit 31 = x^0).
__host__ __device__ inline uint32_t multmodp(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (uint32_t m = 1u << 31; m; m >>= 1) {
    if (a & m) p ^= b;
    b = (b & 1u) ? (b >> 1) ^ kPoly : b >> 1;
  }
  return p;
}

struct X2n {
  uint32_t t[64];  // t[k] = x^(2^k) mod P
};

X2n make_x2n() {
  X2n x{};
  uint32_t p = 1u << 30;  // x^1
  x.t[0] = p;
  for (int k = 1; k < 64; ++k) x.t[k] = p = multmodp(p, p);
  return x;
}

__constant__ X2n d_x2n;

// x^(8n) mod P
__host__ __device__ inline uint32_t x8nmodp(uint64_t n, const uint32_t* t) {
  uint32_t p = 1u << 31;  // x^0
  int k = 3;
  while (n) {
    if (n & 1) p = multmodp(t[k], p);
    n >>= 1;
    ++k;
  }
  return p;
}

__global__ __launch_bounds__(kThreads) void crc32_chunks_kernel(const CrcArgs a) {
  __shared__ uint32_t tab[4][256];
  for (int i = threadIdx.x; i < 256; i += kThreads) {
    uint32_t c = (uint32_t)i;
    for (int j = 0; j < 8; ++j) c = (c & 1u) ? (c >> 1) ^ kPoly : c >> 1;
    tab[0][i] = c;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 256; i += kThreads) {
    uint32_t c = tab[0][i];
    for (int s = 1; s < 4; ++s) {
      c = (c >> 8) ^ tab[0][c & 0xFF];
      tab[s][i] = c;
    }
  }
  __syncthreads();

  const size_t start = ((size_t)blockIdx.x * kThreads + threadIdx.x) * kChunk;
  if (start >= a.len) return;
  const size_t end = start + kChunk < a.len ? start + kChunk : a.len;
  const uint8_t* p = a.ptr[blockIdx.y];
  uint32_t crc = 0;
  size_t i = start;
  for (; i + 16 <= end; i += 16) {
    const u32x4 v = *reinterpret_cast<const u32x4_ua*>(p + i);
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      crc ^= v[w];
      crc = tab[3][crc & 0xFF] ^ tab[2][(crc >> 8) & 0xFF] ^ tab[1][(crc >> 16) & 0xFF] ^ tab[0][crc >> 24];
    }
  }
  for (; i < end; ++i) crc = (crc >> 8) ^ tab[0][(crc ^ p[i]) & 0xFF];
  if (end < a.len) crc = multmodp(x8nmodp(a.len - end, d_x2n.t), crc);
  if (start == 0) crc ^= a.fin;
  atomicXor(a.out + a.idx[blockIdx.y], crc);
}

}  // namespace

hipError_t launch_crc32_to(const uint8_t* const* ptrs, size_t len, int n, uint32_t* out, const uint32_t* idx,
                           uint32_t fin, hipStream_t stream) {
  static const X2n host_x2n = make_x2n();
  hipError_t e = hipMemcpyToSymbolAsync(HIP_SYMBOL(d_x2n), &host_x2n, sizeof(X2n), 0,
                                        hipMemcpyHostToDevice, stream);
  if (e != hipSuccess || len == 0 || n == 0) return e;
  const size_t blocks = (len + kChunk * kThreads - 1) / (kChunk * kThreads);
  CrcArgs a;
  a.len = len;
  a.out = out;
  a.fin = fin;
  a.pad = 0;
  for (int s0 = 0; s0 < n; s0 += kSlots) {
    const int ns = std::min(kSlots, n - s0);
    for (int s = 0; s < ns; ++s) {
      a.ptr[s] = ptrs[s0 + s];
      a.idx[s] = idx ? idx[s0 + s] : (uint32_t)(s0 + s);
    }
    hipLaunchKernelGGL(crc32_chunks_kernel, dim3((unsigned)blocks, (unsigned)ns), dim3(kThreads), 0,
                       stream, a);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_crc32(const uint8_t* const* ptrs, size_t len, int n, uint32_t* out,
                        hipStream_t stream) {
  hipError_t e = hipMemsetAsync(out, 0, sizeof(uint32_t) * (size_t)n, stream);
  if (e != hipSuccess) return e;
  return launch_crc32_to(ptrs, len, n, out, nullptr, 0u, stream);
}

uint32_t crc32_finalize(uint32_t raw, size_t len) {
  static const X2n host_x2n = make_x2n();
  if (len == 0) return 0;
  return ~(multmodp(x8nmodp(len, host_x2n.t), 0xFFFFFFFFu) ^ raw);
}

}  // namespace cfsec
