// gf_kernels.hip -- gfx950 kernels for GF(2^8) Reed-Solomon shard coding.
//
// Replaces the CPU kernels of klauspost/reedsolomon v1.11.7 (the generated
// mulAvxTwo_RxC / mulGFNI_RxC_64 families in KRS/galois_gen_amd64.s and the
// galMulSlice[Xor] tails in KRS/galois_amd64.go:57-122) with one HBM-streaming
// kernel per output-row count.
//
// Arithmetic.  GF(2^8) multiplication by a constant is linear over GF(2), so a
// byte x is split into bit fields x = x[2:0] | x[5:3] | x[7:6] and
//     c*x = T0_c[x[2:0]] ^ T1_c[x[5:3]] ^ T2_c[x[7:6]]
// with 8-, 8- and 4-entry product tables.  An 8-entry byte table is exactly
// what one v_perm_b32 indexes: the two table dwords are the perm's data
// operands and the 3-bit fields (one per byte of the lane's dword) its
// selector, so one VALU op looks up 4 bytes at once.  Per (coefficient, dword)
// the cost is 3 v_perm_b32 + 2 XORs (fused into v_bitop3_b32 by the compiler);
// per input dword the 3 selectors cost 5 ops, amortised over all outputs.
// No MFMA: GF arithmetic is not an FP/int contraction.
//
// Data movement.  Each lane owns 16 consecutive bytes of the shard (one
// global_load_dwordx4 per input row, one global_store_dwordx4 per output row),
// so a 256-thread workgroup streams 4 KiB columns of every row and every byte
// of HBM is touched exactly once: read k*len, write m*len (verify: read
// (k+m)*len, write nothing).  The product tables are rebuilt per workgroup in
// LDS from the coefficient matrix carried in the kernel argument block, which
// keeps the launch free of device allocations and host->device copies (so it
// is safe under concurrent callers and hipGraph capture).
#include "kernels.hpp"

#include <algorithm>

namespace cfsec {
namespace {

constexpr int kMaxK = 32;       // inputs per launch (larger k: input chunks + accumulate)
constexpr int kMaxM = 32;       // outputs per launch
constexpr int kPtrSlots = 300;  // shard pointers carried per launch
constexpr int kThreads = 256;
constexpr int kLaneBytes = 16;
constexpr size_t kBlockBytes = size_t(kThreads) * kLaneBytes;

struct __attribute__((aligned(16))) GfArgs {
  uint64_t len;
  uint32_t k, m, nstripes, pad0;
  uint32_t* flags;
  uint8_t coef[kMaxM * kMaxK];     // m x k, row stride k
  const uint8_t* ptr[kPtrSlots];   // [nstripes*k inputs][nstripes*m outputs]
};
static_assert(sizeof(GfArgs) <= 3584, "kernel argument block must stay below 4 KiB");

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_ua __attribute__((aligned(1)));  // shard rows may start at any byte

__device__ __forceinline__ uint32_t gf_xtime(uint32_t v) {
  v <<= 1;
  return (v & 0x100u) ? (v ^ 0x11Du) : v;  // KRS/galois.go:25 polynomial 0x11D
}

template <bool TAIL>
__device__ __forceinline__ u32x4 load16(const uint8_t* p, size_t rem) {
  if constexpr (!TAIL) {
    return *reinterpret_cast<const u32x4_ua*>(p);
  } else {
    uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if ((size_t)i < rem) w[i >> 2] |= (uint32_t)p[i] << (8 * (i & 3));
    return u32x4{w[0], w[1], w[2], w[3]};
  }
}

template <bool TAIL>
__device__ __forceinline__ void store16(uint8_t* p, u32x4 v, size_t rem) {
  if constexpr (!TAIL) {
    *reinterpret_cast<u32x4_ua*>(p) = v;
  } else {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if ((size_t)i < rem) p[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
  }
}

template <int M, MatVecMode MODE, bool TAIL>
__device__ __forceinline__ void matvec_body(const GfArgs& a, const u32x4* __restrict__ tab01,
                                            const uint32_t* __restrict__ tab2,
                                            const uint8_t* const* in, uint8_t* const* out,
                                            size_t off, size_t rem, int stripe) {
  const int k = (int)a.k;
  u32x4 acc[M];
#pragma unroll
  for (int r = 0; r < M; ++r) acc[r] = u32x4{0u, 0u, 0u, 0u};

  u32x4 x = load16<TAIL>(in[0] + off, rem);
  for (int c = 0; c < k; ++c) {
    u32x4 xn = x;
    if (c + 1 < k) xn = load16<TAIL>(in[c + 1] + off, rem);  // one row ahead
    const u32x4 s0 = x & 0x07070707u;
    const u32x4 s1 = (x >> 3) & 0x07070707u;
    const u32x4 s2 = (x >> 6) & 0x03030303u;
    const u32x4* tq = tab01 + c * M;
    const uint32_t* t2p = tab2 + c * M;
#pragma unroll
    for (int r = 0; r < M; ++r) {
      const u32x4 q = tq[r];
      const uint32_t t2 = t2p[r];
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const uint32_t p0 = __builtin_amdgcn_perm(q.y, q.x, s0[w]);
        const uint32_t p1 = __builtin_amdgcn_perm(q.w, q.z, s1[w]);
        const uint32_t p2 = __builtin_amdgcn_perm(0u, t2, s2[w]);
        // acc ^ p0 ^ p1 in one v_bitop3_b32 (truth table 0x96 = 3-input XOR)
        acc[r][w] = __builtin_amdgcn_bitop3_b32(acc[r][w], p0, p1, 0x96) ^ p2;
      }
    }
    x = xn;
  }

  const int m = (int)a.m;
  if constexpr (MODE == MatVecMode::kVerify) {
    uint32_t diff = 0;
#pragma unroll
    for (int r = 0; r < M; ++r) {
      if (r < m) {
        const u32x4 y = load16<TAIL>(out[r] + off, rem);
        const u32x4 d = acc[r] ^ y;
        diff |= d.x | d.y | d.z | d.w;
      }
    }
    if (diff) atomicOr(a.flags + stripe, 1u);
  } else {
#pragma unroll
    for (int r = 0; r < M; ++r) {
      if (r < m) {
        u32x4 v = acc[r];
        if constexpr (MODE == MatVecMode::kAccum) v ^= load16<TAIL>(out[r] + off, rem);
        store16<TAIL>(out[r] + off, v, rem);
      }
    }
  }
}

template <int M, MatVecMode MODE>
__global__ __launch_bounds__(kThreads) void gf_matvec_kernel(const GfArgs a) {
  __shared__ u32x4 tab01[kMaxK * M];  // {T0[0..3], T0[4..7], T1[0..3], T1[4..7]} per (c, r)
  __shared__ uint32_t tab2[kMaxK * M];  // T2[0..3] per (c, r)

  const int k = (int)a.k;
  for (int i = threadIdx.x; i < k * M; i += kThreads) {
    const int c = i / M;
    const int r = i - c * M;
    uint32_t p[8];
    p[0] = (r < (int)a.m) ? a.coef[r * k + c] : 0u;
#pragma unroll
    for (int j = 1; j < 8; ++j) p[j] = gf_xtime(p[j - 1]);  // coef * 2^j
    uint32_t t0lo = 0, t0hi = 0, t1lo = 0, t1hi = 0, t2 = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const uint32_t v0 = ((e & 1) ? p[0] : 0u) ^ ((e & 2) ? p[1] : 0u) ^ ((e & 4) ? p[2] : 0u);
      const uint32_t v1 = ((e & 1) ? p[3] : 0u) ^ ((e & 2) ? p[4] : 0u) ^ ((e & 4) ? p[5] : 0u);
      if (e < 4) {
        const uint32_t v2 = ((e & 1) ? p[6] : 0u) ^ ((e & 2) ? p[7] : 0u);
        t0lo |= v0 << (8 * e);
        t1lo |= v1 << (8 * e);
        t2 |= v2 << (8 * e);
      } else {
        t0hi |= v0 << (8 * (e - 4));
        t1hi |= v1 << (8 * (e - 4));
      }
    }
    tab01[i] = u32x4{t0lo, t0hi, t1lo, t1hi};
    tab2[i] = t2;
  }
  __syncthreads();

  const int stripe = blockIdx.y;
  const size_t off = ((size_t)blockIdx.x * kThreads + threadIdx.x) * kLaneBytes;
  if (off >= a.len) return;
  const uint8_t* const* in = a.ptr + (size_t)stripe * k;
  uint8_t* const* out = const_cast<uint8_t* const*>(a.ptr + (size_t)a.nstripes * k + (size_t)stripe * a.m);
  const size_t rem = a.len - off;
  if (rem >= (size_t)kLaneBytes)
    matvec_body<M, MODE, false>(a, tab01, tab2, in, out, off, kLaneBytes, stripe);
  else
    matvec_body<M, MODE, true>(a, tab01, tab2, in, out, off, rem, stripe);
}

template <MatVecMode MODE>
hipError_t launch_mode(int mpad, const GfArgs& a, dim3 grid, hipStream_t st) {
#define CFSEC_CASE(MV)                                                              \
  case MV:                                                                          \
    hipLaunchKernelGGL((gf_matvec_kernel<MV, MODE>), grid, dim3(kThreads), 0, st, a); \
    break;
  switch (mpad) {
    CFSEC_CASE(1) CFSEC_CASE(2) CFSEC_CASE(3) CFSEC_CASE(4) CFSEC_CASE(5) CFSEC_CASE(6)
    CFSEC_CASE(8) CFSEC_CASE(10) CFSEC_CASE(12) CFSEC_CASE(16) CFSEC_CASE(20)
    CFSEC_CASE(24) CFSEC_CASE(32)
    default: return hipErrorInvalidValue;
  }
#undef CFSEC_CASE
  return hipGetLastError();
}

int pad_outputs(int m) {
  static const int kSizes[] = {1, 2, 3, 4, 5, 6, 8, 10, 12, 16, 20, 24, 32};
  for (int s : kSizes)
    if (s >= m) return s;
  return -1;
}

}  // namespace

hipError_t launch_matvec(const MatVecJob& job, hipStream_t stream) {
  if (job.k <= 0 || job.m < 0 || job.nstripes < 0 || !job.coef || !job.in || !job.out)
    return hipErrorInvalidValue;
  if (job.m == 0 || job.nstripes == 0 || job.len == 0) return hipSuccess;
  if (job.mode == MatVecMode::kVerify && (job.k > kMaxK || !job.flags)) return hipErrorInvalidValue;

  const size_t blocks_x = (job.len + kBlockBytes - 1) / kBlockBytes;
  if (blocks_x > 0x7fffffffu) return hipErrorInvalidValue;

  GfArgs a;
  for (int r0 = 0; r0 < job.m; r0 += kMaxM) {
    const int mc = std::min(kMaxM, job.m - r0);
    for (int c0 = 0; c0 < job.k; c0 += kMaxK) {
      const int kc = std::min(kMaxK, job.k - c0);
      MatVecMode mode = job.mode;
      if (mode == MatVecMode::kStore && c0 > 0) mode = MatVecMode::kAccum;
      const int per_stripe = kc + mc;
      const int stripes_per_launch = std::min(kPtrSlots / per_stripe, 65535);
      for (int s0 = 0; s0 < job.nstripes; s0 += stripes_per_launch) {
        const int ns = std::min(stripes_per_launch, job.nstripes - s0);
        a.len = job.len;
        a.k = (uint32_t)kc;
        a.m = (uint32_t)mc;
        a.nstripes = (uint32_t)ns;
        a.pad0 = 0;
        a.flags = job.flags ? job.flags + s0 : nullptr;
        for (int r = 0; r < mc; ++r)
          for (int c = 0; c < kc; ++c)
            a.coef[r * kc + c] = job.coef[(size_t)(r0 + r) * job.k + (c0 + c)];
        for (int s = 0; s < ns; ++s) {
          for (int c = 0; c < kc; ++c)
            a.ptr[s * kc + c] = job.in[(size_t)(s0 + s) * job.k + c0 + c];
          for (int r = 0; r < mc; ++r)
            a.ptr[ns * kc + s * mc + r] = job.out[(size_t)(s0 + s) * job.m + r0 + r];
        }
        const dim3 grid((unsigned)blocks_x, (unsigned)ns);
        const int mpad = pad_outputs(mc);
        hipError_t e;
        switch (mode) {
          case MatVecMode::kStore: e = launch_mode<MatVecMode::kStore>(mpad, a, grid, stream); break;
          case MatVecMode::kAccum: e = launch_mode<MatVecMode::kAccum>(mpad, a, grid, stream); break;
          default: e = launch_mode<MatVecMode::kVerify>(mpad, a, grid, stream); break;
        }
        if (e != hipSuccess) return e;
      }
    }
  }
  return hipSuccess;
}

}  // namespace cfsec
