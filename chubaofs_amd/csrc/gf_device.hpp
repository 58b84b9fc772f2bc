// gf_device.hpp -- device side of the GF(2^8) matrix x shard-vector kernel.
//
// Included by gf_kernels.hip (the product launcher) and by the tools/ A/B harnesses, so a
// tuned policy is exactly the code that ships.
//
// See gf_kernels.hip for the arithmetic (3-bit split tables + v_perm_b32) and the data
// movement.  Policy knobs (template parameters of matvec):
//   M   output rows per wave (accumulators live in VGPRs: 4*M)
//   OS  waves of a workgroup that share one column chunk, each owning M of the M*OS output
//       rows (large m: keeps per-wave accumulators + tables small; the inputs the sharing
//       waves re-read come from L1)
//   W   16-B chunks per lane per tile (chunk w sits w*step bytes further on)
//   G   input rows whose loads are issued together before any is consumed
//   PERSIST  grid-stride over (stripe, tile) pairs; tables built once per workgroup
//   NTL/NTS  non-temporal loads / stores (streaming data, touched once)
//   XCD remap blockIdx so each XCD walks a contiguous run of tiles (T1 swizzle)
//   WAVEC    chunk w of a lane sits w*1 KiB on inside its wave's own run (else the
//            workgroup sweeps the tile W times)
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "kernels.hpp"

namespace cfsec {
namespace dev {

constexpr int kMaxK = 32;       // inputs per launch
constexpr int kMaxM = 32;       // outputs per launch
constexpr int kPtrSlots = 288;  // shard pointers per launch
constexpr int kLenSlots = 32;   // per-stripe lengths per launch (heterogeneous batches)
constexpr int kThreads = 256;
constexpr int kLaneBytes = 16;

// Shard pointers of stripe s, row j:
//   explicit table (sstride == 0): ptr[s*k + j] (inputs), ptr[tab*k + s*m + r] (outputs)
//   affine batch   (sstride != 0): ptr[j] + s*sstride, table holds stripe 0 only (tab == 1),
//                                  so one launch covers any number of stripes.
// Stripe lengths: every stripe is `len` bytes, or (varlen != 0, explicit table only) stripe s is
// slen[s] bytes and `len` is the longest (it sizes the grid; tiles past a stripe's end exit).
struct __attribute__((aligned(16))) GfArgs {
  uint64_t len;
  uint32_t k, m, nstripes, tiles_per_stripe;  // tiles_per_stripe: in units of the kernel's tile
  uint32_t* flags;
  int64_t sstride;                 // byte distance between consecutive stripes (affine batch)
  uint32_t tab;                    // stripes held in ptr[]
  uint16_t nstore;                 // kStoreVerify: outputs [0, nstore) are stored, [nstore, m) compared
  uint16_t varlen;                 // nonzero: per-stripe lengths in slen[]
  uint32_t pstore, pcmp;           // repair_dy16: parity rows stored / compared
  uint32_t* zw;                    // repair_dy16: nzw words workgroup (0, 0) zeroes (checksum words)
  uint32_t nzw;
  uint8_t src[16];                 // repair_dy16: input slot of data row i (16 + j: missing row j)
  uint8_t coef[kMaxM * kMaxK];    // m x k, row stride k
  uint32_t slen[kLenSlots];
  const uint8_t* ptr[kPtrSlots];  // [tab*k inputs][tab*m outputs]
};
static_assert(sizeof(GfArgs) <= 3584, "kernel argument block must stay below 4 KiB");
// Register-table launches of the fixed-K kernels (gf_fixed.hpp): the packed tables start this many
// bytes into coef[], 16-byte aligned within the block
constexpr size_t kRegTabOff = (16 - offsetof(GfArgs, coef) % 16) % 16;

// Bytes in stripe s of the launch.
__device__ __forceinline__ uint64_t stripe_len(const GfArgs& a, uint32_t s) {
  return a.varlen ? (uint64_t)a.slen[s] : a.len;
}

// Output row r of the launch is compared, not stored.
template <MatVecMode MODE>
__device__ __forceinline__ bool row_compared(const GfArgs& a, int r) {
  if constexpr (MODE == MatVecMode::kVerify) return true;
  else if constexpr (MODE == MatVecMode::kStoreVerify) return r >= (int)a.nstore;
  else return false;
}

// A Verify mismatch in stripe s: flags[s] = 1.  The words only ever hold 0 or 1, so a store is the
// OR the semantics ask for (no read-modify-write), and it may target pinned host words directly
// (batch.cpp: a synchronous batch's per-item flags, no gather launch), where an atomic RMW would
// need PCIe atomics.
__device__ __forceinline__ void set_flag(uint32_t* flags, uint32_t s) {
  __hip_atomic_store(flags + s, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_ua __attribute__((aligned(1)));  // shard rows may start at any byte

__device__ __forceinline__ uint32_t gf_xtime(uint32_t v) {
  v <<= 1;
  return (v & 0x100u) ? (v ^ 0x11Du) : v;  // KRS/galois.go:25 polynomial 0x11D
}

template <bool NT>
__device__ __forceinline__ u32x4 ld16(const uint8_t* p) {
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const u32x4_ua*>(p));
  else return *reinterpret_cast<const u32x4_ua*>(p);
}

template <bool NT>
__device__ __forceinline__ void st16(uint8_t* p, u32x4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<u32x4_ua*>(p));
  else *reinterpret_cast<u32x4_ua*>(p) = v;
}

// 16-byte vector store with explicit gfx950 cache-policy bits (SP = 0: none, 1: nt, 2: sc1, 3: sc0 sc1,
// 4: nt sc1, 5: nt sc0 sc1, 6: sc0).
//
// The store-data hazard (round 6): a store of more than 64 bits reads its data VGPRs after it issues,
// and on gfx940+ a VALU write of one of them within 2 wait states changes what it stores (LLVM
// GCNHazardRecognizer::createsVALUHazard).  hipcc pads the stores it emits itself, but an inline-asm
// store is opaque to the hazard recognizer, so the asm forms here end in `s_nop 1` (2 wait states)
// inside the string, and the non-temporal form -- the shipped policy -- is the compiler's own store.
// Without that, whether a kernel stored the right bytes depended on its schedule: round 5's "wrong
// rows, not understood" (a compile-time output count in matvec_k, a second instantiation of the
// lookup kernel's body) were schedules that put a VALU write of a store's data right behind it, and six
// shipped (K, 1) kStoreVerify kernels had one too (tools/store_hazard_check.py checks a built library).
template <int SP>
__device__ __forceinline__ void st16_pol(uint8_t* p, u32x4 v) {
  if constexpr (SP == 1) __builtin_nontemporal_store(v, reinterpret_cast<u32x4_ua*>(p));
  else if constexpr (SP == 0) asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
  else if constexpr (SP == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
  else if constexpr (SP == 3)
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
  else if constexpr (SP == 4)
    asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
  else if constexpr (SP == 5)
    asm volatile("global_store_dwordx4 %0, %1, off nt sc0 sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
  else asm volatile("global_store_dwordx4 %0, %1, off sc0\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

// 16-byte load at base + off through a raw buffer descriptor with explicit cache-policy bits
// (measurement variants; aux: 1 = sc0, 2 = nt, 16 = sc1).
template <int LP>
__device__ __forceinline__ u32x4 ld16_pol(const uint8_t* base, uint32_t off) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), (short)0, -1, 0x00020000);
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, LP);
  return u32x4{v[0], v[1], v[2], v[3]};
}

// Output-row store of the fixed-K and dyadic kernels: non-temporal (nt).  Measured with no
// Infinity-Cache reuse between launches (tools/rot_probe.hip, profiles/r02/rot_probe.txt): nt
// 69.1 %, sc1 67.8 %, plain 61.2 % of 8 TB/s on the EC12P4 step kernel.  (Round 1 picked sc1 on a
// bench that re-read its own outputs, where leaving them in the cache paid.)
#ifndef CFSEC_STORE_POL
#define CFSEC_STORE_POL 1  // st16_pol policy of the output stores (1 = nt)
#endif
template <bool NTS>
__device__ __forceinline__ void st16_out(uint8_t* p, u32x4 v) {
  if constexpr (NTS) st16_pol<CFSEC_STORE_POL>(p, v);
  else st16<false>(p, v);
}

// Bytes [0, rem) of a 16-byte chunk, zero above (the tail of a shard).
__device__ __forceinline__ u32x4 ld_tail(const uint8_t* p, size_t rem) {
  uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if ((size_t)i < rem) w[i >> 2] |= (uint32_t)p[i] << (8 * (i & 3));
  return u32x4{w[0], w[1], w[2], w[3]};
}

// ld_tail of a row's last piece (p + rem is the row's end, rem < 16): with a row of at least 16
// bytes, one 16-byte load of the row's last 16 bytes shifted down by 16 - rem bytes, zeros in --
// the byte loads' 16 dependent round trips made the lane holding a row's end a straggler that ended
// a launch late (the fused checksum kernels, whose pieces cannot overlap their neighbours' bytes).
__device__ __forceinline__ u32x4 ld_tail_row(const uint8_t* p, size_t rem, uint64_t len) {
  if (len < 16) return ld_tail(p, rem);
  const u32x4 v = ld16<true>(p + rem - 16);
  const uint32_t s = 16u - (uint32_t)rem, d = s >> 2, b = s & 3u;
  const uint32_t w[5] = {v.x, v.y, v.z, v.w, 0u};
  uint32_t a[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) a[j] = b ? __builtin_amdgcn_alignbyte(w[j + 1], w[j], b) : w[j];
  const uint32_t r0 = d == 0 ? a[0] : d == 1 ? a[1] : d == 2 ? a[2] : a[3];
  const uint32_t r1 = d == 0 ? a[1] : d == 1 ? a[2] : d == 2 ? a[3] : 0u;
  const uint32_t r2 = d == 0 ? a[2] : d == 1 ? a[3] : 0u;
  const uint32_t r3 = d == 0 ? a[3] : 0u;
  return u32x4{r0, r1, r2, r3};
}

__device__ __forceinline__ void st_tail(uint8_t* p, u32x4 v, size_t rem) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if ((size_t)i < rem) p[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
}

// Full lane chunks of LW dwords (16, 8 or 4 bytes) for the fixed-K and 16x16-dyadic kernels.
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef u32x2 u32x2_ua __attribute__((aligned(1)));
typedef uint32_t u32_ua __attribute__((aligned(1)));

template <int LW, bool NT>
__device__ __forceinline__ void ld_chunk(const uint8_t* p, uint32_t (&x)[LW]) {
  static_assert(LW == 1 || LW == 2 || LW == 4, "lane chunk of 1, 2 or 4 dwords");
  if constexpr (LW == 4) {
    const u32x4 v = ld16<NT>(p);
    x[0] = v.x, x[1] = v.y, x[2] = v.z, x[3] = v.w;
  } else if constexpr (LW == 1) {
    x[0] = NT ? __builtin_nontemporal_load(reinterpret_cast<const u32_ua*>(p)) : *reinterpret_cast<const u32_ua*>(p);
  } else {
    const u32x2 v = NT ? __builtin_nontemporal_load(reinterpret_cast<const u32x2_ua*>(p))
                       : *reinterpret_cast<const u32x2_ua*>(p);
    x[0] = v.x, x[1] = v.y;
  }
}

template <int LW, bool NTS, int SP = CFSEC_STORE_POL>
__device__ __forceinline__ void st_chunk(uint8_t* p, const uint32_t (&x)[LW]) {
  if constexpr (LW == 4) {
    if constexpr (NTS) st16_pol<SP>(p, u32x4{x[0], x[1], x[2], x[3]});
    else st16<false>(p, u32x4{x[0], x[1], x[2], x[3]});
  } else if constexpr (LW == 1) {
    if constexpr (NTS) __builtin_nontemporal_store(x[0], reinterpret_cast<u32_ua*>(p));
    else *reinterpret_cast<u32_ua*>(p) = x[0];
  } else if constexpr (NTS) {
    __builtin_nontemporal_store(u32x2{x[0], x[1]}, reinterpret_cast<u32x2_ua*>(p));
  } else {
    *reinterpret_cast<u32x2_ua*>(p) = u32x2{x[0], x[1]};
  }
}

// Lane chunk of the fixed-K kernel for K inputs and M outputs per wave: 16 bytes, or 8 where the
// wave holds many output rows -- K + M chunks of accumulators and inputs at 16 B per lane need
// 130-210 VGPRs for M >= 10 (2-3 waves per SIMD), at 8 B half of that.
#ifndef CFSEC_LANE8_MIN_M
#define CFSEC_LANE8_MIN_M 10
#endif
constexpr int fixed_lane_dwords(int K, int M) { return M >= CFSEC_LANE8_MIN_M ? 2 : 4; }

// Tiles one workgroup of the fixed-K kernel codes, in sequence, for M <= CFSEC_FIXED_TPW_MAXM: a
// single-output matrix (the LRC local stripes) does K loads and one store per lane, so the table
// build and barrier are a visible share of a one-tile workgroup.
#ifndef CFSEC_FIXED_TPW
#define CFSEC_FIXED_TPW 1
#endif
#ifndef CFSEC_FIXED_TPW_MAXM
#define CFSEC_FIXED_TPW_MAXM 1
#endif
constexpr int fixed_tiles_per_wg(int M) { return M <= CFSEC_FIXED_TPW_MAXM ? CFSEC_FIXED_TPW : 1; }

// Product tables of one coefficient:
//   t01 = {T0[0..3], T0[4..7], T1[0..3], T1[4..7]},  t2 = T2[0..3]
// with T0[e] = coef*e, T1[e] = coef*(e<<3), T2[e] = coef*(e<<6).
__device__ __forceinline__ void coef_tables(uint32_t coef, u32x4& t01, uint32_t& t2) {
  uint32_t p[8];
  p[0] = coef;
#pragma unroll
  for (int j = 1; j < 8; ++j) p[j] = gf_xtime(p[j - 1]);  // coef * 2^j
  uint32_t t0lo = 0, t0hi = 0, t1lo = 0, t1hi = 0, tt2 = 0;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const uint32_t v0 = ((e & 1) ? p[0] : 0u) ^ ((e & 2) ? p[1] : 0u) ^ ((e & 4) ? p[2] : 0u);
    const uint32_t v1 = ((e & 1) ? p[3] : 0u) ^ ((e & 2) ? p[4] : 0u) ^ ((e & 4) ? p[5] : 0u);
    if (e < 4) {
      const uint32_t v2 = ((e & 1) ? p[6] : 0u) ^ ((e & 2) ? p[7] : 0u);
      t0lo |= v0 << (8 * e);
      t1lo |= v1 << (8 * e);
      tt2 |= v2 << (8 * e);
    } else {
      t0hi |= v0 << (8 * (e - 4));
      t1hi |= v1 << (8 * (e - 4));
    }
  }
  t01 = u32x4{t0lo, t0hi, t1lo, t1hi};
  t2 = tt2;
}

// Product tables for coefficient (c, r) at LDS slot c*MT + r (MT = output rows per block).
template <int MT>
__device__ __forceinline__ void build_tables(int k, int m, const uint8_t* coef, u32x4* tab01, uint32_t* tab2) {
  for (int i = threadIdx.x; i < k * MT; i += (int)blockDim.x) {
    const int c = i / MT;
    const int r = i - c * MT;
    coef_tables((r < m) ? coef[r * k + c] : 0u, tab01[i], tab2[i]);
  }
}

template <int MT>
__device__ __forceinline__ void build_tables(const GfArgs& a, u32x4* tab01, uint32_t* tab2) {
  build_tables<MT>((int)a.k, (int)a.m, a.coef, tab01, tab2);
}

// acc[r] ^= coef(c, r) * x for the wave's M outputs; x is 16 bytes of input row c and
// tq/t2p point at this wave's first output of input row c.
template <int M>
__device__ __forceinline__ void mac_row(u32x4 (&acc)[M], u32x4 x, const u32x4* __restrict__ tq,
                                        const uint32_t* __restrict__ t2p) {
  const u32x4 s0 = x & 0x07070707u;
  const u32x4 s1 = (x >> 3) & 0x07070707u;
  const u32x4 s2 = (x >> 6) & 0x03030303u;
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
}

// Store / accumulate / compare the wave's outputs og .. og+M-1 (rows past a.m are padding).
template <int M, MatVecMode MODE, bool NTL, bool NTS>
__device__ __forceinline__ void finish(const GfArgs& a, u32x4 (&acc)[M], uint8_t* const* out,
                                       int og, size_t off, uint32_t& diff) {
  const int m = (int)a.m;
#pragma unroll
  for (int r = 0; r < M; ++r) {
    if (og + r < m) {
      uint8_t* p = out[og + r] + off;
      if (row_compared<MODE>(a, og + r)) {
        const u32x4 d = acc[r] ^ ld16<NTL>(p);
        diff |= d.x | d.y | d.z | d.w;
      } else {
        u32x4 v = acc[r];
        if constexpr (MODE == MatVecMode::kAccum) v ^= ld16<NTL>(p);
        st16<NTS>(p, v);
      }
    }
  }
}

// One lane's chunk at the end of a shard (rem < 16 bytes): byte stores; the loads are one 16-byte
// load of the row's last 16 bytes shifted down (ld_tail_row; `len` is the row's length), not 16
// dependent byte loads per row.
template <int M, int MT, MatVecMode MODE>
__device__ __forceinline__ void lane_tail(const GfArgs& a, const u32x4* tab01, const uint32_t* tab2,
                                          const uint8_t* const* in, uint8_t* const* out, int og,
                                          size_t off, size_t rem, uint64_t len, uint32_t& diff) {
  const int k = (int)a.k, m = (int)a.m;
  u32x4 acc[M];
#pragma unroll
  for (int r = 0; r < M; ++r) acc[r] = u32x4{0u, 0u, 0u, 0u};
  for (int c = 0; c < k; ++c)
    mac_row<M>(acc, ld_tail_row(in[c] + off, rem, len), tab01 + c * MT + og, tab2 + c * MT + og);
#pragma unroll
  for (int r = 0; r < M; ++r) {
    if (og + r < m) {
      uint8_t* p = out[og + r] + off;
      if (row_compared<MODE>(a, og + r)) {
        const u32x4 d = acc[r] ^ ld_tail_row(p, rem, len);
        diff |= d.x | d.y | d.z | d.w;
      } else {
        u32x4 v = acc[r];
        if constexpr (MODE == MatVecMode::kAccum) v ^= ld_tail_row(p, rem, len);
        st_tail(p, v, rem);
      }
    }
  }
}

// lane_tail for a compile-time input count, one input row at a time (a rolled loop: unrolled, every
// row's 16 byte loads were hoisted together and this rarely-taken path set the kernel's register
// count -- C4's (8, 1) kernel 72 VGPRs against 48 for the full-tile path)
template <int K, int M, int MT, MatVecMode MODE>
__device__ __forceinline__ void lane_tail_k(const GfArgs& a, const u32x4* tab01, const uint32_t* tab2,
                                            const uint8_t* const* in, uint8_t* const* out, int og,
                                            size_t off, size_t rem, uint32_t& diff) {
  const int m = (int)a.m;
  u32x4 acc[M];
#pragma unroll
  for (int r = 0; r < M; ++r) acc[r] = u32x4{0u, 0u, 0u, 0u};
#pragma unroll 1
  for (int c = 0; c < K; ++c)
    mac_row<M>(acc, ld_tail(in[c] + off, rem), tab01 + c * MT + og, tab2 + c * MT + og);
#pragma unroll
  for (int r = 0; r < M; ++r) {
    if (og + r < m) {
      uint8_t* p = out[og + r] + off;
      if (row_compared<MODE>(a, og + r)) {
        const u32x4 d = acc[r] ^ ld_tail(p, rem);
        diff |= d.x | d.y | d.z | d.w;
      } else {
        st_tail(p, acc[r], rem);
      }
    }
  }
}

// Full tile: W chunks per lane, all in bounds.  Input rows are loaded G at a time.
template <int M, int MT, MatVecMode MODE, int W, int G, bool NTL, bool NTS>
__device__ __forceinline__ void lane_tile(const GfArgs& a, const u32x4* tab01, const uint32_t* tab2,
                                          const uint8_t* const* in, uint8_t* const* out, int og,
                                          size_t off, size_t kStep, uint32_t& diff) {
  const int k = (int)a.k;
  u32x4 acc[W][M];
#pragma unroll
  for (int w = 0; w < W; ++w)
#pragma unroll
    for (int r = 0; r < M; ++r) acc[w][r] = u32x4{0u, 0u, 0u, 0u};
  for (int c0 = 0; c0 < k; c0 += G) {
    u32x4 x[G][W];
#pragma unroll
    for (int g = 0; g < G; ++g)
      if (c0 + g < k)
#pragma unroll
        for (int w = 0; w < W; ++w) x[g][w] = ld16<NTL>(in[c0 + g] + off + w * kStep);
#pragma unroll
    for (int g = 0; g < G; ++g)
      if (c0 + g < k)
#pragma unroll
        for (int w = 0; w < W; ++w)
          mac_row<M>(acc[w], x[g][w], tab01 + (c0 + g) * MT + og, tab2 + (c0 + g) * MT + og);
  }
#pragma unroll
  for (int w = 0; w < W; ++w) finish<M, MODE, NTL, NTS>(a, acc[w], out, og, off + w * kStep, diff);
}

// acc[r][w] ^= coef(c, r) * x[w] on plain dword arrays (the fixed-K tile's form of mac_row).
template <int M, int W = 4>
__device__ __forceinline__ void mac_row_k(uint32_t (&acc)[M][W], const uint32_t (&x)[W],
                                          const u32x4* __restrict__ tq, const uint32_t* __restrict__ t2p) {
  uint32_t s0[W], s1[W], s2[W];
#pragma unroll
  for (int w = 0; w < W; ++w) {
    s0[w] = x[w] & 0x07070707u;
    s1[w] = (x[w] >> 3) & 0x07070707u;
    s2[w] = (x[w] >> 6) & 0x03030303u;
  }
#pragma unroll
  for (int r = 0; r < M; ++r) {
    const u32x4 q = tq[r];
    const uint32_t t2 = t2p[r];
#pragma unroll
    for (int w = 0; w < W; ++w) {
      const uint32_t p0 = __builtin_amdgcn_perm(q.y, q.x, s0[w]);
      const uint32_t p1 = __builtin_amdgcn_perm(q.w, q.z, s1[w]);
      const uint32_t p2 = __builtin_amdgcn_perm(0u, t2, s2[w]);
      acc[r][w] = __builtin_amdgcn_bitop3_b32(acc[r][w], p0, p1, 0x96) ^ p2;
    }
  }
}

// Two input rows at once: acc ^= coef(a, r)*xa ^ coef(b, r)*xb.  The six table lookups per output
// dword fold into acc with three 3-input XORs (v_bitop3_b32 0x96) instead of four XOR ops for
// two single rows: 9 VALU ops per (output, dword, row pair) instead of 10.
template <int M, int W = 4>
__device__ __forceinline__ void mac_pair_k(uint32_t (&acc)[M][W], const uint32_t (&xa)[W],
                                           const uint32_t (&xb)[W], const u32x4* __restrict__ tqa,
                                           const uint32_t* __restrict__ t2a, const u32x4* __restrict__ tqb,
                                           const uint32_t* __restrict__ t2b) {
  uint32_t a0[W], a1[W], a2[W], b0[W], b1[W], b2[W];
#pragma unroll
  for (int w = 0; w < W; ++w) {
    a0[w] = xa[w] & 0x07070707u;
    a1[w] = (xa[w] >> 3) & 0x07070707u;
    a2[w] = (xa[w] >> 6) & 0x03030303u;
    b0[w] = xb[w] & 0x07070707u;
    b1[w] = (xb[w] >> 3) & 0x07070707u;
    b2[w] = (xb[w] >> 6) & 0x03030303u;
  }
#pragma unroll
  for (int r = 0; r < M; ++r) {
    const u32x4 qa = tqa[r], qb = tqb[r];
    const uint32_t ta = t2a[r], tb = t2b[r];
#pragma unroll
    for (int w = 0; w < W; ++w) {
      const uint32_t u = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_perm(qa.y, qa.x, a0[w]),
                                                     __builtin_amdgcn_perm(qa.w, qa.z, a1[w]),
                                                     __builtin_amdgcn_perm(0u, ta, a2[w]), 0x96);
      const uint32_t v = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_perm(qb.y, qb.x, b0[w]),
                                                     __builtin_amdgcn_perm(qb.w, qb.z, b1[w]),
                                                     __builtin_amdgcn_perm(0u, tb, b2[w]), 0x96);
      acc[r][w] = __builtin_amdgcn_bitop3_b32(acc[r][w], u, v, 0x96);
    }
  }
}

// Full tile for a compile-time input count K, one 16-B chunk per lane at byte `loff` of every row.
// The rows a lane touches (K inputs, then in verify mode the M rows it compares) form one load
// sequence in which row c+D is issued before row c is consumed, so D loads per wave stay in
// flight while the multiply runs.  The order is enforced, not hoped for: with the whole tile in
// one basic block the scheduler otherwise hoists every load and table read to the top (270-356
// VGPRs for K=12, M=4: one or two waves per SIMD), so each row ends by pinning the accumulators
// (empty asm) behind a sched_barrier, and the row pointers (uniform: SGPR bases, 32-bit lane
// offsets) are loaded once up front.  tools/gf_pipe.hip measured the effect.
// PIN: the product tables are uniform values (register tables, matvec_k REG) -- read with the row
// pointers, before the first barrier, so that both arrive in one round trip.
template <int K, int M, int MT, MatVecMode MODE, int D, bool NTL, bool NTS, bool PAIR = true, int LW = 4,
          int SP = CFSEC_STORE_POL, bool PIN = false>
__device__ __forceinline__ void lane_tile_k(int m, int nstore, const u32x4* tab01_in, const uint32_t* tab2_in,
                                            const uint8_t* const* in, uint8_t* const* out, int og,
                                            int64_t sbase, uint32_t loff, uint32_t& diff) {
  static_assert(D >= 2, "the fixed-K tile consumes input rows in pairs, a pair ahead");
  constexpr bool kVer = MODE == MatVecMode::kVerify;
  constexpr bool kMix = MODE == MatVecMode::kStoreVerify;  // rows < nstore stored, the rest compared
  if constexpr (kVer) nstore = 0;
  else if constexpr (!kMix) nstore = m;
  constexpr int R = K + (kVer || kMix ? M : 0);  // rows loaded
  const uint8_t* row[R];
#pragma unroll
  for (int c = 0; c < K; ++c) row[c] = in[c] + sbase;
#pragma unroll
  for (int r = 0; r < R - K; ++r) row[K + r] = out[og + r < m ? og + r : og] + sbase;
  u32x4 p01[PIN ? K * MT : 1];
  uint32_t p2[PIN ? K * MT : 1];
  if constexpr (PIN) {
#pragma unroll
    for (int i = 0; i < K * MT; ++i) {
      p01[i] = tab01_in[i];
      p2[i] = tab2_in[i];
      asm volatile("" : "+s"(p01[i].x), "+s"(p01[i].y), "+s"(p01[i].z), "+s"(p01[i].w), "+s"(p2[i]));
    }
  }
  const u32x4* tab01 = PIN ? p01 : tab01_in;
  const uint32_t* tab2 = PIN ? p2 : tab2_in;
  __builtin_amdgcn_sched_barrier(0);

  uint32_t acc[M][LW];
#pragma unroll
  for (int r = 0; r < M; ++r)
#pragma unroll
    for (int w = 0; w < LW; ++w) acc[r][w] = 0u;
  uint32_t x[R][LW];
  const auto load = [&](int c) {
    if (c >= K && (og + (c - K) >= m || og + (c - K) < nstore)) return;  // padding / stored row
    ld_chunk<LW, NTL>(row[c] + loff, x[c]);
  };
  const auto pin = [&]() {
#pragma unroll
    for (int r = 0; r < M; ++r)
#pragma unroll
      for (int w = 0; w < LW; ++w) asm volatile("" : "+v"(acc[r][w]));
  };
#pragma unroll
  for (int c = 0; c < D && c < R; ++c) load(c);
  // inputs two rows per step, an odd K's last row alone
#pragma unroll
  for (int c = 0; c + 1 < K; c += 2) {
    if (c + D < R) load(c + D);
    if (c + D + 1 < R) load(c + D + 1);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (PAIR) {
      mac_pair_k<M>(acc, x[c], x[c + 1], tab01 + c * MT + og, tab2 + c * MT + og, tab01 + (c + 1) * MT + og,
                    tab2 + (c + 1) * MT + og);
    } else {
      mac_row_k<M>(acc, x[c], tab01 + c * MT + og, tab2 + c * MT + og);
      pin();
      mac_row_k<M>(acc, x[c + 1], tab01 + (c + 1) * MT + og, tab2 + (c + 1) * MT + og);
    }
    pin();
    __builtin_amdgcn_sched_barrier(0);
  }
  if constexpr (K % 2 == 1) {
    constexpr int c = K - 1;  // rows up to c + D - 1 are loaded or in flight
    if (c + D < R) load(c + D);
    __builtin_amdgcn_sched_barrier(0);
    mac_row_k<M>(acc, x[c], tab01 + c * MT + og, tab2 + c * MT + og);
    pin();
    __builtin_amdgcn_sched_barrier(0);
  }
  // verify: compare the computed rows with the stored ones
#pragma unroll
  for (int c = K; c < R; ++c) {
    if (c + D < R) load(c + D);
    __builtin_amdgcn_sched_barrier(0);
    if (og + (c - K) < m && og + (c - K) >= nstore) {
      const int r = c - K;
#pragma unroll
      for (int w = 0; w < LW; ++w) diff |= acc[r][w] ^ x[c][w];
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  if constexpr (!kVer) {
#pragma unroll
    for (int r = 0; r < M; ++r) {
      if (og + r < m && og + r < nstore) {
        uint8_t* p = out[og + r] + sbase + loff;
        if constexpr (MODE == MatVecMode::kAccum) {
          uint32_t y[LW];
          ld_chunk<LW, NTL>(p, y);
#pragma unroll
          for (int w = 0; w < LW; ++w) acc[r][w] ^= y[w];
        }
        st_chunk<LW, NTS, SP>(p, acc[r]);
      }
    }
  }
}

// Kernel body for a compile-time input count (a.k == K, a.len < 4 GiB): 256-thread workgroups,
// one chunk of LW dwords per lane, tile = (256/OS)*4*LW bytes of every row, grid (tiles,
// stripes); otherwise as matvec below.
template <int K, int M, MatVecMode MODE, int D, int OS, bool NTL = true, bool NTS = true, bool PAIR = true,
          int LW = 4, int TPW = 1, bool REG = false, int SP = CFSEC_STORE_POL>
__device__ __forceinline__ void matvec_k(const GfArgs& a) {
  static_assert(!REG || OS == 1, "register tables: one wave per column chunk");
  static_assert(MODE != MatVecMode::kAccum, "the clamped row end re-codes bytes: stores and compares only");
  constexpr int MT = M * OS;
  // REG: the host packed each coefficient's tables into the argument block's coef area, from byte
  // kRegTabOff (16-byte aligned in the block): t01 of coefficient (c, r) as the (c * M + r)-th
  // u32x4, then the t2 words -- read straight from the argument block (scalar loads), no LDS build,
  // no barrier (single-output products: 0.65 -> 0.74-0.77 of 8 TB/s, tools/c4l_pattern_probe.hip)
  // The full-tile path takes them as register copies made up front (read through the argument-block
  // pointer inside the tile, each row's table waited for its own scalar load: 57 vs 51 us on C4's
  // (8, 1)); the rarely-taken tail path indexes the argument block row by row.
  __shared__ u32x4 lds01[REG ? 1 : K * MT];
  __shared__ uint32_t lds2[REG ? 1 : K * MT];
  const u32x4* ktab01 = reinterpret_cast<const u32x4*>(a.coef + kRegTabOff);
  const uint32_t* ktab2 = reinterpret_cast<const uint32_t*>(a.coef + kRegTabOff + 16 * K * MT);
  u32x4 reg01[REG ? K * MT : 1];
  uint32_t reg2[REG ? K * MT : 1];
  if constexpr (REG) {
#pragma unroll
    for (int i = 0; i < K * MT; ++i) {
      reg01[i] = ktab01[i];
      reg2[i] = ktab2[i];
    }
  } else {
    build_tables<MT>(a, lds01, lds2);
    __syncthreads();
  }
  const u32x4* tab01 = REG ? reg01 : lds01;
  const uint32_t* tab2 = REG ? reg2 : lds2;
  const u32x4* tail01 = REG ? ktab01 : lds01;
  const uint32_t* tail2 = REG ? ktab2 : lds2;

  const int wave = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
  const int og = (wave % OS) * M;
  const int cw = wave / OS;
  constexpr uint32_t kLB = 4 * LW;  // bytes per lane chunk
  constexpr uint32_t kTile = uint32_t(kThreads / OS) * kLB;
  // 2-D grid (x: runs of TPW tiles of a stripe, y: stripes): a division of blockIdx.x would expand
  // to VALU code and drag the row pointers into VGPRs
  const uint32_t stripe = blockIdx.y;
  // Every argument word the row pointers and the stripe's length depend on, read in one round (the
  // empty asm makes all of them live at once, so no load waits behind a branch on another): a
  // workgroup codes one tile, so each dependent round trip to the argument block before its first
  // row load shows (the stripe's length is selected, not branched on)
  uint32_t varlen = a.varlen, tab = a.tab;
  uint32_t slen = a.slen[stripe < (uint32_t)kLenSlots ? stripe : (uint32_t)kLenSlots - 1];
  uint64_t len0 = a.len;
  int64_t sstride = a.sstride;
  asm volatile("" : "+s"(varlen), "+s"(tab), "+s"(slen), "+s"(len0), "+s"(sstride));
  const uint32_t mrows = a.m;
  const uint64_t len = varlen ? (uint64_t)slen : len0;
  const size_t tstripe = sstride ? 0 : (size_t)stripe;
  const int64_t sbase = (int64_t)stripe * sstride;
  const uint8_t* const* in = a.ptr + tstripe * K;
  uint8_t* const* out = const_cast<uint8_t* const*>(a.ptr + (size_t)tab * K + tstripe * mrows);
  uint32_t diff = 0;
#pragma unroll 1
  for (int j = 0; j < TPW; ++j) {
    const uint32_t tile = blockIdx.x * TPW + j;
    if (TPW > 1 && tile >= a.tiles_per_stripe) break;
    const uint32_t off = tile * kTile + (uint32_t)(cw * 64 + lane) * kLB;
    // (m stays the launch's run-time value although it equals M here.  Round 5 saw the compile-time M
    // return wrong rows -- the store-data hazard of st16_pol, above; with hazard-free stores that
    // form is bit-exact and measured no faster, profiles/r06/shape_sweep_store_variants.txt)
    // The ragged end of a row: the lane holding it codes the last full chunk of the row instead
    // (clamped to end at len: its bytes before the end repeat its neighbour's, with the same values --
    // plain stores and compares, never an accumulate), so every lane takes the one full-chunk path.
    // A per-lane byte tail beside it cost 10 % on C4's (8, 1) product (56 vs 50 us,
    // tools/c4l_pattern_probe.hip "regx F1" / "F8"); rows shorter than a chunk keep the byte path,
    // under a branch uniform over the stripe.
    if (og < (int)mrows && off < len) {
      if (len >= kLB) {
        const uint32_t loff = (uint64_t)off + kLB <= len ? off : (uint32_t)(len - kLB);
        lane_tile_k<K, M, MT, MODE, D, NTL, NTS, PAIR, LW, SP>((int)mrows, (int)a.nstore, tab01, tab2, in, out, og,
                                                               sbase, loff, diff);
      } else {
        lane_tail_k<K, M, MT, MODE>(a, tail01, tail2, in, out, og, (size_t)sbase + off, len - off, diff);
      }
    }
  }
  if constexpr (MODE == MatVecMode::kVerify || MODE == MatVecMode::kStoreVerify) {
    if (diff) dev::set_flag(a.flags, stripe);
  }
}

// Kernel body.  A tile is (blockDim.x/OS)*16*W bytes of every row of one stripe; wave v of the
// workgroup covers column chunk v/OS of it and output rows (v%OS)*M .. +M.
template <int M, MatVecMode MODE, int W, int G, bool PERSIST, bool NTL, bool NTS, bool XCD,
          bool WAVEC = false, int OS = 1>
__device__ __forceinline__ void matvec(const GfArgs& a) {
  constexpr int MT = M * OS;  // output rows per workgroup
  __shared__ u32x4 tab01[kMaxK * MT];
  __shared__ uint32_t tab2[kMaxK * MT];
  build_tables<MT>(a, tab01, tab2);
  __syncthreads();

  const int wave = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
  const int og = (wave % OS) * M;   // this wave's first output row
  const int cw = wave / OS;         // this wave's column chunk
  const size_t col_threads = size_t(blockDim.x) / OS;
  const size_t kStep = WAVEC ? size_t(64) * kLaneBytes : col_threads * kLaneBytes;
  const size_t kTile = col_threads * kLaneBytes * W;
  const size_t lane_off = WAVEC ? (size_t)cw * (64 * kLaneBytes * W) + (size_t)lane * kLaneBytes
                                : ((size_t)cw * 64 + lane) * kLaneBytes;
  const uint32_t tps = a.tiles_per_stripe;
  const uint32_t ntiles = tps * a.nstripes;
  uint32_t diff = 0;
  uint32_t first = blockIdx.x;
  if constexpr (XCD) {
    // blocks b and b+8 share an XCD: give XCD x the contiguous run [x*per, (x+1)*per)
    const uint32_t nb = gridDim.x, per = nb / 8;
    if (per && blockIdx.x < per * 8) first = (blockIdx.x % 8) * per + blockIdx.x / 8;
  }
  for (uint32_t t = first; t < ntiles; t += (PERSIST ? gridDim.x : ntiles)) {
    const int stripe = (int)(t / tps);
    const size_t tile = t - (size_t)stripe * tps;
    // explicit table: this stripe's own pointers; affine batch: stripe 0's plus a byte offset
    const size_t tstripe = a.sstride ? 0 : (size_t)stripe;
    const size_t soff = (size_t)((int64_t)stripe * a.sstride);
    const uint8_t* const* in = a.ptr + tstripe * a.k;
    uint8_t* const* out = const_cast<uint8_t* const*>(a.ptr + (size_t)a.tab * a.k + tstripe * a.m);
    const size_t off = tile * kTile + lane_off;  // byte offset inside the shard
    const uint64_t len = stripe_len(a, (uint32_t)stripe);
    if (og < (int)a.m) {  // waves whose output rows are all padding have nothing to do
      if (off + (W - 1) * kStep + kLaneBytes <= len) {
        lane_tile<M, MT, MODE, W, G, NTL, NTS>(a, tab01, tab2, in, out, og, soff + off, kStep, diff);
      } else {
#pragma unroll
        for (int w = 0; w < W; ++w) {
          const size_t o = off + w * kStep;
          if (o + kLaneBytes <= len) {
            lane_tile<M, MT, MODE, 1, G, NTL, NTS>(a, tab01, tab2, in, out, og, soff + o, kStep, diff);
          } else if (o < len) {
            // The ragged end of a row: stores and compares code the row's last full chunk instead (its
            // bytes before the end repeat a neighbour's, with the same values), as the fixed-K, dyadic
            // and lookup kernels do; an accumulate cannot re-code bytes and keeps the byte stores.
            if (MODE != MatVecMode::kAccum && len >= kLaneBytes)
              lane_tile<M, MT, MODE, 1, G, NTL, NTS>(a, tab01, tab2, in, out, og, soff + (len - kLaneBytes), kStep,
                                                     diff);
            else
              lane_tail<M, MT, MODE>(a, tab01, tab2, in, out, og, soff + o, len - o, len, diff);
          }
        }
      }
    }
    if constexpr (MODE == MatVecMode::kVerify || MODE == MatVecMode::kStoreVerify) {
      if (diff) {
        dev::set_flag(a.flags, stripe);
        diff = 0;
      }
    }
  }
}

}  // namespace dev
}  // namespace cfsec
