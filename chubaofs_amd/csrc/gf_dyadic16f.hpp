// gf_dyadic16f.hpp -- the 16x16-dyadic kernels of gf_dyadic16.hpp with every multiplicand kept as
// its three v_perm selector fields ("field form") instead of a byte vector.
//
// A product c * x takes three v_perm_b32 lookups whose selectors are the bit fields of x:
// a = x & 0x07070707 ([2:0]), b = (x >> 3) & 0x07070707 ([5:3]), c = (x >> 6) & 0x03030303 ([7:6]),
// 5 VALU ops per dword.  The fields are GF(2)-linear in x -- fields(x ^ y) = fields(x) ^ fields(y)
// -- so the XOR combinations the dyadic recursion multiplies (S = X + Y, Y_lo + Y_hi, the leaves'
// u = x0^x1^x2^x3, s = x1^x3, v = x2^x3) can be formed on the fields directly: 3 XORs (one
// v_bitop3_b32 per field for a 3-term sum) instead of 1 XOR + 5 selector ops per combination.  The
// 16 inputs' fields are computed once; the byte form is never rebuilt.
//
// Measured (PMC, profiles/r04/pmc_c5.txt): the byte-form repair kernel of C5's tasklet issues ~1500
// VALU ops per dword column and runs VALU-issue-bound (98.4 M wave-instructions for 175 us at the
// measured v_perm / v_bitop3 rate); ~28 % of them formed selectors, ~7 % were v_cndmask of the
// run-time data-row permutation, which this form replaces by loading inputs in data-row slots and
// one uniform branch per missing row.  The cost is registers: 3 per multiplicand dword instead of 1,
// hence 4-byte lanes (W = 1) by default.
#pragma once
#include "gf_dyadic16.hpp"

namespace cfsec {
namespace dev {

template <int W>
struct Fld {
  uint32_t a[W], b[W], c[W];
};

template <int W>
__device__ __forceinline__ void to_fields(const uint32_t (&x)[W], Fld<W>& f) {
#pragma unroll
  for (int w = 0; w < W; ++w) {
    f.a[w] = x[w] & 0x07070707u;
    f.b[w] = (x[w] >> 3) & 0x07070707u;
    f.c[w] = (x[w] >> 6) & 0x03030303u;
  }
}

template <int W>
__device__ __forceinline__ void fxor(Fld<W>& d, const Fld<W>& s) {
#pragma unroll
  for (int w = 0; w < W; ++w) {
    d.a[w] ^= s.a[w];
    d.b[w] ^= s.b[w];
    d.c[w] ^= s.c[w];
  }
}

template <int W>
__device__ __forceinline__ Fld<W> fsum2(const Fld<W>& x, const Fld<W>& y) {
  Fld<W> r;
#pragma unroll
  for (int w = 0; w < W; ++w) {
    r.a[w] = x.a[w] ^ y.a[w];
    r.b[w] = x.b[w] ^ y.b[w];
    r.c[w] = x.c[w] ^ y.c[w];
  }
  return r;
}

template <int W>
__device__ __forceinline__ Fld<W> fsum3(const Fld<W>& x, const Fld<W>& y, const Fld<W>& z) {
  Fld<W> r;
#pragma unroll
  for (int w = 0; w < W; ++w) {
    r.a[w] = x3(x.a[w], y.a[w], z.a[w]);
    r.b[w] = x3(x.b[w], y.b[w], z.b[w]);
    r.c[w] = x3(x.c[w], y.c[w], z.c[w]);
  }
  return r;
}

// The three partial lookups of coefficient (q, t2) times the multiplicand with fields f.
template <int W>
__device__ __forceinline__ void flook(const u32x4 q, uint32_t t2, const Fld<W>& f, ProdW<W>& p) {
#pragma unroll
  for (int w = 0; w < W; ++w) {
    p.a[w] = __builtin_amdgcn_perm(q.y, q.x, f.a[w]);
    p.b[w] = __builtin_amdgcn_perm(q.w, q.z, f.b[w]);
    p.c[w] = __builtin_amdgcn_perm(0u, t2, f.c[w]);
  }
}

// acc[r] ^= coef(a, r) * xa ^ coef(b, r) * xb for M rows (tables at tqa/t2a, tqb/t2b, row stride 1)
template <int M, int W>
__device__ __forceinline__ void fmac_pair(uint32_t (&acc)[M][W], const Fld<W>& xa, const Fld<W>& xb,
                                          const u32x4* tqa, const uint32_t* t2a, const u32x4* tqb,
                                          const uint32_t* t2b) {
#pragma unroll
  for (int r = 0; r < M; ++r) {
    ProdW<W> pa, pb;
    flook(tqa[r], t2a[r], xa, pa);
    flook(tqb[r], t2b[r], xb, pb);
#pragma unroll
    for (int w = 0; w < W; ++w)
      acc[r][w] = x3(acc[r][w], x3(pa.a[w], pa.b[w], pa.c[w]), x3(pb.a[w], pb.b[w], pb.c[w]));
  }
}

// The 4x4 dyadic product of gf_dyadic.hpp dy_col4 on field-form inputs (MB row blocks).
template <int MB, bool PIN, int W>
__device__ __forceinline__ void fdy_col4(uint32_t (&acc)[4 * MB][W], const Fld<W>& f0, const Fld<W>& f1,
                                         const Fld<W>& f2, const Fld<W>& f3, const u32x4* tq, const uint32_t* t2p,
                                         int stride) {
  const Fld<W> s = fsum2(f1, f3), v = fsum2(f2, f3), u = fsum3(f0, f2, s);  // u = x0^x1^x2^x3
#pragma unroll
  for (int rb = 0; rb < MB; ++rb) {
    const u32x4* q = tq + rb * stride;
    const uint32_t* t = t2p + rb * stride;
    uint32_t ps[W], ps2[W], c0[W], c1[W];
    {
      ProdW<W> p;
      flook(q[2], t[2], s, p);  // (h0^h1) s
#pragma unroll
      for (int w = 0; w < W; ++w) ps[w] = x3(p.a[w], p.b[w], p.c[w]);
      flook(q[5], t[5], s, p);  // (h2^h3) s
#pragma unroll
      for (int w = 0; w < W; ++w) ps2[w] = x3(p.a[w], p.b[w], p.c[w]);
      ProdW<W> py, p6, p7;
      flook(q[8], t[8], f3, py);  // (g0^g1) x3
      flook(q[6], t[6], v, p6);   // g0 v
      flook(q[7], t[7], v, p7);   // g1 v
#pragma unroll
      for (int w = 0; w < W; ++w) {
        const uint32_t qy = x3(py.a[w], py.b[w], py.c[w]);
        c0[w] = x3(p6.a[w], p6.b[w], p6.c[w]) ^ qy;
        c1[w] = x3(p7.a[w], p7.b[w], p7.c[w]) ^ qy;
      }
    }
    if constexpr (PIN) {
#pragma unroll
      for (int w = 0; w < W; ++w) asm volatile("" : "+v"(ps[w]), "+v"(ps2[w]), "+v"(c0[w]), "+v"(c1[w]));
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      ProdW<W> p;
      const int qi = j < 2 ? j : j + 1;  // h0, h1, h2, h3 at slots 0, 1, 3, 4
      flook(q[qi], t[qi], u, p);
      const uint32_t* sh = j < 2 ? ps : ps2;
      const uint32_t* cc = (j & 1) ? c1 : c0;
#pragma unroll
      for (int w = 0; w < W; ++w)
        acc[4 * rb + j][w] = x3(x3(acc[4 * rb + j][w], p.a[w], p.b[w]), x3(p.c[w], sh[w], cc[w]), 0u);
      if constexpr (PIN) {
#pragma unroll
        for (int w = 0; w < W; ++w) asm volatile("" : "+v"(acc[4 * rb + j][w]));
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
}

template <bool PIN, int W>
__device__ __forceinline__ void fleaf4(VecW4<W>& acc, const Fld<W>* f, const u32x4* tab01, const uint32_t* tab2,
                                       int leaf) {
  fdy_col4<1, PIN, W>(acc, f[0], f[1], f[2], f[3], tab01 + leaf * 9, tab2 + leaf * 9, 0);
}

// dy16_rows on field-form inputs f[16] (the 16 data rows, clobbered): rows 16.. (the R4 4x4 row
// blocks, then the E plain rows) first, then the 16x16 block; put(r, chunk) receives each row.
template <int R4, int E, bool PIN, int W, class Put>
__device__ __forceinline__ void fdy16_rows(Fld<W> (&f)[16], const u32x4* tab01, const uint32_t* tab2, Put&& put) {
  constexpr int K = 16, N4 = R4 * 4 * 9;
  constexpr int NA = 16 + (4 * R4 > E ? 4 * R4 : E);
  uint32_t acc[NA][W];
#pragma unroll
  for (int r = 0; r < NA; ++r)
#pragma unroll
    for (int w = 0; w < W; ++w) acc[r][w] = 0u;
  const auto sb = [&]() {
    if constexpr (PIN) __builtin_amdgcn_sched_barrier(0);
  };
  sb();
  if constexpr (R4 > 0) {
    const u32x4* tq = tab01 + kDy16Leaves;
    const uint32_t* tt = tab2 + kDy16Leaves;
    auto& racc = reinterpret_cast<uint32_t(&)[4 * R4][W]>(acc[16]);
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      fdy_col4<R4, PIN, W>(racc, f[4 * cb], f[4 * cb + 1], f[4 * cb + 2], f[4 * cb + 3], tq + cb * 9, tt + cb * 9,
                           4 * 9);
      sb();
    }
#pragma unroll
    for (int r = 16; r < 16 + 4 * R4; ++r) put(r, acc[r]);
    sb();
#pragma unroll
    for (int r = 16; r < NA; ++r)
#pragma unroll
      for (int w = 0; w < W; ++w) acc[r][w] = 0u;
  }
  if constexpr (E > 0) {
    auto& eacc = reinterpret_cast<uint32_t(&)[E][W]>(acc[16]);
    constexpr int ND = kDy16Leaves + N4;
#pragma unroll
    for (int c = 0; c < K; c += 2) {
      fmac_pair<E, W>(eacc, f[c], f[c + 1], tab01 + ND + c * E, tab2 + ND + c * E, tab01 + ND + (c + 1) * E,
                      tab2 + ND + (c + 1) * E);
      if constexpr (PIN)
#pragma unroll
        for (int e = 0; e < E; ++e)
#pragma unroll
          for (int w = 0; w < W; ++w) asm volatile("" : "+v"(eacc[e][w]));
      sb();
    }
#pragma unroll
    for (int e = 0; e < E; ++e) put(16 + 4 * R4 + e, acc[16 + e]);
    sb();
  }
  // the 16x16 block: S = X + Y into f[0..7]
#pragma unroll
  for (int j = 0; j < 8; ++j) fxor(f[j], f[j + 8]);
  // rows 8..15 = C Y, C = A + B (leaves 3..5)
  fleaf4<PIN, W>(v4<W>(acc[12]), f + 12, tab01, tab2, 4);  // C_c Y_hi
#pragma unroll
  for (int r = 8; r < 12; ++r)
#pragma unroll
    for (int w = 0; w < W; ++w) acc[r][w] = acc[r + 4][w];
#pragma unroll
  for (int j = 8; j < 12; ++j) fxor(f[j], f[j + 4]);  // Y_lo + Y_hi
  fleaf4<PIN, W>(v4<W>(acc[8]), f + 8, tab01, tab2, 3);   // C_a
  fleaf4<PIN, W>(v4<W>(acc[12]), f + 8, tab01, tab2, 5);  // C_b
#pragma unroll
  for (int r = 0; r < 8; ++r)
#pragma unroll
    for (int w = 0; w < W; ++w) acc[r][w] = acc[r + 8][w];
  {
    uint32_t tmp[4][W];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int w = 0; w < W; ++w) tmp[r][w] = 0u;
    fleaf4<PIN, W>(tmp, f + 4, tab01, tab2, 1);  // A_c S_hi
    xor_into<W>(v4<W>(acc[0]), tmp);
    xor_into<W>(v4<W>(acc[4]), tmp);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int w = 0; w < W; ++w) tmp[r][w] = 0u;
    fleaf4<PIN, W>(tmp, f + 4, tab01, tab2, 7);  // B_c S_hi
    xor_into<W>(v4<W>(acc[8]), tmp);
    xor_into<W>(v4<W>(acc[12]), tmp);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) fxor(f[j], f[j + 4]);  // S_lo + S_hi
  fleaf4<PIN, W>(v4<W>(acc[0]), f + 0, tab01, tab2, 0);   // A_a
  fleaf4<PIN, W>(v4<W>(acc[4]), f + 0, tab01, tab2, 2);   // A_b
  fleaf4<PIN, W>(v4<W>(acc[8]), f + 0, tab01, tab2, 6);   // B_a
  fleaf4<PIN, W>(v4<W>(acc[12]), f + 0, tab01, tab2, 8);  // B_b
#pragma unroll
  for (int r = 0; r < 16; ++r) put(r, acc[r]);
}

// Field-form repair_dy16 (gf_dyadic16.hpp) over input slots in data-row order: slot i holds data row
// i when it is present, else one of the ND parity rows the decode reads; src[j] (j < ND) is the data
// row of missing row j; the decode rows' coefficients are in slot order.  TPW tiles per workgroup
// (one after the other), so the product tables built per workgroup serve TPW * 256 * 4W bytes of
// every row.
template <int ND, int E, bool PIN = true, int W = 1, int TPW = 2>
__device__ __forceinline__ void repair_dy16f(const GfArgs& a) {
  constexpr int K = 16, NDY = kDy16Leaves + 36 + K * E, NT = NDY + K * (ND > 0 ? ND : 1), MO = ND + 20 + E;
  constexpr uint32_t kLane = 4 * W;
  __shared__ u32x4 tab01[NT];
  __shared__ uint32_t tab2[NT];
  build_dy16_tables<1, E>(a.coef, tab01, tab2);
  for (int i = threadIdx.x; i < K * ND; i += (int)blockDim.x)  // slot NDY + c * ND + j: decode row j, slot c
    coef_tables(a.coef[(20 + E + i % ND) * K + i / ND], tab01[NDY + i], tab2[NDY + i]);
  __syncthreads();

  if (a.zw && blockIdx.x == 0 && blockIdx.y == 0)  // the batch's checksum words (gf_device.hpp GfArgs)
    for (uint32_t i = threadIdx.x; i < a.nzw; i += blockDim.x) a.zw[i] = 0u;
  const uint32_t stripe = blockIdx.y;
  const size_t ts = a.sstride ? 0 : (size_t)stripe;
  const int64_t sbase = (int64_t)stripe * a.sstride;
  const uint64_t slen = stripe_len(a, stripe);
  const uint8_t* const* in = a.ptr + ts * K;
  uint8_t* const* out = const_cast<uint8_t* const*>(a.ptr + (size_t)a.tab * K + ts * MO);
  const uint32_t pstore = a.pstore, pcmp = a.pcmp;
  uint32_t diff = 0;
  for (int tt = 0; tt < TPW; ++tt) {
    const uint32_t off = (blockIdx.x * TPW + tt) * (256u * kLane) + (uint32_t)threadIdx.x * kLane;
    const bool full = (uint64_t)off + kLane <= slen;
    const size_t rem = off < slen ? (size_t)(slen - off) : 0;
    if (!(full || rem)) break;
    const auto sb = [&]() {
      if constexpr (PIN) __builtin_amdgcn_sched_barrier(0);
    };
    Fld<W> f[K];
    {
      uint32_t x[K][W];
#pragma unroll
      for (int c = 0; c < K; ++c) ld_lane<W>(in[c] + sbase + off, full, rem, x[c]);
#pragma unroll
      for (int c = 0; c < K; ++c) to_fields<W>(x[c], f[c]);
    }
    sb();
    if constexpr (ND > 0) {
      uint32_t rec[ND][W];
#pragma unroll
      for (int j = 0; j < ND; ++j)
#pragma unroll
        for (int w = 0; w < W; ++w) rec[j][w] = 0u;
#pragma unroll
      for (int c = 0; c < K; c += 2) {
        fmac_pair<ND, W>(rec, f[c], f[c + 1], tab01 + NDY + c * ND, tab2 + NDY + c * ND, tab01 + NDY + (c + 1) * ND,
                         tab2 + NDY + (c + 1) * ND);
        if constexpr (PIN)
#pragma unroll
          for (int j = 0; j < ND; ++j)
#pragma unroll
            for (int w = 0; w < W; ++w) asm volatile("" : "+v"(rec[j][w]));
        sb();
      }
#pragma unroll
      for (int j = 0; j < ND; ++j) st_lane<W>(out[j] + sbase + off, full, rem, rec[j]);
      // missing data row j replaces the parity input in its slot: one uniform branch per row (the
      // asm keeps it a branch -- as a select it costs 3W v_cndmask per slot)
#pragma unroll
      for (int j = 0; j < ND; ++j) {
        Fld<W> rf;
        to_fields<W>(rec[j], rf);
        const uint32_t m = a.src[j];
#pragma unroll
        for (int i = 0; i < K; ++i) {
          if (m == (uint32_t)i) {
            asm volatile("" ::: "memory");
            f[i] = rf;
          }
        }
      }
      sb();
    }
    const uint8_t* spare = in[0] + sbase + off;  // just read: what rows not compared load instead
    fdy16_rows<1, E, PIN, W>(f, tab01, tab2, [&](int r, const uint32_t (&v)[W]) {
      const bool cmp = (pcmp >> r) & 1u;
      const uint8_t* p = cmp ? (const uint8_t*)out[ND + r] + sbase + off : spare;
      uint32_t y[W];
      ld_lane<W>(p, full, rem, y);
      const uint32_t msk = cmp ? ~0u : 0u;
#pragma unroll
      for (int w = 0; w < W; ++w) diff |= (y[w] ^ v[w]) & msk;
      if ((pstore >> r) & 1u) st_lane<W>(out[ND + r] + sbase + off, full, rem, v);
    });
  }
  if (diff) dev::set_flag(a.flags, stripe);
}

// Field-form matvec_dy16 (EC16P20 encode, the EC16P20L2 fused encode) with TPW tiles per workgroup.
template <int M, int R4, int E, MatVecMode MODE, bool PIN = true, int W = 1, int TPW = 2>
__device__ __forceinline__ void matvec_dy16f(const GfArgs& a) {
  constexpr int K = 16, N4 = R4 * 4 * 9;
  constexpr uint32_t kLane = 4 * W;
  static_assert(M == 16 + 4 * R4 + E, "dyadic-16 shape");
  constexpr bool kVer = MODE == MatVecMode::kVerify;
  __shared__ u32x4 tab01[kDy16Leaves + N4 + K * E];
  __shared__ uint32_t tab2[kDy16Leaves + N4 + K * E];
  build_dy16_tables<R4, E>(a.coef, tab01, tab2);
  __syncthreads();

  const uint32_t stripe = blockIdx.y;
  const size_t ts = a.sstride ? 0 : (size_t)stripe;
  const int64_t sbase = (int64_t)stripe * a.sstride;
  const uint64_t slen = stripe_len(a, stripe);
  const uint8_t* row[K + M];
#pragma unroll
  for (int c = 0; c < K; ++c) row[c] = a.ptr[ts * K + c] + sbase;
#pragma unroll
  for (int r = 0; r < M; ++r) row[K + r] = a.ptr[(size_t)a.tab * K + ts * M + r] + sbase;
  __builtin_amdgcn_sched_barrier(0);
  uint32_t diff = 0;
  for (int tt = 0; tt < TPW; ++tt) {
    const uint32_t off = (blockIdx.x * TPW + tt) * (256u * kLane) + (uint32_t)threadIdx.x * kLane;
    const bool full = (uint64_t)off + kLane <= slen;
    const size_t rem = off < slen ? (size_t)(slen - off) : 0;
    if (!(full || rem)) break;
    Fld<W> f[K];
    {
      uint32_t x[K][W];
#pragma unroll
      for (int c = 0; c < K; ++c) ld_lane<W>(row[c] + off, full, rem, x[c]);
#pragma unroll
      for (int c = 0; c < K; ++c) to_fields<W>(x[c], f[c]);
    }
    fdy16_rows<R4, E, PIN, W>(f, tab01, tab2, [&](int r, const uint32_t (&v)[W]) {
      uint8_t* p = const_cast<uint8_t*>(row[K + r]) + off;
      if constexpr (kVer) {
        uint32_t y[W];
        ld_lane<W>(p, full, rem, y);
#pragma unroll
        for (int w = 0; w < W; ++w) diff |= y[w] ^ v[w];
      } else {
        st_lane<W>(p, full, rem, v);
      }
    });
  }
  if constexpr (kVer) {
    if (diff) dev::set_flag(a.flags, stripe);
  }
}

}  // namespace dev
}  // namespace cfsec
