// gf_dyadic.hpp -- GF(2^8) matrix x shard-vector products for matrices made of dyadic blocks.
//
// The parity rows of the Vandermonde-derived systematic matrix of klauspost/reedsolomon
// (KRS/reedsolomon.go:220-244, evaluation points 0..n-1) have block structure: M[r][c] =
// L(p_r) / ((p_r + p_c) L'(p_c)) is a scaled Cauchy form, and where the points of a block of B
// rows and B columns are cosets of {0..B-1} (an additive subgroup of GF(2^8)) the scale is
// constant on the block and 1/(p_r + p_c) depends on r ^ c only:  M[r0+i][c0+j] = h[i ^ j].
// EC12P4, EC16P4 and EC16P20 parity are made of 4x4 dyadic blocks, EC6P6 / EC6P10 / EC10P4 of
// 2x2 ones, and so are the decode matrices of coset-aligned erasures (EC12P4's worst case
// {0,1,2,3} included).  A dyadic block needs fewer products:
//   [a b; b a] [x; y] = [a(x+y) + (a+b)y ; b(x+y) + (a+b)y]            3 products instead of 4
//   [A B; B A] [X; Y] = [A(X+Y) + (A+B)Y ; B(X+Y) + (A+B)Y]            on 2x2 blocks: 9 instead of 16
// GF(2^8) arithmetic is exact, so the bytes are those of the plain product; the launcher checks
// the structure on the actual coefficient matrix and takes these kernels only when it holds.
//
// Per 4x4 block and dword: multiplicands u = x0^x1^x2^x3, s = x1^x3, v = x2^x3, x3 (their
// v_perm selectors cost what 4 input rows cost), then 27 v_perm_b32 + 19 three-input XORs for 4
// outputs, against 48 + 24 for the plain tile (gf_device.hpp lane_tile_k).
#pragma once
#include "gf_device.hpp"

namespace cfsec {
namespace dev {

template <int B>
struct Dy;
template <>
struct Dy<2> {
  static constexpr int NC = 3;  // a, b, a^b
};
template <>
struct Dy<4> {
  static constexpr int NC = 9;  // h0, h1, h0^h1, h2, h3, h2^h3, g0=h0^h2, g1=h1^h3, g0^g1
};

template <int B>
__device__ __forceinline__ uint32_t dy_coef(const uint8_t* h, int q) {
  if constexpr (B == 2) {
    return q == 0 ? h[0] : q == 1 ? h[1] : (uint32_t)(h[0] ^ h[1]);
  } else {
    switch (q) {
      case 0: return h[0];
      case 1: return h[1];
      case 2: return h[0] ^ h[1];
      case 3: return h[2];
      case 4: return h[3];
      case 5: return h[2] ^ h[3];
      case 6: return h[0] ^ h[2];
      case 7: return h[1] ^ h[3];
      default: return h[0] ^ h[1] ^ h[2] ^ h[3];
    }
  }
}

// Product tables of every derived coefficient: slot (rb*KB + cb)*NC + q for row block rb, column
// block cb (coef: (MD + E) x K row-major, first row of each block read).  Row blocks MB .. MBP-1 pad
// the last wave's share with zero tables, so no wave indexes past the arrays.  The E plain rows
// after the MD dyadic ones follow at slot MBP*KB*NC + c*E + e.
template <int K, int MD, int B, int MBP, int E>
__device__ __forceinline__ void build_dy_tables(const uint8_t* coef, u32x4* tab01, uint32_t* tab2) {
  constexpr int KB = K / B, MB = MD / B, NC = Dy<B>::NC, ND = MBP * KB * NC;
  for (int i = threadIdx.x; i < ND + K * E; i += (int)blockDim.x) {
    uint32_t cf = 0;
    if (i < ND) {
      const int q = i % NC, blk = i / NC, cb = blk % KB, rb = blk / KB;
      cf = rb < MB ? dy_coef<B>(coef + (rb * B) * K + cb * B, q) : 0u;
    } else if constexpr (E > 0) {
      const int c = (i - ND) / E, e = (i - ND) % E;
      cf = coef[(MD + e) * K + c];
    }
    coef_tables(cf, tab01[i], tab2[i]);
  }
}

// v_perm selectors of W dwords per lane (W = 4: 16 bytes, the shipped width; W = 2: 8 bytes)
template <int W = 4>
struct SelW {
  uint32_t s0[W], s1[W], s2[W];
};
using Sel = SelW<4>;

template <int W>
__device__ __forceinline__ void selectors(const uint32_t (&x)[W], SelW<W>& s) {
#pragma unroll
  for (int w = 0; w < W; ++w) {
    s.s0[w] = x[w] & 0x07070707u;
    s.s1[w] = (x[w] >> 3) & 0x07070707u;
    s.s2[w] = (x[w] >> 6) & 0x03030303u;
  }
}

// The three partial lookups of coefficient q times the multiplicand whose selectors are s.
template <int W = 4>
struct ProdW {
  uint32_t a[W], b[W], c[W];
};
using Prod = ProdW<4>;

template <int W>
__device__ __forceinline__ void lookups(const u32x4 q, uint32_t t2, const SelW<W>& s, ProdW<W>& p) {
#pragma unroll
  for (int w = 0; w < W; ++w) {
    p.a[w] = __builtin_amdgcn_perm(q.y, q.x, s.s0[w]);
    p.b[w] = __builtin_amdgcn_perm(q.w, q.z, s.s1[w]);
    p.c[w] = __builtin_amdgcn_perm(0u, t2, s.s2[w]);
  }
}

__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// B = 2, all row blocks of one column block: tq/t2p point at (rb=0, cb) slot 0; row blocks are
// kb*NC slots apart.
template <int MB, bool PIN = true>
__device__ __forceinline__ void dy_col2(uint32_t (&acc)[2 * MB][4], const uint32_t (&x0)[4],
                                        const uint32_t (&x1)[4], const u32x4* tq, const uint32_t* t2p,
                                        int stride) {
  uint32_t u[4];
#pragma unroll
  for (int w = 0; w < 4; ++w) u[w] = x0[w] ^ x1[w];
  Sel su, sy;
  selectors(u, su);
  selectors(x1, sy);
#pragma unroll
  for (int rb = 0; rb < MB; ++rb) {
    const u32x4* q = tq + rb * stride;
    const uint32_t* t = t2p + rb * stride;
    Prod pa, pb, pc;
    lookups(q[0], t[0], su, pa);
    lookups(q[1], t[1], su, pb);
    lookups(q[2], t[2], sy, pc);
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const uint32_t c = x3(pc.a[w], pc.b[w], pc.c[w]);
      acc[2 * rb][w] = x3(x3(acc[2 * rb][w], pa.a[w], pa.b[w]), pa.c[w], c);
      acc[2 * rb + 1][w] = x3(x3(acc[2 * rb + 1][w], pb.a[w], pb.b[w]), pb.c[w], c);
    }
  }
}

// B = 4, all row blocks of one column block.
template <int MB, bool PIN = true, int W = 4>
__device__ __forceinline__ void dy_col4(uint32_t (&acc)[4 * MB][W], const uint32_t (&x0)[W],
                                        const uint32_t (&x1)[W], const uint32_t (&x2)[W],
                                        const uint32_t (&x3v)[W], const u32x4* tq, const uint32_t* t2p,
                                        int stride) {
  uint32_t u[W], s[W], v[W];
#pragma unroll
  for (int w = 0; w < W; ++w) {
    s[w] = x1[w] ^ x3v[w];
    v[w] = x2[w] ^ x3v[w];
    u[w] = x3(x0[w], x2[w], s[w]);  // x0^x1^x2^x3
  }
  SelW<W> su, ss, sv, sy;
#pragma unroll
  for (int rb = 0; rb < MB; ++rb) {
    const u32x4* q = tq + rb * stride;
    const uint32_t* t = t2p + rb * stride;
    uint32_t ps[W], ps2[W], c0[W], c1[W];
    {
      ProdW<W> p;
      selectors(s, ss);
      lookups(q[2], t[2], ss, p);  // (h0^h1) s
#pragma unroll
      for (int w = 0; w < W; ++w) ps[w] = x3(p.a[w], p.b[w], p.c[w]);
      lookups(q[5], t[5], ss, p);  // (h2^h3) s
#pragma unroll
      for (int w = 0; w < W; ++w) ps2[w] = x3(p.a[w], p.b[w], p.c[w]);
      if constexpr (PIN) {
#pragma unroll
        for (int w = 0; w < W; ++w) asm volatile("" : "+v"(ps[w]), "+v"(ps2[w]));
        __builtin_amdgcn_sched_barrier(0);
      }
      ProdW<W> py, p6, p7;
      selectors(x3v, sy);
      selectors(v, sv);
      lookups(q[8], t[8], sy, py);  // (g0^g1) x3
      lookups(q[6], t[6], sv, p6);  // g0 v
      lookups(q[7], t[7], sv, p7);  // g1 v
#pragma unroll
      for (int w = 0; w < W; ++w) {
        const uint32_t qy = x3(py.a[w], py.b[w], py.c[w]);
        c0[w] = x3(p6.a[w], p6.b[w], p6.c[w]) ^ qy;
        c1[w] = x3(p7.a[w], p7.b[w], p7.c[w]) ^ qy;
      }
    }
    if constexpr (PIN) {
#pragma unroll
      for (int w = 0; w < W; ++w) asm volatile("" : "+v"(c0[w]), "+v"(c1[w]));
      __builtin_amdgcn_sched_barrier(0);
    }
    selectors(u, su);
    // one output at a time: out_j ^= h_j u ^ (shared s term) ^ (shared x3/v term)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      ProdW<W> p;
      const int qi = j < 2 ? j : j + 1;  // h0, h1, h2, h3 live at slots 0, 1, 3, 4
      lookups(q[qi], t[qi], su, p);
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

// Waves per column chunk (OS) and column chunks per workgroup (CW) of the dyadic kernels: each
// wave owns RBW row blocks.  The shipped kernels keep all row blocks in one wave (RBW = MB, OS = 1):
// splitting them over waves re-reads every input once per wave and lost 25 % on EC16P20 even
// though one wave holding 20 accumulators runs at 1-2 waves per SIMD (tools/gf_dy_probe.hip).
template <int M, int B, int RBW_ = 64>
struct DyShape {
  static constexpr int MB = M / B;
  static constexpr int RBW = RBW_ < MB ? RBW_ : MB;
  static constexpr int OS = (MB + RBW - 1) / RBW;
  static constexpr int CW = OS >= 4 ? 1 : 4 / OS;
  static constexpr int kThreadsPerWg = 64 * OS * CW;
  static constexpr int kTileBytes = 64 * kLaneBytes * CW;
};

// Kernel body: compile-time K inputs, M outputs of which the first M - E are made of dyadic blocks
// of B and the last E are plain rows (the local parities of a fused LRC encode: EC16P20L2 is 20
// dyadic global rows + 2 local rows); grid (tiles, stripes), DyShape threads; wave w handles
// column chunk w / OS and row blocks (w % OS) * RBW .. +RBW (plain rows: single-wave shapes only),
// one 16-byte chunk per lane per row, column blocks loaded one block ahead.
template <int K, int M, int B, MatVecMode MODE, bool NTS = true, bool NTL = true, int RBW_ = 64, int E = 0,
          bool PIN = true, int SP = -1, int LP = -1>
__device__ __forceinline__ void matvec_dy(const GfArgs& a) {
  constexpr int MD = M - E;
  static_assert(K % B == 0 && MD % B == 0 && (B == 2 || B == 4), "dyadic shape");
  using Sh = DyShape<MD, B, RBW_>;
  static_assert(E == 0 || Sh::OS == 1, "plain rows ride along single-wave shapes only");
  static_assert(MODE == MatVecMode::kStore || MODE == MatVecMode::kVerify, "the clamped row end: stores, compares");
  constexpr int KB = K / B, MB = MD / B, NC = Dy<B>::NC, RBW = Sh::RBW, MW = RBW * B;
  constexpr int MBP = Sh::OS * RBW;  // row blocks incl. the last wave's padding
  constexpr int ND = MBP * KB * NC;  // dyadic table slots; the plain rows' follow
  constexpr bool kVer = MODE == MatVecMode::kVerify;
  __shared__ u32x4 tab01[ND + K * E];
  __shared__ uint32_t tab2[ND + K * E];
  build_dy_tables<K, MD, B, MBP, E>(a.coef, tab01, tab2);
  __syncthreads();

  const int wave = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
  const int rb0 = (wave % Sh::OS) * RBW;  // first row block of this wave
  const int cw = wave / Sh::OS;
  if (rb0 >= MB) return;  // padding wave (no barrier follows)
  const int nrb = MB - rb0 < RBW ? MB - rb0 : RBW;
  const uint32_t stripe = blockIdx.y, tile = blockIdx.x;
  const size_t ts = a.sstride ? 0 : (size_t)stripe;
  const int64_t sbase = (int64_t)stripe * a.sstride;
  uint32_t off = tile * (uint32_t)Sh::kTileBytes + (uint32_t)(cw * 64 + lane) * kLaneBytes;
  const uint8_t* row[K + MW + E];
#pragma unroll
  for (int c = 0; c < K; ++c) row[c] = a.ptr[ts * K + c] + sbase;
#pragma unroll
  for (int r = 0; r < MW; ++r) {
    const int o = rb0 * B + (r < nrb * B ? r : 0);
    row[K + r] = a.ptr[(size_t)a.tab * K + ts * M + o] + sbase;
  }
#pragma unroll
  for (int e = 0; e < E; ++e) row[K + MW + e] = a.ptr[(size_t)a.tab * K + ts * M + MD + e] + sbase;
  __builtin_amdgcn_sched_barrier(0);

  constexpr int MA = MW + E;  // accumulators: dyadic rows, then plain rows
  uint32_t acc[MA][4];
#pragma unroll
  for (int r = 0; r < MA; ++r)
#pragma unroll
    for (int w = 0; w < 4; ++w) acc[r][w] = 0u;
  const auto pin = [&]() {
    if constexpr (PIN) {
#pragma unroll
      for (int r = 0; r < MA; ++r)
        asm volatile("" : "+v"(acc[r][0]), "+v"(acc[r][1]), "+v"(acc[r][2]), "+v"(acc[r][3]));
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  const auto sb = [&]() {
    if constexpr (PIN) __builtin_amdgcn_sched_barrier(0);
  };
  // The ragged end of a row: the lane holding it codes the row's last full 16-byte chunk instead (its
  // bytes before the end repeat its neighbour's, same values: stores and compares only), so in rows of
  // at least 16 bytes no lane takes the byte path -- whose dependent byte loads made each row's last
  // workgroup a straggler that ended the launch late (gf_lut.hpp).  One body, `off` moved.
  const uint64_t slen = stripe_len(a, stripe);
  const bool inrow = off < slen;
  if (inrow && slen >= kLaneBytes && (uint64_t)off + kLaneBytes > slen) off = (uint32_t)(slen - kLaneBytes);
  const bool full = (uint64_t)off + kLaneBytes <= slen;
  const size_t rem = inrow ? (size_t)(slen - off) : 0;
  uint32_t diff = 0;
  if (full || rem) {
    uint32_t x[K][4];
    const auto load = [&](int c) {
      u32x4 v;
      if constexpr (LP >= 0) v = full ? ld16_pol<LP>(row[c], off) : ld_tail(row[c] + off, rem);  // probes
      else v = full ? ld16<NTL>(row[c] + off) : ld_tail(row[c] + off, rem);
      x[c][0] = v.x;
      x[c][1] = v.y;
      x[c][2] = v.z;
      x[c][3] = v.w;
    };
#pragma unroll
    for (int c = 0; c < B; ++c) load(c);
    const u32x4* tq = tab01 + rb0 * KB * NC;
    const uint32_t* tt = tab2 + rb0 * KB * NC;
#pragma unroll
    for (int cb = 0; cb < KB; ++cb) {
      if (cb + 1 < KB)
#pragma unroll
        for (int c = 0; c < B; ++c) load((cb + 1) * B + c);
      sb();
      const int c0 = cb * B;
      auto& dacc = reinterpret_cast<uint32_t(&)[MW][4]>(acc);
      if constexpr (B == 2)
        dy_col2<RBW, PIN>(dacc, x[c0], x[c0 + 1], tq + cb * NC, tt + cb * NC, KB * NC);
      else
        dy_col4<RBW, PIN>(dacc, x[c0], x[c0 + 1], x[c0 + 2], x[c0 + 3], tq + cb * NC, tt + cb * NC, KB * NC);
      pin();
      if constexpr (E > 0) {
        auto& eacc = reinterpret_cast<uint32_t(&)[E][4]>(acc[MW]);
#pragma unroll
        for (int c = c0; c < c0 + B; c += 2) {
          mac_pair_k<E>(eacc, x[c], x[c + 1], tab01 + ND + c * E, tab2 + ND + c * E, tab01 + ND + (c + 1) * E,
                        tab2 + ND + (c + 1) * E);
          pin();
        }
      }
    }
#pragma unroll
    for (int r = 0; r < MA; ++r) {
      if (r < MW && r >= nrb * B) continue;
      uint8_t* p = const_cast<uint8_t*>(row[K + r]) + off;
      const u32x4 v = u32x4{acc[r][0], acc[r][1], acc[r][2], acc[r][3]};
      if constexpr (kVer) {
        const u32x4 d = v ^ (full ? ld16<true>(p) : ld_tail(p, rem));
        diff |= d.x | d.y | d.z | d.w;
      } else if (full) {
        if constexpr (SP >= 0) st16_pol<SP>(p, v);  // probe variants
        else st16_out<NTS>(p, v);
      } else {
        st_tail(p, v, rem);
      }
    }
  }
  if constexpr (kVer) {
    if (diff) dev::set_flag(a.flags, stripe);
  }
}

}  // namespace dev
}  // namespace cfsec
