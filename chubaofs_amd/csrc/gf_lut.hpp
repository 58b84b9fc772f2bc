// gf_lut.hpp -- GF(2^8) matrix x shard-vector product from LDS lookups (gfx950), for matrices with
// many outputs per input (EC15P12, EC12P9 and their repairs).
//
// The v_perm_b32 product (gf_device.hpp) costs 4.5 half-rate VALU per (coefficient, dword): ~1.1
// wave-instruction per output byte, so its cost grows with m and the wide shapes are VALU-issue-
// bound (EC15P12 at 40 % of the HBM roofline).  Here the products of one input byte
// with ALL m coefficients of its column come from two table reads: T_c[h][n] holds, as bytes r of
// its EW words, coef[r][c] * (n << 4h) for the two nibbles h of the byte.  A 16-entry table of EW
// words spans 16*EW banks; ds_read_b32 / b64 / b128 (EW = 1 / 2 / 4) serve lane groups of 32 / 32 / 16
// over 32 / 64 / 64 banks (MI355X_MICROARCH.md §LDS), so every read is conflict-free, and costs
// 2 / 2 / 4 LDS cycles for up to 4 / 8 / 16 outputs.  The products accumulate byte-transposed
// (acc[p][q] byte i = output 4q+i at byte p of the lane's 16-byte chunk) and are transposed back
// once per chunk (8 v_perm_b32 per 4 outputs x 16 bytes).  Per input byte: 2 reads + EW XOR3;
// the VALU no longer scales with 1.1 m, the LDS pipe takes the lookups.
//
// The tables depend only on the coefficients: built per workgroup from the argument block --
// 8 packed powers coef*2^i of each 4-output column group first, then every entry as an XOR of at
// most 4 of them.
#pragma once
#include <hip/hip_runtime.h>

#include "gf_device.hpp"
#include "kernels.hpp"

namespace cfsec {
namespace lut {

using dev::u32x4;

// Entry words for m outputs: 1 (m <= 4), 2 (m <= 8), 4 (m <= 16; a 12-byte entry would take
// ds_read_b96, 8 LDS cycles per read).
constexpr int entry_words(int m) { return m <= 4 ? 1 : (m <= 8 ? 2 : 4); }

// 4 packed GF(2^8) doublings (polynomial 0x11D, KRS/galois.go:25)
__device__ __forceinline__ uint32_t xtime4(uint32_t v) {
  return ((v << 1) & 0xFEFEFEFEu) ^ (((v >> 7) & 0x01010101u) * 0x1Du);
}

// T_c[h][n] word q (c < K, h < 2, n < 16, q < EW) at word index ((c*2 + h)*16 + n)*EW + q.
// (the first M rows of a coefficient matrix with row stride KS)
template <int K, int M, int KS>
__device__ __forceinline__ void build_lut(const uint8_t* coef, uint32_t* T, uint32_t* pw) {
  constexpr int EW = entry_words(M), NQ = (M + 3) / 4;
  // pw[(c*NQ + q)*8 + i] = bytes b of coef[4q+b][c] * 2^i (rows past M: 0)
  for (int t = threadIdx.x; t < K * NQ; t += (int)blockDim.x) {
    const int c = t / NQ, q = t - (t / NQ) * NQ;
    uint32_t v = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b)
      if (4 * q + b < M) v |= (uint32_t)coef[(4 * q + b) * KS + c] << (8 * b);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      pw[t * 8 + i] = v;
      v = xtime4(v);
    }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < K * 2 * 16 * EW; t += (int)blockDim.x) {
    const int q = t % EW, n = (t / EW) & 15, h = (t / (16 * EW)) & 1, c = t / (32 * EW);
    uint32_t v = 0;
    if (q < NQ) {
      const uint32_t* p = pw + (c * NQ + q) * 8 + 4 * h;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if ((n >> i) & 1) v ^= p[i];
    }
    T[t] = v;
  }
}

template <int EW>
struct Entry {
  uint32_t w[EW];
};

// One table read: EW words at byte offset `off` (a multiple of 4*EW) of T.
template <int EW>
__device__ __forceinline__ Entry<EW> ld_entry(const char* T, uint32_t off) {
  Entry<EW> e;
  if constexpr (EW == 1) {
    e.w[0] = *reinterpret_cast<const uint32_t*>(T + off);
  } else if constexpr (EW == 2) {
    const dev::u32x2 v = *reinterpret_cast<const dev::u32x2*>(T + off);
    e.w[0] = v.x;
    e.w[1] = v.y;
  } else {
    const u32x4 v = *reinterpret_cast<const u32x4*>(T + off);
    e.w[0] = v.x;
    e.w[1] = v.y;
    e.w[2] = v.z;
    e.w[3] = v.w;
  }
  return e;
}

// o[i][w] byte b = byte i of g[4w + b]: 4 outputs x 4 LW bytes from the byte-transposed words.
template <int LW = 4>
__device__ __forceinline__ void untranspose4(const uint32_t (&g)[4 * LW], uint32_t (&o)[4][LW]) {
#pragma unroll
  for (int w = 0; w < LW; ++w) {
    const uint32_t a = g[4 * w], b = g[4 * w + 1], c = g[4 * w + 2], d = g[4 * w + 3];
    const uint32_t ab_lo = __builtin_amdgcn_perm(b, a, 0x05010400u), cd_lo = __builtin_amdgcn_perm(d, c, 0x05010400u);
    const uint32_t ab_hi = __builtin_amdgcn_perm(b, a, 0x07030602u), cd_hi = __builtin_amdgcn_perm(d, c, 0x07030602u);
    o[0][w] = __builtin_amdgcn_perm(cd_lo, ab_lo, 0x05040100u);
    o[1][w] = __builtin_amdgcn_perm(cd_lo, ab_lo, 0x07060302u);
    o[2][w] = __builtin_amdgcn_perm(cd_hi, ab_hi, 0x05040100u);
    o[3][w] = __builtin_amdgcn_perm(cd_hi, ab_hi, 0x07060302u);
  }
}

#ifndef CFSEC_LUT_LOOKAHEAD
#define CFSEC_LUT_LOOKAHEAD 2
#endif
// Verify: the compared rows' loads issued right after the last input row's (overlapping the last
// D + 1 columns' lookups) instead of after the product, where the held words fit: EC16P20's 8-row
// repair verify 77 -> 69 us, EC15P12 verify 72 -> 66 us; at 32-36 held words (EC16P20 16 rows,
// EC12P9) the occupancy halves and Verify slows 1.4-2.4x, and K = 16, M = 12 takes 106 VGPRs
// (profiles/r05/lut_verify_early_loads.txt).  0 = off (A/B).
#ifndef CFSEC_LUT_VPRE
#define CFSEC_LUT_VPRE 1
#endif
#ifndef CFSEC_LUT_VPRE_MAXW
#define CFSEC_LUT_VPRE_MAXW 24  // compared words per lane held early, at most
#endif

// One 16-byte chunk of every row at byte `off` of the stripe (all in bounds, or the tail chunk with
// rem < 16 valid bytes).  Outputs [0, ML) come from the lookups, [ML, M) from the v_perm product
// (tab01 / tab2 of gf_device.hpp, slot c * MP + r), which keeps both the LDS pipe and the VALU busy:
// per input byte the lookups cost the LDS 2 reads of ~3.2 effective cycles (b64, measured:
// tools/lds_rate.hip) and the VALU ~13 cycles for 8 outputs, the v_perm product ~4.7 VALU cycles
// per output.  MODE: kStore (outputs written), kVerify (compared: diff), kStoreVerify (rows < nstore
// written, the rest compared).
// FULL: the caller guarantees a whole chunk (rem == 4 * LW), so the tail paths are not compiled in.
template <int K, int M, int ML, MatVecMode MODE, int LA = CFSEC_LUT_LOOKAHEAD, int LW = 4, bool FULL = false>
__device__ __forceinline__ void lut_chunk(const char* T, const u32x4* tab01, const uint32_t* tab2,
                                          const uint8_t* const* in, uint8_t* const* out, int nstore, int64_t sbase,
                                          uint32_t off, uint32_t rem, uint32_t& diff) {
  constexpr int EW = entry_words(ML), NQ = (ML + 3) / 4, EB = 4 * EW, MP = M - ML;
  constexpr int D = LA < K ? LA : K;
  constexpr int SHIFT = EW == 1 ? 2 : (EW == 2 ? 3 : 4);  // log2 of the entry bytes
  constexpr int NP = 4 * LW;                              // bytes per lane chunk
  const bool full = FULL || rem >= (uint32_t)NP;
  uint32_t acc[NP][NQ > 0 ? NQ : 1];
  uint32_t accp[MP > 0 ? MP : 1][LW];
#pragma unroll
  for (int p = 0; p < NP; ++p)
#pragma unroll
    for (int q = 0; q < NQ; ++q) acc[p][q] = 0u;
#pragma unroll
  for (int r = 0; r < MP; ++r)
#pragma unroll
    for (int w = 0; w < LW; ++w) accp[r][w] = 0u;
  uint32_t x[K][LW];
  constexpr bool kPre = CFSEC_LUT_VPRE && MODE == MatVecMode::kVerify && M * LW <= CFSEC_LUT_VPRE_MAXW &&
                          K * M <= 180;
  uint32_t y[kPre ? M : 1][LW];
  const auto load = [&](int c) {
    if (full) {
      dev::ld_chunk<LW, true>(in[c] + sbase + off, x[c]);
    } else {
      const u32x4 v = dev::ld_tail(in[c] + sbase + off, rem);
      const uint32_t t[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int w = 0; w < LW; ++w) x[c][w] = t[w];
    }
  };
#pragma unroll
  for (int c = 0; c < D; ++c) load(c);
#pragma unroll
  for (int c = 0; c < K; ++c) {
    if (c + D < K) load(c + D);
    if constexpr (kPre) {
      if (c == K - D - 1 || (D >= K && c == 0)) {
#pragma unroll
        for (int r = 0; r < M; ++r) {
          const uint8_t* p = out[r] + sbase + off;
          if (full) {
            dev::ld_chunk<LW, true>(p, y[r]);
          } else {
            const u32x4 v = dev::ld_tail(p, rem);
            const uint32_t t[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int w = 0; w < LW; ++w) y[r][w] = t[w];
          }
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (NQ > 0) {
      const char* tc = T + c * 2 * 16 * EB;
#pragma unroll
      for (int w = 0; w < LW; ++w) {
        // byte j of lo / hi = EB x (low / high nibble of byte j): the entry's byte offset
        uint32_t lo, hi;
        if constexpr (SHIFT == 4) {
          lo = (x[c][w] << 4) & 0xF0F0F0F0u;
          hi = x[c][w] & 0xF0F0F0F0u;
        } else {
          lo = (x[c][w] << SHIFT) & (0x0F0F0F0Fu << SHIFT);
          hi = (x[c][w] >> (4 - SHIFT)) & (0x0F0F0F0Fu << SHIFT);
        }
        asm volatile("" : "+v"(lo), "+v"(hi));
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const Entry<EW> el = ld_entry<EW>(tc, (lo >> (8 * j)) & 0xFFu);
          const Entry<EW> eh = ld_entry<EW>(tc + 16 * EB, (hi >> (8 * j)) & 0xFFu);
#pragma unroll
          for (int q = 0; q < NQ; ++q)
            acc[4 * w + j][q] = __builtin_amdgcn_bitop3_b32(acc[4 * w + j][q], el.w[q], eh.w[q], 0x96);
        }
      }
#pragma unroll
      for (int p = 0; p < NP; ++p)
#pragma unroll
        for (int q = 0; q < NQ; ++q) asm volatile("" : "+v"(acc[p][q]));
    }
    if constexpr (MP > 0) {
      dev::mac_row_k<MP, LW>(accp, x[c], tab01 + c * MP, tab2 + c * MP);
#pragma unroll
      for (int r = 0; r < MP; ++r)
#pragma unroll
        for (int w = 0; w < LW; ++w) asm volatile("" : "+v"(accp[r][w]));
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  constexpr bool kVer = MODE == MatVecMode::kVerify, kMix = MODE == MatVecMode::kStoreVerify;
  const auto finish = [&](int r, const uint32_t (&o)[LW]) {
    uint8_t* p = out[r] + sbase + off;
    const bool cmp = kVer || (kMix && r >= nstore);
    if constexpr (kPre) {
      uint32_t d = 0;
#pragma unroll
      for (int w = 0; w < LW; ++w) d |= o[w] ^ y[r][w];
      diff |= d;  // (the tail's bytes past rem: zeros in both)
      return;
    }
    if (full) {
      if (cmp) {
        uint32_t y[LW];
        dev::ld_chunk<LW, true>(p, y);
#pragma unroll
        for (int w = 0; w < LW; ++w) diff |= o[w] ^ y[w];
      } else {
        dev::st_chunk<LW, true>(p, o);
      }
    } else {
      uint32_t t[4] = {0u, 0u, 0u, 0u};
#pragma unroll
      for (int w = 0; w < LW; ++w) t[w] = o[w];
      const u32x4 v{t[0], t[1], t[2], t[3]};
      if (cmp) {
        const u32x4 d = v ^ dev::ld_tail(p, rem);
        diff |= d.x | d.y | d.z | d.w;
      } else {
        dev::st_tail(p, v, rem);
      }
    }
  };
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    uint32_t g[NP];
#pragma unroll
    for (int p = 0; p < NP; ++p) g[p] = acc[p][q];
    uint32_t o[4][LW];
    untranspose4<LW>(g, o);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (4 * q + i < ML) finish(4 * q + i, o[i]);
  }
#pragma unroll
  for (int r = 0; r < MP; ++r) finish(ML + r, accp[r]);
}

// Grid (tiles, stripes), 256 threads, one tile (256 lanes x 4 LW bytes) of every row per workgroup (GfArgs as the
// fixed-K kernel: a.k == K, a.m == M, a.len < 4 GiB).
template <int K, int M, int ML, MatVecMode MODE, int LA = CFSEC_LUT_LOOKAHEAD, int LW = 4>
__global__ __launch_bounds__(256) void gf_lut_kernel(const dev::GfArgs a) {
  constexpr int EW = entry_words(ML), NQ = (ML + 3) / 4, MP = M - ML;
  __shared__ __attribute__((aligned(16))) uint32_t T[NQ > 0 ? K * 2 * 16 * EW : 4];
  __shared__ uint32_t pw[NQ > 0 ? K * NQ * 8 : 1];
  __shared__ u32x4 tab01[MP > 0 ? K * MP : 1];
  __shared__ uint32_t tab2[MP > 0 ? K * MP : 1];
  if constexpr (MP > 0) {
    for (int i = threadIdx.x; i < K * MP; i += 256) {
      const int c = i / MP, r = i - (i / MP) * MP;
      dev::coef_tables(a.coef[(ML + r) * K + c], tab01[i], tab2[i]);
    }
  }
  if constexpr (NQ > 0) build_lut<K, ML, K>(a.coef, T, pw);
  __syncthreads();
  const uint32_t stripe = blockIdx.y, tile = blockIdx.x;
  const size_t ts = a.sstride ? 0 : (size_t)stripe;
  const int64_t sbase = (int64_t)stripe * a.sstride;
  const uint8_t* const* in = a.ptr + ts * K;
  uint8_t* const* out = const_cast<uint8_t* const*>(a.ptr + (size_t)a.tab * K + ts * M);
  constexpr uint32_t kLB = 4u * LW;  // bytes per lane chunk
  const uint32_t off = tile * (256u * kLB) + threadIdx.x * kLB;
  const uint64_t len = dev::stripe_len(a, stripe);
  uint32_t diff = 0;
  // The ragged end of a row: the lane holding it codes the row's last full chunk instead (its bytes
  // before the end repeat its neighbour's, same values: stores and compares only), so in rows of at
  // least one chunk no lane takes the byte path.  That path -- 16 dependent byte loads per input row
  // -- made the row's last workgroup a straggler, and the last stripe's last one ended the launch
  // ~10 us late: EC15P12 encode 75.6 -> 65.8 us, EC12P9 56.6 -> 46.6 (tools/gf_shapes.hip,
  // profiles/r05/shape_sweep_lut_clamp.txt).  Whole chunks take a byte-path-free instantiation of the
  // body (FULL: no tail loads or stores compiled in, fewer registers): EC16P20's 16-row repair verify
  // 128 -> 101 us, EC12P9 encode 46.5 -> 44.0, EC15P12 66.3 -> 63.4, EC16P20's 8-row repair 73.3 ->
  // 70.8 (profiles/r06/shape_sweep_store_variants.txt).  Round 5 measured this form returning wrong
  // rows -- the inline-asm store hazard of gf_device.hpp st16_pol, since removed.
  static_assert(MODE != MatVecMode::kAccum, "the clamped row end re-codes bytes: stores and compares only");
  if ((uint64_t)off < len) {
    const uint32_t loff = len >= kLB && (uint64_t)off + kLB > len ? (uint32_t)(len - kLB) : off;
    const uint32_t rem = (uint64_t)loff + kLB <= len ? kLB : (uint32_t)(len - loff);
    const char* t = reinterpret_cast<const char*>(T);
    if (rem == kLB)
      lut_chunk<K, M, ML, MODE, LA, LW, true>(t, tab01, tab2, in, out, (int)a.nstore, sbase, loff, rem, diff);
    else
      lut_chunk<K, M, ML, MODE, LA, LW, false>(t, tab01, tab2, in, out, (int)a.nstore, sbase, loff, rem, diff);
  }
  if constexpr (MODE == MatVecMode::kVerify || MODE == MatVecMode::kStoreVerify) {
    if (diff) dev::set_flag(a.flags, stripe);
  }
}

}  // namespace lut
}  // namespace cfsec
