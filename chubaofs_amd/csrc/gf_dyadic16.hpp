// gf_dyadic16.hpp -- GF(2^8) products for 16-input matrices whose first 16 rows form one 16x16
// dyadic block: the EC16P20 parity (KRS buildMatrix(16, 36) rows 16..31 over data 0..15; parity
// points 16..31 are the coset 16 + {0..15} of the additive subgroup {0..15}, see gf_dyadic.hpp),
// followed by 4x4-dyadic row blocks (rows 32..35) and, for the fused EC16P20L2 encode, 2 plain
// local rows.
//
// A dyadic block M[i][j] = h[i ^ j] of size 2n is [[A, B], [B, A]] with A, B dyadic of size n, and
//   [A B; B A] [X; Y] = [A S + C Y ; B S + C Y],   S = X + Y,  C = A + B
// so a 16x16 block costs 3 products of 8x8 blocks, each 3 products of 4x4 blocks: 9 leaf 4x4
// products of 9 GF multiplies (dy_col4) = 81 multiplies for 256 coefficients, against 16 x 9 = 144
// when the block is cut into 4x4 dyadic blocks.  The leaves' first rows are XOR combinations of h
// (dy16_coef); the arithmetic is exact, so the bytes equal the plain product.
#pragma once
#include "gf_dyadic.hpp"

namespace cfsec {
namespace dev {

// Leaf l = 3 * l1 + l2 of the 16x16 block with first row h[0..15]: l1 picks the 8x8 block
// (0: A = h[0..7], 1: C = A + B, 2: B = h[8..15]), l2 the 4x4 block of that (0: its first half,
// 1: the sum of its halves, 2: its second half); returns derived coefficient q of the leaf.
__device__ __forceinline__ uint32_t dy16_coef(const uint8_t* h, int leaf, int q) {
  const int l1 = leaf / 3, l2 = leaf % 3;
  uint8_t x8[8], g[4];
#pragma unroll
  for (int j = 0; j < 8; ++j) x8[j] = l1 == 0 ? h[j] : l1 == 1 ? (uint8_t)(h[j] ^ h[j + 8]) : h[j + 8];
#pragma unroll
  for (int j = 0; j < 4; ++j) g[j] = l2 == 0 ? x8[j] : l2 == 1 ? (uint8_t)(x8[j] ^ x8[j + 4]) : x8[j + 4];
  return dy_coef<4>(g, q);
}

constexpr int kDy16Leaves = 81;  // 9 leaves x 9 derived coefficients

// Table slots: [0, 81) the leaves; then R4 row blocks x 4 column blocks x 9 of the 4x4 rows; then
// K * E plain-row coefficients (slot c * E + e).
template <int R4, int E>
__device__ __forceinline__ void build_dy16_tables(const uint8_t* coef, u32x4* tab01, uint32_t* tab2) {
  constexpr int K = 16, N4 = R4 * 4 * 9;
  for (int i = threadIdx.x; i < kDy16Leaves + N4 + K * E; i += (int)blockDim.x) {
    uint32_t cf = 0;
    if (i < kDy16Leaves) {
      cf = dy16_coef(coef, i / 9, i % 9);
    } else if (i < kDy16Leaves + N4) {
      const int j = i - kDy16Leaves, q = j % 9, blk = j / 9, cb = blk % 4, rb = blk / 4;
      cf = dy_coef<4>(coef + (16 + 4 * rb) * K + 4 * cb, q);
    } else if constexpr (E > 0) {
      const int j = i - kDy16Leaves - N4, c = j / E, e = j % E;
      cf = coef[(16 + 4 * R4 + e) * K + c];
    }
    coef_tables(cf, tab01[i], tab2[i]);
  }
}

// Lane chunks of W dwords (W = 4: 16 bytes per lane; W = 2: 8 bytes, half the registers)
template <int W>
using VecW4 = uint32_t[4][W];

template <int W>
__device__ __forceinline__ VecW4<W>& v4(uint32_t (&a)[W]) { return reinterpret_cast<VecW4<W>&>(a); }

// acc (4 rows) ^= leaf * [v[0..3]]
template <bool PIN, int W>
__device__ __forceinline__ void leaf4(VecW4<W>& acc, VecW4<W>& v, const u32x4* tab01, const uint32_t* tab2, int leaf) {
  dy_col4<1, PIN>(acc, v[0], v[1], v[2], v[3], tab01 + leaf * 9, tab2 + leaf * 9, 0);
}

template <int W>
__device__ __forceinline__ void xor_into(VecW4<W>& dst, const VecW4<W>& src) {
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int w = 0; w < W; ++w) dst[r][w] ^= src[r][w];
}

// W-dword lane chunk loads and stores, the shard tail byte-wise
template <int W>
__device__ __forceinline__ void ld_lane(const uint8_t* p, bool full, size_t rem, uint32_t (&x)[W]) {
  if (full) {
    ld_chunk<W, true>(p, x);
  } else {
    const u32x4 v = ld_tail(p, rem < 4 * W ? rem : 4 * W);
#pragma unroll
    for (int w = 0; w < W; ++w) x[w] = v[w];
  }
}

#ifndef CFSEC_DY16_ST_NT
#define CFSEC_DY16_ST_NT 1  // non-temporal output stores (0: plain, the A/B of tools/dy16_st_ab.sh)
#endif
template <int W>
__device__ __forceinline__ void st_lane(uint8_t* p, bool full, size_t rem, const uint32_t (&x)[W]) {
  if (full) {
    st_chunk<W, (bool)CFSEC_DY16_ST_NT>(p, x);
  } else {
    u32x4 v{0u, 0u, 0u, 0u};
#pragma unroll
    for (int w = 0; w < W; ++w) v[w] = x[w];
    st_tail(p, v, rem < 4 * W ? rem : 4 * W);
  }
}

// The rows of a 16-input matrix opening with a 16x16 dyadic block: 16 + 4 R4 + E rows from the 16
// input chunks x (clobbered), each handed to put(r, chunk) as soon as it is final.  Rows 16.. (the
// 4x4 row blocks, then the E plain rows) come first, from the original inputs, one group at a time
// in acc[16..]; then the 16x16 block into acc[0..15].
struct NoHook {
  __device__ __forceinline__ void operator()() const {}
};

// hook() runs after rows 16.. and before the 16x16 block (repair_dy16: the compared rows' loads)
template <int R4, int E, bool PIN, int W, class Put, class Hook = NoHook>
__device__ __forceinline__ void dy16_rows(uint32_t (&x)[16][W], const u32x4* tab01, const uint32_t* tab2, Put&& put,
                                          Hook&& hook = Hook()) {
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
      dy_col4<R4, PIN>(racc, x[4 * cb], x[4 * cb + 1], x[4 * cb + 2], x[4 * cb + 3], tq + cb * 9, tt + cb * 9, 4 * 9);
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
    for (int c = 0; c < K; ++c) {
      mac_row_k<E>(eacc, x[c], tab01 + ND + c * E, tab2 + ND + c * E);
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
  hook();
  // the 16x16 block: S = X + Y into x[0..7]
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int w = 0; w < W; ++w) x[j][w] ^= x[j + 8][w];
  // rows 8..15 = C Y, C = A + B (leaves 3..5): the 8x8 recursion on Y, rows 8..15 start at zero
  leaf4<PIN, W>(v4<W>(acc[12]), v4<W>(x[12]), tab01, tab2, 4);  // C_c Y_hi
#pragma unroll
  for (int r = 8; r < 12; ++r)
#pragma unroll
    for (int w = 0; w < W; ++w) acc[r][w] = acc[r + 4][w];
#pragma unroll
  for (int j = 8; j < 12; ++j)
#pragma unroll
    for (int w = 0; w < W; ++w) x[j][w] ^= x[j + 4][w];  // Y_lo + Y_hi (Y is dead after this)
  leaf4<PIN, W>(v4<W>(acc[8]), v4<W>(x[8]), tab01, tab2, 3);    // C_a
  leaf4<PIN, W>(v4<W>(acc[12]), v4<W>(x[8]), tab01, tab2, 5);   // C_b
  // rows 0..7 = C Y as well, then += A S; rows 8..15 += B S
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
    leaf4<PIN, W>(tmp, v4<W>(x[4]), tab01, tab2, 1);  // A_c S_hi
    xor_into<W>(v4<W>(acc[0]), tmp);
    xor_into<W>(v4<W>(acc[4]), tmp);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int w = 0; w < W; ++w) tmp[r][w] = 0u;
    leaf4<PIN, W>(tmp, v4<W>(x[4]), tab01, tab2, 7);  // B_c S_hi
    xor_into<W>(v4<W>(acc[8]), tmp);
    xor_into<W>(v4<W>(acc[12]), tmp);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int w = 0; w < W; ++w) x[j][w] ^= x[j + 4][w];  // S_lo + S_hi, shared by A and B
  leaf4<PIN, W>(v4<W>(acc[0]), v4<W>(x[0]), tab01, tab2, 0);   // A_a
  leaf4<PIN, W>(v4<W>(acc[4]), v4<W>(x[0]), tab01, tab2, 2);   // A_b
  leaf4<PIN, W>(v4<W>(acc[8]), v4<W>(x[0]), tab01, tab2, 6);   // B_a
  leaf4<PIN, W>(v4<W>(acc[12]), v4<W>(x[0]), tab01, tab2, 8);  // B_b
#pragma unroll
  for (int r = 0; r < 16; ++r) put(r, acc[r]);
}

// Kernel body: 16 inputs, M = 16 + 4 R4 + E outputs; 256-thread workgroups, each lane one chunk of
// W dwords of every row (tile 256 * 4W bytes), grid (tiles, stripes).
template <int M, int R4, int E, MatVecMode MODE, bool PIN = true, int W = 4>
__device__ __forceinline__ void matvec_dy16(const GfArgs& a) {
  constexpr int K = 16, N4 = R4 * 4 * 9;
  constexpr uint32_t kLane = 4 * W;
  static_assert(M == 16 + 4 * R4 + E, "dyadic-16 shape");
  constexpr bool kVer = MODE == MatVecMode::kVerify;
  __shared__ u32x4 tab01[kDy16Leaves + N4 + K * E];
  __shared__ uint32_t tab2[kDy16Leaves + N4 + K * E];
  build_dy16_tables<R4, E>(a.coef, tab01, tab2);
  __syncthreads();

  const uint32_t stripe = blockIdx.y, tile = blockIdx.x;
  const size_t ts = a.sstride ? 0 : (size_t)stripe;
  const int64_t sbase = (int64_t)stripe * a.sstride;
  uint32_t off = tile * (256u * kLane) + (uint32_t)threadIdx.x * kLane;
  const uint8_t* row[K + M];
#pragma unroll
  for (int c = 0; c < K; ++c) row[c] = a.ptr[ts * K + c] + sbase;
#pragma unroll
  for (int r = 0; r < M; ++r) row[K + r] = a.ptr[(size_t)a.tab * K + ts * M + r] + sbase;
  __builtin_amdgcn_sched_barrier(0);

  // the ragged end of a row as the row's last full lane chunk (gf_dyadic.hpp matvec_dy): no lane of a
  // row of at least one chunk takes the byte path
  const uint64_t slen = stripe_len(a, stripe);
  const bool inrow = off < slen;
  if (inrow && slen >= kLane && (uint64_t)off + kLane > slen) off = (uint32_t)(slen - kLane);
  const bool full = (uint64_t)off + kLane <= slen;
  const size_t rem = inrow ? (size_t)(slen - off) : 0;
  uint32_t diff = 0;
  if (full || rem) {
    uint32_t x[K][W];
#pragma unroll
    for (int c = 0; c < K; ++c) ld_lane<W>(row[c] + off, full, rem, x[c]);
    // store (or compare) output row r as soon as it is final, so its registers are free for the
    // 16x16 block's temporaries
    dy16_rows<R4, E, PIN, W>(x, tab01, tab2, [&](int r, const uint32_t (&v)[W]) {
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

// Reconstruct (+ Verify) of a stripe of the 16 + 20 code (EC16P20 and EC16P20L2's global stripe)
// whose first 16 present shards are ND < 5 parity rows and the 16 - ND surviving data rows: the
// ND missing data rows from their decode rows (16 ND products), then all 20 parity rows from the
// 16 data rows through the 16x16 dyadic block (117 products) -- every parity row the reference's
// Reconstruct writes is stored, every one its Verify reads is compared, the rest dropped.  The plain
// reconstruct-and-verify product over the first 16 present rows takes 16 per output row: 320 for
// the 4-erasure repair of a tasklet bid (2 data + 2 parity missing, 16 compared).
// E extra rows over the data follow the parity rows (EC16P20L2: its 2 local parities, so the
// global pass also does the local Verify, lrcencoder.go:89-131): E more plain rows of the 16 data
// chunks, like the fused LRC encode (dy16_rows).
// Args: coef rows 0..19 the parity matrix, rows 20..20+E-1 the extra rows, then the decode rows;
// ptr per stripe: the 16 inputs, then ND + 20 + E outputs (the missing data rows, parity rows
// 0..19, the extra rows); src[i] = the input slot of data row i, or 16 + j for missing data row j;
// pstore / pcmp: parity (bits 0..19) and extra (20..) rows stored / compared.
// SLOTS: the inputs come in data-row slots (slot i = data row i when present, else the parity row
// standing in for a missing one; the decode rows' coefficients in slot order; src[j] = the data row
// of missing row j, gf_dy16.hip to_slot_order): missing row j then replaces its slot's input through
// one uniform branch, where the run-time permutation of the first-16-present order costs v_cndmask
// selects on every data row (~100 VALU ops per dword column, PMC: profiles/r04).
// PF: the compared rows of the 16x16 block are loaded before the block is computed (else each when
// its row is final, all 16 at the end of the block: their latency exposed once per lane chunk).
template <int ND, int E, bool PIN = true, int W = 2, bool SLOTS = false, bool PF = false>
__device__ __forceinline__ void repair_dy16(const GfArgs& a) {
  constexpr int K = 16, NDY = kDy16Leaves + 36 + K * E, NT = NDY + K * (ND > 0 ? ND : 1), MO = ND + 20 + E;
  constexpr uint32_t kLane = 4 * W;
  __shared__ u32x4 tab01[NT];
  __shared__ uint32_t tab2[NT];
  build_dy16_tables<1, E>(a.coef, tab01, tab2);
  for (int i = threadIdx.x; i < K * ND; i += (int)blockDim.x)  // slot NDY + c * ND + j: decode row j, column c
    coef_tables(a.coef[(20 + E + i % ND) * K + i / ND], tab01[NDY + i], tab2[NDY + i]);
  __syncthreads();

  if (a.zw && blockIdx.x == 0 && blockIdx.y == 0)  // the batch's checksum words (gf_device.hpp GfArgs)
    for (uint32_t i = threadIdx.x; i < a.nzw; i += blockDim.x) a.zw[i] = 0u;
  const uint32_t stripe = blockIdx.y, tile = blockIdx.x;
  const size_t ts = a.sstride ? 0 : (size_t)stripe;
  const int64_t sbase = (int64_t)stripe * a.sstride;
  uint32_t off = tile * (256u * kLane) + (uint32_t)threadIdx.x * kLane;
  // the ragged end of a row as the row's last full lane chunk (gf_dyadic.hpp matvec_dy): no lane of a
  // row of at least one chunk takes the byte path
  const uint64_t slen = stripe_len(a, stripe);
  const bool inrow = off < slen;
  if (inrow && slen >= kLane && (uint64_t)off + kLane > slen) off = (uint32_t)(slen - kLane);
  const bool full = (uint64_t)off + kLane <= slen;
  const size_t rem = inrow ? (size_t)(slen - off) : 0;
  uint32_t diff = 0;
  if (full || rem) {
    const uint8_t* const* in = a.ptr + ts * K;
    uint8_t* const* out = const_cast<uint8_t* const*>(a.ptr + (size_t)a.tab * K + ts * MO);
    const auto sb = [&]() {
      if constexpr (PIN) __builtin_amdgcn_sched_barrier(0);
    };
    uint32_t x[K][W];
#pragma unroll
    for (int c = 0; c < K; ++c) ld_lane<W>(in[c] + sbase + off, full, rem, x[c]);
    sb();
    if constexpr (ND > 0) {
      // the missing data rows, stored
      uint32_t rec[ND][W];
#pragma unroll
      for (int j = 0; j < ND; ++j)
#pragma unroll
        for (int w = 0; w < W; ++w) rec[j][w] = 0u;
#pragma unroll
      for (int c = 0; c < K; ++c) {
        mac_row_k<ND>(rec, x[c], tab01 + NDY + c * ND, tab2 + NDY + c * ND);
        if constexpr (PIN)
#pragma unroll
          for (int j = 0; j < ND; ++j)
#pragma unroll
            for (int w = 0; w < W; ++w) asm volatile("" : "+v"(rec[j][w]));
        sb();
      }
#pragma unroll
      for (int j = 0; j < ND; ++j) st_lane<W>(out[j] + sbase + off, full, rem, rec[j]);
      if constexpr (SLOTS) {
        // missing row j replaces the parity input in its slot: a uniform branch (the asm keeps it
        // one -- as a select it costs W v_cndmask per slot)
#pragma unroll
        for (int j = 0; j < ND; ++j) {
          const uint32_t m = a.src[j];
#pragma unroll
          for (int i = 0; i < K; ++i) {
            if (m == (uint32_t)i) {
              asm volatile("" ::: "memory");
#pragma unroll
              for (int w = 0; w < W; ++w) x[i][w] = rec[j][w];
            }
          }
        }
      } else {
        // the data rows in order, in place: data row i is input slot i - (missing rows below i),
        // so from the top down no slot is overwritten before it is read
#pragma unroll
        for (int i = K - 1; i >= 0; --i) {
          const uint32_t s = a.src[i];
#pragma unroll
          for (int d = 0; d <= ND; ++d)
            if (i - d >= 0 && s == (uint32_t)(i - d))
#pragma unroll
              for (int w = 0; w < W; ++w) x[i][w] = x[i - d][w];
#pragma unroll
          for (int j = 0; j < ND; ++j)
            if (s == (uint32_t)(K + j))
#pragma unroll
              for (int w = 0; w < W; ++w) x[i][w] = rec[j][w];
        }
      }
      sb();
    }
    const uint32_t pstore = a.pstore, pcmp = a.pcmp;
    const uint8_t* spare = in[0] + sbase + off;  // just read: what rows not compared load instead
    uint32_t yb[PF ? 16 : 1][W];                 // PF: the 16x16 block's compared rows
    const auto load_cmp = [&](int r, uint32_t (&y)[W]) {
      // every row loads (its own chunk if compared, else the input chunk above, a cache hit) and
      // the mask picks: no branch around the loads, so the compiler issues a group of them before
      // the first wait (a branch per row exposed one load latency per compared row: +45 % time)
      const bool cmp = (pcmp >> r) & 1u;
      if constexpr (SLOTS)  // the row base chosen on the scalar unit, then the lane offset
        ld_lane<W>((cmp ? (const uint8_t*)out[ND + r] : in[0]) + sbase + off, full, rem, y);
      else
        ld_lane<W>(cmp ? (const uint8_t*)out[ND + r] + sbase + off : spare, full, rem, y);
    };
    dy16_rows<1, E, PIN, W>(
        x, tab01, tab2,
        [&](int r, const uint32_t (&v)[W]) {
          uint8_t* p = out[ND + r] + sbase + off;
          uint32_t y[W];
          if (PF && r < 16) {
#pragma unroll
            for (int w = 0; w < W; ++w) y[w] = yb[PF ? r : 0][w];
          } else {
            load_cmp(r, y);
          }
          const uint32_t msk = ((pcmp >> r) & 1u) ? ~0u : 0u;
#pragma unroll
          for (int w = 0; w < W; ++w) diff |= (y[w] ^ v[w]) & msk;
          if ((pstore >> r) & 1u) st_lane<W>(p, full, rem, v);
        },
        [&]() {
          if constexpr (PF) {
#pragma unroll
            for (int r = 0; r < 16; ++r) load_cmp(r, yb[r]);
          }
        });
  }
  if (diff) dev::set_flag(a.flags, stripe);
}

}  // namespace dev
}  // namespace cfsec
