// gf_crc.hpp -- fused GF(2^8) matrix x shard-vector product + shard CRC32-IEEE (gfx950).
//
// CubeFS checksums every shard right after coding it: access computes crc32.ChecksumIEEE of
// each data and parity shard after Encode (blobstore/access/stream_put.go:249-253) and blobnode
// checksums shards around a repair (blobnode/work_shard_recover.go:335-342, 668-683).  As a
// separate pass that re-reads every shard from HBM.  This kernel checksums the 16-byte pieces
// the GF tile already holds in registers, so an encode with checksums moves exactly the bytes
// of the plain encode ("CRC fused: +0 bytes").
//
// CRC algebra (Go hash/crc32 IEEE: reflected polynomial 0xEDB88320, bit 31 = x^0).  f(r, B) is
// the register after feeding bytes B from register r with no pre/post inversion; f(r, B) =
// shift(r, |B|) ^ f(0, B) with shift(v, n) = v * x^(8n) mod P, and
// ChecksumIEEE(M) = f(0, M) ^ shift(~0, |M|) ^ ~0.
//
// Work split.  A workgroup owns `tpw` consecutive 4 KiB tiles of one stripe; thread j holds
// bytes [16j, 16j+16) of every row of each tile (the fixed-K GF tile of gf_device.hpp).  Per
// checksummed row it keeps a Horner register over its pieces, R <- f(shift(R, 4080), piece):
// 20 independent byte-table lookups per 16 bytes (crc_step below).  After
// its last tile the thread moves R from its piece end to the tile end e (x^(8*16*(255-j)), a
// 32-column GF(2) basis read once from global memory), the 256 threads XOR-reduce, and one
// multiply by x^(8(S - e)) moves the sum to the shard end (a host constant per workgroup;
// negative for the zero-padded last tile -- x is invertible mod P).  Workgroups XOR their words
// into the shard's word (atomicXor) and workgroup 0 also folds in shift(~0, S) ^ ~0, so the word
// ends as crc32.ChecksumIEEE with no finalize pass.
#pragma once
#include <hip/hip_runtime.h>

#include "gf_device.hpp"
#include "gf_dyadic.hpp"
#include "kernels.hpp"

namespace cfsec {
namespace crcdev {

using dev::u32x4;

constexpr uint32_t kPoly = 0xEDB88320u;
constexpr int kTile = 4096;            // bytes per row per tile: 256 threads x 16 B
constexpr int kMaxK = 18, kMaxM = 12, kPtrSlots = 96, kMaxGroups = 384;  // m = 12: EC6P10L2's fused encode
constexpr int kByteTabWords = 20 * 256;  // F0..F15: bytes of a 16-B piece;  G0..G3: register bytes
constexpr int kNibTabWords = 40 * 16;    // N0..N31: nibbles of a 16-B piece;  H0..H7: register nibbles
constexpr int kFiveFields = 7;           // per 32-bit word: six 5-bit fields + one 2-bit field
constexpr int kFiveTabWords = 5 * kFiveFields * 32;  // Q(w, f): 4 piece words + the register word
constexpr int kTabWords = kByteTabWords + kNibTabWords + kFiveTabWords;  // device table block, the basis follows
constexpr int kBasisWords = 256 * 32;  // thread j: the 32 columns of shift(., 16*(255-j))
constexpr int kShiftWords = 256;  // after the basis: [j] = x^(8*16*(255-j)), its column x^0 (coalesced)

struct __attribute__((aligned(16))) GfCrcArgs {
  uint64_t len;
  uint32_t k, m, tiles, tpw;
  int64_t sstride;       // affine batch: byte distance between stripes (0: explicit table)
  uint32_t tab, fin;     // stripes held in ptr[]; shift(~0, len) ^ ~0
  uint32_t* crc;         // [stripe][crc_stride] checksum words, zeroed by the launcher
  const uint32_t* tabs;  // device: kTabWords + kBasisWords + kShiftWords
  uint32_t crc_stride, pad0;
  uint8_t slot[kMaxK + kMaxM];  // checksum word of kernel row i (inputs 0..k-1, outputs k..)
  uint8_t coef[kMaxM * kMaxK];
  const uint8_t* ptr[kPtrSlots];  // [tab*k inputs][tab*m outputs], as GfArgs
  uint32_t gconst[kMaxGroups];    // x^(8(len - e_g)) mod P for workgroup g
};
static_assert(sizeof(GfCrcArgs) <= 3584, "kernel argument block must stay below 4 KiB");

// Two equivalent Horner steps R <- f(shift(R, 4080), d) over a thread's next 16-byte piece d,
// which sits 4080 bytes after its previous one.  The byte-table step costs 20 LDS reads and ~30
// VALU; its random byte indices into 256-word tables conflict (~2.6 LDS cycles per read per lane
// group).  The nibble-table step costs 40 conflict-free reads and ~80 VALU.  Kernels whose VALU
// is already busy with the GF product (gf_crc_kernel) take the byte step; the CRC-only kernels
// (crc32.hip, crc32block.hip) take the nibble step (profiles/r01/crc_nibble_ab.txt: also the
// earlier slice-by-8 byte step, whose three dependent LDS rounds per piece cost 1-8 %).

// Byte tables ct (kByteTabWords): f(shift(R, 4080), d) = shift(R, 4096) ^ f(0, d) as the XOR of
// 20 independent words, F_j[b] = f(0, the piece with byte j = b, all else 0) and
// G_q[b] = shift(b << 8q, 4096): one LDS round per piece instead of three dependent ones.
__device__ __forceinline__ uint32_t crc_step(const uint32_t* ct, uint32_t r, const uint32_t (&d)[4]) {
  const uint32_t v[5] = {d[0], d[1], d[2], d[3], r};
  uint32_t t[20];
#pragma unroll
  for (int w = 0; w < 5; ++w)
#pragma unroll
    for (int j = 0; j < 4; ++j) t[4 * w + j] = ct[(4 * w + j) * 256 + ((v[w] >> (8 * j)) & 0xFFu)];
  uint32_t u[7];
#pragma unroll
  for (int i = 0; i < 6; ++i) u[i] = __builtin_amdgcn_bitop3_b32(t[3 * i], t[3 * i + 1], t[3 * i + 2], 0x96);
  u[6] = t[18] ^ t[19];
  return __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(u[0], u[1], u[2], 0x96),
                                     __builtin_amdgcn_bitop3_b32(u[3], u[4], u[5], 0x96), u[6], 0x96);
}

// Nibble tables nt (kNibTabWords): f(shift(R, 4080), d) = shift(R, 4096) ^ f(0, d), both
// GF(2)-linear, as the XOR of 40 words: N_p[n] = f(0, the piece with nibble p = n, all else 0)
// for the 32 nibbles of d, H_q[n] = shift(n << 4q, 4096) for the 8 nibbles of R.  A 16-word
// table lies in 16 distinct banks of ds_read_b32's 32, so lanes either hit distinct banks or
// broadcast one word: no conflicts.  The 40 reads are independent (R is not folded into the
// data first), so the Horner chain through R is one LDS round per piece.
__device__ __forceinline__ uint32_t nib_word(const uint32_t* t, uint32_t scaled) {
  return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(t) + scaled);
}

__device__ __forceinline__ uint32_t crc_step_nib(const uint32_t* nt, uint32_t r, const uint32_t (&d)[4]) {
  const uint32_t v[5] = {d[0], d[1], d[2], d[3], r};
  uint32_t t[40];
#pragma unroll
  for (int w = 0; w < 5; ++w) {
    // byte j of lo / hi = 4 x (low / high nibble of byte j): one byte extract per address.  The
    // empty asm keeps the compiler from re-forming each address as its own shift + mask.
    uint32_t lo = (v[w] << 2) & 0x3C3C3C3Cu, hi = (v[w] >> 2) & 0x3C3C3C3Cu;
    asm volatile("" : "+v"(lo), "+v"(hi));
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      t[8 * w + 2 * j] = nib_word(nt + (8 * w + 2 * j) * 16, (lo >> (8 * j)) & 0xFFu);
      t[8 * w + 2 * j + 1] = nib_word(nt + (8 * w + 2 * j + 1) * 16, (hi >> (8 * j)) & 0xFFu);
    }
  }
  // three-input XORs (v_bitop3_b32): 40 -> 1 in 20 instructions
  uint32_t u[14];
#pragma unroll
  for (int i = 0; i < 13; ++i) u[i] = __builtin_amdgcn_bitop3_b32(t[3 * i], t[3 * i + 1], t[3 * i + 2], 0x96);
  u[13] = t[39];
  const uint32_t a0 = __builtin_amdgcn_bitop3_b32(u[0], u[1], u[2], 0x96);
  const uint32_t a1 = __builtin_amdgcn_bitop3_b32(u[3], u[4], u[5], 0x96);
  const uint32_t a2 = __builtin_amdgcn_bitop3_b32(u[6], u[7], u[8], 0x96);
  const uint32_t a3 = __builtin_amdgcn_bitop3_b32(u[9], u[10], u[11], 0x96);
  const uint32_t a4 = __builtin_amdgcn_bitop3_b32(u[12], u[13], a0, 0x96);
  return __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(a1, a2, a3, 0x96), a4, 0u, 0x96);
}

// 5-bit tables ft (kFiveTabWords, at kByteTabWords + kNibTabWords in the device block): the same
// step as the XOR of 35 words.  Each 32-bit word v of (d0..d3, R) is cut into fields at bits 0, 5,
// ..., 25 (5 bits) and 30 (2 bits); Q(w, f)[e] = the step's image of word w = e << 5f, all else 0.
// A table of at most 32 words sits in 32 distinct banks, so ds_read_b32 (2 x 32-lane groups,
// bank = word mod 32) never conflicts: 35 LDS cycles-per-group per piece against ~20 x 3.1 for the
// byte step (SQ_LDS_BANK_CONFLICT, profiles/r01/pmc_lds_conflicts_crc.txt) and 40 for the nibble
// step.  Addresses cost one VALU each: the odd fields (5, 15, 25) are extracted from v & mO and
// the even ones (10, 20, 30) from v & mE, 7 bits starting 2 below the field, whose two low bits
// belong to a field the mask cleared -- so the extract is already the byte offset 4 * field.
// Field 0 takes a shift + mask.
template <int W>
__device__ __forceinline__ void five_word(const uint32_t* ft, uint32_t v, uint32_t* t) {
  uint32_t e = v & 0xC1F07C00u, o = v & 0x3E0F83E0u;
  asm volatile("" : "+v"(e), "+v"(o));  // keep the masked copies (no re-formed shift + mask per field)
  const uint32_t off[kFiveFields] = {(v << 2) & 0x7Cu,       __builtin_amdgcn_ubfe(o, 3, 7),
                                     __builtin_amdgcn_ubfe(e, 8, 7),  __builtin_amdgcn_ubfe(o, 13, 7),
                                     __builtin_amdgcn_ubfe(e, 18, 7), __builtin_amdgcn_ubfe(o, 23, 7),
                                     __builtin_amdgcn_ubfe(e, 28, 4)};
#pragma unroll
  for (int f = 0; f < kFiveFields; ++f) t[f] = nib_word(ft + (W * kFiveFields + f) * 32, off[f]);
}

__device__ __forceinline__ uint32_t crc_step5(const uint32_t* ft, uint32_t r, const uint32_t (&d)[4]) {
  uint32_t t[5 * kFiveFields];
  five_word<0>(ft, d[0], t);
  five_word<1>(ft, d[1], t + kFiveFields);
  five_word<2>(ft, d[2], t + 2 * kFiveFields);
  five_word<3>(ft, d[3], t + 3 * kFiveFields);
  five_word<4>(ft, r, t + 4 * kFiveFields);
  // 35 -> 1 in 17 three-input XORs
  uint32_t u[12];
#pragma unroll
  for (int i = 0; i < 11; ++i) u[i] = __builtin_amdgcn_bitop3_b32(t[3 * i], t[3 * i + 1], t[3 * i + 2], 0x96);
  u[11] = t[33] ^ t[34];
  const uint32_t a0 = __builtin_amdgcn_bitop3_b32(u[0], u[1], u[2], 0x96);
  const uint32_t a1 = __builtin_amdgcn_bitop3_b32(u[3], u[4], u[5], 0x96);
  const uint32_t a2 = __builtin_amdgcn_bitop3_b32(u[6], u[7], u[8], 0x96);
  const uint32_t a3 = __builtin_amdgcn_bitop3_b32(u[9], u[10], u[11], 0x96);
  return __builtin_amdgcn_bitop3_b32(a0, a1, a2 ^ a3, 0x96);
}

// The fused product+CRC kernel's step: 5-bit tables by default (CFSEC_FUSED_STEP=0: byte tables,
// for A/B probes).
#ifndef CFSEC_FUSED_STEP
#define CFSEC_FUSED_STEP 1
#endif
#if CFSEC_FUSED_STEP
constexpr int kFusedTabBase = kByteTabWords + kNibTabWords, kFusedTabWords = kFiveTabWords;
__device__ __forceinline__ uint32_t fused_step(const uint32_t* ct, uint32_t r, const uint32_t (&d)[4]) {
  return crc_step5(ct, r, d);
}
#else
constexpr int kFusedTabBase = 0, kFusedTabWords = kByteTabWords;
__device__ __forceinline__ uint32_t fused_step(const uint32_t* ct, uint32_t r, const uint32_t (&d)[4]) {
  return crc_step(ct, r, d);
}
#endif

// The CRC-only kernels' step (crc32.hip, crc32block.hip): 5-bit tables by default
// (CFSEC_CRC_ONLY_STEP=0: nibble tables, for A/B probes).
#ifndef CFSEC_CRC_ONLY_STEP
#define CFSEC_CRC_ONLY_STEP 1
#endif
#if CFSEC_CRC_ONLY_STEP
constexpr int kOnlyTabBase = kByteTabWords + kNibTabWords, kOnlyTabWords = kFiveTabWords;
__device__ __forceinline__ uint32_t only_step(const uint32_t* ct, uint32_t r, const uint32_t (&d)[4]) {
  return crc_step5(ct, r, d);
}
#else
constexpr int kOnlyTabBase = kByteTabWords, kOnlyTabWords = kNibTabWords;
__device__ __forceinline__ uint32_t only_step(const uint32_t* ct, uint32_t r, const uint32_t (&d)[4]) {
  return crc_step_nib(ct, r, d);
}
#endif

// a * b mod P (reflected: bit 31 = x^0)
__device__ __forceinline__ uint32_t mulmod(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (uint32_t bit = 0x80000000u; bit; bit >>= 1) {
    if (a & bit) p ^= b;
    b = (b >> 1) ^ ((b & 1u) ? kPoly : 0u);
  }
  return p;
}

// One tile of the product for this thread (bytes [off, off+16) of every row) plus the Horner
// step of every checksummed row.  Full pieces take the pipelined path: input rows are loaded D
// rows ahead of the product, and the last D loads of a tile fetch the first rows of the thread's
// next tile when that one is full too (`next`; then `pre` says those rows are already in x).  The
// thread holding the shard end (or past it) reads/writes only bytes < len and checksums the piece
// zero-padded, which is what the negative group shift undoes.
#ifndef CFSEC_CRC_LOOKAHEAD
#define CFSEC_CRC_LOOKAHEAD 2
#endif
template <int K, int M, bool CIN>
__device__ __forceinline__ void crc_tile(uint64_t len, const u32x4* tab01, const uint32_t* tab2,
                                         const uint32_t* ct, const uint8_t* const (&row)[K + M],
                                         uint32_t off, bool pre, bool next, uint32_t (&x)[K][4],
                                         uint32_t (&R)[(CIN ? K : 0) + M]) {
  constexpr int RO = CIN ? K : 0;  // register of output row 0
  constexpr int D = CFSEC_CRC_LOOKAHEAD < K ? CFSEC_CRC_LOOKAHEAD : K;
  static_assert(K % 2 == 0 && D % 2 == 0, "row pairs");
  uint32_t acc[M][4];
#pragma unroll
  for (int r = 0; r < M; ++r)
#pragma unroll
    for (int w = 0; w < 4; ++w) acc[r][w] = 0u;
  const auto pin = [&]() {
#pragma unroll
    for (int r = 0; r < M; ++r)
      asm volatile("" : "+v"(acc[r][0]), "+v"(acc[r][1]), "+v"(acc[r][2]), "+v"(acc[r][3]));
  };
  if ((uint64_t)off + dev::kLaneBytes <= len) {
    const auto load = [&](int c, uint32_t o) {
      const u32x4 v = dev::ld16<true>(row[c] + o);
      x[c][0] = v.x;
      x[c][1] = v.y;
      x[c][2] = v.z;
      x[c][3] = v.w;
    };
    if (!pre)
#pragma unroll
      for (int c = 0; c < D; ++c) load(c, off);
#pragma unroll
    for (int c = 0; c < K; c += 2) {
#pragma unroll
      for (int j = c + D; j < c + D + 2; ++j) {
        if (j < K) load(j, off);
        else if (next) load(j - K, off + kTile);
      }
      __builtin_amdgcn_sched_barrier(0);
      dev::mac_pair_k<M>(acc, x[c], x[c + 1], tab01 + c * M, tab2 + c * M, tab01 + (c + 1) * M,
                         tab2 + (c + 1) * M);
      pin();
      if constexpr (CIN) {
        R[c] = fused_step(ct, R[c], x[c]);
        R[c + 1] = fused_step(ct, R[c + 1], x[c + 1]);
        asm volatile("" : "+v"(R[c]), "+v"(R[c + 1]));
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int r = 0; r < M; ++r)
      dev::st16_out<true>(const_cast<uint8_t*>(row[K + r]) + off, u32x4{acc[r][0], acc[r][1], acc[r][2], acc[r][3]});
  } else {
    const size_t rem = off < len ? (size_t)(len - off) : 0;
    for (int c = 0; c < K; ++c) {
      uint32_t xv[4] = {0u, 0u, 0u, 0u};
      if (rem) {
        const u32x4 v = dev::ld_tail_row(row[c] + off, rem, len);
        xv[0] = v.x;
        xv[1] = v.y;
        xv[2] = v.z;
        xv[3] = v.w;
      }
      dev::mac_row_k<M>(acc, xv, tab01 + c * M, tab2 + c * M);
      if constexpr (CIN) R[c] = fused_step(ct, R[c], xv);
    }
    if (rem)
#pragma unroll
      for (int r = 0; r < M; ++r)
        dev::st_tail(const_cast<uint8_t*>(row[K + r]) + off, u32x4{acc[r][0], acc[r][1], acc[r][2], acc[r][3]},
                     rem);
  }
#pragma unroll
  for (int r = 0; r < M; ++r) R[RO + r] = fused_step(ct, R[RO + r], acc[r]);
}

// The product of a dyadic matrix in the fused kernel (gf_dyadic.hpp): 4x4 blocks for 4 outputs
// (EC12P4 / EC16P4 encode and their coset-aligned repairs: dy_col4, 9 products per block instead of
// 16), 2x2 blocks for 6 outputs of 6 inputs (EC6P6 encode: dy_col2, 3 instead of 4); rows loaded one
// column block ahead, the CRC step of each block's input rows after its product.  The kernel is
// VALU-issue-bound (§4.1 of DESIGN.md), so fewer products pay even at 3 waves per SIMD (144 VGPRs):
// EC12P4 8 x 64 MiB encode + CRC 242 -> 224 us (profiles/r02/fused_crc_ab.txt).
// E > 0: the last E of the M rows are plain rows over the inputs (the local parities of the fused
// EC6P10L2 encode: 10 dyadic global rows + 2 local rows, every one of its 18 shards checksummed as
// access's Put does, stream_put.go:249-253), on the loaded inputs of each column block.
template <int K, int M, int B, bool CIN, int E = 0>
__device__ __forceinline__ void crc_tile_dy(uint64_t len, const u32x4* tab01, const uint32_t* tab2,
                                            const uint32_t* ct, const uint8_t* const (&row)[K + M],
                                            uint32_t off, uint32_t (&R)[(CIN ? K : 0) + M]) {
  constexpr int MD = M - E;
  constexpr int RO = CIN ? K : 0, KB = K / B, MB = MD / B, NC = dev::Dy<B>::NC, ND = MB * KB * NC;
  static_assert(K % B == 0 && MD % B == 0 && (B == 2 || (B == 4 && M == 4 && E == 0)), "dyadic shape");
  static_assert(E == 0 || B == 2, "plain rows ride along the 2x2-dyadic product");
  uint32_t acc[M][4];
#pragma unroll
  for (int r = 0; r < M; ++r)
#pragma unroll
    for (int w = 0; w < 4; ++w) acc[r][w] = 0u;
  const auto product = [&](int cb, uint32_t (&xs)[B][4]) {
    if constexpr (B == 4) {
      dev::dy_col4<1, true>(acc, xs[0], xs[1], xs[2], xs[3], tab01 + cb * NC, tab2 + cb * NC, KB * NC);
    } else {
      dev::dy_col2<MB, true>(reinterpret_cast<uint32_t(&)[MD][4]>(acc), xs[0], xs[1], tab01 + cb * NC,
                             tab2 + cb * NC, KB * NC);
      if constexpr (E > 0) {
        const int c = B * cb;
        dev::mac_pair_k<E>(reinterpret_cast<uint32_t(&)[E][4]>(acc[MD]), xs[0], xs[1], tab01 + ND + c * E,
                           tab2 + ND + c * E, tab01 + ND + (c + 1) * E, tab2 + ND + (c + 1) * E);
      }
    }
  };
  if ((uint64_t)off + dev::kLaneBytes <= len) {
    uint32_t x[K][4];
    const auto load = [&](int c) {
      const u32x4 v = dev::ld16<true>(row[c] + off);
      x[c][0] = v.x;
      x[c][1] = v.y;
      x[c][2] = v.z;
      x[c][3] = v.w;
    };
#pragma unroll
    for (int c = 0; c < B; ++c) load(c);
#pragma unroll
    for (int cb = 0; cb < KB; ++cb) {
      if (cb + 1 < KB)
#pragma unroll
        for (int c = 0; c < B; ++c) load(B * cb + B + c);
      __builtin_amdgcn_sched_barrier(0);
      product(cb, reinterpret_cast<uint32_t(&)[B][4]>(x[B * cb]));
#pragma unroll
      for (int r = 0; r < M; ++r) asm volatile("" : "+v"(acc[r][0]), "+v"(acc[r][1]), "+v"(acc[r][2]), "+v"(acc[r][3]));
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (CIN) {
#pragma unroll
        for (int c = B * cb; c < B * cb + B; ++c) {
          R[c] = fused_step(ct, R[c], x[c]);
          asm volatile("" : "+v"(R[c]));
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int r = 0; r < M; ++r)
      dev::st16_out<true>(const_cast<uint8_t*>(row[K + r]) + off, u32x4{acc[r][0], acc[r][1], acc[r][2], acc[r][3]});
  } else {
    const size_t rem = off < len ? (size_t)(len - off) : 0;
    for (int cb = 0; cb < KB; ++cb) {
      uint32_t x[B][4];
      for (int c = 0; c < B; ++c) {
        const u32x4 v = rem ? dev::ld_tail_row(row[B * cb + c] + off, rem, len) : u32x4{0u, 0u, 0u, 0u};
        x[c][0] = v.x;
        x[c][1] = v.y;
        x[c][2] = v.z;
        x[c][3] = v.w;
      }
      product(cb, x);
      if constexpr (CIN)
        for (int c = 0; c < B; ++c) R[B * cb + c] = fused_step(ct, R[B * cb + c], x[c]);
    }
    if (rem)
#pragma unroll
      for (int r = 0; r < M; ++r)
        dev::st_tail(const_cast<uint8_t*>(row[K + r]) + off, u32x4{acc[r][0], acc[r][1], acc[r][2], acc[r][3]}, rem);
  }
#pragma unroll
  for (int r = 0; r < M; ++r) R[RO + r] = fused_step(ct, R[RO + r], acc[r]);
}

// The end of a fused kernel: every Horner register R[i] (row i of the checksummed rows, inputs first
// when CIN) moves from this thread's last piece end to its workgroup's tile end, the workgroup
// XOR-reduces, one multiply by the host constant moves the sum to the shard end, and the word is
// XOR-ed into the row's checksum.
template <int K, int NR, bool CIN>
__device__ __forceinline__ void crc_epilogue(const GfCrcArgs& a, const uint32_t (&R)[NR], uint32_t (&red)[4][NR],
                                             uint32_t g, uint32_t stripe, uint32_t tid, bool live = true) {
  const u32x4* basis = reinterpret_cast<const u32x4*>(a.tabs + kTabWords + tid * 32);
  uint32_t col[32];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const u32x4 v = basis[q];
    col[4 * q] = v.x;
    col[4 * q + 1] = v.y;
    col[4 * q + 2] = v.z;
    col[4 * q + 3] = v.w;
  }
  const int wave = (int)(tid >> 6), lane = (int)(tid & 63);
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    uint32_t o = 0;
#pragma unroll
    for (int b = 0; b < 32; ++b) o ^= (0u - ((R[i] >> b) & 1u)) & col[b];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) o ^= (uint32_t)__shfl_xor((int)o, d);
    if (lane == 0) red[wave][i] = o;
  }
  __syncthreads();
  if (live && (int)tid < NR) {
    const int i = (int)tid;
    uint32_t v = red[0][i] ^ red[1][i] ^ red[2][i] ^ red[3][i];
    v = mulmod(a.gconst[g], v);
    if (g == 0) v ^= a.fin;
    atomicXor(a.crc + (size_t)stripe * a.crc_stride + a.slot[CIN ? i : K + i], v);
  }
}

// DY: a.coef is M x K made of DY x DY dyadic blocks (checked by the launcher; 0: plain product),
// the last E rows plain (DY = 2 only); the register allocation aims at 4 waves per SIMD, 3 for the
// dyadic products
template <int K, int M, bool CIN, int DY, int E = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(DY ? 3 : 4, 8))) void gf_crc_kernel(const GfCrcArgs a) {
  constexpr int NR = (CIN ? K : 0) + M;  // checksummed rows
  __shared__ u32x4 tab01[K * M];
  __shared__ uint32_t tab2[K * M];
  __shared__ uint32_t ct[kFusedTabWords];
  __shared__ uint32_t red[4][NR];
  constexpr bool kDy = DY != 0;
  if constexpr (kDy)
    dev::build_dy_tables<K, M - E, (DY ? DY : 1), (M - E) / (DY ? DY : 1), E>(a.coef, tab01, tab2);
  else
    dev::build_tables<M>(K, M, a.coef, tab01, tab2);
  for (int i = threadIdx.x; i < kFusedTabWords; i += 256) ct[i] = a.tabs[kFusedTabBase + i];
  __syncthreads();

  const uint32_t g = blockIdx.x, stripe = blockIdx.y;
  const size_t ts = a.sstride ? 0 : (size_t)stripe;
  const int64_t sbase = (int64_t)stripe * a.sstride;
  const uint8_t* row[K + M];
#pragma unroll
  for (int c = 0; c < K; ++c) row[c] = a.ptr[ts * K + c] + sbase;
#pragma unroll
  for (int r = 0; r < M; ++r) row[K + r] = a.ptr[(size_t)a.tab * K + ts * M + r] + sbase;
  uint32_t R[NR];
#pragma unroll
  for (int i = 0; i < NR; ++i) R[i] = 0u;
  const uint32_t t0 = g * a.tpw;
  const uint32_t t1 = min(t0 + a.tpw, a.tiles);
  const uint32_t lanepos = threadIdx.x * dev::kLaneBytes;
  uint32_t x[K][4];
  bool pre = false;
  for (uint32_t t = t0; t < t1; ++t) {
    const uint32_t off = t * kTile + lanepos;
    // the next tile is full for this thread: its first rows are fetched during this one
    const bool next = t + 1 < t1 && (uint64_t)off + kTile + dev::kLaneBytes <= a.len;
    if constexpr (kDy) crc_tile_dy<K, M, DY, CIN, E>(a.len, tab01, tab2, ct, row, off, R);
    else crc_tile<K, M, CIN>(a.len, tab01, tab2, ct, row, off, pre, next, x, R);
    pre = next && (uint64_t)off + dev::kLaneBytes <= a.len;
  }
  crc_epilogue<K, NR, CIN>(a, R, red, g, stripe, threadIdx.x);
}

// ---------------------------------------------------------------------------------------------
// Product and checksum from one set of lookups (m <= 4 outputs: 8-byte entries; m <= 12: 16-byte).
//
// The CRC step needs a table lookup per field of every piece anyway; a ds_read_b64 costs the LDS
// the same 2 cycles as a ds_read_b32 (bank = dword mod 64 per 32-lane group, MI355X_MICROARCH.md
// §LDS) and a 16-entry table of 8-byte entries spans the 64 banks once, so nibble lookups are
// conflict-free and can return two words: E_c[p][h][n] = (f(0, the piece whose byte p is n << 4h),
// the m products coef[r][c] * (n << 4h) as bytes r of the second word).  Per 16-byte piece of input
// row c: 32 lookups give the row's CRC step (XOR of the first words) and the 16 bytes' products for
// every output (XOR-accumulated byte-transposed: g[p] byte r = output r's byte p), so the GF product
// costs no v_perm_b32 at all -- the fused kernel was VALU-issue-bound on half-rate v_perm /
// v_bitop3.  Output rows are transposed once per tile (8 v_perm per dword) and
// checksummed through the first words of E_0 (ds_read_b32 at the entry stride: 16 distinct banks, no
// conflicts).  The Horner jump shift(R, 4096) takes the 5-bit tables of the register word (7 reads).
// E is 4 KiB per input row (K = 12: 48 KiB; 3 workgroups per CU).
//
// Round 6: up to 12 outputs with 16-byte entries (the CRC word + three product words, one
// ds_read_b128 per nibble, 16 entries span the 64 banks four times over at 16 B: still one cycle per
// quarter-wave, no conflicts; a b96 read would cost 8 LDS cycles, so m = 5..8 pad to 16 B too), for
// EC6P10L2's fused LRC encode with all 18 checksums (C4; stream_put.go:249-253): 6 inputs x 12
// outputs, E = 6 x 8 KiB.  The v_perm form of that kernel issued 2750 VALU per 64-lane column (the
// 2x2-dyadic product plus 18 rows of 5-bit Horner steps, profiles/r05/pmc_c4_crc_probe.txt).
__device__ __forceinline__ uint32_t gf_mul_dev(uint32_t c, uint32_t v) {
  uint32_t p = 0;
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    if ((v >> b) & 1u) p ^= c;
    c = dev::gf_xtime(c);
  }
  return p;
}

constexpr int lds_nq(int M) { return (M + 3) / 4; }       // product words per entry
constexpr int lds_ew(int M) { return M <= 4 ? 2 : 4; }    // entry words: CRC word + products (padded)
constexpr int lds_row_bytes(int M) { return 16 * 2 * 16 * 4 * lds_ew(M); }  // E_c: 16 pos x 2 nibbles x 16
constexpr int kLdsRowBytes = lds_row_bytes(4);

template <int EW>
struct LdsEnt {
  uint32_t w[EW];
};

template <int EW>
__device__ __forceinline__ LdsEnt<EW> ld_ent(const char* p) {
  LdsEnt<EW> e;
  if constexpr (EW == 2) {
    const dev::u32x2 v = *reinterpret_cast<const dev::u32x2*>(p);
    e.w[0] = v.x;
    e.w[1] = v.y;
  } else {
    const u32x4 v = *reinterpret_cast<const u32x4*>(p);
    e.w[0] = v.x;
    e.w[1] = v.y;
    e.w[2] = v.z;
    e.w[3] = v.w;
  }
  return e;
}

// Byte j of lo / hi = the entry offset (4 * EW * nibble) of the low / high nibble of byte j of v.
template <int EW>
__device__ __forceinline__ void ent_offsets(uint32_t v, uint32_t& lo, uint32_t& hi) {
  if constexpr (EW == 2) {
    lo = (v << 3) & 0x78787878u;
    hi = (v >> 1) & 0x78787878u;
  } else {
    lo = (v << 4) & 0xF0F0F0F0u;
    hi = v & 0xF0F0F0F0u;
  }
  asm volatile("" : "+v"(lo), "+v"(hi));
}

// shift(r, 4096) from the 5-bit tables of the register word (rt = Q(4, .), 7 x 32 words)
__device__ __forceinline__ uint32_t rshift4096(const uint32_t* rt, uint32_t r) {
  uint32_t t[kFiveFields];
  five_word<0>(rt, r, t);
  return __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(t[0], t[1], t[2], 0x96),
                                     __builtin_amdgcn_bitop3_b32(t[3], t[4], t[5], 0x96), t[6], 0x96);
}

// Output dwords from the byte-transposed accumulators: o[r][w] byte i = byte r of g[4w + i].
template <int M>
__device__ __forceinline__ void untranspose(const uint32_t (&g)[16], uint32_t (&o)[M][4]) {
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const uint32_t a = g[4 * w], b = g[4 * w + 1], c = g[4 * w + 2], d = g[4 * w + 3];
    const uint32_t ab_lo = __builtin_amdgcn_perm(b, a, 0x05010400u);  // a0 b0 a1 b1
    const uint32_t cd_lo = __builtin_amdgcn_perm(d, c, 0x05010400u);  // c0 d0 c1 d1
    o[0][w] = __builtin_amdgcn_perm(cd_lo, ab_lo, 0x05040100u);       // a0 b0 c0 d0
    if constexpr (M > 1) o[1][w] = __builtin_amdgcn_perm(cd_lo, ab_lo, 0x07060302u);
    if constexpr (M > 2) {
      const uint32_t ab_hi = __builtin_amdgcn_perm(b, a, 0x07030602u);  // a2 b2 a3 b3
      const uint32_t cd_hi = __builtin_amdgcn_perm(d, c, 0x07030602u);
      o[2][w] = __builtin_amdgcn_perm(cd_hi, ab_hi, 0x05040100u);
      if constexpr (M > 3) o[3][w] = __builtin_amdgcn_perm(cd_hi, ab_hi, 0x07060302u);
    }
  }
}

#ifndef CFSEC_LDS_LOOKAHEAD
#define CFSEC_LDS_LOOKAHEAD 4
#endif
// Lookups in flight: the 8 reads of word step s + P are issued before word step s is consumed
// (a step = one dword of one row's piece), so a wave keeps ~8P reads outstanding instead of
// draining its LDS queue after every few (lgkmcnt counts to 15).  P = 0: each step's 8 reads, then
// their use.  The 16-byte entries take P = 0 by default: P = 1 holds 64 VGPRs of entries.
#ifndef CFSEC_LDS_PIPE
#define CFSEC_LDS_PIPE 1
#endif
#ifndef CFSEC_LDS_PIPE_W
#define CFSEC_LDS_PIPE_W 0
#endif
// Output rows' checksums from the 5-bit tables (35 conflict-free reads per 16-byte piece, the
// register jump included) instead of E_0's nibble words + the jump (32 + 7).  Bit 0: the 8-byte-entry
// kernels (m <= 4), bit 1: the 16-byte-entry kernels.
#ifndef CFSEC_LDS_OUT5
#define CFSEC_LDS_OUT5 0
#endif
template <int M>
constexpr bool lds_out5() {
  return (CFSEC_LDS_OUT5 >> (lds_ew(M) == 2 ? 0 : 1)) & 1;
}

template <int K, int M, bool CIN>
__device__ __forceinline__ void crc_tile_lds(uint64_t len, const char* E, const uint32_t* ft, const uint32_t* rt,
                                             const uint8_t* const (&row)[K + M], uint32_t off, bool pre, bool next,
                                             uint32_t (&x)[K][4], uint32_t (&R)[(CIN ? K : 0) + M]) {
  constexpr int RO = CIN ? K : 0;
  constexpr int D = CFSEC_LDS_LOOKAHEAD < K ? CFSEC_LDS_LOOKAHEAD : K;
  constexpr int NQ = lds_nq(M), EW = lds_ew(M), EB = 4 * EW, RB = lds_row_bytes(M);
  constexpr int P = EW == 2 ? CFSEC_LDS_PIPE : CFSEC_LDS_PIPE_W;
  uint32_t g[16][NQ];
#pragma unroll
  for (int p = 0; p < 16; ++p)
#pragma unroll
    for (int q = 0; q < NQ; ++q) g[p][q] = 0u;
  // one pipelined pass; the thread holding the shard end (or past it) loads its piece
  // byte-granular, zero-padded
  const bool full = (uint64_t)off + dev::kLaneBytes <= len;
  const uint32_t rem = full ? 16u : (off < len ? (uint32_t)(len - off) : 0u);
  const auto load = [&](int c, uint32_t o, bool f) {
    u32x4 v;
    if (f) v = dev::ld16<true>(row[c] + o);
    else v = rem ? dev::ld_tail_row(row[c] + o, rem, len) : u32x4{0u, 0u, 0u, 0u};
    x[c][0] = v.x;
    x[c][1] = v.y;
    x[c][2] = v.z;
    x[c][3] = v.w;
  };
  const auto load_ahead = [&](int c) {  // the row D after input row c
    const int j = c + D;
    if (j < K) load(j, off, full);
    else if (next) load(j - K, off + kTile, true);
  };
  if (!pre)
#pragma unroll
    for (int c = 0; c < D; ++c) load(c, off, full);
  {
    // input steps s = 4c + w: 8 entry reads each (+ the 7 register-shift reads of row c at w = 0)
    LdsEnt<EW> L[P + 1][8];
    uint32_t rs[2][kFiveFields];
    uint32_t cr0 = 0u, cr1 = 0u;
    const auto issue = [&](int s) {
      const int c = s >> 2, w = s & 3;
      if (w == 0) {
        load_ahead(c);
        if constexpr (CIN) five_word<0>(rt, R[c], rs[c & 1]);
      }
      uint32_t lo, hi;
      ent_offsets<EW>(x[c][w], lo, hi);
      const char* t = E + c * RB + 4 * w * (32 * EB);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        L[s % (P + 1)][2 * j] = ld_ent<EW>(t + j * (32 * EB) + ((lo >> (8 * j)) & 0xFFu));
        L[s % (P + 1)][2 * j + 1] = ld_ent<EW>(t + j * (32 * EB) + 16 * EB + ((hi >> (8 * j)) & 0xFFu));
      }
    };
    const auto consume = [&](int s) {
      const int c = s >> 2, w = s & 3;
      const LdsEnt<EW>(&l)[8] = L[s % (P + 1)];
      uint32_t& cr = (w & 1) ? cr1 : cr0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        cr = __builtin_amdgcn_bitop3_b32(cr, l[2 * j].w[0], l[2 * j + 1].w[0], 0x96);
#pragma unroll
        for (int q = 0; q < NQ; ++q)
          g[4 * w + j][q] = __builtin_amdgcn_bitop3_b32(g[4 * w + j][q], l[2 * j].w[1 + q], l[2 * j + 1].w[1 + q], 0x96);
      }
      if (w == 3) {
        if constexpr (CIN) {
          const uint32_t(&t)[kFiveFields] = rs[c & 1];
          R[c] = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(cr0, cr1, t[0], 0x96),
                                             __builtin_amdgcn_bitop3_b32(t[1], t[2], t[3], 0x96),
                                             __builtin_amdgcn_bitop3_b32(t[4], t[5], t[6], 0x96), 0x96);
          asm volatile("" : "+v"(R[c]));  // computed here, not sunk to its next use (the reads would stay live)
        }
        cr0 = cr1 = 0u;
      }
#pragma unroll
      for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int q = 0; q < NQ; ++q) asm volatile("" : "+v"(g[4 * w + p][q]));
    };
#pragma unroll
    for (int s = 0; s < P && s < 4 * K; ++s) issue(s);
#pragma clang loop unroll(full)
    for (int s = 0; s < 4 * K; ++s) {
      if (s + P < 4 * K) issue(s + P);
      __builtin_amdgcn_sched_barrier(0);
      consume(s);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // output rows, one quad of the byte-transposed accumulators at a time: transposed back, stored,
  // checksummed through the CRC words of E_0 (output steps s = 4r + w: 8 ds_read_b32 each)
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    constexpr int kLast = M - 4 * (NQ - 1);
    uint32_t gq[16];
#pragma unroll
    for (int p = 0; p < 16; ++p) gq[p] = g[p][q];
    uint32_t o[4][4];
    untranspose<4>(gq, o);
    const int mq = q + 1 < NQ ? 4 : kLast;  // rows of this quad
    if (full) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (r < mq)
          dev::st16_out<true>(const_cast<uint8_t*>(row[K + 4 * q + r]) + off, u32x4{o[r][0], o[r][1], o[r][2], o[r][3]});
    } else if (rem) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (r < mq)
          dev::st_tail(const_cast<uint8_t*>(row[K + 4 * q + r]) + off, u32x4{o[r][0], o[r][1], o[r][2], o[r][3]}, rem);
    }
    if constexpr (lds_out5<M>()) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (r < mq) {
          R[RO + 4 * q + r] = crc_step5(ft, R[RO + 4 * q + r], o[r]);
          asm volatile("" : "+v"(R[RO + 4 * q + r]));
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      continue;
    }
    uint32_t L[P + 1][8];
    uint32_t rs[4][kFiveFields];
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (r < mq) five_word<0>(rt, R[RO + 4 * q + r], rs[r]);
    uint32_t cr0 = 0u, cr1 = 0u;
    const int ns = 4 * mq;
    const auto issue = [&](int s) {
      const int r = s >> 2, w = s & 3;
      uint32_t lo, hi;
      ent_offsets<EW>(o[r][w], lo, hi);
      const char* t = E + 4 * w * (32 * EB);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        L[s % (P + 1)][2 * j] = *reinterpret_cast<const uint32_t*>(t + j * (32 * EB) + ((lo >> (8 * j)) & 0xFFu));
        L[s % (P + 1)][2 * j + 1] =
            *reinterpret_cast<const uint32_t*>(t + j * (32 * EB) + 16 * EB + ((hi >> (8 * j)) & 0xFFu));
      }
    };
    const auto consume = [&](int s) {
      const int r = s >> 2, w = s & 3;
      const uint32_t(&l)[8] = L[s % (P + 1)];
      uint32_t& cr = (w & 1) ? cr1 : cr0;
#pragma unroll
      for (int j = 0; j < 4; ++j) cr = __builtin_amdgcn_bitop3_b32(cr, l[2 * j], l[2 * j + 1], 0x96);
      if (w == 3) {
        const uint32_t(&t)[kFiveFields] = rs[r];
        R[RO + 4 * q + r] = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(cr0, cr1, t[0], 0x96),
                                                        __builtin_amdgcn_bitop3_b32(t[1], t[2], t[3], 0x96),
                                                        __builtin_amdgcn_bitop3_b32(t[4], t[5], t[6], 0x96), 0x96);
        asm volatile("" : "+v"(R[RO + 4 * q + r]));
        cr0 = cr1 = 0u;
      }
    };
#pragma unroll
    for (int s = 0; s < P && s < 16; ++s)
      if (s < ns) issue(s);
#pragma clang loop unroll(full)
    for (int s = 0; s < 16; ++s) {
      if (s < ns) {
        if (s + P < ns) issue(s + P);
        __builtin_amdgcn_sched_barrier(0);
        consume(s);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
}

// V: 256-thread virtual groups per workgroup, each an independent run of tiles with its own
// epilogue; they share one copy of E (the LDS, not the registers, bounds the waves per CU).
#ifndef CFSEC_LDS_V
#define CFSEC_LDS_V 1
#endif
#ifndef CFSEC_LDS_WPE
#define CFSEC_LDS_WPE 3
#endif
constexpr int kLdsV = CFSEC_LDS_V;
template <int K, int M, bool CIN>
__global__ __launch_bounds__(256 * kLdsV) __attribute__((amdgpu_waves_per_eu(CFSEC_LDS_WPE, 8))) void gf_crc_lds_kernel(
    const GfCrcArgs a) {
  static_assert(M >= 1 && M <= 12, "an entry holds at most 12 products");
  constexpr int NR = (CIN ? K : 0) + M;
  constexpr int NT = 256 * kLdsV;
  constexpr int NQ = lds_nq(M), EW = lds_ew(M);
  __shared__ u32x4 E[K * lds_row_bytes(M) / 16];
  constexpr bool kO5 = lds_out5<M>();
  constexpr int kFtWords = (kO5 ? 5 : 1) * kFiveFields * 32, kGfWords = K * 32 * NQ;
  // the register word's 5-bit tables Q(4, .) (kO5: all five words' tables, Q(4, .) last; the product
  // words gfw, needed only while E is built, then live in the same words, so E_c + tables stay
  // within a third of the LDS)
  constexpr bool kShare = kO5 && kGfWords <= kFtWords;
  __shared__ uint32_t ft[kFtWords];
  __shared__ uint32_t gfw_own[kShare ? 1 : kGfWords];
  uint32_t* gfw = kShare ? ft : gfw_own;
  const uint32_t* rt = ft + (kO5 ? 4 * kFiveFields * 32 : 0);
  __shared__ uint32_t red[kLdsV][4][NR];
  // gfw[(c * 32 + h * 16 + n) * NQ + q]: the products of input row c's coefficients of outputs
  // 4q .. 4q + 3 with n << 4h
  for (int i = threadIdx.x; i < K * 32 * NQ; i += NT) {
    const int q = i % NQ, e = i / NQ, c = e >> 5;
    const uint32_t v = (uint32_t)(e & 15) << (4 * ((e >> 4) & 1));
    uint32_t w = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b)
      if (4 * q + b < M) w |= gf_mul_dev(a.coef[(4 * q + b) * K + c], v) << (8 * b);
    gfw[i] = w;
  }
  if constexpr (!kShare)
    for (int i = threadIdx.x; i < kFtWords; i += NT)
      ft[i] = a.tabs[kByteTabWords + kNibTabWords + (kO5 ? 0 : 4 * kFiveFields * 32) + i];
  __syncthreads();
  // E_c[q][n] (q = 2p + h) = (N_q[n], gfw[c][h][n][..]); N_q are the device block's nibble tables
  // (entry i & 511 of E_c takes N word i & 511: a thread meets at most two of them)
  const uint32_t* nt = a.tabs + kByteTabWords;
  const uint32_t nA = nt[threadIdx.x & 511], nB = nt[(threadIdx.x + 256) & 511];
  uint32_t* Ew = reinterpret_cast<uint32_t*>(E);
  for (int i = threadIdx.x; i < K * 512; i += NT) {
    const int c = i >> 9, q = (i >> 4) & 31, n = i & 15;
    const uint32_t* pw = gfw + (c * 32 + (q & 1) * 16 + n) * NQ;
    uint32_t* dst = Ew + (size_t)i * EW;
    dst[0] = (i & 511) == (int)(threadIdx.x & 511) ? nA : nB;
#pragma unroll
    for (int w = 1; w < EW; ++w) dst[w] = w - 1 < NQ ? pw[w - 1] : 0u;
  }
  __syncthreads();
  if constexpr (kShare) {
    for (int i = threadIdx.x; i < kFtWords; i += NT) ft[i] = a.tabs[kByteTabWords + kNibTabWords + i];
    __syncthreads();
  }

  const uint32_t vg = threadIdx.x >> 8, tid = threadIdx.x & 255;
  const uint32_t g = blockIdx.x * kLdsV + vg, stripe = blockIdx.y;
  const size_t ts = a.sstride ? 0 : (size_t)stripe;
  const int64_t sbase = (int64_t)stripe * a.sstride;
  const uint8_t* row[K + M];
#pragma unroll
  for (int c = 0; c < K; ++c) row[c] = a.ptr[ts * K + c] + sbase;
#pragma unroll
  for (int r = 0; r < M; ++r) row[K + r] = a.ptr[(size_t)a.tab * K + ts * M + r] + sbase;
  uint32_t R[NR];
#pragma unroll
  for (int i = 0; i < NR; ++i) R[i] = 0u;
  const uint32_t t0 = g * a.tpw;
  const uint32_t t1 = min(t0 + a.tpw, a.tiles);
  const uint32_t lanepos = tid * dev::kLaneBytes;
  uint32_t x[K][4];
  bool pre = false;
  for (uint32_t t = t0; t < t1; ++t) {
    const uint32_t off = t * kTile + lanepos;
    const bool next = t + 1 < t1 && (uint64_t)off + kTile + dev::kLaneBytes <= a.len;
    crc_tile_lds<K, M, CIN>(a.len, reinterpret_cast<const char*>(E), ft, rt, row, off, pre, next, x, R);
    pre = next && (uint64_t)off + dev::kLaneBytes <= a.len;
  }
  crc_epilogue<K, NR, CIN>(a, R, red[vg], g, stripe, tid, t0 < a.tiles);
}

// Launch gf_crc_kernel<K, m, CIN> (instantiated for m = 1..6 in gf_crc_k<K>.hip); dy: the dyadic
// block size of the product (4: m = 4, K a multiple of 4; 2: K = m = 6; 0: plain); dy = -1: the
// lookup-product kernel gf_crc_lds_kernel (m <= 4; K = 6, m = 12 with the inputs checksummed).
template <int K, bool CIN>
hipError_t launch_crc_k(int m, const GfCrcArgs& a, dim3 grid, hipStream_t st, int dy) {
  if (dy == -1) {
    if constexpr (K > 16) {
      return hipErrorInvalidValue;  // E would pass 64 KiB
    } else {
      switch (m) {
        case 1: hipLaunchKernelGGL((gf_crc_lds_kernel<K, 1, CIN>), grid, dim3(256 * kLdsV), 0, st, a); break;
        case 2: hipLaunchKernelGGL((gf_crc_lds_kernel<K, 2, CIN>), grid, dim3(256 * kLdsV), 0, st, a); break;
        case 3: hipLaunchKernelGGL((gf_crc_lds_kernel<K, 3, CIN>), grid, dim3(256 * kLdsV), 0, st, a); break;
        case 4: hipLaunchKernelGGL((gf_crc_lds_kernel<K, 4, CIN>), grid, dim3(256 * kLdsV), 0, st, a); break;
        case 12:
          if constexpr (K == 6 && CIN) {  // EC6P10L2's fused LRC encode + its 18 checksums
            hipLaunchKernelGGL((gf_crc_lds_kernel<K, 12, CIN>), grid, dim3(256 * kLdsV), 0, st, a);
            break;
          }
          return hipErrorInvalidValue;
        default: return hipErrorInvalidValue;
      }
      return hipGetLastError();
    }
  }
  if constexpr (K % 4 == 0) {
    if (dy == 4 && m == 4) {
      hipLaunchKernelGGL((gf_crc_kernel<K, 4, CIN, 4>), grid, dim3(256), 0, st, a);
      return hipGetLastError();
    }
  }
  if constexpr (K == 6) {
    if (dy == 2 && m == 6) {
      hipLaunchKernelGGL((gf_crc_kernel<K, 6, CIN, 2>), grid, dim3(256), 0, st, a);
      return hipGetLastError();
    }
    if constexpr (CIN) {
      if (dy == 2 && m == 12) {  // EC6P10L2 fused encode (every shard checksummed): 10 dyadic + 2 local rows
        hipLaunchKernelGGL((gf_crc_kernel<K, 12, CIN, 2, 2>), grid, dim3(256), 0, st, a);
        return hipGetLastError();
      }
    }
  }
  if (dy) return hipErrorInvalidValue;
  switch (m) {
#define CFSEC_CRC_CASE(MV)                                                                       \
  case MV:                                                                                       \
    hipLaunchKernelGGL((gf_crc_kernel<K, MV, CIN, 0>), grid, dim3(256), 0, st, a);           \
    break;
    CFSEC_CRC_CASE(1) CFSEC_CRC_CASE(2) CFSEC_CRC_CASE(3) CFSEC_CRC_CASE(4) CFSEC_CRC_CASE(5)
    CFSEC_CRC_CASE(6)
#undef CFSEC_CRC_CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace crcdev

// gf_crc.hip: the lookup tables (kTabWords + kBasisWords + kShiftWords) on the current device, uploaded once
// per device; x^e mod P for any integer e (negative: powers of x^-1).
hipError_t crc_device_tables(const uint32_t** out);
uint32_t crc_xpow(int64_t e);
uint32_t crc_mulmod(uint32_t a, uint32_t b);  // a * b mod P

namespace crcdev {

// Workgroups of gf_crc_lds_kernel<K, m, CIN> resident per CU (its LDS table bounds them), 0 if none.
template <int K, bool CIN>
int lds_blocks_per_cu(int m) {
  if constexpr (K > 16) {
    return 0;
  } else {
    const void* f = nullptr;
    switch (m) {
      case 1: f = reinterpret_cast<const void*>(&gf_crc_lds_kernel<K, 1, CIN>); break;
      case 2: f = reinterpret_cast<const void*>(&gf_crc_lds_kernel<K, 2, CIN>); break;
      case 3: f = reinterpret_cast<const void*>(&gf_crc_lds_kernel<K, 3, CIN>); break;
      case 4: f = reinterpret_cast<const void*>(&gf_crc_lds_kernel<K, 4, CIN>); break;
      case 12:
        if constexpr (K == 6 && CIN) {
          f = reinterpret_cast<const void*>(&gf_crc_lds_kernel<K, 12, CIN>);
          break;
        }
        return 0;
      default: return 0;
    }
    int n = 0;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, f, 256 * kLdsV, 0) == hipSuccess ? n : 0;
  }
}

#define CFSEC_CRC_EXTERN(K)                                                                         \
  extern template hipError_t launch_crc_k<K, true>(int, const GfCrcArgs&, dim3, hipStream_t, int);  \
  extern template hipError_t launch_crc_k<K, false>(int, const GfCrcArgs&, dim3, hipStream_t, int); \
  extern template int lds_blocks_per_cu<K, true>(int);                                              \
  extern template int lds_blocks_per_cu<K, false>(int);

}  // namespace crcdev
}  // namespace cfsec

#define CFSEC_CRC_INSTANTIATE(K)                                                                     \
  namespace cfsec {                                                                                  \
  namespace crcdev {                                                                                 \
  template hipError_t launch_crc_k<K, true>(int, const GfCrcArgs&, dim3, hipStream_t, int);        \
  template hipError_t launch_crc_k<K, false>(int, const GfCrcArgs&, dim3, hipStream_t, int);       \
  template int lds_blocks_per_cu<K, true>(int);                                                      \
  template int lds_blocks_per_cu<K, false>(int);                                                     \
  }                                                                                                  \
  }
