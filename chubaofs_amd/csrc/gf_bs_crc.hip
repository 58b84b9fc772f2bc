// gf_bs_crc.hip -- fused encode + crc32.ChecksumIEEE of every shard on the bit-sliced networks
// (round 6): EC6P10L2's fused LRC encode with all 18 checksums (C4's put; access checksums every shard
// right after Encode, blobstore/access/stream_put.go:249-253) and EC12P4's encode with its 16.
//
// The lookup-product kernel (gf_crc.hpp gf_crc_lds_kernel) gets the products and the input rows'
// checksums from one LDS read per nibble but pays a second round of lookups for every output row's
// checksum: for C4 the output rows are half of its LDS cycles and it is LDS-bound at 0.39 of 8 TB/s.
// Here the product is the bit-sliced XOR network (gf_bitslice.hpp: no lookups at all) and every
// checksum is taken from the bit planes the network already holds:
//
//   A lane's 32 bytes of a row (bytes 16 l .. and 1024 + 16 l .. of a 2 KiB column tile) become 8
//   plane words (bs_transpose8: bit 8q + i of plane j = bit j of chunk byte 4i + q).  The CRC is
//   GF(2)-linear in those 256 bits, so the lane's term f(0, a) * x^(8 * 1024) ^ f(0, b) is the XOR
//   of 56 lookups: each plane word cut into 5-bit fields (bits 0, 5, ..., 25, then 30-31), table
//   (j, f) holding the images of field f of plane j -- 32-word tables, conflict-free for ds_read_b32
//   (a lane group's addresses fall in 32 distinct banks or broadcast).  The input planes come from
//   the transposes the network needs anyway, the output planes are its output before the transpose
//   back; no row is re-read and no product byte is looked up.
//
// Work split: each wave owns one block of consecutive 2 KiB column tiles (possibly crossing stripe
// ends).  Per checksummed row a lane keeps a Horner register R <- shift(R, 2048) ^ term (the jump
// from the register's 5-bit tables, 7 lookups); where the block or a stripe ends (a segment), each
// lane moves R to the tile's end with its own 32-column basis (shift by 16 (63 - l) bytes), the wave
// XOR-reduces, lane r takes row r's word to the row's end (x^(8 (2048 (tps - 1 - c) - pad)), pad the
// zero-padded bytes of a partial last tile -- negative exponents are powers of x^-1) and XORs it into
// the row's checksum word; the segment that starts at a row's first byte also folds in
// shift(~0, S) ^ ~0, so the words end as ChecksumIEEE with no finalize pass.
//
// Rows may start at any byte (the batch seam hands over shards at odd offsets): unaligned 16-byte
// register loads, no LDS-DMA.  A stripe's partial last tile takes byte-granular tail loads and stores.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <type_traits>
#include <vector>

#include "bs_net_ec12p4.hpp"
#include "bs_net_ec6p10l2.hpp"
#include "gf256.hpp"
#include "gf_bitslice.hpp"
#include "gf_launch.hpp"

namespace cfsec {

uint32_t crc_xpow(int64_t e);                 // gf_crc.hip: x^e mod P (e < 0: powers of x^-1)
uint32_t crc_mulmod(uint32_t a, uint32_t b);  // a * b mod P (reflected)

namespace {

using dev::u32x4;
constexpr int kBcWaves = 4;       // waves per workgroup (tables shared by the workgroup)
constexpr int kBcPtr = 96;        // row pointers per launch (explicit tables: 96 / (k + m) stripes)
constexpr int kBcFields = 7;      // 5-bit fields of a word: bits 0, 5, ..., 25, then 30-31
constexpr int kBcPlaneTabs = 8 * kBcFields;       // plane j, field f: table j * 7 + f
constexpr int kBcJump = kBcPlaneTabs;             // 7 tables: the register moved 2048 bytes on
constexpr int kBcTabs = kBcPlaneTabs + kBcFields;  // 63 x 32 words
// The plane-residue form (bc_w_kernel): 4 table sets of the bit-0 plane's images (set q moved
// 2048 (3 - q) bytes on), the register moved 8192 bytes on, the lane tree's 6 levels (16 * 2^k bytes)
constexpr int kBwSets = 4;
constexpr int kBwJump = kBwSets * kBcFields, kBwTree = kBwJump + kBcFields;
constexpr int kBwTabs = kBwTree + 6 * kBcFields;  // 77 x 32 words, after the kBcTabs of the per-row form
constexpr int kBcPow = 64;        // tile-power tables: x^(8 * 2048 * i * 64^d) for d = 0, 1, 2
constexpr uint32_t kBcPoly = 0xEDB88320u;
constexpr uint64_t kBcTile = 2048;

struct __attribute__((aligned(16))) BcArgs {
  uint64_t len;          // bytes per row
  int64_t sstride;       // affine batch: stripe s's row i at ptr[i] + s * sstride (0: explicit table)
  uint32_t tps, ntiles;  // 2 KiB column tiles per stripe (the last one may be partial), in the launch
  uint32_t tab, crc_stride;
  uint32_t fin, pad0;    // shift(~0, len) ^ ~0
  uint32_t* crc;         // [stripe][crc_stride] checksum words (XOR-accumulated)
  const uint32_t* tabs;  // kBcTabs x 32 words
  const uint32_t* lbasis;  // lane l: the 32 columns of the multiply by x^(8 * 16 * (63 - l))
  uint8_t slot[32];      // checksum word of kernel row i (inputs, then outputs)
  // tile j's end to the row's end is x^(8 (2048 e - pad)), e = tps - 1 - j:
  // pw[0][e % 64] (pad folded in) * pw[1][(e / 64) % 64] * pw[2][e / 4096]
  uint32_t pw[3][kBcPow];
  uint32_t negq[kBwSets];  // the plane-residue form: x^(-8 * 2048 * (3 - q)), a segment ending at set q
  uint32_t* scr;           // the plane-residue form: [stripe][8 k] residues at the row end (XOR-accumulated)
  const uint8_t* ptr[kBcPtr];  // [tab * k inputs][tab * m outputs] (affine: tab = 1)
};
static_assert(sizeof(BcArgs) <= 3584, "kernel argument block below 4 KiB");

__device__ __forceinline__ uint32_t bc_x3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// XOR of the 7 lookups of word v's 5-bit fields in tables tb[f * 32] (gf_crc.hpp five_word's masked
// copies: each v_bfe_u32 yields the byte offset 4 * field)
__device__ __forceinline__ uint32_t bc_five7(const uint32_t* tb, uint32_t v) {
  uint32_t e = v & 0xC1F07C00u, o = v & 0x3E0F83E0u;
  asm volatile("" : "+v"(e), "+v"(o));
  const uint32_t off[7] = {(v << 2) & 0x7Cu,           __builtin_amdgcn_ubfe(o, 3, 7),  __builtin_amdgcn_ubfe(e, 8, 7),
                           __builtin_amdgcn_ubfe(o, 13, 7), __builtin_amdgcn_ubfe(e, 18, 7), __builtin_amdgcn_ubfe(o, 23, 7),
                           __builtin_amdgcn_ubfe(e, 28, 4)};
  uint32_t t[7];
#pragma unroll
  for (int f = 0; f < 7; ++f)
    t[f] = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(tb + f * 32) + off[f]);
  return bc_x3(bc_x3(t[0], t[1], t[2]), bc_x3(t[3], t[4], t[5]), t[6]);
}

#ifndef CFSEC_BW_WPE
#define CFSEC_BW_WPE 2  // waves per SIMD the plane-residue form is compiled for (its 48 registers + the network's)
#endif
#ifndef CFSEC_BC_PROBE
#define CFSEC_BC_PROBE 0  // timing probes only (wrong words): bit 0 no input-row terms, bit 1 no output-row terms
#endif

// The lane's term of a row from its 8 planes p: 56 lookups, BC_PL planes' worth in flight at a time
#ifndef CFSEC_BC_PL
#define CFSEC_BC_PL 2
#endif
__device__ __forceinline__ uint32_t bc_planes(const uint32_t* tb, const uint32_t (&p)[8]) {
  uint32_t u = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    u ^= bc_five7(tb + j * kBcFields * 32, p[j]);
    asm volatile("" : "+v"(u));  // XOR-ed here: sunk to the row's next use, the lookups' words stay live (spills)
    if ((j + 1) % CFSEC_BC_PL == 0) __builtin_amdgcn_sched_barrier(0);
  }
  return u;
}

// a * b mod P (reflected: bit 31 = x^0)
__device__ __forceinline__ uint32_t bc_mulmod(uint32_t a, uint32_t b) {
  uint32_t p = 0;
#pragma unroll
  for (int i = 31; i >= 0; --i) {
    p ^= (a >> i & 1u) ? b : 0u;
    b = (b >> 1) ^ ((b & 1u) ? kBcPoly : 0u);
  }
  return p;
}

// A lane's 16 bytes of a row at byte po: whole, the row's last partial piece, or past the end (zeros)
__device__ __forceinline__ u32x4 bc_ld(const uint8_t* row, uint64_t po, uint64_t len) {
  if (po + 16 <= len) return dev::ld16<true>(row + po);
  if (po < len) return dev::ld_tail_row(row + po, (size_t)(len - po), len);
  return u32x4{0u, 0u, 0u, 0u};
}
__device__ __forceinline__ void bc_st(uint8_t* row, uint64_t po, uint64_t len, u32x4 v) {
  if (po + 16 <= len) dev::st16<true>(row + po, v);
  else if (po < len) dev::st_tail(row + po, v, (size_t)(len - po));
}

template <class Net, int M>
__global__ __launch_bounds__(64 * kBcWaves) __attribute__((amdgpu_waves_per_eu(3, 3))) void gf_bs_crc_kernel(
    const BcArgs a) {
  constexpr int K = Net::K;
  constexpr int NR = K + M;  // checksummed rows: the inputs, then the outputs
  static_assert(NR <= 32, "one lane per row's word");
  __shared__ uint32_t tb[kBcTabs * 32];
  __shared__ uint32_t slot[32];  // the rows' word offsets, indexed per lane at the segment ends
  for (uint32_t i = threadIdx.x; i < kBcTabs * 8; i += blockDim.x)
    reinterpret_cast<u32x4*>(tb)[i] = reinterpret_cast<const u32x4*>(a.tabs)[i];
  if (threadIdx.x == 0)  // constant indices: a lane-indexed read of the argument block would copy it to scratch
#pragma unroll
    for (int i = 0; i < NR; ++i) slot[i] = a.slot[i];
  __syncthreads();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * kBcWaves, wid = blockIdx.x * kBcWaves + wave;
  const uint32_t t0 = (uint32_t)((uint64_t)a.ntiles * wid / nw), t1 = (uint32_t)((uint64_t)a.ntiles * (wid + 1) / nw);
  if (t0 >= t1) return;  // no barrier below
  const uint64_t len = a.len;
  const uint32_t tps = a.tps;
  const auto in_row = [&](uint32_t s, int i) -> const uint8_t* {
    return a.sstride ? a.ptr[i] + (int64_t)s * a.sstride : a.ptr[(size_t)s * K + i];
  };
  const auto out_row = [&](uint32_t s, int r) -> uint8_t* {
    return const_cast<uint8_t*>(a.sstride ? a.ptr[K + r] + (int64_t)s * a.sstride
                                          : a.ptr[(size_t)a.tab * K + (size_t)s * M + r]);
  };
  uint32_t R[NR];
#pragma unroll
  for (int i = 0; i < NR; ++i) R[i] = 0u;
  bool first = t0 % tps == 0;  // the current segment starts at its row's first byte
  // one column tile: loads, transposes, the inputs' terms, the network, the outputs' terms and stores
  // (FULL: every piece in bounds -- straight-line code; else the stripe's partial last tile)
  const auto tile = [&](uint32_t s, uint64_t po, auto full_tag) {
    constexpr bool FULL = decltype(full_tag)::value;
    uint32_t x[8 * K];
#pragma unroll
    for (int i = 0; i < K; ++i) {
      const uint8_t* p = in_row(s, i);
      const u32x4 lo = FULL ? dev::ld16<true>(p + po) : bc_ld(p, po, len),
                  hi = FULL ? dev::ld16<true>(p + po + 1024) : bc_ld(p, po + 1024, len);
      x[8 * i] = lo.x; x[8 * i + 1] = lo.y; x[8 * i + 2] = lo.z; x[8 * i + 3] = lo.w;
      x[8 * i + 4] = hi.x; x[8 * i + 5] = hi.y; x[8 * i + 6] = hi.z; x[8 * i + 7] = hi.w;
    }
#pragma unroll
    for (int i = 0; i < K; ++i) {
      dev::bs_transpose8(&x[8 * i]);
      uint32_t(&pl)[8] = *reinterpret_cast<uint32_t(*)[8]>(&x[8 * i]);
      if constexpr (!(CFSEC_BC_PROBE & 1)) R[i] ^= bc_planes(tb, pl);
      asm volatile("" : "+v"(R[i]));
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (Net::Paired) dev::bs_pair_basis<K>(x);
    __builtin_amdgcn_sched_barrier(0);
    Net::template net<M>(x, [&](int r, uint32_t (&o)[8]) {
      if constexpr (!(CFSEC_BC_PROBE & 2)) R[K + r] ^= bc_planes(tb, o);
      asm volatile("" : "+v"(R[K + r]));
      dev::bs_transpose8(o);
      uint8_t* p = out_row(s, r);
      if constexpr (FULL) {
        dev::st16<true>(p + po, u32x4{o[0], o[1], o[2], o[3]});
        dev::st16<true>(p + po + 1024, u32x4{o[4], o[5], o[6], o[7]});
      } else {
        bc_st(p, po, len, u32x4{o[0], o[1], o[2], o[3]});
        bc_st(p, po + 1024, len, u32x4{o[4], o[5], o[6], o[7]});
      }
    });
  };
  for (uint32_t t = t0; t < t1; ++t) {
    const uint32_t s = t / tps, c = t - s * tps;
    const uint64_t po = (uint64_t)c * kBcTile + lane * 16;
    if ((uint64_t)(c + 1) * kBcTile <= len) tile(s, po, std::true_type{});  // wave-uniform
    else tile(s, po, std::false_type{});
    if (t + 1 == t1 || c + 1 == tps) {
      // segment end: every lane's registers to the tile end, the wave's sum, lane r's row r to the
      // row end, into the row's word
      uint32_t col[32];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const u32x4 v = reinterpret_cast<const u32x4*>(a.lbasis + lane * 32)[q];
        col[4 * q] = v.x; col[4 * q + 1] = v.y; col[4 * q + 2] = v.z; col[4 * q + 3] = v.w;
      }
      uint32_t mine = 0;
#pragma unroll
      for (int i = 0; i < NR; ++i) {
        uint32_t v = 0;
#pragma unroll
        for (int b = 0; b < 32; ++b) v ^= (uint32_t)((int32_t)(R[i] << (31 - b)) >> 31) & col[b];
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) v ^= (uint32_t)__shfl_xor((int)v, d, 64);
        mine = lane == (uint32_t)i ? v : mine;
        R[i] = 0u;
      }
      const uint32_t e = tps - 1 - c;
      const uint32_t k = bc_mulmod(bc_mulmod(a.pw[0][e % kBcPow], a.pw[1][(e / kBcPow) % kBcPow]),
                                   a.pw[2][e / (kBcPow * kBcPow)]);
      uint32_t w = bc_mulmod(mine, k);
      if (first) w ^= a.fin;
      if (lane < (uint32_t)NR) atomicXor(a.crc + (size_t)s * a.crc_stride + slot[lane], w);
      first = true;  // a later segment of this wave starts a stripe
    } else {
#pragma unroll
      for (int i = 0; i < NR; ++i) R[i] = bc_five7(tb + kBcJump * 32, R[i]);
    }
  }
}

// ---- the plane-residue form (EC6P10L2's fused LRC encode: 12 outputs over 6 inputs) ----
// Every output row's checksum is a GF(2)-linear function of the input rows' bit planes: with
// W(c, j) = f(0, the row whose byte p is bit j of data row c's byte p), bit t of a byte at position p
// contributes x^-t times what bit 0 there does, and bit t of g * d = XOR over j of bit t of g * 2^j
// times bit j of d, so
//     raw crc(output r) = XOR over c, j of W(c, j) * P(r, c, j),  P = XOR over t of [bit t of g_rc * 2^j] x^-t
//     raw crc(input c)  = XOR over j of W(c, j) * x^-j.
// So the kernel keeps the 8 k plane residues W (48 Horner registers for k = 6: 336 lookups per tile
// instead of the per-row form's 18 x 56) and no output row is looked up at all.  Per lane, tiles
// c = 4g .. 4g + 3 take table set c % 4 (their images pre-moved to the group's last tile), so the
// registers jump once per 4 tiles.  At a segment end the 64 lanes fold by recursive halving (lane
// pairs, then quads, ...: each step keeps half the registers, 63 register-shifts by the tree tables
// in all, instead of a 32-column basis per register), the lane holding residue i moves it to the row
// end and XORs it into scr[stripe][i]; bc_w_combine then forms the k + m checksums per stripe.
template <class Net, int M>
__global__ __launch_bounds__(64 * kBcWaves) __attribute__((amdgpu_waves_per_eu(CFSEC_BW_WPE, 3))) void bc_w_kernel(
    const BcArgs a) {
  constexpr int K = Net::K;
  constexpr int NW = 8 * K;  // plane residues
  static_assert(NW <= 64, "one lane per residue after the fold");
  __shared__ uint32_t tb[kBwTabs * 32];
  for (uint32_t i = threadIdx.x; i < kBwTabs * 8; i += blockDim.x)
    reinterpret_cast<u32x4*>(tb)[i] = reinterpret_cast<const u32x4*>(a.tabs + kBcTabs * 32)[i];
  __syncthreads();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * kBcWaves, wid = blockIdx.x * kBcWaves + wave;
  const uint32_t t0 = (uint32_t)((uint64_t)a.ntiles * wid / nw), t1 = (uint32_t)((uint64_t)a.ntiles * (wid + 1) / nw);
  if (t0 >= t1) return;  // no barrier below
  const uint64_t len = a.len;
  const uint32_t tps = a.tps;
  const auto in_row = [&](uint32_t s, int i) -> const uint8_t* {
    return a.sstride ? a.ptr[i] + (int64_t)s * a.sstride : a.ptr[(size_t)s * K + i];
  };
  const auto out_row = [&](uint32_t s, int r) -> uint8_t* {
    return const_cast<uint8_t*>(a.sstride ? a.ptr[K + r] + (int64_t)s * a.sstride
                                          : a.ptr[(size_t)a.tab * K + (size_t)s * M + r]);
  };
  uint32_t W[NW];
#pragma unroll
  for (int i = 0; i < NW; ++i) W[i] = 0u;
  const auto tile = [&](uint32_t s, uint64_t po, const uint32_t* tq, auto full_tag) {
    constexpr bool FULL = decltype(full_tag)::value;
    uint32_t x[8 * K];
#pragma unroll
    for (int i = 0; i < K; ++i) {
      const uint8_t* p = in_row(s, i);
      const u32x4 lo = FULL ? dev::ld16<true>(p + po) : bc_ld(p, po, len),
                  hi = FULL ? dev::ld16<true>(p + po + 1024) : bc_ld(p, po + 1024, len);
      x[8 * i] = lo.x; x[8 * i + 1] = lo.y; x[8 * i + 2] = lo.z; x[8 * i + 3] = lo.w;
      x[8 * i + 4] = hi.x; x[8 * i + 5] = hi.y; x[8 * i + 6] = hi.z; x[8 * i + 7] = hi.w;
    }
#pragma unroll
    for (int i = 0; i < K; ++i) {
      dev::bs_transpose8(&x[8 * i]);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        W[8 * i + j] ^= bc_five7(tq, x[8 * i + j]);
        asm volatile("" : "+v"(W[8 * i + j]));
        if (j & 1) __builtin_amdgcn_sched_barrier(0);
      }
    }
    if constexpr (Net::Paired) dev::bs_pair_basis<K>(x);
    __builtin_amdgcn_sched_barrier(0);
    Net::template net<M>(x, [&](int r, uint32_t (&o)[8]) {
      dev::bs_transpose8(o);
      uint8_t* p = out_row(s, r);
      if constexpr (FULL) {
        dev::st16<true>(p + po, u32x4{o[0], o[1], o[2], o[3]});
        dev::st16<true>(p + po + 1024, u32x4{o[4], o[5], o[6], o[7]});
      } else {
        bc_st(p, po, len, u32x4{o[0], o[1], o[2], o[3]});
        bc_st(p, po + 1024, len, u32x4{o[4], o[5], o[6], o[7]});
      }
    });
  };
  for (uint32_t t = t0; t < t1; ++t) {
    const uint32_t s = t / tps, c = t - s * tps, q = c % kBwSets;
    const uint64_t po = (uint64_t)c * kBcTile + lane * 16;
    const uint32_t* tq = tb + q * kBcFields * 32;
    if ((uint64_t)(c + 1) * kBcTile <= len) tile(s, po, tq, std::true_type{});  // wave-uniform
    else tile(s, po, tq, std::false_type{});
    if (t + 1 == t1 || c + 1 == tps) {
      // segment end: the lanes' registers folded by recursive halving -- at level k lane pairs l,
      // l ^ 2^k swap halves of their registers, and each keeps the sum of one half, the earlier
      // group's value moved 16 * 2^k bytes on -- until lane l holds residue bitrev6(l) at the tile's
      // (the group's last tile's) end
      uint32_t v[64];
#pragma unroll
      for (int i = 0; i < 64; ++i) v[i] = i < NW ? W[i] : 0u;
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        const int half = 32 >> k;
        const bool up = (lane >> k) & 1u;
#pragma unroll
        for (int i = 0; i < half; ++i) {
          const uint32_t send = up ? v[i] : v[half + i], keep = up ? v[half + i] : v[i];
          const uint32_t recv = (uint32_t)__shfl_xor((int)send, 1 << k, 64);
          const uint32_t lo = up ? recv : keep, hi = up ? keep : recv;
          v[i] = bc_five7(tb + (kBwTree + k * kBcFields) * 32, lo) ^ hi;
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      // the group's last tile's end to the row's end: x^(8 (2048 (tps - 1 - c) - pad)) x^(-8 * 2048 * (3 - q))
      const uint32_t e = tps - 1 - c;
      const uint32_t f = bc_mulmod(bc_mulmod(a.pw[0][e % kBcPow], a.pw[1][(e / kBcPow) % kBcPow]),
                                   bc_mulmod(a.pw[2][e / (kBcPow * kBcPow)], a.negq[q]));
      const uint32_t idx = __builtin_bitreverse32(lane) >> 26;
      if (idx < (uint32_t)NW) atomicXor(a.scr + (size_t)s * NW + idx, bc_mulmod(v[0], f));
#pragma unroll
      for (int i = 0; i < NW; ++i) W[i] = 0u;
    } else if (q == kBwSets - 1) {
#pragma unroll
      for (int i = 0; i < NW; ++i) W[i] = bc_five7(tb + kBwJump * 32, W[i]);
    }
  }
}

// Per stripe: row r's checksum = fin ^ XOR over i of scr[i] * P(r, i) (256 threads: the (r, i)
// products spread over them, XOR-reduced per row in LDS); poly[r * NW + i] = P(r, i)
struct BwCombineArgs {
  const uint32_t* scr;   // [stripe][nw]
  const uint32_t* poly;  // [nr][nw]
  uint32_t* crc;         // [stripe][crc_stride]
  uint32_t nw, nr, crc_stride, fin;
  uint8_t slot[32];
};
__global__ __launch_bounds__(256) void bc_w_combine(const BwCombineArgs c) {
  __shared__ uint32_t acc[32];
  const uint32_t s = blockIdx.x;
  if (threadIdx.x < 32) acc[threadIdx.x] = 0u;
  __syncthreads();
  const uint32_t n = c.nw * c.nr;
  for (uint32_t j = threadIdx.x; j < n; j += blockDim.x) {
    const uint32_t r = j / c.nw, i = j - r * c.nw;
    const uint32_t v = bc_mulmod(c.scr[(size_t)s * c.nw + i], c.poly[j]);
    if (v) atomicXor(&acc[r], v);
  }
  __syncthreads();
  if (threadIdx.x < c.nr) {
    uint32_t sl = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i)  // constant indices into the argument block
      if (threadIdx.x == (uint32_t)i) sl = c.slot[i];
    atomicXor(c.crc + (size_t)s * c.crc_stride + sl, acc[threadIdx.x] ^ c.fin);
  }
}

// ---- host side ----
uint32_t env_mask(const char* name, uint32_t dflt) {
  const char* v = std::getenv(name);
  return v && *v ? (uint32_t)std::strtoul(v, nullptr, 0) : dflt;
}
// CFSEC_BS_CRC: bit 0 EC6P10L2's fused LRC encode (6 x 12), bit 1 EC12P4 (12 x 4), bit 2 the 6 x 12
// in the per-row form instead of the plane-residue form; 0 keeps the lookup-product kernels (A/B)
#ifndef CFSEC_BS_CRC_DEFAULT
#define CFSEC_BS_CRC_DEFAULT 5
#endif
uint32_t bs_crc_mask() {
  static const uint32_t v = env_mask("CFSEC_BS_CRC", CFSEC_BS_CRC_DEFAULT);
  return v;
}

template <class Net>
bool rows_equal(const uint8_t* coef, int m) {
  const uint8_t* w = Net::rows();
  return std::memcmp(coef, w, (size_t)m * Net::K) == 0;
}

// f(0, one byte b)
uint32_t crc_byte(uint32_t b) {
  uint32_t c = b;
  for (int q = 0; q < 8; ++q) c = (c & 1u) ? (c >> 1) ^ kBcPoly : c >> 1;
  return c;
}

// The device table block: the per-row form's kBcTabs tables, then the plane-residue form's kBwTabs
std::vector<uint32_t> bc_host_tables() {
  std::vector<uint32_t> t((size_t)(kBcTabs + kBwTabs) * 32, 0u);
  // C(k, j): bit j of chunk byte k, the chunk's bytes at 0..15 and 1024..1039 of a 1040-byte span
  uint32_t C[32][8];
  for (int k = 0; k < 32; ++k) {
    const int64_t follow = k < 16 ? 1039 - k : 31 - k;
    const uint32_t sh = crc_xpow(8 * follow);
    for (int j = 0; j < 8; ++j) C[k][j] = crc_mulmod(sh, crc_byte(1u << j));
  }
  const uint32_t k2048 = crc_xpow(8 * 2048);
  for (int f = 0; f < kBcFields; ++f) {
    const int nb = f < 6 ? 5 : 2;
    for (uint32_t e = 0; e < (1u << nb); ++e) {
      for (int j = 0; j < 8; ++j) {
        uint32_t v = 0;
        for (int b = 0; b < nb; ++b)
          if (e >> b & 1u) {
            const int bit = 5 * f + b, q = bit >> 3, i = bit & 7;  // plane bit 8q + i = byte 4i + q
            v ^= C[4 * i + q][j];
          }
        t[(size_t)(j * kBcFields + f) * 32 + e] = v;
      }
      t[(size_t)(kBcJump + f) * 32 + e] = crc_mulmod(k2048, e << (5 * f));
      uint32_t* w = t.data() + (size_t)kBcTabs * 32;
      for (int q = 0; q < kBwSets; ++q)  // bit-0 plane images, moved 2048 (3 - q) bytes on
        w[(size_t)(q * kBcFields + f) * 32 + e] =
            crc_mulmod(crc_xpow(8ll * 2048 * (kBwSets - 1 - q)), t[(size_t)(0 * kBcFields + f) * 32 + e]);
      w[(size_t)(kBwJump + f) * 32 + e] = crc_mulmod(crc_xpow(8ll * 2048 * kBwSets), e << (5 * f));
      for (int k = 0; k < 6; ++k)
        w[(size_t)(kBwTree + k * kBcFields + f) * 32 + e] = crc_mulmod(crc_xpow(8ll * (16 << k)), e << (5 * f));
    }
  }
  return t;
}

// P(r, i) of the plane-residue form for a network's rows (bc_w_kernel): rows 0..k-1 the inputs
// (x^-j on their own residues), then the m outputs
template <class Net, int M>
std::vector<uint32_t> bw_host_poly() {
  constexpr int K = Net::K, NW = 8 * K;
  const GF& gf = GF::get();
  const uint8_t* rows = Net::rows();
  std::vector<uint32_t> p((size_t)(K + M) * NW, 0u);
  uint32_t xneg[8];
  for (int t = 0; t < 8; ++t) xneg[t] = crc_xpow(-t);
  for (int r = 0; r < K + M; ++r)
    for (int c = 0; c < K; ++c)
      for (int j = 0; j < 8; ++j) {
        const uint32_t prod = r < K ? (r == c ? 1u << j : 0u) : gf.mul(rows[(size_t)(r - K) * K + c], (uint8_t)(1u << j));
        uint32_t v = 0;
        for (int t = 0; t < 8; ++t)
          if (prod >> t & 1u) v ^= xneg[t];
        p[(size_t)r * NW + 8 * c + j] = v;
      }
  return p;
}

struct BcDev {
  std::mutex mu;
  uint32_t* tab = nullptr;
  uint32_t* lbasis = nullptr;
  uint32_t* poly6 = nullptr;  // bw_host_poly<BsEc6p10l2, 12>
  bool pool = false;          // the default memory pool keeps freed scratch (release threshold set)
};

hipError_t bc_device(const uint32_t** tab, const uint32_t** lbasis, const uint32_t** poly6 = nullptr) {
  static BcDev per[64];
  int d = 0;
  hipError_t e = hipGetDevice(&d);
  if (e != hipSuccess) return e;
  if (d < 0 || d >= 64) return hipErrorInvalidDevice;
  BcDev& c = per[d];
  std::lock_guard<std::mutex> lk(c.mu);
  const auto upload = [&](const std::vector<uint32_t>& h, uint32_t** out) -> hipError_t {
    uint32_t* p = nullptr;
    hipError_t r = hipMalloc(reinterpret_cast<void**>(&p), h.size() * 4);
    if (r != hipSuccess) return r;
    if ((r = hipMemcpy(p, h.data(), h.size() * 4, hipMemcpyHostToDevice)) != hipSuccess) {
      (void)hipFree(p);
      return r;
    }
    *out = p;
    return hipSuccess;
  };
  if (!c.tab && (e = upload(bc_host_tables(), &c.tab)) != hipSuccess) return e;
  if (!c.lbasis) {
    std::vector<uint32_t> h(64 * 32);
    for (int l = 0; l < 64; ++l) {
      const uint32_t k = crc_xpow(8ll * 16 * (63 - l));
      for (int b = 0; b < 32; ++b) h[(size_t)l * 32 + b] = crc_mulmod(k, 1u << b);
    }
    if ((e = upload(h, &c.lbasis)) != hipSuccess) return e;
  }
  if (poly6 && !c.poly6 && (e = upload(bw_host_poly<dev::BsEc6p10l2, 12>(), &c.poly6)) != hipSuccess) return e;
  if (poly6 && !c.pool) {  // stream-ordered scratch (hipMallocAsync) without a trip to the driver per call
    hipMemPool_t mp = nullptr;
    uint64_t keep = 64ull << 20;
    if (hipDeviceGetDefaultMemPool(&mp, d) == hipSuccess)
      (void)hipMemPoolSetAttribute(mp, hipMemPoolAttrReleaseThreshold, &keep);
    (void)hipGetLastError();
    c.pool = true;
  }
  *tab = c.tab;
  *lbasis = c.lbasis;
  if (poly6) *poly6 = c.poly6;
  return hipSuccess;
}

int64_t bc_affine_stride(const MatVecJob& job) {  // as gf_crc.hip's
  if (job.nstripes < 2) return 0;
  const auto addr = [](const void* p) { return (int64_t)(uintptr_t)p; };
  const int64_t ss = addr(job.in[job.k]) - addr(job.in[0]);
  if (ss == 0) return 0;
  for (int s = 1; s < job.nstripes; ++s) {
    for (int c = 0; c < job.k; ++c)
      if (addr(job.in[(size_t)s * job.k + c]) != addr(job.in[c]) + s * ss) return 0;
    for (int r = 0; r < job.m; ++r)
      if (addr(job.out[(size_t)s * job.m + r]) != addr(job.out[r]) + s * ss) return 0;
  }
  return ss;
}

template <class Net, int M, bool W = false>
int bc_groups() {  // resident workgroups on the device (one wave of workgroups)
  static std::mutex mu;
  static std::map<int, int> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  std::lock_guard<std::mutex> l(mu);
  auto it = cache.find(dev);
  if (it != cache.end()) return it->second;
  int per = 0, cus = 0;
  const void* f = nullptr;
  if constexpr (W) f = reinterpret_cast<const void*>(&bc_w_kernel<Net, M>);
  else f = reinterpret_cast<const void*>(&gf_bs_crc_kernel<Net, M>);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, f, 64 * kBcWaves, 0) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
    (void)hipGetLastError();
    per = 0;
  }
  const int n = per > 0 && cus > 0 ? per * cus : 768;
  cache.emplace(dev, n);
  return n;
}

template <class Net, int M>
hipError_t bc_launch(const MatVecJob& job, uint32_t* crc, int crc_stride, const int* slot, hipStream_t st) {
  constexpr int K = Net::K;
  BcArgs a{};
  hipError_t e = bc_device(&a.tabs, &a.lbasis);
  if (e != hipSuccess) return e;
  const uint64_t len = job.len;
  const uint64_t tps = (len + kBcTile - 1) / kBcTile;
  const int64_t pad = (int64_t)(tps * kBcTile - len);
  const uint32_t x1 = crc_xpow(8 * (int64_t)kBcTile), x64 = crc_xpow(8 * (int64_t)kBcTile * kBcPow),
                 x4096 = crc_xpow(8 * (int64_t)kBcTile * kBcPow * kBcPow);
  uint32_t p0 = crc_xpow(-8 * pad), p1 = 0x80000000u, p2 = 0x80000000u;
  for (int i = 0; i < kBcPow; ++i) {
    a.pw[0][i] = p0;
    a.pw[1][i] = p1;
    a.pw[2][i] = p2;
    p0 = crc_mulmod(p0, x1);
    p1 = crc_mulmod(p1, x64);
    p2 = crc_mulmod(p2, x4096);
  }
  a.len = len;
  a.tps = (uint32_t)tps;
  a.crc_stride = (uint32_t)crc_stride;
  a.fin = crc32_shift_ones((size_t)len);
  for (int i = 0; i < K + M; ++i) a.slot[i] = (uint8_t)slot[i];
  const int64_t ss = bc_affine_stride(job);
  a.sstride = ss;
  const int per = ss ? job.nstripes : kBcPtr / (K + M);
  const int groups = bc_groups<Net, M>();
  for (int s0 = 0; s0 < job.nstripes; s0 += per) {
    const int ns = std::min(per, job.nstripes - s0);
    const int tab = ss ? 1 : ns;
    a.tab = (uint32_t)tab;
    a.crc = crc + (size_t)s0 * crc_stride;
    for (int s = 0; s < tab; ++s) {
      for (int c = 0; c < K; ++c) a.ptr[s * K + c] = job.in[(size_t)(s0 + s) * K + c];
      for (int r = 0; r < M; ++r) a.ptr[tab * K + s * M + r] = job.out[(size_t)(s0 + s) * M + r];
    }
    const uint64_t nt = tps * (uint64_t)ns;
    a.ntiles = (uint32_t)nt;
    const unsigned grid = (unsigned)std::min<uint64_t>((uint64_t)groups, (nt + kBcWaves - 1) / kBcWaves);
    hipLaunchKernelGGL((gf_bs_crc_kernel<Net, M>), dim3(grid), dim3(64 * kBcWaves), 0, st, a);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  return hipSuccess;
}

// The plane-residue form: scratch residues per stripe (stream-ordered allocation), the main launches,
// one combine launch; false in *ok when the scratch cannot be had (the caller takes the per-row form)
template <class Net, int M>
hipError_t bw_launch(const MatVecJob& job, uint32_t* crc, int crc_stride, const int* slot, hipStream_t st, bool* ok) {
  constexpr int K = Net::K, NW = 8 * K;
  *ok = false;
  BcArgs a{};
  const uint32_t* poly = nullptr;
  hipError_t e = bc_device(&a.tabs, &a.lbasis, &poly);
  if (e != hipSuccess) return e;
  const size_t bytes = (size_t)job.nstripes * NW * 4;
  uint32_t* scr = nullptr;
  if (hipMallocAsync(reinterpret_cast<void**>(&scr), bytes, st) != hipSuccess || !scr) {
    (void)hipGetLastError();
    return hipSuccess;
  }
  *ok = true;
  if ((e = hipMemsetAsync(scr, 0, bytes, st)) != hipSuccess) {
    (void)hipFreeAsync(scr, st);
    return e;
  }
  const uint64_t len = job.len;
  const uint64_t tps = (len + kBcTile - 1) / kBcTile;
  const int64_t pad = (int64_t)(tps * kBcTile - len);
  const uint32_t x1 = crc_xpow(8 * (int64_t)kBcTile), x64 = crc_xpow(8 * (int64_t)kBcTile * kBcPow),
                 x4096 = crc_xpow(8 * (int64_t)kBcTile * kBcPow * kBcPow);
  uint32_t p0 = crc_xpow(-8 * pad), p1 = 0x80000000u, p2 = 0x80000000u;
  for (int i = 0; i < kBcPow; ++i) {
    a.pw[0][i] = p0;
    a.pw[1][i] = p1;
    a.pw[2][i] = p2;
    p0 = crc_mulmod(p0, x1);
    p1 = crc_mulmod(p1, x64);
    p2 = crc_mulmod(p2, x4096);
  }
  for (int q = 0; q < kBwSets; ++q) a.negq[q] = crc_xpow(-8ll * 2048 * (kBwSets - 1 - q));
  a.len = len;
  a.tps = (uint32_t)tps;
  const int64_t ss = bc_affine_stride(job);
  a.sstride = ss;
  const int per = ss ? job.nstripes : kBcPtr / (K + M);
  const int groups = bc_groups<Net, M, true>();
  for (int s0 = 0; s0 < job.nstripes && e == hipSuccess; s0 += per) {
    const int ns = std::min(per, job.nstripes - s0);
    const int tab = ss ? 1 : ns;
    a.tab = (uint32_t)tab;
    a.scr = scr + (size_t)s0 * NW;
    for (int s = 0; s < tab; ++s) {
      for (int c = 0; c < K; ++c) a.ptr[s * K + c] = job.in[(size_t)(s0 + s) * K + c];
      for (int r = 0; r < M; ++r) a.ptr[tab * K + s * M + r] = job.out[(size_t)(s0 + s) * M + r];
    }
    const uint64_t nt = tps * (uint64_t)ns;
    a.ntiles = (uint32_t)nt;
    const unsigned grid = (unsigned)std::min<uint64_t>((uint64_t)groups, (nt + kBcWaves - 1) / kBcWaves);
    hipLaunchKernelGGL((bc_w_kernel<Net, M>), dim3(grid), dim3(64 * kBcWaves), 0, st, a);
    e = hipGetLastError();
  }
  if (e == hipSuccess) {
    BwCombineArgs c{};
    c.scr = scr;
    c.poly = poly;
    c.crc = crc;
    c.nw = NW;
    c.nr = K + M;
    c.crc_stride = (uint32_t)crc_stride;
    c.fin = crc32_shift_ones((size_t)len);
    for (int i = 0; i < K + M; ++i) c.slot[i] = (uint8_t)slot[i];
    hipLaunchKernelGGL(bc_w_combine, dim3((unsigned)job.nstripes), dim3(256), 0, st, c);
    e = hipGetLastError();
  }
  const hipError_t f = hipFreeAsync(scr, st);
  return e != hipSuccess ? e : f;
}

}  // namespace

bool bs_crc_matches(int k, int m, const uint8_t* coef) {
  if (!coef) return false;
  const uint32_t mask = bs_crc_mask();
  if ((mask & 1u) && k == 6 && m == 12) return rows_equal<dev::BsEc6p10l2>(coef, 12);
  if ((mask & 2u) && k == 12 && m == 4) return rows_equal<dev::BsEc12p4>(coef, 4);
  return false;
}

hipError_t launch_bs_crc(const MatVecJob& job, uint32_t* crc, int crc_stride, const int* slot, hipStream_t st) {
  if (!crc || !slot || !bs_crc_matches(job.k, job.m, job.coef) || job.len == 0 ||
      (job.len + kBcTile - 1) / kBcTile > (uint64_t)kBcPow * kBcPow * kBcPow ||
      (job.len + kBcTile - 1) / kBcTile * (uint64_t)std::max(job.nstripes, 1) > 0xFFFFFFFFull || crc_stride > 256)
    return hipErrorInvalidValue;
  for (int i = 0; i < job.k + job.m; ++i)
    if (slot[i] < 0 || slot[i] >= crc_stride) return hipErrorInvalidValue;
  static const bool trace = env_mask("CFSEC_TRACE_CRC", 0) != 0;
  if (trace) std::fprintf(stderr, "cfsec: bs crc k=%d m=%d stripes=%d len=%llu\n", job.k, job.m, job.nstripes,
                          (unsigned long long)job.len);
  if (job.k == 6) {
    if (!(bs_crc_mask() & 4u)) {  // the plane-residue form (bit 2: the per-row form, A/B)
      bool ok = false;
      const hipError_t e = bw_launch<dev::BsEc6p10l2, 12>(job, crc, crc_stride, slot, st, &ok);
      if (ok || e != hipSuccess) return e;
    }
    return bc_launch<dev::BsEc6p10l2, 12>(job, crc, crc_stride, slot, st);
  }
  return bc_launch<dev::BsEc12p4, 4>(job, crc, crc_stride, slot, st);
}

bool bs_crc_takes(const MatVecJob& job, int crc_stride, const int* slot) {
  if (!slot || slot[0] < 0 || job.len == 0 || crc_stride > 256 || !bs_crc_matches(job.k, job.m, job.coef)) return false;
  const uint64_t tps = (job.len + kBcTile - 1) / kBcTile;
  return tps <= (uint64_t)kBcPow * kBcPow * kBcPow && tps * (uint64_t)std::max(job.nstripes, 1) <= 0xFFFFFFFFull;
}

}  // namespace cfsec
