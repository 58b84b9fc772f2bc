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
// Work split: W waves per stripe (the launch's waves over its stripes, capped at the stripe's tiles),
// wave j taking tiles j, j + W, j + 2W, ... -- neighbouring waves on neighbouring tiles.  Per checksummed
// row a lane keeps a Horner register R <- shift(R, 2048 W) ^ term (the jump from the register's 5-bit
// tables, 7 lookups, rebuilt per launch for its stride); after the wave's last tile of a stripe the 64
// lanes fold by recursive halving (lookups in the lane tree's tables), lane r holds row r's sum at the
// tile's end, takes it to the row's end (x^(8 (2048 (tps - 1 - c) - pad)), pad the zero-padded bytes of
// a partial last tile -- negative exponents are powers of x^-1) and XORs it into the row's checksum
// word; the wave holding tile 0 also folds in shift(~0, S) ^ ~0, so the words end as ChecksumIEEE with
// no finalize pass.  Measured (C4's put batch, 48 x 699,051 B, tools/c4_crc_probe.py): blocks of
// consecutive tiles per wave 195 us, this order 189 us, with the tree fold 184-186 us (a 32-column basis
// per register: 189); 1-4 tiles per wave and stripe 194-249 us (more folds); the product alone in this
// structure 156 us, in gf_bs_kernel's every-nw-th-tile order 143 us (that order leaves no run of one
// row per wave for the Horner registers).  EC12P4 with its input rows' registers in LDS (LI below, 3
// waves per SIMD): in the shape sweep 64 MiB blobs 190 us against 207 on the lookup-product kernel,
// 4 MiB blobs 194 vs 185, but in the bench's rotated batches no faster (encode_crc_roofline_frac
// 0.473-0.481 vs 0.479-0.482, the ec seam 0.463-0.466 vs 0.471-0.475: profiles/r06/bs_crc/
// bench_ec12p4_ab.txt); with the remainder tiles as tail waves (below) it won there too (0.484 -> 0.506)
// and is routed by default.  The 16 + 20 code (EC16P20 / EC16P20L2's fused encode, all 36 / 38 rows
// checksummed) had no fused form: 256 VGPRs with 79 spilled at 2 waves per SIMD, still 243.6 -> 218.5 us
// (EC16P20L2, 64 x 262,144) and 227.5 -> 206.5 us (EC16P20) against the product + separate pass
// (profiles/r06/bs_crc/shape_sweep_ec16.txt).  A plane-residue form -- the 12 output checksums as linear functions of
// the 6 input rows' 48 bit-plane residues, 3x fewer lookups -- ran at 192-211 us (2 waves per SIMD at
// 172 VGPRs) and was dropped.
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

#include "bs_net_ec10p4.hpp"
#include "bs_net_ec3p3.hpp"
#include "bs_net_ec4p4.hpp"
#include "bs_net_ec4p4l2.hpp"
#include "bs_net_ec6p3l3.hpp"
#include "bs_net_ec6p6l9.hpp"
#include "bs_net_ec6p8l10.hpp"
#include "bs_net_ec12p4.hpp"
#include "bs_net_ec12p9.hpp"
#include "bs_net_ec15p12.hpp"
#include "bs_net_ec16p20l2.hpp"
#include "bs_net_ec6p10l2.hpp"
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
constexpr int kBcTree = kBcJump + kBcFields;       // the lane tree's 6 levels: shift by 16 * 2^k bytes
constexpr int kBcTabs = kBcTree + 6 * kBcFields;   // 105 x 32 words
constexpr int kBcPow = 64;        // tile-power tables: x^(8 * 2048 * i * 64^d) for d = 0, 1, 2
constexpr uint32_t kBcPoly = 0xEDB88320u;
constexpr uint64_t kBcTile = 2048;

struct __attribute__((aligned(16))) BcArgs {
  uint64_t len;          // bytes per row
  int64_t sstride;       // affine batch: stripe s's row i at ptr[i] + s * sstride (0: explicit table)
  uint32_t tps, ntiles;  // 2 KiB column tiles per stripe (the last one may be partial), in the launch
  uint32_t tab, crc_stride;
  uint32_t nst, wps, groups;  // the per-row form: stripes, waves per stripe W, wave groups (<= nst)
  uint32_t xjump;             // the per-row form: x^(8 * 2048 * W)
  uint32_t fin;               // shift(~0, len) ^ ~0
  uint32_t bend;              // tiles [0, bend) of a stripe go round the W waves (bend = W floor(tps / W))
  uint32_t tail, tblk;        // the stripes' last tps - bend tiles: one per wave of workgroups >= tblk
  uint32_t pad0;
  uint32_t* crc;         // [stripe][crc_stride] checksum words (XOR-accumulated)
  const uint32_t* tabs;  // kBcTabs x 32 words
  uint8_t slot[40];      // checksum word of kernel row i (inputs, then outputs)
  // tile j's end to the row's end is x^(8 (2048 e - pad)), e = tps - 1 - j:
  // pw[0][e % 64] (pad folded in) * pw[1][(e / 64) % 64] * pw[2][e / 4096]
  uint32_t pw[3][kBcPow];
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

#ifndef CFSEC_BC_LO
#define CFSEC_BC_LO 1  // the 16 + 20 code's output rows' registers in LDS too (A/B)
#endif
#ifndef CFSEC_BC_WPE
#define CFSEC_BC_WPE 3  // waves per SIMD the per-row form is compiled for
#endif
#ifndef CFSEC_BC_PROBE
#define CFSEC_BC_PROBE 0  // timing probes only (wrong words): bit 0 no input-row terms, bit 1 no output-row terms,
                          // bit 2 no register jumps
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

// CRC = false: the product alone (bs_plain_matches: the wide LRC modes, whose fused rows outgrow
// the fixed-K kernels' 12 outputs and ran as two products)
template <class Net, int M, bool CRC = true>
__global__ __launch_bounds__(64 * kBcWaves) __attribute__((amdgpu_waves_per_eu(
    Net::K > 12 || (Net::K > 8 && M > 4) || M > 12 ? 2 : CFSEC_BC_WPE, 4))) void gf_bs_crc_kernel(const BcArgs a) {
  constexpr int K = Net::K;
  constexpr int NR = K + M;  // checksummed rows: the inputs, then the outputs
  static_assert(NR <= 64, "one lane per row's word");
  // the rows padded for the lane fold: log2(NP) halving levels then 6 - log2(NP) lane butterflies, NP -
  // 1 + 6 - log2(NP) register-steps (8 rows: 10 instead of the 32 a 32-row padding took)
#ifndef CFSEC_BC_NPMIN
#define CFSEC_BC_NPMIN 8
#endif
  constexpr int NP = NR <= CFSEC_BC_NPMIN ? CFSEC_BC_NPMIN : NR <= 16 ? (16 > CFSEC_BC_NPMIN ? 16 : CFSEC_BC_NPMIN)
                     : NR <= 32 ? 32 : 64;
  constexpr int LG = NP == 8 ? 3 : NP == 16 ? 4 : NP == 32 ? 5 : 6;
  __shared__ uint32_t tb[CRC ? kBcTabs * 32 : 1];  // planes, the jump, the lane tree
  __shared__ uint32_t slot[64];  // the rows' word offsets, indexed per lane at the segment ends
  // LI (k > 8: the 16 + 20 code, 38 registers beside 128 input planes): the input rows' Horner registers
  // live in LDS across the network -- read, jumped and updated at each tile's input phase -- instead of
  // in VGPRs the network needs (79 spilled at 2 waves per SIMD otherwise)
  constexpr bool LI = CRC && K > 8;
  // LO (k > 12 or m > 12: the 16 + 20 code, EC6P6L9, EC6P8L10): the output rows' registers too, read, jumped and updated where the
  // network emits each row
  constexpr bool LO = CRC && (K > 12 || M > 12) && CFSEC_BC_LO;
  constexpr int NL = (LI ? K : 0) + (LO ? M : 0);  // rows whose registers live in LDS
  // row i's LDS slot (in_lds(i)): the inputs first when LI, then the outputs when LO
  const auto in_lds = [](int i) { return (LI && i < K) || (LO && i >= K); };
  const auto lds_row = [](int i) { return i < K ? i : (LI ? K : 0) + (i - K); };
  __shared__ uint32_t rin[NL ? kBcWaves * NL * 64 : 1];
  if constexpr (CRC) {
    for (uint32_t i = threadIdx.x; i < kBcPlaneTabs * 8; i += blockDim.x)
      reinterpret_cast<u32x4*>(tb)[i] = reinterpret_cast<const u32x4*>(a.tabs)[i];
    for (uint32_t i = threadIdx.x; i < 6 * kBcFields * 8; i += blockDim.x)
      reinterpret_cast<u32x4*>(tb + kBcTree * 32)[i] = reinterpret_cast<const u32x4*>(a.tabs + kBcTree * 32)[i];
    // the register's jump over the launch's tile stride (2048 W bytes): table (kBcJump + f)[e] =
    // shift(e << 5f, 2048 W), built here from x^(8 * 2048 * W)
    for (uint32_t i = threadIdx.x; i < kBcFields * 32; i += blockDim.x)
      tb[kBcJump * 32 + i] = bc_mulmod((i & 31u) << (5 * (i >> 5)), a.xjump);
    if (threadIdx.x == 0)  // constant indices: a lane-indexed read of the argument block would copy it to scratch
#pragma unroll
      for (int i = 0; i < NR; ++i) slot[i] = a.slot[i];
    __syncthreads();
  }
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t wid = blockIdx.x * kBcWaves + wave;
  // wave (g, j) = (wid / W, wid % W) takes tiles j, j + W, ... (< bend) of stripes g, g + groups, ...;
  // a tail wave (workgroups from tblk on, dispatched as the round waves retire) one tile >= bend
  const uint32_t W = a.wps, g0 = wid / W, j = wid - g0 * W;
  const bool tailw = blockIdx.x >= a.tblk;
  const uint32_t tq = (blockIdx.x - a.tblk) * kBcWaves + wave;  // tail waves: stripe tq / tail's tile
  if (tailw ? tq >= a.tail * a.nst : g0 >= a.groups) return;  // no barrier below
  const uint64_t len = a.len;
  const uint32_t tps = a.tps;
  if (!tailw && j >= tps) return;
  const auto in_row = [&](uint32_t s, int i) -> const uint8_t* {
    return a.sstride ? a.ptr[i] + (int64_t)s * a.sstride : a.ptr[(size_t)s * K + i];
  };
  const auto out_row = [&](uint32_t s, int r) -> uint8_t* {
    return const_cast<uint8_t*>(a.sstride ? a.ptr[K + r] + (int64_t)s * a.sstride
                                          : a.ptr[(size_t)a.tab * K + (size_t)s * M + r]);
  };
  uint32_t R[NR];
  bool fresh = true;  // LI: the wave's first tile of a stripe (the LDS registers hold nothing yet)
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
      if constexpr (!CRC) {
      } else if constexpr (LI) {
        uint32_t* ri = rin + (wave * NL + i) * 64 + lane;
        uint32_t v = fresh ? 0u : (CFSEC_BC_PROBE & 4) ? *ri : bc_five7(tb + kBcJump * 32, *ri);
        if constexpr (!(CFSEC_BC_PROBE & 1)) v ^= bc_planes(tb, pl);
        *ri = v;
      } else {
        if constexpr (!(CFSEC_BC_PROBE & 1)) R[i] ^= bc_planes(tb, pl);
        asm volatile("" : "+v"(R[i]));
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (Net::Paired) dev::bs_pair_basis<K>(x);
    __builtin_amdgcn_sched_barrier(0);
    Net::template net<M>(x, [&](int r, uint32_t (&o)[8]) {
      if constexpr (!CRC) {
      } else if constexpr (LO) {
        uint32_t* ri = rin + (wave * NL + lds_row(K + r)) * 64 + lane;
        uint32_t v = fresh ? 0u : (CFSEC_BC_PROBE & 4) ? *ri : bc_five7(tb + kBcJump * 32, *ri);
        if constexpr (!(CFSEC_BC_PROBE & 2)) v ^= bc_planes(tb, o);
        *ri = v;
      } else {
        if constexpr (!(CFSEC_BC_PROBE & 2)) R[K + r] ^= bc_planes(tb, o);
        asm volatile("" : "+v"(R[K + r]));
      }
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
  const uint32_t s0 = tailw ? tq / a.tail : g0, sstep = tailw ? a.nst : a.groups;
  const uint32_t c0 = tailw ? a.bend + (tq - s0 * a.tail) : j, cend = tailw ? c0 + 1 : a.bend;
  for (uint32_t s = s0; s < a.nst; s += sstep) {
#pragma unroll
    for (int i = 0; i < NR; ++i) R[i] = 0u;
    fresh = true;
    uint32_t c = c0;
    for (;;) {
      const uint64_t po = (uint64_t)c * kBcTile + lane * 16;
      if ((uint64_t)(c + 1) * kBcTile <= len) tile(s, po, std::true_type{});  // wave-uniform
      else tile(s, po, std::false_type{});
      if (c + W >= cend) break;
      c += W;
      if constexpr (CRC) {
#pragma unroll
        for (int i = 0; i < NR; ++i)
          if (!in_lds(i) && !(CFSEC_BC_PROBE & 4)) R[i] = bc_five7(tb + kBcJump * 32, R[i]);
      }
      fresh = false;
    }
    if constexpr (!CRC) continue;
    // the stripe's end of this wave: the 64 lanes' registers folded by recursive halving -- at level k
    // lane pairs l, l ^ 2^k swap halves of their registers and each keeps the sum of one half, the
    // earlier group's value moved 16 * 2^k bytes on (7 lookups); the NP padded registers are one per
    // lane after log2(NP) levels, the rest combine whole lane groups (32 rows: 32 register-steps in all
    // instead of a 32-column basis per register) -- so lane l holds row bitrev(l mod NP)'s sum
    uint32_t mine;
    {
      uint32_t v[NP];
#pragma unroll
      for (int i = 0; i < NP; ++i) v[i] = i < NR ? (in_lds(i) ? rin[(wave * NL + lds_row(i)) * 64 + lane] : R[i]) : 0u;
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        const int half = NP >> (k + 1) ? NP >> (k + 1) : 1;  // past log2(NP): whole registers combined
        const bool halving = (NP >> (k + 1)) != 0;
        const bool up = (lane >> k) & 1u;
#pragma unroll
        for (int i = 0; i < half; ++i) {
          const uint32_t send = !halving ? v[i] : (up ? v[i] : v[half + i]);
          const uint32_t keep = !halving ? v[i] : (up ? v[half + i] : v[i]);
          const uint32_t recv = (uint32_t)__shfl_xor((int)send, 1 << k, 64);
          const uint32_t lo = up ? recv : keep, hi = up ? keep : recv;
          v[i] = bc_five7(tb + (kBcTree + k * kBcFields) * 32, lo) ^ hi;
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      mine = v[0];
    }
    // lane l holds row bitrev(l mod NP) (log2(NP) bits)
    const uint32_t row = __builtin_bitreverse32(lane & (NP - 1u)) >> (32 - LG);
    const uint32_t e = tps - 1 - c;
    const uint32_t k = bc_mulmod(bc_mulmod(a.pw[0][e % kBcPow], a.pw[1][(e / kBcPow) % kBcPow]),
                                 a.pw[2][e / (kBcPow * kBcPow)]);
    uint32_t w = bc_mulmod(mine, k);
    if (!tailw && j == 0) w ^= a.fin;
    if (lane < (uint32_t)NP && row < (uint32_t)NR) atomicXor(a.crc + (size_t)s * a.crc_stride + slot[row], w);
  }
}


// ---- host side ----
uint32_t env_mask(const char* name, uint32_t dflt) {
  const char* v = std::getenv(name);
  return v && *v ? (uint32_t)std::strtoul(v, nullptr, 0) : dflt;
}
// CFSEC_BS_CRC: bit 0 EC6P10L2's fused LRC encode (6 x 12), bit 1 EC12P4 (12 x 4; bit 3 the same),
// bit 2 EC16P20 / EC16P20L2 (16 x 20 / 22), bit 4 EC6P8, EC6P10, EC12P9, EC15P12, EC10P4, EC4P4,
// EC3P3 and the LRC modes EC6P3L3, EC4P4L2, EC6P6L9, EC6P8L10 (the product + separate pass, or for
// EC6P3L3 the v_perm fused kernel, otherwise), bit 5 the product alone for EC6P6L9 / EC6P8L10's plain
// fused encodes, bit 6 EC6P6 and EC16P4 (the EC6P10L2 / 16 + 20 networks' first rows; their v_perm
// fused kernels before: EC6P6's 1 MiB-blob put 152 -> 131 us, EC16P4 105 -> 103, the put-batch probe
// 124 -> 117, profiles/r06/bs_crc/ec6p6_ec16p4_ab.txt) -- all on by default --, bit 7 EC6P3 (off: 62 vs
// 64 us); 0 keeps the lookup-product kernels / the separate pass (A/B).
// EC12P4 was off until the remainder tiles became tail waves: the bench's fused encode + CRC 0.484 ->
// 0.506, the ec seam 0.478 -> 0.498 (profiles/r06/bs_crc/bench_ec12p4_tail_ab.txt); 4 MiB blobs 183 ->
// 178 us in the shape sweep (shape_sweep_ec12p4_tail.txt)
#ifndef CFSEC_BS_CRC_DEFAULT
#define CFSEC_BS_CRC_DEFAULT 119
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

// The device table block: the 56 plane tables, the 2048-byte jump (the kernel rebuilds it for its
// tile stride), the lane tree's 6 levels
std::vector<uint32_t> bc_host_tables() {
  std::vector<uint32_t> t((size_t)kBcTabs * 32, 0u);
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
      for (int k = 0; k < 6; ++k)
        t[(size_t)(kBcTree + k * kBcFields + f) * 32 + e] = crc_mulmod(crc_xpow(8ll * (16 << k)), e << (5 * f));
    }
  }
  return t;
}

struct BcDev {
  std::mutex mu;
  uint32_t* tab = nullptr;
};

hipError_t bc_device(const uint32_t** tab) {
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
  *tab = c.tab;
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

template <class Net, int M, bool CRC = true>
int bc_groups() {  // resident workgroups on the device (one wave of workgroups)
  static std::mutex mu;
  static std::map<int, int> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  std::lock_guard<std::mutex> l(mu);
  auto it = cache.find(dev);
  if (it != cache.end()) return it->second;
  int per = 0, cus = 0;
  const void* f = reinterpret_cast<const void*>(&gf_bs_crc_kernel<Net, M, CRC>);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, f, 64 * kBcWaves, 0) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
    (void)hipGetLastError();
    per = 0;
  }
  const int n = per > 0 && cus > 0 ? per * cus : 768;
  cache.emplace(dev, n);
  return n;
}

template <class Net, int M, bool CRC = true>
hipError_t bc_launch(const MatVecJob& job, uint32_t* crc, int crc_stride, const int* slot, hipStream_t st) {
  constexpr int K = Net::K;
  BcArgs a{};
  hipError_t e = bc_device(&a.tabs);
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
  if (CRC)
    for (int i = 0; i < K + M; ++i) a.slot[i] = (uint8_t)slot[i];
  const int64_t ss = bc_affine_stride(job);
  a.sstride = ss;
  const int per = ss ? job.nstripes : kBcPtr / (K + M);
  const int groups = bc_groups<Net, M, CRC>();
  for (int s0 = 0; s0 < job.nstripes; s0 += per) {
    const int ns = std::min(per, job.nstripes - s0);
    const int tab = ss ? 1 : ns;
    a.tab = (uint32_t)tab;
    a.crc = CRC ? crc + (size_t)s0 * crc_stride : nullptr;
    for (int s = 0; s < tab; ++s) {
      for (int c = 0; c < K; ++c) a.ptr[s * K + c] = job.in[(size_t)(s0 + s) * K + c];
      for (int r = 0; r < M; ++r) a.ptr[tab * K + s * M + r] = job.out[(size_t)(s0 + s) * M + r];
    }
    const uint64_t nt = tps * (uint64_t)ns;
    a.ntiles = (uint32_t)nt;
    // W waves per stripe, each taking every W-th tile (neighbouring waves on neighbouring tiles of
    // one stripe; a wave's tiles 2048 W bytes apart, one checksum fold per wave and stripe)
    const uint64_t nw = (uint64_t)groups * kBcWaves;
    uint64_t W = std::min<uint64_t>(tps, std::max<uint64_t>(1, nw / (uint64_t)ns));
    static const uint32_t tpw_env = env_mask("CFSEC_BC_TPW", 0);  // tiles per wave and stripe (A/B)
    if (tpw_env) W = std::min<uint64_t>(nw, (tps + tpw_env - 1) / tpw_env);
    const uint64_t ng = std::min<uint64_t>((uint64_t)ns, nw / W);
    a.nst = (uint32_t)ns;
    a.wps = (uint32_t)W;
    a.groups = (uint32_t)ng;
    a.xjump = crc_xpow(8 * (int64_t)kBcTile * (int64_t)W);
    unsigned grid = (unsigned)((ng * W + kBcWaves - 1) / kBcWaves);
    // the remainder tps mod W: in W-strided rounds a third of the waves take one tile more, and a SIMD
    // whose 3 waves all do leaves the launch a tile late (C4: 320 tiles per row 160 us, 321 tiles 178,
    // profiles/r06/bs_crc/c4_tail_tiles.txt); as one tile per extra wave those tiles go wherever
    // waves retire first: C4 187 -> 176 us per put batch, EC6P6L9 158 -> 151, EC12P9 184 -> 173,
    // EC16P20L2 (32 x 699,051) 330 -> 305; moving a whole round more to tail waves: 181 (C4); plain
    // products unchanged (profiles/r06/bs_crc/tail_waves_ab.txt).  CFSEC_BC_TAIL: the largest remainder
    // (percent of W) taken this way (0: the strided rounds only)
    static const uint32_t tail_pct = env_mask("CFSEC_BC_TAIL", 100);
    const uint64_t rem = tps % W;
    a.bend = (uint32_t)tps;
    a.tail = 0;
    a.tblk = grid;
    if (rem && rem * 100 <= (uint64_t)tail_pct * W) {
      a.bend = (uint32_t)(tps - rem);
      a.tail = (uint32_t)rem;
      grid += (unsigned)((rem * ns + kBcWaves - 1) / kBcWaves);
    }
    if (env_mask("CFSEC_TRACE_CRC", 0))
      std::fprintf(stderr, "cfsec: bs launch stripes=%d tps=%llu W=%llu groups=%llu tail=%u\n", ns,
                   (unsigned long long)tps, (unsigned long long)W, (unsigned long long)ng, a.tail);
    hipLaunchKernelGGL((gf_bs_crc_kernel<Net, M, CRC>), dim3(grid), dim3(64 * kBcWaves), 0, st, a);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace

bool bs_crc_matches(int k, int m, const uint8_t* coef) {
  if (!coef) return false;
  const uint32_t mask = bs_crc_mask();
  if ((mask & 1u) && k == 6 && m == 12) return rows_equal<dev::BsEc6p10l2>(coef, 12);
  if ((mask & 10u) && k == 12 && m == 4) return rows_equal<dev::BsEc12p4>(coef, 4);
  if ((mask & 4u) && k == 16 && (m == 20 || m == 22)) return rows_equal<dev::BsEc16p20l2>(coef, m);
  if (mask & 16u) {  // the other RS modes' encodes (EC6P8 / EC6P10 on the EC6P10L2 network's first rows;
                     // EC6P6, EC16P4, EC6P3: bits 6, 7 below)
    if (k == 6 && (m == 8 || m == 10)) return rows_equal<dev::BsEc6p10l2>(coef, m);
    if (k == 12 && m == 9) return rows_equal<dev::BsEc12p9>(coef, 9);
    if (k == 15 && m == 12) return rows_equal<dev::BsEc15p12>(coef, 12);
    if (k == 10 && m == 4) return rows_equal<dev::BsEc10p4>(coef, 4);
    if (k == 4 && m == 4) return rows_equal<dev::BsEc4p4>(coef, 4);
    if (k == 3 && m == 3) return rows_equal<dev::BsEc3p3>(coef, 3);
    // the other LRC modes' fused encodes (global + every AZ's local rows over the data)
    if (k == 6 && m == 6 && rows_equal<dev::BsEc6p3l3>(coef, 6)) return true;
    if (k == 4 && m == 6) return rows_equal<dev::BsEc4p4l2>(coef, 6);
    if (k == 6 && m == 15) return rows_equal<dev::BsEc6p6l9>(coef, 15);
    if (k == 6 && m == 18) return rows_equal<dev::BsEc6p8l10>(coef, 18);
  }
  // EC6P6 and EC16P4 (bit 6), EC6P3 (bit 7): the first rows of the EC6P10L2 / 16 + 20 networks
  if ((mask & 64u) && k == 6 && m == 6) return rows_equal<dev::BsEc6p10l2>(coef, 6);
  if ((mask & 64u) && k == 16 && m == 4) return rows_equal<dev::BsEc16p20l2>(coef, 4);
  if ((mask & 128u) && k == 6 && m == 3) return rows_equal<dev::BsEc6p10l2>(coef, 3);
  return false;
}

hipError_t launch_bs_crc(const MatVecJob& job, uint32_t* crc, int crc_stride, const int* slot, hipStream_t st) {
  if (!crc || !slot || !bs_crc_matches(job.k, job.m, job.coef) || job.len == 0 ||
      (job.len + kBcTile - 1) / kBcTile > (uint64_t)kBcPow * kBcPow * kBcPow ||
      (job.len + kBcTile - 1) / kBcTile * (uint64_t)std::max(job.nstripes, 1) > 0xFFFFFFFFull || crc_stride > 256)
    return hipErrorInvalidValue;
  for (int i = 0; i < job.k + job.m; ++i)
    if (slot[i] < 0 || slot[i] >= crc_stride) return hipErrorInvalidValue;
  if (env_mask("CFSEC_TRACE_CRC", 0))  // read per call: tests turn it on mid-process
    std::fprintf(stderr, "cfsec: bs crc k=%d m=%d stripes=%d len=%llu\n", job.k, job.m, job.nstripes,
                          (unsigned long long)job.len);
  if (job.k == 6 && job.m == 12) return bc_launch<dev::BsEc6p10l2, 12>(job, crc, crc_stride, slot, st);
  if (job.k == 6 && job.m == 6 && rows_equal<dev::BsEc6p3l3>(job.coef, 6))
    return bc_launch<dev::BsEc6p3l3, 6>(job, crc, crc_stride, slot, st);
  if (job.k == 6 && job.m == 6) return bc_launch<dev::BsEc6p10l2, 6>(job, crc, crc_stride, slot, st);
  if (job.k == 6 && job.m == 3) return bc_launch<dev::BsEc6p10l2, 3>(job, crc, crc_stride, slot, st);
  if (job.k == 16 && job.m == 4) return bc_launch<dev::BsEc16p20l2, 4>(job, crc, crc_stride, slot, st);
  if (job.k == 6 && job.m == 15) return bc_launch<dev::BsEc6p6l9, 15>(job, crc, crc_stride, slot, st);
  if (job.k == 6 && job.m == 18) return bc_launch<dev::BsEc6p8l10, 18>(job, crc, crc_stride, slot, st);
  if (job.k == 4 && job.m == 6) return bc_launch<dev::BsEc4p4l2, 6>(job, crc, crc_stride, slot, st);
  if (job.k == 6 && job.m == 10) return bc_launch<dev::BsEc6p10l2, 10>(job, crc, crc_stride, slot, st);
  if (job.k == 6) return bc_launch<dev::BsEc6p10l2, 8>(job, crc, crc_stride, slot, st);
  if (job.k == 12 && job.m == 9) return bc_launch<dev::BsEc12p9, 9>(job, crc, crc_stride, slot, st);
  if (job.k == 15) return bc_launch<dev::BsEc15p12, 12>(job, crc, crc_stride, slot, st);
  if (job.k == 10) return bc_launch<dev::BsEc10p4, 4>(job, crc, crc_stride, slot, st);
  if (job.k == 4) return bc_launch<dev::BsEc4p4, 4>(job, crc, crc_stride, slot, st);
  if (job.k == 3) return bc_launch<dev::BsEc3p3, 3>(job, crc, crc_stride, slot, st);
  if (job.k == 16 && job.m == 22) return bc_launch<dev::BsEc16p20l2, 22>(job, crc, crc_stride, slot, st);
  if (job.k == 16) return bc_launch<dev::BsEc16p20l2, 20>(job, crc, crc_stride, slot, st);
  return bc_launch<dev::BsEc12p4, 4>(job, crc, crc_stride, slot, st);
}

// The product alone on the bit-sliced kernel for the wide LRC modes' fused encodes (EC6P6L9 6 x 15,
// EC6P8L10 6 x 18: over the fixed-K kernels' 12 outputs they ran as two products): a 32-bid put batch
// (32 x 699,051 B) 173 -> 117 and 190 -> 128 us (profiles/r06/bs_crc/lrc_modes_put_batch.txt);
// CFSEC_BS_CRC bit 5
bool bs_plain_matches(int k, int m, const uint8_t* coef) {
  if (!coef || !(bs_crc_mask() & 32u) || k != 6) return false;
  if (m == 15) return rows_equal<dev::BsEc6p6l9>(coef, 15);
  if (m == 18) return rows_equal<dev::BsEc6p8l10>(coef, 18);
  return false;
}

hipError_t launch_bs_plain(const MatVecJob& job, hipStream_t st) {
  // (the caller has resolved the mode to a plain store: kStore, or kStoreVerify storing every row)
  if (!bs_plain_matches(job.k, job.m, job.coef) || job.len == 0 || job.lens ||
      (job.len + kBcTile - 1) / kBcTile > (uint64_t)kBcPow * kBcPow * kBcPow ||
      (job.len + kBcTile - 1) / kBcTile * (uint64_t)std::max(job.nstripes, 1) > 0xFFFFFFFFull)
    return hipErrorInvalidValue;
  if (env_mask("CFSEC_TRACE_CRC", 0))
    std::fprintf(stderr, "cfsec: bs plain k=%d m=%d stripes=%d len=%llu\n", job.k, job.m, job.nstripes,
                 (unsigned long long)job.len);
  if (job.m == 15) return bc_launch<dev::BsEc6p6l9, 15, false>(job, nullptr, 0, nullptr, st);
  return bc_launch<dev::BsEc6p8l10, 18, false>(job, nullptr, 0, nullptr, st);
}

bool bs_crc_takes(const MatVecJob& job, int crc_stride, const int* slot) {
  if (!slot || slot[0] < 0 || job.len == 0 || crc_stride > 256 || !bs_crc_matches(job.k, job.m, job.coef)) return false;
  const uint64_t tps = (job.len + kBcTile - 1) / kBcTile;
  return tps <= (uint64_t)kBcPow * kBcPow * kBcPow && tps * (uint64_t)std::max(job.nstripes, 1) <= 0xFFFFFFFFull;
}

}  // namespace cfsec
