// gf_bs16.hip -- the EC16P20 / EC16P20L2 parity as a bit-sliced XOR network (gf_bitslice.hpp,
// bs_net_ec16p20l2.hpp): the encodes' whole 2 KiB column runs; the launcher (gf_kernels.hip) sends
// the rest of each row (and every other matrix) to the dyadic kernels.
//
// Persistent waves, 8 per CU (2 per SIMD at <= 256 VGPRs: the 128 input planes of a 32-byte column
// stay in registers).  While a wave runs the network on its tile, data rows 0-7 of its next tile
// are copied into its 16 KiB of LDS by global_load_lds (no VGPRs); rows 8-15 are loaded at the
// tile's top, where the other wave of the SIMD covers their latency.  EC16P20L2's fused encode,
// 64 x 262,144: 131.9 us against 148.6 us for the 16x16-dyadic v_perm kernel (profiles/r04/
// bs_probe.txt); it issues ~40 % fewer VALU instructions at 2 instead of 4 waves per SIMD.
// The network takes its inputs in the paired basis (gf_bitslice.hpp bs_pair_basis): each dyadic
// row pair of the 20 global rows then shares the half over the odd columns, 3262 instead of 3904
// XOR ops per 32-byte column for the 22 rows.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstddef>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

#include "bs_net_ec16p20l2.hpp"
#include "gf_bitslice.hpp"
#include "gf256.hpp"
#include "gf_launch.hpp"

namespace cfsec {

namespace {
constexpr int kBsK = 16, kBsPrefetch = 8, kBsWaves = 8;
// LDS-DMA cache policy (gf_bitslice.hpp bs_glds_row): encode default, repair non-temporal (A/B)
#ifndef CFSEC_BS_ENC_GLDS
#define CFSEC_BS_ENC_GLDS 0
#endif
#ifndef CFSEC_BS_REP_GLDS
#define CFSEC_BS_REP_GLDS 2
#endif
#ifndef CFSEC_BS_ENC_LDNT
#define CFSEC_BS_ENC_LDNT 1  // register loads of the rows not prefetched: non-temporal (A/B)
#endif
#ifndef CFSEC_BS_REP_LDNT
#define CFSEC_BS_REP_LDNT 1
#endif
// row pointers (and the repair's row masks) re-read where used: the repair 1-2 % faster, the encode
// no faster (profiles/r04/bs_reload_ab.txt), A/B
#ifndef CFSEC_BS_REP_RELOAD
#define CFSEC_BS_REP_RELOAD 1
#endif
#ifndef CFSEC_BS_ENC_RELOAD
#define CFSEC_BS_ENC_RELOAD 0
#endif
constexpr int kBsEncGlds = CFSEC_BS_ENC_GLDS, kBsRepGlds = CFSEC_BS_REP_GLDS;

// Both kernels end their tile loop with an LDS-DMA re-prefetch in flight (branch-free: the last
// tile re-reads itself).  s_endpgm does not wait for it, and once every wave of the workgroup has
// ended its 160 KiB of LDS goes to the next workgroup placed on the CU -- possibly another launch's,
// whose freshly prefetched slots the late DMA then overwrites.  Round 4's false ErrVerify (two
// processes, or two streams, repairing at once; profiles/r05/stale_dma_probe.txt) was this.  So
// every wave drains its vector memory operations before it ends.  CFSEC_BS_DRAIN=0: the round-4
// form (A/B and the reproduction only).
#ifndef CFSEC_BS_DRAIN
#define CFSEC_BS_DRAIN 1
#endif
__device__ __forceinline__ void bs_drain_exit() {
  if constexpr (CFSEC_BS_DRAIN) __builtin_amdgcn_s_waitcnt(dev::bs_waitcnt_vm(0));
}

// Row pointer j of the kernels' GfArgs (their first argument, at offset 0 of the argument segment)
// by a scalar load whose offset the compiler cannot see through: the kernels name up to 40 rows,
// and held across the tile loop their pointers (with the per-row conditions) outgrow the SGPRs --
// the spilled ones come back through v_readlane, ~240 per tile in the repair kernel.  Re-read
// where used, they cost a scalar-cache load each.
__device__ __forceinline__ const uint8_t* bs_kernarg_ptr(uint32_t j) {
  typedef const __attribute__((address_space(4))) uint64_t ku64;
  uint32_t w = __builtin_amdgcn_readfirstlane((uint32_t)(offsetof(dev::GfArgs, ptr) / 8) + j);
  asm volatile("" : "+s"(w));
  return reinterpret_cast<const uint8_t*>(((ku64*)__builtin_amdgcn_kernarg_segment_ptr())[w]);
}
constexpr bool kBsEncLdNt = CFSEC_BS_ENC_LDNT, kBsRepLdNt = CFSEC_BS_REP_LDNT;

// A row-offset table in device memory (TAB 2 launches): row i of stripe s at base + dtab[s * (K +
// M) + i] -- stripes whose shards each sit at their own address, any number per launch
struct BsTabArgs {
  const uint8_t* base;
  const uint32_t* dtab;
};

// Encode: Net's K inputs -> its first M rows (K <= 16: 8 K input planes in registers)
// (GfArgs must stay the first parameter: bs_kernarg_ptr reads it at offset 0 of the arguments)
template <class Net, int M, int TAB>
__global__ __launch_bounds__(64 * kBsWaves) __attribute__((amdgpu_waves_per_eu(2, 2))) void gf_bs_kernel(
    const dev::GfArgs a, const BsTabArgs tb, uint32_t tiles_per_stripe, uint32_t ntiles) {
  using namespace dev;
  constexpr int K = Net::K, PF = K < kBsPrefetch ? K : kBsPrefetch;
  constexpr int NW = 2 * (K - PF) + 2 * M;  // vector memory ops a tile issues after its prefetch
  __shared__ __attribute__((aligned(16))) uint8_t lds[kBsWaves][PF * kBsWaveBytes];
  // the wave index as a scalar: tiles, stripes and row pointers are then wave-uniform (scalar loads
  // of the pointer table, no vector memory operations besides the shard copies counted below)
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  uint8_t* pre = lds[wave];
  const uint32_t nw = gridDim.x * kBsWaves;
  // row i of stripe s (inputs 0..K-1, then outputs), at the lane's first byte of column tile c
  // row pointer j of the argument block, re-read where used (bs_kernarg_ptr)
  const auto ptr_at = [&](uint32_t j) -> const uint8_t* {
    if constexpr (CFSEC_BS_ENC_RELOAD) return bs_kernarg_ptr(j);
    else return a.ptr[j];
  };
  const auto row = [&](uint32_t s, int i, uint32_t c) -> uint8_t* {
    const uint8_t* base;
    if constexpr (TAB == 2) {
      typedef const __attribute__((address_space(4))) uint32_t cu32;
      uint32_t w = __builtin_amdgcn_readfirstlane(s * (uint32_t)(K + M) + (uint32_t)i);
      asm volatile("" : "+s"(w));
      base = tb.base + ((cu32*)tb.dtab)[w];  // a scalar load: the table is read-only for the launch
    } else if (i < K) {
      base = a.sstride ? ptr_at(i) + (int64_t)s * a.sstride : ptr_at(s * K + i);
    } else {
      base = a.sstride ? ptr_at(K + (i - K)) + (int64_t)s * a.sstride : ptr_at(a.tab * K + s * M + (i - K));
    }
    return const_cast<uint8_t*>(base) + (size_t)c * kBsWaveBytes + lane * 16;
  };
  const auto prefetch = [&](uint32_t t) {
    const uint32_t s = t / tiles_per_stripe, c = t % tiles_per_stripe;
#pragma unroll
    for (int i = 0; i < PF; ++i) bs_glds_row<kBsEncGlds>(row(s, i, c), pre + i * kBsWaveBytes);
  };
  uint32_t t = blockIdx.x * kBsWaves + wave;
  if (t >= ntiles) return;  // no barrier in this kernel: idle waves leave at once
  prefetch(t);
  __builtin_amdgcn_s_waitcnt(bs_waitcnt_vm(0));
  for (; t < ntiles; t += nw) {
    const uint32_t s = t / tiles_per_stripe, c = t % tiles_per_stripe;
    uint32_t x[8 * K];
#pragma unroll
    for (int i = PF; i < K; ++i) bs_ld_row<kBsEncLdNt>(row(s, i, c), &x[8 * i]);
    // the prefetched rows were issued before the previous tile's stores and these loads, and
    // vector memory operations retire in issue order
    __builtin_amdgcn_s_waitcnt(bs_waitcnt_vm(NW > 63 ? 63 : NW));
#pragma unroll
    for (int i = 0; i < PF; ++i) bs_lds_row(pre + i * kBsWaveBytes, lane, &x[8 * i]);
    __builtin_amdgcn_s_waitcnt(kBsWaitLgkm0);
#pragma unroll
    for (int i = 0; i < K; ++i) bs_transpose8(&x[8 * i]);
    if constexpr (Net::Paired) bs_pair_basis<K>(x);
    __builtin_amdgcn_sched_barrier(0);
    prefetch(t + nw < ntiles ? t + nw : t);  // branch-free: nothing sinks below it (the last re-reads)
    __builtin_amdgcn_sched_barrier(0);
    Net::template net<M>(x, [&](int r, uint32_t (&o)[8]) {
      bs_transpose8(o);
      bs_st_row(row(s, K + r, c), o);
    });
  }
  // the last tile's re-prefetch is still in flight: the wave's LDS must not be handed to the next
  // workgroup on this CU (another launch's) while a DMA can still land in it (bs_drain_exit)
  bs_drain_exit();
}

// Reconstruct + Verify of the 16 + 20 code (C5's repair pass) in the same form, the syndrome way:
//   1. the 16 data slots as planes, a missing data row's slot loaded from a zero buffer;
//   2. s_q = stored(prow[q]) ^ (row prow[q] of the network over the present data): the stand-in
//      parities' syndromes, = A d with A the nd x nd block of the parity matrix at those rows and
//      the missing columns;
//   3. d = A^-1 s in byte form (v_perm products, tables from the host), stored, transposed and
//      written into their (zero) slots and the paired basis' pair sums -- no register indexing;
//   4. the full network: each parity (and extra) row stored (pstore), compared with its stored copy
//      through a 3-deep LDS ring filled by global_load_lds 2 compared rows ahead (pcmp; a mismatch
//      sets the stripe's flag), or skipped (the stand-ins, consistent by construction).
// Slots 0-6 of the next tile are prefetched into LDS during the network, slots 7-15 and the
// stand-ins load at the tile's top; 20 KiB of LDS per wave, 8 waves per CU.  C5's tasklet:
// 158.7-161.6 us against 173.0 us for the dyadic repair kernel (profiles/r04/bs_probe.txt).
struct BsRepairArgs {
  uint8_t slot[4];      // missing data row q (its slot), q < nd <= kBsRepairMaxNd
  uint8_t prow[4];      // the parity row standing in for it (input 16 - nd + q)
  dev::u32x4 t01[16];   // A^-1 product tables, entry j * 4 + q (gf_device.hpp coef_tables layout)
  uint32_t t2[16];
  const uint8_t* zero;  // kBsWaveBytes of zeros
  const uint8_t* base;  // TAB: row (s, i) at base + the 32-bit offset s * (16 + ND + M) + i of the table
  const uint32_t* dtab; // TAB 2: that table in device memory (TAB 1: in the argument block)
  // CRC launches (the rebuilt shards' crc32.ChecksumIEEE in the same pass): checksummed row k of
  // stripe s XOR-accumulates into crcw[s * crc_stride + crc_slot[k]] (zeroed before the launch)
  uint32_t* crcw;
  const uint32_t* ctab;  // kBsCrcTabs 5-bit tables (bs_crc_tables)
  const uint32_t* cpow;  // tiles_per_stripe words: x^(8 * 2048 * j) mod P
  uint32_t crc_stride, crc_ones;  // crc_ones: shift(~0, S) ^ ~0, folded in by each row's first segment
  uint8_t crc_slot[4];
  const uint32_t* lbasis;  // P2 launches: lane l's 32 columns of shift(., 16 * (63 - l)) (bs_crc_device)
  const uint32_t* ccols;   // P2 launches: tile j's 32 columns of the multiply by x^(8 * 2048 * j), j < tps
  uint32_t xjump;          // CRC launches: x^(8 * 2048 * W), W the waves per stripe (bs_rep_waves)
};

// TAB launches keep their row offsets where a repair launch does not read its GfArgs: from coef to
// the end of ptr (coef, slen, padding, ptr: the struct's last fields, in that order)
constexpr size_t kBsTabOff = offsetof(dev::GfArgs, coef);
static_assert(offsetof(dev::GfArgs, slen) > kBsTabOff && offsetof(dev::GfArgs, ptr) > offsetof(dev::GfArgs, slen) &&
                  offsetof(dev::GfArgs, ptr) + sizeof(dev::GfArgs::ptr) + 16 > sizeof(dev::GfArgs) && kBsTabOff % 4 == 0,
              "GfArgs: coef, slen, ptr last");
static_assert(sizeof(dev::GfArgs) + sizeof(BsRepairArgs) + 8 <= 4096, "repair kernel arguments within 4 KiB");
constexpr int kBsTabWords = (int)((offsetof(dev::GfArgs, ptr) + sizeof(dev::GfArgs::ptr) - kBsTabOff) / 4);

// word j of the kernel arguments' table area, by an opaque scalar load (as bs_kernarg_ptr)
__device__ __forceinline__ uint32_t bs_kernarg_u32(uint32_t j) {
  typedef const __attribute__((address_space(4))) uint32_t ku32;
  uint32_t w = __builtin_amdgcn_readfirstlane((uint32_t)(kBsTabOff / 4) + j);
  asm volatile("" : "+s"(w));
  return ((ku32*)__builtin_amdgcn_kernarg_segment_ptr())[w];
}

#ifndef CFSEC_BS_PF
#define CFSEC_BS_PF 7  // slots prefetched into LDS per wave (A/B)
#endif
#ifndef CFSEC_BS_RING
#define CFSEC_BS_RING 3  // LDS ring of compared rows per wave (A/B)
#endif
#ifndef CFSEC_BS_REP_ST
#define CFSEC_BS_REP_ST 0  // rebuilt rows: 0 non-temporal stores, 1 plain (the checksum pass may find them cached)
#endif
#ifndef CFSEC_BS_SKIPZ
#define CFSEC_BS_SKIPZ 1  // missing slots (zero planes) skip their transpose (A/B)
#endif
#ifndef CFSEC_BS_INS
#define CFSEC_BS_INS 1  // a solved row into its slot: 0 masked XOR over every slot, 1 uniform branch (A/B)
#endif
#ifndef CFSEC_BS_DEBUG_FLAGS
// 1: a failed compare writes 0x80000000 | row << 24 | column tile (the stripe's first mismatching
// compared row of the lane that wrote last) instead of 1 into the stripe's flag word (diagnosis)
#define CFSEC_BS_DEBUG_FLAGS 0
#endif
#ifndef CFSEC_BS_PERBID
#define CFSEC_BS_PERBID 0  // timing probe: the repair's tiles in per-stripe order (see the kernel)
#endif
#ifndef CFSEC_BS_BLOCKED
#define CFSEC_BS_BLOCKED 0  // 1: every repair launch maps each wave to a block of consecutive tiles (A/B)
#endif
constexpr int kRepPrefetch = CFSEC_BS_PF, kRepRing = CFSEC_BS_RING;
static_assert(kRepRing >= 3 || kRepRing == 2, "ring of 2 or more rows");

// ---- the rebuilt shards' checksums inside the repair pass (CRC launches) ----
// crc32.ChecksumIEEE(M) = f(0, M) ^ shift(~0, |M|) ^ ~0 (gf_crc.hpp's algebra, reflected: bit 31 =
// x^0).  A CRC launch gives each wave one block of consecutive column tiles (one stripe, or two when
// the block crosses a stripe end) instead of every nw-th tile, so each lane keeps a Horner register
// per checksummed row over its tiles: R <- shift(R, 2048) ^ shift(f(0, a), 1024) ^ f(0, b), with a,
// b its two 16-byte pieces (bytes 16 l and 1024 + 16 l of the tile) -- 63 lookups in 5-bit tables
// per row and tile.  At a segment's end the 64 lanes' registers fold in a 6-level tree over lane
// pairs (shift by 16 * 2^k bytes, 7 lookups a level), one multiply moves the sum from the segment's
// last tile to the row's end, and lane 0 XORs it into the row's word.  At most kBsCrcRows rows per
// stripe (C5: 2 data + 2 parity rows); the launch needs 16 KiB of LDS for the tables, so its waves
// prefetch one slot fewer.
constexpr int kBsCrcRows = 4;
static_assert(kBsRepairTileBytes == dev::kBsWaveBytes && kBsRepairMaxMissing == kBsRepairMaxNd, "kernels.hpp mirrors");
constexpr int kBsCrcTabA = 0, kBsCrcTabB = 28, kBsCrcTabR = 56, kBsCrcTabTree = 63, kBsCrcTabs = 105;
constexpr int kBsCrcLdsBytes = kBsCrcTabs * 32 * 4;
constexpr int kRepPrefetchCrc = CFSEC_BS_PF - 1;
constexpr uint32_t kBsCrcPoly = 0xEDB88320u;

// XOR of the 7 lookups of word v's 5-bit fields (bits 0, 5, ..., 25 and 30) in tables tb[f * 32]
// (gf_crc.hpp five_word: the masked copies make each extract the byte offset 4 * field)
__device__ __forceinline__ uint32_t bs_five7(const uint32_t* tb, uint32_t v) {
  uint32_t e = v & 0xC1F07C00u, o = v & 0x3E0F83E0u;
  asm volatile("" : "+v"(e), "+v"(o));
  const uint32_t off[7] = {(v << 2) & 0x7Cu,           __builtin_amdgcn_ubfe(o, 3, 7),  __builtin_amdgcn_ubfe(e, 8, 7),
                           __builtin_amdgcn_ubfe(o, 13, 7), __builtin_amdgcn_ubfe(e, 18, 7), __builtin_amdgcn_ubfe(o, 23, 7),
                           __builtin_amdgcn_ubfe(e, 28, 4)};
  uint32_t t[7];
#pragma unroll
  for (int f = 0; f < 7; ++f)
    t[f] = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(tb + f * 32) + off[f]);
  return dev::bs_x3(dev::bs_x3(t[0], t[1], t[2]), dev::bs_x3(t[3], t[4], t[5]), t[6]);
}

// a lane's contribution of one 32-byte row tile o (bytes, as stored): shift(f(0, a), 1024) ^ f(0, b)
__device__ __forceinline__ uint32_t bs_crc_tile(const uint32_t* ct, const uint32_t* o) {
  const uint32_t* ta = ct + kBsCrcTabA * 32;
  const uint32_t* tb = ct + kBsCrcTabB * 32;
  return dev::bs_x3(dev::bs_x3(bs_five7(ta, o[0]), bs_five7(ta + 224, o[1]), bs_five7(ta + 448, o[2])),
                    dev::bs_x3(bs_five7(ta + 672, o[3]), bs_five7(tb, o[4]), bs_five7(tb + 224, o[5])),
                    bs_five7(tb + 448, o[6]) ^ bs_five7(tb + 672, o[7]));
}

// bs_crc_tile word by word (7 lookups in flight at a time): inside the network, where the registers
// are spent
__device__ __forceinline__ uint32_t bs_crc_tile_seq(const uint32_t* ct, const uint32_t* o) {
  uint32_t u = 0;
#pragma unroll
  for (int w = 0; w < 8; ++w) {
    u ^= bs_five7(ct + (w < 4 ? kBsCrcTabA + 7 * w : kBsCrcTabB + 7 * (w - 4)) * 32, o[w]);
    __builtin_amdgcn_sched_barrier(0);
  }
  return u;
}

// a * b mod P (reflected)
__device__ __forceinline__ uint32_t bs_mulmod(uint32_t a, uint32_t b) {
  uint32_t p = 0;
#pragma unroll
  for (int i = 31; i >= 0; --i) {
    p ^= (a >> i & 1u) ? b : 0u;
    b = (b >> 1) ^ ((b & 1u) ? kBsCrcPoly : 0u);
  }
  return p;
}

// the 64 lanes' registers (lane l's bytes before lane l + 1's, 16-byte units) folded into one word,
// in every lane: level k combines lane groups of 2^k, the lower group shifted by 16 * 2^k bytes
__device__ __forceinline__ uint32_t bs_crc_lanes(const uint32_t* ct, uint32_t v, uint32_t lane) {
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const uint32_t other = (uint32_t)__shfl_xor((int)v, 1 << k, 64);
    const bool upper = lane >> k & 1u;
    const uint32_t lo = upper ? other : v, hi = upper ? v : other;
    v = bs_five7(ct + (kBsCrcTabTree + 7 * k) * 32, lo) ^ hi;
  }
  return v;
}

__device__ __forceinline__ void bs_st_rebuilt(uint8_t* p, const uint32_t* o) {
  if constexpr (CFSEC_BS_REP_ST) {
    *reinterpret_cast<dev::u32x4*>(p) = dev::u32x4{o[0], o[1], o[2], o[3]};
    *reinterpret_cast<dev::u32x4*>(p + 1024) = dev::u32x4{o[4], o[5], o[6], o[7]};
  } else {
    dev::bs_st_row(p, o);
  }
}

__device__ __forceinline__ void bs_mul_acc8(uint32_t* acc, const uint32_t* s0, const uint32_t* s1, const uint32_t* s2,
                                            const dev::u32x4 q, uint32_t t2) {
#pragma unroll
  for (int w = 0; w < 8; ++w)
    acc[w] = dev::bs_x3(acc[w], __builtin_amdgcn_perm(q.y, q.x, s0[w]), __builtin_amdgcn_perm(q.w, q.z, s1[w])) ^
             __builtin_amdgcn_perm(0u, t2, s2[w]);
}

// (GfArgs must stay the first parameter: bs_kernarg_ptr / bs_kernarg_u32 read it at offset 0 of
// the arguments)
// P2 (round 6, CFSEC_BS_REPAIR_CRC=2): the rebuilt rows' checksums as a second phase of each wave --
// after its last tile it re-reads the rows it stored (2 KiB of each per tile, from L2 / the Infinity
// Cache), takes each lane's 32 bytes through the 5-bit tables (bs_crc_tile, its own copy in its LDS
// slice), moves the lane's term to the tile's end by a per-lane GF(2) basis (64 VALU, no lookups),
// XOR-reduces the wave and moves the tile's term to the row's end (x^(8 * 2048 * j), scalar): no
// Horner registers through the network, the tile order unchanged, no second launch, and the waves
// that finish first checksum while the others still repair.  (The tile-to-row-end multiply is done
// per lane from the tile's 32 columns in scalar registers before the wave's XOR: as a scalar
// bit-serial multiply after it, 256 SALU per row and tile that a CU issues for all its waves, the
// phase cost 34 us per C5 call instead of the separate pass's 20.)
template <int M, int ND, int TAB, bool CRC = false, bool P2 = false>
__global__ __launch_bounds__(64 * kBsWaves) __attribute__((amdgpu_waves_per_eu(2, 2))) void gf_bs16_repair_kernel(
    const dev::GfArgs a, const BsRepairArgs r, uint32_t tiles_per_stripe, uint32_t ntiles) {
  static_assert(!(CRC && P2), "one checksum form per launch");
  using namespace dev;
  constexpr int MO = ND + M;  // output rows per stripe: missing data rows, 20 parity rows, extras
  constexpr int PF = CRC ? kRepPrefetchCrc : kRepPrefetch;
  constexpr int kWaveLds = (PF + kRepRing) * kBsWaveBytes;
  // one LDS array (a second __shared__ object can cost a vmcnt(0) before the first ds_read)
  __shared__ __attribute__((aligned(16))) uint8_t lds[kBsWaves * kWaveLds + (CRC ? kBsCrcLdsBytes : 0)];
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  uint8_t* pre = lds + wave * kWaveLds;
  uint8_t* ring = pre + PF * kBsWaveBytes;
  const uint32_t* ct = reinterpret_cast<const uint32_t*>(lds + kBsWaves * kWaveLds);
  const uint32_t nw = gridDim.x * kBsWaves;
  if constexpr (CRC) {  // the checksum tables, once per workgroup (before any wave may leave)
    uint32_t* ctw = reinterpret_cast<uint32_t*>(lds + kBsWaves * kWaveLds);
    for (uint32_t i = threadIdx.x; i < kBsCrcTabs * 8; i += blockDim.x)
      reinterpret_cast<u32x4*>(ctw)[i] = reinterpret_cast<const u32x4*>(r.ctab)[i];
    __syncthreads();
    // a wave's tiles of a stripe are W apart (per-stripe order below): the register's jump table moves
    // it 2048 W bytes on instead of 2048
    for (uint32_t i = threadIdx.x; i < 7 * 32; i += blockDim.x)
      ctw[kBsCrcTabR * 32 + i] = bs_mulmod((i & 31u) << (5 * (i >> 5)), r.xjump);
    __syncthreads();
  }
  if (blockIdx.x == 0)  // the checksum words the pass after this one accumulates into
    for (uint32_t i = threadIdx.x; i < a.nzw; i += blockDim.x) a.zw[i] = 0u;
  // affine batches: row i of stripe s at ptr[i] + s * sstride; TAB: at base + its table offset
  const auto row_ptr = [&](uint32_t s, int i) -> const uint8_t* {
    if constexpr (TAB == 2) {
      typedef const __attribute__((address_space(4))) uint32_t cu32;
      uint32_t w = __builtin_amdgcn_readfirstlane(s * (uint32_t)(kBsK + ND + M) + (uint32_t)i);
      asm volatile("" : "+s"(w));
      return r.base + ((cu32*)r.dtab)[w];  // a scalar load: the table is read-only for the launch
    } else if constexpr (TAB == 1) {
      return r.base + bs_kernarg_u32(s * (uint32_t)(kBsK + ND + M) + (uint32_t)i);
    } else if constexpr (CFSEC_BS_REP_RELOAD) {
      return bs_kernarg_ptr(i) + (int64_t)s * a.sstride;
    } else {
      return a.ptr[i] + (int64_t)s * a.sstride;
    }
  };
  const auto input = [&](uint32_t s, int i, uint32_t c) -> const uint8_t* {
    return row_ptr(s, i) + (size_t)c * kBsWaveBytes + lane * 16;
  };
  const auto output = [&](uint32_t s, int o, uint32_t c) -> uint8_t* {
    return const_cast<uint8_t*>(row_ptr(s, kBsK + o)) + (size_t)c * kBsWaveBytes + lane * 16;
  };
  const auto slot_ptr = [&](uint32_t s, int i, uint32_t c) -> const uint8_t* {  // data row i, or zeros
    const int src = a.src[i];
    return src < kBsK ? input(s, src, c) : r.zero + lane * 16;
  };
  const auto prefetch = [&](uint32_t t) {
    const uint32_t s = t / tiles_per_stripe, c = t % tiles_per_stripe;
#pragma unroll
    for (int i = 0; i < PF; ++i) bs_glds_row<kBsRepGlds>(slot_ptr(s, i, c), pre + i * kBsWaveBytes);
  };
  // tiles: every nw-th (t0 = the wave's index); CRC launches: per-stripe order (W waves per stripe,
  // each on every W-th tile of its stripes: one run of one row per wave for the Horner registers, +2 %
  // against the every-nw-th order on C5, profiles/r06/c5_perbid_order.txt; blocks of consecutive tiles,
  // round 5's CRC order, cost 8 %)
  constexpr bool kBlocked = CFSEC_BS_BLOCKED && !CRC;
  const uint32_t wid = blockIdx.x * kBsWaves + wave;
  const uint32_t per_wave = kBlocked ? (ntiles + nw - 1) / nw : 0;
  uint32_t t = kBlocked ? wid * per_wave : wid;
  const uint32_t t_end = kBlocked ? min(t + per_wave, ntiles) : ntiles, t_step = kBlocked ? 1u : nw;
  // CFSEC_BS_PERBID (timing probe, no checksum form): W = nw / stripes waves per stripe, wave (g, j)
  // on tiles j, j + W, ... of stripes g, g + nw / W, ... -- the order a per-row checksum run needs
  constexpr bool kPerBid = (CRC || CFSEC_BS_PERBID) && !kBlocked;
  const uint32_t nst = ntiles / tiles_per_stripe;
  const uint32_t pbW = kPerBid ? max(1u, min(tiles_per_stripe, nw / max(nst, 1u))) : 1u, pbG = nw / pbW;
  const auto next_tile = [&](uint32_t u) -> uint32_t {
    if constexpr (!kPerBid) return u + t_step;
    const uint32_t su = u / tiles_per_stripe, cu = u - su * tiles_per_stripe + pbW;
    if (cu < tiles_per_stripe) return su * tiles_per_stripe + cu;
    const uint32_t s2 = su + pbG;
    return s2 < nst ? s2 * tiles_per_stripe + (wid % pbW) : ntiles;
  };
  if constexpr (kPerBid) {
    if (wid / pbW >= pbG || wid % pbW >= tiles_per_stripe) return;
    t = (wid / pbW) * tiles_per_stripe + wid % pbW;
    if (t >= ntiles) return;
  }
  if (t >= t_end) return;
  prefetch(t);
  __builtin_amdgcn_s_waitcnt(bs_waitcnt_vm(0));
  // CRC: each checksummed row's Horner register (lane-wise), the rows' count, the segment's first tile
  uint32_t R[kBsCrcRows] = {};
  uint32_t ncrc = 0, seg_c0 = t % tiles_per_stripe;
  if constexpr (CRC) {
    ncrc = (uint32_t)ND + (uint32_t)__builtin_popcount(a.pstore);
    ncrc = __builtin_amdgcn_readfirstlane(ncrc);
  }
  (void)ncrc;
  (void)seg_c0;
  for (; t < t_end; t = next_tile(t)) {
    const uint32_t s = t / tiles_per_stripe, c = t % tiles_per_stripe;
    uint32_t x[128];
    uint32_t y[ND > 0 ? ND : 1][8];
#pragma unroll
    for (int i = PF; i < kBsK; ++i) bs_ld_row<kBsRepLdNt>(slot_ptr(s, i, c), &x[8 * i]);
#pragma unroll
    for (int q = 0; q < ND; ++q) bs_ld_row<kBsRepLdNt>(input(s, kBsK - ND + q, c), y[q]);
    // the prefetched slots were issued before everything since (in-order retirement)
    __builtin_amdgcn_s_waitcnt(bs_waitcnt_vm(2 * (kBsK - PF + ND)));
#pragma unroll
    for (int i = 0; i < PF; ++i) bs_lds_row(pre + i * kBsWaveBytes, lane, &x[8 * i]);
    __builtin_amdgcn_s_waitcnt(kBsWaitLgkm0);
    __builtin_amdgcn_sched_barrier(0);
    // which slots are present, one bit each, re-read per tile (opaque) like the row masks
    uint32_t present = 0;
#pragma unroll
    for (int i = 0; i < kBsK; ++i) present |= (a.src[i] < kBsK ? 1u : 0u) << i;
    present = __builtin_amdgcn_readfirstlane(present);
    if constexpr (CFSEC_BS_REP_RELOAD) asm volatile("" : "+s"(present));
#pragma unroll
    for (int i = 0; i < kBsK; ++i)
      if (CFSEC_BS_SKIPZ == 0 || (present >> i & 1)) bs_transpose8(&x[8 * i]);  // a missing slot's zeros need none
    if constexpr (BsEc16p20l2::Paired) bs_pair_basis<kBsK>(x);
    if constexpr (ND > 0) {
      // 2. syndromes of the stand-ins over the present data (missing slots are zero planes), in
      // bytes: the row's planes transposed back and XOR-ed into the stored copy
#pragma unroll
      for (int q = 0; q < ND; ++q) {
        uint32_t o[8];
        bs_row_ec16p20l2_rt(r.prow[q], x, o);
        bs_transpose8(o);
#pragma unroll
        for (int w = 0; w < 8; ++w) y[q][w] ^= o[w];
      }
      // 3. d = A^-1 s, stored, into its slot (the slot bytes re-read per tile, as the row masks)
      uint32_t slots = (uint32_t)r.slot[0] | (uint32_t)r.slot[1] << 8 | (uint32_t)r.slot[2] << 16 | (uint32_t)r.slot[3] << 24;
      if constexpr (CFSEC_BS_REP_RELOAD) asm volatile("" : "+s"(slots));
#pragma unroll
      for (int j = 0; j < ND; ++j) {
        const uint32_t slot_j = slots >> (8 * j) & 0xFFu;
        uint32_t d[8];
#pragma unroll
        for (int w = 0; w < 8; ++w) d[w] = 0u;
#pragma unroll
        for (int q = 0; q < ND; ++q) {
          uint32_t s0[8], s1[8], s2[8];
#pragma unroll
          for (int w = 0; w < 8; ++w) {
            s0[w] = y[q][w] & 0x07070707u;
            s1[w] = (y[q][w] >> 3) & 0x07070707u;
            s2[w] = (y[q][w] >> 6) & 0x03030303u;
          }
          bs_mul_acc8(d, s0, s1, s2, r.t01[j * 4 + q], r.t2[j * 4 + q]);
        }
        bs_st_rebuilt(output(s, j, c), d);
        bs_transpose8(d);
#pragma unroll
        for (int i = 0; i < kBsK; ++i) {
          // the slot held zero planes; in the paired basis the even slot of its pair holds the
          // pair's sum, which takes d too (both slots of a pair missing: d_even ^ d_odd there)
          const int e = BsEc16p20l2::Paired ? (i & ~1) : i;  // folds after the unroll
          if constexpr (CFSEC_BS_INS == 1) {
            if (i == slot_j) {  // uniform: one slot's moves
#pragma unroll
              for (int w = 0; w < 8; ++w) x[8 * e + w] ^= d[w];
              if (e != i)
#pragma unroll
                for (int w = 0; w < 8; ++w) x[8 * i + w] = d[w];
            }
          } else {
            const uint32_t m = i == slot_j ? ~0u : 0u;
#pragma unroll
            for (int w = 0; w < 8; ++w) x[8 * e + w] ^= d[w] & m;
            if (e != i)
#pragma unroll
              for (int w = 0; w < 8; ++w) x[8 * i + w] ^= d[w] & m;
          }
        }
      }
    }
    // ring: the first two compared rows; then the next tile's slots
    uint32_t pend = a.pcmp, q_issue = 0, q_read = 0;
    const auto issue_ring = [&]() {
      if (pend) {
        const int p = __builtin_ctz(pend);
        pend &= pend - 1;
        bs_glds_row<kBsRepGlds>(output(s, ND + p, c), ring + (q_issue % kRepRing) * kBsWaveBytes);
        ++q_issue;
      }
    };
    issue_ring();
    issue_ring();
    __builtin_amdgcn_sched_barrier(0);
    prefetch(next_tile(t) < t_end ? next_tile(t) : t);
    __builtin_amdgcn_sched_barrier(0);
    uint32_t diff = 0, first_bad = 0;
    (void)first_bad;
    // the row masks re-read per tile (opaque): hoisted, their 44 per-row conditions outlive the
    // SGPRs as 64-bit lane masks and come back through v_readlane
    uint32_t pst = a.pstore, pcm = a.pcmp;
    if constexpr (CFSEC_BS_REP_RELOAD) asm volatile("" : "+s"(pst), "+s"(pcm));
    bs_net_ec16p20l2<M>(x, [&](int p, uint32_t (&o)[8]) {
      if (pst >> p & 1) {
        bs_transpose8(o);
        bs_st_rebuilt(output(s, ND + p, c), o);
        if constexpr (CRC) {  // checksummed row ND + (stored parity rows before p)
          const uint32_t k = (uint32_t)ND + (uint32_t)__builtin_popcount(pst & ((1u << p) - 1u));
          __builtin_amdgcn_sched_barrier(0);  // in the middle of the network: no lookups hoisted into it
          const uint32_t u = bs_crc_tile_seq(ct, o);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int kk = ND; kk < kBsCrcRows; ++kk)
            if (k == (uint32_t)kk) R[kk] ^= u;
        }
      } else if (pcm >> p & 1) {
        // this row's copy; the next compared row's may still fly (anything issued between them is
        // waited for too: retirement is in order)
        if (q_issue - q_read > 1) __builtin_amdgcn_s_waitcnt(bs_waitcnt_vm(2));
        else __builtin_amdgcn_s_waitcnt(bs_waitcnt_vm(0));
        uint32_t v[8];
        bs_lds_row(ring + (q_read % kRepRing) * kBsWaveBytes, lane, v);
        __builtin_amdgcn_s_waitcnt(kBsWaitLgkm0);
        ++q_read;
        issue_ring();
        bs_transpose8(v);
        uint32_t dd = 0;
#pragma unroll
        for (int w = 0; w < 8; ++w) dd |= v[w] ^ o[w];
        if constexpr (CFSEC_BS_DEBUG_FLAGS)
          if (dd && !first_bad) first_bad = 0x80000000u | (uint32_t)p << 24 | (c & 0xFFFFFFu);
        diff |= dd;
      }
    });
    if (diff) {
      if constexpr (CFSEC_BS_DEBUG_FLAGS) __hip_atomic_store(a.flags + s, first_bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      else set_flag(a.flags, s);
    }
    if constexpr (CRC && ND > 0) {
      // the rebuilt data rows' checksums after the network, from their planes in x (kept as bytes
      // through the network they spill): an odd slot holds d, an even slot the pair sum d ^ x_odd
      uint32_t slots = (uint32_t)r.slot[0] | (uint32_t)r.slot[1] << 8;
      if constexpr (CFSEC_BS_REP_RELOAD) asm volatile("" : "+s"(slots));
#pragma unroll
      for (int j = 0; j < ND; ++j) {
        const uint32_t slot_j = slots >> (8 * j) & 0xFFu;
        uint32_t d[8];
#pragma unroll
        for (int w = 0; w < 8; ++w) d[w] = 0u;
#pragma unroll
        for (int i = 0; i < kBsK; ++i)
          if (i == slot_j) {  // uniform
#pragma unroll
            for (int w = 0; w < 8; ++w)
              d[w] = (BsEc16p20l2::Paired && !(i & 1)) ? x[8 * i + w] ^ x[8 * (i + 1) + w] : x[8 * i + w];
          }
        bs_transpose8(d);
        R[j] ^= bs_crc_tile_seq(ct, d);
      }
    }
    if constexpr (CRC) {
      const uint32_t tn = next_tile(t);
      if (tn >= t_end || tn / tiles_per_stripe != s) {
        // the segment [seg_c0, c] of stripe s: lanes folded, moved to the row's end, XOR-ed into the
        // row's word (the row's first segment also folds in shift(~0, S) ^ ~0)
        const uint32_t mv = r.cpow[tiles_per_stripe - 1 - c];
#pragma unroll
        for (int k = 0; k < kBsCrcRows; ++k) {
          if ((uint32_t)k < ncrc) {
            uint32_t v = bs_mulmod(bs_crc_lanes(ct, R[k], lane), mv);
            if (seg_c0 == 0) v ^= r.crc_ones;
            if (lane == 0) atomicXor(r.crcw + (size_t)s * r.crc_stride + r.crc_slot[k], v);
          }
          R[k] = 0u;
        }
        seg_c0 = tn % tiles_per_stripe;  // the next segment's first tile
      } else {
        // the next tile of this segment: every register moves 2048 W bytes on (the rebuilt jump table)
#pragma unroll
        for (int k = 0; k < kBsCrcRows; ++k)
          if ((uint32_t)k < ncrc) R[k] = bs_five7(ct + kBsCrcTabR * 32, R[k]);
      }
    }
  }
#ifndef CFSEC_BS_P2_PROBE
#define CFSEC_BS_P2_PROBE 0  // 1: plain stores for the atomics, 2: phase 2 skipped (timing probes only)
#endif
  if constexpr (P2 && CFSEC_BS_P2_PROBE != 2) {
    // phase 2: the checksummed rows of this wave's own tiles (written by its own stores above)
    // its stores and the last re-prefetch complete: the rows re-read below come from L2 (this CU never
    // read them before, so no L1 line is stale; an agent-scope acquire here -- an L2 invalidate per
    // wave -- measured +18 us on C5's call)
    __builtin_amdgcn_s_waitcnt(bs_waitcnt_vm(0));
    uint32_t* tb = reinterpret_cast<uint32_t*>(pre);     // tables A and B (56 x 32 words) in its own slice
    constexpr int kTabVec = (kBsCrcTabR - kBsCrcTabA) * 8;
    static_assert(kTabVec * 16 <= kWaveLds, "the tables fit the wave's LDS slice");
    for (uint32_t i = lane; i < (uint32_t)kTabVec; i += 64)
      reinterpret_cast<u32x4*>(tb)[i] = reinterpret_cast<const u32x4*>(r.ctab)[i];
    uint32_t col[32];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const u32x4 v = reinterpret_cast<const u32x4*>(r.lbasis + lane * 32)[q];
      col[4 * q] = v.x;
      col[4 * q + 1] = v.y;
      col[4 * q + 2] = v.z;
      col[4 * q + 3] = v.w;
    }
    __builtin_amdgcn_s_waitcnt(kBsWaitLgkm0);  // the table stores before any lane's lookups (one wave: in order)
    uint32_t pst = a.pstore;
    if constexpr (CFSEC_BS_REP_RELOAD) asm volatile("" : "+s"(pst));
    const uint32_t ncrc = __builtin_amdgcn_readfirstlane((uint32_t)ND + (uint32_t)__builtin_popcount(pst));
    int orow[kBsCrcRows];  // output row of checksummed row k: the rebuilt data rows, then the stored parities
    {
      uint32_t rest = pst;
#pragma unroll
      for (int k = 0; k < kBsCrcRows; ++k) {
        orow[k] = k;
        if (k >= ND && rest) {
          orow[k] = ND + __builtin_ctz(rest);
          rest &= rest - 1;
        }
      }
    }
    // a tile's checksummed rows, loaded one tile ahead (the re-reads' latency under the previous
    // tile's lookups)
    uint32_t cur[kBsCrcRows][8], nxt[kBsCrcRows][8];
    const auto load_tile = [&](uint32_t tt, uint32_t (&buf)[kBsCrcRows][8]) {
      const uint32_t s = tt / tiles_per_stripe, c = tt % tiles_per_stripe;
#pragma unroll
      for (int k = 0; k < kBsCrcRows; ++k)
        if ((uint32_t)k < ncrc) bs_ld_row<false>(output(s, orow[k], c), buf[k]);
    };
    if (wid < ntiles) load_tile(wid, cur);
    for (uint32_t t2 = wid; t2 < ntiles; t2 += nw) {
      if (t2 + nw < ntiles) load_tile(t2 + nw, nxt);
      const uint32_t s = t2 / tiles_per_stripe, c = t2 % tiles_per_stripe;
      uint32_t m[kBsCrcRows];
#pragma unroll
      for (int k = 0; k < kBsCrcRows; ++k) {
        m[k] = 0u;
        if ((uint32_t)k < ncrc) {
          const uint32_t u = bs_crc_tile(tb, cur[k]);
#pragma unroll
          for (int b = 0; b < 32; ++b) m[k] ^= (0u - ((u >> b) & 1u)) & col[b];  // the lane's term to the tile's end
        }
      }
      // the tile's end to the row's end, lane by lane (linear: the wave's sum moves the same), by the
      // tile's 32 columns in scalar registers -- a scalar bit-serial multiply per row and tile cost
      // 256 SALU, which one CU issues for all its waves (~13 us of C5's call)
      const uint32_t* cc = r.ccols + (size_t)(tiles_per_stripe - 1 - c) * 32;
      uint32_t scol[32];
#pragma unroll
      for (int b = 0; b < 32; ++b) scol[b] = __builtin_amdgcn_readfirstlane(cc[b]);
#pragma unroll
      for (int k = 0; k < kBsCrcRows; ++k) {
        uint32_t z = 0;
#pragma unroll
        for (int b = 0; b < 32; ++b) z ^= (0u - ((m[k] >> b) & 1u)) & scol[b];
        m[k] = z;
      }
      // the wave's sums, the rows' four reductions interleaved
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1)
#pragma unroll
        for (int k = 0; k < kBsCrcRows; ++k) m[k] ^= (uint32_t)__shfl_xor((int)m[k], d, 64);
#pragma unroll
      for (int k = 0; k < kBsCrcRows; ++k) {
        if ((uint32_t)k < ncrc) {
          uint32_t w = m[k];
          if (c == 0) w ^= r.crc_ones;
#if CFSEC_BS_P2_PROBE == 1  // timing probe only (wrong words): a plain store instead of the atomic
          if (lane == 0) r.crcw[(size_t)s * r.crc_stride + r.crc_slot[k]] = w;
#else
          if (lane == 0) atomicXor(r.crcw + (size_t)s * r.crc_stride + r.crc_slot[k], w);
#endif
        }
      }
#pragma unroll
      for (int k = 0; k < kBsCrcRows; ++k)
#pragma unroll
        for (int w = 0; w < 8; ++w) cur[k][w] = nxt[k][w];
    }
  }
  bs_drain_exit();
}

int cu_count() {
  static int n[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!n[dev]) {
    int v = 0;
    n[dev] = hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0 ? v : 256;
  }
  return n[dev];
}
}  // namespace

namespace {
template <class Net>
bool rows_match(const uint8_t* coef, int m) {
  const uint8_t* w = Net::rows();
  for (int i = 0; i < m * Net::K; ++i)
    if (coef[i] != w[i]) return false;
  return true;
}

template <class Net, int M, int TAB = 0>
hipError_t launch_net(const dev::GfArgs& a, unsigned grid, uint32_t tps, uint32_t nt, hipStream_t st,
                      BsTabArgs tb = {nullptr, nullptr}) {
  hipLaunchKernelGGL((gf_bs_kernel<Net, M, TAB>), dim3(grid), dim3(64 * kBsWaves), 0, st, a, tb, tps, nt);
  return hipGetLastError();
}
}  // namespace

// EC15P12 / EC12P9 networks (tools/gen_bs_net.py ec15p12 | ec12p9) run 13-23 % slower than the
// lookup-product kernel on their shapes (profiles/r04/bsk_ab.txt: 2-3 tiles per wave, and the row
// tails need a second launch), so only the 16 + 20 code takes this route.
bool bs_matches(const uint8_t* coef, int m, int k) {
  if (k == 16 && (m == 20 || m == 22)) return rows_match<dev::BsEc16p20l2>(coef, m);
  return false;
}

hipError_t launch_bs(int k, int m, const dev::GfArgs& a, unsigned ns, uint64_t len, hipStream_t st) {
  const uint32_t tps = (uint32_t)(len / dev::kBsWaveBytes);
  const uint64_t ntiles = (uint64_t)tps * ns;
  if (tps == 0 || ntiles > 0xFFFFFFFFull || (len % dev::kBsWaveBytes)) return hipErrorInvalidValue;
  const unsigned grid = (unsigned)std::min<uint64_t>((uint64_t)cu_count(), (ntiles + kBsWaves - 1) / kBsWaves);
  const uint32_t nt = (uint32_t)ntiles;
  if (k == 16 && m == 20) return launch_net<dev::BsEc16p20l2, 20>(a, grid, tps, nt, st);
  if (k == 16 && m == 22) return launch_net<dev::BsEc16p20l2, 22>(a, grid, tps, nt, st);
  return hipErrorInvalidValue;
}

namespace {
// kBsWaveBytes of zeros on the current device (the missing slots' loads), allocated once
const uint8_t* zero_tile() {
  static std::mutex mu;
  static const uint8_t* z[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> lk(mu);
  if (!z[dev]) {
    void* p = nullptr;
    if (hipMalloc(&p, dev::kBsWaveBytes) != hipSuccess) return nullptr;
    if (hipMemset(p, 0, dev::kBsWaveBytes) != hipSuccess) {
      (void)hipFree(p);
      return nullptr;
    }
    z[dev] = static_cast<const uint8_t*>(p);
  }
  return z[dev];
}

void coef_tables_host(uint8_t c, dev::u32x4& t01, uint32_t& t2) {  // gf_device.hpp coef_tables
  const GF& gf = GF::get();
  uint32_t p[8];
  p[0] = c;
  for (int j = 1; j < 8; ++j) p[j] = gf.mul((uint8_t)p[j - 1], 2);
  uint32_t t0lo = 0, t0hi = 0, t1lo = 0, t1hi = 0, tt2 = 0;
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
  t01 = dev::u32x4{t0lo, t0hi, t1lo, t1hi};
  t2 = tt2;
}

template <int M, int TAB, bool CRC = false, bool P2 = false>
hipError_t launch_rep_m(int nd, const dev::GfArgs& a, const BsRepairArgs& r, unsigned grid, uint32_t tps,
                        uint32_t nt, hipStream_t st) {
  switch (nd) {
    case 0:
      hipLaunchKernelGGL((gf_bs16_repair_kernel<M, 0, TAB, CRC, P2>), dim3(grid), dim3(64 * kBsWaves), 0, st, a, r, tps, nt);
      break;
    case 1:  // (no CRC form: one missing data row spills ~130 VGPRs with the checksums, the separate pass is faster)
      if constexpr (CRC) return hipErrorInvalidValue;
      else hipLaunchKernelGGL((gf_bs16_repair_kernel<M, 1, TAB, CRC, P2>), dim3(grid), dim3(64 * kBsWaves), 0, st, a, r, tps, nt);
      break;
    case 2:
      hipLaunchKernelGGL((gf_bs16_repair_kernel<M, 2, TAB, CRC, P2>), dim3(grid), dim3(64 * kBsWaves), 0, st, a, r, tps, nt);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// the repair launch with the checksum form r asks for (rep_crc_args): none, Horner in the network
// (crc mode 1), or the second phase (mode 2)
template <int M, int TAB>
hipError_t launch_rep_crc(int nd, int mode, const dev::GfArgs& a, const BsRepairArgs& r, unsigned grid, uint32_t tps,
                          uint32_t nt, hipStream_t st) {
  if (mode == 2) return launch_rep_m<M, TAB, false, true>(nd, a, r, grid, tps, nt, st);
  if (mode == 1) return launch_rep_m<M, TAB, true>(nd, a, r, grid, tps, nt, st);
  return launch_rep_m<M, TAB>(nd, a, r, grid, tps, nt, st);
}

// ---- host side of the fused checksums (bs_crc_tile / bs_crc_lanes) ----
uint32_t crc_mulmod(uint32_t a, uint32_t b) {  // reflected: bit 31 = x^0
  uint32_t p = 0;
  for (uint32_t bit = 0x80000000u; bit; bit >>= 1) {
    if (a & bit) p ^= b;
    b = (b >> 1) ^ ((b & 1u) ? kBsCrcPoly : 0u);
  }
  return p;
}
uint32_t crc_xpow(uint64_t e) {  // x^e mod P
  uint32_t base = 0x40000000u, p = 0x80000000u;
  for (; e; e >>= 1) {
    if (e & 1) p = crc_mulmod(p, base);
    base = crc_mulmod(base, base);
  }
  return p;
}
// f(0, the 16-byte piece whose word w is v, the rest 0)
uint32_t crc_piece_word(int w, uint32_t v) {
  uint32_t c = 0;
  for (int i = 0; i < 16; ++i) {
    c ^= i / 4 == w ? (v >> (8 * (i % 4))) & 0xFFu : 0u;
    for (int q = 0; q < 8; ++q) c = (c & 1u) ? (c >> 1) ^ kBsCrcPoly : c >> 1;
  }
  return c;
}
// kBsCrcTabs tables of 32 words, table (g, f) at (g * 7 + f) * 32 for field f (bits 5f..) of word g:
// a pieces (their image moved 1024 bytes on), b pieces, the register moved 2048 bytes on, and the
// lane tree's levels (moved 16 * 2^k bytes on)
std::vector<uint32_t> bs_crc_host_tables() {
  std::vector<uint32_t> t((size_t)kBsCrcTabs * 32, 0u);
  const uint32_t k1024 = crc_xpow(8 * 1024), k2048 = crc_xpow(8 * 2048);
  for (int f = 0; f < 7; ++f)
    for (uint32_t e = 0; e < (f < 6 ? 32u : 4u); ++e) {
      const uint32_t v = e << (5 * f);
      for (int w = 0; w < 4; ++w) {
        const uint32_t img = crc_piece_word(w, v);
        t[(size_t)((kBsCrcTabA + 7 * w + f) * 32 + e)] = crc_mulmod(k1024, img);
        t[(size_t)((kBsCrcTabB + 7 * w + f) * 32 + e)] = img;
      }
      t[(size_t)((kBsCrcTabR + f) * 32 + e)] = crc_mulmod(k2048, v);
      for (int k = 0; k < 6; ++k) t[(size_t)((kBsCrcTabTree + 7 * k + f) * 32 + e)] = crc_mulmod(crc_xpow(8ull * (16u << k)), v);
    }
  return t;
}

// the tables on the current device (uploaded once), and x^(8 * 2048 * j), j < tps (once per tps)
struct BsCrcDev {
  std::mutex mu;
  uint32_t* tab = nullptr;
  uint32_t* lbasis = nullptr;
  std::map<uint32_t, uint32_t*> pow, cols;
};
hipError_t bs_crc_device(uint32_t tps, const uint32_t** tab, const uint32_t** pw, const uint32_t** lbasis,
                         const uint32_t** ccols) {
  static BsCrcDev per[64];
  int d = 0;
  hipError_t e = hipGetDevice(&d);
  if (e != hipSuccess) return e;
  if (d < 0 || d >= 64) return hipErrorInvalidDevice;
  BsCrcDev& c = per[d];
  std::lock_guard<std::mutex> lk(c.mu);
  if (!c.tab) {
    const std::vector<uint32_t> h = bs_crc_host_tables();
    uint32_t* p = nullptr;
    if ((e = hipMalloc(reinterpret_cast<void**>(&p), h.size() * 4)) != hipSuccess) return e;
    if ((e = hipMemcpy(p, h.data(), h.size() * 4, hipMemcpyHostToDevice)) != hipSuccess) {
      (void)hipFree(p);
      return e;
    }
    c.tab = p;
  }
  if (!c.lbasis) {  // lane l: the columns (bit b of a word) of the multiply by x^(8 * 16 * (63 - l))
    std::vector<uint32_t> h(64 * 32);
    for (int l = 0; l < 64; ++l) {
      const uint32_t k = crc_xpow(8ull * 16 * (63 - l));
      for (int b = 0; b < 32; ++b) h[(size_t)l * 32 + b] = crc_mulmod(k, 1u << b);
    }
    uint32_t* p = nullptr;
    if ((e = hipMalloc(reinterpret_cast<void**>(&p), h.size() * 4)) != hipSuccess) return e;
    if ((e = hipMemcpy(p, h.data(), h.size() * 4, hipMemcpyHostToDevice)) != hipSuccess) {
      (void)hipFree(p);
      return e;
    }
    c.lbasis = p;
  }
  auto it = c.pow.find(tps);
  if (it == c.pow.end()) {
    std::vector<uint32_t> h(tps);
    const uint32_t k = crc_xpow(8ull * 2048);
    uint32_t v = 0x80000000u;  // x^0
    for (uint32_t j = 0; j < tps; ++j, v = crc_mulmod(v, k)) h[j] = v;
    uint32_t* p = nullptr;
    if ((e = hipMalloc(reinterpret_cast<void**>(&p), (size_t)tps * 4)) != hipSuccess) return e;
    if ((e = hipMemcpy(p, h.data(), (size_t)tps * 4, hipMemcpyHostToDevice)) != hipSuccess) {
      (void)hipFree(p);
      return e;
    }
    it = c.pow.emplace(tps, p).first;
  }
  auto jt = c.cols.find(tps);
  if (jt == c.cols.end()) {  // tile j: the columns (bit b) of the multiply by x^(8 * 2048 * j)
    std::vector<uint32_t> h((size_t)tps * 32);
    const uint32_t k = crc_xpow(8ull * 2048);
    uint32_t v = 0x80000000u;
    for (uint32_t j = 0; j < tps; ++j, v = crc_mulmod(v, k))
      for (int b = 0; b < 32; ++b) h[(size_t)j * 32 + b] = crc_mulmod(v, 1u << b);
    uint32_t* p = nullptr;
    if ((e = hipMalloc(reinterpret_cast<void**>(&p), h.size() * 4)) != hipSuccess) return e;
    if ((e = hipMemcpy(p, h.data(), h.size() * 4, hipMemcpyHostToDevice)) != hipSuccess) {
      (void)hipFree(p);
      return e;
    }
    jt = c.cols.emplace(tps, p).first;
  }
  *tab = c.tab;
  *pw = it->second;
  *lbasis = c.lbasis;
  *ccols = jt->second;
  return hipSuccess;
}

// the CRC fields of a repair launch, or false (not eligible: more than kBsCrcRows checksummed rows,
// a zeroing request the atomics would race with, too many tiles per stripe for the table)
bool rep_crc_args(int nd, const dev::GfArgs& a, uint64_t len, const BsCrcReq* crc, uint32_t* words, BsRepairArgs& r) {
  if (!crc || !words || a.nzw || (nd == 1 && crc->mode == 1) || (crc->mode != 1 && crc->mode != 2)) return false;
  const int ncrc = nd + __builtin_popcount(a.pstore);
  if (ncrc != crc->nrows || ncrc > kBsCrcRows || len % dev::kBsWaveBytes || len / dev::kBsWaveBytes > (1u << 20))
    return false;
  const uint32_t tps = (uint32_t)(len / dev::kBsWaveBytes);
  if (bs_crc_device(tps, &r.ctab, &r.cpow, &r.lbasis, &r.ccols) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  r.crcw = words;
  r.crc_stride = crc->stride;
  r.crc_ones = crc32_shift_ones((size_t)len);
  for (int k = 0; k < 4; ++k) r.crc_slot[k] = crc->slot[k];
  return true;
}

// x^(8 * 2048 * W) for a CRC launch of `grid` workgroups: W waves per stripe, as the kernel computes it
uint32_t bs_rep_xjump(unsigned grid, uint32_t tps, uint64_t ntiles) {
  const uint64_t nw = (uint64_t)grid * kBsWaves, nst = tps ? ntiles / tps : 0;
  const uint64_t W = std::max<uint64_t>(1, std::min<uint64_t>(tps, nw / std::max<uint64_t>(nst, 1)));
  return crc_xpow(8ull * 2048 * W);
}

bool rep_args(int nd, const uint8_t* missing, const uint8_t* prow, const uint8_t* ainv, BsRepairArgs& r) {
  for (int q = 0; q < nd; ++q) {
    r.slot[q] = missing[q];
    r.prow[q] = prow[q];
    for (int j = 0; j < nd; ++j) coef_tables_host(ainv[j * 4 + q], r.t01[j * 4 + q], r.t2[j * 4 + q]);
  }
  r.zero = zero_tile();
  return r.zero != nullptr;
}
}  // namespace

hipError_t launch_bs16_repair(int nd, int ne, const uint8_t* missing, const uint8_t* prow, const uint8_t* ainv,
                              const dev::GfArgs& a, unsigned ns, uint64_t len, hipStream_t st, const BsCrcReq* crc,
                              uint32_t* crc_words, bool* crc_done) {
  const uint32_t tps = (uint32_t)(len / dev::kBsWaveBytes);
  const uint64_t ntiles = (uint64_t)tps * ns;
  if (crc_done) *crc_done = false;
  if (nd < 0 || nd > kBsRepairMaxNd || (ne != 0 && ne != 2) || a.tab != 1 || tps == 0 || ntiles > 0xFFFFFFFFull ||
      (len % dev::kBsWaveBytes) || (a.pcmp && !a.flags))
    return hipErrorInvalidValue;
  BsRepairArgs r{};
  if (!rep_args(nd, missing, prow, ainv, r)) return hipErrorOutOfMemory;
  const unsigned grid = (unsigned)std::min<uint64_t>((uint64_t)cu_count(), (ntiles + kBsWaves - 1) / kBsWaves);
  if (rep_crc_args(nd, a, len, crc, crc_words, r)) {
    r.xjump = bs_rep_xjump(grid, tps, ntiles);
    const hipError_t e = ne == 2 ? launch_rep_crc<22, 0>(nd, crc->mode, a, r, grid, tps, (uint32_t)ntiles, st)
                                 : launch_rep_crc<20, 0>(nd, crc->mode, a, r, grid, tps, (uint32_t)ntiles, st);
    if (e == hipSuccess && crc_done) *crc_done = true;
    return e;
  }
  return ne == 2 ? launch_rep_m<22, 0>(nd, a, r, grid, tps, (uint32_t)ntiles, st)
                 : launch_rep_m<20, 0>(nd, a, r, grid, tps, (uint32_t)ntiles, st);
}

int bs_tab_stripes(int mo) { return kBsTabWords / (kBsK + mo); }

// The row-offset tables (TAB 2: any number of stripes in one launch): a ring of kBsDevTables per
// device, each slot a table in mapped, coherent host memory that the kernel reads directly (no copy
// launch: a blit copy into a device twin, read through another XCD's L2 by the next kernel's scalar
// loads, is the one cross-launch hand-off this path had, and round 4's and round 5's false Verify
// flags on the scattered layout came only from it; the direct read measured the same time per call,
// profiles/r05/scattered_c5_upload.txt "host"), free again once the launch that read it has
// completed (its event, polled).  A launch takes a free slot without
// waiting; only when every slot is still in flight -- the host kBsDevTables launches ahead of the
// GPU, e.g. back-to-back asynchronous tasklets -- does it wait for the oldest one, a bounded queue's
// backpressure (the argument-block fallback measured 0.147 -> 0.205 ms per scattered C5 call when
// taken instead).  CFSEC_BS_DTAB=0 keeps the argument-block table (A/B).
#ifndef CFSEC_BS_DTAB
#define CFSEC_BS_DTAB 1
#endif
constexpr int kBsDevTables = 8;
constexpr size_t kBsDevTableMin = 64 * 1024;  // words per slot: growth (a hipFree) stays rare
struct BsDevTable {
  uint32_t* host = nullptr;
  uint32_t* dev = nullptr;
  size_t cap = 0;
  hipEvent_t done = nullptr;
  bool pending = false;
  bool dead = false;  // a launch may still read it and no event says when it ends: never reused
  uint64_t seq = 0;   // when it was last taken
};
struct BsDevTables {
  std::mutex mu;
  BsDevTable slot[kBsDevTables];
  uint64_t next = 0;
};

BsDevTables* dev_tables() {
  static BsDevTables t[64];
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= 64) return nullptr;
  return &t[d];
}

// A free slot with room for n words (under the ring's mutex) -- with every slot in flight, the oldest
// once its launch completes -- or nullptr (no memory, a failed event)
BsDevTable* dev_table_reserve(BsDevTables& r, size_t n) {
  BsDevTable* t = nullptr;
  BsDevTable* oldest = nullptr;
  for (BsDevTable& c : r.slot) {
    if (c.dead) continue;
    if (c.pending) {
      const hipError_t q = hipEventQuery(c.done);
      if (q == hipErrorNotReady) {
        if (!oldest || c.seq < oldest->seq) oldest = &c;
        continue;
      }
      if (q != hipSuccess) return nullptr;
      c.pending = false;
    }
    if (!t || (t->cap < n && c.cap >= n)) t = &c;  // prefer a slot that needs no growth
    if (t->cap >= n) break;
  }
  if (!t && oldest) {  // the host is kBsDevTables launches ahead: wait for the oldest
    if (hipEventSynchronize(oldest->done) != hipSuccess) return nullptr;
    oldest->pending = false;
    t = oldest;
  }
  if (!t) return nullptr;
  t->seq = ++r.next;
  if (!t->done && hipEventCreateWithFlags(&t->done, hipEventDisableTiming) != hipSuccess) return nullptr;
  if (n <= t->cap) return t;
  if (t->host) (void)hipHostFree(t->host);
  t->host = nullptr;
  t->dev = nullptr;
  t->cap = 0;
  const size_t cap = std::max<size_t>(n, kBsDevTableMin);
  if (hipHostMalloc(reinterpret_cast<void**>(&t->host), cap * 4, hipHostMallocMapped | hipHostMallocCoherent) !=
      hipSuccess)
    return nullptr;
  if (hipHostGetDevicePointer(reinterpret_cast<void**>(&t->dev), t->host, 0) != hipSuccess) {
    (void)hipGetLastError();
    (void)hipHostFree(t->host);
    t->host = nullptr;
    return nullptr;
  }
  t->cap = cap;
  return t;
}

// After a launch that reads dt's table: the event that frees the slot.  If it cannot be recorded the
// launch may still be reading the row offsets, so the slot is not handed out again before the stream
// has drained (or ever, when even that fails) -- a later reservation would rewrite the mapped table
// under the kernel.
hipError_t dev_table_fence(BsDevTable* dt, hipStream_t st) {
  const hipError_t e = hipEventRecord(dt->done, st);
  if (e == hipSuccess) {
    dt->pending = true;
    return hipSuccess;
  }
  if (hipStreamSynchronize(st) != hipSuccess) dt->dead = true;
  return e;
}

hipError_t launch_bs16_repair_tab(int nd, int ne, const uint8_t* missing, const uint8_t* prow, const uint8_t* ainv,
                                  const dev::GfArgs& a, const uint8_t* const* rows, unsigned ns, uint64_t len,
                                  hipStream_t st, bool* ok, const BsCrcReq* crc, uint32_t* crc_words,
                                  bool* crc_done) {
  const int mo = nd + 20 + ne, per = bs_tab_stripes(mo);
  const uint32_t tps = (uint32_t)(len / dev::kBsWaveBytes);
  *ok = false;
  if (crc_done) *crc_done = false;
  if (nd < 0 || nd > kBsRepairMaxNd || (ne != 0 && ne != 2) || tps == 0 || (len % dev::kBsWaveBytes) ||
      (a.pcmp && !a.flags) || !rows || ns == 0)
    return hipErrorInvalidValue;
  const size_t nrows = (size_t)ns * (kBsK + mo);
  uintptr_t lo = ~(uintptr_t)0, hi = 0;
  for (size_t i = 0; i < nrows; ++i) {
    lo = std::min(lo, (uintptr_t)rows[i]);
    hi = std::max(hi, (uintptr_t)rows[i]);
  }
  if (hi - lo > 0xFFFFFFFFull) return hipSuccess;  // not ok: the caller keeps its route
  *ok = true;
  BsRepairArgs r{};
  if (!rep_args(nd, missing, prow, ainv, r)) return hipErrorOutOfMemory;
  r.base = reinterpret_cast<const uint8_t*>(lo);
  static thread_local dev::GfArgs t;
  std::memcpy(&t, &a, sizeof(dev::GfArgs));
  t.sstride = 0;
  t.tab = 1;
  if (BsDevTables* ring = CFSEC_BS_DTAB && ns > (unsigned)per ? dev_tables() : nullptr) {
    std::lock_guard<std::mutex> lk(ring->mu);
    if (BsDevTable* dt = dev_table_reserve(*ring, nrows)) {
      for (size_t i = 0; i < nrows; ++i) dt->host[i] = (uint32_t)((uintptr_t)rows[i] - lo);
      std::atomic_thread_fence(std::memory_order_release);  // the table before the launch that reads it
      hipError_t e = hipSuccess;
      r.dtab = dt->dev;
      t.nstripes = ns;
      const uint64_t ntiles = (uint64_t)tps * ns;
      if (ntiles > 0xFFFFFFFFull) return hipErrorInvalidValue;
      const unsigned grid = (unsigned)std::min<uint64_t>((uint64_t)cu_count(), (ntiles + kBsWaves - 1) / kBsWaves);
      const bool fused = rep_crc_args(nd, t, len, crc, crc_words, r);
      const int mode = fused ? crc->mode : 0;
      r.xjump = bs_rep_xjump(grid, tps, ntiles);
      e = ne == 2 ? launch_rep_crc<22, 2>(nd, mode, t, r, grid, tps, (uint32_t)ntiles, st)
                  : launch_rep_crc<20, 2>(nd, mode, t, r, grid, tps, (uint32_t)ntiles, st);
      if (e != hipSuccess) return e;
      if (fused && crc_done) *crc_done = true;
      return dev_table_fence(dt, st);
    }
  }
  for (unsigned s0 = 0; s0 < ns; s0 += (unsigned)per) {
    const unsigned n = std::min<unsigned>((unsigned)per, ns - s0);
    uint32_t off[kBsTabWords];
    for (size_t i = 0; i < (size_t)n * (kBsK + mo); ++i)
      off[i] = (uint32_t)((uintptr_t)rows[(size_t)s0 * (kBsK + mo) + i] - lo);
    std::memcpy(reinterpret_cast<uint8_t*>(&t) + kBsTabOff, off, (size_t)n * (kBsK + mo) * 4);
    t.flags = a.flags ? a.flags + s0 : nullptr;
    t.nstripes = n;
    const uint64_t ntiles = (uint64_t)tps * n;
    const unsigned grid = (unsigned)std::min<uint64_t>((uint64_t)cu_count(), (ntiles + kBsWaves - 1) / kBsWaves);
    const hipError_t e = ne == 2 ? launch_rep_m<22, 1>(nd, t, r, grid, tps, (uint32_t)ntiles, st)
                                 : launch_rep_m<20, 1>(nd, t, r, grid, tps, (uint32_t)ntiles, st);
    if (e != hipSuccess) return e;
    t.zw = nullptr;  // the first launch zeroed them
    t.nzw = 0;
  }
  return hipSuccess;
}


hipError_t launch_bs_tab(int k, int m, const dev::GfArgs& a, const uint8_t* const* rows, unsigned ns, uint64_t len,
                         hipStream_t st, bool* ok) {
  *ok = false;
  const uint32_t tps = (uint32_t)(len / dev::kBsWaveBytes);
  const uint64_t ntiles = (uint64_t)tps * ns;
  if (k != 16 || (m != 20 && m != 22) || tps == 0 || ntiles > 0xFFFFFFFFull || (len % dev::kBsWaveBytes) || !rows ||
      ns == 0)
    return hipErrorInvalidValue;
  const size_t nrows = (size_t)ns * (k + m);
  uintptr_t lo = ~(uintptr_t)0, hi = 0;
  for (size_t i = 0; i < nrows; ++i) {
    lo = std::min(lo, (uintptr_t)rows[i]);
    hi = std::max(hi, (uintptr_t)rows[i]);
  }
  if (hi - lo > 0xFFFFFFFFull) return hipSuccess;  // not ok: the caller keeps its route
  BsDevTables* ring = dev_tables();
  if (!ring) return hipSuccess;
  std::lock_guard<std::mutex> lk(ring->mu);
  BsDevTable* dt = dev_table_reserve(*ring, nrows);
  if (!dt) return hipSuccess;  // not ok: every table in flight, the caller keeps its route
  for (size_t i = 0; i < nrows; ++i) dt->host[i] = (uint32_t)((uintptr_t)rows[i] - lo);
  std::atomic_thread_fence(std::memory_order_release);  // the table before the launch that reads it
  *ok = true;
  static thread_local dev::GfArgs t;
  std::memcpy(&t, &a, sizeof(dev::GfArgs));
  t.sstride = 0;
  t.tab = 1;
  t.nstripes = ns;
  const BsTabArgs tb{reinterpret_cast<const uint8_t*>(lo), dt->dev};
  const unsigned grid = (unsigned)std::min<uint64_t>((uint64_t)cu_count(), (ntiles + kBsWaves - 1) / kBsWaves);
  hipError_t e = m == 22 ? launch_net<dev::BsEc16p20l2, 22, 2>(t, grid, tps, (uint32_t)ntiles, st, tb)
                         : launch_net<dev::BsEc16p20l2, 20, 2>(t, grid, tps, (uint32_t)ntiles, st, tb);
  if (e != hipSuccess) return e;
  return dev_table_fence(dt, st);
}

}  // namespace cfsec
