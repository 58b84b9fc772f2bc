// crc32.hip -- standalone shard CRC32-IEEE on gfx950: Go's crc32.ChecksumIEEE of each shard
// (reflected polynomial 0xEDB88320, register preset ~0, final inversion), for shards no coding
// kernel touches -- cfsec_crc32_ieee_batch, and the checksum pass after a product whose shape
// the fused kernel (gf_crc.hpp) does not cover.
//
// Same algebra and work split as the fused kernel, without the product: a workgroup owns `tpw`
// consecutive 4 KiB tiles of one shard, thread j a 16-byte piece of each (coalesced 16-B loads,
// the next tile's piece in flight while this one is folded), Horner R <- f(shift(R, 4080), piece)
// with the conflict-free nibble tables (gf_crc.hpp crc_step_nib), a per-thread basis multiply to the tile end, a workgroup XOR
// reduction and one multiply by x^(8(S - e)) to the shard end, then atomicXor into the shard's
// word.  `fin` (crc32_shift_ones(S), or 0 for the raw word) is folded in by workgroup 0.
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "gf_crc.hpp"
#include "kernels.hpp"

namespace cfsec {
namespace {

using crcdev::kBasisWords;
using crcdev::kMaxGroups;
using crcdev::kTabWords;
using crcdev::kTile;
using dev::u32x4;
// Argument block: the fixed fields, then a flexible area of words holding the group constants
// gconst[0 .. ng) (x^(8(len - e_g)) mod P, the same for every shard) followed by the shard pointers
// and their output words: a launch carries as many shards as fit beside its ng constants (256 shards
// at ng = 16: a repair tasklet's rebuilt rows in one launch).
constexpr int kFlexWords = 800;

struct __attribute__((aligned(16))) CrcArgs {
  uint64_t len;
  int64_t sstride;               // affine list: shard i at ptr[0] + i*sstride, word idx[0] + i
  uint32_t tiles, tpw;
  uint32_t* out;
  const uint32_t* tabs;
  uint32_t fin, ng;              // ng: workgroups per shard (group constants in flex[0 .. ng))
  uint32_t pw, iw;               // word offsets of the pointer (8-byte) and index arrays in flex
  uint32_t pad[2];
  uint32_t flex[kFlexWords];
};
static_assert(sizeof(CrcArgs) <= 3584, "kernel argument block must stay below 4 KiB");

__device__ __forceinline__ const uint8_t* shard_ptr(const CrcArgs& a, uint32_t i) {
  return reinterpret_cast<const uint8_t* const*>(a.flex + a.pw)[i];
}

#ifndef CFSEC_CRC_LDNT
#define CFSEC_CRC_LDNT 1  // shard loads non-temporal (A/B: rows a repair pass just wrote)
#endif
__device__ __forceinline__ void piece(const uint8_t* p, uint64_t len, uint32_t off, uint32_t (&d)[4]) {
  if ((uint64_t)off + dev::kLaneBytes <= len) {
    const u32x4 v = dev::ld16<CFSEC_CRC_LDNT != 0>(p + off);
    d[0] = v.x, d[1] = v.y, d[2] = v.z, d[3] = v.w;
  } else {
    const size_t rem = off < len ? (size_t)(len - off) : 0;  // zero padding past the shard end
    const u32x4 v = rem ? dev::ld_tail_row(p + off, rem, len) : u32x4{0u, 0u, 0u, 0u};
    d[0] = v.x, d[1] = v.y, d[2] = v.z, d[3] = v.w;
  }
}

// The loads of CFSEC_CRC_AHEAD tiles are issued before any of them is folded (each thread's pieces
// are independent loads; only the fold is a chain), so short runs -- a repair tasklet's 256 rebuilt
// shards of 64 tiles, 8 per workgroup -- keep 8 loads per thread in flight instead of one.
// CFSEC_CRC_DIAG (timing probes only, wrong words): 1 drops the alignment-basis multiply, 2 the fold
#ifndef CFSEC_CRC_DIAG
#define CFSEC_CRC_DIAG 0
#endif
#ifndef CFSEC_CRC_AHEAD
#define CFSEC_CRC_AHEAD 8
#endif
__global__ __launch_bounds__(256) void crc32_horner_kernel(const CrcArgs a) {
  constexpr int A = CFSEC_CRC_AHEAD;
  __shared__ uint32_t ct[crcdev::kOnlyTabWords];
  __shared__ uint32_t red[4];
  for (int i = threadIdx.x; i < crcdev::kOnlyTabWords; i += 256) ct[i] = a.tabs[crcdev::kOnlyTabBase + i];
  __syncthreads();
  const uint32_t g = blockIdx.x, sh = blockIdx.y;
  const uint8_t* p = a.sstride ? shard_ptr(a, 0) + (int64_t)sh * a.sstride : shard_ptr(a, sh);
  const uint32_t t0 = g * a.tpw, t1 = min(t0 + a.tpw, a.tiles);
  const uint32_t lanepos = threadIdx.x * dev::kLaneBytes;
  uint32_t R = 0;
  for (uint32_t t = t0; t < t1; t += A) {
    uint32_t buf[A][4];
#pragma unroll
    for (int k = 0; k < A; ++k)
      if (t + k < t1) piece(p, a.len, (t + k) * kTile + lanepos, buf[k]);
#pragma unroll
    for (int k = 0; k < A; ++k)
      if (t + k < t1) {
#if CFSEC_CRC_DIAG == 2
        R = (R << 1 | R >> 31) ^ buf[k][0] ^ buf[k][1] ^ buf[k][2] ^ buf[k][3];
#else
        R = crcdev::only_step(ct, R, buf[k]);
#endif
      }
  }
  const u32x4* basis = reinterpret_cast<const u32x4*>(a.tabs + kTabWords + threadIdx.x * 32);
  uint32_t o = 0;
#if CFSEC_CRC_DIAG == 1
  o = R;
#else
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const u32x4 v = basis[q];
    o ^= (0u - ((R >> (4 * q)) & 1u)) & v.x;
    o ^= (0u - ((R >> (4 * q + 1)) & 1u)) & v.y;
    o ^= (0u - ((R >> (4 * q + 2)) & 1u)) & v.z;
    o ^= (0u - ((R >> (4 * q + 3)) & 1u)) & v.w;
  }
#endif
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) o ^= (uint32_t)__shfl_xor((int)o, d);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = o;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t v = crcdev::mulmod(a.flex[g], red[0] ^ red[1] ^ red[2] ^ red[3]);
    if (g == 0) v ^= a.fin;
    const uint32_t* idx = a.flex + a.iw;
    atomicXor(a.out + (a.sstride ? idx[0] + sh : idx[sh]), v);
  }
}

// CFSEC_CRC32_GROUPS_PROBE: re-read on every launch (A/B of the workgroup count in one process)
uint32_t probe_groups() {
  const char* v = std::getenv("CFSEC_CRC32_GROUPS_PROBE");
  return v && *v ? (uint32_t)std::strtoul(v, nullptr, 10) : 0u;
}

}  // namespace

hipError_t launch_crc32_to(const uint8_t* const* ptrs, size_t len, int n, uint32_t* out, const uint32_t* idx,
                           uint32_t fin, hipStream_t stream) {
  if (len == 0 || n == 0) return hipSuccess;
  if (len > 0xFFFFFFFFull - kTile || !ptrs || !out) return hipErrorInvalidValue;
  CrcArgs a{};
  hipError_t e = crc_device_tables(&a.tabs);
  if (e != hipSuccess) return e;
  const uint32_t tiles = (uint32_t)((len + kTile - 1) / kTile);
  // one launch for an equally spaced list (a pitched stripe batch) with consecutive words
  const auto at = [&](int i) { return (int64_t)(uintptr_t)ptrs[i]; };
  int64_t stride = n > 1 ? at(1) - at(0) : 0;
  for (int i = 1; i < n && stride; ++i)
    if (at(i) - at(0) != stride * i || (idx && idx[i] != idx[0] + (uint32_t)i)) stride = 0;
  if (n > 65535) stride = 0;
  // ~4096 workgroups in all, but each folding >= 16 tiles: its fixed cost (the 32-word alignment
  // basis of every thread, 32 KiB from L2, and the step table) must not outweigh its tiles.  Round 3,
  // event-timed (tools/crc_pass_probe.hip, profiles/r03/crc_pass.txt): a tasklet's 256 rebuilt rows
  // of 64 tiles 21 us at 4 workgroups per row vs 34 us at 16; 128 rows of 1366 tiles 126 us at 32
  // per row (5.67 TB/s) vs 132-134 at 8-16.  Then as many shards per launch as fit beside the group
  // constants.
  const uint32_t total = probe_groups() ? probe_groups() : 4096u;
  const uint32_t want = std::max<uint32_t>(1, std::min<uint32_t>(total / (uint32_t)n, tiles / 16));
  uint32_t groups = std::min<uint32_t>({tiles, want, (uint32_t)kMaxGroups});
  const uint32_t tpw = (tiles + groups - 1) / groups;
  groups = (tiles + tpw - 1) / tpw;
  const uint32_t pw = (groups + 1) & ~1u;                       // pointers 8-byte aligned
  const int slots = (int)((kFlexWords - pw) / 3);              // 2 words of pointer + 1 of index
  const int per_launch = stride ? n : std::min(n, slots);
  a.len = len;
  a.sstride = stride;
  a.tiles = tiles;
  a.tpw = tpw;
  a.out = out;
  a.fin = fin;
  a.ng = groups;
  a.pw = pw;
  a.iw = pw + 2 * (uint32_t)(stride ? 1 : per_launch);
  for (uint32_t g = 0; g < groups; ++g) {
    const int64_t end = (int64_t)std::min<uint64_t>((uint64_t)(g + 1) * tpw, tiles) * kTile;
    a.flex[g] = crc_xpow(8 * ((int64_t)len - end));
  }
  for (int s0 = 0; s0 < n; s0 += per_launch) {
    const int ns = std::min(per_launch, n - s0);
    const uint8_t** pp = reinterpret_cast<const uint8_t**>(a.flex + a.pw);
    uint32_t* ip = a.flex + a.iw;
    for (int s = 0; s < (stride ? 1 : ns); ++s) {
      pp[s] = ptrs[s0 + s];
      ip[s] = idx ? idx[s0 + s] : (uint32_t)(s0 + s);
    }
    hipLaunchKernelGGL(crc32_horner_kernel, dim3(groups, (unsigned)ns), dim3(256), 0, stream, a);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_crc32(const uint8_t* const* ptrs, size_t len, int n, uint32_t* out,
                        hipStream_t stream) {
  hipError_t e = hipMemsetAsync(out, 0, sizeof(uint32_t) * (size_t)n, stream);
  if (e != hipSuccess) return e;
  return launch_crc32_to(ptrs, len, n, out, nullptr, 0u, stream);
}

uint32_t crc32_finalize(uint32_t raw, size_t len) {
  if (len == 0) return 0;
  return raw ^ crc32_shift_ones(len);
}

}  // namespace cfsec
