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
constexpr int kSlots = 160;

struct __attribute__((aligned(16))) CrcArgs {
  uint64_t len;
  int64_t sstride;               // affine list: shard i at ptr[0] + i*sstride, word idx[0] + i
  uint32_t tiles, tpw;
  uint32_t* out;
  const uint32_t* tabs;
  uint32_t fin, pad;
  const uint8_t* ptr[kSlots];
  uint32_t idx[kSlots];          // output word of shard i
  uint32_t gconst[kMaxGroups];   // x^(8(len - e_g)) mod P
};
static_assert(sizeof(CrcArgs) <= 3584, "kernel argument block must stay below 4 KiB");

__device__ __forceinline__ void piece(const uint8_t* p, uint64_t len, uint32_t off, uint32_t (&d)[4]) {
  if ((uint64_t)off + dev::kLaneBytes <= len) {
    const u32x4 v = dev::ld16<true>(p + off);
    d[0] = v.x, d[1] = v.y, d[2] = v.z, d[3] = v.w;
  } else {
    const size_t rem = off < len ? (size_t)(len - off) : 0;  // zero padding past the shard end
    const u32x4 v = rem ? dev::ld_tail(p + off, rem) : u32x4{0u, 0u, 0u, 0u};
    d[0] = v.x, d[1] = v.y, d[2] = v.z, d[3] = v.w;
  }
}

__global__ __launch_bounds__(256) void crc32_horner_kernel(const CrcArgs a) {
  __shared__ uint32_t ct[crcdev::kOnlyTabWords];
  __shared__ uint32_t red[4];
  for (int i = threadIdx.x; i < crcdev::kOnlyTabWords; i += 256) ct[i] = a.tabs[crcdev::kOnlyTabBase + i];
  __syncthreads();
  const uint32_t g = blockIdx.x, sh = blockIdx.y;
  const uint8_t* p = a.sstride ? a.ptr[0] + (int64_t)sh * a.sstride : a.ptr[sh];
  const uint32_t t0 = g * a.tpw, t1 = min(t0 + a.tpw, a.tiles);
  const uint32_t lanepos = threadIdx.x * dev::kLaneBytes;
  uint32_t R = 0, cur[4], nxt[4];
  piece(p, a.len, t0 * kTile + lanepos, cur);
  for (uint32_t t = t0; t < t1; ++t) {
    if (t + 1 < t1) piece(p, a.len, (t + 1) * kTile + lanepos, nxt);
    R = crcdev::only_step(ct, R, cur);
#pragma unroll
    for (int w = 0; w < 4; ++w) cur[w] = nxt[w];
  }
  const u32x4* basis = reinterpret_cast<const u32x4*>(a.tabs + kTabWords + threadIdx.x * 32);
  uint32_t o = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const u32x4 v = basis[q];
    o ^= (0u - ((R >> (4 * q)) & 1u)) & v.x;
    o ^= (0u - ((R >> (4 * q + 1)) & 1u)) & v.y;
    o ^= (0u - ((R >> (4 * q + 2)) & 1u)) & v.z;
    o ^= (0u - ((R >> (4 * q + 3)) & 1u)) & v.w;
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) o ^= (uint32_t)__shfl_xor((int)o, d);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = o;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t v = crcdev::mulmod(a.gconst[g], red[0] ^ red[1] ^ red[2] ^ red[3]);
    if (g == 0) v ^= a.fin;
    atomicXor(a.out + (a.sstride ? a.idx[0] + sh : a.idx[sh]), v);
  }
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
  const int per_launch = stride ? n : kSlots;
  // ~2048 workgroups in all, each keeping >= 1 tile
  const uint32_t want = std::max<uint32_t>(1, 2048u / (uint32_t)n);
  uint32_t groups = std::min<uint32_t>({tiles, want, (uint32_t)kMaxGroups});
  const uint32_t tpw = (tiles + groups - 1) / groups;
  groups = (tiles + tpw - 1) / tpw;
  a.len = len;
  a.sstride = stride;
  a.tiles = tiles;
  a.tpw = tpw;
  a.out = out;
  a.fin = fin;
  for (uint32_t g = 0; g < groups; ++g) {
    const int64_t end = (int64_t)std::min<uint64_t>((uint64_t)(g + 1) * tpw, tiles) * kTile;
    a.gconst[g] = crc_xpow(8 * ((int64_t)len - end));
  }
  for (int s0 = 0; s0 < n; s0 += per_launch) {
    const int ns = std::min(per_launch, n - s0);
    for (int s = 0; s < std::min(ns, kSlots); ++s) {
      a.ptr[s] = ptrs[s0 + s];
      a.idx[s] = idx ? idx[s0 + s] : (uint32_t)(s0 + s);
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
