// crc32block.hip -- blobstore/common/crc32block framing on gfx950.
//
// A framed object is a run of blocks of block_len bytes (default 64 KiB, a positive multiple of
// 4096, util.go:22-36): each block is the little-endian crc32.ChecksumIEEE of its payload followed
// by the payload, block_len - 4 bytes except in the last block (block.go:34-49, encode.go:87-109,
// decode.go:85-108).  Blobnode frames every shard it stores -- and takes crc32.ChecksumIEEE of the
// whole shard on the way (core/storage/datafile.go:345-373) -- and checks the frames of the range
// it reads back (datafile.go:406-426 -> Decoder.Reader, decode.go:122-146).
//
// One kernel does both directions: workgroup w owns block b0 + w, streams its payload in 4 KiB
// tiles (thread j: the 16-byte piece j of each tile, the next tile's piece in flight), folds every
// piece into a Horner register with the slice-by-8 LDS tables of the shard CRC kernels (gf_crc.hpp:
// R <- f(shift(R, 4080), piece)), and copies the piece to its destination.  After the last tile a
// per-thread basis moves R to the tile end, the workgroup XOR-reduces, and one multiply by
// x^(8(plen - tiles*4096)) (a negative power: the zero padding of the last tile) gives the raw
// (zero-preset) CRC of the payload; XOR-ing shift(~0, plen) ^ ~0 makes it ChecksumIEEE.  Encode
// writes that in front of the block; decode compares it with the stored word and atomicMin's the
// block index into `bad`.  The whole-object checksum is the XOR of every block's raw CRC moved to
// the object end, x^(8 * bytes after the block) -- computed per block from a table of x^(8P 2^i).
// Every payload byte is read once and written once.
#include <algorithm>

#include "gf_crc.hpp"
#include "kernels.hpp"

namespace cfsec {
namespace {

using crcdev::kTabWords;
using crcdev::kTile;
using dev::u32x4;

struct __attribute__((aligned(16))) BlockArgs {
  const uint8_t* in;  // payload of launch block w at in + w*in_stride + in_off
  uint8_t* out;       // its payload byte o at out + w*out_stride + out_off + o, if lo <= b*P + o < hi
  const uint32_t* tabs;
  uint32_t* bad;      // decode: smallest mismatching launch block index
  uint32_t* whole;    // encode, optional: raw CRC of the whole object, atomicXor-accumulated
  int64_t in_stride, in_off, out_stride, out_off;
  uint64_t size, lo, hi;  // payload size of the object; copied payload range
  uint64_t b0, nblk;      // first block of the launch; blocks in the object
  uint32_t P;             // payload bytes of a full block
  uint32_t encode;        // 1: write the checksum at out + w*out_stride; 0: check in + w*in_stride
  uint32_t gconst[2], fin[2];  // [full block, last block]
  uint32_t xlast;              // x^(8 * payload of the last block)
  uint32_t xpow2[40];          // x^(8 P 2^i) for 2^i <= nblk
};

__device__ __forceinline__ void load_piece(const uint8_t* p, uint32_t plen, uint32_t off, uint32_t (&d)[4]) {
  u32x4 v{0u, 0u, 0u, 0u};
  if (off + dev::kLaneBytes <= plen)
    v = dev::ld16<true>(p + off);
  else if (off < plen)
    v = dev::ld_tail(p + off, plen - off);  // zero padding past the payload end
  d[0] = v.x, d[1] = v.y, d[2] = v.z, d[3] = v.w;
}

__global__ __launch_bounds__(256) void crc32block_kernel(const BlockArgs a) {
  __shared__ uint32_t ct[kTabWords];
  __shared__ uint32_t red[4];
  for (int i = threadIdx.x; i < kTabWords; i += 256) ct[i] = a.tabs[i];
  __syncthreads();
  const uint32_t w = blockIdx.x;
  const uint64_t b = a.b0 + w;
  const uint64_t q0 = b * a.P;  // payload coordinate of the block's first byte
  const uint32_t plen = (uint32_t)min<uint64_t>(a.P, a.size - q0);
  const int last = plen != a.P ? 1 : 0;
  const uint8_t* src = a.in + (int64_t)w * a.in_stride + a.in_off;
  const int64_t dbase = (int64_t)w * a.out_stride + a.out_off;  // out offset of payload byte 0
  const uint32_t tiles = (plen + kTile - 1) / kTile;
  const uint32_t lanepos = threadIdx.x * dev::kLaneBytes;
  uint32_t R = 0, cur[4], nxt[4];
  load_piece(src, plen, lanepos, cur);
  for (uint32_t t = 0; t < tiles; ++t) {
    const uint32_t o = t * kTile + lanepos;
    if (t + 1 < tiles) load_piece(src, plen, o + kTile, nxt);
    R = crcdev::crc_step(ct, R, cur);
    if (o < plen) {
      const uint64_t q = q0 + o;
      const uint32_t n = min<uint32_t>(dev::kLaneBytes, plen - o);
      if (n == dev::kLaneBytes && q >= a.lo && q + n <= a.hi) {
        dev::st16<true>(a.out + dbase + o, u32x4{cur[0], cur[1], cur[2], cur[3]});
      } else {
        for (uint32_t j = 0; j < n; ++j)
          if (q + j >= a.lo && q + j < a.hi) a.out[dbase + o + j] = (uint8_t)(cur[j >> 2] >> (8 * (j & 3)));
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) cur[i] = nxt[i];
  }
  const u32x4* basis = reinterpret_cast<const u32x4*>(a.tabs + kTabWords + threadIdx.x * 32);
  uint32_t v = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const u32x4 bv = basis[q];
    v ^= (0u - ((R >> (4 * q)) & 1u)) & bv.x;
    v ^= (0u - ((R >> (4 * q + 1)) & 1u)) & bv.y;
    v ^= (0u - ((R >> (4 * q + 2)) & 1u)) & bv.z;
    v ^= (0u - ((R >> (4 * q + 3)) & 1u)) & bv.w;
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v ^= (uint32_t)__shfl_xor((int)v, d);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t raw = crcdev::mulmod(a.gconst[last], red[0] ^ red[1] ^ red[2] ^ red[3]);
    const uint32_t crc = raw ^ a.fin[last];
    if (a.encode) {
      uint8_t* h = a.out + (int64_t)w * a.out_stride;
      for (int j = 0; j < 4; ++j) h[j] = (uint8_t)(crc >> (8 * j));
      if (a.whole) {
        // bytes after block b: none for the last block, else the last block's payload plus
        // nblk - 2 - b full blocks
        uint32_t s = raw;
        if (b + 1 < a.nblk) {
          s = crcdev::mulmod(s, a.xlast);
          uint64_t e = a.nblk - 2 - b;
          for (int i = 0; e; e >>= 1, ++i)
            if (e & 1) s = crcdev::mulmod(s, a.xpow2[i]);
        }
        atomicXor(a.whole, s);
      }
    } else {
      const uint8_t* h = a.in + (int64_t)w * a.in_stride;
      const uint32_t stored = h[0] | (uint32_t)h[1] << 8 | (uint32_t)h[2] << 16 | (uint32_t)h[3] << 24;
      if (stored != crc) atomicMin(a.bad, w);
    }
  }
}

}  // namespace

bool crc32block_valid_len(int64_t block_len) { return block_len > 0 && block_len % 4096 == 0; }

hipError_t launch_crc32block(const Crc32BlockJob& j, hipStream_t stream) {
  if (!crc32block_valid_len(j.block_len) || j.size < 0 || j.block_len > 0xFFFFFFFFll) return hipErrorInvalidValue;
  const int64_t P = j.block_len - 4;
  const int64_t nblk = (j.size + P - 1) / P;
  BlockArgs a{};
  a.size = (uint64_t)j.size;
  a.P = (uint32_t)P;
  a.nblk = (uint64_t)nblk;
  a.encode = j.encode ? 1u : 0u;
  int64_t b0 = 0, nb = 0;
  if (j.encode) {
    nb = nblk;
    a.lo = 0, a.hi = (uint64_t)j.size;
    a.in_stride = P, a.in_off = 0;
    a.out_stride = j.block_len, a.out_off = 4;
  } else {
    if (j.from < 0 || j.from > j.to || j.to > j.size) return hipErrorInvalidValue;
    // Decoder.Reader (decode.go:122-146) reads from the block holding `from` through the block
    // holding to-1; with from == to it still reads (and checks) the first block when it has to
    // skip into it (rangeReader.Read, decode.go:110-120)
    b0 = j.from / P;
    const int64_t b1 = j.from < j.to ? (j.to - 1) / P : (j.from % P ? b0 : b0 - 1);
    nb = b1 - b0 + 1;
    a.lo = (uint64_t)j.from, a.hi = (uint64_t)j.to;
    a.in_stride = j.block_len, a.in_off = 4;
    a.out_stride = P, a.out_off = b0 * P - j.from;
  }
  if (nb <= 0) return hipSuccess;
  if (nb > 0x7FFFFFFF || !j.in || (!j.out && (j.encode || j.to > j.from)) || (!j.encode && !j.bad))
    return hipErrorInvalidValue;
  // decode: j.in is the framed object; the launch starts at block b0
  a.in = j.encode ? j.in : j.in + b0 * j.block_len;
  a.out = j.out;
  a.bad = j.bad;
  a.whole = j.encode ? j.whole : nullptr;
  a.b0 = (uint64_t)b0;
  hipError_t e = crc_device_tables(&a.tabs);
  if (e != hipSuccess) return e;
  const int64_t plens[2] = {P, j.size - (nblk - 1) * P};
  for (int i = 0; i < 2; ++i) {
    const int64_t tiles = (plens[i] + kTile - 1) / kTile;
    a.gconst[i] = crc_xpow(8 * (plens[i] - tiles * kTile));
    a.fin[i] = crc32_shift_ones((size_t)plens[i]);
  }
  a.xlast = crc_xpow(8 * plens[1]);
  for (int i = 0; i < 40 && (int64_t(1) << i) <= nblk; ++i) a.xpow2[i] = crc_xpow(8 * P * (int64_t(1) << i));
  hipLaunchKernelGGL(crc32block_kernel, dim3((unsigned)nb), dim3(256), 0, stream, a);
  return hipGetLastError();
}

}  // namespace cfsec
