// crc32block.hip -- blobstore/common/crc32block framing on gfx950.
//
// A framed object is a run of blocks of block_len bytes (default 64 KiB, a positive multiple of
// 4096, util.go:22-36): each block is the little-endian crc32.ChecksumIEEE of its payload followed
// by the payload, block_len - 4 bytes except in the last block (block.go:34-49, encode.go:87-109,
// decode.go:85-108).  Blobnode frames every shard it stores -- and takes crc32.ChecksumIEEE of the
// whole shard on the way (core/storage/datafile.go:345-373) -- and checks the frames of the range
// it reads back (datafile.go:406-426 -> Decoder.Reader, decode.go:122-146).
//
// One kernel does both directions over a batch of equally sized objects (grid y): workgroup (w, y)
// owns block b0 + w of object y, streams its payload in 4 KiB tiles cut at 16-byte boundaries of
// the destination (thread j: the 16-byte piece j of each tile, the next tile's piece in flight;
// loads may be unaligned, stores are aligned), folds every
// piece into a Horner register with the nibble LDS tables of the shard CRC kernels (gf_crc.hpp
// crc_step_nib: R <- f(shift(R, 4080), piece)), and copies the piece to its destination.  After the last tile a
// per-thread basis moves R to the tile end, the workgroup XOR-reduces, and one multiply by
// x^(8(plen - tiles*4096)) (a negative power: the zero padding of the last tile) gives the raw
// (zero-preset) CRC of the payload; XOR-ing shift(~0, plen) ^ ~0 makes it ChecksumIEEE.  Encode
// writes that in front of the block; decode compares it with the stored word and atomicMin's the
// block index into `bad`.  The whole-object checksum is the XOR of every block's raw CRC moved to
// the object end, x^(8 * bytes after the block) -- computed per block from a table of x^(8P 2^i) --
// with shift(~0, size) ^ ~0 folded in by the last block, so the accumulated word is ChecksumIEEE.
// Every payload byte is read once and written once.
#include <algorithm>
#include <cstdlib>

#include "gf_crc.hpp"
#include "kernels.hpp"

namespace cfsec {
namespace blk {

using crcdev::kTabWords;
using crcdev::kTile;
using dev::u32x4;

constexpr int kSlots = 128;  // objects per launch (a whole 8-stripe EC12P4 batch: 128 shards)
constexpr int kRing = 4;    // tiles in flight per thread
constexpr int kAfter = 200;  // objects of up to 200 blocks (12.5 MiB at 64 KiB) move a block's CRC in one multiply

struct __attribute__((aligned(16))) BlockArgs {
  const uint8_t* in[kSlots];  // object y: payload of launch block w at in[y] + w*in_stride + in_off
  uint8_t* out[kSlots];       // its payload byte o at out[y] + w*out_stride + out_off + o, if lo <= b*P + o < hi
  const uint32_t* tabs;
  uint32_t* bad;      // decode: [object] smallest mismatching launch block index
  uint32_t* whole;    // encode, optional: [object] raw CRC of the whole object, atomicXor-accumulated
  int64_t in_stride, in_off, out_stride, out_off;
  uint64_t size, lo, hi;  // payload size of the object; copied payload range
  uint64_t b0, nblk;      // first block of the launch; blocks in the object
  uint32_t nb, items;     // blocks per object in the launch; nb * objects
  uint32_t P;             // payload bytes of a full block
  uint32_t encode;        // 1: write the checksum at out + w*out_stride; 0: check in + w*in_stride
  uint32_t gconst[2][16];      // [full block, last block][h]: x^(8(plen + h - tiles*4096))
  uint32_t gc4k[2][16][2];     // block kernel, h = 16a + b < 4096: [last][b][tiles - ceil((plen+b)/4096)]:
                               // x^(8(plen + b - tiles*4096)); times x^(8*16a) it is gconst
  uint32_t fin[2];             // [full block, last block]: shift(~0, plen) ^ ~0
  uint32_t xlast;              // x^(8 * payload of the last block)
  uint32_t xlen[2];            // x^(8 plen): [full block, last block]
  uint32_t ipw;                // items per workgroup
  uint32_t whole_fin;          // shift(~0, size) ^ ~0
  uint32_t xpow2[40];          // x^(8 P 2^i) for 2^i <= nblk
  uint32_t nafter;             // entries of xafter (0: nblk too large, use xlast and xpow2)
  uint32_t xafter[kAfter];     // [r]: x^(8 * payload bytes after block r - 1), 1 <= r < nblk
};
static_assert(sizeof(BlockArgs) <= 3584, "kernel argument block must stay below 4 KiB");

// Bytes [lo, hi) of the 16 at p, zero elsewhere.
__device__ __forceinline__ u32x4 ld_range(const uint8_t* p, uint32_t lo, uint32_t hi) {
  uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (uint32_t i = 0; i < 16; ++i)
    if (i >= lo && i < hi) w[i >> 2] |= (uint32_t)p[i] << (8 * (i & 3));
  return u32x4{w[0], w[1], w[2], w[3]};
}

// Piece p of a block: the 16 payload positions 16p - h .. 16p - h + 15, i.e. one 16-byte-aligned
// chunk of the destination (h = destination misalignment of payload byte 0), so every full store
// is aligned; positions outside [0, plen) read as zero (leading zeros leave a zero-preset CRC
// unchanged, trailing ones are taken out by gconst).
__device__ __forceinline__ void load_piece(const uint8_t* src, uint32_t plen, uint32_t h, uint32_t p,
                                           uint32_t (&d)[4]) {
  const int64_t first = (int64_t)16 * p - h;  // payload index of byte 0 of the piece
  u32x4 v{0u, 0u, 0u, 0u};
  if (first >= 0 && first + 16 <= plen)
    v = dev::ld16<true>(src + first);
  else if (first < (int64_t)plen)
    v = ld_range(src + first, first < 0 ? (uint32_t)-first : 0u, (uint32_t)min<int64_t>(16, plen - first));
  d[0] = v.x, d[1] = v.y, d[2] = v.z, d[3] = v.w;
}

// STORE / CRC / EPI off, SRCALIGN on: measurement variants for tools/blk_probe.hip (the product
// runs STORE, CRC and EPI on, pieces aligned to the destination).
template <bool STORE = true, bool CRC = true, bool EPI = true, bool SRCALIGN = false, bool NTS = true>
__global__ __launch_bounds__(256) void crc32block_kernel(const BlockArgs a) {
  __shared__ uint32_t ct[crcdev::kOnlyTabWords];
  __shared__ uint32_t red[4];
  for (int i = threadIdx.x; i < crcdev::kOnlyTabWords; i += 256) ct[i] = a.tabs[crcdev::kOnlyTabBase + i];
  // this thread's x^(8*16*(255 - j)): moves its Horner register from its piece to the tile end
  // (gf_crc.hip host_tables; one coalesced word per thread -- reading column x^0 of the
  // per-thread basis instead, 128 B apart, cost one L2 request per thread per block)
  const uint32_t kj = a.tabs[kTabWords + crcdev::kBasisWords + threadIdx.x];
  __syncthreads();
  // work items (launch block w, object y), y-major; a workgroup takes a run of consecutive ones,
  // so the table load above is paid once per workgroup and the whole-object checksum is a Horner
  // sum over the run (acc <- acc * x^(8 plen) ^ raw) moved to the object end once per run
  const uint32_t it0 = blockIdx.x * a.ipw, it1 = min(it0 + a.ipw, a.items);
  uint32_t acc = 0, run_y = 0xFFFFFFFFu, run_end = 0;  // thread 0: the run's raw CRC, object, next block
  const auto flush = [&]() {
    if (threadIdx.x != 0 || !a.whole || run_y == 0xFFFFFFFFu) return;
    uint32_t s = acc;
    if (run_end == a.nblk) {
      s ^= a.whole_fin;  // the run ends the object: fold in the conditioning once per object
    } else if (run_end < a.nafter) {
      s = crcdev::mulmod(s, a.xafter[run_end]);  // one multiply: thread 0's work is serial
    } else {
      // bytes after the run: nblk - 1 - run_end full blocks, then the last block's payload
      s = crcdev::mulmod(s, a.xlast);
      uint64_t e = a.nblk - 1 - run_end;
      for (int i = 0; e; e >>= 1, ++i)
        if (e & 1) s = crcdev::mulmod(s, a.xpow2[i]);
    }
    atomicXor(a.whole + run_y, s);
  };
  for (uint32_t it = it0; it < it1; ++it) {
    const uint32_t y = it / a.nb, w = it - y * a.nb;
    if (y != run_y) {
      flush();
      acc = 0;
      run_y = y;
    }
    const uint8_t* const in = a.in[y];
    uint8_t* const out = a.out[y];
    const uint64_t b = a.b0 + w;
    const uint64_t q0 = b * a.P;  // payload coordinate of the block's first byte
    const uint32_t plen = (uint32_t)min<uint64_t>(a.P, a.size - q0);
    const int last = plen != a.P ? 1 : 0;
    const uint8_t* src = in + (int64_t)w * a.in_stride + a.in_off;
    const int64_t dbase = (int64_t)w * a.out_stride + a.out_off;  // out offset of payload byte 0
    const uint32_t h = SRCALIGN ? (uint32_t)((uintptr_t)src & 15u) : (uint32_t)(((uintptr_t)out + (uint64_t)dbase) & 15u);
    const uint32_t tiles = (plen + h + kTile - 1) / kTile;
    // kRing tiles' pieces in flight per thread, in a ring of registers named at compile time (the
    // tile loop is unrolled by kRing): moving a register that an outstanding load targets would
    // make the wave wait for that load, which is what a rotating prefetch buffer does
    uint32_t R = 0, ring[kRing][4];
#pragma unroll
    for (int k = 0; k < kRing; ++k)
      if (k < (int)tiles) load_piece(src, plen, h, threadIdx.x + 256 * k, ring[k]);
    for (uint32_t t0 = 0; t0 < tiles; t0 += kRing) {
#pragma unroll
      for (int k = 0; k < kRing; ++k) {
        const uint32_t t = t0 + k;
        if (t < tiles) {
          uint32_t (&cur)[4] = ring[k];
          const uint32_t p = t * 256 + threadIdx.x;
          if constexpr (CRC) R = crcdev::only_step(ct, R, cur);
          else R ^= cur[0] ^ cur[1] ^ cur[2] ^ cur[3];
          const int64_t first = (int64_t)16 * p - h;
          if (STORE && first < (int64_t)plen) {
            const int64_t q = (int64_t)q0 + first;  // payload coordinate of the piece's byte 0
            uint8_t* dp = out + (dbase + first);    // 16-byte aligned
            if (first >= 0 && first + 16 <= plen && q >= (int64_t)a.lo && q + 16 <= (int64_t)a.hi) {
              dev::st16_out<NTS>(dp, u32x4{cur[0], cur[1], cur[2], cur[3]});
            } else {
              for (int j = 0; j < 16; ++j)
                if (first + j >= 0 && first + j < plen && q + j >= (int64_t)a.lo && q + j < (int64_t)a.hi)
                  dp[j] = (uint8_t)(cur[j >> 2] >> (8 * (j & 3)));
            }
          }
          if (t + kRing < tiles) load_piece(src, plen, h, p + 256 * kRing, cur);
        }
      }
    }
    if constexpr (!EPI) {
      if (R == 0x12345678u) a.bad[0] = R;  // keep the loads live
      run_y = 0xFFFFFFFFu;
      continue;
    }
    uint32_t v = crcdev::mulmod(kj, R);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v ^= (uint32_t)__shfl_xor((int)v, d);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint32_t raw = crcdev::mulmod(a.gconst[last][h], red[0] ^ red[1] ^ red[2] ^ red[3]);
      const uint32_t crc = raw ^ a.fin[last];
      if (a.encode) {
        uint8_t* hdr = out + (int64_t)w * a.out_stride;
        for (int j = 0; j < 4; ++j) hdr[j] = (uint8_t)(crc >> (8 * j));
        if (a.whole) acc = (acc ? crcdev::mulmod(acc, a.xlen[last]) : 0u) ^ raw;  // first block of a run: acc = 0
        run_end = (uint32_t)b + 1;
      } else {
        const uint8_t* hdr = in + (int64_t)w * a.in_stride;
        const uint32_t stored = hdr[0] | (uint32_t)hdr[1] << 8 | (uint32_t)hdr[2] << 16 | (uint32_t)hdr[3] << 24;
        if (stored != crc) atomicMin(a.bad + y, w);
      }
    }
    __syncthreads();  // red[] is reused by the next item
  }
  flush();
}

// The shipped kernel.  Blocks go to workgroups in order (consecutive workgroups take consecutive
// blocks, so the workgroups in flight sweep one compact region of HBM: runs of blocks per workgroup
// spread them over hundreds of MiB and measured 18-60 % slower, profiles/r02/blk_probe.txt), either
// one block per workgroup or (STRIDE) a resident grid striding over the blocks, which loads the
// next block's first tiles before the current block's epilogue.  The epilogue keeps its serial
// work off the barrier: every wave moves its reduced register to the block end itself (the
// x^(8*16*(255-j)) and x^(8(plen - tiles*4096)) multiplies are linear, so they distribute over the
// XOR), and in encode also to the object end and into the whole-object word; after one barrier
// thread 0 only XORs four words and stores or compares the header.
template <int RING, bool NTS = true, bool STRIDE = false>
__global__ __launch_bounds__(256) void crc32block_block_kernel(const BlockArgs a) {
  __shared__ uint32_t ct[crcdev::kOnlyTabWords];
  __shared__ uint32_t redb[2][8];  // per wave: its share of the block's raw CRC, and of the object's
  for (int i = threadIdx.x; i < crcdev::kOnlyTabWords; i += 256) ct[i] = a.tabs[crcdev::kOnlyTabBase + i];
  const uint32_t tid = threadIdx.x;
  const uint32_t kj = a.tabs[kTabWords + crcdev::kBasisWords + tid];
  __syncthreads();
  uint32_t it = blockIdx.x;
  if (it >= a.items) return;  // whole workgroup: no barrier follows

  // Decode writes the payloads of consecutive blocks back to back, so the 128-byte line holding
  // the seam between two blocks gets bytes of both.  Written by two workgroups (two L2s), it would
  // reach HBM as two partial-line writes (profiles/r02/blk_probe.txt: 57 % of 8 TB/s against 62 %
  // with the seams apart).  So each seam line has one writer: a block stores from the first line
  // boundary of its payload [sbeg) and on through the next block's first bytes up to the next line
  // boundary [send), those taken from the next block's frame.
  struct Blk {
    uint32_t y, w, plen, h, tiles, stored;
    int last;
    uint64_t b, q0;
    const uint8_t* src;
    int64_t dbase;
    uint32_t sbeg, send, lim;  // stored payload range [sbeg, send); main loop stores below lim
  };
  const auto make = [&](uint32_t item) {
    Blk k;
    k.y = item / a.nb;
    k.w = item - k.y * a.nb;
    k.b = a.b0 + k.w;
    k.q0 = k.b * a.P;
    k.plen = (uint32_t)min<uint64_t>(a.P, a.size - k.q0);
    k.last = k.plen != a.P ? 1 : 0;
    k.src = a.in[k.y] + (int64_t)k.w * a.in_stride + a.in_off;
    k.dbase = (int64_t)k.w * a.out_stride + a.out_off;
    // pieces are cut at 16-byte boundaries of the destination and tiles at its 4 KiB boundaries
    // (decode's payloads sit at 65532-byte steps: tiles across 4 KiB boundaries of the written
    // side measured 56 % of 8 TB/s against 61 % aligned, profiles/r02/blk_probe.txt)
    k.h = (uint32_t)(((uintptr_t)a.out[k.y] + (uint64_t)k.dbase) & (kTile - 1));
    k.tiles = (k.plen + k.h + kTile - 1) / kTile;
    k.sbeg = 0, k.send = k.plen, k.lim = k.plen;
    if (!a.encode) {
      const uint64_t d0 = (uintptr_t)a.out[k.y] + (uint64_t)k.dbase;  // destination of payload byte 0
      if (k.w > 0) k.sbeg = (uint32_t)((128u - (d0 & 127u)) & 127u);
      if (k.w + 1 < a.nb) {
        const uint64_t next = min<uint64_t>(a.P, a.size - k.q0 - k.plen);  // the next block's payload
        k.send = k.plen + (uint32_t)min<uint64_t>((128u - ((d0 + k.plen) & 127u)) & 127u, next);
        k.lim = k.plen - ((k.plen + k.h) & 15u);  // the piece across the seam goes with the tail
      }
    }
    // decode: the stored checksum, fetched up front (read at the end it is one more dependent
    // global load on the workgroup's critical path)
    k.stored = 0;
    if (!a.encode && tid == 0) {
      const uint8_t* hdr = a.in[k.y] + (int64_t)k.w * a.in_stride;
      k.stored = hdr[0] | (uint32_t)hdr[1] << 8 | (uint32_t)hdr[2] << 16 | (uint32_t)hdr[3] << 24;
    }
    return k;
  };
  uint32_t ring[RING][4];
  const auto prefetch = [&](const Blk& k) {
#pragma unroll
    for (int r = 0; r < RING; ++r)
      if (r < (int)k.tiles) load_piece(k.src, k.plen, k.h, tid + 256 * r, ring[r]);
  };
  Blk cur = make(it);
  prefetch(cur);
  for (uint32_t parity = 0;; parity ^= 1u) {
    uint8_t* const out = a.out[cur.y];
    uint32_t R = 0;
    // piece t*256 + tid: Horner step, then the copy to the destination
    const auto piece = [&](uint32_t t, uint32_t (&pc)[4]) {
      const uint32_t p = t * 256 + tid;
      R = crcdev::only_step(ct, R, pc);
      const int64_t first = (int64_t)16 * p - cur.h;
      if (first + 16 > (int64_t)cur.sbeg && first < (int64_t)cur.lim) {  // sbeg > 0 is a piece boundary
        const int64_t q = (int64_t)cur.q0 + first;
        uint8_t* dp = out + (cur.dbase + first);  // 16-byte aligned
        if (first >= 0 && first + 16 <= cur.lim && q >= (int64_t)a.lo && q + 16 <= (int64_t)a.hi) {
          dev::st16_out<NTS>(dp, u32x4{pc[0], pc[1], pc[2], pc[3]});
        } else {
          for (int j = 0; j < 16; ++j)
            if (first + j >= 0 && first + j < cur.lim && q + j >= (int64_t)a.lo && q + j < (int64_t)a.hi)
              dp[j] = (uint8_t)(pc[j >> 2] >> (8 * (j & 3)));
        }
      }
    };
    for (uint32_t t0 = 0; t0 < cur.tiles; t0 += RING) {
#pragma unroll
      for (int r = 0; r < RING; ++r) {
        const uint32_t t = t0 + r;
        if (t < cur.tiles) {
          piece(t, ring[r]);
          if (t + RING < cur.tiles) load_piece(cur.src, cur.plen, cur.h, t * 256 + tid + 256 * RING, ring[r]);
        }
      }
    }
    if (cur.send > cur.lim) {  // decode: the pieces from lim to the seam line's end, one per thread
      const uint32_t nx = (cur.send - cur.lim + 15u) >> 4;
      if (tid < nx) {
        const int64_t first = (int64_t)cur.lim + 16 * tid;
        const uint32_t own = (uint32_t)max<int64_t>(0, min<int64_t>(16, (int64_t)cur.plen - first));
        const uint8_t* nsrc = cur.src + a.in_stride;  // the next block's payload
        const u32x4 v = ld_range(cur.src + first, 0, own) | ld_range(nsrc + (first - (int64_t)cur.plen), own,
                                                                   (uint32_t)min<int64_t>(16, (int64_t)cur.send - first));
        const int64_t q = (int64_t)cur.q0 + first;
        uint8_t* dp = out + (cur.dbase + first);
        if (first + 16 <= cur.send && q >= (int64_t)a.lo && q + 16 <= (int64_t)a.hi) {
          dev::st16_out<NTS>(dp, v);
        } else {
          const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
          for (int j = 0; j < 16; ++j)
            if (first + j < cur.send && q + j >= (int64_t)a.lo && q + j < (int64_t)a.hi)
              dp[j] = (uint8_t)(w4[j >> 2] >> (8 * (j & 3)));
        }
      }
    }
    const uint32_t nit = it + gridDim.x;
    const bool more = STRIDE && nit < a.items;
    Blk nxt{};
    if (more) {
      nxt = make(nit);
      prefetch(nxt);
    }
    uint32_t* red = redb[parity];  // the other buffer may still be read by thread 0 of the last block
    uint32_t v = crcdev::mulmod(kj, R);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v ^= (uint32_t)__shfl_xor((int)v, d);
    if ((tid & 63) == 0) {
      // this wave's share of the block's raw CRC: x^(8(plen + h - tiles*4096)) from the host's
      // factor for h mod 16 and x^(8*16*(h >> 4)), a word of the per-thread shift table
      const uint32_t b16 = cur.h & 15u, dt = cur.tiles - ((cur.plen + b16 + kTile - 1) / kTile);
      const uint32_t g = crcdev::mulmod(a.gc4k[cur.last][b16][dt], a.tabs[kTabWords + crcdev::kBasisWords + 255 - (cur.h >> 4)]);
      const uint32_t raw = crcdev::mulmod(g, v);
      red[tid >> 6] = raw;
      if (a.encode && a.whole) {
        uint32_t s = raw;  // the share moved to the object end
        if (cur.b + 1 < a.nblk) {
          if (cur.b + 1 < a.nafter) {
            s = crcdev::mulmod(s, a.xafter[cur.b + 1]);
          } else {
            s = crcdev::mulmod(s, a.xlast);
            uint64_t e = a.nblk - 2 - cur.b;
            for (int q = 0; e; e >>= 1, ++q)
              if (e & 1) s = crcdev::mulmod(s, a.xpow2[q]);
          }
        }
        red[4 + (tid >> 6)] = s;
      }
    }
    __syncthreads();
    if (tid == 0) {
      const uint32_t crc = red[0] ^ red[1] ^ red[2] ^ red[3] ^ a.fin[cur.last];
      if (a.encode) {
        uint8_t* hdr = out + (int64_t)cur.w * a.out_stride;
        for (int j = 0; j < 4; ++j) hdr[j] = (uint8_t)(crc >> (8 * j));
        // one atomic per block (the four waves' shares XOR-ed here: many adders on one word are slow)
        if (a.whole)
          atomicXor(a.whole + cur.y, red[4] ^ red[5] ^ red[6] ^ red[7] ^ (cur.b + 1 == a.nblk ? a.whole_fin : 0u));
      } else if (cur.stored != crc) {
        atomicMin(a.bad + cur.y, cur.w);
      }
    }
    if (!more) break;
    cur = nxt;
    it = nit;
  }
}

}  // namespace blk

using blk::BlockArgs;
using blk::kSlots;

bool crc32block_valid_len(int64_t block_len) { return block_len > 0 && block_len % 4096 == 0; }

namespace blk {
// Workgroups of crc32block_block_kernel<RING, NTS, true> resident on the current device at once.
template <int RING, bool NTS>
unsigned resident_groups() {
  int dev = 0, cus = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, crc32block_block_kernel<RING, NTS, true>, 256, 0) != hipSuccess)
    return 0;
  return (unsigned)std::max(cus * per, 1);
}

template <bool STORE, bool CRC, bool EPI = true, bool SRCALIGN = false, bool ONE = true, bool NTS = true,
          int RING = kRing, bool FASTEPI = true, bool STRIDE = false, bool SEAMLESS_PROBE = false>
hipError_t launch(const Crc32BlockJob& j, hipStream_t stream) {
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
    // probe only (tools/blk_probe): destination blocks block_len apart, so no 128-byte line is
    // shared by two blocks' payloads -- not the unframed layout
    if (SEAMLESS_PROBE) a.out_stride = j.block_len;
  }
  if (nb <= 0 || j.n == 0) return hipSuccess;
  if (nb > 0xFFFFFFFFll / kSlots || j.n < 0 || !j.in || (!j.out && (j.encode || j.to > j.from)) || (!j.encode && !j.bad))
    return hipErrorInvalidValue;
  a.bad = j.bad;
  a.whole = j.encode ? j.whole : nullptr;
  a.b0 = (uint64_t)b0;
  hipError_t e = crc_device_tables(&a.tabs);
  if (e != hipSuccess) return e;
  const int64_t plens[2] = {P, j.size - (nblk - 1) * P};
  for (int i = 0; i < 2; ++i) {
    for (int h = 0; h < 16; ++h) {
      const int64_t tiles = (plens[i] + h + kTile - 1) / kTile;
      a.gconst[i][h] = crc_xpow(8 * (plens[i] + h - tiles * kTile));
      for (int dt = 0; dt < 2; ++dt) a.gc4k[i][h][dt] = crc_xpow(8 * (plens[i] + h - (tiles + dt) * kTile));
    }
    a.fin[i] = crc32_shift_ones((size_t)plens[i]);
  }
  a.xlast = crc_xpow(8 * plens[1]);
  a.xlen[0] = crc_xpow(8 * plens[0]);
  a.xlen[1] = a.xlast;
  a.whole_fin = crc32_shift_ones((size_t)j.size);
  for (int i = 0; i < 40 && (int64_t(1) << i) <= nblk; ++i) a.xpow2[i] = crc_xpow(8 * P * (int64_t(1) << i));
  if (nblk <= kAfter) {
    a.nafter = (uint32_t)nblk;
    const uint32_t xp = crc_xpow(8 * P);
    uint32_t v = a.xlast;  // after block nblk - 2: the last block's payload
    for (int64_t r = nblk - 1; r >= 1; --r) {
      a.xafter[r] = v;
      v = crc_mulmod(v, xp);
    }
  }
  for (int y0 = 0; y0 < j.n; y0 += kSlots) {
    const int ny = std::min(kSlots, j.n - y0);
    for (int y = 0; y < ny; ++y) {
      if (!j.in[y0 + y] || ((!j.out || !j.out[y0 + y]) && (j.encode || j.to > j.from))) return hipErrorInvalidValue;
      // decode: in[] are the framed objects; the launch starts at block b0
      a.in[y] = j.encode ? j.in[y0 + y] : j.in[y0 + y] + b0 * j.block_len;
      a.out[y] = j.out ? j.out[y0 + y] : nullptr;
    }
    a.nb = (uint32_t)nb;
    a.items = (uint32_t)(nb * ny);
    // one block per workgroup measured best (tools/blk_probe.hip, profiles/r01/crc32block_probe.txt:
    // runs of ~5 blocks per workgroup, sharing one table load, were 5-10 % slower)
    a.ipw = ONE ? 1u : (a.items + 2047) / 2048;
    const unsigned grid = (a.items + a.ipw - 1) / a.ipw;
    if (FASTEPI && ONE && EPI && STORE && CRC && STRIDE) {
      // a resident grid, every workgroup the same number of blocks
      static thread_local int cached_dev = -1;
      static thread_local unsigned cap = 0;
      int dev = 0;
      if (hipGetDevice(&dev) == hipSuccess && dev != cached_dev) {
        cap = resident_groups<RING, NTS>();
        cached_dev = dev;
      }
      // CFSEC_BLK_GRID=1: the whole resident grid, (items mod cap) workgroups taking one block more, so
      // every CU holds as many workgroups; 0: as few workgroups as give every one the same count (A/B)
      static const bool full = [] {
        const char* v = std::getenv("CFSEC_BLK_GRID");
        return !(v && v[0] == '0');
      }();
      const unsigned per = cap ? (a.items + cap - 1) / cap : 1;
      const unsigned g = full && cap ? std::min(cap, a.items) : (a.items + per - 1) / per;
      hipLaunchKernelGGL((crc32block_block_kernel<RING, NTS, true>), dim3(g), dim3(256), 0, stream, a);
    } else if (FASTEPI && ONE && EPI && STORE && CRC)
      hipLaunchKernelGGL((crc32block_block_kernel<RING, NTS, false>), dim3(a.items), dim3(256), 0, stream, a);
    else
      hipLaunchKernelGGL((crc32block_kernel<STORE, CRC, EPI, SRCALIGN, NTS>), dim3(grid), dim3(256), 0, stream, a);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (a.bad) a.bad += ny;
    if (a.whole) a.whole += ny;
  }
  return hipSuccess;
}

}  // namespace blk

// shipped: the resident-grid kernel with 8 tiles in flight per thread (tools/blk_probe,
// profiles/r02/blk_probe.txt: encode 62 %, decode 58 % of 8 TB/s against 60 / 57 % one block per
// workgroup)
hipError_t launch_crc32block(const Crc32BlockJob& j, hipStream_t stream) {
  return blk::launch<true, true, true, false, true, true, 8, true, true>(j, stream);
}

}  // namespace cfsec
