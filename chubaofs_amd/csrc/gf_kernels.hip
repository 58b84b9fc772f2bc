// gf_kernels.hip -- gfx950 kernels for GF(2^8) Reed-Solomon shard coding (launcher).
//
// Replaces the CPU kernels of klauspost/reedsolomon v1.11.7 (the generated
// mulAvxTwo_RxC / mulGFNI_RxC_64 families in KRS/galois_gen_amd64.s and the
// galMulSlice[Xor] tails in KRS/galois_amd64.go:57-122) with one HBM-streaming
// kernel per output-row count.  Device code: gf_device.hpp.
//
// Arithmetic.  GF(2^8) multiplication by a constant is linear over GF(2), so a
// byte x is split into bit fields x = x[2:0] | x[5:3] | x[7:6] and
//     c*x = T0_c[x[2:0]] ^ T1_c[x[5:3]] ^ T2_c[x[7:6]]
// with 8-, 8- and 4-entry product tables.  An 8-entry byte table is exactly
// what one v_perm_b32 indexes: the two table dwords are the perm's data
// operands and the 3-bit fields (one per byte of the lane's dword) its
// selector, so one VALU op looks up 4 bytes at once.  Per (coefficient, dword)
// the cost is 3 v_perm_b32 + v_bitop3_b32 + v_xor; per input dword the 3
// selectors cost 5 ops, amortised over all outputs.  No MFMA: GF arithmetic is
// not an FP/int contraction.
//
// Data movement.  Each lane owns 16 consecutive bytes of the shard (one
// global_load_dwordx4 per input row, one global_store_dwordx4 per output row),
// so a workgroup streams whole 1 KiB-per-wave runs of every row and every byte
// of HBM is touched exactly once: read k*len, write m*len (verify: read
// (k+m)*len, write nothing).  Loads and stores are non-temporal (each byte is
// touched once).  The product tables are rebuilt per workgroup in LDS from the
// coefficient matrix carried in the kernel argument block, which keeps the
// launch free of device allocations and host->device copies (safe under
// concurrent callers and hipGraph capture).
//
// Kernel families, first match wins:
//   lookup-product (gf_lut.hpp): the products of each input byte with a whole column from two LDS
//                table reads, for the shapes lut_outputs() names (EC12P9, EC15P12, EC16P20(L2)
//                repairs of 5-16 shards, non-dyadic k = 6 products); CFSEC_LUT=0 disables (A/B)
//   16x16-dyadic (gf_dyadic16.hpp): EC16P20's 20 parity rows
//   dyadic-block (gf_dyadic.hpp): 4x4 / 2x2 dyadic matrices (code-mode encodes, coset-aligned
//                repairs, fused LRC encodes with 2 plain rows)
//   fixed-K (gf_fixed.hpp, every code-mode input count k in {3,4,6,7,8,10,12,15,16,18}, m up to
//                fixed_max_m(k)): 256-thread workgroups, 1 chunk per lane, all outputs in one
//                wave, rows pipelined 2 ahead with the issue order pinned (tools/gf_pipe.hip:
//                +6% over the runtime-k loop on EC12P4)
//   runtime-k (any other k, or k > 32 chunked with accumulate): policies from
//                tools/gf_variants.hip -- store/accum 256-thread, 1 chunk per lane, one row at a
//                time; verify 128-thread, 2 chunks per lane, rows loaded in pairs
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "gf_device.hpp"
#include "gf_launch.hpp"
#include "gf_lut_launch.hpp"
#include "kernels.hpp"

namespace cfsec {
namespace {

using dev::GfArgs;
constexpr int kStoreW = 1;
constexpr int kVerifyW = 2;

#ifndef CFSEC_SPLIT_G
#define CFSEC_SPLIT_G 1  // input rows loaded together by output-split (compute-heavy) kernels
#endif

template <int M, int OS, MatVecMode MODE>
__global__ __launch_bounds__(256) void gf_matvec_kernel(const GfArgs a) {
  constexpr int G = OS > 1 ? CFSEC_SPLIT_G : 1;
  if constexpr (MODE == MatVecMode::kVerify || MODE == MatVecMode::kStoreVerify)
    dev::matvec<M, MODE, kVerifyW, 2, false, true, true, false, false, OS>(a);
  else
    dev::matvec<M, MODE, kStoreW, G, false, true, true, false, false, OS>(a);
}

template <MatVecMode MODE>
hipError_t launch_fixed(int k, int m, const GfArgs& a, dim3 grid, hipStream_t st) {
  switch (k) {
    case 3: return launch_k<3, MODE>(m, a, grid, st);
    case 4: return launch_k<4, MODE>(m, a, grid, st);
    case 6: return launch_k<6, MODE>(m, a, grid, st);
    case 7: return launch_k<7, MODE>(m, a, grid, st);
    case 8: return launch_k<8, MODE>(m, a, grid, st);
    case 10: return launch_k<10, MODE>(m, a, grid, st);
    case 15: return launch_k<15, MODE>(m, a, grid, st);
    case 12: return launch_k<12, MODE>(m, a, grid, st);
    case 16: return launch_k<16, MODE>(m, a, grid, st);
    case 18: return launch_k<18, MODE>(m, a, grid, st);
    default: return hipErrorInvalidValue;
  }
}

template <MatVecMode MODE>
hipError_t launch_mode(Shape sh, const GfArgs& a, dim3 grid, int threads, hipStream_t st) {
#define CFSEC_CASE(MV, OSV)                                                                      \
  case MV * 8 + OSV:                                                                             \
    hipLaunchKernelGGL((gf_matvec_kernel<MV, OSV, MODE>), grid, dim3(threads), 0, st, a);        \
    break;
  switch (sh.M * 8 + sh.OS) {
    CFSEC_CASE(1, 1) CFSEC_CASE(2, 1) CFSEC_CASE(3, 1) CFSEC_CASE(4, 1) CFSEC_CASE(5, 1)
    CFSEC_CASE(6, 1) CFSEC_CASE(4, 2) CFSEC_CASE(5, 2) CFSEC_CASE(6, 2) CFSEC_CASE(4, 4)
    CFSEC_CASE(5, 4) CFSEC_CASE(6, 4) CFSEC_CASE(8, 4)
    default: return hipErrorInvalidValue;
  }
#undef CFSEC_CASE
  return hipGetLastError();
}

// Byte distance between consecutive stripes when every stripe of the job has the same
// relative row layout (input rows c0..c0+kc, output rows r0..r0+mc); 0 otherwise.  Such a
// batch (e.g. stripes carved from one pitched HBM buffer) runs as a single launch whatever its
// stripe count; anything else is carried as an explicit pointer table, kPtrSlots per launch.
int64_t affine_stride(const MatVecJob& job, int c0, int kc, int r0, int mc) {
  if (job.nstripes < 2 || job.lens) return 0;
  const auto addr = [](const void* p) { return (int64_t)(uintptr_t)p; };
  const int64_t ss = addr(job.in[job.k + c0]) - addr(job.in[c0]);
  if (ss == 0) return 0;
  for (int s = 1; s < job.nstripes; ++s) {
    for (int c = c0; c < c0 + kc; ++c)
      if (addr(job.in[(size_t)s * job.k + c]) != addr(job.in[c]) + s * ss) return 0;
    for (int r = r0; r < r0 + mc; ++r)
      if (addr(job.out[(size_t)s * job.m + r]) != addr(job.out[r]) + s * ss) return 0;
  }
  return ss;
}

}  // namespace

// The bit-sliced EC16P20(L2) encode (gf_bs16.hip) for this launch: the network's matrix and
// 16-byte aligned rows (global_load_lds and the 16-byte accesses); CFSEC_BS16=0 disables it (A/B).
static const bool kBs16 = [] {
  const char* v = std::getenv("CFSEC_BS16");
  return !(v && v[0] == '0');
}();
// ... and its pointer-table form for repairs of stripes at unrelated addresses; CFSEC_BS_TAB=0
// leaves those to the dyadic kernel (A/B)
static const bool kBsTab = [] {
  const char* v = std::getenv("CFSEC_BS_TAB");
  return !(v && v[0] == '0');
}();
static bool aligned16(const dev::GfArgs& a, int nptr) {
  if (a.sstride & 15) return false;
  for (int i = 0; i < nptr; ++i)
    if (reinterpret_cast<uintptr_t>(a.ptr[i]) & 15) return false;
  return true;
}
static bool bs_ok(const dev::GfArgs& a, int k, int m, int tab) {
  return bs_matches(a.coef, m, k) && aligned16(a, tab * (k + m));
}

hipError_t launch_matvec(const MatVecJob& job, hipStream_t stream) {
  using dev::kMaxK;
  using dev::kMaxM;
  using dev::kPtrSlots;
  if (job.k <= 0 || job.m < 0 || job.nstripes < 0 || !job.coef || !job.in || !job.out)
    return hipErrorInvalidValue;
  MatVecMode jmode = job.mode;
  if (jmode == MatVecMode::kStoreVerify) {
    if (job.nstore < 0 || job.nstore > job.m) return hipErrorInvalidValue;
    if (job.nstore == job.m) jmode = MatVecMode::kStore;
    else if (job.nstore == 0) jmode = MatVecMode::kVerify;
    else if (job.m > kMaxM) return hipErrorInvalidValue;  // the stored/compared split lives in one launch
  }
  uint64_t maxlen = job.len;
  if (job.lens) {
    maxlen = 0;
    for (int s = 0; s < job.nstripes; ++s) maxlen = std::max<uint64_t>(maxlen, job.lens[s]);
    if (maxlen > 0xFFFFFFFFull) return hipErrorInvalidValue;  // slen[] is 32-bit
  }
  if (job.m == 0 || job.nstripes == 0 || maxlen == 0) return hipSuccess;
  // the wide LRC modes' fused encodes (EC6P6L9, EC6P8L10): one bit-sliced product instead of two passes
  if (jmode == MatVecMode::kStore && !job.lens && bs_plain_matches(job.k, job.m, job.coef))
    return launch_bs_plain(job, stream);
  if ((jmode == MatVecMode::kVerify || jmode == MatVecMode::kStoreVerify) && (job.k > kMaxK || !job.flags))
    return hipErrorInvalidValue;

  GfArgs a;
  for (int r0 = 0; r0 < job.m; r0 += kMaxM) {
    const int mc = std::min(kMaxM, job.m - r0);
    for (int c0 = 0; c0 < job.k; c0 += kMaxK) {
      const int kc = std::min(kMaxK, job.k - c0);
      MatVecMode mode = jmode;
      if (mode == MatVecMode::kStore && c0 > 0) mode = MatVecMode::kAccum;
      const bool verify = mode == MatVecMode::kVerify || mode == MatVecMode::kStoreVerify;
      const Shape sh = choose(mc);
      // the code-mode input counts take the fixed-K pipelined kernels (256 threads, one wave per
      // column chunk holding every output, 1 chunk per lane); anything else the runtime-k
      // kernel, whose verify policy is 128-thread workgroups with 2 chunks per lane unless the
      // outputs are split over waves
      const bool fixed = fixed_k(kc) && kc == job.k && mc <= fixed_max_m(kc) && mode != MatVecMode::kAccum &&
                         maxlen <= 0xFFFFFFFFull - 4096;  // 32-bit lane offsets
      const int threads = (!fixed && verify && sh.OS == 1) ? 128 : 256;
      // matrices of 4x4 / 2x2 dyadic blocks (encode of every code mode but the LRC local stripes,
      // coset-aligned reconstructs such as EC12P4's worst case) take the reduced-product kernel
      static const bool kLut = [] {
        const char* v = std::getenv("CFSEC_LUT");
        return !(v && v[0] == '0');
      }();
      DyPlan dy{0, 0};
      bool dy16 = false;
      if (fixed && r0 == 0 && mc == job.m && mode != MatVecMode::kStoreVerify) {
        std::vector<uint8_t> sub((size_t)mc * kc);
        for (int r = 0; r < mc; ++r)
          for (int c = 0; c < kc; ++c) sub[(size_t)r * kc + c] = job.coef[(size_t)r * job.k + c];
        dy16 = dyadic16_plan(sub.data(), mc, kc);
        if (!dy16) dy = dyadic_plan(sub.data(), mc, kc);
      }
      const bool lut = kLut && fixed && lut_outputs(kc, mc, dy16 || dy.B != 0) > 0;
      const size_t tile = fixed ? size_t(256) * 4 * dev::fixed_lane_dwords(kc, mc)
                                : size_t(threads / sh.OS) * dev::kLaneBytes * (verify ? kVerifyW : kStoreW);
      const int per_stripe = kc + mc;
      const int64_t sstride = affine_stride(job, c0, kc, r0, mc);
      int stripes_per_launch = sstride ? job.nstripes : kPtrSlots / per_stripe;
      if (job.lens) stripes_per_launch = std::min(stripes_per_launch, dev::kLenSlots);
      const size_t tiles = (maxlen + tile - 1) / tile;  // (varlen: per launch below)
      // one launch covers tiles * stripes workgroups: keep that in a 32-bit grid
      stripes_per_launch = (int)std::min<size_t>(stripes_per_launch, std::max<size_t>(1, 0x7fffffffu / tiles));
      if (fixed) stripes_per_launch = std::min(stripes_per_launch, 65535);  // grid.y = stripes
      if (tiles > 0x7fffffffu) return hipErrorInvalidValue;
      // stripes at unrelated addresses (more than one argument block holds) of the bit-sliced
      // encode shapes: one launch through a device table of row offsets for the whole 2 KiB column
      // runs (launch_bs_tab); the chunks below then code only the rows' tails
      uint64_t tab_full = 0;
      if (!sstride && mode == MatVecMode::kStore && !job.lens && kBs16 && kBsTab && c0 == 0 && r0 == 0 &&
          kc == job.k && mc == job.m && job.nstripes > stripes_per_launch && job.len >= kBs16Tile &&
          bs_matches(job.coef, mc, kc)) {
        static thread_local std::vector<const uint8_t*> rows;
        rows.resize((size_t)job.nstripes * per_stripe);
        bool al = true;
        for (int s = 0; s < job.nstripes; ++s) {
          for (int c = 0; c < kc; ++c) rows[(size_t)s * per_stripe + c] = job.in[(size_t)s * job.k + c];
          for (int r = 0; r < mc; ++r) rows[(size_t)s * per_stripe + kc + r] = job.out[(size_t)s * job.m + r];
        }
        for (const uint8_t* p : rows) al = al && !(reinterpret_cast<uintptr_t>(p) & 15);
        if (al) {
          a.flags = nullptr;
          a.pstore = a.pcmp = 0;
          bool ok = false;
          const uint64_t full = job.len / kBs16Tile * kBs16Tile;
          const hipError_t e = launch_bs_tab(kc, mc, a, rows.data(), (unsigned)job.nstripes, full, stream, &ok);
          if (e != hipSuccess) return e;
          if (ok) tab_full = full;
          if (ok && full == job.len) continue;
        }
      }
      for (int s0 = 0; s0 < job.nstripes; s0 += stripes_per_launch) {
        const int ns = std::min(stripes_per_launch, job.nstripes - s0);
        const int tab = sstride ? 1 : ns;  // stripes held in the pointer table
        uint64_t llen = job.len;
        if (job.lens) {
          llen = 0;
          for (int s = 0; s < ns; ++s) {
            a.slen[s] = (uint32_t)job.lens[s0 + s];
            llen = std::max<uint64_t>(llen, job.lens[s0 + s]);
          }
          if (llen == 0) continue;
        }
        size_t ltiles = (llen + tile - 1) / tile;
        a.len = llen;
        a.k = (uint32_t)kc;
        a.m = (uint32_t)mc;
        a.nstripes = (uint32_t)ns;
        a.tiles_per_stripe = (uint32_t)ltiles;
        a.flags = job.flags ? job.flags + s0 : nullptr;
        a.sstride = sstride;
        a.tab = (uint32_t)tab;
        a.nstore = (uint16_t)(mode == MatVecMode::kStoreVerify ? job.nstore - r0 : 0);
        a.varlen = job.lens ? 1 : 0;
        for (int r = 0; r < mc; ++r)
          for (int c = 0; c < kc; ++c)
            a.coef[r * kc + c] = job.coef[(size_t)(r0 + r) * job.k + (c0 + c)];
        for (int s = 0; s < tab; ++s) {
          for (int c = 0; c < kc; ++c)
            a.ptr[s * kc + c] = job.in[(size_t)(s0 + s) * job.k + c0 + c];
          for (int r = 0; r < mc; ++r)
            a.ptr[tab * kc + s * mc + r] = job.out[(size_t)(s0 + s) * job.m + r0 + r];
        }
        hipError_t e;
        // encodes of the bit-sliced shapes (gf_bs16.hip: EC16P20, EC16P20L2's fused encode) with 16-byte
        // aligned rows: the whole 2 KiB column runs through the network, the rest of each row through
        // the kernel chosen below
        const uint64_t full = mode == MatVecMode::kStore && !tab_full && !job.lens && kBs16 && c0 == 0 && r0 == 0 &&
                                      kc == job.k && mc == job.m && bs_ok(a, kc, mc, tab)
                                  ? llen / kBs16Tile * kBs16Tile
                                  : 0;
        // Verify of the same shapes: the bit-sliced repair kernel with nothing missing, every row compared
        const uint64_t vfull = mode == MatVecMode::kVerify && full == 0 && !job.lens && kBs16 && c0 == 0 &&
                                       r0 == 0 && kc == 16 && kc == job.k && mc == job.m && tab == 1 &&
                                       a.flags && bs_ok(a, kc, mc, tab)
                                   ? llen / kBs16Tile * kBs16Tile
                                   : 0;
        if (vfull) {
          a.pstore = 0;
          a.pcmp = (1u << mc) - 1;
          for (int i = 0; i < 16; ++i) a.src[i] = (uint8_t)i;
          a.zw = nullptr;
          a.nzw = 0;
          e = launch_bs16_repair(0, mc - 20, nullptr, nullptr, nullptr, a, (unsigned)ns, vfull, stream);
          if (e != hipSuccess) return e;
        }
        if (full || vfull || tab_full) {
          if (full) {
            e = launch_bs(kc, mc, a, (unsigned)ns, full, stream);
            if (e != hipSuccess) return e;
          }
          const uint64_t done = full ? full : vfull ? vfull : tab_full;
          if (done == llen) continue;
          for (int i = 0; i < tab * (kc + mc); ++i) a.ptr[i] += done;
          llen -= done;
          ltiles = (llen + tile - 1) / tile;
          a.len = llen;
          a.tiles_per_stripe = (uint32_t)ltiles;
        }
        const dim3 grid((unsigned)(ltiles * ns));
        if (lut) {
          const size_t lt = lut_tile_bytes(kc);
          const dim3 lgrid((unsigned)((llen + lt - 1) / lt), (unsigned)ns);
          e = launch_lut(kc, mc, mode, a, lgrid, stream);
          if (e != hipSuccess) return e;
          continue;
        }
        if (fixed && dy16) {
          e = launch_dy16(mc, mode, a, (unsigned)ns, stream);
          if (e != hipSuccess) return e;
          continue;
        }
        if (fixed && dy.B) {
          e = kc == 6    ? launch_dy<6>(mc, dy.B, dy.E, mode, a, (unsigned)ns, stream)
              : kc == 12 ? launch_dy<12>(mc, dy.B, dy.E, mode, a, (unsigned)ns, stream)
                         : launch_dy<16>(mc, dy.B, dy.E, mode, a, (unsigned)ns, stream);
          if (e != hipSuccess) return e;
          continue;
        }
        if (fixed) {
          const dim3 grid2((unsigned)ltiles, (unsigned)ns);
          e = mode == MatVecMode::kVerify        ? launch_fixed<MatVecMode::kVerify>(kc, mc, a, grid2, stream)
              : mode == MatVecMode::kStoreVerify ? launch_fixed<MatVecMode::kStoreVerify>(kc, mc, a, grid2, stream)
                                                 : launch_fixed<MatVecMode::kStore>(kc, mc, a, grid2, stream);
          if (e != hipSuccess) return e;
          continue;
        }
        switch (mode) {
          case MatVecMode::kStore: e = launch_mode<MatVecMode::kStore>(sh, a, grid, threads, stream); break;
          case MatVecMode::kAccum: e = launch_mode<MatVecMode::kAccum>(sh, a, grid, threads, stream); break;
          case MatVecMode::kStoreVerify:
            e = launch_mode<MatVecMode::kStoreVerify>(sh, a, grid, threads, stream);
            break;
          default: e = launch_mode<MatVecMode::kVerify>(sh, a, grid, threads, stream); break;
        }
        if (e != hipSuccess) return e;
      }
    }
  }
  return hipSuccess;
}

namespace {
constexpr int kGatherSlots = 256;  // items and words per gather launch (argument block < 3 KiB)
struct GatherArgs {
  uint32_t* tmp;
  uint32_t* out;
  uint32_t nitems;
  uint32_t acc;
  uint32_t item[kGatherSlots];
  uint32_t word[kGatherSlots];
  uint16_t first[kGatherSlots + 1];
};

// One thread per item: OR of its tasks' words, which are reset to 0.
__global__ __launch_bounds__(kGatherSlots) void flag_gather_kernel(const GatherArgs a) {
  const uint32_t o = threadIdx.x;
  if (o >= a.nitems) return;
  uint32_t v = 0;
  for (int j = a.first[o]; j < a.first[o + 1]; ++j) {
    v |= a.tmp[a.word[j]];
    a.tmp[a.word[j]] = 0;
  }
  uint32_t* p = a.out + a.item[o];
  *p = a.acc ? (*p | (v != 0 ? 1u : 0u)) : (v != 0 ? 1u : 0u);
}
}  // namespace

namespace {
__global__ __launch_bounds__(256) void stream_copy_kernel(const dev::u32x4* __restrict__ src, dev::u32x4* __restrict__ dst,
                                                          size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}
}  // namespace

hipError_t launch_stream_copy(void* dst, const void* src, size_t bytes, hipStream_t stream) {
  if ((bytes & 15) || ((uintptr_t)dst & 15) || ((uintptr_t)src & 15) || (bytes && (!dst || !src)))
    return hipErrorInvalidValue;
  if (bytes == 0) return hipSuccess;
  const size_t n = bytes / 16;
  // 8192 x 256 threads: tools/rot_probe.hip's flat copy (32 resident workgroups per CU)
  const unsigned grid = (unsigned)std::min<size_t>(8192, (n + 255) / 256);
  hipLaunchKernelGGL(stream_copy_kernel, dim3(grid), dim3(256), 0, stream, static_cast<const dev::u32x4*>(src),
                     static_cast<dev::u32x4*>(dst), n);
  return hipGetLastError();
}

hipError_t launch_flag_gather(uint32_t* tmp, uint32_t* out, const int* item, const int* word, int n,
                              bool accumulate, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  if (!tmp || !out || !item || !word) return hipErrorInvalidValue;
  GatherArgs a;
  a.tmp = tmp;
  a.out = out;
  a.acc = accumulate ? 1u : 0u;
  int j = 0;
  while (j < n) {
    // one launch: whole items only, up to kGatherSlots items and kGatherSlots words
    int ni = 0, nw = 0;
    a.first[0] = 0;
    while (j < n && ni < kGatherSlots) {
      int e = j;
      while (e < n && item[e] == item[j]) ++e;
      if (e - j > kGatherSlots) return hipErrorInvalidValue;
      if (nw + (e - j) > kGatherSlots) break;
      a.item[ni] = (uint32_t)item[j];
      for (int q = j; q < e; ++q) a.word[nw++] = (uint32_t)word[q];
      a.first[++ni] = (uint16_t)nw;
      j = e;
    }
    a.nitems = (uint32_t)ni;
    hipLaunchKernelGGL(flag_gather_kernel, dim3(1), dim3(kGatherSlots), 0, stream, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_dy16_repair(const Dy16RepairJob& job, hipStream_t stream) {
  using dev::kPtrSlots;
  const int nd = job.nd, ne = job.e, mo = nd + 20 + ne;
  if (nd < 0 || nd > 4 || (ne != 0 && ne != 2) || job.nstripes < 0 || !job.coef || !job.in || !job.out ||
      (job.pcmp && !job.flags) || (job.pstore | job.pcmp) >> (20 + ne))
    return hipErrorInvalidValue;
  if (job.nstripes == 0) return hipSuccess;
  uint64_t maxlen = job.len;
  if (job.lens) {
    maxlen = 0;
    for (int s = 0; s < job.nstripes; ++s) maxlen = std::max<uint64_t>(maxlen, job.lens[s]);
  }
  if (maxlen == 0) return hipSuccess;
  if (maxlen > 0xFFFFFFFFull - 4096) return hipErrorInvalidValue;  // 32-bit lane offsets, slen[]
  // one stride between stripes on every row: one affine launch
  int64_t sstride = 0;
  if (job.nstripes > 1 && !job.lens) {
    const auto addr = [](const void* p) { return (int64_t)(uintptr_t)p; };
    sstride = addr(job.in[16]) - addr(job.in[0]);
    for (int s = 1; s < job.nstripes && sstride; ++s) {
      for (int c = 0; c < 16 && sstride; ++c)
        if (addr(job.in[(size_t)s * 16 + c]) != addr(job.in[c]) + s * sstride) sstride = 0;
      for (int r = 0; r < mo && sstride; ++r)
        if (addr(job.out[(size_t)s * mo + r]) != addr(job.out[r]) + s * sstride) sstride = 0;
    }
  }
  int per = sstride ? std::min(job.nstripes, 65535) : kPtrSlots / (16 + mo);
  if (job.lens) per = std::min(per, dev::kLenSlots);
  dev::GfArgs a;
  a.k = 16;
  a.m = (uint32_t)mo;
  a.sstride = sstride;
  a.nstore = 0;
  a.pstore = job.pstore;
  a.pcmp = job.pcmp;
  a.zw = job.zero_words;
  a.nzw = job.nzero;
  std::memcpy(a.src, job.src, 16);
  std::memcpy(a.coef, job.coef, (size_t)(20 + ne + nd) * 16);
  // Stripes at unrelated addresses (every shard its own buffer, as blobnode assembles a bid): the
  // bit-sliced repair over a table of 32-bit row offsets, ~20 stripes per launch, for the whole
  // 2 KiB column runs; the dyadic kernel below then covers only the rows' tails.
  // the stored rows' checksums in the bit-sliced pass: rows = the missing data rows then the stored
  // parity rows, in order (gf_bs16.hip's checksummed rows)
  BsCrcReq crc_req;
  if (job.crc_words && job.crc_done && !job.lens && job.syn && nd <= kBsRepairMaxNd) {
    const int ncrc = nd + __builtin_popcount(job.pstore);
    if (ncrc >= 1 && ncrc <= 4) {
      crc_req.nrows = ncrc;
      crc_req.stride = job.crc_stride;
      crc_req.mode = job.crc_mode;
      for (int q = 0; q < 4; ++q) crc_req.slot[q] = job.crc_slot[q];
    }
  }
  uint64_t tab_full = 0;
  // CFSEC_BS_FORCE_TAB=1 (A/B, read once): affine batches through the table launch too
  static const bool kForceTab = [] {
    const char* v = std::getenv("CFSEC_BS_FORCE_TAB");
    return v && v[0] == '1';
  }();
  if ((!sstride || kForceTab) && job.nstripes > 1 && job.syn && kBs16 && nd <= kBsRepairMaxNd && !job.lens && kBsTab &&
      bs_matches(job.coef, 20 + ne, 16) && job.len >= kBs16Tile) {
    static thread_local std::vector<const uint8_t*> rows;
    rows.resize((size_t)job.nstripes * (16 + mo));
    bool al = true;
    for (int s = 0; s < job.nstripes; ++s) {
      for (int c = 0; c < 16; ++c) rows[(size_t)s * (16 + mo) + c] = job.in[(size_t)s * 16 + c];
      for (int r = 0; r < mo; ++r) rows[(size_t)s * (16 + mo) + 16 + r] = job.out[(size_t)s * mo + r];
    }
    for (const uint8_t* p : rows) al = al && !(reinterpret_cast<uintptr_t>(p) & 15);
    if (al) {
      uint8_t missing[4] = {};
      for (int i = 0; i < 16; ++i)
        if (job.src[i] >= 16) missing[job.src[i] - 16] = (uint8_t)i;
      dev::GfArgs t = a;
      t.flags = job.flags;
      bool ok = false, fused = false;
      const uint64_t full = job.len / kBs16Tile * kBs16Tile;
      const bool want_crc = crc_req.nrows && full == job.len;
      if (want_crc) {  // the words are zeroed by the caller: no in-kernel zeroing to race the atomics
        t.zw = nullptr;
        t.nzw = 0;
      }
      const hipError_t e = launch_bs16_repair_tab(nd, ne, missing, job.prow, job.ainv, t, rows.data(),
                                                  (unsigned)job.nstripes, full, stream, &ok,
                                                  want_crc ? &crc_req : nullptr, job.crc_words, &fused);
      if (e != hipSuccess) return e;
      if (fused)
        for (int s = 0; s < job.nstripes; ++s) job.crc_done[s] = 1;
      if (ok) {
        tab_full = full;
        a.zw = nullptr;  // the first launch zeroed them
        a.nzw = 0;
        if (full == job.len) return hipSuccess;
      }
    }
  }
  for (int s0 = 0; s0 < job.nstripes; s0 += per) {
    const int ns = std::min(per, job.nstripes - s0);
    const int tab = sstride ? 1 : ns;
    uint64_t llen = job.len;
    a.varlen = job.lens ? 1 : 0;
    if (job.lens) {
      llen = 0;
      for (int s = 0; s < ns; ++s) {
        a.slen[s] = (uint32_t)job.lens[s0 + s];
        llen = std::max<uint64_t>(llen, job.lens[s0 + s]);
      }
      if (llen == 0) continue;
    }
    a.len = llen;
    a.nstripes = (uint32_t)ns;
    a.tab = (uint32_t)tab;
    a.flags = job.flags ? job.flags + s0 : nullptr;
    for (int s = 0; s < tab; ++s) {
      for (int c = 0; c < 16; ++c) a.ptr[s * 16 + c] = job.in[(size_t)(s0 + s) * 16 + c];
      for (int r = 0; r < mo; ++r) a.ptr[tab * 16 + s * mo + r] = job.out[(size_t)(s0 + s) * mo + r];
    }
    // the syndrome form of the bit-sliced network (gf_bs16.hip) for the whole 2 KiB column runs of
    // 16-byte aligned rows, the dyadic repair kernel for the rest of each row
    const uint64_t full = job.syn && kBs16 && nd <= kBsRepairMaxNd && tab == 1 && !tab_full && !job.lens &&
                                  bs_matches(job.coef, 20 + ne, 16) && aligned16(a, tab * (16 + mo))
                              ? llen / kBs16Tile * kBs16Tile
                              : 0;
    if (full) {
      uint8_t missing[4] = {};
      for (int i = 0; i < 16; ++i)
        if (job.src[i] >= 16) missing[job.src[i] - 16] = (uint8_t)i;
      const bool want_crc = crc_req.nrows && full == llen;
      bool fused = false;
      const dev::GfArgs* ra = &a;
      static thread_local dev::GfArgs nz;
      if (want_crc && a.nzw) {  // the words are zeroed by the caller: no in-kernel zeroing to race the atomics
        std::memcpy(&nz, &a, sizeof(dev::GfArgs));
        nz.zw = nullptr;
        nz.nzw = 0;
        ra = &nz;
      }
      const hipError_t e = launch_bs16_repair(nd, ne, missing, job.prow, job.ainv, *ra, (unsigned)ns, full, stream,
                                              want_crc ? &crc_req : nullptr,
                                              want_crc ? job.crc_words + (size_t)s0 * job.crc_stride : nullptr, &fused);
      if (e != hipSuccess) return e;
      if (fused)
        for (int s = 0; s < ns; ++s) job.crc_done[s0 + s] = 1;
    }
    const uint64_t done = full ? full : tab_full;  // columns the bit-sliced kernel covered
    if (done < llen) {
      const dev::GfArgs* ta = &a;
      static thread_local dev::GfArgs tail;
      if (done) {
        std::memcpy(&tail, &a, sizeof(dev::GfArgs));
        for (int i = 0; i < tab * (16 + mo); ++i) tail.ptr[i] = a.ptr[i] + done;
        tail.len = llen - done;
        ta = &tail;
      }
      const hipError_t e = launch_dy16_repair_args(nd, ne, *ta, (unsigned)ns, stream);
      if (e != hipSuccess) return e;
    }
    a.zw = nullptr;  // the first launch zeroed them
    a.nzw = 0;
  }
  return hipSuccess;
}

}  // namespace cfsec
