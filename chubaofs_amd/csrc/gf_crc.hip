// gf_crc.hip -- host side of the fused matvec + shard CRC32 kernels (device code: gf_crc.hpp).
#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>
#include <vector>

#include "gf_crc.hpp"
#include "gf_launch.hpp"

namespace cfsec {
namespace crcdev {
CFSEC_CRC_EXTERN(6)
CFSEC_CRC_EXTERN(8)
CFSEC_CRC_EXTERN(12)
CFSEC_CRC_EXTERN(16)
CFSEC_CRC_EXTERN(18)
}  // namespace crcdev

namespace {

using crcdev::GfCrcArgs;
constexpr uint32_t kX0 = 0x80000000u;    // x^0 (reflected)
constexpr uint32_t kX1 = 0x40000000u;    // x^1
constexpr uint32_t kXInv = 0xDB710641u;  // x^-1 mod P: the y with y*x = x^0 (P has a constant term)

uint32_t mulmod(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (uint32_t bit = kX0; bit; bit >>= 1) {
    if (a & bit) p ^= b;
    b = (b >> 1) ^ ((b & 1u) ? crcdev::kPoly : 0u);
  }
  return p;
}

// x^e mod P for any integer e (e < 0: powers of x^-1).
uint32_t xpow(int64_t e) {
  uint32_t base = e >= 0 ? kX1 : kXInv;
  uint64_t n = e >= 0 ? (uint64_t)e : (uint64_t)(-e);
  uint32_t p = kX0;
  while (n) {
    if (n & 1) p = mulmod(p, base);
    base = mulmod(base, base);
    n >>= 1;
  }
  return p;
}

std::vector<uint32_t> host_tables() {
  std::vector<uint32_t> t(crcdev::kTabWords + crcdev::kBasisWords + crcdev::kShiftWords);
  const uint32_t k4096 = xpow(8 * 4096);
  for (int j = 0; j < 16; ++j)  // Fj[b] = f(0, 16-byte piece with byte j = b, the rest 0)
    for (uint32_t b = 0; b < 256; ++b) {
      uint32_t c = 0;
      for (int i = 0; i < 16; ++i) {
        c ^= i == j ? b : 0u;
        for (int q = 0; q < 8; ++q) c = (c & 1u) ? (c >> 1) ^ crcdev::kPoly : c >> 1;
      }
      t[j * 256 + b] = c;
    }
  for (int q = 0; q < 4; ++q)  // Gq[b] = shift(b << 8q, 4096)
    for (uint32_t b = 0; b < 256; ++b) t[(16 + q) * 256 + b] = mulmod(k4096, b << (8 * q));
  uint32_t* nt = t.data() + crcdev::kByteTabWords;
  for (int p = 0; p < 32; ++p)  // Np[n] = f(0, 16-byte piece with nibble p = n, the rest 0)
    for (uint32_t n = 0; n < 16; ++n) {
      uint8_t piece[16] = {};
      piece[p / 2] = (uint8_t)(n << (4 * (p & 1)));
      uint32_t c = 0;
      for (uint8_t b : piece) {
        c ^= b;
        for (int i = 0; i < 8; ++i) c = (c & 1u) ? (c >> 1) ^ crcdev::kPoly : c >> 1;
      }
      nt[p * 16 + n] = c;
    }
  for (int q = 0; q < 8; ++q)  // Hq[n] = shift(n << 4q, 4096)
    for (uint32_t n = 0; n < 16; ++n) nt[(32 + q) * 16 + n] = mulmod(k4096, n << (4 * q));
  uint32_t* ft = nt + crcdev::kNibTabWords;
  for (int w = 0; w < 5; ++w)  // Q(w, f)[e]: word w of (d0..d3, R) = e << 5f, the rest 0
    for (int f = 0; f < crcdev::kFiveFields; ++f)
      for (uint32_t e = 0; e < (f < 6 ? 32u : 4u); ++e) {
        const uint32_t v = e << (5 * f);
        uint32_t c = 0;
        if (w == 4) {
          c = mulmod(k4096, v);
        } else {
          for (int i = 0; i < 16; ++i) {
            c ^= i / 4 == w ? (v >> (8 * (i % 4))) & 0xFFu : 0u;
            for (int q = 0; q < 8; ++q) c = (c & 1u) ? (c >> 1) ^ crcdev::kPoly : c >> 1;
          }
        }
        ft[(w * crcdev::kFiveFields + f) * 32 + e] = c;
      }
  for (int j = 0; j < 256; ++j) {  // basis of shift(., 16*(255-j)) for thread j
    const uint32_t kj = xpow(8LL * 16 * (255 - j));
    for (int i = 0; i < 32; ++i) t[crcdev::kTabWords + j * 32 + i] = mulmod(kj, 1u << i);
    t[crcdev::kTabWords + crcdev::kBasisWords + j] = kj;
  }
  return t;
}

}  // namespace

// The lookup tables on the current device, uploaded once per device.
hipError_t crc_device_tables(const uint32_t** out) {
  static std::mutex mu;
  static std::map<int, uint32_t*> per_device;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> l(mu);
  auto it = per_device.find(dev);
  if (it == per_device.end()) {
    static const std::vector<uint32_t> host = host_tables();
    uint32_t* d = nullptr;
    e = hipMalloc(reinterpret_cast<void**>(&d), host.size() * 4);
    if (e != hipSuccess) return e;
    e = hipMemcpy(d, host.data(), host.size() * 4, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      (void)hipFree(d);
      return e;
    }
    it = per_device.emplace(dev, d).first;
  }
  *out = it->second;
  return hipSuccess;
}

uint32_t crc_xpow(int64_t e) { return xpow(e); }
uint32_t crc_mulmod(uint32_t a, uint32_t b) { return mulmod(a, b); }

namespace {

uint32_t env_u32(const char* name, uint32_t dflt) {
  const char* v = std::getenv(name);
  return v && *v ? (uint32_t)std::strtoul(v, nullptr, 10) : dflt;
}

// As gf_kernels.hip's affine_stride, for the whole job.
int64_t affine_stride(const MatVecJob& job) {
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

template <bool CIN>
int lds_per_cu(int k, int m) {
  static std::mutex mu;
  static std::map<std::pair<int, int>, int> cache;  // (device, k * 64 + m)
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  std::lock_guard<std::mutex> l(mu);
  const auto key = std::make_pair(dev, k * 64 + m);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  int n = 0;
  switch (k) {
    case 6: n = crcdev::lds_blocks_per_cu<6, CIN>(m); break;
    case 8: n = crcdev::lds_blocks_per_cu<8, CIN>(m); break;
    case 12: n = crcdev::lds_blocks_per_cu<12, CIN>(m); break;
    case 16: n = crcdev::lds_blocks_per_cu<16, CIN>(m); break;
    default: n = 0;
  }
  cache.emplace(key, n);
  return n;
}

template <bool CIN>
hipError_t launch_crc(int k, int m, const GfCrcArgs& a, dim3 grid, hipStream_t st, int dy) {
  switch (k) {
    case 6: return crcdev::launch_crc_k<6, CIN>(m, a, grid, st, dy);
    case 8: return crcdev::launch_crc_k<8, CIN>(m, a, grid, st, dy);
    case 12: return crcdev::launch_crc_k<12, CIN>(m, a, grid, st, dy);
    case 16: return crcdev::launch_crc_k<16, CIN>(m, a, grid, st, dy);
    case 18: return crcdev::launch_crc_k<18, CIN>(m, a, grid, st, dy);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

// The lookup-product fused kernel (gf_crc_lds_kernel): m <= 4, k <= 16, and (round 6) k = 6, m = 12 --
// EC6P10L2's fused LRC encode with every shard checksummed, any 6 x 12 matrix (CFSEC_CRC_LDS=0 /
// CFSEC_CRC_LDS12=0 keep the v_perm kernels for A/B, which need the 2x2-dyadic + 2 plain-row form).
static bool crc_lds_on() {
  static const bool v = env_u32("CFSEC_CRC_LDS", 1) != 0;
  return v;
}
static bool crc_lds12_on() {
  static const bool v = crc_lds_on() && env_u32("CFSEC_CRC_LDS12", 1) != 0;
  return v;
}

bool matvec_crc_supported(int k, int m, size_t len, const uint8_t* coef) {
  // the fused kernels exist for the input counts of the code modes of SURVEY §8, m <= 6 outputs, and
  // EC6P10L2's fused encode (6 x (10 dyadic + 2 local) rows)
  if (m < 1 || len > 0xFFFFFFFFull - crcdev::kTile) return false;
  if (bs_crc_matches(k, m, coef)) return true;  // the bit-sliced fused kernels (gf_bs_crc.hip)
  const bool crc_k = k == 6 || k == 8 || k == 12 || k == 16 || k == 18;
  if (!crc_k) return false;
  if (m <= 6) return true;
  if (k == 6 && m == 12 && crc_lds12_on()) return true;
  if (k == 6 && m == 12 && coef) {
    const DyPlan dp = dyadic_plan(coef, m, k);
    return dp.B == 2 && dp.E == 2;
  }
  return false;
}

uint32_t crc32_shift_ones(size_t len) { return mulmod(xpow(8 * (int64_t)len), 0xFFFFFFFFu) ^ 0xFFFFFFFFu; }

bool matvec_crc_accepts(const MatVecJob& job, int crc_stride, const int* slot) {
  if (job.mode != MatVecMode::kStore || !matvec_crc_supported(job.k, job.m, job.len, job.coef) || !slot ||
      crc_stride <= 0 || crc_stride > 256 || job.nstripes < 0 || !job.coef || !job.in || !job.out)
    return false;
  const bool cin = slot[0] >= 0;
  for (int i = 0; i < job.k + job.m; ++i) {
    const bool want = i >= job.k || cin;
    if (want && (slot[i] < 0 || slot[i] >= crc_stride)) return false;
  }
  // EC6P10L2's fused encode is instantiated with its inputs checksummed only (every shard, as Put does)
  return !(job.m > 6 && !cin);
}

hipError_t launch_matvec_crc(const MatVecJob& job, uint32_t* crc, int crc_stride, const int* slot,
                             hipStream_t stream, bool zero) {
  if (!crc || !matvec_crc_accepts(job, crc_stride, slot)) return hipErrorInvalidValue;
  const int k = job.k, m = job.m;
  const bool cin = slot[0] >= 0;
  hipError_t e = zero ? hipMemsetAsync(crc, 0, sizeof(uint32_t) * (size_t)crc_stride * job.nstripes, stream)
                      : hipSuccess;
  if (e != hipSuccess || job.nstripes == 0 || job.len == 0) return e;
  // EC6P10L2's fused LRC encode and EC12P4's encode with every shard checksummed: the bit-sliced
  // network, checksums from its bit planes (gf_bs_crc.hip, round 6)
  if (cin && bs_crc_takes(job, crc_stride, slot)) return launch_bs_crc(job, crc, crc_stride, slot, stream);

  GfCrcArgs a{};
  e = crc_device_tables(&a.tabs);
  if (e != hipSuccess) return e;
  const uint32_t tiles = (uint32_t)((job.len + crcdev::kTile - 1) / crcdev::kTile);
  const int64_t sstride = affine_stride(job);
  const int per = sstride ? job.nstripes : crcdev::kPtrSlots / (k + m);
  const int stripes_per_launch = std::min(per, 65535);
  for (int r = 0; r < m; ++r)
    for (int c = 0; c < k; ++c) a.coef[r * k + c] = job.coef[(size_t)r * k + c];
  // matrices of dyadic blocks the v_perm kernel has a reduced-product form for: 4 outputs of 4x4
  // blocks (EC12P4 / EC16P4 encode, coset-aligned repairs), 6 x 6 of 2x2 blocks (EC6P6 encode)
  const DyPlan dp = (m == 4 && k % 4 == 0) || (k == 6 && (m == 6 || m == 12)) ? dyadic_plan(a.coef, m, k)
                                                                             : DyPlan{0, 0};
#ifndef CFSEC_CRC_DY2
#define CFSEC_CRC_DY2 1  // A/B switch for the 2x2 form
#endif
  int dy = dp.E == 0 && ((dp.B == 4 && m == 4) || (CFSEC_CRC_DY2 && dp.B == 2 && m == 6 && k == 6)) ? dp.B : 0;
  if (k == 6 && m == 12 && dp.B == 2 && dp.E == 2) {  // EC6P10L2 fused encode + its 18 checksums
    if (!cin) return hipErrorInvalidValue;             // (the only form instantiated: inputs checksummed)
    dy = 2;
  }
  // m <= 4, k <= 16: the lookup-product kernel (gf_crc_lds_kernel; CFSEC_CRC_LDS=0 keeps the v_perm
  // kernels for A/B): EC12P4 8 x 64 MiB encode + 16 checksums 225-230 -> 200 us
  // (profiles/r03/crc_lds_ab*.txt)
  if (crc_lds_on() && m <= 4 && k <= 16) dy = -1;
  // EC6P10L2's fused LRC encode + 18 checksums (C4) on the same lookup kernel with 16-byte entries
  // (round 6): C4's put batch 245 -> 211 us per call against the v_perm form (profiles/r06/c4_crc_lds12.txt)
  if (crc_lds12_on() && k == 6 && m == 12 && cin) dy = -1;
  // Workgroups per launch.  The v_perm kernels: ~1024, each folding ~11 tiles per row before its
  // per-thread basis epilogue (16 rows x 32 columns); 512 / 2048 / 4096 were 3-7 % slower
  // (profiles/r01/crc_wgs_sweep.txt).  The lookup kernel: exactly the resident count (its 48-64 KiB
  // LDS table allows 2-3 per CU), so no second partial wave of workgroups: 768 vs 1024 for k = 12
  // is 200 vs 220 us.  CFSEC_CRC_GROUPS overrides (probes).
#ifndef CFSEC_CRC_GROUPS
#define CFSEC_CRC_GROUPS 1024
#endif
  static const uint32_t kGroupsEnv = env_u32("CFSEC_CRC_GROUPS", 0);
  uint32_t total = CFSEC_CRC_GROUPS;
  if (dy == -1) {
    const int per_cu = cin ? lds_per_cu<true>(k, m) : lds_per_cu<false>(k, m);
    int dev = 0, cus = 0;
    if (per_cu > 0 && hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0)
      total = (uint32_t)(per_cu * cus * crcdev::kLdsV);
  }
  if (kGroupsEnv) total = kGroupsEnv;
  const uint32_t want = std::max<uint32_t>(1, total / (uint32_t)std::min(job.nstripes, stripes_per_launch));
  uint32_t groups = std::min<uint32_t>({tiles, want, (uint32_t)crcdev::kMaxGroups});
  const uint32_t tpw = (tiles + groups - 1) / groups;
  groups = (tiles + tpw - 1) / tpw;

  a.len = job.len;
  a.k = (uint32_t)k;
  a.m = (uint32_t)m;
  a.tiles = tiles;
  a.tpw = tpw;
  a.sstride = sstride;
  a.fin = crc32_shift_ones(job.len);
  a.crc_stride = (uint32_t)crc_stride;
  for (int i = 0; i < k + m; ++i) a.slot[i] = (uint8_t)std::max(slot[i], 0);
  for (uint32_t g = 0; g < groups; ++g) {
    const int64_t end = (int64_t)std::min<uint64_t>((uint64_t)(g + 1) * tpw, tiles) * crcdev::kTile;
    a.gconst[g] = xpow(8 * ((int64_t)job.len - end));
  }
  for (int s0 = 0; s0 < job.nstripes; s0 += stripes_per_launch) {
    const int ns = std::min(stripes_per_launch, job.nstripes - s0);
    const int tab = sstride ? 1 : ns;
    a.tab = (uint32_t)tab;
    a.crc = crc + (size_t)s0 * crc_stride;
    for (int s = 0; s < tab; ++s) {
      for (int c = 0; c < k; ++c) a.ptr[s * k + c] = job.in[(size_t)(s0 + s) * k + c];
      for (int r = 0; r < m; ++r) a.ptr[tab * k + s * m + r] = job.out[(size_t)(s0 + s) * m + r];
    }
    // the lookup kernel runs kLdsV virtual groups per workgroup (a trailing one past the tiles idles)
    const dim3 grid(dy == -1 ? (groups + crcdev::kLdsV - 1) / crcdev::kLdsV : groups, (unsigned)ns);
    e = cin ? launch_crc<true>(k, m, a, grid, stream, dy) : launch_crc<false>(k, m, a, grid, stream, dy);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace cfsec
