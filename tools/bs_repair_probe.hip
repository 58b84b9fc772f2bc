// bs_repair_probe.hip -- C5's repair pass in bit-sliced form (dev probe, round 4).
//
// The EC16P20L2 tasklet of BASELINE config 5 (64 bids x S = 262,144, rows {0,1,16,17} lost):
// per bid, the reference's Reconstruct then Verify.  Bit-sliced form (chubaofs_amd/csrc/bs_net_ec16p20l2.hpp):
//   1. the 16 input slots (present data rows in their slots, the first nd present parities standing
//      in for the missing data rows) as bit planes; the stand-ins' planes set aside, their slots zeroed;
//   2. syndromes: s_k = stored(p_k) ^ row p_k of the network over the present data;
//   3. the missing data rows d = A^-1 s in byte form (A: the nd x nd block of the parity matrix at
//      rows p_k, columns of the missing data; v_perm products with run-time tables), stored, and
//      transposed into their slots;
//   4. the full network: each parity row stored (rebuilt) or compared with its stored copy (Verify;
//      the p_k rows hold by construction and are skipped).
// Persistent waves, 8 per CU (2 per SIMD); the next tile's slots 0-6 are prefetched into LDS by
// global_load_lds while the network runs, slots 7-15 are loaded at the tile's top, and each compared
// row comes through a 3-deep LDS ring filled 2 compared rows ahead.  Every wait on those copies is a
// conservative s_waitcnt (vector memory operations retire in issue order).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../chubaofs_amd/csrc bs_repair_probe.hip -o bs_repair_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "bs_net_ec16p20l2.hpp"

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

constexpr int K = 16, NP = 22, ROWS = K + NP, NB = 64, NT = 3;
constexpr size_t S = 262144;
constexpr int kWT = 2048;                   // bytes per row per wave tile (64 lanes x 32 B)
constexpr int NPF = 7;                      // slots prefetched into LDS
constexpr int kRing = 3;                    // LDS ring of compared rows
constexpr int kWaveLds = (NPF + kRing) * kWT;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct RepairArgs {
  uint8_t* base;            // bid b, row r at base + (b * ROWS + r) * S
  uint32_t* flags;          // per bid, set when Verify fails
  const uint8_t* zero;      // kWT zero bytes: the missing data rows' slots load from here
  uint32_t ntiles;
  int nd;
  uint8_t slot[4];          // missing data row k (its slot)
  uint8_t prow[4];          // the parity row standing in for it (0..21)
  uint32_t pstore, pcmp;    // parity rows stored / compared
  u32x4 t01[16];            // A^-1 product tables, entry j * 4 + k
  uint32_t t2[16];
};

__device__ __forceinline__ void swapmove(uint32_t& a, uint32_t& b, int s, uint32_t m) {
  const uint32_t t = ((a >> s) ^ b) & m;
  b ^= t;
  a ^= t << s;
}
__device__ __forceinline__ void transpose8(uint32_t* w) {
#pragma unroll
  for (int i = 0; i < 8; i += 2) swapmove(w[i], w[i + 1], 1, 0x55555555u);
#pragma unroll
  for (int i = 0; i < 8; ++i)
    if (!(i & 2)) swapmove(w[i], w[i + 2], 2, 0x33333333u);
#pragma unroll
  for (int i = 0; i < 4; ++i) swapmove(w[i], w[i + 4], 4, 0x0F0F0F0Fu);
}
__device__ __forceinline__ u32x4 ld16nt(const uint8_t* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
}
__device__ __forceinline__ void st16nt(uint8_t* p, u32x4 v) {
  __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
}
__device__ __forceinline__ void glds16(const uint8_t* g, uint8_t* l) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}
// a row's 32 lane bytes: [16 lane, +16) and [1024 + 16 lane, +16) of the wave's 2 KiB
__device__ __forceinline__ void ld_row(const uint8_t* p, uint32_t* x) {
  const u32x4 a = ld16nt(p), b = ld16nt(p + 1024);
  x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
}
__device__ __forceinline__ void lds_row(const uint8_t* l, uint32_t lane, uint32_t* x) {
  const u32x4 a = *reinterpret_cast<const u32x4*>(l + lane * 16), b = *reinterpret_cast<const u32x4*>(l + 1024 + lane * 16);
  x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
}
__device__ __forceinline__ void st_row(uint8_t* p, const uint32_t* o) {
  st16nt(p, u32x4{o[0], o[1], o[2], o[3]});
  st16nt(p + 1024, u32x4{o[4], o[5], o[6], o[7]});
}
__device__ __forceinline__ void glds_row(const uint8_t* g, uint8_t* l) {
  glds16(g, l);
  glds16(g + 1024, l + 1024);
}
constexpr unsigned waitcnt_vm(unsigned n) { return (n & 0xFu) | (0x7u << 4) | (0xFu << 8) | ((n >> 4) << 14); }

// acc ^= c * v over 8 dwords (v_perm 3-bit-field products; q/t2: c's tables)
__device__ __forceinline__ void mul_acc8(uint32_t* acc, const uint32_t* s0, const uint32_t* s1, const uint32_t* s2,
                                         const u32x4 q, uint32_t t2) {
#pragma unroll
  for (int w = 0; w < 8; ++w)
    acc[w] = cfsec::dev::bs_x3(acc[w], __builtin_amdgcn_perm(q.y, q.x, s0[w]), __builtin_amdgcn_perm(q.w, q.z, s1[w])) ^
             __builtin_amdgcn_perm(0u, t2, s2[w]);
}

template <int ND>
__device__ __forceinline__ void solve(const RepairArgs& a, uint32_t (&x)[128], uint32_t (&y)[4][8], uint8_t* const* mrow,
                                      size_t off) {
  // y[k]: syndrome planes -> bytes; d_j = sum_k Ainv[j][k] * s_k
  uint32_t d[ND][8];
#pragma unroll
  for (int j = 0; j < ND; ++j)
#pragma unroll
    for (int w = 0; w < 8; ++w) d[j][w] = 0u;
#pragma unroll
  for (int k = 0; k < ND; ++k) {
    transpose8(y[k]);
    uint32_t s0[8], s1[8], s2[8];
#pragma unroll
    for (int w = 0; w < 8; ++w) {
      s0[w] = y[k][w] & 0x07070707u;
      s1[w] = (y[k][w] >> 3) & 0x07070707u;
      s2[w] = (y[k][w] >> 6) & 0x03030303u;
    }
#pragma unroll
    for (int j = 0; j < ND; ++j) mul_acc8(d[j], s0, s1, s2, a.t01[j * 4 + k], a.t2[j * 4 + k]);
  }
#pragma unroll
  for (int j = 0; j < ND; ++j) {
    st_row(mrow[j] + off, d[j]);
    transpose8(d[j]);
    // into its slot (zero so far): x ^= d & mask, the mask uniform per slot -- no register indexing
#pragma unroll
    for (int i = 0; i < K; ++i) {
      const uint32_t m = i == a.slot[j] ? ~0u : 0u;
#pragma unroll
      for (int w = 0; w < 8; ++w) x[8 * i + w] ^= d[j][w] & m;
      if (cfsec::dev::kBsEc16p20l2Paired && !(i & 1))  // paired basis: an odd slot's d joins its pair's sum too
#pragma unroll
        for (int w = 0; w < 8; ++w) x[8 * i + w] ^= d[j][w] & (i + 1 < 16 && a.slot[j] == i + 1 ? ~0u : 0u);
    }
  }
}

template <int ND>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void bs_repair(const RepairArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[8][kWaveLds];
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint8_t* in_l = lds[wave];
  uint8_t* ring = lds[wave] + NPF * kWT;
  constexpr uint32_t tpb = (uint32_t)(S / kWT);
  const uint32_t nw = gridDim.x * 8;
  const auto row_ptr = [&](uint32_t t, int r) { return a.base + ((size_t)(t / tpb) * ROWS + r) * S + (size_t)(t % tpb) * kWT; };
  const auto slot_ptr = [&](uint32_t t, int i) -> const uint8_t* {  // data row i, or zeros where it is missing
    bool miss = false;
#pragma unroll
    for (int k = 0; k < ND; ++k) miss |= a.slot[k] == i;
    return miss ? a.zero : row_ptr(t, i);
  };
  uint32_t t = blockIdx.x * 8 + wave;
  if (t < a.ntiles) {
#pragma unroll
    for (int i = 0; i < NPF; ++i) glds_row(slot_ptr(t, i) + lane * 16, in_l + i * kWT);
  }
  for (; t < a.ntiles; t += nw) {
    const uint32_t bid = t / tpb;
    uint32_t x[128];
    uint32_t y[4][8];  // the stand-in parity rows
#pragma unroll
    for (int i = NPF; i < K; ++i) ld_row(slot_ptr(t, i) + lane * 16, &x[8 * i]);
#pragma unroll
    for (int k = 0; k < ND; ++k) ld_row(row_ptr(t, K + a.prow[k]) + lane * 16, y[k]);
    __builtin_amdgcn_s_waitcnt(waitcnt_vm(2 * (K - NPF + ND)));  // the prefetched slots (and everything before them)
#pragma unroll
    for (int i = 0; i < NPF; ++i) lds_row(in_l + i * kWT, lane, &x[8 * i]);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < K; ++i) transpose8(&x[8 * i]);
    if constexpr (cfsec::dev::kBsEc16p20l2Paired)  // the network header's paired basis
      for (int c = 0; c < K; c += 2)
        for (int j = 0; j < 8; ++j) x[8 * c + j] ^= x[8 * (c + 1) + j];
    // 1-3: syndromes and the missing data rows
    uint8_t* mrow[4];
    if constexpr (ND > 0) {
#pragma unroll
      for (int k = 0; k < ND; ++k) {
        transpose8(y[k]);
        uint32_t o[8];
        cfsec::dev::bs_row_ec16p20l2_rt(a.prow[k], x, o);  // the row over the present data only
#pragma unroll
        for (int w = 0; w < 8; ++w) y[k][w] ^= o[w];
        mrow[k] = row_ptr(t, a.slot[k]) + lane * 16;
      }
      solve<ND>(a, x, y, mrow, 0);
    }
    // ring: the first two compared rows
    uint32_t pend = a.pcmp;  // compared rows whose ring copy is not issued yet
    uint32_t q_issue = 0, q_read = 0;
    const auto issue_ring = [&]() {
      if (pend) {
        const int r = __builtin_ctz(pend);
        pend &= pend - 1;
        glds_row(row_ptr(t, K + r) + lane * 16, ring + (q_issue % kRing) * kWT);
        ++q_issue;
      }
    };
    issue_ring();
    issue_ring();
    __builtin_amdgcn_sched_barrier(0);
    // the next tile's prefetch
    const uint32_t tn = t + nw < a.ntiles ? t + nw : t;
#pragma unroll
    for (int i = 0; i < NPF; ++i) glds_row(slot_ptr(tn, i) + lane * 16, in_l + i * kWT);
    __builtin_amdgcn_sched_barrier(0);
    uint32_t diff = 0;
    cfsec::dev::bs_net_ec16p20l2(x, [&](int r, uint32_t (&o)[8]) {
      if (a.pstore >> r & 1) {
        transpose8(o);
        st_row(row_ptr(t, K + r) + lane * 16, o);
      } else if (a.pcmp >> r & 1) {
        if (q_issue - q_read > 1) __builtin_amdgcn_s_waitcnt(waitcnt_vm(2));  // this row's copy; the next may fly
        else __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
        uint32_t v[8];
        lds_row(ring + (q_read % kRing) * kWT, lane, v);
        __builtin_amdgcn_s_waitcnt(0xC07F);
        ++q_read;
        issue_ring();
        transpose8(v);
#pragma unroll
        for (int w = 0; w < 8; ++w) diff |= v[w] ^ o[w];
      }
    });
    if (diff) a.flags[bid] = 1u;
  }
}

// encode (the golden codeword): bs_probe's kernel on this layout
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void bs_encode(uint8_t* base) {
  const uint32_t stripe = blockIdx.y;
  const size_t off = ((size_t)blockIdx.x * 256 + threadIdx.x) * 32;
  uint8_t* row0 = base + (size_t)stripe * ROWS * S;
  uint32_t x[128];
#pragma unroll
  for (int c = 0; c < K; ++c) {
    const u32x4 p = ld16nt(row0 + c * S + off), q = ld16nt(row0 + c * S + off + 16);
    x[8 * c + 0] = p.x; x[8 * c + 1] = p.y; x[8 * c + 2] = p.z; x[8 * c + 3] = p.w;
    x[8 * c + 4] = q.x; x[8 * c + 5] = q.y; x[8 * c + 6] = q.z; x[8 * c + 7] = q.w;
    transpose8(&x[8 * c]);
  }
  if constexpr (cfsec::dev::kBsEc16p20l2Paired)
    for (int c = 0; c < K; c += 2)
      for (int j = 0; j < 8; ++j) x[8 * c + j] ^= x[8 * (c + 1) + j];
  cfsec::dev::bs_net_ec16p20l2(x, [&](int r, uint32_t (&o)[8]) {
    transpose8(o);
    uint8_t* p = row0 + (size_t)(K + r) * S + off;
    st16nt(p, u32x4{o[0], o[1], o[2], o[3]});
    st16nt(p + 16, u32x4{o[4], o[5], o[6], o[7]});
  });
}

__global__ void fill(uint32_t* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t v = (uint32_t)i * 2654435761u ^ seed;
    v ^= v >> 15; v *= 0x2c1b3c6du; v ^= v >> 12;
    p[i] = v;
  }
}

static uint8_t gmul(uint8_t a, uint8_t b) {
  uint8_t p = 0;
  while (b) {
    if (b & 1) p ^= a;
    a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1D : 0));
    b >>= 1;
  }
  return p;
}
static uint8_t ginv(uint8_t a) {
  for (int b = 1; b < 256; ++b)
    if (gmul(a, (uint8_t)b) == 1) return (uint8_t)b;
  return 0;
}
static void coef_tables(uint8_t c, u32x4& t01, uint32_t& t2) {  // gf_device.hpp coef_tables on the host
  uint32_t p[8];
  p[0] = c;
  for (int j = 1; j < 8; ++j) p[j] = gmul((uint8_t)p[j - 1], 2);
  uint32_t t0lo = 0, t0hi = 0, t1lo = 0, t1hi = 0, tt2 = 0;
  for (int e = 0; e < 8; ++e) {
    const uint32_t v0 = ((e & 1) ? p[0] : 0u) ^ ((e & 2) ? p[1] : 0u) ^ ((e & 4) ? p[2] : 0u);
    const uint32_t v1 = ((e & 1) ? p[3] : 0u) ^ ((e & 2) ? p[4] : 0u) ^ ((e & 4) ? p[5] : 0u);
    if (e < 4) {
      const uint32_t v2 = ((e & 1) ? p[6] : 0u) ^ ((e & 2) ? p[7] : 0u);
      t0lo |= v0 << (8 * e); t1lo |= v1 << (8 * e); tt2 |= v2 << (8 * e);
    } else {
      t0hi |= v0 << (8 * (e - 4)); t1hi |= v1 << (8 * (e - 4));
    }
  }
  t01 = u32x4{t0lo, t0hi, t1lo, t1hi};
  t2 = tt2;
}

int main() {
  const size_t bytes = (size_t)NB * ROWS * S;
  std::vector<uint8_t*> bufs(NT);
  std::vector<uint8_t*> gold(NT);
  const int bad[4] = {0, 1, K + 0, K + 1};
  for (int t = 0; t < NT; ++t) {
    CK(hipMalloc(&bufs[t], bytes));
    CK(hipMalloc(&gold[t], (size_t)NB * 4 * S));
    fill<<<4096, 256>>>((uint32_t*)bufs[t], bytes / 4, 0x9E3779B9u * (t + 1));
    hipLaunchKernelGGL(bs_encode, dim3((unsigned)(S / 8192), NB), dim3(256), 0, 0, bufs[t]);
    for (int b = 0; b < NB; ++b)
      for (int i = 0; i < 4; ++i)
        CK(hipMemcpy(gold[t] + ((size_t)b * 4 + i) * S, bufs[t] + ((size_t)b * ROWS + bad[i]) * S, S, hipMemcpyDeviceToDevice));
  }
  uint32_t* flags;
  CK(hipMalloc(&flags, NB * 4));
  uint8_t* zero;
  CK(hipMalloc(&zero, kWT));
  CK(hipMemset(zero, 0, kWT));
  CK(hipDeviceSynchronize());
  // the plan of {0,1,16,17}: missing data 0, 1 in slots 0, 1; stand-ins: parity rows 2, 3 (the first
  // two present); rebuilt parities 0, 1; compared: every other parity row
  RepairArgs ra{};
  ra.flags = flags;
  ra.zero = zero;
  ra.ntiles = (uint32_t)(NB * (S / kWT));
  ra.nd = 2;
  ra.slot[0] = 0; ra.slot[1] = 1;
  ra.prow[0] = 2; ra.prow[1] = 3;
  ra.pstore = 0x3u;
  ra.pcmp = ((1u << NP) - 1) & ~0xFu;
  const uint8_t (*M)[16] = cfsec::dev::kBsEc16p20l2Rows;
  // A = M[p_k][slot_j] (k rows, j columns); A^-1 by 2x2 formula
  const uint8_t a00 = M[2][0], a01 = M[2][1], a10 = M[3][0], a11 = M[3][1];
  const uint8_t det = gmul(a00, a11) ^ gmul(a01, a10), id = ginv(det);
  const uint8_t inv[2][2] = {{gmul(a11, id), gmul(a01, id)}, {gmul(a10, id), gmul(a00, id)}};  // d = inv * s
  for (int j = 0; j < 2; ++j)
    for (int k = 0; k < 2; ++k) coef_tables(inv[j][k], ra.t01[j * 4 + k], ra.t2[j * 4 + k]);
  int dev = 0, ncu = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const auto zero_bad = [&](int t) {
    for (int b = 0; b < NB; ++b)
      for (int i = 0; i < 4; ++i) CK(hipMemset(bufs[t] + ((size_t)b * ROWS + bad[i]) * S, 0, S));
  };
  const auto check = [&](int t) {
    std::vector<uint8_t> h(S), g(S);
    long nbad = 0;
    for (int b = 0; b < NB; ++b)
      for (int i = 0; i < 4; ++i) {
        CK(hipMemcpy(h.data(), bufs[t] + ((size_t)b * ROWS + bad[i]) * S, S, hipMemcpyDeviceToHost));
        CK(hipMemcpy(g.data(), gold[t] + ((size_t)b * 4 + i) * S, S, hipMemcpyDeviceToHost));
        if (memcmp(h.data(), g.data(), S) && nbad++ < 4) printf("bid %d row %d differs\n", b, bad[i]);
      }
    return nbad;
  };
  long nbad = 0;
  for (int t = 0; t < NT; ++t) {
    zero_bad(t);
    CK(hipMemset(flags, 0, NB * 4));
    ra.base = bufs[t];
    hipLaunchKernelGGL(bs_repair<2>, dim3(ncu), dim3(512), 0, 0, ra);
    CK(hipDeviceSynchronize());
    nbad += check(t);
    std::vector<uint32_t> fl(NB);
    CK(hipMemcpy(fl.data(), flags, NB * 4, hipMemcpyDeviceToHost));
    for (int b = 0; b < NB; ++b)
      if (fl[b]) { printf("tasklet %d bid %d: Verify flag set on a codeword\n", t, b); ++nbad; }
  }
  // Verify must fail where a survivor is corrupted: a compared parity (bid 5, parity 9) and a
  // present data row (bid 9, row 7), then everything restored
  {
    uint8_t* p1 = bufs[0] + ((size_t)5 * ROWS + K + 9) * S + 12345;
    uint8_t* p2 = bufs[0] + ((size_t)9 * ROWS + 7) * S + 200001;
    uint8_t o1, o2, v;
    CK(hipMemcpy(&o1, p1, 1, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&o2, p2, 1, hipMemcpyDeviceToHost));
    v = o1 ^ 0x40; CK(hipMemcpy(p1, &v, 1, hipMemcpyHostToDevice));
    v = o2 ^ 0x01; CK(hipMemcpy(p2, &v, 1, hipMemcpyHostToDevice));
    CK(hipMemset(flags, 0, NB * 4));
    ra.base = bufs[0];
    hipLaunchKernelGGL(bs_repair<2>, dim3(ncu), dim3(512), 0, 0, ra);
    CK(hipDeviceSynchronize());
    std::vector<uint32_t> fl(NB);
    CK(hipMemcpy(fl.data(), flags, NB * 4, hipMemcpyDeviceToHost));
    for (int b = 0; b < NB; ++b)
      if ((fl[b] != 0) != (b == 5 || b == 9)) { printf("corruption test: bid %d flag %u\n", b, fl[b]); ++nbad; }
    CK(hipMemcpy(p1, &o1, 1, hipMemcpyHostToDevice));
    CK(hipMemcpy(p2, &o2, 1, hipMemcpyHostToDevice));
  }
  printf("repair check: %s\n", nbad ? "FAIL" : "ok (rows {0,1,16,17} of every bid == golden, Verify flags as expected)");
  if (nbad) return 1;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double algo = (double)NB * 38 * S;
  for (int i = 0; i < 300; ++i) { ra.base = bufs[i % NT]; hipLaunchKernelGGL(bs_repair<2>, dim3(ncu), dim3(512), 0, 0, ra); }
  for (int rep = 0; rep < 8; ++rep) {
    for (int i = 0; i < 6; ++i) { ra.base = bufs[i % NT]; hipLaunchKernelGGL(bs_repair<2>, dim3(ncu), dim3(512), 0, 0, ra); }
    CK(hipEventRecord(e0, 0));
    const int n = 30;
    for (int i = 0; i < n; ++i) { ra.base = bufs[i % NT]; hipLaunchKernelGGL(bs_repair<2>, dim3(ncu), dim3(512), 0, 0, ra); }
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / n;
    printf("bs_repair C5 (64 bids, {0,1,16,17}, Reconstruct + Verify): %8.1f us  %5.1f %% of 8 TB/s (38 rows per bid)\n", us,
           algo / us / 8e4);
  }
  return 0;
}
