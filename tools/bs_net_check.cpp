// bs_net_check.cpp -- host check of a generated bit-sliced network header (dev tool, round 4):
// random bytes for the 16 data rows of one lane, the planes built by the same 8x8 bit transpose
// the kernels use (paired basis when the header says so), every row of the network emitted and
// transposed back, compared byte by byte with the GF(2^8)/0x11D matrix product.
//   g++ -O1 -std=c++17 -I../chubaofs_amd/csrc -DBS_NET_HDR='"bs_net_ec16p20l2.hpp"' bs_net_check.cpp -o /tmp/bs_net_check
// (another network: -DBS_NET_CAP=Ec6p10l2 -DBS_NET_LOW=ec6p10l2 with its header)
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define __device__
#define __forceinline__ inline
#define CFSEC_BS_X3
#define __builtin_amdgcn_sched_barrier(x) ((void)0)
namespace cfsec { namespace dev { inline uint32_t bs_x3(uint32_t a, uint32_t b, uint32_t c) { return a ^ b ^ c; } } }
#include BS_NET_HDR
#ifndef BS_NET_CAP
#define BS_NET_CAP Ec16p20l2
#define BS_NET_LOW ec16p20l2
#endif
#define BS_CAT3(a, b, c) a##b##c
#define BS_PASTE3(a, b, c) BS_CAT3(a, b, c)
#define BS_NET_TYPE BS_PASTE3(Bs, BS_NET_CAP, )
#define BS_NET_ROWS BS_PASTE3(kBs, BS_NET_CAP, Rows)
#define BS_NET_FN BS_PASTE3(bs_net_, BS_NET_LOW, )
#define BS_NET_ROW_RT BS_PASTE3(bs_row_, BS_NET_LOW, _rt)

static void swapmove(uint32_t& a, uint32_t& b, int s, uint32_t m) {
  const uint32_t t = ((a >> s) ^ b) & m;
  b ^= t;
  a ^= t << s;
}
static void transpose8(uint32_t* w) {
  for (int i = 0; i < 8; i += 2) swapmove(w[i], w[i + 1], 1, 0x55555555u);
  for (int i = 0; i < 8; ++i)
    if (!(i & 2)) swapmove(w[i], w[i + 2], 2, 0x33333333u);
  for (int i = 0; i < 4; ++i) swapmove(w[i], w[i + 4], 4, 0x0F0F0F0Fu);
}
static uint8_t gmul(uint8_t a, uint8_t b) {
  uint8_t p = 0;
  for (int i = 0; i < 8; ++i) {
    if (b & 1) p ^= a;
    b >>= 1;
    a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1D : 0));
  }
  return p;
}

int main() {
  using namespace cfsec::dev;
  constexpr int K = BS_NET_TYPE::K, M = BS_NET_TYPE::M;
  srand(12345);
  long bad = 0;
  for (int trial = 0; trial < 200; ++trial) {
    uint8_t in[K][32];
    for (int c = 0; c < K; ++c)
      for (int b = 0; b < 32; ++b) in[c][b] = (uint8_t)rand();
    uint32_t x[8 * K];
    for (int c = 0; c < K; ++c) {
      for (int w = 0; w < 8; ++w)
        x[8 * c + w] = in[c][4 * w] | in[c][4 * w + 1] << 8 | in[c][4 * w + 2] << 16 | (uint32_t)in[c][4 * w + 3] << 24;
      transpose8(&x[8 * c]);
    }
    if (BS_NET_TYPE::Paired)
      for (int c = 0; c < K; c += 2)
        for (int j = 0; j < 8; ++j) x[8 * c + j] ^= x[8 * (c + 1) + j];
    int seen = 0;
    BS_NET_FN<M>(x, [&](int r, uint32_t (&o)[8]) {
      ++seen;
      uint32_t v[8];
      for (int w = 0; w < 8; ++w) v[w] = o[w];
      transpose8(v);
      for (int b = 0; b < 32; ++b) {
        uint8_t want = 0;
        for (int c = 0; c < K; ++c) want ^= gmul(BS_NET_ROWS[r][c], in[c][b]);
        const uint8_t got = (uint8_t)(v[b / 4] >> (8 * (b % 4)));
        bad += got != want;
      }
    });
    // the run-time single rows too
    for (int r = 0; r < M; ++r) {
      uint32_t o[8];
      BS_NET_ROW_RT(r, x, o);
      transpose8(o);
      for (int b = 0; b < 32; ++b) {
        uint8_t want = 0;
        for (int c = 0; c < K; ++c) want ^= gmul(BS_NET_ROWS[r][c], in[c][b]);
        bad += (uint8_t)(o[b / 4] >> (8 * (b % 4))) != want;
      }
    }
    if (seen != M) { printf("emitted %d rows of %d\n", seen, M); return 1; }
  }
  printf("%s: %s (%ld bad bytes)\n", BS_NET_HDR, bad ? "FAIL" : "ok", bad);
  return bad != 0;
}
