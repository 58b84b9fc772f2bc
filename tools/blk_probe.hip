// blk_probe.hip -- where the crc32block framing kernel's time goes (dev tool): the shipped kernel
// against its CRC-only and copy-only variants and the standalone shard CRC, on blobnode's write
// batch (16 shards x 8 EC12P4 stripes of S = 5,592,406 bytes, 64 KiB blocks).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../chubaofs_amd/csrc blk_probe.hip \
//         -L../chubaofs_amd -lcfsec -Wl,-rpath,'$ORIGIN/../chubaofs_amd' -o blk_probe
#include <algorithm>
#include <cstdio>
#include <functional>
#include <string>
#include <vector>

#include "../chubaofs_amd/csrc/crc32block.hip"

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

__global__ void fill(uint32_t* p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    p[i] = (uint32_t)(z ^ (z >> 31));
  }
}

// flat copy of n16 16-byte chunks with the source / destination offset by SOFF / DOFF bytes
template <int SOFF, int DOFF>
__global__ __launch_bounds__(256) void kcopy(const uint8_t* s, uint8_t* d, size_t n16) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256)
    cfsec::dev::st16<true>(d + DOFF + 16 * i, cfsec::dev::ld16<true>(s + SOFF + 16 * i));
}

int main(int argc, char** argv) {
  const int64_t S = argc > 1 ? atoll(argv[1]) : 5592406;
  const int n = argc > 2 ? atoi(argv[2]) : 128;
  const int64_t L = argc > 3 ? atoll(argv[3]) : 65536, flen = S + 4 * ((S + L - 5) / (L - 4));
  const int64_t pitch = (S + 255) / 256 * 256, fpitch = (flen + 255) / 256 * 256;
  // three buffer sets used in rotation: no launch finds its data in the 256 MB Infinity Cache
  constexpr int NB = 3;
  uint8_t *pays[NB], *frms[NB], *seams[NB];
  const int64_t spitch = (S + L - 5) / (L - 4) * L;  // the no-seams probe: destination blocks L apart
  uint32_t* words;
  CK(hipMalloc(&words, 4 * 4096));
  std::vector<std::vector<const uint8_t*>> ins(NB, std::vector<const uint8_t*>(n)), fins(NB, std::vector<const uint8_t*>(n));
  std::vector<std::vector<uint8_t*>> outs(NB, std::vector<uint8_t*>(n)), fouts(NB, std::vector<uint8_t*>(n)),
      souts(NB, std::vector<uint8_t*>(n));
  for (int b = 0; b < NB; ++b) {
    CK(hipMalloc(&pays[b], pitch * n));
    CK(hipMalloc(&frms[b], fpitch * n));
    CK(hipMalloc(&seams[b], spitch * n));
    fill<<<2048, 256>>>((uint32_t*)pays[b], pitch * n / 4);
    for (int i = 0; i < n; ++i) {
      ins[b][i] = pays[b] + i * pitch, outs[b][i] = frms[b] + i * fpitch;
      fins[b][i] = frms[b] + i * fpitch, fouts[b][i] = pays[b] + i * pitch;
      souts[b][i] = seams[b] + i * spitch;
    }
  }
  uint8_t* pay = pays[0];
  uint8_t* frm = frms[0];
  int rot = 0;
  cfsec::Crc32BlockJob j;
  j.n = n;
  j.in = ins[0].data();
  j.out = outs[0].data();
  j.size = S;
  j.block_len = L;
  j.whole = words;
  const auto J = [&](bool enc) {
    cfsec::Crc32BlockJob k = j;
    const int b = rot++ % NB;
    k.encode = enc;
    k.in = enc ? ins[b].data() : fins[b].data();
    k.out = enc ? outs[b].data() : fouts[b].data();
    k.whole = enc ? words : nullptr;
    k.bad = enc ? nullptr : words;
    k.from = 0;
    k.to = S;
    return k;
  };
  const auto Jseam = [&]() {  // decode into destination blocks L apart (launch<..., SEAMLESS_PROBE>)
    cfsec::Crc32BlockJob k = J(false);
    k.out = souts[(rot - 1) % NB].data();
    return k;
  };
  struct V {
    std::string name;
    std::function<void()> f;
    double bytes;
  };
  const double pb = double(S) * n;
  std::vector<V> vs = {
      {"enc old epilogue", [&] { CK((cfsec::blk::launch<true, true, true, false, true, true, 4, false>(J(true), 0))); }, 2 * pb},
      {"enc new epi R4", [&] { CK((cfsec::blk::launch<true, true, true, false, true, true, 4, true>(J(true), 0))); }, 2 * pb},
      {"enc new epi R6", [&] { CK((cfsec::blk::launch<true, true, true, false, true, true, 6, true>(J(true), 0))); }, 2 * pb},
      {"enc new epi R8", [&] { CK((cfsec::blk::launch<true, true, true, false, true, true, 8, true>(J(true), 0))); }, 2 * pb},
      {"enc stride R4", [&] { CK((cfsec::blk::launch<true, true, true, false, true, true, 4, true, true>(J(true), 0))); }, 2 * pb},
      {"enc stride R6", [&] { CK((cfsec::blk::launch<true, true, true, false, true, true, 6, true, true>(J(true), 0))); }, 2 * pb},
      {"enc stride R8", [&] { CK((cfsec::blk::launch<true, true, true, false, true, true, 8, true, true>(J(true), 0))); }, 2 * pb},
      {"enc new epi R2", [&] { CK((cfsec::blk::launch<true, true, true, false, true, true, 2, true>(J(true), 0))); }, 2 * pb},
      {"dec stride R4", [&] { CK((cfsec::blk::launch<true, true, true, false, true, true, 4, true, true>(J(false), 0))); }, 2 * pb},
      {"dec stride R8", [&] { CK((cfsec::blk::launch<true, true, true, false, true, true, 8, true, true>(J(false), 0))); }, 2 * pb},
      {"dec stride R8 no seams", [&] { CK((cfsec::blk::launch<true, true, true, false, true, true, 8, true, true, true>(Jseam(), 0))); }, 2 * pb},
      {"dec old epilogue", [&] { CK((cfsec::blk::launch<true, true, true, false, true, true, 4, false>(J(false), 0))); }, 2 * pb},
      {"dec new epi R4", [&] { CK((cfsec::blk::launch<true, true, true, false, true, true, 4, true>(J(false), 0))); }, 2 * pb},
      {"dec new epi R8", [&] { CK((cfsec::blk::launch<true, true, true, false, true, true, 8, true>(J(false), 0))); }, 2 * pb},
      {"shipped enc", [&] { CK(cfsec::launch_crc32block(J(true), 0)); }, 2 * pb},
      {"shipped dec", [&] { CK(cfsec::launch_crc32block(J(false), 0)); }, 2 * pb},
      {"crc only (no store)", [&] { CK((cfsec::blk::launch<false, true>(j, 0))); }, pb},
      {"copy only (no crc)", [&] { CK((cfsec::blk::launch<true, false>(j, 0))); }, 2 * pb},
      {"copy, src-aligned", [&] { CK((cfsec::blk::launch<true, false, true, true>(j, 0))); }, 2 * pb},
      {"copy, no epilogue", [&] { CK((cfsec::blk::launch<true, false, false>(j, 0))); }, 2 * pb},
      {"copy, runs of blocks", [&] { CK((cfsec::blk::launch<true, false, true, false, false>(j, 0))); }, 2 * pb},
      {"crc, no epilogue", [&] { CK((cfsec::blk::launch<false, true, false>(j, 0))); }, pb},
      {"crc+store, runs", [&] { CK((cfsec::blk::launch<true, true, true, false, false>(j, 0))); }, 2 * pb},
      {"copy, no epi, plain st", [&] { CK((cfsec::blk::launch<true, false, false, false, true, false>(j, 0))); }, 2 * pb},
      {"copy, no epi, runs, pl", [&] { CK((cfsec::blk::launch<true, false, false, false, false, false>(j, 0))); }, 2 * pb},
      {"crc+st, plain st", [&] { CK((cfsec::blk::launch<true, true, true, false, true, false>(j, 0))); }, 2 * pb},
      {"crc+st, no epi, plain", [&] { CK((cfsec::blk::launch<true, true, false, false, true, false>(j, 0))); }, 2 * pb},
      {"shipped, no shard crc", [&] { cfsec::Crc32BlockJob j2 = j; j2.whole = nullptr; CK((cfsec::blk::launch<true, true>(j2, 0))); }, 2 * pb},
      {"flat copy aligned", [&] { kcopy<0, 0><<<4096, 256>>>(pay, frm, (size_t)(pb / 16) - 1); }, 2 * pb},
      {"flat copy src+4", [&] { kcopy<4, 0><<<4096, 256>>>(pay, frm, (size_t)(pb / 16) - 1); }, 2 * pb},
      {"flat copy dst+4", [&] { kcopy<0, 4><<<4096, 256>>>(pay, frm, (size_t)(pb / 16) - 1); }, 2 * pb},
      {"flat copy both+4", [&] { kcopy<4, 4><<<4096, 256>>>(pay, frm, (size_t)(pb / 16) - 1); }, 2 * pb},
      {"standalone shard crc", [&] { CK(cfsec::launch_crc32(ins[0].data(), S, n, words, 0)); }, pb},
  };
  {  // the grid-stride kernel frames exactly like the old per-block kernel
    std::vector<uint8_t> want((size_t)fpitch * n), got((size_t)fpitch * n);
    std::vector<uint32_t> w1(n), w2(n);
    cfsec::Crc32BlockJob k = j;
    k.encode = true;
    CK(hipMemset(frm, 0, fpitch * n));
    CK(hipMemset(words, 0, 4 * n));
    CK((cfsec::blk::launch<true, true, true, false, true, true, 4, false>(k, 0)));
    CK(hipMemcpy(want.data(), frm, want.size(), hipMemcpyDeviceToHost));
    CK(hipMemcpy(w1.data(), words, 4 * n, hipMemcpyDeviceToHost));
    CK(hipMemset(frm, 0, fpitch * n));
    CK(hipMemset(words, 0, 4 * n));
    CK((cfsec::blk::launch<true, true, true, false, true, true, 4, true, true>(k, 0)));
    CK(hipMemcpy(got.data(), frm, got.size(), hipMemcpyDeviceToHost));
    CK(hipMemcpy(w2.data(), words, 4 * n, hipMemcpyDeviceToHost));
    printf("stride kernel == old kernel: framed %s, whole-shard crc %s\n", want == got ? "yes" : "NO",
           w1 == w2 ? "yes" : "NO");
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 100; ++i) vs[0].f();
  std::vector<std::vector<float>> t(vs.size());
  for (int r = 0; r < 15; ++r)
    for (size_t v = 0; v < vs.size(); ++v) {
      vs[v].f();
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < 10; ++i) vs[v].f();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[v].push_back(ms / 10);
    }
  printf("S=%lld shards=%d block=%lld  payload %.1f MB\n", (long long)S, n, (long long)L, pb / 1e6);
  for (size_t v = 0; v < vs.size(); ++v) {
    std::sort(t[v].begin(), t[v].end());
    const double ms = t[v][t[v].size() / 2];
    printf("%-24s median %8.1f us  payload %7.1f GB/s  HBM %6.1f%% of 8 TB/s\n", vs[v].name.c_str(), ms * 1e3,
           pb / (ms * 1e-3) / 1e9, 100 * vs[v].bytes / (ms * 1e-3) / 8e12);
  }
  return 0;
}
