/*
 * cpu_simd.c -- BENCH INFRASTRUCTURE: the CPU baseline bench.py times beside the GPU.
 *
 * The reference library (Go + Go assembler) cannot run here or on the GPU box (no Go
 * toolchain), so this is a C restatement of the strategy klauspost/reedsolomon v1.11.7
 * uses on amd64 -- labelled "port" in bench.py's cpu_baseline, never the product:
 *   - AVX2 split-nibble tiles (VPSHUFB on low/high nibble tables, VPXOR accumulate),
 *     <= 10 inputs x <= 10 outputs per tile, first tile stores and later tiles XOR
 *     (KRS/galois_gen_amd64.s mulAvxTwo_RxC[Xor], planned by codeSomeShardsAVXP,
 *     KRS/reedsolomon.go:985-1134; tile matrix layout genAvx2Matrix, KRS/galois.go:908-935)
 *   - AVX-512 GFNI tiles (VGF2P8AFFINEQB with the 8x8 bit matrices of
 *     KRS/galois.go:937), used when inputs and outputs are both <= 10
 *     (canGFNI, KRS/reedsolomon.go:792-796; galMulSlicesGFNI)
 *   - the byte range split into 64-B aligned pieces over at most `threads` workers,
 *     each walking perRound sub-chunks (KRS/reedsolomon.go:968-980, 1072-1133);
 *     reference caps: 4 workers with GFNI, 8 with AVX2 (:551-557)
 *   - tails below 32/64 bytes through the scalar mulTable (galMulSlice[Xor]).
 * Results are checked against the scalar oracle by tests/test_oracle.py.
 */
#include <immintrin.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

void oracle_tables(uint8_t* log_t, uint8_t* exp_t, uint8_t* inv_t, uint8_t* mul_t, uint8_t* mul_lo,
                   uint8_t* mul_hi, uint64_t* gfni);

static uint8_t MUL[256][256], MLO[256][16], MHI[256][16];
static uint64_t GFNI_M[256];
static int g_ready = 0;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;
static void init_once(void) {
  oracle_tables(NULL, NULL, NULL, &MUL[0][0], &MLO[0][0], &MHI[0][0], GFNI_M);
  g_ready = 1;
}

int cpu_has_gfni(void) {
  __builtin_cpu_init();
  return __builtin_cpu_supports("gfni") && __builtin_cpu_supports("avx512bw") &&
         __builtin_cpu_supports("avx512f");
}
int cpu_has_avx2(void) {
  __builtin_cpu_init();
  return __builtin_cpu_supports("avx2");
}

#define MAXT 10

/* ---------------- AVX2 tile: out[r] (^)= sum_c M[r][c] * in[c] over [start, stop) --------------- */
__attribute__((target("avx2"))) static size_t tile_avx2(const uint8_t* mat /* nin*nout*64 */, int nin,
                                                        int nout, uint8_t* const* in, uint8_t* const* out,
                                                        size_t start, size_t stop, int xor_out) {
  const __m256i mask = _mm256_set1_epi8(0x0f);
  size_t off = start;
  for (; off + 32 <= stop; off += 32) {
    __m256i acc[MAXT];
    for (int r = 0; r < nout; r++)
      acc[r] = xor_out ? _mm256_loadu_si256((const __m256i*)(out[r] + off)) : _mm256_setzero_si256();
    for (int c = 0; c < nin; c++) {
      const __m256i x = _mm256_loadu_si256((const __m256i*)(in[c] + off));
      const __m256i lo = _mm256_and_si256(x, mask);
      const __m256i hi = _mm256_and_si256(_mm256_srli_epi64(x, 4), mask);
      const uint8_t* t = mat + (size_t)(c * nout) * 64;
      for (int r = 0; r < nout; r++, t += 64) {
        const __m256i L = _mm256_load_si256((const __m256i*)t);
        const __m256i H = _mm256_load_si256((const __m256i*)(t + 32));
        acc[r] = _mm256_xor_si256(acc[r], _mm256_xor_si256(_mm256_shuffle_epi8(L, lo), _mm256_shuffle_epi8(H, hi)));
      }
    }
    for (int r = 0; r < nout; r++) _mm256_storeu_si256((__m256i*)(out[r] + off), acc[r]);
  }
  return off;
}

/* ---------------- GFNI tile (64 B per step) ---------------- */
__attribute__((target("avx512f,avx512bw,gfni"))) static size_t tile_gfni(const uint64_t* mat /* nin*nout */,
                                                                         int nin, int nout, uint8_t* const* in,
                                                                         uint8_t* const* out, size_t start,
                                                                         size_t stop, int xor_out) {
  size_t off = start;
  for (; off + 64 <= stop; off += 64) {
    __m512i acc[MAXT];
    for (int r = 0; r < nout; r++)
      acc[r] = xor_out ? _mm512_loadu_si512((const void*)(out[r] + off)) : _mm512_setzero_si512();
    for (int c = 0; c < nin; c++) {
      const __m512i x = _mm512_loadu_si512((const void*)(in[c] + off));
      for (int r = 0; r < nout; r++)
        acc[r] = _mm512_xor_si512(acc[r], _mm512_gf2p8affine_epi64_epi8(x, _mm512_set1_epi64((long long)mat[c * nout + r]), 0));
    }
    for (int r = 0; r < nout; r++) _mm512_storeu_si512((void*)(out[r] + off), acc[r]);
  }
  return off;
}

static void scalar_rows(const uint8_t* rows, int k, int nout, uint8_t* const* in, uint8_t* const* out,
                        size_t start, size_t stop) {
  for (int r = 0; r < nout; r++)
    for (int c = 0; c < k; c++) {
      const uint8_t* mt = MUL[rows[r * k + c]];
      if (c == 0) for (size_t i = start; i < stop; i++) out[r][i] = mt[in[c][i]];
      else for (size_t i = start; i < stop; i++) out[r][i] ^= mt[in[c][i]];
    }
}

typedef struct {
  int in0, nin, out0, nout, first;
  uint8_t* avx2;   /* nin*nout*64, 32-B aligned */
  uint64_t gfni[MAXT * MAXT];
} tile_plan;

typedef struct {
  const uint8_t* rows;
  int k, m;
  uint8_t* const* in;
  uint8_t* const* out;
  tile_plan* plan;
  int nplan;
  int use_gfni;
  size_t per_round;
  size_t start, stop;
} job;

static void run_range(const job* j) {
  for (size_t ls = j->start; ls < j->stop;) {
    size_t le = ls + j->per_round;
    if (le > j->stop) le = j->stop;
    size_t done = ls;
    for (int p = 0; p < j->nplan; p++) {
      const tile_plan* t = &j->plan[p];
      size_t e = j->use_gfni ? tile_gfni(t->gfni, t->nin, t->nout, j->in + t->in0, j->out + t->out0, ls, le, !t->first)
                             : tile_avx2(t->avx2, t->nin, t->nout, j->in + t->in0, j->out + t->out0, ls, le, !t->first);
      done = e;
    }
    if (done < le) scalar_rows(j->rows, j->k, j->m, j->in, j->out, done, le);
    ls = le;
  }
}

static void* worker(void* p) {
  run_range((const job*)p);
  return NULL;
}

/*
 * outputs[r] = XOR_c rows[r*k + c] * inputs[c] over len bytes, klauspost-style.
 * threads: worker count (the reference uses <= 4 with GFNI, <= 8 with AVX2).
 * force: 0 = reference selection, 1 = AVX2 tiles, 2 = GFNI tiles (<=10x10 only).
 */
int cpu_code_some_shards(const uint8_t* rows, int k, int m, uint8_t* const* in, uint8_t* const* out,
                         size_t len, int threads, int force) {
  pthread_once(&g_once, init_once);
  if (k <= 0 || m <= 0 || len == 0) return 0;
  int use_gfni = cpu_has_gfni() && k <= MAXT && m <= MAXT;
  if (force == 1) use_gfni = 0;
  if (force == 2) {
    if (!(cpu_has_gfni() && k <= MAXT && m <= MAXT)) return -1;
    use_gfni = 1;
  }
  if (!use_gfni && !cpu_has_avx2()) return -1;
  /* plan: tiles of <= 10 inputs x <= 10 outputs, inner loop over the smaller side */
  tile_plan plan[64];
  int np = 0;
  for (int o0 = 0; o0 < m; o0 += MAXT)
    for (int i0 = 0; i0 < k; i0 += MAXT) {
      tile_plan* t = &plan[np++];
      t->in0 = i0;
      t->nin = k - i0 < MAXT ? k - i0 : MAXT;
      t->out0 = o0;
      t->nout = m - o0 < MAXT ? m - o0 : MAXT;
      t->first = i0 == 0;
      t->avx2 = (uint8_t*)aligned_alloc(64, (size_t)t->nin * t->nout * 64);
      for (int r = 0; r < t->nout; r++)
        for (int c = 0; c < t->nin; c++) {
          const uint8_t coef = rows[(o0 + r) * k + i0 + c];
          uint8_t* d = t->avx2 + (size_t)(c * t->nout + r) * 64;
          memcpy(d, MLO[coef], 16);
          memcpy(d + 16, MLO[coef], 16);
          memcpy(d + 32, MHI[coef], 16);
          memcpy(d + 48, MHI[coef], 16);
          t->gfni[c * t->nout + r] = GFNI_M[coef];
        }
    }
  /* perRound: L1D (48 KiB assumed) / (inputs + outputs of a tile), 64-B aligned */
  size_t div = (size_t)((k < MAXT ? k : MAXT) + (m < MAXT ? m : MAXT));
  size_t per_round = ((48 * 1024 / div) + 63) & ~(size_t)63;
  if (threads < 1) threads = 1;
  size_t chunk = (len + threads - 1) / threads;
  chunk = (chunk + 63) & ~(size_t)63;
  job jobs[256];
  pthread_t tids[256];
  int nj = 0;
  for (size_t s = 0; s < len && nj < 256; s += chunk) {
    job* j = &jobs[nj++];
    j->rows = rows; j->k = k; j->m = m; j->in = in; j->out = out;
    j->plan = plan; j->nplan = np; j->use_gfni = use_gfni; j->per_round = per_round;
    j->start = s;
    j->stop = s + chunk < len ? s + chunk : len;
  }
  for (int i = 1; i < nj; i++) pthread_create(&tids[i], NULL, worker, &jobs[i]);
  run_range(&jobs[0]);
  for (int i = 1; i < nj; i++) pthread_join(tids[i], NULL);
  for (int p = 0; p < np; p++) free(plan[p].avx2);
  return use_gfni ? 2 : 1;
}
