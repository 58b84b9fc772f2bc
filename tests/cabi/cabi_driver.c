/*
 * cabi_driver.c -- a plain C caller of libcfsec.so, doing what the cgo shim (go/cfsec) does:
 * cfsec_shard vectors over host memory (pageable Go-heap-like buffers and cfsec_host_alloc pinned
 * ones), reedsolomon.Encoder calls, ec.Encoder calls for an LRC mode, the blobnode repair batch,
 * crc32block framing, and the error codes the shim maps back to Go sentinels.
 *
 * It never loads PyTorch, so the library runs on /opt/rocm's HIP runtime -- the runtime a Go/C
 * process gets (every Python GPU test imports torch first and runs on torch's bundled runtime).
 * tests/test_gpu_cabi.py runs it in a subprocess and checks every record it writes against the
 * oracle.  Test infrastructure: built by __graft_entry__.build(), never shipped.
 *
 * usage: cabi_driver <out file>
 * out: records {char name[16]; uint64 len; bytes[len]}.
 */
#define _GNU_SOURCE
#include <link.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/cfsec.h"

static FILE* out;

static void rec(const char* name, const void* p, uint64_t n) {
  char nm[16] = {0};
  strncpy(nm, name, 15);
  fwrite(nm, 1, 16, out);
  fwrite(&n, 8, 1, out);
  if (n) fwrite(p, 1, n, out);
}

static void rec_int(const char* name, int v) { rec(name, &v, 4); }

static uint64_t sm_state;
static uint8_t sm_byte(void) { /* splitmix64 */
  uint64_t z = (sm_state += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return (uint8_t)((z ^ (z >> 31)) & 0xFF);
}

#define CHECK(x)                                                                  \
  do {                                                                            \
    int st_ = (x);                                                                \
    if (st_ != CFSEC_OK) {                                                        \
      fprintf(stderr, "%s:%d %s -> %s (%s)\n", __FILE__, __LINE__, #x,           \
              cfsec_status_name(st_), cfsec_last_error());                        \
      exit(2);                                                                    \
    }                                                                             \
  } while (0)

/* The HIP runtime this process mapped (evidence of which runtime served the calls). */
static char hip_path[512];
static int find_hip(struct dl_phdr_info* info, size_t size, void* data) {
  (void)size;
  (void)data;
  if (info->dlpi_name && strstr(info->dlpi_name, "libamdhip64")) {
    strncpy(hip_path, info->dlpi_name, sizeof hip_path - 1);
    return 1;
  }
  return 0;
}

int main(int argc, char** argv) {
  if (argc != 2) return 1;
  out = fopen(argv[1], "wb");
  if (!out) return 1;
  rec("version", cfsec_version(), strlen(cfsec_version()));
  rec_int("devices", cfsec_device_count());

  /* ---- reedsolomon.Encoder, EC12P4, pageable host memory ---- */
  enum { K = 12, M = 4, T = 16 };
  const size_t S = 100003;
  cfsec_rs* rs = NULL;
  CHECK(cfsec_rs_new(K, M, -1, &rs));
  uint8_t* page = malloc(T * S);
  sm_state = 0xCF5EC000u;
  for (size_t i = 0; i < K * S; ++i) page[i] = sm_byte();
  memset(page + K * S, 0, M * S);
  cfsec_shard sh[T];
  for (int i = 0; i < T; ++i) sh[i] = (cfsec_shard){page + i * S, S, S};
  CHECK(cfsec_rs_encode(rs, sh, T, CFSEC_MEM_HOST, NULL));
  rec("enc_page", page, T * S);
  int ok = 0;
  CHECK(cfsec_rs_verify(rs, sh, T, CFSEC_MEM_HOST, NULL, &ok));
  rec_int("verify_ok", ok);
  page[K * S + 7] ^= 1;
  CHECK(cfsec_rs_verify(rs, sh, T, CFSEC_MEM_HOST, NULL, &ok));
  rec_int("verify_bad", ok);
  page[K * S + 7] ^= 1;

  /* ---- the same on pinned memory (the resourcepool.NewMemPoolWith hook) ---- */
  uint8_t* pin = NULL;
  CHECK(cfsec_host_alloc(T * S, (void**)&pin));
  memcpy(pin, page, K * S);
  memset(pin + K * S, 0xEE, M * S);
  for (int i = 0; i < T; ++i) sh[i] = (cfsec_shard){pin + i * S, S, S};
  CHECK(cfsec_rs_encode(rs, sh, T, CFSEC_MEM_HOST, NULL));
  rec("enc_pin", pin, T * S);
  uint32_t crcs[T];
  CHECK(cfsec_rs_encode_crc(rs, sh, T, CFSEC_MEM_HOST, NULL, crcs));
  rec("enc_crc", crcs, sizeof crcs);

  /* ---- Reconstruct: erase {0, 5, 13}, len 0 with cap kept ---- */
  const int erased[3] = {0, 5, 13};
  for (int e = 0; e < 3; ++e) {
    memset(page + erased[e] * S, 0, S);
    sh[erased[e]] = (cfsec_shard){page + erased[e] * S, 0, S};
  }
  for (int i = 0; i < T; ++i)
    if (sh[i].len) sh[i] = (cfsec_shard){page + i * S, S, S};
  CHECK(cfsec_rs_reconstruct(rs, sh, T, CFSEC_MEM_HOST, NULL));
  rec("rec_page", page, T * S);
  int lens_ok = 1;
  for (int i = 0; i < T; ++i) lens_ok &= sh[i].len == S;
  rec_int("rec_lens", lens_ok);

  /* ---- error codes the shim maps to Go sentinels ---- */
  for (int i = 0; i < T; ++i) sh[i] = (cfsec_shard){page + i * S, S, S};
  sh[3].len = S - 1;
  rec_int("err_size", cfsec_rs_encode(rs, sh, T, CFSEC_MEM_HOST, NULL));
  for (int i = 0; i < T; ++i) sh[i] = (cfsec_shard){page + i * S, i < 5 ? 0 : S, S};
  rec_int("err_few", cfsec_rs_reconstruct(rs, sh, T, CFSEC_MEM_HOST, NULL));
  rec_int("err_num", cfsec_rs_encode(rs, sh, T - 1, CFSEC_MEM_HOST, NULL));
  cfsec_rs* bad = NULL;
  rec_int("err_new", cfsec_rs_new(0, 4, -1, &bad));
  rec_int("err_max", cfsec_rs_new(200, 100, -1, &bad));

  /* ---- ec.Encoder, EC6P10L2 (LRC), host memory ---- */
  cfsec_tactic t;
  CHECK(cfsec_codemode_tactic(4, &t));
  cfsec_ec* lrc = NULL;
  CHECK(cfsec_ec_new(&t, 1, 0, -1, &lrc));
  const int LT = t.n + t.m + t.l;
  const size_t LS = 4097;
  uint8_t* lbuf = calloc(LT, LS);
  for (size_t i = 0; i < (size_t)t.n * LS; ++i) lbuf[i] = sm_byte();
  cfsec_shard lsh[64];
  for (int i = 0; i < LT; ++i) lsh[i] = (cfsec_shard){lbuf + i * LS, LS, LS};
  CHECK(cfsec_ec_encode(lrc, lsh, LT, CFSEC_MEM_HOST, NULL));
  rec("lrc_enc", lbuf, LT * LS);
  CHECK(cfsec_ec_verify(lrc, lsh, LT, CFSEC_MEM_HOST, NULL, &ok));
  rec_int("lrc_ok", ok);

  /* ---- blobnode repair batch: 3 EC12P4 bids of different sizes and bad sets ---- */
  cfsec_tactic t12;
  CHECK(cfsec_codemode_tactic(9, &t12));
  cfsec_ec* ec12 = NULL;
  CHECK(cfsec_ec_new(&t12, 0, 0, -1, &ec12));
  const size_t bs[3] = {1024, 23, 65536 + 5};
  uint8_t* bb[3];
  cfsec_shard bsh[3 * T];
  for (int b = 0; b < 3; ++b) {
    bb[b] = malloc(T * bs[b]);
    for (size_t i = 0; i < K * bs[b]; ++i) bb[b][i] = sm_byte();
    for (int i = 0; i < T; ++i) bsh[b * T + i] = (cfsec_shard){bb[b] + i * bs[b], bs[b], bs[b]};
    CHECK(cfsec_ec_encode(ec12, bsh + b * T, T, CFSEC_MEM_HOST, NULL));
  }
  for (int b = 0; b < 3; ++b) rec("batch_good", bb[b], T * bs[b]);
  const int bad_idx[] = {1, 2, 3, 4, 0, 15, 7, 9, 12};
  const int bad_off[] = {0, 4, 6, 9};
  for (int j = 0; j < 9; ++j) {
    int b = j < 4 ? 0 : j < 6 ? 1 : 2;
    memset(bb[b] + bad_idx[j] * bs[b], 0, bs[b]);
  }
  bb[2][14 * bs[2] + 100] ^= 0x40; /* bid 2: parity 14, one of the first 12 present, goes bad */
  int bst[3] = {-1, -1, -1};
  CHECK(cfsec_ec_reconstruct_batch(ec12, bsh, T, 3, bad_idx, bad_off, 1, CFSEC_MEM_HOST, bst));
  for (int b = 0; b < 3; ++b) rec("batch_after", bb[b], T * bs[b]);
  rec("batch_status", bst, sizeof bst);

  /* ---- blobnode's tasklet with per-shard buffers (ShardsBuf, work_shard_recover.go:711-716) from
   * cfsec_host_alloc: a non-contiguous vector of page-locked shards, which the Go 1.17 shim passes
   * as a C array of C pointers with no staging (vec_copy.go) -- coded in place over PCIe ---- */
  {
    enum { NB = 2 };
    const size_t PS = 6000 + 3;
    uint8_t* ps[NB][64];
    cfsec_shard psh[NB * 64];
    for (int b = 0; b < NB; ++b)
      for (int i = 0; i < LT; ++i) {
        CHECK(cfsec_host_alloc(PS, (void**)&ps[b][i]));
        for (size_t j = 0; j < PS; ++j) ps[b][i][j] = i < t.n ? sm_byte() : 0;
        psh[b * LT + i] = (cfsec_shard){ps[b][i], PS, PS};
      }
    for (int b = 0; b < NB; ++b) CHECK(cfsec_ec_encode(lrc, psh + b * LT, LT, CFSEC_MEM_HOST, NULL));
    for (int b = 0; b < NB; ++b)
      for (int i = 0; i < LT; ++i) rec("pv_good", ps[b][i], PS);
    const int pb[] = {0, 7, 16, 3, 17};
    const int po[] = {0, 3, 5};
    for (int b = 0; b < NB; ++b)
      for (int j = po[b]; j < po[b + 1]; ++j) memset(ps[b][pb[j]], 0x3C, PS);
    ps[1][9][11] ^= 0x80; /* bid 1: a corrupted surviving global parity -> ErrVerify */
    int pst[NB] = {-1, -1};
    uint32_t pcrc[NB * 64];
    CHECK(cfsec_ec_reconstruct_batch_crc(lrc, psh, LT, NB, pb, po, 1, CFSEC_MEM_HOST, pst, pcrc));
    for (int b = 0; b < NB; ++b)
      for (int i = 0; i < LT; ++i) rec("pv_after", ps[b][i], PS);
    rec("pv_st", pst, sizeof pst);
    rec("pv_crc", pcrc, sizeof(uint32_t) * NB * LT);
    for (int b = 0; b < NB; ++b)
      for (int i = 0; i < LT; ++i) CHECK(cfsec_host_free(ps[b][i]));
  }

  /* ---- contiguous stripes (ec.Buffer layout): the Go 1.17 cgo path, one pointer per call ---- */
  {
    /* EC6P10L2 stripe of 4097-byte shards at stride 4100 inside one pageable allocation */
    const size_t CS = 4097, CST = 4100;
    uint8_t* cb = calloc((size_t)LT, CST);
    for (int i = 0; i < t.n; ++i)
      for (size_t j = 0; j < CS; ++j) cb[i * CST + j] = sm_byte();
    CHECK(cfsec_ec_encode_contig(lrc, cb, CS, CST, LT, CFSEC_MEM_HOST, NULL));
    rec("ct_enc", cb, (size_t)LT * CST);
    CHECK(cfsec_ec_verify_contig(lrc, cb, CS, CST, LT, CFSEC_MEM_HOST, NULL, &ok));
    rec_int("ct_ok", ok);
    const int cbad[3] = {1, 7, LT - 1}; /* a data, a global and a local parity shard */
    for (int e = 0; e < 3; ++e) memset(cb + cbad[e] * CST, 0xA5, CS);
    CHECK(cfsec_ec_reconstruct_contig(lrc, cb, CS, CST, LT, cbad, 3, 0, CFSEC_MEM_HOST, NULL));
    rec("ct_rec", cb, (size_t)LT * CST);
    /* reedsolomon seam: EC12P4 on pinned memory, shards packed, {2, 14} missing */
    uint8_t* rp = NULL;
    CHECK(cfsec_host_alloc(T * 5000, (void**)&rp));
    for (size_t i = 0; i < K * 5000; ++i) rp[i] = sm_byte();
    CHECK(cfsec_rs_encode_contig(rs, rp, 5000, 5000, T, CFSEC_MEM_HOST, NULL));
    rec("ct_rs_enc", rp, T * 5000);
    const int miss[2] = {2, 14};
    memset(rp + 2 * 5000, 0, 5000);
    memset(rp + 14 * 5000, 0, 5000);
    CHECK(cfsec_rs_reconstruct_contig(rs, rp, 5000, 5000, T, miss, 2, 0, CFSEC_MEM_HOST, NULL));
    rec("ct_rs_rec", rp, T * 5000);
    CHECK(cfsec_host_free(rp));
    /* encode batch of 3 stripes in one allocation, with checksums */
    const size_t BS = 3000, BST = 3 * (size_t)LT * BS;
    uint8_t* eb = calloc(3, (size_t)LT * BS);
    (void)BST;
    for (int s = 0; s < 3; ++s)
      for (size_t j = 0; j < (size_t)t.n * BS; ++j) eb[(size_t)s * LT * BS + j] = sm_byte();
    int est[3] = {-1, -1, -1};
    uint32_t ecrc[3 * 64];
    CHECK(cfsec_ec_encode_batch_contig(lrc, eb, BS, BS, (size_t)LT * BS, LT, 3, CFSEC_MEM_HOST, est, ecrc));
    rec("ct_batch", eb, 3 * (size_t)LT * BS);
    rec("ct_batch_st", est, sizeof est);
    rec("ct_batch_crc", ecrc, sizeof(uint32_t) * 3 * LT);
    /* repair tasklet of 2 bids at offsets in one allocation, sizes 3000 and 1500 */
    const uint64_t boff[2] = {0, (uint64_t)LT * 3000 + 64};
    const uint64_t bsz[2] = {3000, 1500};
    uint8_t* rb = calloc(1, boff[1] + (size_t)LT * 1500);
    memcpy(rb, eb, (size_t)LT * 3000);
    int one = 0;
    uint8_t* s1 = rb + boff[1];
    for (size_t j = 0; j < (size_t)t.n * 1500; ++j) s1[j] = sm_byte();
    CHECK(cfsec_ec_encode_contig(lrc, s1, 1500, 1500, LT, CFSEC_MEM_HOST, NULL));
    (void)one;
    rec("ct_tasklet_good", rb, boff[1] + (size_t)LT * 1500);
    const int tb[] = {0, 16, 5, 17};
    const int to[] = {0, 2, 4};
    memset(rb + 0 * 3000, 0, 3000);
    memset(rb + 16 * 3000, 0, 3000);
    memset(s1 + 5 * 1500, 0, 1500);
    memset(s1 + 17 * 1500, 0, 1500);
    int tst[2] = {-1, -1};
    uint32_t tcrc[2 * 64];
    CHECK(cfsec_ec_reconstruct_batch_contig(lrc, rb, boff, bsz, LT, 2, tb, to, 1, CFSEC_MEM_HOST, tst, tcrc));
    rec("ct_tasklet", rb, boff[1] + (size_t)LT * 1500);
    rec("ct_tasklet_st", tst, sizeof tst);
    rec("ct_tasklet_crc", tcrc, sizeof(uint32_t) * 2 * LT);
    rec_int("ct_err_overlap", cfsec_ec_encode_contig(lrc, cb, CS, CS - 1, LT, CFSEC_MEM_HOST, NULL));
    free(cb);
    free(eb);
    free(rb);
  }

  /* ---- crc32block framing (blobnode datafile) ---- */
  const int64_t PL = 200000;
  const int64_t FL = cfsec_crc32block_encode_size(PL, 65536);
  uint8_t* payload = malloc(PL);
  uint8_t* framed = malloc(FL);
  for (int64_t i = 0; i < PL; ++i) payload[i] = sm_byte();
  uint32_t shard_crc = 0;
  CHECK(cfsec_crc32block_encode(payload, PL, 65536, framed, &shard_crc, CFSEC_MEM_HOST, -1, NULL));
  rec("blk_payload", payload, PL);
  rec("blk_framed", framed, FL);
  rec("blk_crc", &shard_crc, 4);
  uint8_t* back = malloc(PL);
  int64_t badblk = 7;
  CHECK(cfsec_crc32block_decode(framed, FL, PL, 65536, 1000, PL, back, &badblk, CFSEC_MEM_HOST, -1, NULL));
  rec("blk_back", back, PL - 1000);
  framed[70000] ^= 1;
  rec_int("blk_mismatch", cfsec_crc32block_decode(framed, FL, PL, 65536, 0, PL, back, &badblk, CFSEC_MEM_HOST, -1, NULL));
  rec_int("blk_badblock", (int)badblk);
  rec_int("blk_short", cfsec_crc32block_decode(framed, FL - 1, PL, 65536, 0, PL, back, &badblk, CFSEC_MEM_HOST, -1, NULL));

  dl_iterate_phdr(find_hip, NULL);
  rec("hip_runtime", hip_path, strlen(hip_path));

  cfsec_ec_free(ec12);
  cfsec_ec_free(lrc);
  cfsec_rs_free(rs);
  CHECK(cfsec_host_free(pin));
  fclose(out);
  return 0;
}
