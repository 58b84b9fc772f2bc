// capi.cpp -- extern "C" boundary declared in include/cfsec.h.
#include <algorithm>
#include <cstdint>
#include <new>
#include <vector>

#include <cstring>

#include "engine.hpp"

namespace cfsec {
const char* last_error_cstr();
uint32_t crc_xpow(int64_t e);                   // gf_crc.hip: x^e mod P
uint32_t crc_mulmod(uint32_t a, uint32_t b);  // a * b mod P
}

using cfsec::ECEncoder;
using cfsec::RSEngine;

struct cfsec_rs {
  std::unique_ptr<RSEngine> e;
};
struct cfsec_ec {
  std::unique_ptr<ECEncoder> e;
};

namespace {

hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

template <class F>
int guarded(F&& f) {
  try {
    return f();
  } catch (const std::bad_alloc&) {
    cfsec::set_last_error("host allocation failed");
    return CFSEC_ERR_DEVICE;
  } catch (...) {
    cfsec::set_last_error("unexpected C++ exception");
    return CFSEC_ERR_DEVICE;
  }
}

// codemode.go:56-79 (the constCodeModeTactic table), keyed by the CodeMode values of
// codemode.go:26-44.
struct ModeRow {
  int mode;
  cfsec_tactic t;
};
const ModeRow kModes[] = {
    {1, {15, 12, 0, 3, 24, 0, 2048}},   // EC15P12
    {2, {6, 6, 0, 3, 11, 0, 2048}},     // EC6P6
    {3, {16, 20, 2, 2, 34, 0, 2048}},   // EC16P20L2
    {4, {6, 10, 2, 2, 14, 0, 2048}},    // EC6P10L2
    {5, {6, 3, 3, 3, 9, 0, 2048}},      // EC6P3L3
    {6, {6, 6, 0, 3, 11, 0, 0}},        // EC6P6Align0
    {7, {6, 6, 0, 3, 11, 0, 512}},      // EC6P6Align512
    {8, {4, 4, 2, 2, 6, 0, 2048}},      // EC4P4L2
    {9, {12, 4, 0, 1, 15, 0, 2048}},    // EC12P4
    {10, {16, 4, 0, 1, 19, 0, 2048}},   // EC16P4
    {11, {3, 3, 0, 1, 5, 0, 2048}},     // EC3P3
    {12, {10, 4, 0, 1, 13, 0, 2048}},   // EC10P4
    {13, {6, 3, 0, 1, 8, 0, 2048}},     // EC6P3
    {14, {12, 9, 0, 3, 20, 0, 2048}},   // EC12P9
    {200, {6, 6, 9, 3, 11, 0, 2048}},   // EC6P6L9
    {201, {6, 8, 10, 2, 13, 0, 0}},     // EC6P8L10
};

// EncodeSize (common/crc32block/util.go:50-57) for a valid block length.
int64_t crc32block_framed(int64_t size, int64_t block_len) {
  const int64_t p = block_len - 4;
  return size + 4 * ((size + p - 1) / p);
}

// Encoder.Encode / Decoder.Reader through launch_crc32block: device pointers in place, page-locked
// host buffers in place (device aliases), other host memory staged through the workspace.
int crc32block_call(bool encode, const uint8_t* src, int64_t src_len, int64_t size, int64_t block_len, int64_t from,
                    int64_t to, uint8_t* dst, uint32_t* shard_crc, int64_t* bad_block, int mem, int device,
                    void* stream) {
  if (!cfsec::crc32block_valid_len(block_len)) return CFSEC_ERR_INVALID_BLOCK;
  if (size < 0 || (mem != CFSEC_MEM_HOST && mem != CFSEC_MEM_DEVICE)) return CFSEC_ERR_INVALID_ARG;
  if (!encode && (from < 0 || from > to || to > size)) return CFSEC_ERR_INVALID_ARG;
  if (bad_block) *bad_block = -1;
  if (shard_crc) *shard_crc = 0;  // crc32.ChecksumIEEE(nil)
  const int64_t P = block_len - 4;
  int64_t b0 = 0, nb = (size + P - 1) / P;  // blocks the call touches
  if (!encode) {
    b0 = from / P;
    const int64_t b1 = from < to ? (to - 1) / P : (from % P ? b0 : b0 - 1);  // see crc32block.hip
    nb = b1 - b0 + 1;
  }
  if (nb <= 0) return CFSEC_OK;
  const int64_t framed = crc32block_framed(size, block_len);
  const int64_t f0 = b0 * block_len, f1 = std::min(framed, (b0 + nb) * block_len);
  const int64_t in_bytes = encode ? size : f1 - f0;
  const int64_t out_bytes = encode ? framed : to - from;
  if (!src || (!dst && out_bytes > 0)) return CFSEC_ERR_INVALID_ARG;
  // Decoder.Reader reads the touched blocks through an io.SectionReader: a framed object that ends
  // before them is io.ErrUnexpectedEOF there (decode.go:94-97, 126-130), ErrShortData here --
  // checked before any copy or launch, so nothing reads past the caller's buffer.
  if (!encode && src_len < f1) {
    cfsec::set_last_error("crc32block decode: framed source shorter than the blocks the range touches");
    return CFSEC_ERR_SHORT_DATA;
  }
  return guarded([&] {
    if (device < 0 && hipGetDevice(&device) != hipSuccess) return (int)CFSEC_ERR_DEVICE;
    cfsec::DeviceContext* ctx = cfsec::DeviceContext::get(device);
    if (!ctx) {
      cfsec::set_last_error("no HIP device available to the cfsec engine");
      return (int)CFSEC_ERR_DEVICE;
    }
    cfsec::DeviceGuard g(device);
    if (!g.ok()) return cfsec::hip_status(hipErrorInvalidDevice, "hipSetDevice");
    const uint8_t* din = src;
    uint8_t* dout = dst;
    bool stage = false;
    if (mem == CFSEC_MEM_HOST) {
      uint8_t *pi = nullptr, *po = nullptr;
      const bool pin_in = cfsec::device_alias(const_cast<uint8_t*>(src) + (encode ? 0 : f0), &pi);
      const bool pin_out = out_bytes == 0 || cfsec::device_alias(dst, &po);
      stage = !(pin_in && pin_out);
      if (!stage) {
        din = encode ? pi : reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(pi) - (uintptr_t)f0);
        dout = po;
      }
    }
    cfsec::DeviceContext::Workspace* ws = nullptr;
    int st = ctx->acquire(stage ? (size_t)(in_bytes + out_bytes) : 0, 2, &ws);
    if (st != CFSEC_OK) return st;
    hipStream_t s = stream ? as_stream(stream) : ws->stream;
    if (!stream && !stage) st = ctx->order_after_default(ws);
    if (st == CFSEC_OK && stage) {
      st = cfsec::hip_status(hipMemcpyAsync(ws->dbuf, src + (encode ? 0 : f0), (size_t)in_bytes, hipMemcpyHostToDevice, s),
                             "hipMemcpyAsync H2D");
      // the launch addresses the framed object from its start; the staged copy begins at block b0
      din = encode ? ws->dbuf : reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(ws->dbuf) - (uintptr_t)f0);
      dout = ws->dbuf + in_bytes;
    }
    if (st == CFSEC_OK) st = cfsec::hip_status(hipMemsetAsync(ws->dflags, 0xFF, 4, s), "hipMemsetAsync");
    if (st == CFSEC_OK) st = cfsec::hip_status(hipMemsetAsync(ws->dflags + 1, 0, 4, s), "hipMemsetAsync");
    cfsec::Crc32BlockJob j;
    j.encode = encode;
    j.n = 1;
    j.in = &din;
    j.out = &dout;
    j.size = size;
    j.block_len = block_len;
    j.from = from;
    j.to = to;
    j.bad = ws->dflags;
    j.whole = (encode && shard_crc) ? ws->dflags + 1 : nullptr;
    if (st == CFSEC_OK) st = cfsec::hip_status(cfsec::launch_crc32block(j, s), "launch_crc32block");
    if (st == CFSEC_OK && stage && out_bytes > 0)
      st = cfsec::hip_status(hipMemcpyAsync(dst, dout, (size_t)out_bytes, hipMemcpyDeviceToHost, s),
                             "hipMemcpyAsync D2H");
    if (st == CFSEC_OK)
      st = cfsec::hip_status(hipMemcpyAsync(ws->hflags, ws->dflags, 8, hipMemcpyDeviceToHost, s), "hipMemcpyAsync D2H");
    const int sync = ctx->finish(ws, s);
    if (st == CFSEC_OK) st = sync;
    if (st == CFSEC_OK) {
      if (encode && shard_crc) *shard_crc = ws->hflags[1];
      if (!encode && ws->hflags[0] != 0xFFFFFFFFu) {
        if (bad_block) *bad_block = b0 + (int64_t)ws->hflags[0];
        st = CFSEC_ERR_MISMATCHED_CRC;
      }
    }
    ctx->release(ws);
    return st;
  });
}

}  // namespace

extern "C" {

const char* cfsec_version(void) { return "cfsec 0.4.0 (gfx950)"; }

const char* cfsec_last_error(void) { return cfsec::last_error_cstr(); }

const char* cfsec_status_name(int status) {
  switch (status) {
    case CFSEC_OK: return "OK";
    case CFSEC_ERR_TOO_FEW_SHARDS: return "ErrTooFewShards";
    case CFSEC_ERR_SHARD_NO_DATA: return "ErrShardNoData";
    case CFSEC_ERR_SHARD_SIZE: return "ErrShardSize";
    case CFSEC_ERR_INV_SHARD_NUM: return "ErrInvShardNum";
    case CFSEC_ERR_MAX_SHARD_NUM: return "ErrMaxShardNum";
    case CFSEC_ERR_SHORT_DATA: return "ErrShortData";
    case CFSEC_ERR_RECONSTRUCT_REQUIRED: return "ErrReconstructRequired";
    case CFSEC_ERR_SINGULAR: return "errSingular";
    case CFSEC_ERR_INVALID_CODE_MODE: return "ErrInvalidCodeMode";
    case CFSEC_ERR_VERIFY: return "ErrVerify";
    case CFSEC_ERR_INVALID_SHARDS: return "ErrInvalidShards";
    case CFSEC_ERR_INVALID_ARG: return "ErrInvalidArg";
    case CFSEC_ERR_DEVICE: return "ErrDevice";
    case CFSEC_ERR_NOT_SUPPORTED: return "ErrNotSupported";
    case CFSEC_ERR_INVALID_BLOCK: return "ErrInvalidBlock";
    case CFSEC_ERR_MISMATCHED_CRC: return "ErrMismatchedCrc";
    default: return "ErrUnknown";
  }
}

int cfsec_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int cfsec_set_sync_poll(int on) { return cfsec::sync_poll_mode().exchange(on ? 1 : 0); }

// ---------------- reedsolomon.Encoder ----------------

int cfsec_rs_new(int data_shards, int parity_shards, int device, cfsec_rs** out) {
  if (!out) return CFSEC_ERR_INVALID_ARG;
  *out = nullptr;
  return guarded([&] {
    std::unique_ptr<RSEngine> e;
    int st = RSEngine::create(data_shards, parity_shards, device, &e);
    if (st != CFSEC_OK) return st;
    *out = new cfsec_rs{std::move(e)};
    return (int)CFSEC_OK;
  });
}

void cfsec_rs_free(cfsec_rs* h) { delete h; }

int cfsec_rs_data_shards(const cfsec_rs* h) { return h ? h->e->k() : -1; }
int cfsec_rs_parity_shards(const cfsec_rs* h) { return h ? h->e->m() : -1; }

int cfsec_rs_matrix(const cfsec_rs* h, uint8_t* out, size_t out_len) {
  if (!h || !out) return CFSEC_ERR_INVALID_ARG;
  const auto& m = h->e->matrix();
  if (out_len < m.v.size()) return CFSEC_ERR_INVALID_ARG;
  std::copy(m.v.begin(), m.v.end(), out);
  return CFSEC_OK;
}

int cfsec_rs_encode(cfsec_rs* h, cfsec_shard* shards, int n, int mem, void* stream) {
  if (!h) return CFSEC_ERR_INVALID_ARG;
  return guarded([&] { return h->e->encode(shards, n, mem, as_stream(stream)); });
}

int cfsec_rs_verify(cfsec_rs* h, cfsec_shard* shards, int n, int mem, void* stream, int* ok) {
  if (!h || !ok) return CFSEC_ERR_INVALID_ARG;
  return guarded([&] {
    bool b = false;
    int st = h->e->verify(shards, n, mem, as_stream(stream), &b);
    *ok = b ? 1 : 0;
    return st;
  });
}

int cfsec_rs_reconstruct(cfsec_rs* h, cfsec_shard* shards, int n, int mem, void* stream) {
  if (!h) return CFSEC_ERR_INVALID_ARG;
  return guarded([&] { return h->e->reconstruct(shards, n, false, mem, as_stream(stream)); });
}

int cfsec_rs_reconstruct_data(cfsec_rs* h, cfsec_shard* shards, int n, int mem, void* stream) {
  if (!h) return CFSEC_ERR_INVALID_ARG;
  return guarded([&] { return h->e->reconstruct(shards, n, true, mem, as_stream(stream)); });
}

int cfsec_rs_split(cfsec_rs* h, uint8_t* data, size_t len, size_t cap, cfsec_shard* out,
                   uint8_t* pad, size_t pad_len, size_t* pad_needed) {
  if (!h) return CFSEC_ERR_INVALID_ARG;
  return guarded([&] { return h->e->split(data, len, cap, out, pad, pad_len, pad_needed); });
}

int cfsec_rs_join(cfsec_rs* h, uint8_t* dst, size_t dst_len, const cfsec_shard* shards, int n,
                  size_t out_size) {
  if (!h || (!shards && n > 0)) return CFSEC_ERR_INVALID_ARG;
  return guarded([&] { return h->e->join(dst, dst_len, shards, n, out_size); });
}

int cfsec_rs_encode_batch(cfsec_rs* h, uint8_t* const* ptrs, size_t shard_size, int nstripes,
                          void* stream) {
  if (!h) return CFSEC_ERR_INVALID_ARG;
  return guarded([&] { return h->e->encode_batch(ptrs, shard_size, nstripes, as_stream(stream)); });
}

int cfsec_rs_verify_batch(cfsec_rs* h, uint8_t* const* ptrs, size_t shard_size, int nstripes,
                          uint32_t* flags, void* stream) {
  if (!h) return CFSEC_ERR_INVALID_ARG;
  return guarded(
      [&] { return h->e->verify_batch(ptrs, shard_size, nstripes, flags, as_stream(stream)); });
}

int cfsec_rs_reconstruct_batch(cfsec_rs* h, uint8_t* const* ptrs, size_t shard_size, int nstripes,
                               const int* erased, int nerased, int data_only, void* stream) {
  if (!h) return CFSEC_ERR_INVALID_ARG;
  return guarded([&] {
    return h->e->reconstruct_batch(ptrs, shard_size, nstripes, erased, nerased, data_only != 0,
                                   as_stream(stream));
  });
}

int cfsec_rs_encode_crc(cfsec_rs* h, cfsec_shard* shards, int n, int mem, void* stream, uint32_t* crcs) {
  if (!h) return CFSEC_ERR_INVALID_ARG;
  return guarded([&] { return h->e->encode_crc(shards, n, mem, as_stream(stream), crcs); });
}

int cfsec_rs_encode_crc_batch(cfsec_rs* h, uint8_t* const* ptrs, size_t shard_size, int nstripes,
                              uint32_t* crcs, void* stream) {
  if (!h) return CFSEC_ERR_INVALID_ARG;
  return guarded([&] { return h->e->encode_crc_batch(ptrs, shard_size, nstripes, crcs, as_stream(stream)); });
}

int cfsec_rs_reconstruct_crc_batch(cfsec_rs* h, uint8_t* const* ptrs, size_t shard_size, int nstripes,
                                   const int* erased, int nerased, int data_only, uint32_t* crcs,
                                   void* stream) {
  if (!h) return CFSEC_ERR_INVALID_ARG;
  return guarded([&] {
    return h->e->reconstruct_crc_batch(ptrs, shard_size, nstripes, erased, nerased, data_only != 0, crcs,
                                       as_stream(stream));
  });
}

// ---------------- stripe batches ----------------

int cfsec_rs_set_devices(cfsec_rs* h, const int* devices, int ndev) {
  if (!h) return CFSEC_ERR_INVALID_ARG;
  return guarded([&] { return h->e->set_devices(devices, ndev); });
}

extern "C++" {
namespace {
std::vector<cfsec_shard*> stripe_views(cfsec_shard* shards, int nstripes, int total) {
  std::vector<cfsec_shard*> v((size_t)std::max(nstripes, 0));
  for (int s = 0; s < nstripes; ++s) v[s] = shards + (size_t)s * total;
  return v;
}
}  // namespace
}

int cfsec_batch_partition(const uint64_t* bytes, int n, int ndev, int* dev) {
  if (n < 0 || ndev <= 0 || (n > 0 && (!bytes || !dev))) return CFSEC_ERR_INVALID_ARG;
  cfsec::partition_stripes(bytes, n, ndev, dev);
  return CFSEC_OK;
}

int cfsec_rs_encode_stripes(cfsec_rs* h, cfsec_shard* shards, int nstripes, int mem, int* status) {
  if (!h || nstripes < 0 || (nstripes > 0 && (!shards || !status))) return CFSEC_ERR_INVALID_ARG;
  return guarded([&] {
    auto v = stripe_views(shards, nstripes, h->e->total());
    return h->e->encode_stripes(v.data(), nstripes, mem, status);
  });
}

int cfsec_rs_verify_stripes(cfsec_rs* h, cfsec_shard* shards, int nstripes, int mem, int* status) {
  if (!h || nstripes < 0 || (nstripes > 0 && (!shards || !status))) return CFSEC_ERR_INVALID_ARG;
  return guarded([&] {
    auto v = stripe_views(shards, nstripes, h->e->total());
    return h->e->verify_stripes(v.data(), nstripes, mem, status);
  });
}

int cfsec_rs_reconstruct_stripes(cfsec_rs* h, cfsec_shard* shards, int nstripes, int verify, int mem,
                                 int* status) {
  if (!h || nstripes < 0 || (nstripes > 0 && (!shards || !status))) return CFSEC_ERR_INVALID_ARG;
  return guarded([&] {
    auto v = stripe_views(shards, nstripes, h->e->total());
    return h->e->reconstruct_stripes(v.data(), nstripes, mem, verify != 0, status);
  });
}

// ---------------- ec.Encoder ----------------

int cfsec_codemode_tactic(int codemode, cfsec_tactic* t) {
  if (!t) return CFSEC_ERR_INVALID_ARG;
  for (const auto& r : kModes)
    if (r.mode == codemode) {
      *t = r.t;
      return CFSEC_OK;
    }
  return CFSEC_ERR_INVALID_CODE_MODE;
}

int cfsec_ec_new(const cfsec_tactic* tactic, int enable_verify, int concurrency, int device,
                 cfsec_ec** out) {
  if (!out) return CFSEC_ERR_INVALID_ARG;
  *out = nullptr;
  if (!tactic) return CFSEC_ERR_INVALID_CODE_MODE;
  return guarded([&] {
    std::unique_ptr<ECEncoder> e;
    int st = ECEncoder::create(*tactic, enable_verify != 0, concurrency, device, &e);
    if (st != CFSEC_OK) return st;
    *out = new cfsec_ec{std::move(e)};
    return (int)CFSEC_OK;
  });
}

void cfsec_ec_free(cfsec_ec* h) { delete h; }

int cfsec_ec_encode(cfsec_ec* h, cfsec_shard* shards, int n, int mem, void* stream) {
  if (!h) return CFSEC_ERR_INVALID_ARG;
  return guarded([&] { return h->e->encode(shards, n, mem, as_stream(stream)); });
}

int cfsec_ec_reconstruct(cfsec_ec* h, cfsec_shard* shards, int n, const int* bad_idx, int nbad,
                         int mem, void* stream) {
  if (!h || (nbad > 0 && !bad_idx) || nbad < 0) return CFSEC_ERR_INVALID_ARG;
  return guarded(
      [&] { return h->e->reconstruct(shards, n, bad_idx, nbad, mem, as_stream(stream)); });
}

int cfsec_ec_reconstruct_data(cfsec_ec* h, cfsec_shard* shards, int n, const int* bad_idx,
                              int nbad, int mem, void* stream) {
  if (!h || (nbad > 0 && !bad_idx) || nbad < 0) return CFSEC_ERR_INVALID_ARG;
  return guarded(
      [&] { return h->e->reconstruct_data(shards, n, bad_idx, nbad, mem, as_stream(stream)); });
}

int cfsec_ec_verify(cfsec_ec* h, cfsec_shard* shards, int n, int mem, void* stream, int* ok) {
  if (!h || !ok) return CFSEC_ERR_INVALID_ARG;
  return guarded([&] {
    bool b = false;
    int st = h->e->verify(shards, n, mem, as_stream(stream), &b);
    *ok = b ? 1 : 0;
    return st;
  });
}

int cfsec_ec_set_devices(cfsec_ec* h, const int* devices, int ndev) {
  if (!h) return CFSEC_ERR_INVALID_ARG;
  return guarded([&] { return h->e->set_devices(devices, ndev); });
}

int cfsec_ec_reconstruct_batch(cfsec_ec* h, cfsec_shard* shards, int n, int nbids, const int* bad_idx,
                               const int* bad_off, int verify, int mem, int* status) {
  if (!h || nbids < 0 || n <= 0 || (nbids > 0 && (!shards || !status || !bad_off))) return CFSEC_ERR_INVALID_ARG;
  if (nbids > 0 && bad_off[0] != 0) return CFSEC_ERR_INVALID_ARG;  // offsets index bad_idx from 0
  for (int b = 0; b < nbids; ++b)
    if (bad_off[b + 1] < bad_off[b] || (bad_off[b + 1] > bad_off[b] && !bad_idx)) return CFSEC_ERR_INVALID_ARG;
  return guarded([&] { return h->e->reconstruct_batch(shards, n, nbids, bad_idx, bad_off, mem, verify != 0, status); });
}

int cfsec_ec_encode_batch(cfsec_ec* h, cfsec_shard* shards, int n, int nstripes, int mem, int* status) {
  if (!h || nstripes < 0 || n <= 0 || (nstripes > 0 && (!shards || !status))) return CFSEC_ERR_INVALID_ARG;
  return guarded([&] { return h->e->encode_batch(shards, n, nstripes, mem, status); });
}

int cfsec_ec_reconstruct_batch_crc(cfsec_ec* h, cfsec_shard* shards, int n, int nbids, const int* bad_idx,
                                   const int* bad_off, int verify, int mem, int* status, uint32_t* crcs) {
  if (!h || nbids < 0 || n <= 0 || (nbids > 0 && (!shards || !status || !bad_off || !crcs)))
    return CFSEC_ERR_INVALID_ARG;
  if (nbids > 0 && bad_off[0] != 0) return CFSEC_ERR_INVALID_ARG;
  for (int b = 0; b < nbids; ++b)
    if (bad_off[b + 1] < bad_off[b] || (bad_off[b + 1] > bad_off[b] && !bad_idx)) return CFSEC_ERR_INVALID_ARG;
  std::memset(crcs, 0, sizeof(uint32_t) * (size_t)nbids * n);
  cfsec::CrcOut c;
  c.words = crcs;
  c.n = (size_t)nbids * n;
  return guarded([&] {
    return h->e->reconstruct_batch(shards, n, nbids, bad_idx, bad_off, mem, verify != 0, status, nullptr, &c);
  });
}

int cfsec_ec_encode_batch_crc(cfsec_ec* h, cfsec_shard* shards, int n, int nstripes, int mem, int* status,
                              uint32_t* crcs) {
  if (!h || nstripes < 0 || n <= 0 || (nstripes > 0 && (!shards || !status || !crcs))) return CFSEC_ERR_INVALID_ARG;
  std::memset(crcs, 0, sizeof(uint32_t) * (size_t)nstripes * n);
  cfsec::CrcOut c;
  c.words = crcs;
  c.n = (size_t)nstripes * n;
  return guarded([&] { return h->e->encode_batch(shards, n, nstripes, mem, status, nullptr, &c); });
}

int cfsec_ec_reconstruct_batch_async(cfsec_ec* h, cfsec_shard* shards, int n, int nbids, const int* bad_idx,
                                     const int* bad_off, int verify, int* status, uint32_t* flags, uint32_t* crcs,
                                     void* stream) {
  if (!h || nbids < 0 || n <= 0 || (nbids > 0 && (!shards || !status || !bad_off))) return CFSEC_ERR_INVALID_ARG;
  if (nbids > 0 && bad_off[0] != 0) return CFSEC_ERR_INVALID_ARG;
  for (int b = 0; b < nbids; ++b)
    if (bad_off[b + 1] < bad_off[b] || (bad_off[b + 1] > bad_off[b] && !bad_idx)) return CFSEC_ERR_INVALID_ARG;
  if (verify && nbids > 0 && !flags) return CFSEC_ERR_INVALID_ARG;
  cfsec::AsyncOut a;
  a.stream = as_stream(stream);
  a.flags = flags;
  cfsec::CrcOut c;
  c.words = crcs;
  c.n = (size_t)nbids * n;
  return guarded([&] {
    return h->e->reconstruct_batch(shards, n, nbids, bad_idx, bad_off, CFSEC_MEM_DEVICE, verify != 0, status, &a,
                                   crcs ? &c : nullptr);
  });
}

int cfsec_ec_encode_batch_async(cfsec_ec* h, cfsec_shard* shards, int n, int nstripes, int* status, uint32_t* flags,
                                uint32_t* crcs, void* stream) {
  if (!h || nstripes < 0 || n <= 0 || (nstripes > 0 && (!shards || !status))) return CFSEC_ERR_INVALID_ARG;
  cfsec::AsyncOut a;
  a.stream = as_stream(stream);
  a.flags = flags;
  cfsec::CrcOut c;
  c.words = crcs;
  c.n = (size_t)nstripes * n;
  return guarded([&] {
    return h->e->encode_batch(shards, n, nstripes, CFSEC_MEM_DEVICE, status, &a, crcs ? &c : nullptr);
  });
}

int cfsec_ec_repair_rows(cfsec_ec* h, const int* bad_idx, int nbad, const int* want, int nwant, int* in_idx,
                         uint8_t* rows) {
  if (!h) return CFSEC_ERR_INVALID_ARG;
  return guarded([&] { return h->e->repair_rows(bad_idx, nbad, want, nwant, in_idx, rows); });
}

int cfsec_ec_matvec_batch(cfsec_ec* h, const uint8_t* coef, int rows, uint8_t* const* ptrs, size_t shard_size,
                          int nstripes, void* stream) {
  if (!h) return CFSEC_ERR_INVALID_ARG;
  return guarded([&] { return h->e->matvec_batch(coef, rows, ptrs, shard_size, nstripes, as_stream(stream)); });
}

int cfsec_ec_shards_in_idc(const cfsec_ec* h, int idx, int* out, int out_cap, int* count) {
  if (!h || !count) return CFSEC_ERR_INVALID_ARG;
  const std::vector<int> v = h->e->shards_in_idc(idx);
  *count = (int)v.size();
  if (out_cap < (int)v.size() || (!out && !v.empty())) return CFSEC_ERR_INVALID_ARG;
  for (size_t i = 0; i < v.size(); ++i) out[i] = v[i];
  return CFSEC_OK;
}

// ---------------- pinned host memory ----------------

int cfsec_host_alloc(size_t size, void** out) {
  if (!out) return CFSEC_ERR_INVALID_ARG;
  *out = nullptr;
  if (size == 0) return CFSEC_OK;
  return guarded([&] {
    const int st = (int)cfsec::hip_status(hipHostMalloc(out, size, hipHostMallocPortable), "hipHostMalloc");
    if (st == CFSEC_OK) cfsec::host_range_add(*out, size);
    return st;
  });
}

int cfsec_host_free(void* p) {
  if (!p) return CFSEC_OK;
  return guarded([&] {
    cfsec::host_range_remove(p);
    return (int)cfsec::hip_status(hipHostFree(p), "hipHostFree");
  });
}

// ---------------- CRC32 ----------------

int cfsec_crc32_ieee_batch(uint8_t* const* ptrs, size_t shard_size, int n, uint32_t* out,
                           int device, void* stream) {
  if ((!ptrs && n > 0) || !out || n < 0) return CFSEC_ERR_INVALID_ARG;
  return guarded([&] {
    if (device < 0 && hipGetDevice(&device) != hipSuccess) return (int)CFSEC_ERR_DEVICE;
    cfsec::DeviceContext* ctx = cfsec::DeviceContext::get(device);
    if (!ctx) {
      cfsec::set_last_error("no HIP device available to the cfsec engine");
      return (int)CFSEC_ERR_DEVICE;
    }
    cfsec::DeviceGuard g(device);
    if (!g.ok()) return cfsec::hip_status(hipErrorInvalidDevice, "hipSetDevice");
    cfsec::DeviceContext::Workspace* ws = nullptr;
    int st = ctx->acquire(0, (size_t)n, &ws);
    if (st != CFSEC_OK) return st;
    hipStream_t s = stream ? as_stream(stream) : ws->stream;
    if (!stream) st = ctx->order_after_default(ws);
    if (st == CFSEC_OK)
      st = cfsec::hip_status(cfsec::launch_crc32(ptrs, shard_size, n, ws->dflags, s), "launch_crc32");
    if (st == CFSEC_OK)
      st = cfsec::hip_status(hipMemcpyAsync(ws->hflags, ws->dflags, 4 * (size_t)n, hipMemcpyDeviceToHost, s),
                             "hipMemcpyAsync D2H");
    const int sync = ctx->finish(ws, s);
    if (st == CFSEC_OK) st = sync;
    if (st == CFSEC_OK)
      for (int i = 0; i < n; ++i) out[i] = cfsec::crc32_finalize(ws->hflags[i], shard_size);
    ctx->release(ws);
    return st;
  });
}

// Checksums of concatenations (host arithmetic in GF(2)[x] mod P, gf_crc.hip's xpow / mulmod):
// ChecksumIEEE(A || B) = ChecksumIEEE(A) * x^(8|B|) ^ ChecksumIEEE(B) -- the init and final XORs of
// the two halves cancel (zlib's crc32_combine identity).
uint32_t cfsec_crc32_combine(uint32_t crc1, uint32_t crc2, int64_t len2) {
  if (len2 <= 0) return crc1 ^ crc2;
  return cfsec::crc_mulmod(cfsec::crc_xpow(8 * len2), crc1) ^ crc2;
}

int cfsec_crc32_shift(uint32_t* words, int n, int64_t nbytes) {
  if ((!words && n > 0) || n < 0 || nbytes < 0) return CFSEC_ERR_INVALID_ARG;
  if (nbytes == 0) return CFSEC_OK;
  const uint32_t xp = cfsec::crc_xpow(8 * nbytes);
  for (int i = 0; i < n; ++i) words[i] = cfsec::crc_mulmod(xp, words[i]);
  return CFSEC_OK;
}

int cfsec_stream_copy(void* dst, const void* src, size_t bytes, void* stream) {
  return guarded([&] {
    return (int)cfsec::hip_status(cfsec::launch_stream_copy(dst, src, bytes, static_cast<hipStream_t>(stream)),
                                  "launch_stream_copy");
  });
}

// ---------------- crc32block ----------------

int64_t cfsec_crc32block_encode_size(int64_t size, int64_t block_len) {
  if (!cfsec::crc32block_valid_len(block_len) || size < 0) return -1;
  return crc32block_framed(size, block_len);
}

int64_t cfsec_crc32block_decode_size(int64_t total, int64_t block_len) {
  if (!cfsec::crc32block_valid_len(block_len) || total < 0) return -1;
  return total - 4 * ((total + block_len - 1) / block_len);  // util.go:59-65
}

int cfsec_crc32block_encode(const uint8_t* src, int64_t size, int64_t block_len, uint8_t* dst,
                            uint32_t* shard_crc, int mem, int device, void* stream) {
  return crc32block_call(true, src, size, size, block_len, 0, size, dst, shard_crc, nullptr, mem, device, stream);
}

int cfsec_crc32block_decode(const uint8_t* src, int64_t src_len, int64_t size, int64_t block_len, int64_t from,
                            int64_t to, uint8_t* dst, int64_t* bad_block, int mem, int device, void* stream) {
  return crc32block_call(false, src, src_len, size, block_len, from, to, dst, nullptr, bad_block, mem, device,
                         stream);
}

int cfsec_crc32block_encode_batch(const uint8_t* const* srcs, uint8_t* const* dsts, int n, int64_t size,
                                  int64_t block_len, uint32_t* shard_crcs, void* stream) {
  if (!cfsec::crc32block_valid_len(block_len)) return CFSEC_ERR_INVALID_BLOCK;
  if (n < 0 || size < 0 || (n > 0 && (!srcs || !dsts))) return CFSEC_ERR_INVALID_ARG;
  return guarded([&] {
    hipStream_t s = as_stream(stream);
    int st = CFSEC_OK;
    if (shard_crcs && n > 0)
      st = cfsec::hip_status(hipMemsetAsync(shard_crcs, 0, 4 * (size_t)n, s), "hipMemsetAsync");
    cfsec::Crc32BlockJob j;
    j.encode = true;
    j.n = n;
    j.in = srcs;
    j.out = dsts;
    j.size = size;
    j.block_len = block_len;
    j.whole = shard_crcs;
    if (st == CFSEC_OK) st = cfsec::hip_status(cfsec::launch_crc32block(j, s), "launch_crc32block");
    return st;
  });
}

int cfsec_crc32block_decode_batch(const uint8_t* const* srcs, int64_t src_len, uint8_t* const* dsts, int n,
                                  int64_t size, int64_t block_len, int64_t from, int64_t to, uint32_t* bad,
                                  void* stream) {
  if (!cfsec::crc32block_valid_len(block_len)) return CFSEC_ERR_INVALID_BLOCK;
  if (n < 0 || size < 0 || from < 0 || from > to || to > size || (n > 0 && (!srcs || !bad)) ||
      (n > 0 && to > from && !dsts))
    return CFSEC_ERR_INVALID_ARG;
  {  // the framed end of the last block the range touches must lie inside every source object
    const int64_t P = block_len - 4, b0 = from / P;
    const int64_t b1 = from < to ? (to - 1) / P : (from % P ? b0 : b0 - 1);
    const int64_t f1 = std::min(crc32block_framed(size, block_len), (b1 + 1) * block_len);
    if (b1 >= b0 && src_len < f1) {
      cfsec::set_last_error("crc32block decode: framed source shorter than the blocks the range touches");
      return CFSEC_ERR_SHORT_DATA;
    }
  }
  return guarded([&] {
    hipStream_t s = as_stream(stream);
    int st = CFSEC_OK;
    if (n > 0) st = cfsec::hip_status(hipMemsetAsync(bad, 0xFF, 4 * (size_t)n, s), "hipMemsetAsync");
    cfsec::Crc32BlockJob j;
    j.encode = false;
    j.n = n;
    j.in = srcs;
    j.out = dsts;
    j.size = size;
    j.block_len = block_len;
    j.from = from;
    j.to = to;
    j.bad = bad;
    if (st == CFSEC_OK) st = cfsec::hip_status(cfsec::launch_crc32block(j, s), "launch_crc32block");
    return st;
  });
}

}  // extern "C"

// ---------------- contiguous stripes (ec.Buffer layout) ----------------

namespace {
// Shard headers of a contiguous stripe: shard i at base + i * stride, `size` bytes, missing[] (when
// given) marked len 0 with their buffer kept as capacity.
int contig_shards(uint8_t* base, size_t size, size_t stride, int n, const int* missing, int nmissing,
                  std::vector<cfsec_shard>* out) {
  if (!base || n <= 0 || size == 0 || stride < size || nmissing < 0 || (nmissing > 0 && !missing))
    return CFSEC_ERR_INVALID_ARG;
  out->assign((size_t)n, cfsec_shard{nullptr, 0, 0});
  for (int i = 0; i < n; ++i) (*out)[i] = cfsec_shard{base + (size_t)i * stride, size, size};
  for (int j = 0; j < nmissing; ++j) {
    if (missing[j] < 0 || missing[j] >= n) return CFSEC_ERR_INVALID_ARG;
    (*out)[missing[j]].len = 0;
  }
  return CFSEC_OK;
}
}  // namespace

int cfsec_rs_encode_contig(cfsec_rs* h, uint8_t* base, size_t shard_size, size_t stride, int n, int mem,
                           void* stream) {
  std::vector<cfsec_shard> v;
  const int st = contig_shards(base, shard_size, stride, n, nullptr, 0, &v);
  if (!h || st != CFSEC_OK) return CFSEC_ERR_INVALID_ARG;
  return cfsec_rs_encode(h, v.data(), n, mem, stream);
}

int cfsec_rs_verify_contig(cfsec_rs* h, uint8_t* base, size_t shard_size, size_t stride, int n, int mem,
                           void* stream, int* ok) {
  std::vector<cfsec_shard> v;
  const int st = contig_shards(base, shard_size, stride, n, nullptr, 0, &v);
  if (!h || st != CFSEC_OK) return CFSEC_ERR_INVALID_ARG;
  return cfsec_rs_verify(h, v.data(), n, mem, stream, ok);
}

int cfsec_rs_reconstruct_contig(cfsec_rs* h, uint8_t* base, size_t shard_size, size_t stride, int n,
                                const int* missing, int nmissing, int data_only, int mem, void* stream) {
  std::vector<cfsec_shard> v;
  const int st = contig_shards(base, shard_size, stride, n, missing, nmissing, &v);
  if (!h || st != CFSEC_OK) return CFSEC_ERR_INVALID_ARG;
  return data_only ? cfsec_rs_reconstruct_data(h, v.data(), n, mem, stream)
                   : cfsec_rs_reconstruct(h, v.data(), n, mem, stream);
}

int cfsec_ec_encode_contig(cfsec_ec* h, uint8_t* base, size_t shard_size, size_t stride, int n, int mem,
                           void* stream) {
  std::vector<cfsec_shard> v;
  const int st = contig_shards(base, shard_size, stride, n, nullptr, 0, &v);
  if (!h || st != CFSEC_OK) return CFSEC_ERR_INVALID_ARG;
  return cfsec_ec_encode(h, v.data(), n, mem, stream);
}

int cfsec_ec_verify_contig(cfsec_ec* h, uint8_t* base, size_t shard_size, size_t stride, int n, int mem,
                           void* stream, int* ok) {
  std::vector<cfsec_shard> v;
  const int st = contig_shards(base, shard_size, stride, n, nullptr, 0, &v);
  if (!h || st != CFSEC_OK) return CFSEC_ERR_INVALID_ARG;
  return cfsec_ec_verify(h, v.data(), n, mem, stream, ok);
}

int cfsec_ec_reconstruct_contig(cfsec_ec* h, uint8_t* base, size_t shard_size, size_t stride, int n,
                                const int* bad_idx, int nbad, int data_only, int mem, void* stream) {
  std::vector<cfsec_shard> v;
  const int st = contig_shards(base, shard_size, stride, n, nullptr, 0, &v);
  if (!h || st != CFSEC_OK) return CFSEC_ERR_INVALID_ARG;
  return data_only ? cfsec_ec_reconstruct_data(h, v.data(), n, bad_idx, nbad, mem, stream)
                   : cfsec_ec_reconstruct(h, v.data(), n, bad_idx, nbad, mem, stream);
}

int cfsec_ec_encode_batch_contig(cfsec_ec* h, uint8_t* base, size_t shard_size, size_t stride, size_t stripe_stride,
                                 int n, int nstripes, int mem, int* status, uint32_t* crcs) {
  if (!h || nstripes < 0 || n <= 0 || (nstripes > 0 && (!base || !status))) return CFSEC_ERR_INVALID_ARG;
  if (nstripes > 1 && stripe_stride < stride * (size_t)n) return CFSEC_ERR_INVALID_ARG;  // stripes overlap
  std::vector<cfsec_shard> all((size_t)nstripes * n), one;
  for (int s = 0; s < nstripes; ++s) {
    if (contig_shards(base + (size_t)s * stripe_stride, shard_size, stride, n, nullptr, 0, &one) != CFSEC_OK)
      return CFSEC_ERR_INVALID_ARG;
    std::copy(one.begin(), one.end(), all.begin() + (size_t)s * n);
  }
  return crcs ? cfsec_ec_encode_batch_crc(h, all.data(), n, nstripes, mem, status, crcs)
              : cfsec_ec_encode_batch(h, all.data(), n, nstripes, mem, status);
}

int cfsec_ec_reconstruct_batch_contig(cfsec_ec* h, uint8_t* base, const uint64_t* bid_off,
                                      const uint64_t* bid_shard_size, int n, int nbids, const int* bad_idx,
                                      const int* bad_off, int verify, int mem, int* status, uint32_t* crcs) {
  if (!h || nbids < 0 || n <= 0 || (nbids > 0 && (!base || !bid_off || !bid_shard_size || !status)))
    return CFSEC_ERR_INVALID_ARG;
  std::vector<cfsec_shard> all((size_t)nbids * n), one;
  for (int b = 0; b < nbids; ++b) {
    const size_t S = (size_t)bid_shard_size[b];
    if (S == 0) {  // a zero-size bid: every shard empty (the reference loop skips those, :730-733)
      for (int i = 0; i < n; ++i) all[(size_t)b * n + i] = cfsec_shard{base + bid_off[b], 0, 0};
      continue;
    }
    if (contig_shards(base + bid_off[b], S, S, n, nullptr, 0, &one) != CFSEC_OK) return CFSEC_ERR_INVALID_ARG;
    std::copy(one.begin(), one.end(), all.begin() + (size_t)b * n);
  }
  return crcs ? cfsec_ec_reconstruct_batch_crc(h, all.data(), n, nbids, bad_idx, bad_off, verify, mem, status, crcs)
              : cfsec_ec_reconstruct_batch(h, all.data(), n, nbids, bad_idx, bad_off, verify, mem, status);
}
