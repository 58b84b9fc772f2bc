// engine.cpp -- RSEngine / ECEncoder / LrcEncoder host logic (see engine.hpp).
#include <atomic>
#include <chrono>
#include <thread>

#include "engine.hpp"

#include <algorithm>
#include <cstring>
#include <map>
#include <shared_mutex>
#include <unordered_map>

namespace cfsec {

namespace {
thread_local std::string t_last_error;
constexpr size_t kSlotAlign = 256;  // staging rows start on 256-B boundaries

size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// KRS/reedsolomon.go:1314-1339 checkShards / shardSize.
Status check_shards(const cfsec_shard* shards, int n, bool nilok, size_t* size) {
  size_t s = 0;
  for (int i = 0; i < n; ++i)
    if (shards[i].len != 0) {
      s = shards[i].len;
      break;
    }
  if (s == 0) return CFSEC_ERR_SHARD_NO_DATA;
  for (int i = 0; i < n; ++i)
    if (shards[i].len != s && (shards[i].len != 0 || !nilok)) return CFSEC_ERR_SHARD_SIZE;
  *size = s;
  return CFSEC_OK;
}

size_t first_size(const cfsec_shard* shards, int n) {
  for (int i = 0; i < n; ++i)
    if (shards[i].len != 0) return shards[i].len;
  return 0;
}

}  // namespace

// ec.fillFullShards (encoder.go:199-210).  Go allocates when cap is short; across the
// C ABI the caller must hand in buffers with enough capacity.
Status fill_full_shards(cfsec_shard* shards, int n) {
  const size_t s = first_size(shards, n);
  for (int i = 0; i < n; ++i)
    if (shards[i].len == 0) {
      if (s != 0 && (shards[i].cap < s || shards[i].data == nullptr)) {
        set_last_error("fillFullShards: shard " + std::to_string(i) + " has cap < shard size");
        return CFSEC_ERR_INVALID_ARG;
      }
      shards[i].len = s;
    }
  return CFSEC_OK;
}

// ec.initBadShards (encoder.go:182-188).
Status init_bad_shards(cfsec_shard* shards, int n, const std::vector<int>& bad) {
  for (int i : bad) {
    if (i < 0 || i >= n) {
      set_last_error("bad shard index out of range");
      return CFSEC_ERR_INVALID_ARG;
    }
    if (shards[i].data != nullptr && shards[i].len != 0 && shards[i].cap > 0) shards[i].len = 0;
  }
  return CFSEC_OK;
}

namespace {

// codemode.Tactic.IsValid (codemode.go:267-271).
bool tactic_valid(const cfsec_tactic& t) {
  return t.n > 0 && t.m > 0 && t.l >= 0 && t.az_count > 0 && t.put_quorum > 0 &&
         t.get_quorum >= 0 && t.min_shard_size >= 0 && t.n % t.az_count == 0 &&
         t.m % t.az_count == 0 && t.l % t.az_count == 0;
}

// codemode.Tactic.GetECLayoutByAZ (codemode.go:274-291).
std::vector<std::vector<int>> layout_by_az(const cfsec_tactic& t) {
  std::vector<std::vector<int>> az(t.az_count);
  const int n = t.n / t.az_count, m = t.m / t.az_count, l = t.l / t.az_count;
  for (int idx = 0; idx < t.az_count; ++idx) {
    for (int i = 0; i < n; ++i) az[idx].push_back(idx * n + i);
    for (int i = 0; i < m; ++i) az[idx].push_back(t.n + idx * m + i);
    for (int i = 0; i < l; ++i) az[idx].push_back(t.n + t.m + idx * l + i);
  }
  return az;
}
}  // namespace

void set_last_error(const std::string& msg) { t_last_error = msg; }
const char* last_error_cstr() { return t_last_error.c_str(); }

Status hip_status(hipError_t e, const char* what) {
  if (e == hipSuccess) return CFSEC_OK;
  set_last_error(std::string(what) + ": " + hipGetErrorString(e));
  return CFSEC_ERR_DEVICE;
}

// ---------------------------------------------------------------- devices

DeviceGuard::DeviceGuard(int device) {
  if (hipGetDevice(&prev_) != hipSuccess) return;
  if (prev_ != device && hipSetDevice(device) != hipSuccess) return;
  ok_ = true;
}
DeviceGuard::~DeviceGuard() {
  if (ok_) {
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && cur != prev_) (void)hipSetDevice(prev_);
  }
}

DeviceContext* DeviceContext::get(int device, int slot) {
  static std::mutex mu;
  static std::map<std::pair<int, int>, std::unique_ptr<DeviceContext>> ctxs;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count || slot < 0) return nullptr;
  std::lock_guard<std::mutex> l(mu);
  auto& p = ctxs[{device, slot}];
  if (!p) p.reset(new DeviceContext(device));
  return p.get();
}

Status DeviceContext::acquire(size_t bytes, size_t nflags, Workspace** out, size_t nbflags, size_t ncrc) {
  Workspace* ws = nullptr;
  bool wait = false;
  {
    std::lock_guard<std::mutex> l(mu_);
    // a workspace an asynchronous call returned is free once its stream has passed the call
    const auto ready = [](Workspace* w) {
      if (!w->pending) return true;
      const hipError_t q = hipEventQuery(w->done);
      if (q == hipErrorNotReady) return false;
      (void)hipGetLastError();
      w->pending = false;
      return true;
    };
    // best fit among the free workspaces
    auto best = free_.end();
    for (auto it = free_.begin(); it != free_.end(); ++it)
      if ((*it)->cap >= bytes && (*it)->nflags >= nflags && (*it)->nbflags >= nbflags && (*it)->ncrc >= ncrc &&
          (best == free_.end() || (*it)->cap < (*best)->cap) && ready(*it))
        best = it;
    if (best == free_.end())
      for (auto it = free_.begin(); it != free_.end() && best == free_.end(); ++it)
        if (ready(*it)) best = it;
    if (best != free_.end()) {
      ws = *best;
      free_.erase(best);
    } else if (all_.size() >= kMaxWorkspaces && !free_.empty()) {
      // every free workspace is still pending on an asynchronous call's stream: wait for the
      // oldest one instead of growing without bound (each holds streams, events, pinned words)
      ws = free_.front();
      free_.erase(free_.begin());
      wait = true;
    } else {
      all_.emplace_back(new Workspace());
      ws = all_.back().get();
    }
  }
  if (wait) {
    if (hipEventSynchronize(ws->done) != hipSuccess) {
      (void)hipGetLastError();
      DeviceGuard dg(device_);
      (void)hipDeviceSynchronize();
    }
    ws->pending = false;
  }
  DeviceGuard g(device_);
  if (!g.ok()) {
    release(ws);
    return hip_status(hipErrorInvalidDevice, "hipSetDevice");
  }
  Status st = CFSEC_OK;
  // Non-blocking streams: work on them does not wait for (or hold up) the legacy default stream,
  // so concurrent callers overlap.  A device-memory call without a caller stream orders itself
  // after the default stream explicitly (order_after_default).
  if (!ws->stream) st = hip_status(hipStreamCreateWithFlags(&ws->stream, hipStreamNonBlocking), "hipStreamCreate");
  if (st == CFSEC_OK && !ws->stream2)
    st = hip_status(hipStreamCreateWithFlags(&ws->stream2, hipStreamNonBlocking), "hipStreamCreate");
  if (st == CFSEC_OK && !ws->ev)
    st = hip_status(hipEventCreateWithFlags(&ws->ev, hipEventDisableTiming), "hipEventCreate");
  if (st == CFSEC_OK && !ws->ev_in)
    st = hip_status(hipEventCreateWithFlags(&ws->ev_in, hipEventDisableTiming), "hipEventCreate");
  if (st == CFSEC_OK && ws->cap < bytes) {
    if (ws->dbuf) (void)hipFree(ws->dbuf);
    ws->dbuf = nullptr;
    ws->cap = 0;
    st = hip_status(hipMalloc(reinterpret_cast<void**>(&ws->dbuf), bytes), "hipMalloc(staging)");
    if (st == CFSEC_OK) ws->cap = bytes;
  }
  if (st == CFSEC_OK && ws->nflags < nflags) {
    const size_t nf = std::max<size_t>(nflags, 64);
    if (ws->dflags) (void)hipFree(ws->dflags);
    if (ws->hflags) (void)hipHostFree(ws->hflags);
    ws->dflags = nullptr;
    ws->hflags = nullptr;
    ws->hflags_dev = nullptr;
    ws->nflags = 0;
    st = hip_status(hipMalloc(reinterpret_cast<void**>(&ws->dflags), nf * 4), "hipMalloc(flags)");
    if (st == CFSEC_OK)
      st = hip_status(hipHostMalloc(reinterpret_cast<void**>(&ws->hflags), nf * 4,
                                    hipHostMallocMapped | hipHostMallocCoherent),
                      "hipHostMalloc(flags)");
    if (st == CFSEC_OK)
      st = hip_status(hipHostGetDevicePointer(reinterpret_cast<void**>(&ws->hflags_dev), ws->hflags, 0),
                      "hipHostGetDevicePointer(flags)");
    if (st == CFSEC_OK) ws->nflags = nf;
  }
  if (st == CFSEC_OK && ws->nbflags < nbflags) {
    const size_t nf = std::max<size_t>(nbflags, 256);
    if (ws->bflags) (void)hipFree(ws->bflags);
    ws->bflags = nullptr;
    ws->nbflags = 0;
    ws->bflags_clean = false;
    st = hip_status(hipMalloc(reinterpret_cast<void**>(&ws->bflags), nf * 4), "hipMalloc(batch flags)");
    if (st == CFSEC_OK) ws->nbflags = nf;
  }
  if (st == CFSEC_OK && ws->bflags && !ws->bflags_clean) {
    // once per allocation (or after a failed call): the gather kernel keeps them zero afterwards
    st = hip_status(hipMemset(ws->bflags, 0, ws->nbflags * 4), "hipMemset(batch flags)");
    if (st == CFSEC_OK) ws->bflags_clean = true;
  }
  if (st == CFSEC_OK && ws->ncrc < ncrc) {
    const size_t nc = std::max<size_t>(ncrc, 256);
    if (ws->dcrc) (void)hipFree(ws->dcrc);
    if (ws->hcrc) (void)hipHostFree(ws->hcrc);
    ws->dcrc = nullptr;
    ws->hcrc = nullptr;
    ws->ncrc = 0;
    st = hip_status(hipMalloc(reinterpret_cast<void**>(&ws->dcrc), nc * 4), "hipMalloc(crc words)");
    if (st == CFSEC_OK)
      st = hip_status(hipHostMalloc(reinterpret_cast<void**>(&ws->hcrc), nc * 4, hipHostMallocCoherent),
                      "hipHostMalloc(crc words)");
    if (st == CFSEC_OK) ws->ncrc = nc;
  }
  if (st == CFSEC_OK && !ws->done)
    st = hip_status(hipEventCreateWithFlags(&ws->done, hipEventDisableTiming), "hipEventCreate");
  if (st != CFSEC_OK) {
    release(ws);
    return st;
  }
  *out = ws;
  return CFSEC_OK;
}

Status DeviceContext::order_after_default(Workspace* ws) {
  // Nothing queued on the legacy null stream is still pending (the common case: a caller that does
  // not use it, e.g. the Go shim on HBM shards): no ordering to add.  Work another thread queues
  // there after this query is concurrent with this call, not before it.  Saves the event record +
  // cross-stream wait, ~6 us of host time and ~3 us of GPU-side dependency per synchronous call
  // (tools/seg_latency.hip: 24-25 -> 13-14 us per NULL-stream ReconstructData of a 64 KiB segment).
  const hipError_t q = hipStreamQuery(nullptr);
  if (q == hipSuccess) return CFSEC_OK;
  if (q != hipErrorNotReady) (void)hipGetLastError();
  // An event recorded on the legacy null stream completes after everything queued before it on
  // that stream and on every blocking stream of the device.
  Status st = hip_status(hipEventRecord(ws->ev_in, nullptr), "hipEventRecord(null stream)");
  if (st == CFSEC_OK) st = hip_status(hipStreamWaitEvent(ws->stream, ws->ev_in, 0), "hipStreamWaitEvent");
  return st;
}

void DeviceContext::release(Workspace* ws) {
  std::lock_guard<std::mutex> l(mu_);
  free_.push_back(ws);
}

// CFSEC_SYNC_POLL=0 (or cfsec_set_sync_poll(0)): hipStreamSynchronize always (A/B, tests)
std::atomic<int>& sync_poll_mode() {
  static std::atomic<int> mode{[] {
    const char* v = std::getenv("CFSEC_SYNC_POLL");
    return (v && v[0] == '0') ? 0 : 1;
  }()};
  return mode;
}

Status DeviceContext::finish(Workspace* ws, hipStream_t stream) {
  const auto blocking = [&] { return hip_status(hipStreamSynchronize(stream), "hipStreamSynchronize"); };
  if (!sync_poll_mode().load(std::memory_order_relaxed)) return blocking();
  if (!ws->hmark) {
    void* h = nullptr;
    if (hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
      (void)hipGetLastError();
      return blocking();
    }
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
      (void)hipGetLastError();
      (void)hipHostFree(h);
      return blocking();
    }
    ws->hmark = static_cast<uint32_t*>(h);
    ws->dmark = static_cast<uint32_t*>(d);
    __atomic_store_n(ws->hmark, 0u, __ATOMIC_RELEASE);
    ws->seq = 0;
  }
  const uint32_t seq = ++ws->seq;
  if (hipStreamWriteValue32(stream, ws->dmark, seq, 0) != hipSuccess) {
    (void)hipGetLastError();
    return blocking();
  }
  // The marker is written after the call's kernels and copies on this stream; the words the caller
  // reads next (hflags, hcrc) are coherent host memory, so they are visible once the marker is.
  // Busy-polling for the first kSpinBusyUs (a call's own latency), yielding the core after that.
  const auto t0 = std::chrono::steady_clock::now();
  bool busy = true;
  for (uint32_t spin = 0;; ++spin) {
    if (__atomic_load_n(ws->hmark, __ATOMIC_ACQUIRE) == seq) return CFSEC_OK;
    if (busy) __builtin_ia32_pause();
    else std::this_thread::yield();
    if ((spin & 255u) == 255u) {
      const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
      if (us > kSpinLimitUs) return blocking();
      busy = us < kSpinBusyUs;
    }
  }
}

void DeviceContext::release_after(Workspace* ws, hipStream_t stream) {
  // if the record fails the stream's work is unknown: wait for the device before reuse
  if (hipEventRecord(ws->done, stream) != hipSuccess) {
    (void)hipGetLastError();
    (void)hipDeviceSynchronize();
    ws->pending = false;
  } else {
    ws->pending = true;
  }
  release(ws);
}

// ---------------------------------------------------------------- inversion cache

bool InversionCache::get(const std::vector<int>& invalid, Matrix* out) const {
  std::shared_lock<std::shared_mutex> l(mu_);
  auto it = map_.find(invalid);
  if (it == map_.end()) return false;
  *out = it->second;
  return true;
}

void InversionCache::put(const std::vector<int>& invalid, const Matrix& m) {
  std::unique_lock<std::shared_mutex> l(mu_);
  map_.emplace(invalid, m);
}

// ---------------------------------------------------------------- RSEngine

Status RSEngine::create(int k, int m, int device, std::unique_ptr<RSEngine>* out) {
  // KRS/reedsolomon.go:413-447.  More than 256 shards switches the reference to its
  // leopard GF(2^16) codec, which CubeFS never reaches (max 38 shards).
  if (k + m > 256) return CFSEC_ERR_NOT_SUPPORTED;
  if (k <= 0 || m < 0) return CFSEC_ERR_INV_SHARD_NUM;
  std::unique_ptr<RSEngine> e(new RSEngine());
  e->k_ = k;
  e->m_ = m;
  if (m > 0) {
    if (!build_matrix(k, k + m, e->mat_)) return CFSEC_ERR_SINGULAR;
  } else {
    e->mat_ = Matrix(k, k);
    for (int i = 0; i < k; ++i) e->mat_.at(i, i) = 1;
  }
  e->parity_ = Matrix(m, k);
  for (int r = 0; r < m; ++r)
    for (int c = 0; c < k; ++c) e->parity_.at(r, c) = e->mat_.at(k + r, c);
  if (device < 0) {
    int cur = 0;
    int count = 0;
    if (hipGetDeviceCount(&count) == hipSuccess && count > 0 && hipGetDevice(&cur) == hipSuccess)
      device = cur;
  }
  // A missing device is reported by the first call that needs it (CFSEC_ERR_DEVICE); the
  // host-only methods (matrix, Split, Join) work without one.
  e->ctx_ = device >= 0 ? DeviceContext::get(device) : nullptr;
  if (e->ctx_) e->devs_.push_back(e->ctx_);
  *out = std::move(e);
  return CFSEC_OK;
}

static Status matvec_with_crc(const MatVecJob& job, uint8_t* const* ptrs, int total, const std::vector<int>& slot,
                              size_t S, uint32_t* crcs, hipStream_t stream);

// The device address of page-locked host memory (hipHostMalloc / cfsec_host_alloc); false for
// pageable memory.
namespace {
struct HostRange {
  size_t size;
  uint8_t* dev;  // device address of the base
};
struct HostRanges {
  std::shared_mutex mu;
  std::map<uintptr_t, HostRange> by_base;
};
HostRanges& host_ranges() {
  static HostRanges r;
  return r;
}
}  // namespace

void host_range_add(void* base, size_t size) {
  hipPointerAttribute_t attr;
  if (!base || hipPointerGetAttributes(&attr, base) != hipSuccess || !attr.devicePointer) {
    (void)hipGetLastError();
    return;
  }
  HostRanges& r = host_ranges();
  std::unique_lock<std::shared_mutex> lk(r.mu);
  r.by_base[(uintptr_t)base] = HostRange{size, static_cast<uint8_t*>(attr.devicePointer)};
}

void host_range_remove(void* base) {
  HostRanges& r = host_ranges();
  std::unique_lock<std::shared_mutex> lk(r.mu);
  r.by_base.erase((uintptr_t)base);
}

// Page-locked staging for small pageable host calls (RSEngine::run): a free list of cfsec-owned
// hipHostMalloc blocks (registered in the host-range registry, so the zero-copy path takes them),
// one per concurrent call, kept for reuse.
namespace {
struct PinnedStages {
  std::mutex mu;
  std::vector<std::pair<uint8_t*, size_t>> free;
};
PinnedStages& pinned_stages() {
  static PinnedStages p;
  return p;
}
}  // namespace

static std::pair<uint8_t*, size_t> pinned_stage_take(size_t bytes) {
  PinnedStages& p = pinned_stages();
  {
    std::lock_guard<std::mutex> lk(p.mu);
    for (size_t i = 0; i < p.free.size(); ++i)
      if (p.free[i].second >= bytes) {
        const auto b = p.free[i];
        p.free.erase(p.free.begin() + (long)i);
        return b;
      }
  }
  const size_t cap = std::max<size_t>(bytes, (size_t)256 << 10);
  void* h = nullptr;
  if (hipHostMalloc(&h, cap, hipHostMallocPortable) != hipSuccess) {
    (void)hipGetLastError();
    return {nullptr, 0};
  }
  host_range_add(h, cap);
  return {static_cast<uint8_t*>(h), cap};
}

static void pinned_stage_give(std::pair<uint8_t*, size_t> b) {
  if (!b.first) return;
  PinnedStages& p = pinned_stages();
  std::lock_guard<std::mutex> lk(p.mu);
  p.free.push_back(b);
}

bool device_alias(uint8_t* p, uint8_t** dptr) {
  {
    HostRanges& r = host_ranges();
    std::shared_lock<std::shared_mutex> lk(r.mu);
    if (!r.by_base.empty()) {
      auto it = r.by_base.upper_bound((uintptr_t)p);
      if (it != r.by_base.begin()) {
        --it;
        const uintptr_t off = (uintptr_t)p - it->first;
        if (off < it->second.size) {
          *dptr = it->second.dev + off;
          return true;
        }
      }
    }
  }
  hipPointerAttribute_t attr;
  if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  if (attr.type != hipMemoryTypeHost || !attr.devicePointer) return false;
  const uint8_t* hbase = static_cast<const uint8_t*>(attr.hostPointer);
  *dptr = static_cast<uint8_t*>(attr.devicePointer) + (hbase ? p - hbase : 0);
  return true;
}

Status RSEngine::run(const Matrix& rows, const std::vector<cfsec_shard*>& ins,
                     const std::vector<cfsec_shard*>& outs, size_t S, int mem, hipStream_t stream,
                     MatVecMode mode, bool* ok) {
  if (ok) *ok = true;
  if (outs.empty() || S == 0) return CFSEC_OK;
  if (!ctx_) {
    set_last_error("no HIP device available to the cfsec engine");
    return CFSEC_ERR_DEVICE;
  }
  if (mem != CFSEC_MEM_HOST && mem != CFSEC_MEM_DEVICE) return CFSEC_ERR_INVALID_ARG;
  for (auto* s : ins)
    if (!s->data) return CFSEC_ERR_INVALID_ARG;
  for (auto* s : outs)
    if (!s->data) return CFSEC_ERR_INVALID_ARG;
  const int nin = (int)ins.size(), nout = (int)outs.size();
  if (rows.rows != nout || rows.cols != nin) return CFSEC_ERR_INVALID_ARG;

  DeviceGuard g(ctx_->device());
  if (!g.ok()) return hip_status(hipErrorInvalidDevice, "hipSetDevice");

  const bool verify = mode == MatVecMode::kVerify;
  const bool host = mem == CFSEC_MEM_HOST;
  const size_t slot = align_up(S, kSlotAlign);
  // Verify with more inputs than one launch carries: compute into staging, then compare.
  const bool two_step_verify = verify && nin > 32;
  if (host) {
    // Page-locked buffers (cfsec_host_alloc) are device-addressable: the kernel reads and writes
    // them over PCIe with no staging copies (tools/bench_host.py: 50.7 GB/s of data for EC12P4
    // encode vs 32.4 through the staged pipeline and 26.7 from pageable memory).
    std::vector<cfsec_shard> zin(nin), zout(nout);
    bool zero_copy = true;
    for (int i = 0; i < nin && zero_copy; ++i) {
      zin[i] = *ins[i];
      zero_copy = device_alias(ins[i]->data, &zin[i].data);
    }
    for (int r = 0; r < nout && zero_copy; ++r) {
      zout[r] = *outs[r];
      zero_copy = device_alias(outs[r]->data, &zout[r].data);
    }
    if (zero_copy) {
      std::vector<cfsec_shard*> pin(nin), pout(nout);
      for (int i = 0; i < nin; ++i) pin[i] = &zin[i];
      for (int r = 0; r < nout; ++r) pout[r] = &zout[r];
      return run(rows, pin, pout, S, CFSEC_MEM_DEVICE, nullptr, mode, ok);
    }
    // Small pageable calls (a degraded range read's segments): the rows copied on the CPU into
    // page-locked staging and coded there in place, instead of HIP's staged copies of pageable memory
    // (~130 us per call whatever the size up to 64 KiB, profiles/r06/bench_s1).
    const size_t total = S * (size_t)(nin + nout);
    if (!two_step_verify && total <= kSmallPageable) {
      std::pair<uint8_t*, size_t> stage = pinned_stage_take(total);
      if (stage.first) {
        std::vector<cfsec_shard> sin(nin), sout(nout);
        std::vector<cfsec_shard*> pin(nin), pout(nout);
        for (int i = 0; i < nin; ++i) {
          std::memcpy(stage.first + S * i, ins[i]->data, S);
          sin[i] = cfsec_shard{stage.first + S * i, S, S};
          pin[i] = &sin[i];
        }
        for (int r = 0; r < nout; ++r) {
          uint8_t* d = stage.first + S * (nin + r);
          if (mode != MatVecMode::kStore) std::memcpy(d, outs[r]->data, S);
          sout[r] = cfsec_shard{d, S, S};
          pout[r] = &sout[r];
        }
        Status st = run(rows, pin, pout, S, CFSEC_MEM_HOST, nullptr, mode, ok);
        if (st == CFSEC_OK && mode != MatVecMode::kVerify)
          for (int r = 0; r < nout; ++r) std::memcpy(outs[r]->data, sout[r].data, S);
        pinned_stage_give(stage);
        return st;
      }
    }
    if (!two_step_verify) return run_host(rows, ins, outs, S, mode, ok);
  }
  size_t staging = host ? slot * size_t(nin + nout) : 0;
  if (two_step_verify) staging += slot * size_t(nout);

  DeviceContext::Workspace* ws = nullptr;
  std::unique_ptr<HostTimer> tm(new HostTimer("  run: acquire"));
  Status st = ctx_->acquire(staging, 1, &ws);
  if (st != CFSEC_OK) return st;
  hipStream_t s = (host || !stream) ? ws->stream : stream;
  if (!host && !stream) st = ctx_->order_after_default(ws);
  tm.reset(new HostTimer("  run: copies + launch"));

  std::vector<const uint8_t*> din(nin);
  std::vector<uint8_t*> dout(nout);
  for (int i = 0; i < nin; ++i) {
    if (host) {
      din[i] = ws->dbuf + slot * i;
      if (st == CFSEC_OK)
        st = hip_status(hipMemcpyAsync(const_cast<uint8_t*>(din[i]), ins[i]->data, S, hipMemcpyHostToDevice, s),
                        "hipMemcpyAsync H2D");
    } else {
      din[i] = ins[i]->data;
    }
  }
  for (int r = 0; r < nout; ++r) {
    if (host) {
      dout[r] = ws->dbuf + slot * (nin + r);
      if (st == CFSEC_OK && mode != MatVecMode::kStore)
        st = hip_status(hipMemcpyAsync(dout[r], outs[r]->data, S, hipMemcpyHostToDevice, s),
                        "hipMemcpyAsync H2D");
    } else {
      dout[r] = outs[r]->data;
    }
  }
  if (st == CFSEC_OK && verify) st = hip_status(hipMemsetAsync(ws->dflags, 0, 4, s), "hipMemsetAsync");
  if (st == CFSEC_OK) {
    MatVecJob job;
    job.k = nin;
    job.m = nout;
    job.coef = rows.v.data();
    job.len = S;
    job.nstripes = 1;
    job.in = din.data();
    job.flags = ws->dflags;
    if (!two_step_verify) {
      job.out = dout.data();
      job.mode = mode;
      st = hip_status(launch_matvec(job, s), "launch_matvec");
    } else {
      uint8_t* tmp0 = ws->dbuf + (host ? slot * size_t(nin + nout) : 0);
      std::vector<uint8_t*> tmp(nout);
      for (int r = 0; r < nout; ++r) tmp[r] = tmp0 + slot * r;
      job.out = tmp.data();
      job.mode = MatVecMode::kStore;
      st = hip_status(launch_matvec(job, s), "launch_matvec");
      if (st == CFSEC_OK) {
        Matrix ident(nout, nout);
        for (int r = 0; r < nout; ++r) ident.at(r, r) = 1;
        std::vector<const uint8_t*> tin(tmp.begin(), tmp.end());
        MatVecJob cmp = job;
        cmp.k = nout;
        cmp.coef = ident.v.data();
        cmp.in = tin.data();
        cmp.out = dout.data();
        cmp.mode = MatVecMode::kVerify;
        st = hip_status(launch_matvec(cmp, s), "launch_matvec(verify)");
      }
    }
  }
  if (st == CFSEC_OK && verify)
    st = hip_status(hipMemcpyAsync(ws->hflags, ws->dflags, 4, hipMemcpyDeviceToHost, s), "hipMemcpyAsync D2H");
  if (st == CFSEC_OK && host && !verify)
    for (int r = 0; r < nout && st == CFSEC_OK; ++r)
      st = hip_status(hipMemcpyAsync(outs[r]->data, dout[r], S, hipMemcpyDeviceToHost, s), "hipMemcpyAsync D2H");
  tm.reset(new HostTimer("  run: finish"));
  const Status sync = ctx_->finish(ws, s);
  tm.reset();
  if (st == CFSEC_OK) st = sync;
  if (st == CFSEC_OK && verify && ok) *ok = ws->hflags[0] == 0;
  ctx_->release(ws);
  return st;
}

namespace {
// Rows of a host call that sit at one stride from each other (ec.Buffer carves its shards at
// stride S from one allocation, common/ec/buf.go:83-84): one 2-D copy moves all of them.
int64_t host_row_stride(const std::vector<cfsec_shard*>& rows) {
  if (rows.size() < 2) return 0;
  const int64_t st = (int64_t)(uintptr_t)rows[1]->data - (int64_t)(uintptr_t)rows[0]->data;
  if (st <= 0) return 0;
  for (size_t i = 2; i < rows.size(); ++i)
    if ((int64_t)(uintptr_t)rows[i]->data - (int64_t)(uintptr_t)rows[0]->data != st * (int64_t)i) return 0;
  return st;
}

hipError_t copy_rows(const std::vector<cfsec_shard*>& rows, int64_t hstride, size_t off, size_t len,
                     uint8_t* dev, size_t dpitch, bool h2d, hipStream_t s) {
  if (rows.empty()) return hipSuccess;
  if (hstride > 0 && (size_t)hstride >= len) {
    return h2d ? hipMemcpy2DAsync(dev, dpitch, rows[0]->data + off, (size_t)hstride, len, rows.size(),
                                  hipMemcpyHostToDevice, s)
               : hipMemcpy2DAsync(rows[0]->data + off, (size_t)hstride, dev, dpitch, len, rows.size(),
                                  hipMemcpyDeviceToHost, s);
  }
  for (size_t i = 0; i < rows.size(); ++i) {
    hipError_t e = h2d ? hipMemcpyAsync(dev + i * dpitch, rows[i]->data + off, len, hipMemcpyHostToDevice, s)
                       : hipMemcpyAsync(rows[i]->data + off, dev + i * dpitch, len, hipMemcpyDeviceToHost, s);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}
}  // namespace

// Host-memory call: the shard columns go through HBM in chunks of kHostChunk bytes per row,
// alternating over two streams, so chunk j+1's host->device copies, chunk j's kernel and chunk
// j-1's device->host copies overlap (the copy engines of each direction and the CUs run
// concurrently; PCIe Gen5 x16 is the bound).  Buffers from cfsec_host_alloc (pinned) DMA
// directly; pageable ones go through HIP's staging.  Chunks of one stream reuse its staging
// region, which that stream's order makes safe.
Status RSEngine::run_host(const Matrix& rows, const std::vector<cfsec_shard*>& ins,
                          const std::vector<cfsec_shard*>& outs, size_t S, MatVecMode mode, bool* ok) {
  const int nin = (int)ins.size(), nout = (int)outs.size();
  const bool verify = mode == MatVecMode::kVerify;
  const size_t chunk = std::min(align_up(S, kSlotAlign), kHostChunk);
  const size_t nchunks = (S + chunk - 1) / chunk;
  const int nlanes = nchunks > 1 ? 2 : 1;
  const size_t per_lane = chunk * size_t(nin + nout);
  DeviceContext::Workspace* ws = nullptr;
  Status st = ctx_->acquire(per_lane * nlanes, 1, &ws);
  if (st != CFSEC_OK) return st;
  hipStream_t lane[2] = {ws->stream, ws->stream2};
  const int64_t in_stride = host_row_stride(ins), out_stride = host_row_stride(outs);
  if (verify) {
    st = hip_status(hipMemsetAsync(ws->dflags, 0, 4, lane[0]), "hipMemsetAsync");
    if (st == CFSEC_OK && nlanes > 1) st = hip_status(hipEventRecord(ws->ev, lane[0]), "hipEventRecord");
    if (st == CFSEC_OK && nlanes > 1) st = hip_status(hipStreamWaitEvent(lane[1], ws->ev, 0), "hipStreamWaitEvent");
  }
  std::vector<const uint8_t*> din(nin);
  std::vector<uint8_t*> dout(nout);
  for (size_t j = 0; j < nchunks && st == CFSEC_OK; ++j) {
    const int l = (int)(j % nlanes);
    hipStream_t s = lane[l];
    uint8_t* base = ws->dbuf + per_lane * l;
    const size_t off = j * chunk, len = std::min(chunk, S - off);
    for (int i = 0; i < nin; ++i) din[i] = base + chunk * i;
    for (int r = 0; r < nout; ++r) dout[r] = base + chunk * (nin + r);
    st = hip_status(copy_rows(ins, in_stride, off, len, base, chunk, true, s), "hipMemcpyAsync H2D");
    if (st == CFSEC_OK && verify)
      st = hip_status(copy_rows(outs, out_stride, off, len, base + chunk * nin, chunk, true, s), "hipMemcpyAsync H2D");
    if (st == CFSEC_OK) {
      MatVecJob job;
      job.k = nin;
      job.m = nout;
      job.coef = rows.v.data();
      job.len = len;
      job.nstripes = 1;
      job.in = din.data();
      job.out = dout.data();
      job.mode = mode;
      job.flags = ws->dflags;
      st = hip_status(launch_matvec(job, s), "launch_matvec");
    }
    if (st == CFSEC_OK && !verify)
      st = hip_status(copy_rows(outs, out_stride, off, len, base + chunk * nin, chunk, false, s), "hipMemcpyAsync D2H");
  }
  if (st == CFSEC_OK && verify && nlanes > 1) {
    st = hip_status(hipEventRecord(ws->ev, lane[1]), "hipEventRecord");
    if (st == CFSEC_OK) st = hip_status(hipStreamWaitEvent(lane[0], ws->ev, 0), "hipStreamWaitEvent");
  }
  if (st == CFSEC_OK && verify)
    st = hip_status(hipMemcpyAsync(ws->hflags, ws->dflags, 4, hipMemcpyDeviceToHost, lane[0]), "hipMemcpyAsync D2H");
  for (int l = 0; l < nlanes; ++l) {
    const Status sync = ctx_->finish(ws, lane[l]);
    if (st == CFSEC_OK) st = sync;
  }
  if (st == CFSEC_OK && verify && ok) *ok = ws->hflags[0] == 0;
  ctx_->release(ws);
  return st;
}

Status RSEngine::encode(cfsec_shard* shards, int n, int mem, hipStream_t stream) {
  if (!shards || n != total()) return CFSEC_ERR_TOO_FEW_SHARDS;
  size_t S = 0;
  Status st = check_shards(shards, n, false, &S);
  if (st != CFSEC_OK) return st;
  std::vector<cfsec_shard*> ins, outs;
  for (int i = 0; i < k_; ++i) ins.push_back(&shards[i]);
  for (int i = k_; i < n; ++i) outs.push_back(&shards[i]);
  return run(parity_, ins, outs, S, mem, stream, MatVecMode::kStore, nullptr);
}

Status RSEngine::encode_crc(cfsec_shard* shards, int n, int mem, hipStream_t stream, uint32_t* crcs) {
  if (!shards || n != total()) return CFSEC_ERR_TOO_FEW_SHARDS;
  if (!crcs) return CFSEC_ERR_INVALID_ARG;
  size_t S = 0;
  Status st = check_shards(shards, n, false, &S);
  if (st != CFSEC_OK) return st;
  if (!ctx_) {
    set_last_error("no HIP device available to the cfsec engine");
    return CFSEC_ERR_DEVICE;
  }
  if (mem != CFSEC_MEM_HOST && mem != CFSEC_MEM_DEVICE) return CFSEC_ERR_INVALID_ARG;
  for (int i = 0; i < n; ++i)
    if (!shards[i].data) return CFSEC_ERR_INVALID_ARG;
  DeviceGuard g(ctx_->device());
  if (!g.ok()) return hip_status(hipErrorInvalidDevice, "hipSetDevice");
  // device addresses of the shards: device memory as is, pinned host pages aliased (zero-copy),
  // pageable host memory staged whole through the workspace
  std::vector<uint8_t*> dptr(n);
  bool staged = false;
  if (mem == CFSEC_MEM_HOST)
    for (int i = 0; i < n && !staged; ++i) staged = !device_alias(shards[i].data, &dptr[i]);
  else
    for (int i = 0; i < n; ++i) dptr[i] = shards[i].data;
  const size_t slot = align_up(S, kSlotAlign);
  DeviceContext::Workspace* ws = nullptr;
  st = ctx_->acquire(staged ? slot * n : 0, (size_t)n, &ws);
  if (st != CFSEC_OK) return st;
  hipStream_t s = (mem == CFSEC_MEM_HOST || !stream) ? ws->stream : stream;
  if (!staged && !stream) st = ctx_->order_after_default(ws);
  if (staged)
    for (int i = 0; i < n; ++i) {
      dptr[i] = ws->dbuf + slot * i;
      if (i < k_ && st == CFSEC_OK)
        st = hip_status(hipMemcpyAsync(dptr[i], shards[i].data, S, hipMemcpyHostToDevice, s), "hipMemcpyAsync H2D");
    }
  if (st == CFSEC_OK && m_ > 0) {
    MatVecJob job;
    job.k = k_;
    job.m = m_;
    job.coef = parity_.v.data();
    job.len = S;
    job.nstripes = 1;
    std::vector<const uint8_t*> in(dptr.begin(), dptr.begin() + k_);
    job.in = in.data();
    job.out = dptr.data() + k_;
    std::vector<int> slots(n);
    for (int i = 0; i < n; ++i) slots[i] = i;
    st = matvec_with_crc(job, dptr.data(), n, slots, S, ws->dflags, s);
  } else if (st == CFSEC_OK) {
    st = hip_status(hipMemsetAsync(ws->dflags, 0, 4 * (size_t)n, s), "hipMemsetAsync");
    std::vector<const uint8_t*> p(dptr.begin(), dptr.end());
    if (st == CFSEC_OK)
      st = hip_status(launch_crc32_to(p.data(), S, n, ws->dflags, nullptr, crc32_shift_ones(S), s), "launch_crc32_to");
  }
  if (st == CFSEC_OK && staged)
    for (int r = k_; r < n && st == CFSEC_OK; ++r)
      st = hip_status(hipMemcpyAsync(shards[r].data, dptr[r], S, hipMemcpyDeviceToHost, s), "hipMemcpyAsync D2H");
  if (st == CFSEC_OK)
    st = hip_status(hipMemcpyAsync(ws->hflags, ws->dflags, 4 * (size_t)n, hipMemcpyDeviceToHost, s), "hipMemcpyAsync D2H");
  const Status sync = ctx_->finish(ws, s);
  if (st == CFSEC_OK) st = sync;
  if (st == CFSEC_OK) std::memcpy(crcs, ws->hflags, 4 * (size_t)n);
  ctx_->release(ws);
  return st;
}

Status RSEngine::verify(cfsec_shard* shards, int n, int mem, hipStream_t stream, bool* ok) {
  *ok = false;
  if (!shards || n != total()) return CFSEC_ERR_TOO_FEW_SHARDS;
  size_t S = 0;
  Status st = check_shards(shards, n, false, &S);
  if (st != CFSEC_OK) return st;
  std::vector<cfsec_shard*> ins, outs;
  for (int i = 0; i < k_; ++i) ins.push_back(&shards[i]);
  for (int i = k_; i < n; ++i) outs.push_back(&shards[i]);
  return run(parity_, ins, outs, S, mem, stream, MatVecMode::kVerify, ok);
}

Status RSEngine::plan_reconstruct(const std::vector<bool>& present, bool data_only, ReconPlan* plan) {
  // KRS/reedsolomon.go:1453-1501: first k present rows in index order; cache key is
  // the invalid rows met before the k-th valid one.
  std::vector<int> invalid;
  plan->valid.clear();
  for (int row = 0; row < total() && (int)plan->valid.size() < k_; ++row) {
    if (present[row]) plan->valid.push_back(row);
    else invalid.push_back(row);
  }
  if ((int)plan->valid.size() < k_) return CFSEC_ERR_TOO_FEW_SHARDS;
  Matrix dec;
  if (!tree_.get(invalid, &dec)) {
    Matrix sub(k_, k_);
    for (int r = 0; r < k_; ++r)
      for (int c = 0; c < k_; ++c) sub.at(r, c) = mat_.at(plan->valid[r], c);
    if (!mat_invert(sub, dec)) return CFSEC_ERR_SINGULAR;
    tree_.put(invalid, dec);
  }
  // Missing data rows: rows of inv(sub) (:1508-1524).  Missing parity rows: the
  // reference recomputes them from all data shards (:1537-1550); the same linear map
  // over the k survivors is parity_row x inv(sub), so one fused pass is bit-exact.
  plan->outputs.clear();
  std::vector<const uint8_t*> rowsrc;
  for (int i = 0; i < k_; ++i)
    if (!present[i]) plan->outputs.push_back(i);
  if (!data_only)
    for (int i = k_; i < total(); ++i)
      if (!present[i]) plan->outputs.push_back(i);
  plan->rows = Matrix((int)plan->outputs.size(), k_);
  const GF& gf = GF::get();
  for (size_t o = 0; o < plan->outputs.size(); ++o) {
    const int idx = plan->outputs[o];
    uint8_t* dst = plan->rows.row((int)o);
    if (idx < k_) {
      std::memcpy(dst, dec.row(idx), k_);
    } else {
      const uint8_t* p = parity_.row(idx - k_);
      for (int c = 0; c < k_; ++c) {
        uint8_t v = 0;
        for (int j = 0; j < k_; ++j) v ^= gf.mul(p[j], dec.at(j, c));
        dst[c] = v;
      }
    }
  }
  return CFSEC_OK;
}

Status RSEngine::reconstruct(cfsec_shard* shards, int n, bool data_only, int mem, hipStream_t stream) {
  if (!shards || n != total()) return CFSEC_ERR_TOO_FEW_SHARDS;
  size_t S = 0;
  Status st = check_shards(shards, n, true, &S);
  if (st != CFSEC_OK) return st;
  std::vector<bool> present(n);
  int npresent = 0, dpresent = 0;
  for (int i = 0; i < n; ++i) {
    present[i] = shards[i].len != 0;
    if (present[i]) {
      ++npresent;
      if (i < k_) ++dpresent;
    }
  }
  if (npresent == n || (data_only && dpresent == k_)) return CFSEC_OK;
  if (npresent < k_) return CFSEC_ERR_TOO_FEW_SHARDS;
  ReconPlan plan;
  {
    HostTimer tp("  reconstruct: plan");
    st = plan_reconstruct(present, data_only, &plan);
  }
  if (st != CFSEC_OK) return st;
  for (int idx : plan.outputs)
    if (!shards[idx].data || shards[idx].cap < S) {
      set_last_error("reconstruct: missing shard " + std::to_string(idx) + " has cap < shard size");
      return CFSEC_ERR_INVALID_ARG;
    }
  std::vector<cfsec_shard*> ins, outs;
  for (int v : plan.valid) ins.push_back(&shards[v]);
  for (int o : plan.outputs) outs.push_back(&shards[o]);
  for (auto* o : outs) o->len = S;  // KRS/reedsolomon.go:1514-1518: shards[i] = shards[i][0:S]
  return run(plan.rows, ins, outs, S, mem, stream, MatVecMode::kStore, nullptr);
}

Status RSEngine::split(uint8_t* data, size_t len, size_t cap, cfsec_shard* out, uint8_t* pad,
                       size_t pad_len, size_t* pad_needed) {
  // KRS/reedsolomon.go:1574-1632
  if (pad_needed) *pad_needed = 0;
  if (len == 0) return CFSEC_ERR_SHORT_DATA;
  if (!data || !out) return CFSEC_ERR_INVALID_ARG;
  if (cap < len) cap = len;
  const int tot = total();
  if (tot == 1) {
    out[0] = cfsec_shard{data, len, cap};
    return CFSEC_OK;
  }
  const size_t per = (len + k_ - 1) / k_;
  const size_t need_total = per * tot;
  size_t eff = len;
  if (cap > len) {
    eff = std::min(cap, need_total);
    std::memset(data + len, 0, eff - len);
  }
  const size_t full = std::min<size_t>(eff / per, tot);
  const size_t npad = tot - full;
  // the padding shards as AllocAligned(npad, per) lays them out (KRS/unsafe.go:17-41): a 64-byte
  // aligned start, each shard at a 64-byte rounded stride with that stride as its capacity
  const size_t each = (per + 63) / 64 * 64;
  if (pad_needed) *pad_needed = npad ? npad * each + 63 : 0;
  if (npad > 0 && (!pad || pad_len < npad * each + 63)) return CFSEC_ERR_INVALID_ARG;
  uint8_t* base = pad;
  if (npad > 0) {
    base = pad + ((64 - (reinterpret_cast<uintptr_t>(pad) & 63)) & 63);
    std::memset(base, 0, npad * each);
    // the partial data after the full shards, copied shard by shard (copy(padding[i], copyFrom))
    size_t from = per * full;
    for (size_t j = 0; j < npad && from < len; ++j) {
      const size_t c = std::min(per, len - from);
      std::memcpy(base + j * each, data + from, c);
      from += c;
    }
  }
  for (size_t i = 0; i < full; ++i) out[i] = cfsec_shard{data + i * per, per, per};
  for (size_t j = 0; j < npad; ++j) out[full + j] = cfsec_shard{base + j * each, per, each};
  return CFSEC_OK;
}

Status RSEngine::join(uint8_t* dst, size_t dst_len, const cfsec_shard* shards, int n, size_t out_size) {
  // KRS/reedsolomon.go:1646-1684
  if (n < k_) return CFSEC_ERR_TOO_FEW_SHARDS;
  size_t size = 0;
  for (int i = 0; i < k_; ++i) {
    if (shards[i].data == nullptr) return CFSEC_ERR_RECONSTRUCT_REQUIRED;
    size += shards[i].len;
    if (size >= out_size) break;
  }
  if (size < out_size) return CFSEC_ERR_SHORT_DATA;
  if (!dst || dst_len < out_size) return CFSEC_ERR_INVALID_ARG;
  size_t write = out_size;
  for (int i = 0; i < k_ && write > 0; ++i) {
    const size_t c = std::min(write, shards[i].len);
    std::memcpy(dst + (out_size - write), shards[i].data, c);
    write -= c;
  }
  return CFSEC_OK;
}

Status RSEngine::encode_batch(uint8_t* const* ptrs, size_t S, int nstripes, hipStream_t stream) {
  if (!ctx_) return CFSEC_ERR_DEVICE;
  if (!ptrs || nstripes < 0) return CFSEC_ERR_INVALID_ARG;
  if (m_ == 0 || nstripes == 0 || S == 0) return CFSEC_OK;
  std::vector<const uint8_t*> in(size_t(nstripes) * k_);
  std::vector<uint8_t*> out(size_t(nstripes) * m_);
  for (int s = 0; s < nstripes; ++s) {
    for (int c = 0; c < k_; ++c) in[size_t(s) * k_ + c] = ptrs[size_t(s) * total() + c];
    for (int r = 0; r < m_; ++r) out[size_t(s) * m_ + r] = ptrs[size_t(s) * total() + k_ + r];
  }
  DeviceGuard g(ctx_->device());
  if (!g.ok()) return hip_status(hipErrorInvalidDevice, "hipSetDevice");
  MatVecJob job;
  job.k = k_;
  job.m = m_;
  job.coef = parity_.v.data();
  job.len = S;
  job.nstripes = nstripes;
  job.in = in.data();
  job.out = out.data();
  return hip_status(launch_matvec(job, stream), "launch_matvec(encode_batch)");
}

Status RSEngine::matvec_batch(const uint8_t* coef, int rows, uint8_t* const* ptrs, size_t S, int nstripes,
                              hipStream_t stream) {
  if (!ctx_) return CFSEC_ERR_DEVICE;
  if (!coef || !ptrs || nstripes < 0 || rows < 0 || rows > 256) return CFSEC_ERR_INVALID_ARG;
  if (rows == 0 || nstripes == 0 || S == 0) return CFSEC_OK;
  const size_t w = (size_t)k_ + rows;
  std::vector<const uint8_t*> in(size_t(nstripes) * k_);
  std::vector<uint8_t*> out(size_t(nstripes) * rows);
  for (int s = 0; s < nstripes; ++s) {
    for (int c = 0; c < k_; ++c) in[size_t(s) * k_ + c] = ptrs[s * w + c];
    for (int r = 0; r < rows; ++r) out[size_t(s) * rows + r] = ptrs[s * w + k_ + r];
  }
  DeviceGuard g(ctx_->device());
  if (!g.ok()) return hip_status(hipErrorInvalidDevice, "hipSetDevice");
  MatVecJob job;
  job.k = k_;
  job.m = rows;
  job.coef = coef;
  job.len = S;
  job.nstripes = nstripes;
  job.in = in.data();
  job.out = out.data();
  return hip_status(launch_matvec(job, stream), "launch_matvec(matvec_batch)");
}

Status RSEngine::verify_batch(uint8_t* const* ptrs, size_t S, int nstripes, uint32_t* flags,
                              hipStream_t stream) {
  if (!ctx_) return CFSEC_ERR_DEVICE;
  if (!ptrs || !flags || nstripes < 0) return CFSEC_ERR_INVALID_ARG;
  if (m_ == 0 || nstripes == 0 || S == 0) return CFSEC_OK;
  if (k_ > 32) return CFSEC_ERR_NOT_SUPPORTED;
  std::vector<const uint8_t*> in(size_t(nstripes) * k_);
  std::vector<uint8_t*> out(size_t(nstripes) * m_);
  for (int s = 0; s < nstripes; ++s) {
    for (int c = 0; c < k_; ++c) in[size_t(s) * k_ + c] = ptrs[size_t(s) * total() + c];
    for (int r = 0; r < m_; ++r) out[size_t(s) * m_ + r] = ptrs[size_t(s) * total() + k_ + r];
  }
  DeviceGuard g(ctx_->device());
  if (!g.ok()) return hip_status(hipErrorInvalidDevice, "hipSetDevice");
  MatVecJob job;
  job.k = k_;
  job.m = m_;
  job.coef = parity_.v.data();
  job.len = S;
  job.nstripes = nstripes;
  job.in = in.data();
  job.out = out.data();
  job.mode = MatVecMode::kVerify;
  job.flags = flags;
  return hip_status(launch_matvec(job, stream), "launch_matvec(verify_batch)");
}

Status RSEngine::reconstruct_batch(uint8_t* const* ptrs, size_t S, int nstripes, const int* erased,
                                   int nerased, bool data_only, hipStream_t stream) {
  if (!ctx_) return CFSEC_ERR_DEVICE;
  if (!ptrs || nstripes < 0 || nerased < 0 || (nerased > 0 && !erased)) return CFSEC_ERR_INVALID_ARG;
  std::vector<bool> present(total(), true);
  for (int i = 0; i < nerased; ++i) {
    if (erased[i] < 0 || erased[i] >= total()) return CFSEC_ERR_INVALID_ARG;
    present[erased[i]] = false;
  }
  int np = 0, dp = 0;
  for (int i = 0; i < total(); ++i)
    if (present[i]) {
      ++np;
      if (i < k_) ++dp;
    }
  if (np == total() || (data_only && dp == k_) || nstripes == 0 || S == 0) return CFSEC_OK;
  if (np < k_) return CFSEC_ERR_TOO_FEW_SHARDS;
  ReconPlan plan;
  Status st = plan_reconstruct(present, data_only, &plan);
  if (st != CFSEC_OK) return st;
  const int nout = (int)plan.outputs.size();
  std::vector<const uint8_t*> in(size_t(nstripes) * k_);
  std::vector<uint8_t*> out(size_t(nstripes) * nout);
  for (int s = 0; s < nstripes; ++s) {
    for (int c = 0; c < k_; ++c) in[size_t(s) * k_ + c] = ptrs[size_t(s) * total() + plan.valid[c]];
    for (int r = 0; r < nout; ++r) out[size_t(s) * nout + r] = ptrs[size_t(s) * total() + plan.outputs[r]];
  }
  DeviceGuard g(ctx_->device());
  if (!g.ok()) return hip_status(hipErrorInvalidDevice, "hipSetDevice");
  MatVecJob job;
  job.k = k_;
  job.m = nout;
  job.coef = plan.rows.v.data();
  job.len = S;
  job.nstripes = nstripes;
  job.in = in.data();
  job.out = out.data();
  return hip_status(launch_matvec(job, stream), "launch_matvec(reconstruct_batch)");
}

// Product + checksums: the fused kernel where it takes the job, else the product then the
// standalone CRC kernel over the same shards (one more read of each).
static Status matvec_with_crc(const MatVecJob& job, uint8_t* const* ptrs, int total, const std::vector<int>& slot,
                              size_t S, uint32_t* crcs, hipStream_t stream) {
  if (matvec_crc_accepts(job, total, slot.data()))
    return hip_status(launch_matvec_crc(job, crcs, total, slot.data(), stream), "launch_matvec_crc");
  Status st = hip_status(launch_matvec(job, stream), "launch_matvec");
  if (st != CFSEC_OK) return st;
  st = hip_status(hipMemsetAsync(crcs, 0, sizeof(uint32_t) * (size_t)total * job.nstripes, stream), "hipMemsetAsync");
  if (st != CFSEC_OK || S == 0) return st;
  std::vector<const uint8_t*> p;
  std::vector<uint32_t> idx;
  const bool cin = slot[0] >= 0;
  for (int s = 0; s < job.nstripes; ++s)
    for (int i = 0; i < job.k + job.m; ++i) {
      if (i < job.k && !cin) continue;
      p.push_back(i < job.k ? job.in[(size_t)s * job.k + i] : job.out[(size_t)s * job.m + i - job.k]);
      idx.push_back((uint32_t)(s * total + slot[i]));
    }
  return hip_status(launch_crc32_to(p.data(), S, (int)p.size(), crcs, idx.data(), crc32_shift_ones(S), stream),
                    "launch_crc32_to");
}

Status RSEngine::encode_crc_batch(uint8_t* const* ptrs, size_t S, int nstripes, uint32_t* crcs,
                                  hipStream_t stream) {
  if (!ctx_) return CFSEC_ERR_DEVICE;
  if (!ptrs || !crcs || nstripes < 0) return CFSEC_ERR_INVALID_ARG;
  if (nstripes == 0) return CFSEC_OK;
  DeviceGuard g(ctx_->device());
  if (!g.ok()) return hip_status(hipErrorInvalidDevice, "hipSetDevice");
  if (m_ == 0 || S == 0) {
    Status st = hip_status(hipMemsetAsync(crcs, 0, 4 * (size_t)total() * nstripes, stream), "hipMemsetAsync");
    if (st != CFSEC_OK || S == 0) return st;
    std::vector<const uint8_t*> p(ptrs, ptrs + (size_t)total() * nstripes);
    return hip_status(launch_crc32_to(p.data(), S, (int)p.size(), crcs, nullptr, crc32_shift_ones(S), stream),
                      "launch_crc32_to");
  }
  std::vector<const uint8_t*> in(size_t(nstripes) * k_);
  std::vector<uint8_t*> out(size_t(nstripes) * m_);
  for (int s = 0; s < nstripes; ++s) {
    for (int c = 0; c < k_; ++c) in[size_t(s) * k_ + c] = ptrs[size_t(s) * total() + c];
    for (int r = 0; r < m_; ++r) out[size_t(s) * m_ + r] = ptrs[size_t(s) * total() + k_ + r];
  }
  MatVecJob job;
  job.k = k_;
  job.m = m_;
  job.coef = parity_.v.data();
  job.len = S;
  job.nstripes = nstripes;
  job.in = in.data();
  job.out = out.data();
  std::vector<int> slot(total());
  for (int i = 0; i < total(); ++i) slot[i] = i;
  return matvec_with_crc(job, ptrs, total(), slot, S, crcs, stream);
}

Status RSEngine::reconstruct_crc_batch(uint8_t* const* ptrs, size_t S, int nstripes, const int* erased,
                                       int nerased, bool data_only, uint32_t* crcs, hipStream_t stream) {
  if (!ctx_) return CFSEC_ERR_DEVICE;
  if (!ptrs || !crcs || nstripes < 0 || nerased < 0 || (nerased > 0 && !erased)) return CFSEC_ERR_INVALID_ARG;
  std::vector<bool> present(total(), true);
  for (int i = 0; i < nerased; ++i) {
    if (erased[i] < 0 || erased[i] >= total()) return CFSEC_ERR_INVALID_ARG;
    present[erased[i]] = false;
  }
  int np = 0;
  for (int i = 0; i < total(); ++i) np += present[i] ? 1 : 0;
  if (np < k_ && nstripes > 0) return CFSEC_ERR_TOO_FEW_SHARDS;
  DeviceGuard g(ctx_->device());
  if (!g.ok()) return hip_status(hipErrorInvalidDevice, "hipSetDevice");
  if (nstripes == 0) return CFSEC_OK;
  ReconPlan plan;
  if (np < total()) {
    Status st = plan_reconstruct(present, data_only, &plan);
    if (st != CFSEC_OK) return st;
  }
  const int nout = (int)plan.outputs.size();
  if (nout == 0 || S == 0)
    return hip_status(hipMemsetAsync(crcs, 0, 4 * (size_t)total() * nstripes, stream), "hipMemsetAsync");
  std::vector<const uint8_t*> in(size_t(nstripes) * k_);
  std::vector<uint8_t*> out(size_t(nstripes) * nout);
  for (int s = 0; s < nstripes; ++s) {
    for (int c = 0; c < k_; ++c) in[size_t(s) * k_ + c] = ptrs[size_t(s) * total() + plan.valid[c]];
    for (int r = 0; r < nout; ++r) out[size_t(s) * nout + r] = ptrs[size_t(s) * total() + plan.outputs[r]];
  }
  MatVecJob job;
  job.k = k_;
  job.m = nout;
  job.coef = plan.rows.v.data();
  job.len = S;
  job.nstripes = nstripes;
  job.in = in.data();
  job.out = out.data();
  std::vector<int> slot(k_ + nout, -1);
  for (int r = 0; r < nout; ++r) slot[k_ + r] = plan.outputs[r];
  return matvec_with_crc(job, ptrs, total(), slot, S, crcs, stream);
}

// ---------------------------------------------------------------- ec.Encoder

Status ECEncoder::create(const cfsec_tactic& t, bool enable_verify, int concurrency, int device,
                         std::unique_ptr<ECEncoder>* out) {
  // ec.NewEncoder, encoder.go:78-112
  if (!tactic_valid(t)) return CFSEC_ERR_INVALID_CODE_MODE;
  if (concurrency <= 0) concurrency = 100;  // defaultConcurrency, encoder.go:29
  std::unique_ptr<RSEngine> engine;
  Status st = RSEngine::create(t.n, t.m, device, &engine);
  if (st != CFSEC_OK) return st;
  std::unique_ptr<ECEncoder> enc;
  if (t.l != 0) {
    std::unique_ptr<RSEngine> local;
    const int ln = (t.n + t.m) / t.az_count, lm = t.l / t.az_count;
    st = RSEngine::create(ln, lm, device, &local);
    if (st != CFSEC_OK) return st;
    auto* lrc = new LrcEncoder();
    // Fused LRC encode rows: global parity, then every AZ's local parity expressed over
    // the N data shards (local parity = localRow x [AZ data, AZ global parity], and the
    // global parity is itself parity_row x data).
    const Matrix& G = engine->matrix();
    const Matrix& Lm = local->matrix();
    lrc->fused_ = Matrix(t.m + t.l, t.n);
    for (int r = 0; r < t.m; ++r)
      for (int c = 0; c < t.n; ++c) lrc->fused_.at(r, c) = G.at(t.n + r, c);
    const GF& gf = GF::get();
    const auto az = layout_by_az(t);
    for (int a = 0; a < t.az_count; ++a)
      for (int j = 0; j < lm; ++j) {
        const int g = t.n + t.m + a * lm + j;
        uint8_t* dst = lrc->fused_.row(t.m + (g - t.n - t.m));
        for (int i = 0; i < ln; ++i) {
          const uint8_t coef = Lm.at(ln + j, i);
          const int member = az[a][i];
          for (int c = 0; c < t.n; ++c) {
            const uint8_t basis = member < t.n ? uint8_t(member == c) : G.at(member, c);
            dst[c] ^= gf.mul(coef, basis);
          }
        }
      }
    lrc->local_ = std::move(local);
    enc.reset(lrc);
  } else {
    enc.reset(new ECEncoder());
  }
  enc->t_ = t;
  enc->enable_verify_ = enable_verify;
  enc->pool_.reset(new BlockingCount(concurrency));
  enc->engine_ = std::move(engine);
  *out = std::move(enc);
  return CFSEC_OK;
}

Status ECEncoder::encode(cfsec_shard* shards, int n, int mem, hipStream_t s) {
  Slot slot(pool_.get());  // encoder.go:114-131
  Status st = engine_->encode(shards, n, mem, s);
  if (st != CFSEC_OK) return st;
  if (enable_verify_) {
    bool ok = false;
    st = engine_->verify(shards, n, mem, s, &ok);
    if (st != CFSEC_OK) return st;
    if (!ok) return CFSEC_ERR_VERIFY;
  }
  return CFSEC_OK;
}

Status ECEncoder::verify(cfsec_shard* shards, int n, int mem, hipStream_t s, bool* ok) {
  Slot slot(pool_.get());  // encoder.go:133-137
  return engine_->verify(shards, n, mem, s, ok);
}

Status ECEncoder::reconstruct(cfsec_shard* shards, int n, const int* bad, int nbad, int mem,
                              hipStream_t s) {
  // encoder.go:139-144
  Status st = init_bad_shards(shards, n, std::vector<int>(bad, bad + nbad));
  if (st != CFSEC_OK) return st;
  Slot slot(pool_.get());
  return engine_->reconstruct(shards, n, false, mem, s);
}

Status ECEncoder::reconstruct_data(cfsec_shard* shards, int n, const int* bad, int nbad, int mem,
                                   hipStream_t s) {
  // encoder.go:146-151
  HostTimer whole("ec reconstruct_data");
  Status st = init_bad_shards(shards, n, std::vector<int>(bad, bad + nbad));
  if (st != CFSEC_OK) return st;
  Slot slot(pool_.get());
  return engine_->reconstruct(shards, n, true, mem, s);
}

bool ECEncoder::row_over_data(int g, uint8_t* dst) const {
  const int N = t_.n, M = t_.m;
  if (g < 0 || g >= N + M) return false;
  for (int c = 0; c < N; ++c) dst[c] = g < N ? uint8_t(g == c) : engine_->matrix().at(g, c);
  return true;
}

bool LrcEncoder::row_over_data(int g, uint8_t* dst) const {
  const int N = t_.n, M = t_.m, L = t_.l;
  if (g < N + M) return ECEncoder::row_over_data(g, dst);
  if (g >= N + M + L) return false;
  std::memcpy(dst, fused_.row(M + g - N - M), N);  // lrcencoder.go: the local parity over the data
  return true;
}

Status ECEncoder::repair_rows(const int* bad, int nbad, const int* want, int nwant, int* in, uint8_t* rows) {
  const int N = t_.n, M = t_.m, L = t_.l;
  if ((nbad && !bad) || nbad < 0 || nwant < 0 || (nwant && (!want || !rows)) || !in) return CFSEC_ERR_INVALID_ARG;
  std::vector<bool> present(N + M, true);
  for (int i = 0; i < nbad; ++i) {
    if (bad[i] < 0 || bad[i] >= N + M + L) return CFSEC_ERR_INVALID_ARG;
    if (bad[i] < N + M) present[bad[i]] = false;
  }
  ReconPlan rp;
  Status st = engine_->plan_reconstruct(present, false, &rp);
  if (st != CFSEC_OK) return st;
  // D: the data over the N inputs (unit rows for surviving data, decode rows for the missing)
  Matrix D(N, N);
  for (int i = 0; i < N; ++i) {
    const auto v = std::find(rp.valid.begin(), rp.valid.end(), i);
    const auto o = std::find(rp.outputs.begin(), rp.outputs.end(), i);
    if (v != rp.valid.end()) D.at(i, (int)(v - rp.valid.begin())) = 1;
    else if (o != rp.outputs.end()) std::memcpy(D.row(i), rp.rows.row((int)(o - rp.outputs.begin())), N);
    else return CFSEC_ERR_INVALID_ARG;
  }
  for (int c = 0; c < N; ++c) in[c] = rp.valid[c];
  const GF& gf = GF::get();
  std::vector<uint8_t> g(N);
  for (int w = 0; w < nwant; ++w) {
    if (!row_over_data(want[w], g.data())) return CFSEC_ERR_INVALID_ARG;
    uint8_t* dst = rows + (size_t)w * N;
    for (int c = 0; c < N; ++c) {
      uint8_t v = 0;
      for (int j = 0; j < N; ++j) v ^= gf.mul(g[j], D.at(j, c));
      dst[c] = v;
    }
  }
  return CFSEC_OK;
}

std::vector<int> ECEncoder::shards_in_idc(int idx) const {
  // encoder.go:169-176
  std::vector<int> v;
  const int ln = t_.n / t_.az_count, lm = t_.m / t_.az_count;
  for (int i = idx * ln; i < (idx + 1) * ln; ++i) v.push_back(i);
  for (int i = t_.n + lm * idx; i < t_.n + lm * (idx + 1); ++i) v.push_back(i);
  return v;
}

// ---------------------------------------------------------------- lrcEncoder

std::vector<int> LrcEncoder::shards_in_idc(int idx) const {
  // lrcencoder.go:236-243 via codemode.LocalStripeInAZ (codemode.go:334-345)
  if (idx < 0 || idx >= t_.az_count) return {};
  return layout_by_az(t_)[idx];
}

Status LrcEncoder::encode(cfsec_shard* shards, int n, int mem, hipStream_t s) {
  // lrcencoder.go:35-82
  const int N = t_.n, M = t_.m, L = t_.l;
  if (!shards || n != N + M + L) return CFSEC_ERR_INVALID_SHARDS;
  Slot slot(pool_.get());
  return encode_stripe(shards, n, mem, s);
}

Status LrcEncoder::encode_stripe(cfsec_shard* shards, int n, int mem, hipStream_t s) {
  const int N = t_.n, M = t_.m, L = t_.l;
  Status st = fill_full_shards(shards, n);
  if (st != CFSEC_OK) return st;
  size_t S = 0;
  st = check_shards(shards, N + M, false, &S);  // global engine.Encode's checkShards
  if (st != CFSEC_OK) return st;
  Status local_err = CFSEC_OK;
  for (int a = 0; a < t_.az_count && local_err == CFSEC_OK; ++a) {
    std::vector<cfsec_shard> ls;
    for (int g : shards_in_idc(a)) ls.push_back(shards[g]);
    size_t ignored;
    local_err = check_shards(ls.data(), (int)ls.size(), false, &ignored);
  }
  std::vector<cfsec_shard*> ins, outs;
  for (int i = 0; i < N; ++i) ins.push_back(&shards[i]);
  if (local_err != CFSEC_OK) {
    // The reference's sequence, step by step: global parity (+ Verify), then every AZ's local
    // task -- task.Run lets each goroutine finish, so the AZs that pass checkShards are encoded
    // -- and the first error in AZ order (oracle/ec_oracle.py: ECOracle.encode).
    st = engine_->encode(shards, N + M, mem, s);
    if (st != CFSEC_OK) return st;
    if (enable_verify_) {
      bool ok = false;
      st = engine_->verify(shards, N + M, mem, s, &ok);
      if (st != CFSEC_OK) return st;
      if (!ok) return CFSEC_ERR_VERIFY;
    }
    Status first = CFSEC_OK;
    for (int a = 0; a < t_.az_count; ++a) {
      std::vector<cfsec_shard> ls;
      for (int g : shards_in_idc(a)) ls.push_back(shards[g]);
      Status e = local_->encode(ls.data(), (int)ls.size(), mem, s);
      if (e == CFSEC_OK && enable_verify_) {
        bool ok = false;
        e = local_->verify(ls.data(), (int)ls.size(), mem, s, &ok);
        if (e == CFSEC_OK && !ok) e = CFSEC_ERR_VERIFY;
      }
      if (first == CFSEC_OK) first = e;
    }
    return first;
  }
  for (int i = N; i < N + M + L; ++i) outs.push_back(&shards[i]);
  st = engine_->run(fused_, ins, outs, S, mem, s, MatVecMode::kStore, nullptr);
  if (st != CFSEC_OK) return st;
  if (enable_verify_) {
    bool ok = false;
    st = engine_->run(fused_, ins, outs, S, mem, s, MatVecMode::kVerify, &ok);
    if (st != CFSEC_OK) return st;
    if (!ok) return CFSEC_ERR_VERIFY;
  }
  return CFSEC_OK;
}

Status LrcEncoder::verify(cfsec_shard* shards, int n, int mem, hipStream_t s, bool* ok) {
  // lrcencoder.go:89-131
  *ok = false;
  Slot slot(pool_.get());
  const int N = t_.n, M = t_.m, L = t_.l;
  if (n == (N + M + L) / t_.az_count) return local_->verify(shards, n, mem, s, ok);
  if (!shards || n != N + M + L) return CFSEC_ERR_INVALID_SHARDS;
  Status st = engine_->verify(shards, N + M, mem, s, ok);
  if (st != CFSEC_OK || !*ok) return st;
  for (int a = 0; a < t_.az_count; ++a) {
    std::vector<cfsec_shard> ls;
    for (int g : shards_in_idc(a)) ls.push_back(shards[g]);
    st = local_->verify(ls.data(), (int)ls.size(), mem, s, ok);
    if (st != CFSEC_OK || !*ok) return st;
  }
  *ok = true;
  return CFSEC_OK;
}

Status LrcEncoder::reconstruct(cfsec_shard* shards, int n, const int* bad, int nbad, int mem,
                               hipStream_t s) {
  // lrcencoder.go:133-186
  const int N = t_.n, M = t_.m, L = t_.l, AZ = t_.az_count;
  if (!shards || n <= 0) return CFSEC_ERR_INVALID_SHARDS;
  Status st = fill_full_shards(shards, n);
  if (st != CFSEC_OK) return st;
  std::vector<int> global_bad;
  for (int i = 0; i < nbad; ++i)
    if (bad[i] < N + M) global_bad.push_back(bad[i]);
  st = init_bad_shards(shards, n, global_bad);
  if (st != CFSEC_OK) return st;
  Slot slot(pool_.get());
  if (n == (N + M + L) / AZ) return local_->reconstruct(shards, n, false, mem, s);
  if (n != N + M + L) return CFSEC_ERR_INVALID_SHARDS;
  st = engine_->reconstruct(shards, N + M, false, mem, s);
  if (st != CFSEC_OK) return st;
  std::map<int, std::vector<int>> local_bad;
  for (int i = 0; i < nbad; ++i) {
    const int b = bad[i];
    if (b >= N + M) {
      const int idc = (b - N - M) * AZ / L;
      local_bad[idc].push_back(b - N - M - L / AZ * idc + (N + M) / AZ);
    }
  }
  // task.Run (util/task/task.go:43-73) runs every AZ's local pass to the end and returns the first
  // error sent; the AZs are disjoint, so running them in AZ order and keeping the lowest AZ's error
  // gives the same bytes (the reference's pick among several failing AZs is scheduling-dependent,
  // oracle/ec_oracle.py takes the lowest AZ as well).
  Status first = CFSEC_OK;
  for (auto& kv : local_bad) {
    // Go copies the slice headers into a fresh [][]byte (lrcencoder.go:236-243); the
    // rebuilt bytes land in the shared buffers, the caller's headers keep their length.
    std::vector<cfsec_shard> ls;
    for (int g : shards_in_idc(kv.first)) ls.push_back(shards[g]);
    st = init_bad_shards(ls.data(), (int)ls.size(), kv.second);
    if (st == CFSEC_OK) st = local_->reconstruct(ls.data(), (int)ls.size(), false, mem, s);
    if (st == CFSEC_ERR_DEVICE) return st;  // the device failed: nothing further is meaningful
    if (first == CFSEC_OK) first = st;
  }
  return first;
}

Status LrcEncoder::reconstruct_data(cfsec_shard* shards, int n, const int* bad, int nbad, int mem,
                                    hipStream_t s) {
  // lrcencoder.go:188-201
  const int N = t_.n, M = t_.m;
  if (!shards || n < N + M) return CFSEC_ERR_INVALID_SHARDS;
  Status st = fill_full_shards(shards, N + M);
  if (st != CFSEC_OK) return st;
  std::vector<int> global_bad;
  for (int i = 0; i < nbad; ++i)
    if (bad[i] < N + M) global_bad.push_back(bad[i]);
  st = init_bad_shards(shards, n, global_bad);
  if (st != CFSEC_OK) return st;
  Slot slot(pool_.get());
  return engine_->reconstruct(shards, N + M, true, mem, s);
}

}  // namespace cfsec
