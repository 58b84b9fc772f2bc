// engine.hpp -- the MI355X erasure-coding engine behind the cfsec C ABI.
//
//   RSEngine   restates reedsolomon.Encoder (KRS/reedsolomon.go) for the default
//              Vandermonde code, with its arithmetic on the GPU.
//   ECEncoder  restates ec.Encoder (blobstore/common/ec/encoder.go) and
//   LrcEncoder the LRC variant (blobstore/common/ec/lrcencoder.go).
#pragma once
#include <atomic>
#include <hip/hip_runtime.h>

#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <vector>

#include "../../include/cfsec.h"
#include "gf256.hpp"
#include "kernels.hpp"

namespace cfsec {

// synchronous calls poll a marker word (1) or hipStreamSynchronize (0): cfsec_set_sync_poll
std::atomic<int>& sync_poll_mode();


using Status = int;  // cfsec_status

void set_last_error(const std::string& msg);
const char* last_error_cstr();

// Host-side phase timing of the batch calls, printed to stderr when CFSEC_HOST_TIMING is set
// (development aid: where a synchronous batch call spends its time besides the kernels).
struct HostTimer {
  const char* name;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  static bool on() {
    static const bool v = std::getenv("CFSEC_HOST_TIMING") != nullptr;
    return v;
  }
  explicit HostTimer(const char* n) : name(n) {}
  ~HostTimer() {
    if (on())
      std::fprintf(stderr, "cfsec host %-28s %8.1f us\n", name,
                   std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  }
};
// ec.initBadShards (encoder.go:182-188) / ec.fillFullShards (encoder.go:199-210), engine.cpp.
Status init_bad_shards(cfsec_shard* shards, int n, const std::vector<int>& bad);
Status fill_full_shards(cfsec_shard* shards, int n);
Status hip_status(hipError_t e, const char* what);
// The device address of page-locked host memory (hipHostMalloc / cfsec_host_alloc); false for
// pageable memory.
bool device_alias(uint8_t* p, uint8_t** dptr);
// The library's own page-locked allocations (cfsec_host_alloc / cfsec_host_free), looked up by
// device_alias before it asks the runtime: hipPointerGetAttributes costs microseconds per shard,
// which a small host-memory call (a degraded range read's segment) pays for every row.
void host_range_add(void* base, size_t size);
void host_range_remove(void* base);

// Per-device streams and staging workspaces, shared by every engine on the device.
class DeviceContext {
 public:
  // nullptr if the device does not exist.  slot > 0: another context on the same device (its own
  // streams and workspaces) -- the multi-device rehearsal of set_devices on a one-GPU machine.
  static DeviceContext* get(int device, int slot = 0);
  int device() const { return device_; }

  struct Workspace {
    uint8_t* dbuf = nullptr;   // device staging buffer
    size_t cap = 0;
    uint32_t* dflags = nullptr;  // device verify flags
    uint32_t* hflags = nullptr;  // pinned host mirror
    size_t nflags = 0;
    hipStream_t stream = nullptr;
    hipStream_t stream2 = nullptr;  // second lane of the chunked host pipeline
    hipEvent_t ev = nullptr;        // orders stream2 after work enqueued on stream
    hipEvent_t ev_in = nullptr;     // orders stream after the legacy default stream (no caller stream)
    // batch calls (batch.cpp run_device): per-task verify words, kept zero between calls (the flag
    // gather kernel resets the words it reads), and the device address of hflags
    uint32_t* bflags = nullptr;
    size_t nbflags = 0;
    bool bflags_clean = false;
    uint32_t* hflags_dev = nullptr;
    // asynchronous calls: the workspace is reused only after `done` (recorded on the caller's
    // stream after the call's last kernel) has completed
    hipEvent_t done = nullptr;
    bool pending = false;
    // batch calls with shard checksums: device words (accumulated by the CRC kernel) + pinned mirror
    uint32_t* dcrc = nullptr;
    uint32_t* hcrc = nullptr;
    size_t ncrc = 0;
    // finish(): a pinned, coherent word the stream writes after its work, polled by the caller
    uint32_t* hmark = nullptr;
    uint32_t* dmark = nullptr;
    uint32_t seq = 0;
  };
  // Wait for everything queued on `stream` so far (a synchronous call's end): the stream writes a
  // sequence number into ws's pinned marker word after its work (hipStreamWriteValue32) and the
  // caller polls it, which returns as soon as the GPU gets there -- hipStreamSynchronize's
  // completion-signal wait returned ~15-20 us later (C4 / C5 calls, profiles/r04).  Falls back to
  // hipStreamSynchronize when the marker cannot be written, and after kSpinLimitUs of polling (a
  // long host batch, a fault: the runtime then reports the error).
  Status finish(Workspace* ws, hipStream_t stream);
  static constexpr double kSpinLimitUs = 20000.0;
  static constexpr double kSpinBusyUs = 200.0;
  // Order ws->stream after the work already queued on the legacy default stream (and, by that
  // stream's semantics, on every blocking stream of the device): a device-memory call made
  // without a caller stream must not read its input before the kernel that produced it ran.
  // The workspace streams themselves are non-blocking, so concurrent callers do not serialise
  // on each other's null-stream work.
  Status order_after_default(Workspace* ws);
  // Check out a workspace with at least `bytes` of staging, `nflags` flag words (device + pinned
  // host) and `nbflags` batch flag words (zero on return).
  Status acquire(size_t bytes, size_t nflags, Workspace** out, size_t nbflags = 0, size_t ncrc = 0);
  void release(Workspace* ws);
  // Return a workspace whose work is still queued on `stream`: it is handed out again only once
  // the stream has passed this point.
  void release_after(Workspace* ws, hipStream_t stream);

 private:
  explicit DeviceContext(int device) : device_(device) {}
  int device_;
  std::mutex mu_;
  std::vector<std::unique_ptr<Workspace>> all_;
  std::vector<Workspace*> free_;  // release order: the front was released first
  // beyond this many workspaces an acquire with every free one still pending (asynchronous calls
  // queued without a sync) waits for the oldest instead of allocating another
  static constexpr size_t kMaxWorkspaces = 64;
};

// Makes `device` current for the scope, restoring the caller's device after.
class DeviceGuard {
 public:
  explicit DeviceGuard(int device);
  ~DeviceGuard();
  bool ok() const { return ok_; }

 private:
  int prev_ = -1;
  bool ok_ = false;
};

// KRS/inversion_tree.go:16-164: decode matrices keyed by the invalid indices seen
// before k valid rows were found; RW-locked for concurrent readers.
class InversionCache {
 public:
  bool get(const std::vector<int>& invalid, Matrix* out) const;
  void put(const std::vector<int>& invalid, const Matrix& m);

 private:
  mutable std::shared_mutex mu_;
  std::map<std::vector<int>, Matrix> map_;
};

// Rows to compute for one reconstruct call (shared by the single and batch paths).
struct ReconPlan {
  std::vector<int> valid;    // k surviving shard indices, first-present order
  std::vector<int> outputs;  // shard indices to rebuild
  Matrix rows;               // outputs.size() x k, over the shards in `valid`
};

// The 16 + 20 code's reconstruct (+ verify) through its 16x16 dyadic parity block
// (Dy16RepairJob): missing data rows from decode rows, then all 20 parity rows from the data.
struct Dy16Plan {
  int nd = 0;             // missing data rows
  int e = 0;              // extra rows (ExtraRows) after the 20 parity rows
  std::vector<int> rows;  // output shard indices: the nd missing data rows, parity rows k .. k+19, extras
  uint8_t src[16] = {};
  uint32_t pstore = 0, pcmp = 0;
  Matrix coef;  // (20 + e + nd) x 16: parity matrix, extra rows, decode rows
  // the syndrome form of the bit-sliced repair (gf_bs16.hip): parity row prow[q] stands in for
  // missing data row rows[q]; the missing rows are ainv (nd x nd) times the stand-ins' syndromes
  bool syn = false;
  uint8_t prow[4] = {};
  uint8_t ainv[16] = {};
};

// Rows beyond a code's own that a Reconstruct + Verify pass can check on the way: row j over the
// k data columns, compared with shard idx[j] of the stripe's shard array.  The LRC local parities
// (LrcEncoder: the global pass also does the per-AZ local Verify, lrcencoder.go:89-131).
struct ExtraRows {
  Matrix rows;
  std::vector<int> idx;
};

// The product one stripe of a heterogeneous batch needs (batch.cpp): rows x shards[in]; rows
// [0, nstore) are written to shards[out[0 .. nstore)), the rest compared with shards[out[nstore ..)]
// (a mismatch raises the stripe's flag).  Shared by every stripe with the same erasure pattern.
struct StripePlan {
  std::vector<int> in;
  std::vector<int> out;
  int nstore = 0;
  int nextra = 0;  // the last nextra rows of out are ExtraRows, compared
  Matrix rows;  // out.size() x in.size()
  std::shared_ptr<const Dy16Plan> dy16;  // set where that product is the cheaper one
};

// The device (0 .. ndev-1) each of n stripes of a host-memory batch runs on: contiguous runs
// balanced by the bytes each stripe moves (cfsec_batch_partition).
void partition_stripes(const uint64_t* bytes, int n, int ndev, int* dev);

// An asynchronous batch call's destination: kernels on `stream`, per-item Verify mismatches OR-ed
// into the device words flags[owner] (the caller zeroes them).
struct AsyncOut {
  hipStream_t stream = nullptr;
  uint32_t* flags = nullptr;
};

// Shard checksums a batch call returns (crc32.ChecksumIEEE, access/stream_put.go:249-253,
// blobnode/work_shard_recover.go:335-342): words[w] for the rows the tasks name (StripeTask::crc);
// host memory for the synchronous calls (words the call does not compute are left alone), device
// memory on the call's stream for the asynchronous ones (zeroed by the call first).
struct CrcOut {
  uint32_t* words = nullptr;
  size_t n = 0;
};

// One stripe of a batch call: its shard vector, the plan, its length, its result.
struct StripeTask {
  cfsec_shard* shards = nullptr;
  const StripePlan* plan = nullptr;
  size_t len = 0;
  int* status = nullptr;        // set to CFSEC_ERR_VERIFY when a compared row mismatches
  int dev = 0;                  // index into the engine's device list
  int phase = 0;                // tasks of phase p run after every task of phase p - 1 (same call)
  int owner = 0;                // batch item: a host batch keeps an item's tasks on one device; the
                                // item's Verify word (asynchronous calls: the caller's flags[owner])
  int crc = 0;                  // checksums: 0 none, 1 the stored rows, 2 every row (inputs + stored)
  int64_t crc_word = 0;         // CrcOut word of shard index 0 of this task's item
  const int* crc_map = nullptr; // shard index -> index in the item (local views), or identity
};

// Plans built for one batch call (stable addresses for the tasks that point at them).
struct PlanStore {
  std::map<std::vector<bool>, std::unique_ptr<StripePlan>> by_pattern;
  std::vector<std::unique_ptr<StripePlan>> other;
  StripePlan* add(const StripePlan& p) {
    other.emplace_back(new StripePlan(p));
    return other.back().get();
  }
};

class RSEngine {
 public:
  static Status create(int k, int m, int device, std::unique_ptr<RSEngine>* out);
  int k() const { return k_; }
  int m() const { return m_; }
  int total() const { return k_ + m_; }
  int device() const { return ctx_ ? ctx_->device() : -1; }
  const Matrix& matrix() const { return mat_; }
  // rows [r0, r0 + nr) of the encoding matrix (the parity rows: matrix_rows(k, m))
  Matrix matrix_rows(int r0, int nr) const {
    Matrix out(nr, k_);
    for (int r = 0; r < nr; ++r)
      for (int c = 0; c < k_; ++c) out.at(r, c) = mat_.at(r0 + r, c);
    return out;
  }

  Status encode(cfsec_shard* shards, int n, int mem, hipStream_t stream);
  // Encode + crc32.ChecksumIEEE of every shard into host crcs[n], one fused pass.
  Status encode_crc(cfsec_shard* shards, int n, int mem, hipStream_t stream, uint32_t* crcs);
  Status verify(cfsec_shard* shards, int n, int mem, hipStream_t stream, bool* ok);
  Status reconstruct(cfsec_shard* shards, int n, bool data_only, int mem, hipStream_t stream);
  Status split(uint8_t* data, size_t len, size_t cap, cfsec_shard* out, uint8_t* pad,
               size_t pad_len, size_t* pad_needed);
  Status join(uint8_t* dst, size_t dst_len, const cfsec_shard* shards, int n, size_t out_size);

  Status encode_batch(uint8_t* const* ptrs, size_t S, int nstripes, hipStream_t stream);
  Status verify_batch(uint8_t* const* ptrs, size_t S, int nstripes, uint32_t* flags,
                      hipStream_t stream);
  Status reconstruct_batch(uint8_t* const* ptrs, size_t S, int nstripes, const int* erased,
                           int nerased, bool data_only, hipStream_t stream);
  // outputs = coef (rows x k) x inputs for every stripe of a device batch: ptrs[s*(k+rows) ..] =
  // the k inputs, then the rows outputs (any rows, e.g. ECEncoder::repair_rows).
  Status matvec_batch(const uint8_t* coef, int rows, uint8_t* const* ptrs, size_t S, int nstripes,
                      hipStream_t stream);
  // The same with crc32.ChecksumIEEE of the shards (fused into the kernel where supported):
  // crcs = device [nstripes * total()]; encode checksums every shard, reconstruct the rebuilt ones
  // (other words 0).
  Status encode_crc_batch(uint8_t* const* ptrs, size_t S, int nstripes, uint32_t* crcs, hipStream_t stream);
  Status reconstruct_crc_batch(uint8_t* const* ptrs, size_t S, int nstripes, const int* erased, int nerased,
                               bool data_only, uint32_t* crcs, hipStream_t stream);

  // Plan the rows of a reconstruct given which shards are present.
  Status plan_reconstruct(const std::vector<bool>& present, bool data_only, ReconPlan* plan);

  // ---- heterogeneous stripe batches (batch.cpp) ----
  // The devices batch entry points spread stripes over (the handle's own device first).
  Status set_devices(const int* devices, int n);
  int ndevices() const { return (int)devs_.size(); }
  // `stripes` holds nst pointers to shard vectors of total() entries; each stripe has its own
  // shard size and missing set.  Per-stripe results go to status[]; the return value reports only
  // failures of the call itself (device errors, bad arguments).
  //   encode:              Encode(shards)                         (KRS/reedsolomon.go:609-625)
  //   verify:              Verify(shards): OK, or CFSEC_ERR_VERIFY when it returns false
  //   reconstruct(verify): Reconstruct(shards) [then Verify(shards)], the blobnode repair step
  //                        (blobnode/work_shard_recover.go:751-760), in one fused pass
  Status encode_stripes(cfsec_shard* const* stripes, int nst, int mem, int* status);
  Status verify_stripes(cfsec_shard* const* stripes, int nst, int mem, int* status);
  Status reconstruct_stripes(cfsec_shard* const* stripes, int nst, int mem, bool verify, int* status);
  // The planning half of reconstruct_stripes: checks every stripe (errors to status[s]), sets the
  // rebuilt shards' lengths and appends the tasks (phase `phase`, and phase + 1 for a split Verify)
  // that run_stripes executes; owner of stripe s = owner0 + s.
  // extra / fuse (optional): stripe s also compares the ExtraRows when fuse[s] (and verify).
  void plan_reconstruct_tasks(cfsec_shard* const* stripes, int nst, bool verify, int* status, int phase,
                              int owner0, PlanStore* store, std::vector<StripeTask>* tasks,
                              const ExtraRows* extra = nullptr, const std::vector<bool>* fuse = nullptr);
  // Run the tasks' products (device memory, pinned host memory in place, pageable host memory
  // through double-buffered staging), tasks partitioned over the devices.
  // async (device memory, the handle's first device): enqueue on async->stream and return; verify
  // mismatches OR 1 into async->flags[owner] instead of setting the tasks' status.
  Status run_stripes(std::vector<StripeTask>& tasks, int mem, const AsyncOut* async = nullptr,
                     const CrcOut* crc = nullptr);
  // Plan of a Reconstruct (+ Verify) over the present shards.
  Status plan_stripe(const std::vector<bool>& present, bool verify, StripePlan* plan,
                     const ExtraRows* extra = nullptr);
  // plan->dy16 where the code and the erasure pattern make that product cheaper (batch.cpp).
  void plan_dy16(const std::vector<bool>& present, const Matrix& dec, StripePlan* plan,
                 const ExtraRows* extra = nullptr) const;
  // The batch calls stripe by stripe through the single-stripe calls (k > kLaunchMaxRows Verify).
  Status stripes_one_by_one(cfsec_shard* const* stripes, int nst, int mem, bool reconstruct, bool verify,
                            int* status);
  // Run a plan's Verify as a separate encode-matrix pass instead of its compared rows.
  bool split_verify(const StripePlan& p) const;

  // Generic "outputs = rows x inputs" over caller shards (host or device memory).
  // mode kVerify: *ok set; outputs are read, not written.
  Status run(const Matrix& rows, const std::vector<cfsec_shard*>& ins,
             const std::vector<cfsec_shard*>& outs, size_t S, int mem, hipStream_t stream,
             MatVecMode mode, bool* ok);

  // Columns of a host-memory call per chunk (bytes per row) through the two-stream pipeline.
  static constexpr size_t kHostChunk = 1 << 20;
  // pageable host calls moving at most this many bytes take the page-locked staging path (run)
  static constexpr size_t kSmallPageable = 1 << 20;

 private:
  Status run_host(const Matrix& rows, const std::vector<cfsec_shard*>& ins,
                  const std::vector<cfsec_shard*>& outs, size_t S, MatVecMode mode, bool* ok);

 public:

 private:
  RSEngine() = default;
  int k_ = 0, m_ = 0;
  Matrix mat_;     // total x k
  Matrix parity_;  // m x k (r.parity, KRS/reedsolomon.go:568-571)
  InversionCache tree_;
  // Reconstruct plans across calls (blobnode's tasklets repeat one erasure pattern call after call):
  // key = the present shards + [extra rows fused] + [verify]; a cached plan is never changed or
  // freed, so concurrent callers share it.  Beyond kMaxCachedPlans patterns a call keeps its own.
  std::mutex plan_mu_;
  std::map<std::vector<bool>, std::unique_ptr<StripePlan>> plan_cache_;
  static constexpr size_t kMaxCachedPlans = 4096;
  const StripePlan* cached_plan(const std::vector<bool>& present, bool fx, bool verify, const ExtraRows* extra,
                                PlanStore* store, Status* st);
  DeviceContext* ctx_ = nullptr;
  std::vector<DeviceContext*> devs_;  // batch devices, ctx_ first
  Status run_device(std::vector<StripeTask*>& tasks, int mem, DeviceContext* ctx, const AsyncOut* async,
                    const CrcOut* crc);
};

// Counting semaphore (util/limit/count.NewBlockingCount, encoder.go:90).
class BlockingCount {
 public:
  explicit BlockingCount(int n) : left_(n) {}
  void acquire() {
    std::unique_lock<std::mutex> l(mu_);
    cv_.wait(l, [&] { return left_ > 0; });
    --left_;
  }
  void release() {
    std::lock_guard<std::mutex> l(mu_);
    ++left_;
    cv_.notify_one();
  }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  int left_;
};

class ECEncoder {
 public:
  static Status create(const cfsec_tactic& t, bool enable_verify, int concurrency, int device,
                       std::unique_ptr<ECEncoder>* out);
  virtual ~ECEncoder() = default;
  virtual Status encode(cfsec_shard* shards, int n, int mem, hipStream_t s);
  virtual Status reconstruct(cfsec_shard* shards, int n, const int* bad, int nbad, int mem,
                             hipStream_t s);
  virtual Status reconstruct_data(cfsec_shard* shards, int n, const int* bad, int nbad, int mem,
                                  hipStream_t s);
  virtual Status verify(cfsec_shard* shards, int n, int mem, hipStream_t s, bool* ok);
  virtual std::vector<int> shards_in_idc(int idx) const;
  const cfsec_tactic& tactic() const { return t_; }
  // Repair over survivors held elsewhere (chubaofs_amd/repair.py ships only the first N present
  // global shards): in[0..N) = the first N global shards not in bad (KRS/reedsolomon.go:1453-1465),
  // rows[w * N ..] = shard want[w] (data, global parity, or an LRC local parity) over them.
  Status repair_rows(const int* bad, int nbad, const int* want, int nwant, int* in, uint8_t* rows);
  Status matvec_batch(const uint8_t* coef, int rows, uint8_t* const* ptrs, size_t S, int nstripes,
                      hipStream_t stream) {
    return engine_->matvec_batch(coef, rows, ptrs, S, nstripes, stream);
  }
  // Devices the batch entry points spread bids over (batch.cpp).
  virtual Status set_devices(const int* devices, int n);
  // blobnode's repair step over a batch of bids (work_shard_recover.go:708-771): for bid b, the
  // n shards at shards[b*n ..], Reconstruct(shards_b, bad_b) then Verify(shards_b), where bad_b =
  // bad[bad_off[b] .. bad_off[b+1]); status[b] = the Reconstruct error, CFSEC_ERR_VERIFY when Verify
  // returns false, or CFSEC_OK.  verify = false: Reconstruct only.
  // async (device memory, asynchronous on async->stream): status[b] gets the planning result at
  // return; a Verify mismatch ORs 1 into async->flags[b] when the stream gets there.
  // crc: the rebuilt shards' checksums into crc->words[b * n + shard] (other words untouched).
  virtual Status reconstruct_batch(cfsec_shard* shards, int n, int nbids, const int* bad, const int* bad_off,
                                   int mem, bool verify, int* status, const AsyncOut* async = nullptr,
                                   const CrcOut* crc = nullptr);
  // Encode over a batch of stripes of n shards each (access puts, stream_put.go:104-143), with
  // the Config's EnableVerify; status[s] as Encode would return it.
  // crc: every shard's checksum after the Encode into crc->words[s * n + shard].
  virtual Status encode_batch(cfsec_shard* shards, int n, int nstripes, int mem, int* status,
                              const AsyncOut* async = nullptr, const CrcOut* crc = nullptr);

 protected:
  // Shard index g (< N + M + L) as a row over the N data shards.
  virtual bool row_over_data(int g, uint8_t* dst) const;
  struct Slot {
    explicit Slot(BlockingCount* p) : p_(p) { p_->acquire(); }
    ~Slot() { p_->release(); }
    BlockingCount* p_;
  };
  cfsec_tactic t_{};
  bool enable_verify_ = false;
  std::unique_ptr<BlockingCount> pool_;
  std::unique_ptr<RSEngine> engine_;
};

class LrcEncoder : public ECEncoder {
 public:
  Status encode(cfsec_shard* shards, int n, int mem, hipStream_t s) override;
  Status reconstruct(cfsec_shard* shards, int n, const int* bad, int nbad, int mem,
                     hipStream_t s) override;
  Status reconstruct_data(cfsec_shard* shards, int n, const int* bad, int nbad, int mem,
                          hipStream_t s) override;
  Status verify(cfsec_shard* shards, int n, int mem, hipStream_t s, bool* ok) override;
  std::vector<int> shards_in_idc(int idx) const override;
  Status set_devices(const int* devices, int n) override;
  Status reconstruct_batch(cfsec_shard* shards, int n, int nbids, const int* bad, const int* bad_off, int mem,
                           bool verify, int* status, const AsyncOut* async = nullptr,
                           const CrcOut* crc = nullptr) override;
  Status encode_batch(cfsec_shard* shards, int n, int nstripes, int mem, int* status,
                      const AsyncOut* async = nullptr, const CrcOut* crc = nullptr) override;

 protected:
  bool row_over_data(int g, uint8_t* dst) const override;

 private:
  // Encode of one full stripe (n == N+M+L) without taking a concurrency slot (the caller holds one).
  Status encode_stripe(cfsec_shard* shards, int n, int mem, hipStream_t s);
  friend class ECEncoder;
  std::unique_ptr<RSEngine> local_;
  Matrix fused_;  // (M+L) x N: global parity rows then local parity rows, over data
};

}  // namespace cfsec
