// batch.cpp -- heterogeneous stripe batches over one or more GPUs (see engine.hpp).
//
// The reference codes one stripe per call: access puts encode one blob at a time
// (access/stream_put.go:104-143, up to 4 in flight per request) and blobnode repairs a tasklet bid
// by bid, each bid with its own shard size and its own missing set, Reconstruct then Verify
// (blobnode/work_shard_recover.go:708-771).  Here a whole batch is one call: stripes with the same
// erasure pattern share one decode plan and run in the same launches (per-stripe lengths in the
// kernel arguments), Reconstruct + Verify is one pass (the stored rows and the compared rows come
// out of one product over the first k present shards), and the stripes are spread over the
// handle's devices, each with its own streams and staging.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <thread>

#include "engine.hpp"

namespace cfsec {
namespace {

constexpr size_t kSlot = 256;                      // staging rows start on 256-B boundaries
constexpr size_t kLaneBudget = size_t(256) << 20;  // staging bytes per lane of a pageable batch

size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// The HIP device that owns device memory p, or -1.
int device_of(const void* p) {
  hipPointerAttribute_t attr;
  if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  if (attr.type != hipMemoryTypeDevice) return -1;
  return attr.device;
}

// KRS/reedsolomon.go:1314-1339 checkShards / shardSize (as engine.cpp's).
Status stripe_size(const cfsec_shard* shards, int n, bool nilok, size_t* size) {
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

// Rows of one device launch group: stripes sharing a plan.
struct Group {
  const StripePlan* plan = nullptr;
  std::vector<StripeTask*> tasks;
  std::vector<const uint8_t*> in;  // [tasks * k]
  std::vector<uint8_t*> out;       // [tasks * m]
  std::vector<uint64_t> lens;
  std::vector<uint8_t*> hout;      // plan->dy16: [tasks * (nd + 20)] its output rows
  int flag0 = 0;                   // first flag word
  uint32_t* direct = nullptr;      // or: task i's Verify word is direct[i] (consecutive items' words)
  uint32_t* zero_words = nullptr;  // dy16: the call's checksum words, zeroed by the group's first launch
  uint32_t nzero = 0;
  // dy16: the stored rows' checksums in the repair pass (dy16_crc_group): task i's checksummed row k
  // into crc_words[i * crc_stride + crc_slot[k]]; crc_done[i] = 1 once a launch accumulated them
  uint32_t* crc_words = nullptr;
  uint32_t crc_stride = 0;
  uint8_t crc_slot[4] = {};
  int crc_mode = 1;
  std::vector<char>* crc_done = nullptr;
};

hipError_t launch_group_run(const Group& g, size_t t0, size_t t1, uint32_t* dflags, hipStream_t s);

// Enqueue one group: maximal runs of stripes that sit at one stride from each other (every row)
// launch as affine batches of any size; the rest as pointer tables.
hipError_t launch_group(const Group& g, uint32_t* dflags, hipStream_t s) {
  const size_t k = g.plan->in.size(), m = g.plan->out.size(), nt = g.tasks.size();
  bool uniform = true;
  for (uint64_t l : g.lens) uniform = uniform && l == g.lens[0];
  if (!uniform || nt < 3) return launch_group_run(g, 0, nt, dflags, s);
  const auto addr = [](const void* p) { return (int64_t)(uintptr_t)p; };
  const auto stride_ok = [&](size_t t, int64_t d) {  // stripe t+1 = stripe t + d on every row
    for (size_t c = 0; c < k; ++c)
      if (addr(g.in[(t + 1) * k + c]) - addr(g.in[t * k + c]) != d) return false;
    for (size_t r = 0; r < m; ++r)
      if (addr(g.out[(t + 1) * m + r]) - addr(g.out[t * m + r]) != d) return false;
    if (g.plan->dy16) {
      const size_t mo = g.plan->dy16->rows.size();
      for (size_t r = 0; r < mo; ++r)
        if (addr(g.hout[(t + 1) * mo + r]) - addr(g.hout[t * mo + r]) != d) return false;
    }
    return true;
  };
  // Runs shorter than kMinRun stripes (separately allocated shards: blobnode's per-vuid buffers)
  // are not launched one by one -- a launch per stripe leaves most of the GPU idle (C5's tasklet
  // with every shard at its own address: 64 launches of 16 workgroups, 1.9 ms) -- but gathered into
  // pointer-table runs, which the launchers split into as many stripes per launch as their argument
  // block holds.
  constexpr size_t kMinRun = 4;
  const auto run_end = [&](size_t t0) {
    size_t t1 = t0 + 1;
    if (t1 < nt) {
      const int64_t d = addr(g.in[t1 * k]) - addr(g.in[t0 * k]);
      while (t1 < nt && d != 0 && stride_ok(t1 - 1, d)) ++t1;
    }
    return t1;
  };
  size_t t0 = 0;
  while (t0 < nt) {
    size_t t1 = run_end(t0);
    if (t1 - t0 < kMinRun) {  // extend over the following short runs
      while (t1 < nt) {
        const size_t t2 = run_end(t1);
        if (t2 - t1 >= kMinRun) break;
        t1 = t2;
      }
    }
    const hipError_t e = launch_group_run(g, t0, t1, dflags, s);
    if (e != hipSuccess) return e;
    t0 = t1;
  }
  return hipSuccess;
}

// Stripes [t0, t1) of a group: the mixed store/compare product, split into a store and a compare
// launch when the rows exceed one launch.
hipError_t launch_group_run(const Group& g, size_t t0, size_t t1, uint32_t* dflags, hipStream_t s) {
  if (const Dy16Plan* d = g.plan->dy16.get()) {
    Dy16RepairJob job;
    job.nd = d->nd;
    job.coef = d->coef.v.data();
    std::memcpy(job.src, d->src, 16);
    job.pstore = d->pstore;
    job.pcmp = d->pcmp;
    if (d->syn) {
      job.syn = true;
      std::memcpy(job.prow, d->prow, 4);
      std::memcpy(job.ainv, d->ainv, 16);
    }
    job.nstripes = (int)(t1 - t0);
    job.in = g.in.data() + t0 * 16;
    job.e = d->e;
    job.out = g.hout.data() + t0 * d->rows.size();
    bool uniform = true;
    for (size_t t = t0; t < t1; ++t) uniform = uniform && g.lens[t] == g.lens[t0];
    job.lens = uniform ? nullptr : g.lens.data() + t0;
    job.len = g.lens[t0];
    job.flags = g.direct ? g.direct + t0 : dflags + g.flag0 + t0;
    if (t0 == 0) {
      job.zero_words = g.zero_words;
      job.nzero = g.nzero;
    }
    if (g.crc_words && g.crc_done) {
      job.crc_words = g.crc_words + t0 * g.crc_stride;
      job.crc_stride = g.crc_stride;
      job.crc_mode = g.crc_mode;
      std::memcpy(job.crc_slot, g.crc_slot, 4);
      job.crc_done = g.crc_done->data() + t0;
    }
    return launch_dy16_repair(job, s);
  }
  MatVecJob job;
  job.k = (int)g.plan->in.size();
  job.m = (int)g.plan->out.size();
  job.coef = g.plan->rows.v.data();
  job.nstripes = (int)(t1 - t0);
  job.in = g.in.data() + t0 * job.k;
  job.out = g.out.data() + t0 * job.m;
  // one length for the run: no per-stripe lengths, so stripes carved from one pitched buffer run
  // as a single affine launch (any number of stripes) instead of 8-32 per launch
  bool uniform = true;
  for (size_t t = t0; t < t1; ++t) uniform = uniform && g.lens[t] == g.lens[t0];
  job.lens = uniform ? nullptr : g.lens.data() + t0;
  job.len = g.lens[t0];
  job.flags = g.direct ? g.direct + t0 : dflags + g.flag0 + t0;
  job.mode = MatVecMode::kStoreVerify;
  job.nstore = g.plan->nstore;
  if (job.m <= kLaunchMaxRows || job.nstore == 0 || job.nstore == job.m) return launch_matvec(job, s);
  // store rows [0, nstore) then compare rows [nstore, m): two jobs over row subsets
  const int k = job.k, m = job.m, ns = job.nstripes, nst = job.nstore;
  std::vector<uint8_t*> o1((size_t)ns * nst), o2((size_t)ns * (m - nst));
  for (int t = 0; t < ns; ++t) {
    for (int r = 0; r < nst; ++r) o1[(size_t)t * nst + r] = job.out[(size_t)t * m + r];
    for (int r = nst; r < m; ++r) o2[(size_t)t * (m - nst) + r - nst] = job.out[(size_t)t * m + r];
  }
  MatVecJob a = job, b = job;
  a.m = nst;
  a.out = o1.data();
  a.mode = MatVecMode::kStore;
  b.m = m - nst;
  b.coef = g.plan->rows.v.data() + (size_t)nst * k;
  b.out = o2.data();
  b.mode = MatVecMode::kVerify;
  hipError_t e = launch_matvec(a, s);
  return e != hipSuccess ? e : launch_matvec(b, s);
}

// A group whose product is a plain store of a shape the fused product + CRC kernels cover (gf_crc.hpp:
// m <= 6, k in {6, 8, 12, 16, 18}, one length) and whose checksum words sit at one stride per task
// (no index remap, no other task of the same bid writing that bid's words) runs as one fused launch:
// the shards are checksummed from the registers the product already holds, instead of a second pass
// that reads every row again (EC12P4 8 x 64 MiB: 130 + 123 us -> ~180 us).  Returns false when the
// group does not qualify (then the product and the separate pass run as before).  The words are
// zeroed by run_device already (the launch skips its own memset).
bool fused_crc_group(const Group& g, uint32_t* dcrc, size_t nwords, const std::map<int, int>& tasks_per_owner,
                     hipStream_t s, Status* st) {
  static const bool kOn = [] {  // CFSEC_BATCH_FUSED_CRC=0: the separate pass always (A/B)
    const char* v = std::getenv("CFSEC_BATCH_FUSED_CRC");
    return !(v && v[0] == '0');
  }();
  const StripePlan& p = *g.plan;
  const int k = (int)p.in.size(), m = (int)p.out.size();
  const size_t nt = g.tasks.size();
  if (!kOn || p.dy16 || p.nstore != m || m == 0 || nt == 0) return false;
  const uint64_t len = g.lens[0];
  if (len == 0 || !matvec_crc_supported(k, m, len, p.rows.v.data())) return false;
  const StripeTask* t0 = g.tasks[0];
  const int mode = t0->crc;  // 2: inputs and outputs, 1: the stored outputs only
  if (mode == 0 || (m > 6 && mode != 2)) return false;  // m = 12 (EC6P10L2 encode): every shard checksummed
  int64_t cs = 0;
  for (size_t i = 0; i < nt; ++i) {
    const StripeTask* t = g.tasks[i];
    if (t->crc != mode || t->crc_map || g.lens[i] != len || tasks_per_owner.at(t->owner) != 1) return false;
    if (i == 1) cs = t->crc_word - t0->crc_word;
    if (i >= 1 && t->crc_word - g.tasks[i - 1]->crc_word != cs) return false;
  }
  int maxrow = 0;
  for (int c : p.in) maxrow = std::max(maxrow, c);
  for (int o : p.out) maxrow = std::max(maxrow, o);
  if (nt == 1) cs = maxrow + 1;
  if (cs <= maxrow || cs > 256 || t0->crc_word < 0 || (size_t)(t0->crc_word + cs * (int64_t)nt) > nwords) return false;
  std::vector<int> slot(k + m);
  for (int c = 0; c < k; ++c) slot[c] = mode == 2 ? p.in[c] : -1;
  for (int r = 0; r < m; ++r) slot[k + r] = p.out[r];
  MatVecJob job;
  job.k = k;
  job.m = m;
  job.coef = p.rows.v.data();
  job.len = len;
  job.nstripes = (int)nt;
  job.in = g.in.data();
  job.out = g.out.data();
  job.mode = MatVecMode::kStore;
  *st = hip_status(launch_matvec_crc(job, dcrc + t0->crc_word, (int)cs, slot.data(), s, false),
                   "launch_matvec_crc(batch)");
  if (std::getenv("CFSEC_TRACE_BATCH"))  // which groups fused, for tests
    std::fprintf(stderr,"cfsec batch: fused crc group k=%d m=%d tasks=%zu len=%llu\n", k, m, nt, (unsigned long long)len);
  return true;
}

// A dy16 (16 + 20 code) repair group whose stored rows -- the rebuilt data rows and the rebuilt parity
// rows, at most 4 per bid (C5's {0, 1, 16, 17}) -- are checksummed by the bit-sliced repair pass
// itself (gf_bs16.hip CRC launches) instead of a second pass over the rebuilt rows: every task one
// checksummed task of its bid (crc == 1, no index remap), one length (a multiple of the kernel's
// 2 KiB tile), the words at one stride.  Sets the group's crc_* fields; the launches report which
// tasks they covered (crc_done), the rest keep the separate pass.  The words must be zeroed before.
bool dy16_crc_group(Group& g, uint32_t* dcrc, size_t nwords, const std::map<int, int>& tasks_per_owner,
                    std::vector<char>* done) {
  // CFSEC_BS_REPAIR_CRC (read per call) = 1: the Horner steps inside the network -- measured slower
  // than the separate pass on C5's tasklet (profiles/r05/c5_repair_crc.txt: 178-183 vs 154-156 us
  // per call): the repair kernel sits at 253 of 256 VGPRs at 2 waves per SIMD, so the Horner
  // registers and lookups spill or serialise, and the block tile order it needs costs 8 % by itself;
  // = 2: each wave checksums the rebuilt rows of its own tiles after its last tile (round 6, a second
  // phase of the same kernel: no launch, no dependence on other waves, the network's registers free)
  const char* on = std::getenv("CFSEC_BS_REPAIR_CRC");
  if (!on || (on[0] != '1' && on[0] != '2')) return false;
  g.crc_mode = on[0] - '0';
  const Dy16Plan* d = g.plan->dy16.get();
  const size_t nt = g.tasks.size();
  if (!d || !d->syn || d->nd > kBsRepairMaxMissing || nt == 0 || !dcrc) return false;
  const uint64_t len = g.lens[0];
  if (len == 0 || len % kBsRepairTileBytes) return false;
  // checksummed rows in the kernel's order: the missing data rows, then the stored parity rows
  std::vector<int> rows;
  for (int j = 0; j < d->nd; ++j) rows.push_back(d->rows[j]);
  for (int p = 0; p < 22; ++p)
    if (d->pstore >> p & 1u) rows.push_back(d->rows[d->nd + p]);
  if (rows.empty() || rows.size() > 4) return false;
  std::vector<int> stored(g.plan->out.begin(), g.plan->out.begin() + g.plan->nstore);
  std::vector<int> sorted_rows = rows;
  std::sort(stored.begin(), stored.end());
  std::sort(sorted_rows.begin(), sorted_rows.end());
  if (stored != sorted_rows) return false;  // the separate pass would checksum other rows
  int64_t cs = 0;
  for (size_t i = 0; i < nt; ++i) {
    const StripeTask* t = g.tasks[i];
    if (t->crc != 1 || t->crc_map || g.lens[i] != len || tasks_per_owner.at(t->owner) != 1) return false;
    if (i == 1) cs = t->crc_word - g.tasks[0]->crc_word;
    if (i >= 1 && t->crc_word - g.tasks[i - 1]->crc_word != cs) return false;
  }
  const int maxrow = *std::max_element(rows.begin(), rows.end());
  if (nt == 1) cs = maxrow + 1;
  const int64_t w0 = g.tasks[0]->crc_word;
  if (cs <= maxrow || maxrow > 255 || w0 < 0 || (size_t)(w0 + cs * (int64_t)nt) > nwords) return false;
  g.crc_words = dcrc + w0;
  g.crc_stride = (uint32_t)cs;
  for (size_t k = 0; k < rows.size(); ++k) g.crc_slot[k] = (uint8_t)rows[k];
  done->assign(nt, 0);
  g.crc_done = done;
  return true;
}

// Group tasks by plan (first appearance order) and give each group consecutive flag words from
// *next_flag; row pointers from ptr(task, shard index).
template <class Ptr>
std::vector<Group> make_groups(const std::vector<StripeTask*>& tasks, int* next_flag, Ptr ptr) {
  std::vector<Group> groups;
  std::map<const StripePlan*, size_t> index;
  for (StripeTask* t : tasks) {
    auto it = index.find(t->plan);
    if (it == index.end()) {
      it = index.emplace(t->plan, groups.size()).first;
      groups.emplace_back();
      groups.back().plan = t->plan;
    }
    groups[it->second].tasks.push_back(t);
  }
  for (Group& g : groups) {
    g.flag0 = *next_flag;
    g.in.reserve(g.tasks.size() * g.plan->in.size());
    g.out.reserve(g.tasks.size() * g.plan->out.size());
    g.lens.reserve(g.tasks.size());
    // dy16 output rows: rows the kernel neither stores nor compares (inputs; parity not verified)
    // get any pointer the task has -- decided once per plan, not per task
    std::vector<int> hrow;
    if (g.plan->dy16)
      for (int idx : g.plan->dy16->rows) {
        const bool known = std::find(g.plan->in.begin(), g.plan->in.end(), idx) != g.plan->in.end() ||
                           std::find(g.plan->out.begin(), g.plan->out.end(), idx) != g.plan->out.end();
        hrow.push_back(known ? idx : g.plan->in[0]);
      }
    g.hout.reserve(g.tasks.size() * hrow.size());
    for (size_t i = 0; i < g.tasks.size(); ++i) {
      StripeTask* t = g.tasks[i];
      for (int c : g.plan->in) g.in.push_back(ptr(t, c));
      for (int o : g.plan->out) g.out.push_back(const_cast<uint8_t*>(ptr(t, o)));
      g.lens.push_back(t->len);
      for (int idx : hrow) g.hout.push_back(const_cast<uint8_t*>(ptr(t, idx)));
    }
    *next_flag += (int)g.tasks.size();
  }
  return groups;
}

}  // namespace

void partition_stripes(const uint64_t* bytes, int n, int ndev, int* dev) {
  // Stripe i goes to the device whose share of the byte total holds the midpoint of stripe i's
  // bytes: contiguous, non-decreasing runs whose loads differ by at most one stripe's bytes.
  long double total = 0;
  for (int i = 0; i < n; ++i) total += bytes[i];
  long double acc = 0;
  for (int i = 0; i < n; ++i) {
    const long double mid = acc + (long double)bytes[i] / 2;
    int d = total > 0 ? (int)(mid * ndev / total) : (int)((long double)i * ndev / std::max(n, 1));
    dev[i] = std::max(0, std::min(ndev - 1, d));
    acc += bytes[i];
  }
}

Status RSEngine::set_devices(const int* devices, int n) {
  if (!devices || n <= 0) return CFSEC_ERR_INVALID_ARG;
  // CFSEC_DEVICE_REHEARSAL=1: a repeated ordinal is another context on that device (own thread,
  // streams and staging), so the multi-device split runs on a one-GPU machine
  const char* reh = std::getenv("CFSEC_DEVICE_REHEARSAL");
  const bool rehearsal = reh && *reh && *reh != '0';
  std::vector<DeviceContext*> v;
  for (int i = 0; i < n; ++i) {
    const int slot = rehearsal ? (int)std::count(devices, devices + i, devices[i]) : 0;
    DeviceContext* c = DeviceContext::get(devices[i], slot);
    if (!c) {
      set_last_error("set_devices: device " + std::to_string(devices[i]) + " does not exist");
      return CFSEC_ERR_DEVICE;
    }
    if (std::find(v.begin(), v.end(), c) != v.end()) return CFSEC_ERR_INVALID_ARG;
    v.push_back(c);
  }
  devs_ = std::move(v);
  return CFSEC_OK;
}

Status RSEngine::plan_stripe(const std::vector<bool>& present, bool verify, StripePlan* plan,
                             const ExtraRows* extra) {
  // KRS/reedsolomon.go:1453-1501: the first k present rows in index order, decode matrix from the
  // inversion cache (key: the invalid rows met before the k-th valid one).
  std::vector<int> invalid;
  plan->in.clear();
  for (int row = 0; row < total() && (int)plan->in.size() < k_; ++row) {
    if (present[row]) plan->in.push_back(row);
    else invalid.push_back(row);
  }
  if ((int)plan->in.size() < k_) return CFSEC_ERR_TOO_FEW_SHARDS;
  Matrix dec;
  if (!tree_.get(invalid, &dec)) {
    Matrix sub(k_, k_);
    for (int r = 0; r < k_; ++r)
      for (int c = 0; c < k_; ++c) sub.at(r, c) = mat_.at(plan->in[r], c);
    if (!mat_invert(sub, dec)) return CFSEC_ERR_SINGULAR;
    tree_.put(invalid, dec);
  }
  // Stored rows: missing data = dec rows (:1508-1524); missing parity = parity x data, the same
  // linear map over the k inputs as parity_row x dec (:1537-1550).  Compared rows (Verify,
  // :1287-1301, after the reconstruct): every present parity shard outside the k inputs against
  // parity_row x dec.  That is the whole of Verify: present data shards are always among the k
  // inputs (they come first), so the data after the reconstruct is exactly dec x inputs, and a
  // parity shard that is an input or was just rebuilt equals its row by construction.
  plan->out.clear();
  for (int i = 0; i < k_; ++i)
    if (!present[i]) plan->out.push_back(i);
  for (int i = k_; i < total(); ++i)
    if (!present[i]) plan->out.push_back(i);
  plan->nstore = (int)plan->out.size();
  if (verify)
    for (int i = k_; i < total(); ++i)
      if (present[i] && std::find(plan->in.begin(), plan->in.end(), i) == plan->in.end()) plan->out.push_back(i);
  // extra rows over the data (LRC local parities): compared like the parity rows above
  plan->nextra = verify && extra ? (int)extra->idx.size() : 0;
  for (int j = 0; j < plan->nextra; ++j) plan->out.push_back(extra->idx[j]);
  plan->rows = Matrix((int)plan->out.size(), k_);
  const GF& gf = GF::get();
  for (size_t o = 0; o < plan->out.size(); ++o) {
    const int idx = plan->out[o];
    uint8_t* dst = plan->rows.row((int)o);
    if (idx < k_) {
      std::memcpy(dst, dec.row(idx), k_);
    } else {
      const int xo = (int)o - ((int)plan->out.size() - plan->nextra);  // extra row, or < 0
      const uint8_t* p = xo >= 0 ? extra->rows.row(xo) : parity_.row(idx - k_);
      for (int c = 0; c < k_; ++c) {
        uint8_t v = 0;
        for (int j = 0; j < k_; ++j) v ^= gf.mul(p[j], dec.at(j, c));
        dst[c] = v;
      }
    }
  }
  plan_dy16(present, dec, plan, plan->nextra ? extra : nullptr);
  return CFSEC_OK;
}

namespace {
// The parity rows of a 16 + 20 code in the form repair_dy16 takes: rows 0..15 one 16x16 dyadic
// block, rows 16..19 4x4 dyadic blocks (KRS buildMatrix(16, 36): gf_dyadic16.hpp).
bool parity_dy16(const Matrix& p) {
  if (p.rows != 20 || p.cols != 16) return false;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j)
      if (p.at(i, j) != p.at(0, i ^ j)) return false;
  for (int c0 = 0; c0 < 16; c0 += 4)
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j)
        if (p.at(16 + i, c0 + j) != p.at(16, c0 + (i ^ j))) return false;
  return true;
}
}  // namespace

void RSEngine::plan_dy16(const std::vector<bool>& present, const Matrix& dec, StripePlan* plan,
                         const ExtraRows* extra) const {
  plan->dy16.reset();
  static const bool off = std::getenv("CFSEC_NO_DY16_REPAIR") != nullptr;  // A/B switch
  if (off || k_ != 16 || m_ != 20 || !parity_dy16(parity_)) return;
  const int e = extra ? (int)extra->idx.size() : 0;
  if (e != 0 && e != 2) return;  // kernels: 0 or 2 extra rows (EC16P20L2's two local parities)
  auto d = std::make_shared<Dy16Plan>();
  for (int i = 0; i < k_; ++i)
    if (!present[i]) d->rows.push_back(i);
  d->nd = (int)d->rows.size();
  d->e = e;
  // products: 16 per decode row + 117 for the 20 parity rows + 16 per extra row, against 16 per
  // output row
  if (d->nd > 4 || 16 * d->nd + 117 + 16 * e >= 16 * (int)plan->out.size()) return;
  for (int r = 0; r < m_; ++r) d->rows.push_back(k_ + r);
  for (int j = 0; j < e; ++j) d->rows.push_back(extra->idx[j]);
  int slot = 0, j = 0;
  for (int i = 0; i < k_; ++i) d->src[i] = present[i] ? (uint8_t)slot++ : (uint8_t)(16 + j++);
  const int nx0 = (int)plan->out.size() - plan->nextra;
  for (size_t o = 0; o < plan->out.size(); ++o) {
    const int idx = plan->out[o];
    if (idx < k_) continue;
    const int bit = (int)o >= nx0 ? 20 + ((int)o - nx0) : idx - k_;
    (o < (size_t)plan->nstore ? d->pstore : d->pcmp) |= 1u << bit;
  }
  d->coef = Matrix(20 + e + d->nd, 16);
  std::memcpy(d->coef.v.data(), parity_.v.data(), 20 * 16);
  for (int q = 0; q < e; ++q) std::memcpy(d->coef.row(20 + q), extra->rows.row(q), 16);
  for (int q = 0; q < d->nd; ++q) std::memcpy(d->coef.row(20 + e + q), dec.row(d->rows[q]), 16);
  // syndrome form: the inputs past the present data rows are the stand-in parities (first-present
  // order); A[q][j] = parity row prow[q] at missing data column rows[j], invertible exactly when the
  // decode is (block elimination of the 16 x 16 input matrix)
  if (plan->in.size() == 16) {
    bool ok = true;
    Matrix A(d->nd, d->nd), Ai;
    for (int q = 0; q < d->nd && ok; ++q) {
      const int p = plan->in[16 - d->nd + q] - k_;
      ok = p >= 0 && p < 20;
      if (ok) {
        d->prow[q] = (uint8_t)p;
        for (int j = 0; j < d->nd; ++j) A.at(q, j) = parity_.at(p, d->rows[j]);
      }
    }
    if (ok && (d->nd == 0 || mat_invert(A, Ai))) {
      for (int j = 0; j < d->nd; ++j)
        for (int q = 0; q < d->nd; ++q) d->ainv[j * 4 + q] = Ai.at(j, q);
      d->syn = true;
    }
  }
  plan->dy16 = std::move(d);
}

Status RSEngine::encode_stripes(cfsec_shard* const* stripes, int nst, int mem, int* status) {
  if (!stripes || !status || nst < 0) return CFSEC_ERR_INVALID_ARG;
  StripePlan plan;
  for (int i = 0; i < k_; ++i) plan.in.push_back(i);
  for (int i = k_; i < total(); ++i) plan.out.push_back(i);
  plan.nstore = m_;
  plan.rows = parity_;
  std::vector<StripeTask> tasks;
  for (int s = 0; s < nst; ++s) {
    status[s] = CFSEC_OK;
    size_t S = 0;
    Status st = stripes[s] ? stripe_size(stripes[s], total(), false, &S) : CFSEC_ERR_INVALID_ARG;
    for (int i = 0; i < total() && st == CFSEC_OK; ++i)
      if (!stripes[s][i].data) st = CFSEC_ERR_INVALID_ARG;
    if (st != CFSEC_OK) {
      status[s] = st;
      continue;
    }
    if (m_ > 0) tasks.push_back(StripeTask{stripes[s], &plan, S, &status[s], 0, 0, s});
  }
  return run_stripes(tasks, mem);
}

Status RSEngine::stripes_one_by_one(cfsec_shard* const* stripes, int nst, int mem, bool reconstruct, bool verify,
                                   int* status) {
  // More inputs than one compare launch carries (k > kLaunchMaxRows): the single-stripe calls,
  // whose Verify stores into staging and compares there (run(): two_step_verify), stripe by stripe.
  for (int s = 0; s < nst; ++s) {
    Status st = stripes[s] ? CFSEC_OK : CFSEC_ERR_INVALID_ARG;
    if (st == CFSEC_OK && reconstruct) st = this->reconstruct(stripes[s], total(), false, mem, nullptr);
    if (st == CFSEC_OK && verify) {
      bool ok = false;
      st = this->verify(stripes[s], total(), mem, nullptr, &ok);
      if (st == CFSEC_OK && !ok) st = CFSEC_ERR_VERIFY;
    }
    if (st == CFSEC_ERR_DEVICE) return st;
    status[s] = st;
  }
  return CFSEC_OK;
}

Status RSEngine::verify_stripes(cfsec_shard* const* stripes, int nst, int mem, int* status) {
  if (!stripes || !status || nst < 0) return CFSEC_ERR_INVALID_ARG;
  if (k_ > kLaunchMaxRows && m_ > 0) return stripes_one_by_one(stripes, nst, mem, false, true, status);
  StripePlan plan;
  for (int i = 0; i < k_; ++i) plan.in.push_back(i);
  for (int i = k_; i < total(); ++i) plan.out.push_back(i);
  plan.nstore = 0;
  plan.rows = parity_;
  std::vector<StripeTask> tasks;
  for (int s = 0; s < nst; ++s) {
    status[s] = CFSEC_OK;
    size_t S = 0;
    Status st = stripes[s] ? stripe_size(stripes[s], total(), false, &S) : CFSEC_ERR_INVALID_ARG;
    for (int i = 0; i < total() && st == CFSEC_OK; ++i)
      if (!stripes[s][i].data) st = CFSEC_ERR_INVALID_ARG;
    if (st != CFSEC_OK) {
      status[s] = st;
      continue;
    }
    if (m_ > 0) tasks.push_back(StripeTask{stripes[s], &plan, S, &status[s], 0, 0, s});
  }
  return run_stripes(tasks, mem);
}

Status RSEngine::reconstruct_stripes(cfsec_shard* const* stripes, int nst, int mem, bool verify, int* status) {
  if (!stripes || !status || nst < 0) return CFSEC_ERR_INVALID_ARG;
  if (verify && k_ > kLaunchMaxRows && m_ > 0) return stripes_one_by_one(stripes, nst, mem, true, true, status);
  PlanStore store;
  std::vector<StripeTask> tasks;
  plan_reconstruct_tasks(stripes, nst, verify, status, 0, 0, &store, &tasks);
  return run_stripes(tasks, mem);
}

void RSEngine::plan_reconstruct_tasks(cfsec_shard* const* stripes, int nst, bool verify, int* status, int phase,
                                      int owner0, PlanStore* store, std::vector<StripeTask>* tasks,
                                      const ExtraRows* extra, const std::vector<bool>* fuse) {
  StripePlan* vplan = nullptr;  // Verify as an encode-matrix pass (split_verify)
  std::map<const StripePlan*, StripePlan*> store_only;
  tasks->reserve(tasks->size() + (size_t)nst);
  // batches mostly repeat one erasure pattern: the previous stripe's plan is checked first
  std::vector<bool> present(total()), last_present;
  const StripePlan* last_plan = nullptr;
  for (int s = 0; s < nst; ++s) {
    status[s] = CFSEC_OK;
    cfsec_shard* sh = stripes[s];
    size_t S = 0;
    Status st = sh ? stripe_size(sh, total(), true, &S) : CFSEC_ERR_INVALID_ARG;
    if (st != CFSEC_OK) {
      status[s] = st;
      continue;
    }
    int np = 0;
    for (int i = 0; i < total(); ++i) {
      present[i] = sh[i].len != 0;
      np += present[i] ? 1 : 0;
    }
    if (np < k_) {
      status[s] = CFSEC_ERR_TOO_FEW_SHARDS;
      continue;
    }
    const bool fx = verify && extra && fuse && (*fuse)[s];
    if (np == total() && (!verify || (m_ == 0 && !fx))) continue;  // Reconstruct of a full stripe is a no-op
    // plans are keyed by the present shards, plus whether the extra rows ride along
    present.push_back(fx);
    if (!last_plan || present != last_present) {
      present.pop_back();
      last_plan = cached_plan(present, fx, verify, fx ? extra : nullptr, store, &st);
      present.push_back(fx);
      last_present = present;
      if (!last_plan) {
        present.pop_back();
        status[s] = st;
        continue;
      }
    }
    present.pop_back();
    const StripePlan* plan = last_plan;
    for (int r = 0; r < plan->nstore && st == CFSEC_OK; ++r)
      if (!sh[plan->out[r]].data || sh[plan->out[r]].cap < S) st = CFSEC_ERR_INVALID_ARG;
    for (int c : plan->in)
      if (!sh[c].data) st = CFSEC_ERR_INVALID_ARG;
    if (st != CFSEC_OK) {
      set_last_error("reconstruct batch: stripe " + std::to_string(s) + " has a missing shard with cap < shard size");
      status[s] = st;
      continue;
    }
    // KRS/reedsolomon.go:1514-1518: shards[i] = shards[i][0:S]
    for (int r = 0; r < plan->nstore; ++r) sh[plan->out[r]].len = S;
    const StripePlan* use = plan;
    if (split_verify(*plan)) {
      // Verify as a second pass over the whole stripe with the encoding matrix instead of compared
      // rows in the reconstruct pass: the compared rows (parity_row x dec over the k inputs) have
      // no structure, the parity rows over the data do (dyadic kernels)
      StripePlan*& so = store_only[plan];
      if (!so) {
        StripePlan cut = *plan;
        cut.dy16.reset();
        cut.out.resize(cut.nstore);
        cut.rows = Matrix(cut.nstore, k_);
        std::memcpy(cut.rows.v.data(), plan->rows.v.data(), (size_t)cut.nstore * k_);
        so = store->add(cut);
      }
      if (!vplan) {
        StripePlan v;
        for (int i = 0; i < k_; ++i) v.in.push_back(i);
        for (int i = k_; i < total(); ++i) v.out.push_back(i);
        v.nstore = 0;
        v.rows = parity_;
        vplan = store->add(v);
      }
      use = so;
      StripeTask vt{sh, vplan, S, &status[s], 0, phase + 1, owner0 + s};
      tasks->push_back(vt);
    }
    if (!use->out.empty()) tasks->push_back(StripeTask{sh, use, S, &status[s], 0, phase, owner0 + s});
  }
}

const StripePlan* RSEngine::cached_plan(const std::vector<bool>& present, bool fx, bool verify,
                                        const ExtraRows* extra, PlanStore* store, Status* st) {
  std::vector<bool> key = present;
  key.push_back(fx);
  key.push_back(verify);
  {
    std::lock_guard<std::mutex> l(plan_mu_);
    auto it = plan_cache_.find(key);
    if (it != plan_cache_.end()) return it->second.get();
  }
  std::unique_ptr<StripePlan> p(new StripePlan());
  *st = plan_stripe(present, verify, p.get(), extra);
  if (*st != CFSEC_OK) return nullptr;
  std::lock_guard<std::mutex> l(plan_mu_);
  auto it = plan_cache_.find(key);  // another caller may have planned it meanwhile
  if (it != plan_cache_.end()) return it->second.get();
  if (plan_cache_.size() < kMaxCachedPlans) return plan_cache_.emplace(std::move(key), std::move(p)).first->second.get();
  return store->add(*p);
}

bool RSEngine::split_verify(const StripePlan& p) const {
  const int checks = (int)p.out.size() - p.nstore;
  if (checks <= 0 || p.nextra > 0) return false;
  static const int mode = [] {
    const char* e = getenv("CFSEC_VERIFY_SPLIT");
    return e ? atoi(e) : -1;
  }();
  if (mode >= 0) return mode != 0;
  return false;
}

Status RSEngine::run_stripes(std::vector<StripeTask>& tasks, int mem, const AsyncOut* async, const CrcOut* crc) {
  if (tasks.empty()) return CFSEC_OK;
  if (devs_.empty()) {
    set_last_error("no HIP device available to the cfsec engine");
    return CFSEC_ERR_DEVICE;
  }
  if (mem != CFSEC_MEM_HOST && mem != CFSEC_MEM_DEVICE) return CFSEC_ERR_INVALID_ARG;
  const int nd = async ? 1 : (int)devs_.size();
  if (mem == CFSEC_MEM_DEVICE && nd == 1) {
    // one device: the batch's memory must live on it (checked on the first stripe; per-stripe
    // pointer queries cost ~1 us each)
    const int d = device_of(tasks[0].shards[tasks[0].plan->in[0]].data);
    if (d != devs_[0]->device()) {
      set_last_error("stripe batch: device memory on device " + std::to_string(d) + ", the handle runs on device " +
                     std::to_string(devs_[0]->device()));
      return CFSEC_ERR_INVALID_ARG;
    }
  } else if (mem == CFSEC_MEM_DEVICE) {
    // device memory runs where it lives
    for (auto& t : tasks) {
      const int d = device_of(t.shards[t.plan->in[0]].data);
      int idx = -1;
      for (int i = 0; i < nd; ++i)
        if (devs_[i]->device() == d) idx = i;
      if (idx < 0) {
        set_last_error("stripe batch: device memory on device " + std::to_string(d) +
                       ", which is not one of the handle's devices");
        return CFSEC_ERR_INVALID_ARG;
      }
      t.dev = idx;
    }
  } else {
    // host memory: contiguous runs of batch items, balanced by the bytes each moves; every task of
    // an item (its phases) on one device, so a later phase reads what an earlier one wrote
    std::map<int, uint64_t> per_owner;
    for (auto& t : tasks) per_owner[t.owner] += uint64_t(t.len) * (t.plan->in.size() + t.plan->out.size());
    std::vector<uint64_t> bytes;
    std::map<int, int> slot;
    for (auto& kv : per_owner) {
      slot[kv.first] = (int)bytes.size();
      bytes.push_back(kv.second);
    }
    std::vector<int> dev(bytes.size());
    partition_stripes(bytes.data(), (int)bytes.size(), nd, dev.data());
    for (auto& t : tasks) t.dev = dev[slot[t.owner]];
  }
  std::vector<std::vector<StripeTask*>> per(nd);
  for (auto& t : tasks) per[t.dev].push_back(&t);
  const bool trace = std::getenv("CFSEC_TRACE_BATCH") != nullptr;  // the split, for tests
  if (trace)
    for (int d = 0; d < nd; ++d) {
      std::set<int> items;
      for (StripeTask* t : per[d]) items.insert(t->owner);
      std::fprintf(stderr, "cfsec batch: device index %d (ordinal %d): %zu tasks, items", d, devs_[d]->device(),
                   per[d].size());
      for (int it : items) std::fprintf(stderr, " %d", it);
      std::fprintf(stderr, "\n");
    }
  std::vector<Status> st(nd, CFSEC_OK);
  std::vector<std::string> err(nd);
  std::vector<std::thread> threads;
  for (int d = 1; d < nd; ++d)
    if (!per[d].empty())
      threads.emplace_back([&, d] {
        st[d] = run_device(per[d], mem, devs_[d], nullptr, crc);
        if (st[d] != CFSEC_OK) err[d] = last_error_cstr();
      });
  if (!per[0].empty()) st[0] = run_device(per[0], mem, devs_[0], async, crc);
  for (auto& th : threads) th.join();
  for (int d = 1; d < nd; ++d)
    if (st[d] != CFSEC_OK && st[0] == CFSEC_OK) {
      set_last_error(err[d]);
      return st[d];
    }
  return st[0];
}

Status RSEngine::run_device(std::vector<StripeTask*>& tasks, int mem, DeviceContext* ctx, const AsyncOut* async,
                            const CrcOut* crc) {
  HostTimer whole("  run_device");
  std::unique_ptr<HostTimer> tm(new HostTimer("    classify + acquire"));
  DeviceGuard g(ctx->device());
  if (!g.ok()) return hip_status(hipErrorInvalidDevice, "hipSetDevice");
  const int n = (int)tasks.size();
  // which stripes the GPU addresses in place (device memory, or page-locked host memory on every
  // row the product touches) and which go through staging (pageable host memory)
  std::vector<StripeTask*> direct, staged;
  std::map<std::pair<const StripeTask*, int>, uint8_t*> alias;
  int nphase = 1, nitems = 0;
  bool checks = false;  // some task compares rows (Verify)
  bool sums = false;    // some task checksums rows
  for (StripeTask* t : tasks) {
    sums = sums || (t->crc && crc && crc->words && crc->n);
    nphase = std::max(nphase, t->phase + 1);
    nitems = std::max(nitems, t->owner + 1);
    checks = checks || t->plan->out.size() > (size_t)t->plan->nstore;
    bool in_place = true;
    if (mem == CFSEC_MEM_HOST) {
      for (int c : t->plan->in) {
        uint8_t* d = nullptr;
        in_place = in_place && device_alias(t->shards[c].data, &d);
        alias[{t, c}] = d;
      }
      for (int o : t->plan->out) {
        uint8_t* d = nullptr;
        in_place = in_place && device_alias(t->shards[o].data, &d);
        alias[{t, o}] = d;
      }
    }
    (in_place ? direct : staged).push_back(t);
  }
  if (async && (!staged.empty() || (checks && !async->flags))) return CFSEC_ERR_INVALID_ARG;
  // staging lanes: each holds whole stripes, at least the largest one
  size_t lane_bytes = 0, staged_total = 0;
  for (StripeTask* t : staged) {
    const size_t b = align_up(t->len, kSlot) * (t->plan->in.size() + t->plan->out.size());
    lane_bytes = std::max(lane_bytes, b);
    staged_total += b;
  }
  if (!staged.empty()) lane_bytes = std::max(lane_bytes, std::min(kLaneBudget, staged_total));
  // two lanes only for staged chunks (a second phase of in-place stripes follows the first on one
  // stream)
  const int nlanes = !staged.empty() && (staged_total > lane_bytes || nphase > 1) ? 2 : 1;
  DeviceContext::Workspace* ws = nullptr;
  Status st = ctx->acquire(lane_bytes * nlanes, (size_t)std::max(n, nitems), &ws, (size_t)n,
                           sums && !async ? crc->n : 0);
  if (st != CFSEC_OK) return st;
  // checksum words: the caller's device array (asynchronous) or the workspace's, zeroed first (the
  // CRC kernel XOR-accumulates)
  uint32_t* dcrc = !sums ? nullptr : async ? crc->words : ws->dcrc;
  // asynchronous calls run on the caller's stream (NULL: the legacy default stream); synchronous
  // ones on the workspace's streams, ordered after the legacy default stream for device memory
  hipStream_t lane[2] = {async ? async->stream : ws->stream, ws->stream2};
  // lane `to` waits for everything queued on lane `from` so far
  const auto join = [&](int from, int to) {
    Status e = hip_status(hipEventRecord(ws->ev, lane[from]), "hipEventRecord");
    if (e == CFSEC_OK) e = hip_status(hipStreamWaitEvent(lane[to], ws->ev, 0), "hipStreamWaitEvent");
    return e;
  };
  if (mem == CFSEC_MEM_DEVICE && !async) st = ctx->order_after_default(ws);
  // Zeroed inline on lane 0: a memset on lane 1 beside the first products, waited for by the first
  // checksum launch, measured slower (C5 +26 instead of +14 us, EC12P4 fused encode + CRC 246
  // instead of 224 us: the cross-stream wait costs more than the 10 KiB fill it hides).  When the
  // first launch is a 16x16-dyadic repair (C5's tasklet) its workgroup (0, 0) zeroes the words and
  // the memset launch goes (zero_first below).
  bool zero_first = false;
  if (sums && nlanes == 1 && nphase == 1 && !direct.empty()) {
    const StripeTask* t0 = direct.front();
    zero_first = t0->plan->dy16 && t0->phase == 0 && crc->n <= 0xFFFFFFFFu;
  }
  if (st == CFSEC_OK && sums && !zero_first)
    st = hip_status(hipMemsetAsync(dcrc, 0, crc->n * 4, lane[0]), "hipMemsetAsync(crc)");
  if (st == CFSEC_OK && nlanes > 1) st = join(0, 1);
  // crc32.ChecksumIEEE of the rows the tasks of a launched part name, on the part's stream, from the
  // same device addresses the product used (staged rows before their lane is reused)
  const auto checksum = [&](const std::vector<StripeTask*>& part, auto ptr, hipStream_t s) -> Status {
    if (!sums) return CFSEC_OK;
    std::map<size_t, std::pair<std::vector<const uint8_t*>, std::vector<uint32_t>>> by_len;
    for (StripeTask* t : part) {
      if (!t->crc || t->len == 0) continue;
      auto& v = by_len[t->len];
      const auto add = [&](int row) {
        const int64_t w = t->crc_word + (t->crc_map ? t->crc_map[row] : row);
        if (w < 0 || (size_t)w >= crc->n) return;
        v.first.push_back(ptr(t, row));
        v.second.push_back((uint32_t)w);
      };
      if (t->crc == 2)
        for (int c : t->plan->in) add(c);
      for (int r = 0; r < t->plan->nstore; ++r) add(t->plan->out[r]);
    }
    for (auto& kv : by_len) {
      const Status e = hip_status(launch_crc32_to(kv.second.first.data(), kv.first, (int)kv.second.first.size(), dcrc,
                                                  kv.second.second.data(), crc32_shift_ones(kv.first), s),
                                  "launch_crc32_to(batch)");
      if (e != CFSEC_OK) return e;
    }
    return CFSEC_OK;
  };
  std::map<int, int> tasks_per_owner;  // a bid with several checksummed tasks keeps the separate pass
  for (StripeTask* t : tasks)          // (EnableVerify's compare task writes no words: not counted)
    if (t->crc) ++tasks_per_owner[t->owner];
  int next_flag = 0;
  // Verify flags.  A group whose tasks belong to consecutive items writes each mismatch straight
  // into the items' words -- the caller's device array (asynchronous) or the pinned host words,
  // zeroed here first (synchronous) -- so no gather launch follows it (C4 / C5: one tasklet group,
  // -4 us of device time per call).  Other groups use per-task words and the gather.
  // CFSEC_BATCH_DIRECT_FLAGS=0: the gather always (A/B).
  static const bool kDirect = [] {
    const char* v = std::getenv("CFSEC_BATCH_DIRECT_FLAGS");
    return !(v && v[0] == '0');
  }();
  uint32_t* fdirect = checks && kDirect ? (async ? async->flags : ws->hflags_dev) : nullptr;
  if (fdirect && !async)
    for (StripeTask* t : tasks) ws->hflags[t->owner] = 0;
  const auto route = [&](std::vector<Group>& groups) {
    if (!fdirect) return;
    for (Group& gr : groups) {
      if (gr.plan->out.size() <= (size_t)gr.plan->nstore) continue;  // nothing compared
      bool consecutive = true;
      for (size_t i = 1; i < gr.tasks.size() && consecutive; ++i)
        consecutive = gr.tasks[i]->owner == gr.tasks[0]->owner + (int)i;
      if (consecutive) gr.direct = fdirect + gr.tasks[0]->owner;
    }
  };
  std::vector<std::pair<StripeTask*, int>> flags;  // (task, flag word; -1: written directly)
  const auto record = [&](const std::vector<Group>& groups) {
    for (const Group& gr : groups)
      for (size_t i = 0; i < gr.tasks.size(); ++i) flags.emplace_back(gr.tasks[i], gr.direct ? -1 : gr.flag0 + (int)i);
  };
  int chunk = 0;
  tm.reset(new HostTimer("    group + launch"));
  for (int ph = 0; ph < nphase && st == CFSEC_OK; ++ph) {
    if (ph > 0 && nlanes > 1) {  // a phase starts after everything of the previous one, on both lanes
      st = join(1, 0);
      if (st == CFSEC_OK) st = join(0, 1);
    }
    // in-place stripes: one set of launches on lane 0
    std::vector<StripeTask*> dph, sph;
    for (StripeTask* t : direct)
      if (t->phase == ph) dph.push_back(t);
    for (StripeTask* t : staged)
      if (t->phase == ph) sph.push_back(t);
    if (st == CFSEC_OK && !dph.empty()) {
      const auto dptr = [&](const StripeTask* t, int idx) {
        return mem == CFSEC_MEM_DEVICE ? (const uint8_t*)t->shards[idx].data : (const uint8_t*)alias[{t, idx}];
      };
      std::unique_ptr<HostTimer> gt(new HostTimer("      make_groups"));
      std::vector<Group> groups = make_groups(dph, &next_flag, dptr);
      route(groups);
      gt.reset();
      // dy16 groups that checksum their rebuilt rows in the repair pass itself
      std::vector<std::vector<char>> crc_done(groups.size());
      bool any_crc_fused = false;
      if (sums)
        for (size_t gi = 0; gi < groups.size(); ++gi)
          any_crc_fused |= dy16_crc_group(groups[gi], dcrc, crc->n, tasks_per_owner, &crc_done[gi]);
      if (zero_first) {  // make_groups keeps first-appearance order: groups[0] holds direct.front()
        if (!groups.empty() && groups[0].plan->dy16 && !any_crc_fused) {
          groups[0].zero_words = dcrc;
          groups[0].nzero = (uint32_t)crc->n;
        } else {  // (the repair pass's checksum atomics must find the words zeroed already)
          st = hip_status(hipMemsetAsync(dcrc, 0, crc->n * 4, lane[0]), "hipMemsetAsync(crc)");
        }
        zero_first = false;
      }
      std::set<const StripeTask*> fused;  // tasks whose checksums a fused product + CRC launch took
      for (size_t gi = 0; gi < groups.size(); ++gi) {
        const Group& gr = groups[gi];
        if (st != CFSEC_OK) break;
        if (sums && fused_crc_group(gr, dcrc, crc->n, tasks_per_owner, lane[0], &st)) {
          fused.insert(gr.tasks.begin(), gr.tasks.end());
          continue;
        }
        {
          HostTimer lt("      launch_group");
          st = hip_status(launch_group(gr, ws->bflags, lane[0]), "launch_matvec(batch)");
        }
        if (gr.crc_done) {
          int nf = 0;
          for (size_t i = 0; i < gr.tasks.size(); ++i)
            if ((*gr.crc_done)[i]) {
              fused.insert(gr.tasks[i]);
              ++nf;
            }
          if (std::getenv("CFSEC_TRACE_BATCH"))
            std::fprintf(stderr, "cfsec batch: repair-pass crc group tasks=%zu fused=%d\n", gr.tasks.size(), nf);
        }
      }
      record(groups);
      if (st == CFSEC_OK) {
        std::vector<StripeTask*> rest;
        for (StripeTask* t : dph)
          if (!fused.count(t)) rest.push_back(t);
        st = checksum(rest, dptr, lane[0]);
      }
    }
    // staged stripes: chunks of whole stripes alternating over the two lanes; each lane copies its
    // chunk in, runs it and copies the stored rows back while the other lane's chunk moves
    size_t i0 = 0;
    for (; st == CFSEC_OK && i0 < sph.size(); ++chunk) {
      const int l = chunk % nlanes;
      hipStream_t s = lane[l];
      uint8_t* base = ws->dbuf + lane_bytes * l;
      size_t used = 0, i1 = i0;
      std::map<std::pair<const StripeTask*, int>, uint8_t*> slot;
      while (i1 < sph.size()) {
        StripeTask* t = sph[i1];
        const size_t sl = align_up(t->len, kSlot);
        const size_t need = sl * (t->plan->in.size() + t->plan->out.size());
        if (i1 > i0 && used + need > lane_bytes) break;
        for (int c : t->plan->in) {
          slot[{t, c}] = base + used;
          used += sl;
        }
        for (int o : t->plan->out) {
          slot[{t, o}] = base + used;
          used += sl;
        }
        ++i1;
      }
      std::vector<StripeTask*> part(sph.begin() + i0, sph.begin() + i1);
      for (StripeTask* t : part) {
        for (int c : t->plan->in)
          if (st == CFSEC_OK)
            st = hip_status(hipMemcpyAsync(slot[{t, c}], t->shards[c].data, t->len, hipMemcpyHostToDevice, s),
                            "hipMemcpyAsync H2D");
        for (size_t r = t->plan->nstore; r < t->plan->out.size(); ++r)
          if (st == CFSEC_OK) {
            const int o = t->plan->out[r];
            st = hip_status(hipMemcpyAsync(slot[{t, o}], t->shards[o].data, t->len, hipMemcpyHostToDevice, s),
                            "hipMemcpyAsync H2D");
          }
      }
      const auto sptr = [&](const StripeTask* t, int idx) { return (const uint8_t*)slot[{t, idx}]; };
      std::vector<Group> groups = make_groups(part, &next_flag, sptr);
      route(groups);
      for (const Group& gr : groups)
        if (st == CFSEC_OK) st = hip_status(launch_group(gr, ws->bflags, s), "launch_matvec(batch)");
      record(groups);
      if (st == CFSEC_OK) st = checksum(part, sptr, s);
      for (StripeTask* t : part)
        for (int r = 0; r < t->plan->nstore && st == CFSEC_OK; ++r) {
          const int o = t->plan->out[r];
          st = hip_status(hipMemcpyAsync(t->shards[o].data, slot[{t, o}], t->len, hipMemcpyDeviceToHost, s),
                          "hipMemcpyAsync D2H");
        }
      i0 = i1;
    }
  }
  if (st == CFSEC_OK && nlanes > 1) st = join(1, 0);
  if (st == CFSEC_OK && sums && !async)
    st = hip_status(hipMemcpyAsync(ws->hcrc, ws->dcrc, crc->n * 4, hipMemcpyDeviceToHost, lane[0]),
                    "hipMemcpyAsync D2H(crc)");
  // Verify flags per batch item, gathered from the per-task words (which the gather resets): into
  // the caller's device array (asynchronous), or straight into the pinned host words (no D2H copy)
  if (st == CFSEC_OK && checks) {
    std::vector<std::pair<int, int>> pairs;
    for (auto& f : flags)
      if (f.second >= 0 && f.first->plan->out.size() > (size_t)f.first->plan->nstore)
        pairs.emplace_back(f.first->owner, f.second);
    std::sort(pairs.begin(), pairs.end());
    std::vector<int> item(pairs.size()), word(pairs.size());
    for (size_t i = 0; i < pairs.size(); ++i) item[i] = pairs[i].first, word[i] = pairs[i].second;
    st = hip_status(launch_flag_gather(ws->bflags, async ? async->flags : ws->hflags_dev, item.data(), word.data(),
                                       (int)pairs.size(), async != nullptr || fdirect != nullptr, lane[0]),
                    "launch_flag_gather");
  }
  if (st != CFSEC_OK) ws->bflags_clean = false;  // some task words may be left set: memset on reuse
  if (async) {
    tm.reset();
    ctx->release_after(ws, lane[0]);
    return st;
  }
  tm.reset(new HostTimer("    sync"));
  for (int l = 0; l < nlanes; ++l) {
    const Status sync = ctx->finish(ws, lane[l]);
    if (st == CFSEC_OK) st = sync;
  }
  tm.reset();
  if (st == CFSEC_OK && checks)
    for (auto& f : flags)
      if (f.first->plan->out.size() > (size_t)f.first->plan->nstore && ws->hflags[f.first->owner] != 0 &&
          *f.first->status == CFSEC_OK)
        *f.first->status = CFSEC_ERR_VERIFY;
  if (st == CFSEC_OK && sums)  // this device's words only (another device of the call fills the rest)
    for (StripeTask* t : tasks) {
      if (!t->crc) continue;
      const auto put = [&](int row) {
        const int64_t w = t->crc_word + (t->crc_map ? t->crc_map[row] : row);
        if (w >= 0 && (size_t)w < crc->n) crc->words[w] = ws->hcrc[w];
      };
      if (t->crc == 2)
        for (int c : t->plan->in) put(c);
      for (int r = 0; r < t->plan->nstore; ++r) put(t->plan->out[r]);
    }
  ctx->release(ws);
  return st;
}

}  // namespace cfsec

// ---------------------------------------------------------------- ec.Encoder batches

namespace cfsec {

namespace {
// Synchronous calls return checksums only for the items that succeeded (the reference checksums
// after a successful Encode / repair): the words of a failed item are zeroed.  (Asynchronous calls
// learn a false Verify on the stream; their caller skips the words of flagged items.)
void clear_failed_crcs(const CrcOut* crc, const AsyncOut* async, const int* status, int nitems, int n) {
  if (!crc || async) return;
  for (int b = 0; b < nitems; ++b)
    if (status[b] != CFSEC_OK)
      for (int i = 0; i < n && (size_t)b * n + i < crc->n; ++i) crc->words[(size_t)b * n + i] = 0;
}
}  // namespace

Status ECEncoder::set_devices(const int* devices, int n) { return engine_->set_devices(devices, n); }

Status LrcEncoder::set_devices(const int* devices, int n) {
  Status st = engine_->set_devices(devices, n);
  return st != CFSEC_OK ? st : local_->set_devices(devices, n);
}

Status ECEncoder::reconstruct_batch(cfsec_shard* shards, int n, int nbids, const int* bad, const int* bad_off,
                                    int mem, bool verify, int* status, const AsyncOut* async, const CrcOut* crc) {
  // encoder.go:139-144 per bid (initBadShards, engine Reconstruct), then encoder.go:133-137 (Verify)
  if (!shards || !status || !bad_off || nbids < 0) return CFSEC_ERR_INVALID_ARG;
  Slot slot(pool_.get());
  std::vector<cfsec_shard*> stripes;
  std::vector<int> pos;
  for (int b = 0; b < nbids; ++b) {
    status[b] = CFSEC_OK;
    cfsec_shard* sh = shards + (size_t)b * n;
    if (n != engine_->total()) {
      status[b] = CFSEC_ERR_TOO_FEW_SHARDS;  // reedsolomon.go:1408-1410
      continue;
    }
    const Status st = init_bad_shards(sh, n, std::vector<int>(bad + bad_off[b], bad + bad_off[b + 1]));
    if (st != CFSEC_OK) {
      status[b] = st;
      continue;
    }
    stripes.push_back(sh);
    pos.push_back(b);
  }
  std::vector<int> st(stripes.size());
  Status rc;
  if (verify && engine_->k() > kLaunchMaxRows) {
    // the single-stripe path is synchronous on its own streams: not for the checksummed or the
    // asynchronous forms (no code mode of SURVEY §8 has more than 16 inputs)
    if (crc || async) return CFSEC_ERR_NOT_SUPPORTED;
    rc = engine_->reconstruct_stripes(stripes.data(), (int)stripes.size(), mem, verify, st.data());
  } else {
    PlanStore store;
    std::vector<StripeTask> tasks;
    engine_->plan_reconstruct_tasks(stripes.data(), (int)stripes.size(), verify, st.data(), 0, 0, &store, &tasks);
    for (auto& t : tasks) {
      t.owner = pos[t.owner];  // the bid: its verify word
      t.crc = crc ? 1 : 0;     // the rebuilt shards' checksums (blobnode ShardCrc32)
      t.crc_word = (int64_t)t.owner * n;
    }
    rc = engine_->run_stripes(tasks, mem, async, crc);
  }
  for (size_t i = 0; i < pos.size(); ++i) status[pos[i]] = st[i];
  clear_failed_crcs(crc, async, status, nbids, n);
  return rc;
}

Status LrcEncoder::reconstruct_batch(cfsec_shard* shards, int n, int nbids, const int* bad, const int* bad_off,
                                     int mem, bool verify, int* status, const AsyncOut* async, const CrcOut* crc) {
  // lrcencoder.go:133-186 per bid, then lrcencoder.go:89-131 (Verify): a local stripe (n = its size)
  // is the local engine alone; a whole stripe is the global engine over its first N+M shards, then
  // each AZ's local engine over that AZ's local stripe -- planned together and run as two phases of
  // one call (one sync), in that order, as the reference runs them.
  if (!shards || !status || !bad_off || nbids < 0) return CFSEC_ERR_INVALID_ARG;
  HostTimer whole("lrc reconstruct_batch");
  const int N = t_.n, M = t_.m, L = t_.l, AZ = t_.az_count;
  const int lsz = (N + M + L) / AZ;
  if (verify && std::max(N, local_->k()) > kLaunchMaxRows) {
    if (crc || async) return CFSEC_ERR_NOT_SUPPORTED;  // synchronous bid-by-bid path only
    // compared rows over more than one launch's inputs: the single calls, bid by bid (each takes
    // its own concurrency slot)
    for (int b = 0; b < nbids; ++b) {
      cfsec_shard* sh = shards + (size_t)b * n;
      Status st = reconstruct(sh, n, bad + bad_off[b], bad_off[b + 1] - bad_off[b], mem, nullptr);
      if (st == CFSEC_OK) {
        bool ok = false;
        st = this->verify(sh, n, mem, nullptr, &ok);
        if (st == CFSEC_OK && !ok) st = CFSEC_ERR_VERIFY;
      }
      if (st == CFSEC_ERR_DEVICE) return st;
      status[b] = st;
    }
    return CFSEC_OK;
  }
  Slot slot(pool_.get());
  std::unique_ptr<HostTimer> ph(new HostTimer("  init/fill"));
  std::vector<cfsec_shard*> stripes;
  std::vector<int> pos;
  for (int b = 0; b < nbids; ++b) {
    status[b] = CFSEC_OK;
    cfsec_shard* sh = shards + (size_t)b * n;
    if (n != lsz && n != N + M + L) {
      status[b] = CFSEC_ERR_INVALID_SHARDS;
      continue;
    }
    Status st = fill_full_shards(sh, n);
    std::vector<int> global_bad;
    for (int i = bad_off[b]; i < bad_off[b + 1]; ++i)
      if (bad[i] < N + M) global_bad.push_back(bad[i]);
    if (st == CFSEC_OK) st = init_bad_shards(sh, n, global_bad);
    if (st != CFSEC_OK) {
      status[b] = st;
      continue;
    }
    stripes.push_back(sh);
    pos.push_back(b);
  }
  if (n == lsz) {  // local stripes: local engine only (lrcencoder.go:93-99, 147-152)
    std::vector<int> st(stripes.size());
    PlanStore store;
    std::vector<StripeTask> tasks;
    local_->plan_reconstruct_tasks(stripes.data(), (int)stripes.size(), verify, st.data(), 0, 0, &store, &tasks);
    for (auto& t : tasks) {
      t.owner = pos[t.owner];
      t.crc = crc ? 1 : 0;
      t.crc_word = (int64_t)t.owner * n;
    }
    const Status rc = local_->run_stripes(tasks, mem, async, crc);
    for (size_t i = 0; i < pos.size(); ++i) status[pos[i]] = st[i];
    clear_failed_crcs(crc, async, status, nbids, n);
    return rc;
  }
  // phase 0 (1): global Reconstruct (+ global Verify) over shards [0, N+M)
  ph.reset(new HostTimer("  global plan"));
  PlanStore gstore, lstore;
  std::vector<StripeTask> tasks;
  std::vector<int> st1(stripes.size());
  // A bid with no bad local shard has its local Verify done in the global pass: every local
  // parity is a fixed row over the data (fused_, as in the fused LRC encode), compared there --
  // the local pass would re-read the 2 x 19 shards of the AZs (C5: 74 -> 38 shard reads per bid).
  ExtraRows extra;
  std::vector<bool> fuse(stripes.size(), false);
  if (verify && L > 0) {
    extra.rows = Matrix(L, N);
    std::memcpy(extra.rows.v.data(), fused_.row(M), (size_t)L * N);
    for (int j = 0; j < L; ++j) extra.idx.push_back(N + M + j);
    for (size_t i = 0; i < stripes.size(); ++i) {
      const cfsec_shard* sh = stripes[i];
      const int b = pos[i];
      bool ok = true;
      for (int j = bad_off[b]; j < bad_off[b + 1]; ++j) ok = ok && bad[j] < N + M;
      size_t S = 0;
      for (int g = 0; g < N + M && !S; ++g) S = sh[g].len;
      for (int j = 0; j < L; ++j) ok = ok && sh[N + M + j].data && sh[N + M + j].len == S && S != 0;
      fuse[i] = ok;
    }
  }
  engine_->plan_reconstruct_tasks(stripes.data(), (int)stripes.size(), verify, st1.data(), 0, 0, &gstore, &tasks,
                                  verify && L > 0 ? &extra : nullptr, &fuse);
  int lphase = 1;
  for (auto& t : tasks) lphase = std::max(lphase, t.phase + 1);
  ph.reset(new HostTimer("  local views + plan"));
  // then every AZ's local stripe (copied headers, lrcencoder.go:236-243) with the rebuilt global
  // shards' lengths already set: local Reconstruct of its bad local shards (index remap
  // lrcencoder.go:161-171) (+ local Verify)
  // per AZ, in bid order: an AZ's views of bids carved from one pitched buffer sit at one stride
  // from each other, so each AZ runs as one affine launch
  // views[a]: AZ a's local stripes of the bids, lsz headers each, back to back
  std::vector<std::vector<cfsec_shard>> views(AZ);
  std::vector<std::vector<size_t>> vowner(AZ);
  std::vector<std::vector<int>> idc(AZ), local_bad(AZ);
  for (int a = 0; a < AZ; ++a) {
    idc[a] = shards_in_idc(a);
    views[a].reserve(stripes.size() * idc[a].size());
    vowner[a].reserve(stripes.size());
  }
  for (size_t i = 0; i < stripes.size(); ++i) {
    if (st1[i] != CFSEC_OK) continue;  // Reconstruct failed: no local pass
    cfsec_shard* sh = stripes[i];
    const int b = pos[i];
    for (auto& v : local_bad) v.clear();
    for (int j = bad_off[b]; j < bad_off[b + 1]; ++j)
      if (bad[j] >= N + M) {
        const int a = (bad[j] - N - M) * AZ / L;
        local_bad[a].push_back(bad[j] - N - M - L / AZ * a + (N + M) / AZ);
      }
    for (int a = 0; a < AZ; ++a) {
      const bool has_bad = !local_bad[a].empty();
      if (!has_bad && (!verify || fuse[i])) continue;  // nothing to rebuild; Verify done (or not asked)
      const size_t at = views[a].size();
      for (int g : idc[a]) views[a].push_back(sh[g]);
      cfsec_shard* ls = views[a].data() + at;
      if (has_bad) {
        const Status s = init_bad_shards(ls, (int)idc[a].size(), local_bad[a]);
        if (s != CFSEC_OK) {
          st1[i] = s;
          views[a].resize(at);
          break;
        }
      }
      vowner[a].push_back(i);
    }
  }
  std::vector<cfsec_shard*> lp;
  std::vector<size_t> owner;
  std::vector<int> vaz;  // the AZ of each local view
  for (int a = 0; a < AZ; ++a)
    for (size_t v = 0; v < vowner[a].size(); ++v) {
      lp.push_back(views[a].data() + v * idc[a].size());
      owner.push_back(vowner[a][v]);
      vaz.push_back(a);
    }
  std::vector<int> st2(lp.size());
  const size_t first_local = tasks.size();
  local_->plan_reconstruct_tasks(lp.data(), (int)lp.size(), verify, st2.data(), lphase, 0, &lstore, &tasks);
  for (size_t t = first_local; t < tasks.size(); ++t) {
    // owner: the bid (a host batch keeps a bid's passes on one device)
    const size_t v = (size_t)(tasks[t].status - st2.data());
    tasks[t].owner = (int)owner[v];
    tasks[t].crc_map = idc[vaz[v]].data();  // local index -> global shard index
  }
  ph.reset();
  for (auto& t : tasks) {
    t.owner = pos[t.owner];  // the bid: its device, its verify word
    t.crc = crc ? 1 : 0;     // rebuilt shards, global or local (blobnode ShardCrc32)
    t.crc_word = (int64_t)t.owner * n;
  }
  const Status rc = engine_->run_stripes(tasks, mem, async, crc);
  // per bid: a Reconstruct error (global, then local) wins over a failed Verify
  std::vector<int> local_err(stripes.size(), CFSEC_OK);
  for (size_t v = 0; v < lp.size(); ++v) {
    int& e = local_err[owner[v]];
    if (st2[v] != CFSEC_OK && (e == CFSEC_OK || (e == CFSEC_ERR_VERIFY && st2[v] != CFSEC_ERR_VERIFY))) e = st2[v];
  }
  for (size_t i = 0; i < stripes.size(); ++i) {
    int s = st1[i];
    if (s == CFSEC_OK || s == CFSEC_ERR_VERIFY) {
      if (local_err[i] != CFSEC_OK && local_err[i] != CFSEC_ERR_VERIFY) s = local_err[i];
      else if (s == CFSEC_OK) s = local_err[i];
    }
    status[pos[i]] = s;
  }
  clear_failed_crcs(crc, async, status, nbids, n);
  return rc;
}

Status ECEncoder::encode_batch(cfsec_shard* shards, int n, int nstripes, int mem, int* status,
                               const AsyncOut* async, const CrcOut* crc) {
  // encoder.go:114-131 per stripe: engine Encode, then Verify when EnableVerify -- the Verify pass in
  // the same call (phase 1), after the encode
  if (!shards || !status || nstripes < 0) return CFSEC_ERR_INVALID_ARG;
  Slot slot(pool_.get());
  const int k = engine_->k(), m = engine_->m(), tot = k + m;
  if (enable_verify_ && k > kLaunchMaxRows) {  // compared rows over more inputs than one launch carries
    if (crc || async) return CFSEC_ERR_NOT_SUPPORTED;  // synchronous stripe-by-stripe path only
    std::vector<cfsec_shard*> stripes;
    std::vector<int> pos;
    for (int s = 0; s < nstripes; ++s) {
      status[s] = n != tot ? CFSEC_ERR_TOO_FEW_SHARDS : CFSEC_OK;
      if (n == tot) stripes.push_back(shards + (size_t)s * n), pos.push_back(s);
    }
    std::vector<int> st(stripes.size());
    Status rc = engine_->encode_stripes(stripes.data(), (int)stripes.size(), mem, st.data());
    std::vector<cfsec_shard*> ok;
    std::vector<size_t> okp;
    for (size_t i = 0; i < stripes.size(); ++i)
      if (st[i] == CFSEC_OK) ok.push_back(stripes[i]), okp.push_back(i);
    std::vector<int> vs(ok.size());
    if (rc == CFSEC_OK) rc = engine_->verify_stripes(ok.data(), (int)ok.size(), mem, vs.data());
    for (size_t i = 0; i < ok.size(); ++i) st[okp[i]] = vs[i];
    for (size_t i = 0; i < pos.size(); ++i) status[pos[i]] = st[i];
    return rc;
  }
  StripePlan plan;
  for (int i = 0; i < k; ++i) plan.in.push_back(i);
  for (int i = k; i < tot; ++i) plan.out.push_back(i);
  plan.nstore = m;
  plan.rows = engine_->matrix_rows(k, m);
  StripePlan vplan = plan;
  vplan.nstore = 0;
  std::vector<StripeTask> tasks;
  for (int s = 0; s < nstripes; ++s) {
    status[s] = CFSEC_OK;
    cfsec_shard* sh = shards + (size_t)s * n;
    if (n != tot) {
      status[s] = CFSEC_ERR_TOO_FEW_SHARDS;  // reedsolomon.go:610-612
      continue;
    }
    size_t S = 0;
    Status st = stripe_size(sh, n, false, &S);
    for (int i = 0; i < n && st == CFSEC_OK; ++i)
      if (!sh[i].data) st = CFSEC_ERR_INVALID_ARG;
    if (st != CFSEC_OK) {
      status[s] = st;
      continue;
    }
    if (m == 0 && !crc) continue;
    tasks.push_back(StripeTask{sh, &plan, S, &status[s], 0, 0, s});
    tasks.back().crc = crc ? 2 : 0;  // every shard (access/stream_put.go:249-253)
    tasks.back().crc_word = (int64_t)s * n;
    if (enable_verify_ && m > 0) tasks.push_back(StripeTask{sh, &vplan, S, &status[s], 0, 1, s});
  }
  const Status rc = engine_->run_stripes(tasks, mem, async, crc);
  clear_failed_crcs(crc, async, status, nstripes, n);
  return rc;
}

Status LrcEncoder::encode_batch(cfsec_shard* shards, int n, int nstripes, int mem, int* status,
                                const AsyncOut* async, const CrcOut* crc) {
  // lrcencoder.go:35-82 per stripe, fused: global parity and every AZ's local parity as one
  // (M+L) x N product over the data (the same rows LrcEncoder::encode launches); EnableVerify
  // compares all M+L rows in a second pass (the reference verifies the global and the local stripes)
  if (!shards || !status || nstripes < 0) return CFSEC_ERR_INVALID_ARG;
  const int N = t_.n, M = t_.m, L = t_.l;
  Slot slot(pool_.get());
  if (enable_verify_ && N > kLaunchMaxRows) {  // the fused Verify's rows exceed one compare launch
    if (crc || async) return CFSEC_ERR_NOT_SUPPORTED;  // synchronous stripe-by-stripe path only
    for (int s = 0; s < nstripes; ++s) {
      status[s] = n != N + M + L ? CFSEC_ERR_INVALID_SHARDS
                                 : encode_stripe(shards + (size_t)s * n, n, mem, async ? async->stream : nullptr);
      if (status[s] == CFSEC_ERR_DEVICE) return status[s];
    }
    return CFSEC_OK;
  }
  StripePlan plan;
  for (int i = 0; i < N; ++i) plan.in.push_back(i);
  for (int i = N; i < N + M + L; ++i) plan.out.push_back(i);
  plan.nstore = M + L;
  plan.rows = fused_;
  std::vector<StripeTask> tasks;
  for (int s = 0; s < nstripes; ++s) {
    status[s] = CFSEC_OK;
    cfsec_shard* sh = shards + (size_t)s * n;
    if (n != N + M + L) {
      status[s] = CFSEC_ERR_INVALID_SHARDS;
      continue;
    }
    Status st = fill_full_shards(sh, n);
    size_t S = 0;
    if (st == CFSEC_OK) st = stripe_size(sh, n, false, &S);
    for (int i = 0; i < n && st == CFSEC_OK; ++i)
      if (!sh[i].data) st = CFSEC_ERR_INVALID_ARG;
    if (st == CFSEC_ERR_SHARD_SIZE && stripe_size(sh, N + M, false, &S) == CFSEC_OK) {
      // only a local shard has another length: the reference still writes the global parity and
      // the AZs that pass their check -- the single-stripe path restates that sequence
      status[s] = encode_stripe(sh, n, mem, async ? async->stream : nullptr);
      continue;
    }
    if (st != CFSEC_OK) {
      status[s] = st;
      continue;
    }
    tasks.push_back(StripeTask{sh, &plan, S, &status[s], 0, 0, s});
    tasks.back().crc = crc ? 2 : 0;  // every shard, global and local (access/stream_put.go:249-253)
    tasks.back().crc_word = (int64_t)s * n;
  }
  StripePlan vplan = plan;
  vplan.nstore = 0;
  if (enable_verify_) {  // the Verify pass in the same call, after the encode (phase 1)
    const size_t ne = tasks.size();
    for (size_t i = 0; i < ne; ++i) {
      StripeTask v = tasks[i];
      v.plan = &vplan;
      v.phase = 1;
      v.crc = 0;
      tasks.push_back(v);
    }
  }
  const Status rc = engine_->run_stripes(tasks, mem, async, crc);
  clear_failed_crcs(crc, async, status, nstripes, n);
  return rc;
}

}  // namespace cfsec
