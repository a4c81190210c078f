// libcordagpu C ABI implementation (host side).  See include/cordagpu.h for the
// contract and the reference call sites each entry point replaces.
//
// Design (MI355X-first):
//  * one context = one HIP device + one non-blocking stream; the process-per-GPU
//    model of the multi-GPU path opens exactly one context per rank;
//  * inputs are copied element-major (what a JVM caller fills) and transposed on
//    the device into word-major SoA, so every kernel load is coalesced;
//  * mixed-scheme batches are partitioned by scheme on the host (index lists),
//    each scheme's kernels run on their subset and scatter verdicts back;
//  * Ed25519 scratch (per-lane tables) is bounded by processing in chunks, so a
//    100M-signature backlog needs ~3 GB of scratch, not 144 GB;
//  * device buffers come from a per-context block cache (freed blocks are kept
//    and reused), so repeated calls do not pay hipMalloc / hipFree;
//  * the transaction path uploads the caller's component arena as is and derives
//    all per-component / per-signature metadata on the device;
//  * no CPU fallback: without a gfx950 device cg_open fails.
#include "cordagpu.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <condition_variable>
#include <functional>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "cg_composite_api.h"
#include "cg_ecdsa_api.h"
#include "cg_kernels.h"
#include "cg_merkle_api.h"
#include "cg_plan.h"

namespace {

using cg::kAsyncArenaMin;
using cg::kEarlyPartMin;
using cg::kEdChunk;
using cg::kEdSplitDefault;
using cg::kEdSplitMin;

struct Stat {
  double ms = 0;
  uint64_t launches = 0;
  uint64_t items = 0;
};

// Host copy workers for staging pageable caller buffers into page-locked memory
// (cg_verify_batch's ring): one memcpy job split over the workers and the caller's
// thread.  A single core copies ~10-20 GB/s; PCIe takes ~57 GB/s.
class CopyPool {
 public:
  struct Piece {
    void* dst;
    const void* src;
    size_t bytes;
  };
  // A worker that cannot be created (resource exhaustion) leaves the pool with the
  // ones that were: the caller's thread copies too, so zero workers still work.
  explicit CopyPool(int workers) {
    for (int t = 0; t < workers; ++t) {
      try {
        th_.emplace_back([this] { loop(); });
      } catch (...) {
        break;
      }
    }
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  // Copies every piece (split into 256 KB tasks: a 12 MB slice is then ~48 tasks over
  // the 8 threads, not 12 tasks in two uneven rounds); returns when all are done.
  void run(const std::vector<Piece>& pieces) {
    std::unique_lock<std::mutex> g(m_);
    tasks_.clear();
    constexpr size_t kTask = 256u << 10;
    for (const Piece& p : pieces)
      for (size_t o = 0; o < p.bytes; o += kTask)
        tasks_.push_back({(char*)p.dst + o, (const char*)p.src + o, std::min(kTask, p.bytes - o)});
    next_ = 0;
    left_ = tasks_.size();
    ++gen_;
    cv_.notify_all();
    work(g);  // the caller copies too
    done_.wait(g, [this] { return left_ == 0; });
  }
  // Runs every function (the caller's thread takes part); returns when all are done.
  void run_fns(const std::vector<std::function<void()>>& fns) {
    std::unique_lock<std::mutex> g(m_);
    tasks_.clear();
    fns_ = &fns;
    next_ = 0;
    left_ = fns.size();
    ++gen_;
    cv_.notify_all();
    work(g);
    done_.wait(g, [this] { return left_ == 0; });
    fns_ = nullptr;
  }
  size_t workers() const { return th_.size(); }

 private:
  void work(std::unique_lock<std::mutex>& g) {
    while (fns_ && next_ < fns_->size()) {
      const size_t t = next_++;
      g.unlock();
      (*fns_)[t]();
      g.lock();
      if (--left_ == 0) done_.notify_all();
    }
    while (next_ < tasks_.size()) {
      const Piece t = tasks_[next_++];
      g.unlock();
      std::memcpy(t.dst, t.src, t.bytes);
      g.lock();
      if (--left_ == 0) done_.notify_all();
    }
  }
  void loop() {
    std::unique_lock<std::mutex> g(m_);
    uint64_t seen = 0;
    for (;;) {
      cv_.wait(g, [&] { return stop_ || gen_ != seen; });
      if (stop_) return;
      seen = gen_;
      work(g);
    }
  }
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  std::vector<Piece> tasks_;
  const std::vector<std::function<void()>>* fns_ = nullptr;
  size_t next_ = 0, left_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

// One long-lived helper thread: runs posted jobs in order.  Its HIP device is set
// once, when it starts (the verify pipeline's upload thread: a thread created per call
// cost ~0.05-0.07 ms before the first copy, r05p spans).
class JobThread {
 public:
  explicit JobThread(int device) : th_([this, device] {
    (void)hipSetDevice(device);
    loop();
  }) {}
  ~JobThread() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    th_.join();
  }
  void post(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> g(m_);
      q_.push_back(std::move(f));
    }
    cv_.notify_all();
  }

 private:
  void loop() {
    std::unique_lock<std::mutex> g(m_);
    for (;;) {
      cv_.wait(g, [&] { return stop_ || !q_.empty(); });
      if (q_.empty()) return;  // (stop_)
      std::function<void()> f = std::move(q_.front());
      q_.erase(q_.begin());
      g.unlock();
      try {
        f();
      } catch (...) {  // (a job reports its own failures; nothing unwinds out of the thread)
      }
      g.lock();
    }
  }
  std::mutex m_;
  std::condition_variable cv_;
  std::vector<std::function<void()>> q_;
  bool stop_ = false;
  std::thread th_;  // (last: started once the members above exist)
};

}  // namespace

struct cg_ctx {
  int device = -1;
  cg::Options opts;  // the CORDA_AMD_* knobs: environment snapshot at cg_open, cg_set_option
  uint32_t n_cu = 256;                  // compute units (hipDeviceProp)
  uint32_t lds_per_cu = 160 * 1024;     // LDS bytes per CU (hipDeviceProp; 160 KB on gfx950)
  uint32_t lds_per_block = 160 * 1024;  // largest LDS request of one block (hipDeviceProp)
  hipStream_t stream = nullptr;
  hipStream_t copy_stream = nullptr;  // host-to-device uploads overlapped with `stream` (tx pipeline)
  hipStream_t hash_stream = nullptr;  // tx pipeline: Merkle ids of chunk k+1 beside chunk k's signatures
  // the ECDSA curves' kernels run on their own streams, concurrently with the Ed25519
  // kernels on `stream` (fork/join events, no host sync).  HIP maps streams onto
  // GPU_MAX_HW_QUEUES hardware queues (default 4): stream, copy_stream, hash_stream
  // and one ECDSA stream fill four, and a fifth stream would share a queue and
  // serialize behind another stream's work (measured: the two curves of a tx chunk
  // alternated).  So the curves get a stream each only when the process allows >= 5
  // queues; otherwise ec_stream[1] aliases ec_stream[0].
  hipStream_t ec_stream[2] = {nullptr, nullptr};
  hipEvent_t ev_fork = nullptr, ev_join[2] = {nullptr, nullptr};
  hipEvent_t ev_keys = nullptr;  // key-reuse path: per-key tables ready (keyprep runs on ec_stream[0])
  hipEvent_t ev_split = nullptr;  // prepared-batch verify: the Ed25519 pieces on hash_stream are done
  hipEvent_t ev_pts_in = nullptr, ev_pts_done = nullptr;  // Ed25519 points kernel beside the hash kernel
  hipEvent_t ev_arena = nullptr;  // one-chunk verify: the deferred arena copy (on hash_stream) is done
  hipEvent_t ev_rows = nullptr;   // one-chunk verify: the raw key / signature rows are on the device
  std::string err;
  int32_t* btab = nullptr;
  // Ed25519 chunk scratch
  uint32_t ed_scap = 0;
  uint32_t* ed_status = nullptr;
  uint32_t* ed_digits = nullptr;
  int32_t* ed_table = nullptr;
  // key-reuse path scratch: per-key tables and decode status
  uint32_t ed_kcap = 0;
  int32_t* ed_ktab = nullptr;
  uint32_t* ed_kstat = nullptr;
  uint32_t* err_flag = nullptr;  // device word raised by kernels on malformed layouts
  // page-locked staging for the host-built index vectors of the tx pipeline, so their
  // uploads are truly asynchronous (a pageable hipMemcpyAsync waits for the stream);
  // grow-only, handed out front to back while pin_active, reset per call
  uint8_t* pin = nullptr;
  size_t pin_cap = 0, pin_used = 0;
  bool pin_active = false;
  uint64_t pin_fallbacks = 0;  // uploads that found the staging area full
  // cg_verify_batch's staging ring for pageable inputs: two page-locked slots (grow-only)
  // filled by the copy workers while the other slot's DMA runs
  uint8_t* ring[2] = {nullptr, nullptr};
  size_t ring_cap = 0;
  // page-locked bounce buffer of the host-buffer verify's verdict download (grow-only)
  uint8_t* dl_pin = nullptr;
  size_t dl_pin_cap = 0;
  CopyPool* pool = nullptr;
  JobThread* uploader = nullptr;  // the verify pipeline's upload thread (created on first use)
  bool profiling = false;
  // cg_set_profiling(ctx, 2): only the "call" span of each cg_verify_batch (two events
  // per call, no per-kernel events, no timeline file): the GPU time of unprofiled-shape
  // calls, so the host's share of a call's wall time can be measured
  bool call_spans_only = false;
  // the "call" span of a profiled cg_verify_batch: begin recorded at entry (the
  // streams are idle then, so it marks the host's entry on the GPU clock), end after
  // the verdicts' D2H copy, just before the final sync (end_call_span)
  hipEvent_t call_begin = nullptr;
  std::map<std::string, Stat> stats;
  std::vector<std::pair<std::string, std::pair<hipEvent_t, hipEvent_t>>> pending;
  std::vector<hipEvent_t> event_pool;
  // ordering-only events (hipEventDisableTiming) of the host-buffer verify pipeline,
  // reused across calls: creating and destroying ~10 per call cost host time after the
  // final sync
  std::vector<hipEvent_t> sync_event_pool;
  cg::EcdsaConsts* ec = nullptr;
  // device block cache: size -> free block; live block -> size
  std::multimap<size_t, void*> free_blocks;
  std::unordered_map<void*, size_t> live_blocks;
  // test hooks (cg_set_debug): Ed25519 lanes forced onto the full-length (h, 1)
  // scalar pair when index % debug_full_mod == 0; the debug_fail_alloc-th device
  // allocation from now fails as out of memory; the next guarded call throws.
  uint32_t debug_full_mod = 0;
  int64_t debug_fail_alloc = 0;
  int debug_throw = 0;
};

namespace {

cg_status fail(cg_ctx* ctx, cg_status code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  return code;
}

cg_status hip_fail(cg_ctx* ctx, hipError_t e, const char* what) {
  std::string m = std::string(what) + ": " + hipGetErrorString(e);
  (void)hipGetLastError();
  return fail(ctx, e == hipErrorOutOfMemory ? CG_E_OUT_OF_MEMORY : CG_E_DEVICE, m);
}

#define CG_TRY(ctx, expr, what)                           \
  do {                                                    \
    hipError_t e_ = (expr);                               \
    if (e_ != hipSuccess) return hip_fail(ctx, e_, what); \
  } while (0)

hipEvent_t take_sync_event(cg_ctx* ctx) {
  if (!ctx->sync_event_pool.empty()) {
    hipEvent_t e = ctx->sync_event_pool.back();
    ctx->sync_event_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
  return e;
}

hipEvent_t take_event(cg_ctx* ctx) {
  if (!ctx->event_pool.empty()) {
    hipEvent_t e = ctx->event_pool.back();
    ctx->event_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

// Profiling span events that will not be pushed as a span (their copy or kernel failed
// or never ran): back to the pool, never to hipEventElapsedTime unrecorded.
void give_back_events(cg_ctx* ctx, hipEvent_t a, hipEvent_t b) {
  if (a) ctx->event_pool.push_back(a);
  if (b) ctx->event_pool.push_back(b);
}

// RAII timing scope around one kernel launch on the context stream (or `s`).
struct Timed {
  cg_ctx* ctx;
  const char* name;
  uint64_t items;
  hipStream_t s;
  hipEvent_t a = nullptr, b = nullptr;
  Timed(cg_ctx* c, const char* n, uint64_t it, hipStream_t st = nullptr)
      : ctx(c), name(n), items(it), s(st ? st : c->stream) {
    if (ctx->profiling) {
      a = take_event(ctx);
      b = take_event(ctx);
      if (a) (void)hipEventRecord(a, s);
    }
  }
  ~Timed() {
    if (ctx->profiling && a && b) {
      (void)hipEventRecord(b, s);
      ctx->pending.push_back({name, {a, b}});
      ctx->stats[name].items += items;
    }
  }
};

void begin_call_span(cg_ctx* ctx) {
  if (!(ctx->profiling || ctx->call_spans_only) || ctx->call_begin) return;
  ctx->call_begin = take_event(ctx);
  if (ctx->call_begin) (void)hipEventRecord(ctx->call_begin, ctx->stream);
}
void end_call_span(cg_ctx* ctx) {
  if (!ctx->call_begin) return;
  hipEvent_t e = take_event(ctx);
  if (e) {
    (void)hipEventRecord(e, ctx->stream);
    ctx->pending.insert(ctx->pending.begin(), {"call", {ctx->call_begin, e}});  // first: the timeline's reference
  } else {
    ctx->event_pool.push_back(ctx->call_begin);
  }
  ctx->call_begin = nullptr;
}

void collect_timings(cg_ctx* ctx) {
  // CORDA_AMD_TIMELINE=<file>: every timed span of the call appended as
  // "name items start_ms end_ms" relative to the call's first span (tools/timeline.py)
  const char* tl_path = ctx->opts.str(cg::OPT_TIMELINE);
  if (tl_path && ctx->profiling && !ctx->pending.empty()) {
    if (FILE* f = std::fopen(tl_path, "a")) {
      const hipEvent_t ref = ctx->pending.front().second.first;
      std::fprintf(f, "# call\n");
      for (auto& p : ctx->pending) {
        float t0 = 0, t1 = 0;
        if (hipEventSynchronize(p.second.second) == hipSuccess &&
            hipEventElapsedTime(&t0, ref, p.second.first) == hipSuccess &&
            hipEventElapsedTime(&t1, ref, p.second.second) == hipSuccess)
          std::fprintf(f, "%s %.4f %.4f\n", p.first.c_str(), t0, t1);
      }
      std::fclose(f);
    }
  }
  for (auto& p : ctx->pending) {
    float ms = 0;
    if (hipEventSynchronize(p.second.second) == hipSuccess &&
        hipEventElapsedTime(&ms, p.second.first, p.second.second) == hipSuccess) {
      Stat& s = ctx->stats[p.first];
      s.ms += ms;
      s.launches += 1;
    }
    ctx->event_pool.push_back(p.second.first);
    ctx->event_pool.push_back(p.second.second);
  }
  ctx->pending.clear();
}

// min(off + len, bytes) without the wrap of off + len (an element or component
// outside the arena is rejected by its own check; this only sizes upload prefixes).
inline uint64_t clamped_end(uint64_t off, uint64_t len, uint64_t bytes) {
  return off >= bytes ? bytes : off + std::min<uint64_t>(len, bytes - off);
}

// ---------------------------------------------------------------- device blocks
// Requests are rounded to 1/8 of their power-of-two size class so that repeated
// batches of similar shape hit the cache; a cached block is reused for requests of
// at least half its size.  All users run on ctx->stream, so reuse is stream-ordered.
size_t round_block(size_t bytes) {
  if (bytes <= 4096) return (bytes + 255) & ~(size_t)255;
  size_t p = 1;
  while (p * 2 <= bytes) p *= 2;
  const size_t q = p / 8;
  return (bytes + q - 1) / q * q;
}

void release_cached(cg_ctx* ctx) {
  for (auto& b : ctx->free_blocks) (void)hipFree(b.second);
  ctx->free_blocks.clear();
}

bool debug_alloc_fails(cg_ctx* ctx) {
  if (ctx->debug_fail_alloc <= 0) return false;
  return --ctx->debug_fail_alloc == 0;
}

cg_status dalloc_bytes(cg_ctx* ctx, void** p, size_t bytes, const char* what) {
  *p = nullptr;
  if (debug_alloc_fails(ctx)) return fail(ctx, CG_E_OUT_OF_MEMORY, std::string(what) + ": injected allocation failure");
  const size_t want = round_block(bytes ? bytes : 1);
  auto it = ctx->free_blocks.lower_bound(want);
  if (it != ctx->free_blocks.end() && it->first <= 2 * want) {
    *p = it->second;
    ctx->live_blocks[it->second] = it->first;
    ctx->free_blocks.erase(it);
    return CG_OK;
  }
  hipError_t e = hipMalloc(p, want);
  if (e == hipErrorOutOfMemory && !ctx->free_blocks.empty()) {
    (void)hipGetLastError();
    (void)hipStreamSynchronize(ctx->stream);
    release_cached(ctx);
    e = hipMalloc(p, want);
  }
  if (e != hipSuccess) {
    *p = nullptr;
    return hip_fail(ctx, e, what);
  }
  ctx->live_blocks[*p] = want;
  return CG_OK;
}

template <typename T>
cg_status dalloc(cg_ctx* ctx, T** p, size_t count, const char* what) {
  void* v = nullptr;
  const cg_status st = dalloc_bytes(ctx, &v, count * sizeof(T), what);
  *p = (T*)v;
  return st;
}

void dfree(cg_ctx* ctx, const void* cp) {
  void* p = const_cast<void*>(cp);
  if (!p) return;
  auto it = ctx->live_blocks.find(p);
  if (it == ctx->live_blocks.end()) {
    (void)hipFree(p);
    return;
  }
  ctx->free_blocks.emplace(it->second, p);
  ctx->live_blocks.erase(it);
}

template <typename T>
cg_status upload(cg_ctx* ctx, T** dst, const T* src, size_t count, const char* what) {
  cg_status st = dalloc(ctx, dst, count, what);
  if (st != CG_OK) return st;
  if (count) CG_TRY(ctx, hipMemcpyAsync(*dst, src, count * sizeof(T), hipMemcpyHostToDevice, ctx->stream), what);
  return CG_OK;
}

// upload() of a host vector that dies before the copy runs: through the pinned
// staging area when the tx pipeline has one active (the copy then never blocks the
// host), else a plain upload followed by the caller's stream sync — or, for a
// MsgSrc::keep_raw batch (no sync), with the vector moved into the batch (idx_kept).
cg_status upload_idx(cg_ctx* ctx, uint32_t** dst, const uint32_t* src, size_t count, const char* what) {
  const size_t bytes = (count * 4 + 255) & ~(size_t)255;
  if (!ctx->pin_active || ctx->pin_used + bytes > ctx->pin_cap) {
    ctx->pin_fallbacks += ctx->pin_active;
    return upload(ctx, dst, src, count, what);
  }
  cg_status st = dalloc(ctx, dst, count, what);
  if (st != CG_OK) return st;
  uint8_t* h = ctx->pin + ctx->pin_used;
  ctx->pin_used += bytes;
  std::memcpy(h, src, count * 4);
  if (count) CG_TRY(ctx, hipMemcpyAsync(*dst, h, count * 4, hipMemcpyHostToDevice, ctx->stream), what);
  return CG_OK;
}

cg_status ensure_ed_scratch(cg_ctx* ctx, uint32_t need, uint32_t limit = kEdChunk) {
  const uint32_t want = std::min(need, limit);
  if (ctx->ed_scap >= want) return CG_OK;
  (void)hipStreamSynchronize(ctx->stream);
  (void)hipStreamSynchronize(ctx->hash_stream);  // (the verify pipeline's second compute stream)
  (void)hipStreamSynchronize(ctx->copy_stream);  // (points kernels beside the hash kernels)
  (void)hipStreamSynchronize(ctx->ec_stream[0]);
  dfree(ctx, ctx->ed_status);
  dfree(ctx, ctx->ed_digits);
  dfree(ctx, ctx->ed_table);
  ctx->ed_status = nullptr;
  ctx->ed_digits = nullptr;
  ctx->ed_table = nullptr;
  ctx->ed_scap = 0;
  cg_status st;
  // status words of the hash phase [0, want) and of the points phase [want, 2 want), the
  // grouped MSM's three lane classes [(2 + c) want, (3 + c) want) and its block counts
  // [5 want, 6 want) (a piece uses fewer words than lanes, from its first lane on)
  if ((st = dalloc(ctx, &ctx->ed_status, 6 * (size_t)want, "alloc ed25519 status")) != CG_OK) return st;
  if ((st = dalloc(ctx, &ctx->ed_digits, cg::ed25519_digit_words() * want, "alloc ed25519 digits")) != CG_OK) return st;
  if ((st = dalloc(ctx, (uint8_t**)&ctx->ed_table, cg::ed25519_table_bytes(want), "alloc ed25519 table")) != CG_OK)
    return st;
  ctx->ed_scap = want;
  return CG_OK;
}

}  // namespace

// Device-resident prepared batch.
struct cg_batch {
  size_t n = 0;
  uint8_t* verdict = nullptr;   // [n]
  bool verdict_owned = true;    // false: a slice of the tx pipeline's verdict array
  uint32_t* bitmap = nullptr;   // [ceil(n/32)]
  uint8_t* arena = nullptr;     // message arena (+16 pad)
  bool arena_owned = true;
  uint64_t* msg_off_all = nullptr;
  uint32_t* msg_len_all = nullptr;
  bool meta_owned = true;
  // Ed25519 subset
  uint32_t n_ed = 0;
  uint32_t* ed_index = nullptr;  // null when the subset is the whole batch in order
  uint32_t* ed_pk = nullptr;
  uint32_t* ed_sig = nullptr;
  uint32_t* ed_sig_len = nullptr;
  uint64_t* ed_msg_off = nullptr;
  uint32_t* ed_msg_len = nullptr;
  // key-reuse path (see key_reuse_mode): distinct-key slot of every Ed25519 element
  // and one element per slot; null key_index = the balanced per-signature path
  uint32_t n_keys = 0;
  uint32_t* ed_key_index = nullptr;
  uint32_t* ed_key_first = nullptr;
  // elements flagged CG_SCHEME_FLAG_KEY_INVALID: their verdict is CG_KEY_INVALID
  uint32_t n_bad = 0;
  uint32_t* bad_index = nullptr;
  // ECDSA subsets (K1, R1)
  cg::EcdsaBatch ec[2];
  // the ECDSA subsets' raw signature rows, compacted per curve (subset order), kept for
  // the K4 DER parse that opens every verify (BC decodes the DER inside each
  // engineVerify call); null in tx-pipeline batches, whose staging parse already sits
  // inside the pipeline's own timed run
  const void* raw_kept[3] = {nullptr, nullptr, nullptr};  // MsgSrc::keep_raw: staging's raw rows
  // MsgSrc::keep_raw: the host index vectors the staging copies read (a plain
  // hipMemcpyAsync when no pinned staging area is active), alive until the batch is freed
  // after the caller's sync
  std::vector<uint32_t> idx_kept[4];
  const uint8_t* arena_pending = nullptr;  // host arena still to upload (launch_verify, beside the points kernel)
  size_t arena_pending_bytes = 0;
  // host msg_off / msg_len still to upload with the arena (an all-Ed25519 in-order batch:
  // only the hash kernel reads them); ed_msg_off / ed_msg_len then alias msg_off_all /
  // msg_len_all instead of being gathered copies
  const uint64_t* meta_pending_off = nullptr;
  const uint32_t* meta_pending_len = nullptr;
  bool ed_meta_alias = false;
  // async arena (async_arena_enabled): the deferred arena and offsets / lengths go up from
  // the upload thread on hash_stream while the calling thread copies the rows; ctx->ev_arena
  // is recorded after them once `done`
  struct ArenaJob {
    std::mutex m;
    std::condition_variable cv;
    bool done = false;
    hipError_t err = hipSuccess;
    hipEvent_t span[2] = {nullptr, nullptr};  // (profiling: the copies' h2d_arena span)
    size_t bytes = 0;
    void wait() {
      std::unique_lock<std::mutex> g(m);
      cv.wait(g, [&] { return done; });
    }
  };
  std::unique_ptr<ArenaJob> arena_job;
  // one-chunk verify of an all-Ed25519 in-order batch: ctx->ev_rows marks the raw rows'
  // arrival (raw_kept[0..1], word strides below), so a latency-mode points kernel can
  // read them without waiting for the staging kernels
  bool rows_event = false;
  uint32_t raw_pk_words = 0, raw_sig_words = 0;
  uint32_t pair_max = 0;  // latency-mode threshold of this batch (MsgSrc::pair_max; 0: the default)
  // early points (early_points_parts): the balanced points kernels already run on
  // ctx->copy_stream and ctx->ev_pts_done marks their end
  bool points_early = false;
  uint8_t* ec_rows[2] = {nullptr, nullptr};     // [ec[c].n][ec_sig_stride]
  uint32_t* ec_row_len[2] = {nullptr, nullptr};  // [ec[c].n], or null: every row is ec_sig_stride long
  size_t ec_sig_stride = 0;
};

namespace {

void batch_free(cg_ctx* ctx, cg_batch* b) {
  if (!b) return;
  if (b->arena_job) {  // (a call that ended before launch_verify joined the arena copy)
    b->arena_job->wait();
    (void)hipStreamSynchronize(ctx->hash_stream);
    give_back_events(ctx, b->arena_job->span[0], b->arena_job->span[1]);
  }
  if (b->verdict_owned) dfree(ctx, b->verdict);
  dfree(ctx, b->bitmap);
  if (b->arena_owned) dfree(ctx, b->arena);
  if (b->meta_owned) {
    dfree(ctx, b->msg_off_all);
    dfree(ctx, b->msg_len_all);
  }
  dfree(ctx, b->ed_index);
  dfree(ctx, b->ed_pk);
  dfree(ctx, b->ed_sig);
  dfree(ctx, b->ed_sig_len);
  if (!b->ed_meta_alias) {
    dfree(ctx, b->ed_msg_off);
    dfree(ctx, b->ed_msg_len);
  }
  dfree(ctx, b->ed_key_index);
  dfree(ctx, b->ed_key_first);
  dfree(ctx, b->bad_index);
  for (auto& e : b->ec)
    for (const void* p : {(const void*)e.index, (const void*)e.q, (const void*)e.rs, (const void*)e.der,
                          (const void*)e.sig_len, (const void*)e.msg_off, (const void*)e.msg_len})
      dfree(ctx, p);
  for (int c = 0; c < 2; ++c) {
    dfree(ctx, b->ec_rows[c]);
    dfree(ctx, b->ec_row_len[c]);
  }
  for (const void* p : b->raw_kept) dfree(ctx, p);
  delete b;
}

// Where a batch's clear data comes from: a host arena with host offsets/lengths
// (cg_verify_batch / cg_batch_create), or a device arena the library owns with
// device-side offsets/lengths (the recomputed tx ids of cg_tx_verify_batch).
struct MsgSrc {
  const uint8_t* host = nullptr;
  uint8_t* dev = nullptr;
  size_t bytes = 0;
  const uint64_t* off_host = nullptr;
  const uint32_t* len_host = nullptr;
  uint64_t* off_dev = nullptr;
  uint32_t* len_dev = nullptr;
  // tx pipeline: the element-major pk / sig / sig_len rows are already on the device
  // (uploaded on copy_stream, complete once raw_ready fires); not owned by the batch
  const uint8_t* pk_dev = nullptr;
  const uint8_t* sig_dev = nullptr;
  const uint32_t* sl_dev = nullptr;
  hipEvent_t raw_ready = nullptr;
  // tx pipeline: verdicts straight into this device slice; staging ends without a
  // host sync (the caller keeps the batch until its own final sync)
  uint8_t* verdict_dev = nullptr;
  bool async = false;
  // one-chunk cg_verify_batch: the raw rows stay with the batch (freed by batch_free
  // after the call's final sync) instead of a host sync at the end of staging
  bool keep_raw = false;
  uint32_t pair_max = 0;  // the batch's latency-mode threshold (0: kEdPairMaxDefault)
  size_t index_base = 0;  // the batch's first element in the caller's (a pipeline chunk): error messages
};

// First element whose message lies outside an arena of `bytes` bytes, or n: a
// branch-free (vectorised) pass, then the exact index only when one exists.
// off > bytes || len > bytes - off: the sum off + len could wrap for a huge off.
size_t first_out_of_arena(const uint64_t* off, const uint32_t* len, size_t n, uint64_t bytes) {
  uint32_t bad = 0;
  for (size_t i = 0; i < n; ++i) bad |= (uint32_t)(off[i] > bytes) | (uint32_t)((uint64_t)len[i] > bytes - off[i]);
  for (size_t i = 0; bad && i < n; ++i)
    if (off[i] > bytes || len[i] > bytes - off[i]) return i;
  return n;
}

std::string out_of_arena_message(size_t i) { return "message out of arena bounds at element " + std::to_string(i); }

// arena_bounds = false: the caller runs the all-Ed25519 arena-bounds pass itself (create_batch's
// BoundsBeside, on the upload thread beside the row copies)
// index_base: the first element's index in the caller's batch (a pipeline chunk), so an
// error names the caller's element.
cg_status check_inputs(cg_ctx* ctx, size_t n, const uint8_t* scheme_id, const uint8_t* pk, size_t pk_stride,
                       const uint8_t* sig, size_t sig_stride, const uint32_t* sig_len, const MsgSrc& m,
                       bool arena_bounds = true, size_t index_base = 0) {
  if (!ctx) return CG_E_INVALID_ARGUMENT;
  if (n > 0xFFFFFFF0ull) return fail(ctx, CG_E_INVALID_ARGUMENT, "batch larger than 2^32 - 16 elements");
  if (n == 0) return CG_OK;
  if (!pk || !sig) return fail(ctx, CG_E_INVALID_ARGUMENT, "null input pointer");
  if (!m.dev && (!m.off_host || !m.len_host)) return fail(ctx, CG_E_INVALID_ARGUMENT, "null input pointer");
  if (!m.dev && m.bytes > 0 && !m.host) return fail(ctx, CG_E_INVALID_ARGUMENT, "null message arena");
  bool has_ed = false, has_ec = false;
  if (!scheme_id) {  // all Ed25519: only the arena bounds
    if (m.off_host && arena_bounds) {
      const size_t i = first_out_of_arena(m.off_host, m.len_host, n, m.bytes);
      if (i < n) return fail(ctx, CG_E_INVALID_ARGUMENT, out_of_arena_message(index_base + i));
    }
    if (pk_stride < 32 || sig_stride < 64)
      return fail(ctx, CG_E_INVALID_ARGUMENT, "Ed25519 needs pk_stride >= 32 and sig_stride >= 64");
    return CG_OK;
  }
  for (size_t i = 0; i < n; ++i) {
    const uint8_t s = scheme_id[i];
    // off > bytes || len > bytes - off: the sum off + len could wrap for a huge off
    if (m.off_host && (m.off_host[i] > m.bytes || m.len_host[i] > m.bytes - m.off_host[i]))
      return fail(ctx, CG_E_INVALID_ARGUMENT, out_of_arena_message(index_base + i));
    if (s & CG_SCHEME_FLAG_KEY_INVALID) continue;  // never read beyond its verdict
    if (s == CG_SCHEME_EDDSA_ED25519_SHA512) has_ed = true;
    if (s == CG_SCHEME_ECDSA_SECP256K1_SHA256 || s == CG_SCHEME_ECDSA_SECP256R1_SHA256) {
      has_ec = true;
      const uint32_t l = sig_len ? sig_len[i] : (uint32_t)sig_stride;
      if (l > sig_stride)
        return fail(ctx, CG_E_INVALID_ARGUMENT,
                    "ECDSA signature longer than sig_stride at element " + std::to_string(index_base + i));
    }
  }
  if (has_ed && (pk_stride < 32 || sig_stride < 64))
    return fail(ctx, CG_E_INVALID_ARGUMENT, "Ed25519 needs pk_stride >= 32 and sig_stride >= 64");
  if (has_ec && pk_stride < 64) return fail(ctx, CG_E_INVALID_ARGUMENT, "ECDSA needs pk_stride >= 64");
  return CG_OK;
}

// Every extern "C" entry point runs inside CG_API_BEGIN / CG_API_END: a C++
// exception (std::bad_alloc from a host-side vector or string, or anything else)
// never unwinds into the caller (a JVM through JNI); it becomes a status code, and
// the context's streams are drained first so no in-flight kernel still uses a
// buffer the caller is about to reuse.
cg_status api_guard_fail(cg_ctx* ctx) noexcept {
  cg_status st = CG_E_DEVICE;
  const char* msg = "internal error (exception caught at the C ABI)";
  try {
    throw;
  } catch (const std::bad_alloc&) {
    st = CG_E_OUT_OF_MEMORY;
    msg = "host allocation failed";
  } catch (...) {
  }
  if (ctx) {
    (void)hipSetDevice(ctx->device);
    for (hipStream_t s : {ctx->stream, ctx->copy_stream, ctx->hash_stream, ctx->ec_stream[0], ctx->ec_stream[1]})
      if (s) (void)hipStreamSynchronize(s);
    try {
      ctx->err = msg;
    } catch (...) {
    }
  }
  return st;
}

void debug_throw_point(cg_ctx* ctx) {
  if (ctx && ctx->debug_throw) {
    ctx->debug_throw = 0;
    throw std::bad_alloc();
  }
}

#define CG_API_BEGIN try {
#define CG_API_END(ctx_)          \
  }                               \
  catch (...) {                   \
    return api_guard_fail(ctx_);  \
  }

}  // namespace

extern "C" {

int cg_abi_version(void) { return CG_ABI_VERSION; }

int cg_device_count(void) {
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return c;
}

cg_status cg_open(int device, cg_ctx** out) {
  CG_API_BEGIN
  if (!out) return CG_E_INVALID_ARGUMENT;
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0) {
    (void)hipGetLastError();
    return CG_E_NO_DEVICE;
  }
  if (device < 0 || device >= count) return CG_E_INVALID_ARGUMENT;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return CG_E_DEVICE;
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return CG_E_NO_DEVICE;
  cg_ctx* ctx = new (std::nothrow) cg_ctx();
  if (!ctx) return CG_E_OUT_OF_MEMORY;
  ctx->device = device;
  ctx->opts.from_env();  // the CORDA_AMD_* knobs, read once (cg_set_option changes them later)
  ctx->n_cu = (uint32_t)std::max(1, prop.multiProcessorCount);
  if (prop.maxSharedMemoryPerMultiProcessor > 0) ctx->lds_per_cu = (uint32_t)prop.maxSharedMemoryPerMultiProcessor;
  if (prop.sharedMemPerBlock > 0) ctx->lds_per_block = (uint32_t)prop.sharedMemPerBlock;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
    delete ctx;
    return CG_E_DEVICE;
  }
  if (hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&ctx->hash_stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&ctx->ec_stream[0], hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_join[0], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_join[1], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_keys, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_split, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_pts_in, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_pts_done, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_arena, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_rows, hipEventDisableTiming) != hipSuccess) {
    cg_close(ctx);
    return CG_E_DEVICE;
  }
  const char* hwq = std::getenv("GPU_MAX_HW_QUEUES");
  if (!hwq || std::atoi(hwq) < 5 ||
      hipStreamCreateWithFlags(&ctx->ec_stream[1], hipStreamNonBlocking) != hipSuccess)
    ctx->ec_stream[1] = ctx->ec_stream[0];
  // the shared Ed25519 base tables (k*B, k*2^128 B) are built on the device, once per context
  if (dalloc(ctx, &ctx->btab, cg::ed25519_btab_words(), "alloc base table") != CG_OK ||
      cg::launch_ed25519_btab_build(ctx->btab, ctx->stream) != hipSuccess ||
      hipStreamSynchronize(ctx->stream) != hipSuccess ||
      dalloc(ctx, &ctx->err_flag, 1, "alloc error flag") != CG_OK) {
    cg_close(ctx);
    return CG_E_DEVICE;
  }
  if (cg::ecdsa_consts_create(&ctx->ec, ctx->stream) != hipSuccess) {
    cg_close(ctx);
    return CG_E_DEVICE;
  }
  *out = ctx;
  return CG_OK;
  CG_API_END(nullptr)
}

void cg_close(cg_ctx* ctx) {
  try {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->copy_stream) (void)hipStreamSynchronize(ctx->copy_stream);
    if (ctx->hash_stream) (void)hipStreamSynchronize(ctx->hash_stream);
    for (hipStream_t es : ctx->ec_stream)
      if (es) (void)hipStreamSynchronize(es);
    collect_timings(ctx);
    cg::ecdsa_consts_free(ctx->ec);
    for (auto& b : ctx->live_blocks) (void)hipFree(b.first);
    ctx->live_blocks.clear();
    release_cached(ctx);
    for (hipEvent_t e : ctx->event_pool) (void)hipEventDestroy(e);
    for (hipEvent_t e : ctx->sync_event_pool) (void)hipEventDestroy(e);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    if (ctx->copy_stream) (void)hipStreamDestroy(ctx->copy_stream);
    if (ctx->hash_stream) (void)hipStreamDestroy(ctx->hash_stream);
    if (ctx->ec_stream[1] && ctx->ec_stream[1] != ctx->ec_stream[0]) (void)hipStreamDestroy(ctx->ec_stream[1]);
    if (ctx->ec_stream[0]) (void)hipStreamDestroy(ctx->ec_stream[0]);
    for (hipEvent_t e : {ctx->ev_fork, ctx->ev_join[0], ctx->ev_join[1], ctx->ev_keys, ctx->ev_split, ctx->ev_pts_in,
                         ctx->ev_pts_done, ctx->ev_arena, ctx->ev_rows})
      if (e) (void)hipEventDestroy(e);
    if (ctx->pin) (void)hipHostFree(ctx->pin);
    for (uint8_t* r : ctx->ring)
      if (r) (void)hipHostFree(r);
    if (ctx->dl_pin) (void)hipHostFree(ctx->dl_pin);
    delete ctx->uploader;
    delete ctx->pool;
    delete ctx;
  } catch (...) {
    // nothing to report from a destructor-like call; never unwind into the caller
  }
}

const char* cg_last_error(const cg_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

cg_status cg_register_host(cg_ctx* ctx, void* ptr, size_t bytes) {
  CG_API_BEGIN
  if (!ctx) return CG_E_INVALID_ARGUMENT;
  if (!ptr || !bytes) return fail(ctx, CG_E_INVALID_ARGUMENT, "null pointer or empty range");
  if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, CG_E_DEVICE, "hipSetDevice");
  CG_TRY(ctx, hipHostRegister(ptr, bytes, hipHostRegisterDefault), "hipHostRegister");
  return CG_OK;
  CG_API_END(ctx)
}

cg_status cg_unregister_host(cg_ctx* ctx, void* ptr) {
  CG_API_BEGIN
  if (!ctx) return CG_E_INVALID_ARGUMENT;
  if (!ptr) return fail(ctx, CG_E_INVALID_ARGUMENT, "null pointer");
  if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, CG_E_DEVICE, "hipSetDevice");
  CG_TRY(ctx, hipHostUnregister(ptr), "hipHostUnregister");
  return CG_OK;
  CG_API_END(ctx)
}

cg_status cg_release_cached(cg_ctx* ctx) {
  CG_API_BEGIN
  if (!ctx) return CG_E_INVALID_ARGUMENT;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  release_cached(ctx);
  return CG_OK;
  CG_API_END(ctx)
}

}  // extern "C"

namespace {

// The knobs of a context (cg_plan.h: each a pure function of ctx->opts, the environment
// snapshot of cg_open plus cg_set_option).
// Key-reuse decision (CORDA_AMD_KEY_REUSE: 0 never, 1 always, else automatic):
// the per-key path pays a decode and four 9-entry tables (~190 doublings) per
// distinct key and saves ~70 doublings, the A decode and the A table per
// signature, so it wins once keys repeat a few times; automatic = n / n_keys >= 8.
int key_reuse_forced(const cg_ctx* ctx) { return cg::key_reuse_forced(ctx->opts); }
uint32_t ed_pair_max(const cg_ctx* ctx, uint32_t call_default = 0) { return cg::ed_pair_max(ctx->opts, call_default); }
// Latency mode: the hash and points kernels run side by side with a few blocks each,
// and the dispatcher packs those blocks onto the same CUs, where they slow each other
// (4,096 signatures: hash 0.16 -> 0.26 ms beside the points kernel, r04r spans).  The
// blocks then reserve LDS (dynamic, unused) so that no CU holds a hash block beside
// another block: hash blocks more than half a CU's LDS, points blocks more than half
// too when every block fits on its own CU, else exactly half (two points blocks may
// share a CU, a hash block never joins them) when that fits; otherwise nothing.
// CORDA_AMD_ED_SPREAD_LDS=0 turns it off.  Sets d.spread_lds / d.spread_lds_hash.
// n_cu: the CUs this piece may count on (inside the two-chunk verify pipeline the other
// chunk's kernels hold about half the chip).
void ed_spread_lds(const cg_ctx* ctx, cg::Ed25519Dev& d, uint64_t points_blocks, uint64_t hash_blocks,
                   uint32_t n_cu) {
  d.spread_lds = d.spread_lds_hash = 0;
  if (!ctx->opts.on(cg::OPT_ED_SPREAD_LDS, true)) return;
  const uint32_t half = ctx->lds_per_cu / 2;
  if (half + 4096 > ctx->lds_per_block) return;  // a block cannot reserve more than half a CU
  if (points_blocks + hash_blocks <= n_cu) {
    d.spread_lds = d.spread_lds_hash = half + 4096;
  } else if ((points_blocks + 1) / 2 + hash_blocks <= n_cu) {
    d.spread_lds = half;
    d.spread_lds_hash = half + 4096;
  }
}
bool ed_overlap_enabled(const cg_ctx* ctx) { return cg::ed_overlap_enabled(ctx->opts); }

bool key_reuse_mode(const cg_ctx* ctx, uint32_t n, uint32_t n_keys) {
  const int forced = key_reuse_forced(ctx);
  if (forced >= 0) return forced == 1;
  return n_keys > 0 && (uint64_t)n_keys * 8 <= n;
}

// Distinct Ed25519 keys of a staged batch (device hash table, stage_kernels.hip);
// keeps key_index / key_first only when the key-reuse path will be used.
// Automatic mode first looks at a pseudo-random sample of the keys on the host: the
// exact device count (which needs a host round trip) only runs when the sample holds
// enough repeats for n / n_keys >= 8 to be plausible (half the birthday-bound
// threshold, so a true reuse batch passes with a wide margin).
bool key_sample_suggests_reuse(const uint8_t* pk, size_t pk_stride, const std::vector<uint32_t>& idx0, uint32_t ne) {
  constexpr uint32_t kSample = 1024;
  if (ne < 8 * kSample) return true;  // small batch: the exact count is cheap
  std::vector<std::array<uint8_t, 32>> keys(kSample);
  for (uint32_t j = 0; j < kSample; ++j) {
    const uint64_t i = ((uint64_t)j * 0x9E3779B1u + 12345u) % ne;
    const size_t e = idx0.size() == ne ? idx0[i] : i;
    std::memcpy(keys[j].data(), pk + e * pk_stride, 32);
  }
  std::sort(keys.begin(), keys.end());
  uint32_t repeats = 0;
  for (uint32_t j = 1; j < kSample; ++j) repeats += keys[j] == keys[j - 1];
  // n_keys ~ kSample^2 / (2 repeats); reuse needs n_keys <= ne / 8
  return (uint64_t)repeats * ne >= (uint64_t)kSample * kSample * 2;
}

// sample: key_sample_suggests_reuse's answer when the caller already has it (-1: unknown)
cg_status stage_key_dedupe(cg_ctx* ctx, cg_batch* b, const uint8_t* pk, size_t pk_stride,
                           const std::vector<uint32_t>& idx0, int sample = -1) {
  const uint32_t ne = b->n_ed;
  const int forced = key_reuse_forced(ctx);
  if (forced == 0 || (ne < 64 && forced != 1)) return CG_OK;
  // automatic mode and a batch the latency mode will verify: the key-reuse path's
  // per-key table build (~190 doublings, one wave per 64 keys) would be the longest
  // chain of the call, and the exact count is a host round trip
  if (forced != 1 && ne <= ed_pair_max(ctx, b->pair_max)) return CG_OK;
  if (forced != 1 && !(sample >= 0 ? sample == 1 : key_sample_suggests_reuse(pk, pk_stride, idx0, ne))) return CG_OK;
  uint32_t tsize = 1;
  while (tsize < 2 * ne) tsize <<= 1;
  uint32_t *table = nullptr, *slot_of = nullptr, *owner = nullptr, *counter = nullptr;
  cg_status st = CG_OK;
  auto done = [&](cg_status r) {
    (void)hipStreamSynchronize(ctx->stream);
    for (const void* p : {(const void*)table, (const void*)slot_of, (const void*)owner, (const void*)counter})
      dfree(ctx, p);
    return r;
  };
  if ((st = dalloc(ctx, &table, tsize, "alloc key table")) != CG_OK || (st = dalloc(ctx, &slot_of, ne, "alloc key slots")) != CG_OK ||
      (st = dalloc(ctx, &owner, tsize, "alloc key owners")) != CG_OK || (st = dalloc(ctx, &counter, 1, "alloc key counter")) != CG_OK ||
      (st = dalloc(ctx, &b->ed_key_index, ne, "alloc key index")) != CG_OK ||
      (st = dalloc(ctx, &b->ed_key_first, ne, "alloc key first")) != CG_OK)
    return done(st);
  hipError_t e = hipMemsetAsync(table, 0, (size_t)tsize * 4, ctx->stream);
  if (e == hipSuccess) e = hipMemsetAsync(counter, 0, 4, ctx->stream);
  if (e == hipSuccess)
    e = cg::launch_key_dedupe(b->ed_pk, ne, ne, table, tsize, slot_of, owner, counter, b->ed_key_index,
                              b->ed_key_first, ctx->stream);
  uint32_t n_keys = 0;
  if (e == hipSuccess) e = hipMemcpyAsync(&n_keys, counter, 4, hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) return done(hip_fail(ctx, e, "key dedupe"));
  if (!key_reuse_mode(ctx, ne, n_keys)) {
    dfree(ctx, b->ed_key_index);
    dfree(ctx, b->ed_key_first);
    b->ed_key_index = b->ed_key_first = nullptr;
    return done(CG_OK);
  }
  b->n_keys = n_keys;
  return done(CG_OK);
}

cg_status ensure_key_scratch(cg_ctx* ctx, uint32_t n_keys) {
  if (ctx->ed_kcap >= n_keys) return CG_OK;
  (void)hipStreamSynchronize(ctx->stream);
  (void)hipStreamSynchronize(ctx->hash_stream);  // (the verify pipeline's second compute stream)
  dfree(ctx, ctx->ed_ktab);
  dfree(ctx, ctx->ed_kstat);
  ctx->ed_ktab = nullptr;
  ctx->ed_kstat = nullptr;
  ctx->ed_kcap = 0;
  cg_status st;
  if ((st = dalloc(ctx, (uint8_t**)&ctx->ed_ktab, cg::ed25519_key_table_bytes(n_keys), "alloc key tables")) != CG_OK ||
      (st = dalloc(ctx, &ctx->ed_kstat, n_keys, "alloc key status")) != CG_OK)
    return st;
  ctx->ed_kcap = n_keys;
  return CG_OK;
}

// A scheme array that names Ed25519 for every element is the batch scheme_id NULL
// describes (include/cordagpu.h): one vectorised pass (~n / 16 ns) lets such a call take
// the Ed25519-only host path — no per-element partition and checks (~3 ns per element:
// 0.2 ms at 65,536), the arena bounds beside the row copies.  Returns the array to use.
const uint8_t* ed25519_only(const uint8_t* scheme_id, size_t n) {
  if (!scheme_id) return nullptr;
  for (size_t i = 0; i < n; i += 4096) {  // (blocks: a mixed batch usually stops at the first)
    const size_t e = std::min(n, i + 4096);
    uint8_t acc = 0;
    for (size_t j = i; j < e; ++j) acc |= (uint8_t)(scheme_id[j] ^ CG_SCHEME_EDDSA_ED25519_SHA512);
    if (acc) return scheme_id;
  }
  return nullptr;
}

// create_batch's arena-bounds pass on the upload thread (see there).  Every exit of
// create_batch waits for a posted pass (the job reads the caller's arrays and this object).
struct BoundsBeside {
  std::mutex m;
  std::condition_variable cv;
  bool posted = false, done = false;
  size_t first_bad = 0;
  bool post(cg_ctx* ctx, const uint64_t* off, const uint32_t* len, size_t n, uint64_t bytes) {
    try {
      if (!ctx->uploader) ctx->uploader = new JobThread(ctx->device);
      ctx->uploader->post([this, off, len, n, bytes] {
        const size_t i = first_out_of_arena(off, len, n, bytes);
        std::lock_guard<std::mutex> g(m);
        first_bad = i;
        done = true;
        cv.notify_all();
      });
    } catch (...) {
      return false;
    }
    posted = true;
    return true;
  }
  size_t wait() {
    std::unique_lock<std::mutex> g(m);
    cv.wait(g, [&] { return done; });
    posted = false;
    return first_bad;
  }
  ~BoundsBeside() {
    if (posted) (void)wait();
  }
};

// Stages a batch (see MsgSrc for where its clear data lives).
cg_status create_batch(cg_ctx* ctx, size_t n, const uint8_t* scheme_id, const uint8_t* pk, size_t pk_stride,
                       const uint8_t* sig, size_t sig_stride, const uint32_t* sig_len, const MsgSrc& m,
                       cg_batch** out) {
  if (!out) return fail(ctx, CG_E_INVALID_ARGUMENT, "null out");
  *out = nullptr;
  // A one-chunk host call of Ed25519 rows (no scheme ids, n >= cg::kBoundsBesideMin: below it
// the pass is ~18 us, less than the thread hand-off would save): the
  // arena-bounds pass over msg_off / msg_len (~0.55 ns per element: 0.15 ms at 2^18, all of
  // it before the first copy) runs on the upload thread while this thread copies the rows
  // and launches the points kernels, which read no message.  The batch is handed out only
  // after the pass has found nothing (the hash kernel, the first reader of a message, is
  // launched later, by launch_verify); a failure returns the same status and message as the
  // synchronous check, after draining what was launched.
  BoundsBeside beside;
  const bool bounds_beside = !scheme_id && m.keep_raw && !m.dev && m.off_host && m.len_host && n >= cg::kBoundsBesideMin;
  cg_status st = check_inputs(ctx, n, scheme_id, pk, pk_stride, sig, sig_stride, sig_len, m, !bounds_beside,
                              m.index_base);
  if (st != CG_OK) return st;
  if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, CG_E_DEVICE, "hipSetDevice");
  if (bounds_beside && !beside.post(ctx, m.off_host, m.len_host, n, m.bytes)) {
    const size_t i = first_out_of_arena(m.off_host, m.len_host, n, m.bytes);  // (no thread: here, now)
    if (i < n) return fail(ctx, CG_E_INVALID_ARGUMENT, out_of_arena_message(i));
  }
  cg_batch* b = new (std::nothrow) cg_batch();
  if (!b) return fail(ctx, CG_E_OUT_OF_MEMORY, "host alloc");
  b->n = n;
  b->pair_max = m.pair_max;
  // raw element-major inputs (temporary)
  uint8_t *pk_raw = nullptr, *sig_raw = nullptr;
  uint32_t* sl_raw = nullptr;
  const bool raw_owned = !m.pk_dev;
  auto free_raw = [&]() {
    if (raw_owned) {
      dfree(ctx, pk_raw);
      dfree(ctx, sig_raw);
      dfree(ctx, sl_raw);
    }
    pk_raw = sig_raw = nullptr;
    sl_raw = nullptr;
  };
  auto bail = [&](cg_status s) {
    (void)hipStreamSynchronize(ctx->stream);
    if (b->points_early) (void)hipStreamSynchronize(ctx->copy_stream);
    free_raw();
    batch_free(ctx, b);
    return s;
  };
  // host-side partition by scheme
  std::vector<uint32_t> idx[3];  // 0: ed25519, 1: K1, 2: R1
  std::vector<uint32_t> bad;     // flagged CG_SCHEME_FLAG_KEY_INVALID
  debug_throw_point(ctx);
  bool ed_identity = true;
  int key_sample = -1;  // key_sample_suggests_reuse's answer, once asked
  bool meta_deferred = false;  // offsets / lengths go up after create_batch (launch_verify or the upload thread)
  size_t n_ed = 0;  // Ed25519 elements (idx[0] stays empty when they are the whole batch in order)
  for (size_t i = 0; scheme_id && i < n; ++i) {
    const uint8_t s = scheme_id ? scheme_id[i] : CG_SCHEME_EDDSA_ED25519_SHA512;
    if (s & CG_SCHEME_FLAG_KEY_INVALID) {
      bad.push_back((uint32_t)i);
    } else if (s == CG_SCHEME_EDDSA_ED25519_SHA512) {
      if (idx[0].size() != i) ed_identity = false;
      idx[0].push_back((uint32_t)i);
    } else if (s == CG_SCHEME_ECDSA_SECP256K1_SHA256) {
      idx[1].push_back((uint32_t)i);
    } else if (s == CG_SCHEME_ECDSA_SECP256R1_SHA256) {
      idx[2].push_back((uint32_t)i);
    }
  }
  // scheme_id NULL: every element is Ed25519, in order — no index vector (an O(n) loop
  // of push_backs was ~0.1-0.2 ms of host time before the first copy at 2^18 elements)
  n_ed = scheme_id ? idx[0].size() : n;
  if (n_ed != n) ed_identity = false;
  const size_t nwords = (n + 31) / 32;
  const uint64_t fallbacks0 = ctx->pin_fallbacks;
  if (m.verdict_dev) {
    b->verdict = m.verdict_dev;
    b->verdict_owned = false;
  } else if ((st = dalloc(ctx, &b->verdict, n, "alloc verdict")) != CG_OK) {
    return bail(st);
  }
  if ((st = dalloc(ctx, &b->bitmap, nwords, "alloc bitmap")) != CG_OK) return bail(st);
  if (m.dev) {
    b->arena = m.dev;  // library-owned device arena (padded by its producer)
    b->arena_owned = false;
    b->msg_off_all = m.off_dev;
    b->msg_len_all = m.len_dev;
    b->meta_owned = false;
  } else {
    if ((st = dalloc(ctx, &b->arena, m.bytes + 16, "alloc arena")) != CG_OK) return bail(st);
    // A one-chunk host verify (m.keep_raw) follows its plan (cg_plan.h plan_verify, from
    // the call's shape as the partition above found it; the key sample only when a
    // choice hinges on it).  An Ed25519-only batch: the message arena goes up later, from
    // launch_verify, once the points kernel (which needs only keys and R) is running —
    // the copy then overlaps it (no ECDSA kernel reads the arena earlier); when every
    // element is Ed25519 in order, its offsets / lengths too: the points kernel starts
    // after the key and signature rows alone (r05: 2^18 x 32 B ids spent ~0.85 ms in
    // copies before the first kernel).
    cg::VerifyPlan plan;
    if (m.keep_raw) {
      cg::VerifyShape shape;
      shape.n = n;
      shape.n_ed = n_ed;
      shape.msg_bytes = m.bytes;
      shape.pk_stride = pk_stride;
      shape.sig_stride = sig_stride;
      shape.sig_len = sig_len != nullptr;
      shape.ecdsa = !idx[1].empty() || !idx[2].empty();
      shape.ed_in_order = ed_identity && bad.empty();
      plan = cg::plan_verify(shape, ctx->opts);
      if (plan.needs_key_sample) {
        shape.keys_repeat = key_sample_suggests_reuse(pk, pk_stride, idx[0], (uint32_t)n_ed) ? 1 : 0;
        key_sample = shape.keys_repeat;
        plan = cg::plan_verify(shape, ctx->opts);
      }
    }
    const bool defer_arena = plan.defer_arena;
    const bool defer_meta = plan.defer_meta;
    meta_deferred = defer_meta;
    Timed t(ctx, "h2d_stage", (defer_arena ? 0 : m.bytes) + (defer_meta ? 0 : 12 * n) +
                                  (raw_owned ? n * (pk_stride + sig_stride + (sig_len ? 4 : 0)) : 0));
    if (defer_arena) {
      b->arena_pending = m.host;
      b->arena_pending_bytes = m.bytes;
    } else if (m.bytes) {
      const hipError_t e = hipMemcpyAsync(b->arena, m.host, m.bytes, hipMemcpyHostToDevice, ctx->stream);
      if (e != hipSuccess) return bail(hip_fail(ctx, e, "upload arena"));
    }
    const hipError_t e = hipMemsetAsync(b->arena + m.bytes, 0, 16, ctx->stream);
    if (e != hipSuccess) return bail(hip_fail(ctx, e, "pad arena"));
    if (defer_meta) {
      if ((st = dalloc(ctx, &b->msg_off_all, n, "alloc msg_off")) != CG_OK ||
          (st = dalloc(ctx, &b->msg_len_all, n, "alloc msg_len")) != CG_OK)
        return bail(st);
      b->meta_pending_off = m.off_host;
      b->meta_pending_len = m.len_host;
    } else {
      if ((st = upload(ctx, &b->msg_off_all, m.off_host, n, "upload msg_off")) != CG_OK) return bail(st);
      if ((st = upload(ctx, &b->msg_len_all, m.len_host, n, "upload msg_len")) != CG_OK) return bail(st);
    }
    if (plan.async_arena) {
      try {
        if (!ctx->uploader) ctx->uploader = new JobThread(ctx->device);
        b->arena_job.reset(new cg_batch::ArenaJob());
        cg_batch::ArenaJob* job = b->arena_job.get();
        uint8_t* arena = b->arena;
        uint64_t* off_d = b->msg_off_all;
        uint32_t* len_d = b->msg_len_all;
        const uint64_t* off_h = b->meta_pending_off;
        const uint32_t* len_h = b->meta_pending_len;
        const uint8_t* host = m.host;
        const size_t bytes = m.bytes;
        hipStream_t hs = ctx->hash_stream;
        hipEvent_t ev = ctx->ev_arena;
        job->bytes = bytes;
        if (ctx->profiling) {
          job->span[0] = take_event(ctx);
          job->span[1] = take_event(ctx);
        }
        ctx->uploader->post([=] {
          if (job->span[0]) (void)hipEventRecord(job->span[0], hs);
          hipError_t e2 = hipMemcpyAsync(arena, host, bytes, hipMemcpyHostToDevice, hs);
          if (e2 == hipSuccess && off_h) e2 = hipMemcpyAsync(off_d, off_h, n * 8, hipMemcpyHostToDevice, hs);
          if (e2 == hipSuccess && len_h) e2 = hipMemcpyAsync(len_d, len_h, n * 4, hipMemcpyHostToDevice, hs);
          if (e2 == hipSuccess && job->span[1]) (void)hipEventRecord(job->span[1], hs);
          if (e2 == hipSuccess) e2 = hipEventRecord(ev, hs);
          std::lock_guard<std::mutex> g(job->m);
          job->err = e2;
          job->done = true;
          job->cv.notify_all();
        });
        b->arena_pending = nullptr;
        b->meta_pending_off = nullptr;
        b->meta_pending_len = nullptr;
      } catch (...) {  // (no thread: the copies stay deferred to launch_verify)
        b->arena_job.reset();
      }
    }
    if (raw_owned) {
      const bool rows_direct = plan.rows_direct && ctx->ev_rows;
      const uint32_t parts = rows_direct ? plan.early_parts : 0;
      const bool split_points = rows_direct && plan.split_points;
      if (split_points) {  // the A half beside the signatures' copy (split_points_enabled)
        if ((st = ensure_ed_scratch(ctx, (uint32_t)n)) != CG_OK ||
            (st = dalloc(ctx, &pk_raw, n * pk_stride, "alloc pk")) != CG_OK ||
            (st = dalloc(ctx, &sig_raw, n * sig_stride, "alloc sig")) != CG_OK)
          return bail(st);
        cg::Ed25519Dev d;
        d.cap = (uint32_t)n;
        d.scap = ctx->ed_scap;
        d.pk_rows = reinterpret_cast<const uint32_t*>(pk_raw);
        d.sig_rows = reinterpret_cast<const uint32_t*>(sig_raw);
        d.pk_row_words = (uint32_t)(pk_stride / 4);
        d.sig_row_words = (uint32_t)(sig_stride / 4);
        d.pstat = ctx->ed_status + ctx->ed_scap;
        d.table = ctx->ed_table;
        for (int half = 0; half < 2; ++half) {
          hipError_t e2 = half ? hipMemcpyAsync(sig_raw, sig, n * sig_stride, hipMemcpyHostToDevice, ctx->stream)
                               : hipMemcpyAsync(pk_raw, pk, n * pk_stride, hipMemcpyHostToDevice, ctx->stream);
          if (e2 == hipSuccess) e2 = hipEventRecord(ctx->ev_rows, ctx->stream);
          if (e2 == hipSuccess) e2 = hipStreamWaitEvent(ctx->copy_stream, ctx->ev_rows, 0);
          if (e2 != hipSuccess) return bail(hip_fail(ctx, e2, "upload rows"));
          b->points_early = true;  // (from here on copy_stream may hold work: bail syncs it)
          Timed t(ctx, half ? "ed25519_points_r" : "ed25519_points_a", n, ctx->copy_stream);
          e2 = cg::launch_ed25519_points_half(d, half, (uint32_t)n, ctx->copy_stream);
          if (e2 != hipSuccess) return bail(hip_fail(ctx, e2, "launch ed25519_points"));
        }
        const hipError_t e2 = hipEventRecord(ctx->ev_pts_done, ctx->copy_stream);
        if (e2 != hipSuccess) return bail(hip_fail(ctx, e2, "points done"));
      } else if (parts > 1) {
        if ((st = ensure_ed_scratch(ctx, (uint32_t)n)) != CG_OK ||
            (st = dalloc(ctx, &pk_raw, n * pk_stride, "alloc pk")) != CG_OK ||
            (st = dalloc(ctx, &sig_raw, n * sig_stride, "alloc sig")) != CG_OK)
          return bail(st);
        for (uint32_t p = 0; p < parts; ++p) {  // part boundaries: whole 256-lane blocks
          const size_t lo = (size_t)(((uint64_t)n * p / parts) & ~(uint64_t)255);
          const size_t hi = p + 1 == parts ? n : (size_t)(((uint64_t)n * (p + 1) / parts) & ~(uint64_t)255);
          hipError_t e2 = hipMemcpyAsync(pk_raw + lo * pk_stride, pk + lo * pk_stride, (hi - lo) * pk_stride,
                                         hipMemcpyHostToDevice, ctx->stream);
          if (e2 == hipSuccess)
            e2 = hipMemcpyAsync(sig_raw + lo * sig_stride, sig + lo * sig_stride, (hi - lo) * sig_stride,
                                hipMemcpyHostToDevice, ctx->stream);
          if (e2 == hipSuccess) e2 = hipEventRecord(ctx->ev_rows, ctx->stream);
          if (e2 == hipSuccess) e2 = hipStreamWaitEvent(ctx->copy_stream, ctx->ev_rows, 0);
          if (e2 != hipSuccess) return bail(hip_fail(ctx, e2, "upload rows"));
          b->points_early = true;  // (from here on copy_stream may hold work: bail syncs it)
          cg::Ed25519Dev d;
          d.cap = (uint32_t)n;
          d.scap = ctx->ed_scap;
          d.pk_rows = reinterpret_cast<const uint32_t*>(pk_raw + lo * pk_stride);
          d.sig_rows = reinterpret_cast<const uint32_t*>(sig_raw + lo * sig_stride);
          d.pk_row_words = (uint32_t)(pk_stride / 4);
          d.sig_row_words = (uint32_t)(sig_stride / 4);
          d.pstat = ctx->ed_status + ctx->ed_scap + lo;
          d.table = ctx->ed_table + cg::ed25519_table_offset((uint32_t)lo);
          Timed t(ctx, "ed25519_points", hi - lo, ctx->copy_stream);
          e2 = cg::launch_ed25519_points(d, (uint32_t)(hi - lo), ctx->copy_stream);
          if (e2 != hipSuccess) return bail(hip_fail(ctx, e2, "launch ed25519_points"));
        }
        const hipError_t e2 = hipEventRecord(ctx->ev_pts_done, ctx->copy_stream);
        if (e2 != hipSuccess) return bail(hip_fail(ctx, e2, "points done"));
      } else {
        if ((st = upload(ctx, &pk_raw, pk, n * pk_stride, "upload pk")) != CG_OK) return bail(st);
        if ((st = upload(ctx, &sig_raw, sig, n * sig_stride, "upload sig")) != CG_OK) return bail(st);
        if (rows_direct && hipEventRecord(ctx->ev_rows, ctx->stream) == hipSuccess) {
          b->rows_event = true;
          b->raw_pk_words = (uint32_t)(pk_stride / 4);
          b->raw_sig_words = (uint32_t)(sig_stride / 4);
        }
      }
      if (sig_len && (st = upload(ctx, &sl_raw, sig_len, n, "upload sig_len")) != CG_OK) return bail(st);
    }
  }
  if (!raw_owned) {
    pk_raw = const_cast<uint8_t*>(m.pk_dev);
    sig_raw = const_cast<uint8_t*>(m.sig_dev);
    sl_raw = const_cast<uint32_t*>(m.sl_dev);
    if (m.raw_ready) {
      const hipError_t e = hipStreamWaitEvent(ctx->stream, m.raw_ready, 0);
      if (e != hipSuccess) return bail(hip_fail(ctx, e, "wait raw rows"));
    }
  } else if (m.dev) {
    if ((st = upload(ctx, &pk_raw, pk, n * pk_stride, "upload pk")) != CG_OK) return bail(st);
    if ((st = upload(ctx, &sig_raw, sig, n * sig_stride, "upload sig")) != CG_OK) return bail(st);
    if (sig_len && (st = upload(ctx, &sl_raw, sig_len, n, "upload sig_len")) != CG_OK) return bail(st);
  }
  if (!bad.empty()) {
    b->n_bad = (uint32_t)bad.size();
    if ((st = upload_idx(ctx, &b->bad_index, bad.data(), bad.size(), "upload key-invalid index")) != CG_OK)
      return bail(st);
  }
  {
    Timed t(ctx, "stage", n);
    // Ed25519 subset -> SoA
    const uint32_t ne = (uint32_t)n_ed;
    b->n_ed = ne;
    if (ne) {
      if (!ed_identity && (st = upload_idx(ctx, &b->ed_index, idx[0].data(), ne, "upload ed index")) != CG_OK)
        return bail(st);
      b->ed_meta_alias = meta_deferred;  // (the offsets / lengths are not on the device yet: no gather)
      if (b->ed_meta_alias) {  // (identity order: the gathered copies would equal them)
        b->ed_msg_off = b->msg_off_all;
        b->ed_msg_len = b->msg_len_all;
      }
      if ((st = dalloc(ctx, &b->ed_pk, (size_t)8 * ne, "alloc ed pk")) != CG_OK ||
          (st = dalloc(ctx, &b->ed_sig, (size_t)16 * ne, "alloc ed sig")) != CG_OK ||
          (st = dalloc(ctx, &b->ed_sig_len, ne, "alloc ed sig_len")) != CG_OK ||
          (!b->ed_meta_alias && (st = dalloc(ctx, &b->ed_msg_off, ne, "alloc ed msg_off")) != CG_OK) ||
          (!b->ed_meta_alias && (st = dalloc(ctx, &b->ed_msg_len, ne, "alloc ed msg_len")) != CG_OK))
        return bail(st);
      hipError_t e = cg::launch_gather_words(pk_raw, pk_stride, 0, 8, b->ed_index, ne, ne, b->ed_pk, ctx->stream);
      if (e == hipSuccess)
        e = cg::launch_gather_words(sig_raw, sig_stride, 0, 16, b->ed_index, ne, ne, b->ed_sig, ctx->stream);
      if (e == hipSuccess)
        e = cg::launch_gather_u32(sl_raw, b->ed_index, ne, b->ed_sig_len, (uint32_t)sig_stride, ctx->stream);
      if (e == hipSuccess && !b->ed_meta_alias)
        e = cg::launch_gather_u64(b->msg_off_all, b->ed_index, ne, b->ed_msg_off, ctx->stream);
      if (e == hipSuccess && !b->ed_meta_alias)
        e = cg::launch_gather_u32(b->msg_len_all, b->ed_index, ne, b->ed_msg_len, 0, ctx->stream);
      if (e != hipSuccess) return bail(hip_fail(ctx, e, "stage ed25519"));
      if ((st = stage_key_dedupe(ctx, b, pk, pk_stride, idx[0], key_sample)) != CG_OK) return bail(st);
    }
    for (int c = 0; c < 2; ++c) {
      const std::vector<uint32_t>& ix = idx[1 + c];
      if (ix.empty()) continue;
      cg::EcdsaBatch& eb = b->ec[c];
      const size_t ne_c = ix.size();
      eb.n = (uint32_t)ne_c;
      eb.scheme = c == 0 ? CG_SCHEME_ECDSA_SECP256K1_SHA256 : CG_SCHEME_ECDSA_SECP256R1_SHA256;
      if ((st = upload_idx(ctx, &eb.index, ix.data(), ne_c, "upload ecdsa index")) != CG_OK ||
          (st = dalloc(ctx, &eb.q, 16 * ne_c, "alloc ecdsa q")) != CG_OK ||
          (st = dalloc(ctx, &eb.rs, 16 * ne_c, "alloc ecdsa rs")) != CG_OK ||
          (st = dalloc(ctx, &eb.der, ne_c, "alloc ecdsa der")) != CG_OK ||
          (st = dalloc(ctx, &eb.sig_len, ne_c, "alloc ecdsa sig_len")) != CG_OK ||
          (st = dalloc(ctx, &eb.msg_off, ne_c, "alloc ecdsa msg_off")) != CG_OK ||
          (st = dalloc(ctx, &eb.msg_len, ne_c, "alloc ecdsa msg_len")) != CG_OK)
        return bail(st);
      hipError_t e = cg::ecdsa_batch_stage(eb, pk_raw, pk_stride, sig_raw, sig_stride, sl_raw, b->msg_off_all,
                                           b->msg_len_all, ctx->stream);
      if (e != hipSuccess) return bail(hip_fail(ctx, e, "stage ecdsa"));
      if (raw_owned) {  // the batch keeps this subset's rows (only) for its per-verify DER parse
        if ((st = dalloc(ctx, &b->ec_rows[c], ne_c * sig_stride, "alloc ecdsa rows")) != CG_OK ||
            (sl_raw && (st = dalloc(ctx, &b->ec_row_len[c], ne_c, "alloc ecdsa row lengths")) != CG_OK))
          return bail(st);
        b->ec_sig_stride = sig_stride;
        e = cg::launch_gather_rows(sig_raw, sig_stride, eb.index, (uint32_t)ne_c, b->ec_rows[c], ctx->stream);
        if (e == hipSuccess && sl_raw)
          e = cg::launch_gather_u32(sl_raw, eb.index, (uint32_t)ne_c, b->ec_row_len[c], 0, ctx->stream);
        if (e != hipSuccess) return bail(hip_fail(ctx, e, "keep ecdsa rows"));
      }
    }
  }
  // the host index vectors die here: wait for the copies that read them (unless every
  // one went through the pinned staging area of an asynchronous tx-pipeline stage, or
  // the batch keeps them: keep_raw)
  if (m.keep_raw && raw_owned) {  // freed with the batch, after the caller's sync
    b->raw_kept[0] = pk_raw;
    b->raw_kept[1] = sig_raw;
    b->raw_kept[2] = sl_raw;
    pk_raw = sig_raw = nullptr;
    sl_raw = nullptr;
  }
  if (m.keep_raw) {  // no sync below: the copies may still read the index vectors
    for (int c = 0; c < 3; ++c) b->idx_kept[c].swap(idx[c]);
    b->idx_kept[3].swap(bad);
  }
  hipError_t e = ((m.async || m.keep_raw) && ctx->pin_fallbacks == fallbacks0) ? hipSuccess
                                                                               : hipStreamSynchronize(ctx->stream);
  free_raw();
  if (e != hipSuccess) return bail(hip_fail(ctx, e, "stage sync"));
  if (beside.posted) {
    const size_t i = beside.wait();
    if (i < n) return bail(fail(ctx, CG_E_INVALID_ARGUMENT, out_of_arena_message(i)));
  }
  if (!m.async && !m.keep_raw && !ctx->call_begin)
    collect_timings(ctx);  // (it waits on every pending span: the pipeline collects at its end)
  *out = b;
  return CG_OK;
}

// ECDSA scratch for one curve; on out-of-memory the context's cached blocks are
// returned to the device and the allocation retried once (as dalloc_bytes does).
cg_status ecdsa_scratch_retry(cg_ctx* ctx, int scheme, uint32_t n, uint32_t* chunk) {
  hipError_t e = debug_alloc_fails(ctx) ? hipErrorOutOfMemory : cg::ecdsa_scratch(ctx->ec, scheme, n, chunk);
  if (e == hipErrorOutOfMemory) {
    (void)hipGetLastError();
    for (hipStream_t s : {ctx->stream, ctx->ec_stream[0], ctx->ec_stream[1]}) (void)hipStreamSynchronize(s);
    release_cached(ctx);
    e = debug_alloc_fails(ctx) ? hipErrorOutOfMemory : cg::ecdsa_scratch(ctx->ec, scheme, n, chunk);
  }
  return e == hipSuccess ? CG_OK : hip_fail(ctx, e, "alloc ecdsa scratch");
}

// Orders ctx->stream after everything the ECDSA streams hold so far.
cg_status join_ecdsa_streams(cg_ctx* ctx) {
  for (int c = 0; c < 2; ++c) {
    CG_TRY(ctx, hipEventRecord(ctx->ev_join[c], ctx->ec_stream[c]), "record ecdsa join");
    CG_TRY(ctx, hipStreamWaitEvent(ctx->stream, ctx->ev_join[c], 0), "join ecdsa");
  }
  return CG_OK;
}

// Launches the verify kernels of a staged batch and the accept bitmap; no sync.
// Every exit — success or error — leaves ctx->stream ordered after the ECDSA
// streams it forked, so the caller's stream-ordered frees (batch_free, the block
// cache) can never hand a buffer to new work while an ECDSA kernel still writes it.
// join_streams = false (the tx pipeline): a successful exit leaves the ECDSA work
// running on its streams and skips the bitmap; the caller joins once after the last
// batch and frees the batches only after its final sync.
// scratch_off / scratch_lanes: the batch's Ed25519 lanes may use scratch lanes
// [scratch_off, scratch_off + scratch_lanes) (0: to the end; the verify pipeline runs
// two chunks at once on disjoint halves); the four-lane latency mode needs 2 n_ed.
// Ed25519 points kernels beside the hash kernels on `pts_stream` (null: after them on
// the same stream); CORDA_AMD_ED_OVERLAP=0 turns it off.


cg_status launch_verify(cg_ctx* ctx, cg_batch* b, int mode, bool join_streams = true, uint32_t scratch_off = 0,
                        hipStream_t pts_stream = nullptr, uint32_t scratch_lanes = 0, bool allow_lanes = true) {
  const size_t n = b->n;
  bool joins[2] = {false, false};
  cg_status st = CG_OK;
  auto join = [&]() {
    for (int c = 0; c < 2; ++c)
      if (joins[c]) {  // recorded here, after whatever this curve's stream got (all of it, or up to a failure)
        hipError_t e = hipEventRecord(ctx->ev_join[c], ctx->ec_stream[c]);
        if (e == hipSuccess) e = hipStreamWaitEvent(ctx->stream, ctx->ev_join[c], 0);
        if (e != hipSuccess) {  // cannot order the streams: wait on the host instead
          (void)hipGetLastError();
          (void)hipStreamSynchronize(ctx->ec_stream[c]);
          if (st == CG_OK) st = hip_fail(ctx, e, "join ecdsa");
        }
        joins[c] = false;
      }
  };
  auto run = [&]() -> cg_status {
    // elements of unsupported schemes keep this value
    CG_TRY(ctx, hipMemsetAsync(b->verdict, CG_UNSUPPORTED, n, ctx->stream), "init verdict");
    // keys the caller could not construct: KEY_INVALID (no verify kernel touches them)
    CG_TRY(ctx, cg::launch_fill_index(b->bad_index, b->n_bad, b->verdict, CG_KEY_INVALID, ctx->stream),
           "launch key-invalid fill");
    CG_TRY(ctx, hipEventRecord(ctx->ev_fork, ctx->stream), "fork ecdsa");
    bool keys_pending = false;
    if (b->n_ed && b->ed_key_index) {
      // key-reuse path: every distinct key decoded once and its tables built once, on
      // ec_stream[0] beside the hash kernel (one wave per 64 keys: latency-bound, it
      // would otherwise serialize ~0.6 ms on the main stream); the points kernel waits
      cg_status s2 = ensure_key_scratch(ctx, b->n_keys);
      if (s2 != CG_OK) return s2;
      hipStream_t ks = ctx->ec_stream[0];
      CG_TRY(ctx, hipStreamWaitEvent(ks, ctx->ev_fork, 0), "fork keyprep");
      joins[0] = true;
      cg::Ed25519Dev kd;
      kd.pk = b->ed_pk;
      kd.cap = b->n_ed;
      kd.ktab = ctx->ed_ktab;
      kd.kstat = ctx->ed_kstat;
      {
        Timed t(ctx, "ed25519_keyprep", b->n_keys, ks);
        CG_TRY(ctx, cg::launch_ed25519_keyprep(kd, b->ed_key_first, b->n_keys, ks), "launch ed25519_keyprep");
      }
      CG_TRY(ctx, hipEventRecord(ctx->ev_keys, ks), "keyprep ready");
      keys_pending = true;
    }
    // ECDSA: each curve on its own stream, forked after the verdict init and joined
    // before the bitmap (the verdict scatters touch disjoint positions); enqueued
    // first so they overlap the Ed25519 kernels below in mixed batches (config 4:
    // 14.9 -> 15.3 M tx/s; per-kernel times then include the overlap)
    for (int c = 0; c < 2; ++c) {
      if (!b->ec[c].n) continue;
      const cg::EcdsaBatch& eb = b->ec[c];
      const char* prep_name = eb.scheme == 2 ? "ecdsa_k1_prep" : "ecdsa_r1_prep";
      const char* msm_name = eb.scheme == 2 ? "ecdsa_k1_msm" : "ecdsa_r1_msm";
      hipStream_t es = ctx->ec_stream[c];
      uint32_t chunk = 0;
      cg_status s2 = ecdsa_scratch_retry(ctx, eb.scheme, eb.n, &chunk);
      if (s2 != CG_OK) return s2;
      CG_TRY(ctx, hipStreamWaitEvent(es, ctx->ev_fork, 0), "fork ecdsa");
      joins[c] = true;  // from here on this curve's stream may hold work: the exit path joins it
      if (b->ec_rows[c]) {  // K4: strict DER -> r, s + status, from the kept (compacted) raw rows
        Timed t(ctx, eb.scheme == 2 ? "ecdsa_k1_der" : "ecdsa_r1_der", eb.n, es);
        CG_TRY(ctx,
               cg::launch_der_parse(eb.scheme, b->ec_rows[c], b->ec_sig_stride, b->ec_row_len[c],
                                    (uint32_t)b->ec_sig_stride, nullptr, eb.n, eb.n, eb.rs, eb.der, es),
               "launch ecdsa der parse");
      }
      for (uint32_t base = 0; base < eb.n; base += chunk) {
        const uint32_t cnt = std::min(chunk, eb.n - base);
        {
          Timed t(ctx, prep_name, cnt, es);
          CG_TRY(ctx, cg::ecdsa_launch_prep(eb, ctx->ec, base, cnt, b->arena, (uint32_t)mode, es), "launch ecdsa prep");
        }
        {
          Timed t(ctx, msm_name, cnt, es);
          CG_TRY(ctx, cg::ecdsa_launch_msm(eb, ctx->ec, base, cnt, b->verdict, es), "launch ecdsa msm");
        }
      }
    }
    if (b->n_ed) {
      const uint32_t pair_max = ed_pair_max(ctx, b->pair_max);
      // four lanes per signature: tables in 2 n_ed scratch slots — grown for it only where
      // this call owns the whole scratch; inside a pipeline only if its region has room
      const bool quad_want = !b->ed_key_index && b->n_ed <= std::min(pair_max, cg::ed_quad_max(ctx->opts));
      const bool oct_want = quad_want && b->n_ed <= cg::ed_oct_max(ctx->opts);
      cg_status s2 = ensure_ed_scratch(
          ctx, quad_want && join_streams && scratch_off == 0 ? (oct_want ? 4 : 2) * b->n_ed : b->n_ed);
      if (s2 != CG_OK) return s2;
      const uint32_t region = scratch_lanes ? scratch_lanes : ctx->ed_scap - scratch_off;
      const bool quad_ok = quad_want && 2 * (uint64_t)b->n_ed <= region;
      const bool oct_ok = oct_want && 4 * (uint64_t)b->n_ed <= region;
      const uint32_t span = ctx->ed_scap - scratch_off;  // scratch lanes this batch may use
      // Large batches run as `split` index pieces alternating between ctx->stream and
      // hash_stream (each piece on its own scratch lanes), so one piece's kernels fill
      // the SIMDs another piece's kernel leaves idle while its last waves drain.  Only
      // when this call owns the streams (join_streams: not inside verify_pipeline).
      uint32_t split = 1;
      if (join_streams && b->n_ed >= 2 * kEdSplitMin && b->n_ed <= span) {
        split = kEdSplitDefault;
        if (ctx->opts.has(cg::OPT_ED_SPLIT)) split = (uint32_t)std::max(1, ctx->opts.i(cg::OPT_ED_SPLIT, 1));
        split = std::min<uint32_t>(split, b->n_ed / kEdSplitMin);
      }
      hipStream_t ed_lane[2] = {ctx->stream, ctx->hash_stream};
      // Points kernel beside the hash kernel on the idle copy stream (this call owns the
      // streams) when the call still waits on host copies — a one-chunk host-buffer call:
      // the points kernel reads the raw rows while the arena goes up.  A resident batch runs
      // it after the hash kernel: side by side the two VALU-bound kernels took longer than
      // one after the other once the hash kernel stopped spilling (r06i, config 2: 99.7 ->
      // 100.9 M/s over three interleaved pairs).  CORDA_AMD_ED_OVERLAP=0: never beside, 2:
      // always (the round-5 plan).
      const int overlap = ctx->opts.i(cg::OPT_ED_OVERLAP, 1);
      const bool copies_pending = b->rows_event || b->points_early || b->arena_pending || b->arena_job;
      hipStream_t pts = pts_stream ? pts_stream
                                   : (join_streams && (overlap >= 2 || (overlap == 1 && copies_pending)) ? ctx->copy_stream
                                                                                                         : nullptr);
      if (split > 1) {
        if (b->arena_job) {  // (never with split pieces: cg_plan.h's static_assert; kept safe anyway)
          b->arena_job->wait();
          const hipError_t e2 = b->arena_job->err;
          give_back_events(ctx, b->arena_job->span[0], b->arena_job->span[1]);
          b->arena_job.reset();
          CG_TRY(ctx, e2, "upload arena");
          CG_TRY(ctx, hipStreamWaitEvent(ctx->stream, ctx->ev_arena, 0), "wait arena");
          CG_TRY(ctx, hipStreamWaitEvent(ctx->hash_stream, ctx->ev_arena, 0), "wait arena");
        }
        if (b->arena_pending) {  // every piece's hash kernel reads the arena: it goes up before the fork
          {
            Timed t(ctx, "h2d_arena", b->arena_pending_bytes);
            CG_TRY(ctx,
                   hipMemcpyAsync(b->arena, b->arena_pending, b->arena_pending_bytes, hipMemcpyHostToDevice,
                                  ctx->stream),
                   "upload arena");
            if (b->meta_pending_off) {
              CG_TRY(ctx, hipMemcpyAsync(b->msg_off_all, b->meta_pending_off, b->n * 8, hipMemcpyHostToDevice,
                                         ctx->stream), "upload msg_off");
              CG_TRY(ctx, hipMemcpyAsync(b->msg_len_all, b->meta_pending_len, b->n * 4, hipMemcpyHostToDevice,
                                         ctx->stream), "upload msg_len");
            }
          }
          b->arena_pending = nullptr;
          b->meta_pending_off = nullptr;
          b->meta_pending_len = nullptr;
          CG_TRY(ctx, hipEventRecord(ctx->ev_arena, ctx->stream), "arena done");
          CG_TRY(ctx, hipStreamWaitEvent(ctx->hash_stream, ctx->ev_arena, 0), "fork ed25519 split");
        }
        CG_TRY(ctx, hipStreamWaitEvent(ctx->hash_stream, ctx->ev_fork, 0), "fork ed25519 split");
      }
      // create_batch's early points kernels cover the whole batch as one balanced piece;
      // any other plan recomputes them, after they are done
      const bool early = b->points_early && pts && split == 1 && !b->ed_key_index && b->n_ed <= span &&
                         !(allow_lanes && b->n_ed <= pair_max);
      if (b->points_early && !early) {
        CG_TRY(ctx, hipStreamWaitEvent(ctx->stream, ctx->ev_pts_done, 0), "join early points");
        if (split > 1) CG_TRY(ctx, hipStreamWaitEvent(ctx->hash_stream, ctx->ev_pts_done, 0), "join early points");
      }
      struct StreamBack {  // ctx->stream is the piece's lane inside the loop; restored on every exit
        cg_ctx* c;
        hipStream_t main;
        ~StreamBack() { c->stream = main; }
      } back{ctx, ctx->stream};
      for (uint32_t base = 0, piece = 0; base < b->n_ed; ++piece) {
        uint32_t cnt = std::min(span, b->n_ed - base);
        if (split > 1)  // piece sizes: whole 256-lane blocks, the last one takes the rest
          cnt = piece + 1 == split ? b->n_ed - base : (uint32_t)(((uint64_t)b->n_ed / split + 255) / 256 * 256);
        ctx->stream = ed_lane[piece & 1 & (split > 1)];
        const uint32_t soff = scratch_off + (split > 1 ? base : 0);  // scratch lanes of this piece
        cg::Ed25519Dev d;
        d.cap = b->n_ed;
        d.scap = ctx->ed_scap;
        d.pk = b->ed_pk + base;
        d.sig = b->ed_sig + base;
        d.sig_len = b->ed_sig_len + base;
        d.arena = b->arena;
        d.msg_off = b->ed_msg_off + base;
        d.msg_len = b->ed_msg_len + base;
        d.status = ctx->ed_status + soff;
        d.pstat = ctx->ed_status + ctx->ed_scap + soff;
        d.digits = ctx->ed_digits + soff;  // rows keep their stride scap
        d.table = ctx->ed_table + cg::ed25519_table_offset(soff);
        d.btab = ctx->btab;
        d.full_mod = ctx->debug_full_mod;
        d.index_base = base;
        if (b->ed_key_index) {
          d.key_index = b->ed_key_index + base;
          d.ktab = ctx->ed_ktab;
          d.kstat = ctx->ed_kstat;
        }
        const bool pair = allow_lanes && !b->ed_key_index && cnt <= pair_max;  // latency mode
        // balanced MSM over lanes grouped by digit count
        if (!pair && !b->ed_key_index && cnt >= cg::ed_bucket_min(ctx->opts)) {
          d.order = ctx->ed_status + 2 * (size_t)ctx->ed_scap + soff;
          d.order_count = ctx->ed_status + 5 * (size_t)ctx->ed_scap + soff;
        }
        // (quad_ok / oct_ok: one piece with 2 / 4 cnt scratch slots in its region)
        const uint32_t lanes = !pair ? 1u : oct_ok && split == 1 ? 8u : quad_ok && split == 1 ? 4u : 2u;
        if (pair)
          ed_spread_lds(ctx, d, ((uint64_t)lanes * cnt + 255) / 256, (cnt + 255) / 256,
                        join_streams ? ctx->n_cu : std::max(1u, ctx->n_cu / 2));
        auto launch_points = [&](hipStream_t ps) -> cg_status {
          Timed t(ctx, lanes == 8   ? "ed25519_points_oct"
                       : lanes == 4 ? "ed25519_points_quad"
                       : pair       ? "ed25519_points_pair"
                                    : "ed25519_points",
                  cnt, ps);
          CG_TRY(ctx, pair ? cg::launch_ed25519_points_lanes(d, cnt, lanes, ps) : cg::launch_ed25519_points(d, cnt, ps),
                 "launch ed25519_points");
          return CG_OK;
        };
        // create_batch's deferred arena (one-chunk verify).  Beside the points kernel (the
        // pts path) an arena of 6 MB or more goes on hash_stream, so its copy starts as soon
        // as it is issued instead of behind the staging kernel on ctx->stream, and the hash
        // kernel waits for it (r04ad: 8,192-65,536 x 1 KB -0.02..0.05 ms; at 4,096 the
        // cross-stream wait cost more than the copy's head start, +0.01 ms).
        // CORDA_AMD_ARENA_BESIDE=0 keeps it on ctx->stream.
        auto upload_pending_arena = [&](bool beside) -> cg_status {
          if (b->arena_job) {  // issued by the upload thread: the hash kernel waits for ev_arena
            b->arena_job->wait();
            const hipError_t e2 = b->arena_job->err;
            if (e2 == hipSuccess && b->arena_job->span[0] && b->arena_job->span[1]) {
              ctx->pending.push_back({"h2d_arena", {b->arena_job->span[0], b->arena_job->span[1]}});
              ctx->stats["h2d_arena"].items += b->arena_job->bytes;
            } else {
              give_back_events(ctx, b->arena_job->span[0], b->arena_job->span[1]);
            }
            b->arena_job.reset();
            CG_TRY(ctx, e2, "upload arena");
            CG_TRY(ctx, hipStreamWaitEvent(ctx->stream, ctx->ev_arena, 0), "wait arena");
            return CG_OK;
          }
          if (!b->arena_pending) return CG_OK;
          const size_t pending = b->arena_pending_bytes + (b->meta_pending_off ? (size_t)12 * b->n : 0);
          hipStream_t as = beside && split == 1 && pending >= ((size_t)6 << 20) &&
                                   ctx->opts.on(cg::OPT_ARENA_BESIDE, true)
                               ? ctx->hash_stream
                               : ctx->stream;
          {
            Timed t(ctx, "h2d_arena", b->arena_pending_bytes, as);
            CG_TRY(ctx, hipMemcpyAsync(b->arena, b->arena_pending, b->arena_pending_bytes, hipMemcpyHostToDevice, as),
                   "upload arena");
            if (b->meta_pending_off) {
              CG_TRY(ctx, hipMemcpyAsync(b->msg_off_all, b->meta_pending_off, b->n * 8, hipMemcpyHostToDevice, as),
                     "upload msg_off");
              CG_TRY(ctx, hipMemcpyAsync(b->msg_len_all, b->meta_pending_len, b->n * 4, hipMemcpyHostToDevice, as),
                     "upload msg_len");
            }
          }
          b->arena_pending = nullptr;
          b->meta_pending_off = nullptr;
          b->meta_pending_len = nullptr;
          if (as != ctx->stream) {
            CG_TRY(ctx, hipEventRecord(ctx->ev_arena, as), "arena done");
            CG_TRY(ctx, hipStreamWaitEvent(ctx->stream, ctx->ev_arena, 0), "wait arena");
          }
          return CG_OK;
        };
        if (early) {  // points already running on copy_stream since the rows' arrival
          if ((s2 = upload_pending_arena(true)) != CG_OK) return s2;
          {
            Timed t(ctx, "ed25519_hash", cnt);
            CG_TRY(ctx, cg::launch_ed25519_hash(d, cnt, (uint32_t)mode, ctx->stream), "launch ed25519_hash");
          }
          CG_TRY(ctx, hipStreamWaitEvent(ctx->stream, ctx->ev_pts_done, 0), "join points");
        } else if (pts) {
          // the points kernel needs only the rows (ready where this lane stands now):
          // it runs on pts beside the hash kernel, and the MSM waits for both.  In a
          // one-chunk call it reads the raw rows and waits only for their copy, not for
          // the staging kernels (r05 spans: 4,096 x 1 KB ~0.05 ms, 65,536 x 32 B ~0.05 ms)
          hipEvent_t in = ctx->ev_pts_in;
          if (b->rows_event && !b->ed_key_index && split == 1 && base == 0 && cnt == b->n_ed) {
            d.pk_rows = static_cast<const uint32_t*>(b->raw_kept[0]);
            d.sig_rows = static_cast<const uint32_t*>(b->raw_kept[1]);
            d.pk_row_words = b->raw_pk_words;
            d.sig_row_words = b->raw_sig_words;
            in = ctx->ev_rows;
          } else {
            CG_TRY(ctx, hipEventRecord(ctx->ev_pts_in, ctx->stream), "fork points");
          }
          CG_TRY(ctx, hipStreamWaitEvent(pts, in, 0), "fork points");
          if (keys_pending && piece == 0) CG_TRY(ctx, hipStreamWaitEvent(pts, ctx->ev_keys, 0), "wait keyprep");
          if ((s2 = launch_points(pts)) != CG_OK) return s2;
          CG_TRY(ctx, hipEventRecord(ctx->ev_pts_done, pts), "points done");
          if ((s2 = upload_pending_arena(true)) != CG_OK) return s2;
          {
            Timed t(ctx, "ed25519_hash", cnt);
            CG_TRY(ctx, cg::launch_ed25519_hash(d, cnt, (uint32_t)mode, ctx->stream), "launch ed25519_hash");
          }
          CG_TRY(ctx, hipStreamWaitEvent(ctx->stream, ctx->ev_pts_done, 0), "join points");
        } else {
          if ((s2 = upload_pending_arena(false)) != CG_OK) return s2;
          {
            Timed t(ctx, "ed25519_hash", cnt);
            CG_TRY(ctx, cg::launch_ed25519_hash(d, cnt, (uint32_t)mode, ctx->stream), "launch ed25519_hash");
          }
          if (keys_pending && piece < std::min<uint32_t>(split, 2))  // each lane's first points kernel
            CG_TRY(ctx, hipStreamWaitEvent(ctx->stream, ctx->ev_keys, 0), "wait keyprep");
          if ((s2 = launch_points(ctx->stream)) != CG_OK) return s2;
        }
        const uint32_t* oi = b->ed_index ? b->ed_index + base : nullptr;
        uint8_t* vd = b->ed_index ? b->verdict : b->verdict + base;
        if (d.order) {
          Timed t(ctx, "ed25519_bucket", cnt);
          CG_TRY(ctx, cg::launch_ed25519_bucket(d, cnt, oi, vd, ctx->stream), "launch ed25519_bucket");
        }
        {
          Timed t(ctx, lanes == 8 ? "ed25519_msm_oct" : lanes == 4 ? "ed25519_msm_quad" : pair ? "ed25519_msm_pair" : "ed25519_msm",
                  cnt);
          CG_TRY(ctx,
                 pair ? cg::launch_ed25519_msm_lanes(d, cnt, lanes, oi, vd, ctx->stream)
                      : cg::launch_ed25519_msm(d, cnt, oi, vd, ctx->stream),
                 "launch ed25519_msm");
        }
        base += cnt;
      }
      ctx->stream = back.main;
      if (split > 1) {  // the main stream continues once the other lane's pieces are done
        CG_TRY(ctx, hipEventRecord(ctx->ev_split, ctx->hash_stream), "split join");
        CG_TRY(ctx, hipStreamWaitEvent(ctx->stream, ctx->ev_split, 0), "split join");
      }
    }
    return CG_OK;
  };
  st = run();
  if (st != CG_OK) {  // a split's other lane or the points stream may hold work
    (void)hipStreamSynchronize(ctx->hash_stream);
    (void)hipStreamSynchronize(ctx->copy_stream);
    if (pts_stream) (void)hipStreamSynchronize(pts_stream);
  }
  if (st != CG_OK || join_streams) join();
  if (st != CG_OK || !join_streams) return st;
  CG_TRY(ctx, cg::launch_verdict_bitmap(b->verdict, (uint32_t)n, b->bitmap, ctx->stream), "launch bitmap");
  return CG_OK;
}

// ------------------------------------------------------------ host-buffer verify
// cg_verify_batch is what a JVM caller hits (Crypto.isValid / doVerify in a loop,
// Crypto.kt:534-541): host buffers in, verdicts out.  Uploading the whole batch and
// then verifying it leaves the GPU idle for the PCIe transfer (~20 ns per 1 KB
// signature at ~57 GB/s, twice the kernels' ~10 ns).  The pipeline cuts the batch
// into index-range chunks: chunk k's rows and the arena prefix its messages reach
// are copied on copy_stream while chunk k-1's kernels run on the compute streams, so
// the call costs the transfer plus the last chunk's kernels.  The last chunk is the
// smallest (`tail` of a regular chunk): only its kernels run after the last byte.
// Consecutive chunks alternate between two compute streams (ctx->stream and
// hash_stream) over disjoint halves of the Ed25519 scratch, so a chunk's kernels
// start as soon as its bytes land instead of queueing behind the previous chunk's
// (each chunk's three kernels are a serial ~1 ms chain per lane, whatever its size).
struct VerifyRun {
  uint8_t* arena = nullptr;
  // every chunk's per-element arrays as one chunk-major block (ChunkRows): a staged
  // chunk's rows go up in one DMA
  uint8_t* rows = nullptr;
  uint8_t* verdict = nullptr;
  uint32_t* bitmap = nullptr;
  std::vector<hipEvent_t> ev;
  std::vector<cg_batch*> batches;  // chunk batches (verdicts are slices of `verdict`)
  void release(cg_ctx* ctx) {
    for (hipStream_t s : {ctx->copy_stream, ctx->hash_stream, ctx->ec_stream[0], ctx->ec_stream[1], ctx->stream})
      (void)hipStreamSynchronize(s);
    for (cg_batch* b : batches) batch_free(ctx, b);
    batches.clear();
    for (hipEvent_t e : ev)
      if (e) ctx->sync_event_pool.push_back(e);  // (idle after the syncs above)
    ev.clear();
    for (const void* p : {(const void*)arena, (const void*)rows, (const void*)verdict, (const void*)bitmap}) dfree(ctx, p);
    arena = rows = verdict = nullptr;
    bitmap = nullptr;
  }
};

// (copy-bound vs compute-bound calls and their chunk bounds: cg_plan.h plan_verify)

// Page-locked host memory (cg_register_host, hipHostMalloc): a copy from it is truly
// asynchronous.  A pageable copy is staged by the runtime and holds the calling thread.
bool host_is_pinned(const void* p) {
  if (!p) return true;
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

// The end of a host-buffer verify: verdicts (and the accept bitmap) to the caller's
// buffers, then the stream sync.  Pageable buffers take the copies through a
// page-locked bounce buffer (DMA, then a host memcpy after the sync): a pageable
// device-to-host copy is staged by the runtime, ~0.17 ms for 262,144 verdicts (r04l
// spans) against ~0.01 ms of DMA.
cg_status download_verdicts(cg_ctx* ctx, uint8_t* verdict_out, const uint8_t* verdict, size_t n,
                            uint32_t* bitmap_out, const uint32_t* bitmap, size_t nwords) {
  const size_t vb = verdict_out ? (n + 255) & ~(size_t)255 : 0, bb = bitmap_out ? nwords * 4 : 0;
  bool bounce = (verdict_out && !host_is_pinned(verdict_out)) || (bitmap_out && !host_is_pinned(bitmap_out));
  if (bounce && ctx->dl_pin_cap < vb + bb) {
    if (ctx->dl_pin) (void)hipHostFree(ctx->dl_pin);  // idle: every earlier call ended with a sync
    ctx->dl_pin = nullptr;
    ctx->dl_pin_cap = 0;
    if (hipHostMalloc((void**)&ctx->dl_pin, vb + bb, hipHostMallocDefault) == hipSuccess) ctx->dl_pin_cap = vb + bb;
    else (void)hipGetLastError();
  }
  bounce = bounce && ctx->dl_pin_cap >= vb + bb;
  uint8_t* vdst = bounce ? ctx->dl_pin : verdict_out;
  uint32_t* bdst = bounce ? reinterpret_cast<uint32_t*>(ctx->dl_pin + vb) : bitmap_out;
  {
    Timed t(ctx, "d2h_verdict", (verdict_out ? n : 0) + bb);
    if (verdict_out) CG_TRY(ctx, hipMemcpyAsync(vdst, verdict, n, hipMemcpyDeviceToHost, ctx->stream), "download verdict");
    if (bitmap_out) CG_TRY(ctx, hipMemcpyAsync(bdst, bitmap, bb, hipMemcpyDeviceToHost, ctx->stream), "download bitmap");
  }
  end_call_span(ctx);
  CG_TRY(ctx, hipStreamSynchronize(ctx->stream), "verify sync");
  if (bounce) {
    if (verdict_out) std::memcpy(verdict_out, vdst, n);
    if (bitmap_out) std::memcpy(bitmap_out, bdst, bb);
  }
  return CG_OK;
}

// A chunk's per-element arrays inside VerifyRun::rows (and inside its ring slot, after
// the arena piece, in the same layout): msg_off, msg_len, key rows, signature rows,
// signature lengths, each 256-byte aligned.
// CG_ROWS_FIRST (pageable pipeline calls): the row arrays (offsets, lengths, keys,
// signatures, signature lengths) live whole-call on the device, chunk 0's slices go up
// with chunk 0 and every later chunk's in one copy per array with chunk 1; chunks 2.. send
// only their arena piece.  Per chunk they were five or six more pageable copies each.
#ifndef CG_ROWS_FIRST
#define CG_ROWS_FIRST 1
#endif
struct ChunkRows {
  size_t off, len, pk, sig, sl, bytes;  // byte offsets from the chunk's base; total size
  ChunkRows(size_t cnt, size_t pk_stride, size_t sig_stride, bool has_sl) {
    auto a = [](size_t x) { return (x + 255) & ~(size_t)255; };
    off = 0;
    len = off + a(cnt * 8);
    pk = len + a(cnt * 4);
    sig = pk + a(cnt * pk_stride);
    sl = sig + a(cnt * sig_stride);
    bytes = sl + (has_sl ? a(cnt * 4) : 0);
  }
};

cg_status verify_pipeline(cg_ctx* ctx, size_t n, int mode, const uint8_t* scheme_id, const uint8_t* pk,
                          size_t pk_stride, const uint8_t* sig, size_t sig_stride, const uint32_t* sig_len,
                          const uint8_t* msg, size_t msg_bytes, const uint64_t* msg_off, const uint32_t* msg_len,
                          const std::vector<size_t>& cb, VerifyRun& r) {
  const size_t K = cb.size() - 1;
  cg_status st;
  std::vector<size_t> rows_at(K + 1, 0);  // chunk k's rows at r.rows + rows_at[k]
  for (size_t k = 0; k < K; ++k)
    rows_at[k + 1] = rows_at[k] + ChunkRows(cb[k + 1] - cb[k], pk_stride, sig_stride, sig_len).bytes;
  if ((st = dalloc(ctx, &r.arena, msg_bytes + 16, "alloc arena")) != CG_OK ||
      (st = dalloc(ctx, &r.rows, rows_at[K], "alloc rows")) != CG_OK ||
      (st = dalloc(ctx, &r.verdict, n, "alloc verdict")) != CG_OK ||
      (st = dalloc(ctx, &r.bitmap, (n + 31) / 32, "alloc bitmap")) != CG_OK)
    return st;
  r.ev.assign(K, nullptr);
  for (hipEvent_t& e : r.ev)
    if (!(e = take_sync_event(ctx))) return fail(ctx, CG_E_DEVICE, "verify pipeline event");
  // the arena's 16-byte tail pad (kernels' vector loads may run past a message end)
  CG_TRY(ctx, hipMemsetAsync(r.arena + msg_bytes, 0, 16, ctx->copy_stream), "pad arena");
  // Chunk k's upload: the arena bytes its messages reach beyond what earlier chunks
  // uploaded (a prefix: an element-ordered arena, what a caller packs, gives even
  // pieces; any layout is correct), then its metadata and rows; event ev[k].
  // End of the arena prefix each chunk's messages reach (clamped: a chunk's offsets are
  // checked against the arena before its copy goes out).
  std::vector<uint64_t> aend(K + 1, 0);
  // Pinned inputs: the copies are asynchronous.  Pageable inputs go up as the runtime's
  // own pageable copies (they hold the issuing thread: the upload thread below), or with
  // CORDA_AMD_VERIFY_RING=1 through the context's two page-locked ring slots, filled by
  // the copy workers (chunk k+1's slot while chunk k's DMA runs; a slot is reused once
  // chunk k-2's copies are done).  The ring was the default until r05: it is as fast
  // where the host's memcpy runs at ~90 GB/s, but it is bound by it, and on three of five
  // r05 boxes the staging ran at 35-50 GB/s (2^18 x 1 KB: 7.5-9.8 ms against 6.9-7.5 for
  // the runtime's copies on the same boxes; r05l/o/p sweeps).
  const bool pinned = host_is_pinned(msg) && host_is_pinned(pk) && host_is_pinned(sig) &&
                      host_is_pinned(msg_off) && host_is_pinned(msg_len) && host_is_pinned(sig_len);
  bool ring = false;
  if (ctx->opts.has(cg::OPT_VERIFY_RING)) ring = !pinned && K > 1 && ctx->opts.on(cg::OPT_VERIFY_RING, false);
  // the copy workers: the ring's host copies, and the arena-end scan below
  if (!ctx->pool && (ring || n >= 65536)) {
    int workers = 7;
    if (ctx->opts.has(cg::OPT_COPY_THREADS)) workers = std::max(0, ctx->opts.i(cg::OPT_COPY_THREADS, 8) - 1);
    ctx->pool = new CopyPool(workers);
  }
  // arena end of each chunk's messages (a prefix scan over every element: on the copy
  // workers when they exist — one thread needed ~0.2 ms of host time before the first
  // DMA at 2^18 elements)
  {
    std::vector<uint64_t> cmax(K, 0);
    auto scan = [&](size_t lo, size_t hi, uint64_t* out) {
      for (size_t k = 0; k < K; ++k) {
        uint64_t u = 0;
        const size_t a = std::max(lo, cb[k]), z = std::min(hi, cb[k + 1]);
        for (size_t i = a; i < z; ++i) u = std::max<uint64_t>(u, clamped_end(msg_off[i], msg_len[i], msg_bytes));
        out[k] = std::max(out[k], u);
      }
    };
    const size_t parts = ctx->pool && n >= 65536 ? ctx->pool->workers() + 1 : 1;
    std::vector<std::vector<uint64_t>> part(parts, std::vector<uint64_t>(K, 0));
    if (parts > 1) {
      std::vector<std::function<void()>> fns;
      for (size_t t = 0; t < parts; ++t)
        fns.push_back([&, t] { scan(n * t / parts, n * (t + 1) / parts, part[t].data()); });
      ctx->pool->run_fns(fns);
    } else {
      scan(0, n, part[0].data());
    }
    for (size_t t = 0; t < parts; ++t)
      for (size_t k = 0; k < K; ++k) cmax[k] = std::max(cmax[k], part[t][k]);
    for (size_t k = 0; k < K; ++k) aend[k + 1] = std::max(aend[k], cmax[k]);
  }
  const size_t row_bytes = 12 + pk_stride + sig_stride + (sig_len ? 4 : 0);
  size_t slot = 0;
  for (size_t k = 0; k < K; ++k)
    slot = std::max(slot, (size_t)((aend[k + 1] - aend[k] + 255) & ~(uint64_t)255) + (rows_at[k + 1] - rows_at[k]));
  if (ring) {
    // The slots stay page-locked until cg_close, so their size is capped
    // (CORDA_AMD_RING_MAX_MB, default 256 MB per slot): a call whose chunk would need
    // more — e.g. an arena packed in reverse element order, whose first chunk's prefix
    // is the whole arena — copies its pageable buffers synchronously instead.
    size_t cap_mb = 256;
    if (ctx->opts.has(cg::OPT_RING_MAX_MB)) cap_mb = (size_t)std::max(1, ctx->opts.i(cg::OPT_RING_MAX_MB, 256));
    if (slot > (cap_mb << 20)) ring = false;
  }
  if (ring) {
    if (ctx->ring_cap < slot) {
      for (uint8_t*& rb : ctx->ring) {
        if (rb) (void)hipHostFree(rb);  // idle: every earlier call ended with a sync
        rb = nullptr;
      }
      ctx->ring_cap = 0;
      if (hipHostMalloc((void**)&ctx->ring[0], slot, hipHostMallocDefault) == hipSuccess &&
          hipHostMalloc((void**)&ctx->ring[1], slot, hipHostMallocDefault) == hipSuccess) {
        ctx->ring_cap = slot;
      } else {
        (void)hipGetLastError();
        for (uint8_t*& rb : ctx->ring) {
          if (rb) (void)hipHostFree(rb);
          rb = nullptr;
        }
      }
    }
    ring = ctx->ring_cap >= slot;
  }
  const bool one_dma = ctx->opts.on(cg::OPT_VERIFY_ONE_DMA, true);
  // whole-call row arrays (CG_ROWS_FIRST; the ring stages each chunk's rows in its layout)
  const bool soa = CG_ROWS_FIRST && !ring && K > 1;
  const ChunkRows all_rows(n, pk_stride, sig_stride, sig_len);  // (fits: <= rows_at[K], one pad per array)
  struct RowPtrs {
    uint8_t *off, *len, *pk, *sig, *sl;
  };
  auto row_ptrs = [&](size_t k) -> RowPtrs {  // chunk k's rows on the device
    const size_t lo = cb[k];
    if (soa)
      return {r.rows + all_rows.off + lo * 8, r.rows + all_rows.len + lo * 4, r.rows + all_rows.pk + lo * pk_stride,
              r.rows + all_rows.sig + lo * sig_stride, r.rows + all_rows.sl + lo * 4};
    const ChunkRows cr(cb[k + 1] - lo, pk_stride, sig_stride, sig_len);
    uint8_t* const rb = r.rows + rows_at[k];
    return {rb + cr.off, rb + cr.len, rb + cr.pk, rb + cr.sig, rb + cr.sl};
  };
  // staging slice size (ring only); CORDA_AMD_VERIFY_SLICE_KB overrides (0: whole chunks)
  size_t slice_bytes = (size_t)12 << 20;
  if (ctx->opts.has(cg::OPT_VERIFY_SLICE_KB)) slice_bytes = (size_t)std::max(0, ctx->opts.i(cg::OPT_VERIFY_SLICE_KB, 0)) << 10;
  // the chunk's inputs are checked just before they go out (the host scan then
  // overlaps the earlier chunks' copies and kernels); an error ends the call
  auto check_chunk = [&](size_t k) -> cg_status {
    const size_t lo = cb[k], hi = cb[k + 1];
    MsgSrc mc;
    mc.host = msg;
    mc.bytes = msg_bytes;
    mc.off_host = msg_off + lo;
    mc.len_host = msg_len + lo;
    return check_inputs(ctx, hi - lo, scheme_id ? scheme_id + lo : nullptr, pk + lo * pk_stride, pk_stride,
                        sig + lo * sig_stride, sig_stride, sig_len ? sig_len + lo : nullptr, mc, true, lo);
  };
  // (device destination, host source, bytes) of chunk k: its arena piece and rows
  auto chunk_pieces = [&](size_t k) {
    size_t lo = cb[k], hi = cb[k + 1];
    std::vector<CopyPool::Piece> pieces = {{r.arena + aend[k], msg + aend[k], (size_t)(aend[k + 1] - aend[k])}};
    if (soa) {  // chunk 0: its own rows; chunk 1: every later chunk's; the rest: none
      if (k > 1) return pieces;
      if (k == 1) hi = n;
    }
    const RowPtrs rp = row_ptrs(k);
    pieces.push_back({rp.off, msg_off + lo, (hi - lo) * 8});
    pieces.push_back({rp.len, msg_len + lo, (hi - lo) * 4});
    pieces.push_back({rp.pk, pk + lo * pk_stride, (hi - lo) * pk_stride});
    pieces.push_back({rp.sig, sig + lo * sig_stride, (hi - lo) * sig_stride});
    if (sig_len) pieces.push_back({rp.sl, sig_len + lo, (hi - lo) * 4});
    return pieces;
  };
  // Issues chunk k's copies on the copy stream and records ev[k] (and the profiling span
  // events a / b when given): ring staging or direct copies.  Touches no context state
  // but the ring and the copy workers, so the upload thread can run it.
  auto issue_chunk = [&](size_t k, hipEvent_t a, hipEvent_t b) -> hipError_t {
    const size_t lo = cb[k], hi = cb[k + 1];
    const ChunkRows cr(hi - lo, pk_stride, sig_stride, sig_len);
    uint8_t* const rb = r.rows + rows_at[k];
    std::vector<CopyPool::Piece> pieces = chunk_pieces(k);
    hipStream_t cs = ctx->copy_stream;
    hipError_t e = hipSuccess;
    if (ring) {  // stage into slot k % 2 (free once chunk k-2's copies are done)
      uint8_t* slot = ctx->ring[k & 1];
      if (k >= 2 && (e = hipEventSynchronize(r.ev[k - 2])) != hipSuccess) return e;
      // the slot: the arena piece, then the rows in their device layout, so the rows
      // go up in one DMA (each extra DMA costs ~9 us of engine time, r04 ubench)
      const size_t abytes = (size_t)(aend[k + 1] - aend[k]), rows0 = (abytes + 255) & ~(size_t)255;
      std::vector<CopyPool::Piece> staged = {{slot, msg + aend[k], abytes}};
      for (size_t i = 1; i < pieces.size(); ++i)
        staged.push_back({slot + rows0 + (size_t)(static_cast<uint8_t*>(pieces[i].dst) - rb), pieces[i].src, pieces[i].bytes});
      if (one_dma && slice_bytes) {
        // staged in slices, each slice's DMA issued as soon as it is in the slot (the
        // first one small): the first DMA starts after ~2 MB of host copying instead of
        // the whole head chunk's, and the copy engine never waits for a whole chunk's
        // staging (r05j timeline, 2^18 x 1 KB: first DMA at 0.17-0.22 ms, then 0.13-0.28
        // ms idle after the head while the next chunk was staged)
        const size_t total = rows0 + cr.bytes;
        if (a) (void)hipEventRecord(a, cs);
        for (size_t x = 0, y; x < total && e == hipSuccess; x = y) {
          y = std::min(total, (x + (k == 0 && x == 0 ? std::min(slice_bytes, (size_t)2 << 20) : slice_bytes) + 4095) &
                                  ~(size_t)4095);
          std::vector<CopyPool::Piece> part;
          for (const CopyPool::Piece& q : staged) {
            const size_t qa = (size_t)(static_cast<uint8_t*>(q.dst) - slot), a2 = std::max(x, qa);
            const size_t z = std::min(y, qa + q.bytes);
            if (a2 < z) part.push_back({slot + a2, static_cast<const uint8_t*>(q.src) + (a2 - qa), z - a2});
          }
          ctx->pool->run(part);
          if (x < abytes)
            e = hipMemcpyAsync(r.arena + aend[k] + x, slot + x, std::min(y, abytes) - x, hipMemcpyHostToDevice, cs);
          if (e == hipSuccess && y > rows0) {
            const size_t a2 = std::max(x, rows0);
            e = hipMemcpyAsync(rb + (a2 - rows0), slot + a2, y - a2, hipMemcpyHostToDevice, cs);
          }
        }
        if (b && e == hipSuccess) (void)hipEventRecord(b, cs);
        pieces.clear();
      } else {
        ctx->pool->run(staged);
        if (one_dma) {
          pieces = {{r.arena + aend[k], slot, abytes}, {rb, slot + rows0, cr.bytes}};
        } else {  // (A/B: one DMA per array, as before)
          for (size_t i = 0; i < pieces.size(); ++i) pieces[i].src = staged[i].dst;
        }
      }
    }
    if (!pieces.empty()) {
      if (a) (void)hipEventRecord(a, cs);
      for (const CopyPool::Piece& p : pieces)
        if (e == hipSuccess && p.bytes) e = hipMemcpyAsync(p.dst, p.src, p.bytes, hipMemcpyHostToDevice, cs);
      if (b && e == hipSuccess) (void)hipEventRecord(b, cs);
    }
    if (e == hipSuccess) e = hipEventRecord(r.ev[k], cs);
    return e;
  };
  auto chunk_span = [&](size_t k, hipEvent_t a, hipEvent_t b) {  // (a profiling span of chunk k's copies)
    if (!a || !b) return;
    ctx->pending.push_back({"h2d_verify", {a, b}});
    ctx->stats["h2d_verify"].items += (aend[k + 1] - aend[k]) + (cb[k + 1] - cb[k]) * row_bytes;
  };
  auto enqueue_upload = [&](size_t k) -> cg_status {
    cg_status cst = check_chunk(k);
    if (cst != CG_OK) return cst;
    hipEvent_t a = ctx->profiling ? take_event(ctx) : nullptr, b = ctx->profiling ? take_event(ctx) : nullptr;
    const hipError_t e = issue_chunk(k, a, b);
    if (e == hipSuccess) chunk_span(k, a, b);
    else give_back_events(ctx, a, b);
    return e == hipSuccess ? CG_OK : hip_fail(ctx, e, "upload chunk");
  };
  // Asynchronous copies (pinned or staged) run one chunk ahead of the kernels, so the
  // copy engine never waits for the host; a copy that holds the host goes after the
  // previous chunk's kernels are enqueued, so they run beside it.

  size_t uploaded = 0;  // chunks whose copies are enqueued (and inputs checked)
  // The upload thread (pageable inputs): every chunk's copies — the ring staging and its
  // DMAs, or the runtime's own pageable copies, which hold the issuing thread for their
  // duration — are issued on a helper thread, chunk after chunk, so the calling thread
  // only checks inputs and enqueues kernels, each chunk's as soon as its copies are
  // issued.  On the calling thread the copy engine idled between chunks while it
  // enqueued the kernels (r05n, no ring: 0.05-0.15 ms per chunk), and with the ring the
  // last chunks' kernels went out late whenever the host copies ran slow (1.5 ms of
  // kernels after the last byte against 0.8 at best).  CORDA_AMD_VERIFY_UPLOAD_THREAD=0
  // keeps the uploads on the calling thread.  `issued` counts the chunks whose ev[k] is
  // recorded.
  bool thread_up = !pinned && K > 1;
  thread_up = thread_up && ctx->opts.on(cg::OPT_VERIFY_UPLOAD_THREAD, true);
  // (with the upload thread the calling thread waits only for the chunk it launches next)
  size_t ahead = thread_up ? 0 : (pinned || ring) ? 2 : 1;
  if (ctx->opts.has(cg::OPT_VERIFY_AHEAD) && !thread_up) ahead = (size_t)std::max(1, ctx->opts.i(cg::OPT_VERIFY_AHEAD, 1));
  struct Uploader {
    std::mutex m;
    std::condition_variable cv;
    size_t issued = 0;
    bool started = false, stop = false, finished = false;
    hipError_t err = hipSuccess;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> spans;  // (profiling) per chunk, pre-taken
    void finish() {  // stop the job (if still running) and wait for its end
      std::unique_lock<std::mutex> g(m);
      if (!started) return;
      stop = true;
      cv.wait(g, [&] { return finished; });
      started = false;
    }
  } up;
  struct UploaderJoin {  // on every exit: the job joined; span events not handed to chunk_span go back
    Uploader& u;
    cg_ctx* c;
    ~UploaderJoin() {
      u.finish();
      for (auto& sp : u.spans) give_back_events(c, sp.first, sp.second);
    }
  } up_join{up, ctx};
  auto upload_through = [&](size_t k) -> cg_status {  // enqueue copies of chunks < min(k, K)
    for (; uploaded < std::min(k, K); ++uploaded) {
      if (!thread_up) {
        cg_status s2 = enqueue_upload(uploaded);
        if (s2 != CG_OK) return s2;
        continue;
      }
      cg_status s2 = check_chunk(uploaded);
      if (s2 != CG_OK) return s2;
      std::unique_lock<std::mutex> g(up.m);
      up.cv.wait(g, [&] { return up.issued > uploaded || up.err != hipSuccess; });
      if (up.issued <= uploaded) return hip_fail(ctx, up.err, "upload chunk");
    }
    return CG_OK;
  };
  if (thread_up) {
    if (ctx->profiling) {
      up.spans.resize(K, {nullptr, nullptr});
      for (auto& sp : up.spans) sp = {take_event(ctx), take_event(ctx)};
    }
    try {
      if (!ctx->uploader) ctx->uploader = new JobThread(ctx->device);
      up.started = true;
      ctx->uploader->post([&] {
        hipError_t e = hipSuccess;
        for (size_t k = 0; k < K && e == hipSuccess; ++k) {
          {
            std::lock_guard<std::mutex> g(up.m);
            if (up.stop) break;
          }
          try {  // (nothing may unwind out of the thread: a host allocation failure ends the uploads)
            e = up.spans.empty() ? issue_chunk(k, nullptr, nullptr)
                                 : issue_chunk(k, up.spans[k].first, up.spans[k].second);
          } catch (...) {
            e = hipErrorOutOfMemory;
          }
          std::lock_guard<std::mutex> g(up.m);
          if (e == hipSuccess) ++up.issued;
          else up.err = e;
          up.cv.notify_all();
        }
        std::lock_guard<std::mutex> g(up.m);
        up.finished = true;
        up.cv.notify_all();
      });
    } catch (...) {  // (a thread that cannot be created: std::system_error)
      up.started = false;
      return fail(ctx, CG_E_DEVICE, "verify upload thread");
    }
  }
  if ((st = upload_through(ahead)) != CG_OK) return st;
  // Scratch sized for the largest chunk first, so no chunk regrows (frees) a buffer
  // an earlier chunk's kernels still use.
  uint32_t max_cnt[3] = {0, 0, 0};
  for (size_t k = 0; k < K; ++k) {
    uint32_t cnt[3] = {scheme_id ? 0u : (uint32_t)(cb[k + 1] - cb[k]), 0, 0};
    for (size_t i = cb[k]; scheme_id && i < cb[k + 1]; ++i) {
      const uint8_t sc = scheme_id ? scheme_id[i] : CG_SCHEME_EDDSA_ED25519_SHA512;
      if (sc == CG_SCHEME_EDDSA_ED25519_SHA512) ++cnt[0];
      else if (sc == CG_SCHEME_ECDSA_SECP256K1_SHA256) ++cnt[1];
      else if (sc == CG_SCHEME_ECDSA_SECP256R1_SHA256) ++cnt[2];
    }
    for (int c = 0; c < 3; ++c) max_cnt[c] = std::max(max_cnt[c], cnt[c]);
  }
  // Latency lanes for pipeline chunks (CORDA_AMD_VERIFY_LANES=0/1 forces): a chunk's
  // two / four / eight lanes per signature cost 1.4-1.7x the MSM instructions; they pay
  // only when the call is bound by its copies (the extra work hides under the next
  // chunk's upload and the last chunk's chain after the last byte is shorter).
  bool lanes = true;
  lanes = ctx->opts.on(cg::OPT_VERIFY_LANES, lanes);
  // two chunks in flight need two disjoint scratch halves; chunks too large for that
  // (> kEdChunk Ed25519 lanes each) run one after the other on ctx->stream
  const bool dual = K > 1 && max_cnt[0] <= kEdChunk && !ctx->opts.has(cg::OPT_VERIFY_SERIAL);
  if (max_cnt[0] &&
      (st = ensure_ed_scratch(ctx, dual ? 2 * max_cnt[0] : max_cnt[0], dual ? 2 * kEdChunk : kEdChunk)) != CG_OK)
    return st;
  for (int c = 0; c < 2; ++c) {
    uint32_t chunk = 0;
    if (max_cnt[1 + c] &&
        (st = ecdsa_scratch_retry(ctx, c == 0 ? CG_SCHEME_ECDSA_SECP256K1_SHA256 : CG_SCHEME_ECDSA_SECP256R1_SHA256,
                                  max_cnt[1 + c], &chunk)) != CG_OK)
      return st;
  }
  // the staging's host index vectors go out through page-locked memory, so no chunk
  // waits on the host for its own copies
  const size_t pin_need = 4 * n + 4 * 256 * K;
  if (ctx->pin_cap < pin_need) {
    if (ctx->pin) (void)hipHostFree(ctx->pin);  // idle: every earlier call ended with a sync
    ctx->pin = nullptr;
    ctx->pin_cap = 0;
    if (hipHostMalloc((void**)&ctx->pin, pin_need, hipHostMallocDefault) == hipSuccess) ctx->pin_cap = pin_need;
    else (void)hipGetLastError();  // no staging: the chunks sync instead
  }
  ctx->pin_used = 0;
  ctx->pin_active = true;
  struct PinOff {
    cg_ctx* c;
    ~PinOff() { c->pin_active = false; }
  } pin_off{ctx};
  // chunk k runs on lane[k % 2]; ctx->stream is swapped for the chunk's staging and
  // launches (every helper enqueues on ctx->stream) and restored on every exit
  hipStream_t lane[2] = {ctx->stream, dual ? ctx->hash_stream : ctx->stream};
  // Ed25519 points kernels beside the hash kernels on the first ECDSA stream when no
  // chunk has ECDSA elements (it is idle then)
  hipStream_t pts = (!max_cnt[1] && !max_cnt[2] && ed_overlap_enabled(ctx)) ? ctx->ec_stream[0] : nullptr;
  struct StreamRestore {
    cg_ctx* c;
    hipStream_t main;
    ~StreamRestore() { c->stream = main; }
  } restore{ctx, ctx->stream};
  hipEvent_t done[2] = {nullptr, nullptr};  // the latest chunk's end on each lane
  for (hipEvent_t& e : done) {
    if (!(e = take_sync_event(ctx))) return fail(ctx, CG_E_DEVICE, "verify pipeline event");
    r.ev.push_back(e);  // returned to the pool by VerifyRun::release, after the syncs
  }
  for (size_t k = 0; k < K; ++k) {
    const size_t lo = cb[k], hi = cb[k + 1];
    if ((st = upload_through(k + 1)) != CG_OK) return st;  // (chunk k's own copy, if not yet)
    if (hi == lo) continue;
    const int L = dual ? (int)(k & 1) : 0;
    ctx->stream = lane[L];
    MsgSrc m;
    m.dev = r.arena;
    m.bytes = msg_bytes;
    const RowPtrs rp = row_ptrs(k);
    m.off_dev = reinterpret_cast<uint64_t*>(rp.off);
    m.len_dev = reinterpret_cast<uint32_t*>(rp.len);
    m.pk_dev = rp.pk;
    m.sig_dev = rp.sig;
    m.sl_dev = sig_len ? reinterpret_cast<const uint32_t*>(rp.sl) : nullptr;
    m.raw_ready = r.ev[k];
    m.verdict_dev = r.verdict + lo;
    m.async = true;
    m.index_base = lo;
    cg_batch* b = nullptr;
    st = create_batch(ctx, hi - lo, scheme_id ? scheme_id + lo : nullptr, pk + lo * pk_stride, pk_stride,
                      sig + lo * sig_stride, sig_stride, sig_len ? sig_len + lo : nullptr, m, &b);
    if (b) r.batches.push_back(b);  // freed after the final sync
    if (st != CG_OK) return st;
    // the key-reuse path's per-key tables are one context-wide buffer: a chunk that
    // builds them waits for the other lane's chunk, which may still read them
    if (dual && b->ed_key_index)
      CG_TRY(ctx, hipStreamWaitEvent(ctx->stream, done[L ^ 1], 0), "verify pipeline wait");
    st = launch_verify(ctx, b, mode, /*join_streams=*/false, dual ? (uint32_t)(L * max_cnt[0]) : 0, pts,
                       dual ? max_cnt[0] : 0, lanes);
    if (st != CG_OK) return st;
    CG_TRY(ctx, hipEventRecord(done[L], ctx->stream), "verify pipeline record");
    if ((st = upload_through(k + 1 + ahead)) != CG_OK) return st;
  }
  ctx->stream = restore.main;
  if (dual) CG_TRY(ctx, hipStreamWaitEvent(ctx->stream, done[1], 0), "verify pipeline join");
  if ((st = join_ecdsa_streams(ctx)) != CG_OK) return st;
  CG_TRY(ctx, cg::launch_verdict_bitmap(r.verdict, (uint32_t)n, r.bitmap, ctx->stream), "launch bitmap");
  if (up.started) {  // (every chunk is issued by now)
    up.finish();
    for (size_t k = 0; k < up.spans.size(); ++k) chunk_span(k, up.spans[k].first, up.spans[k].second);
    up.spans.clear();
  }
  return CG_OK;
}

}  // namespace

extern "C" {

cg_status cg_batch_create(cg_ctx* ctx, size_t n, const uint8_t* scheme_id, const uint8_t* pk, size_t pk_stride,
                          const uint8_t* sig, size_t sig_stride, const uint32_t* sig_len, const uint8_t* msg,
                          size_t msg_bytes, const uint64_t* msg_off, const uint32_t* msg_len, cg_batch** out) {
  CG_API_BEGIN
  scheme_id = ed25519_only(scheme_id, n);
  MsgSrc m;
  m.host = msg;
  m.bytes = msg_bytes;
  m.off_host = msg_off;
  m.len_host = msg_len;
  return create_batch(ctx, n, scheme_id, pk, pk_stride, sig, sig_stride, sig_len, m, out);
  CG_API_END(ctx)
}

cg_status cg_batch_verify(cg_ctx* ctx, cg_batch* b, int mode, uint8_t* verdict_out, uint32_t* accept_bitmap_out,
                          void* device_bitmap_out) {
  CG_API_BEGIN
  if (!ctx || !b) return fail(ctx, CG_E_INVALID_ARGUMENT, "null context or batch");
  if (mode != CG_MODE_IS_VALID && mode != CG_MODE_DO_VERIFY) return fail(ctx, CG_E_INVALID_ARGUMENT, "bad mode");
  if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, CG_E_DEVICE, "hipSetDevice");
  const size_t n = b->n;
  if (n == 0) return CG_OK;
  cg_status st = launch_verify(ctx, b, mode);
  if (st != CG_OK) return st;
  const size_t nwords = (n + 31) / 32;
  if (device_bitmap_out)
    CG_TRY(ctx, hipMemcpyAsync(device_bitmap_out, b->bitmap, nwords * 4, hipMemcpyDeviceToDevice, ctx->stream),
           "copy device bitmap");
  st = download_verdicts(ctx, verdict_out, b->verdict, n, accept_bitmap_out, b->bitmap, nwords);
  if (st != CG_OK) return st;
  collect_timings(ctx);
  return CG_OK;
  CG_API_END(ctx)
}

size_t cg_batch_size(const cg_batch* b) { return b ? b->n : 0; }

void cg_batch_destroy(cg_ctx* ctx, cg_batch* b) {
  try {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    if (b && b->points_early) (void)hipStreamSynchronize(ctx->copy_stream);  // (a verify that never joined them)
    batch_free(ctx, b);
  } catch (...) {
    api_guard_fail(ctx);
  }
}

cg_status cg_verify_batch(cg_ctx* ctx, size_t n, int mode, const uint8_t* scheme_id, const uint8_t* pk,
                          size_t pk_stride, const uint8_t* sig, size_t sig_stride, const uint32_t* sig_len,
                          const uint8_t* msg, size_t msg_bytes, const uint64_t* msg_off, const uint32_t* msg_len,
                          uint8_t* verdict_out, uint32_t* accept_bitmap_out) {
  CG_API_BEGIN
  if (!ctx) return CG_E_INVALID_ARGUMENT;
  if (n && !verdict_out) return fail(ctx, CG_E_INVALID_ARGUMENT, "null verdict_out");
  if (n == 0) return CG_OK;
  if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, CG_E_DEVICE, "hipSetDevice");
  begin_call_span(ctx);
  scheme_id = ed25519_only(scheme_id, n);
  struct CallSpanEnd {  // an early error return drops the span
    cg_ctx* c;
    ~CallSpanEnd() {
      if (c->call_begin) c->event_pool.push_back(c->call_begin);
      c->call_begin = nullptr;
    }
  } call_span_end{ctx};
  // the call's plan (cg_plan.h): copy-bound or compute-bound by bytes per element, chunk
  // bounds; a one-chunk call's own choices are made in create_batch once the partition
  // has found the scheme mix
  cg::VerifyShape shape;
  shape.n = n;
  shape.msg_bytes = msg_bytes;
  shape.pk_stride = pk_stride;
  shape.sig_stride = sig_stride;
  shape.sig_len = sig_len != nullptr;
  const cg::VerifyPlan plan = cg::plan_verify(shape, ctx->opts);
  const std::vector<size_t>& cb = plan.chunks;
  if (cb.size() == 2) {  // one chunk: stage, then verify, with one host sync at the end
    MsgSrc m;
    m.host = msg;
    m.bytes = msg_bytes;
    m.off_host = msg_off;
    m.len_host = msg_len;
    m.keep_raw = true;
    m.pair_max = plan.pair_max;
    cg_batch* b = nullptr;
    cg_status st = create_batch(ctx, n, scheme_id, pk, pk_stride, sig, sig_stride, sig_len, m, &b);
    if (st != CG_OK) return st;
    st = cg_batch_verify(ctx, b, mode, verdict_out, accept_bitmap_out, nullptr);
    cg_batch_destroy(ctx, b);
    return st;
  }
  if (mode != CG_MODE_IS_VALID && mode != CG_MODE_DO_VERIFY) return fail(ctx, CG_E_INVALID_ARGUMENT, "bad mode");
  if (n > 0xFFFFFFF0ull) return fail(ctx, CG_E_INVALID_ARGUMENT, "batch larger than 2^32 - 16 elements");
  if (!pk || !sig || !msg_off || !msg_len || (msg_bytes > 0 && !msg))
    return fail(ctx, CG_E_INVALID_ARGUMENT, "null input pointer");
  cg_status st = CG_OK;
  if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, CG_E_DEVICE, "hipSetDevice");
  VerifyRun r;
  struct RunGuard {  // also on an exception caught by CG_API_END (release is idempotent)
    VerifyRun& r;
    cg_ctx* c;
    ~RunGuard() { r.release(c); }
  } guard{r, ctx};
  st = verify_pipeline(ctx, n, mode, scheme_id, pk, pk_stride, sig, sig_stride, sig_len, msg, msg_bytes, msg_off,
                       msg_len, cb, r);
  if (st == CG_OK) st = download_verdicts(ctx, verdict_out, r.verdict, n, accept_bitmap_out, r.bitmap, (n + 31) / 32);
  r.release(ctx);
  collect_timings(ctx);
  return st;
  CG_API_END(ctx)
}

cg_status cg_der_parse_batch(cg_ctx* ctx, size_t n, const uint8_t* scheme_id, const uint8_t* sig,
                             size_t sig_stride, const uint32_t* sig_len, uint8_t* rs_out, uint8_t* status_out) {
  CG_API_BEGIN
  if (!ctx) return CG_E_INVALID_ARGUMENT;
  if (n == 0) return CG_OK;
  if (!sig || !rs_out || !status_out) return fail(ctx, CG_E_INVALID_ARGUMENT, "null pointer");
  if (n > 0xFFFFFFF0ull) return fail(ctx, CG_E_INVALID_ARGUMENT, "batch too large");
  for (size_t i = 0; sig_len && i < n; ++i)
    if (sig_len[i] > sig_stride) return fail(ctx, CG_E_INVALID_ARGUMENT, "signature longer than sig_stride");
  if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, CG_E_DEVICE, "hipSetDevice");
  std::vector<uint32_t> idx[2];
  for (size_t i = 0; i < n; ++i)
    idx[(scheme_id && (scheme_id[i] & 0x7F) == CG_SCHEME_ECDSA_SECP256K1_SHA256) ? 0 : 1].push_back((uint32_t)i);
  uint8_t* sig_d = nullptr;
  uint32_t *sl_d = nullptr, *rs_d = nullptr, *st_d = nullptr, *ix_d = nullptr;
  cg_status st = CG_OK;
  auto cleanup = [&]() {
    (void)hipStreamSynchronize(ctx->stream);
    dfree(ctx, sig_d); dfree(ctx, sl_d); dfree(ctx, rs_d); dfree(ctx, st_d); dfree(ctx, ix_d);
  };
  if ((st = upload(ctx, &sig_d, sig, n * sig_stride, "upload sig")) != CG_OK ||
      (sig_len && (st = upload(ctx, &sl_d, sig_len, n, "upload sig_len")) != CG_OK) ||
      (st = dalloc(ctx, &rs_d, 16 * n, "alloc rs")) != CG_OK || (st = dalloc(ctx, &st_d, n, "alloc status")) != CG_OK ||
      (st = dalloc(ctx, &ix_d, n, "alloc index")) != CG_OK) {
    cleanup();
    return st;
  }
  // results are written in subset order; scatter back on the host
  std::vector<uint32_t> rs_h(16 * n), st_h(n);
  size_t done = 0;
  for (int c = 0; c < 2; ++c) {
    const uint32_t m = (uint32_t)idx[c].size();
    if (!m) continue;
    hipError_t e = hipMemcpyAsync(ix_d + done, idx[c].data(), (size_t)m * 4, hipMemcpyHostToDevice, ctx->stream);
    {
      Timed t(ctx, "der_parse", m);
      if (e == hipSuccess)
        e = cg::launch_der_parse(c == 0 ? 2 : 3, sig_d, sig_stride, sl_d, (uint32_t)sig_stride, ix_d + done, m, m,
                                 rs_d + 16 * done, st_d + done, ctx->stream);
    }
    if (e == hipSuccess)
      e = hipMemcpyAsync(rs_h.data() + 16 * done, rs_d + 16 * done, (size_t)16 * m * 4, hipMemcpyDeviceToHost,
                         ctx->stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(st_h.data() + done, st_d + done, (size_t)m * 4, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) {
      cleanup();
      return hip_fail(ctx, e, "der parse");
    }
    for (uint32_t j = 0; j < m; ++j) {
      const size_t dst = idx[c][j];
      status_out[dst] = (uint8_t)st_h[done + j];
      for (int half = 0; half < 2; ++half)
        for (int w = 0; w < 8; ++w) {
          const uint32_t limb = rs_h[16 * done + (size_t)(8 * half + w) * m + j];
          uint8_t* o = rs_out + dst * 64 + 32 * half + 4 * (7 - w);  // big-endian bytes
          o[0] = (uint8_t)(limb >> 24); o[1] = (uint8_t)(limb >> 16); o[2] = (uint8_t)(limb >> 8); o[3] = (uint8_t)limb;
        }
    }
    done += m;
  }
  cleanup();
  collect_timings(ctx);
  return CG_OK;
  CG_API_END(ctx)
}

cg_status cg_set_profiling(cg_ctx* ctx, int enable) {
  CG_API_BEGIN
  if (!ctx) return CG_E_INVALID_ARGUMENT;
  collect_timings(ctx);
  ctx->profiling = enable == 1;
  ctx->call_spans_only = enable == 2;
  return CG_OK;
  CG_API_END(ctx)
}

cg_status cg_kernel_stats(cg_ctx* ctx, const char* kernel, double* total_ms, uint64_t* launches, uint64_t* items) {
  CG_API_BEGIN
  if (!ctx || !kernel) return CG_E_INVALID_ARGUMENT;
  collect_timings(ctx);
  auto it = ctx->stats.find(kernel);
  const Stat s = it == ctx->stats.end() ? Stat() : it->second;
  if (total_ms) *total_ms = s.ms;
  if (launches) *launches = s.launches;
  if (items) *items = s.items;
  return CG_OK;
  CG_API_END(ctx)
}

cg_status cg_reset_stats(cg_ctx* ctx) {
  CG_API_BEGIN
  if (!ctx) return CG_E_INVALID_ARGUMENT;
  collect_timings(ctx);
  ctx->stats.clear();
  return CG_OK;
  CG_API_END(ctx)
}

cg_status cg_set_debug(cg_ctx* ctx, int option, int64_t value) {
  CG_API_BEGIN
  if (!ctx) return CG_E_INVALID_ARGUMENT;
  switch (option) {
    case CG_DEBUG_FORCE_FULL_LENGTH:
      if (value < 0 || value > 0xffffffffll) return fail(ctx, CG_E_INVALID_ARGUMENT, "bad modulus");
      ctx->debug_full_mod = (uint32_t)value;
      return CG_OK;
    case CG_DEBUG_FAIL_ALLOC:
      ctx->debug_fail_alloc = value;
      return CG_OK;
    case CG_DEBUG_THROW:
      ctx->debug_throw = value != 0;
      return CG_OK;
    case CG_DEBUG_FORCE_GLV_FALLBACK:
      if (value < 0 || value > 0xffffffffll) return fail(ctx, CG_E_INVALID_ARGUMENT, "bad modulus");
      cg::ecdsa_set_debug_glv(ctx->ec, (uint32_t)value);
      return CG_OK;
    default:
      return fail(ctx, CG_E_INVALID_ARGUMENT, "unknown debug option");
  }
  CG_API_END(ctx)
}

cg_status cg_set_option(cg_ctx* ctx, const char* key, const char* value) {
  CG_API_BEGIN
  if (!ctx) return CG_E_INVALID_ARGUMENT;
  const int o = cg::Options::find(key);
  if (o < 0) return fail(ctx, CG_E_INVALID_ARGUMENT, std::string("unknown option ") + (key ? key : "(null)"));
  ctx->opts.assign(o, value);
  return CG_OK;
  CG_API_END(ctx)
}

}  // extern "C"

namespace {

// Device buffers of one tx-id computation (K5 + K6) and of the signature
// metadata derived from it.
struct TxDev {
  uint8_t* arena = nullptr;
  uint64_t* comp_off = nullptr;
  uint32_t *comp_len = nullptr, *comp_start = nullptr, *comp_tx = nullptr, *salts = nullptr, *leaves = nullptr;
  uint8_t* ids = nullptr;  // 32 B per tx (+16 pad): digest byte order
  uint32_t* sig_start = nullptr;
  uint64_t* sig_moff = nullptr;
  uint32_t* sig_mlen = nullptr;
  uint32_t *order = nullptr, *leaf_hist = nullptr;  // leaf kernel work order (length buckets)
  uint8_t *raw_pk = nullptr, *raw_sig = nullptr;     // tx pipeline: signature rows, element-major
  uint32_t* raw_sl = nullptr;
  void release(cg_ctx* ctx) {
    for (const void* p : {(const void*)arena, (const void*)comp_off, (const void*)comp_len, (const void*)comp_start,
                          (const void*)comp_tx, (const void*)salts, (const void*)leaves, (const void*)ids,
                          (const void*)sig_start, (const void*)sig_moff, (const void*)sig_mlen, (const void*)order,
                          (const void*)leaf_hist, (const void*)raw_pk, (const void*)raw_sig, (const void*)raw_sl})
      dfree(ctx, p);
    *this = TxDev();
  }
};

// Host-side validation is O(n_tx): monotone comp_start / sig_start.  Component
// bounds are checked by the leaf kernel (error flag, read back by the caller).
// Leaf hashes of the components of txs [t0, t1) and their Merkle roots (the arena
// bytes of those components must be on the device, in stream order).
cg_status hash_txs(cg_ctx* ctx, TxDev& d, size_t arena_bytes, const uint32_t* comp_start, size_t t0, size_t t1,
                   hipStream_t s = nullptr) {
  if (!s) s = ctx->stream;
  const uint32_t c0 = comp_start[t0], c1 = comp_start[t1];
  {
    Timed t(ctx, "merkle_leaf", c1 - c0, s);
    CG_TRY(ctx, cg::launch_merkle_leaf(d.arena, arena_bytes, d.comp_off, d.comp_len, d.comp_start, d.comp_tx, d.salts,
                                       nullptr, c0, c1, d.leaves, ctx->err_flag, s, d.order + c0,
                                       d.leaf_hist),
           "launch merkle_leaf");
  }
  {
    Timed t(ctx, "merkle_tree", t1 - t0, s);
    CG_TRY(ctx, cg::launch_merkle_tree(d.leaves, d.comp_start + t0, (uint32_t)(t1 - t0), (uint32_t*)d.ids + 8 * t0,
                                       s),
           "launch merkle_tree");
  }
  return CG_OK;
}

// upload_arena = false: everything but the arena upload and the hashing (the
// pipelined cg_tx_verify_batch streams the arena in chunks and hashes per chunk).
cg_status compute_txids(cg_ctx* ctx, size_t n_tx, const uint8_t* arena, size_t arena_bytes, const uint64_t* comp_off,
                        const uint32_t* comp_len, const uint32_t* comp_start, const uint8_t* salts,
                        const uint32_t* sig_start, TxDev& d, bool* any_empty, bool upload_arena = true) {
  if (n_tx > 0xFFFFFFF0ull) return fail(ctx, CG_E_INVALID_ARGUMENT, "too many transactions");
  if (!comp_start || !salts || (comp_start[n_tx] && (!comp_off || !comp_len || !arena)))
    return fail(ctx, CG_E_INVALID_ARGUMENT, "null pointer");
  *any_empty = false;
  for (size_t t = 0; t < n_tx; ++t) {
    if (comp_start[t + 1] < comp_start[t]) return fail(ctx, CG_E_INVALID_ARGUMENT, "comp_start not monotone");
    if (comp_start[t + 1] == comp_start[t]) *any_empty = true;
    if (sig_start && sig_start[t + 1] < sig_start[t]) return fail(ctx, CG_E_INVALID_ARGUMENT, "sig_start not monotone");
  }
  const uint32_t c_end = comp_start[n_tx];
  const size_t n_comp = c_end;
  const size_t n_sig = sig_start ? sig_start[n_tx] : 0;
  cg_status st;
  if ((st = dalloc(ctx, &d.arena, arena_bytes + 16, "alloc tx arena")) != CG_OK ||
      (st = upload(ctx, &d.comp_off, comp_off, n_comp, "upload comp_off")) != CG_OK ||
      (st = upload(ctx, &d.comp_len, comp_len, n_comp, "upload comp_len")) != CG_OK ||
      (st = upload(ctx, &d.comp_start, comp_start, n_tx + 1, "upload comp_start")) != CG_OK ||
      (st = upload(ctx, &d.salts, (const uint32_t*)salts, 8 * n_tx, "upload salts")) != CG_OK ||
      (st = dalloc(ctx, &d.comp_tx, n_comp, "alloc comp_tx")) != CG_OK ||
      (st = dalloc(ctx, &d.leaves, 8 * n_comp, "alloc leaves")) != CG_OK ||
      (st = dalloc(ctx, &d.order, n_comp + 1, "alloc leaf order")) != CG_OK ||
      (st = dalloc(ctx, &d.leaf_hist, 32, "alloc leaf bins")) != CG_OK ||
      (st = dalloc(ctx, &d.ids, 32 * n_tx + 16, "alloc ids")) != CG_OK)
    return st;
  if (sig_start && ((st = upload(ctx, &d.sig_start, sig_start, n_tx + 1, "upload sig_start")) != CG_OK ||
                    (st = dalloc(ctx, &d.sig_moff, n_sig, "alloc sig msg_off")) != CG_OK ||
                    (st = dalloc(ctx, &d.sig_mlen, n_sig, "alloc sig msg_len")) != CG_OK))
    return st;
  if (upload_arena && arena_bytes)
    CG_TRY(ctx, hipMemcpyAsync(d.arena, arena, arena_bytes, hipMemcpyHostToDevice, ctx->stream), "upload tx arena");
  CG_TRY(ctx, hipMemsetAsync(d.arena + arena_bytes, 0, 16, ctx->stream), "pad tx arena");
  CG_TRY(ctx, hipMemsetAsync(d.ids, 0, 32 * n_tx + 16, ctx->stream), "zero ids");
  CG_TRY(ctx, hipMemsetAsync(ctx->err_flag, 0, 4, ctx->stream), "zero error flag");
  CG_TRY(ctx, cg::launch_tx_index(d.comp_start, d.sig_start, (uint32_t)n_tx, d.comp_tx, d.sig_moff, d.sig_mlen,
                                  ctx->stream), "launch tx_index");
  if (upload_arena) return hash_txs(ctx, d, arena_bytes, comp_start, 0, n_tx);
  return CG_OK;
}

// The transaction pipeline of cg_tx_verify_batch: the component arena is streamed
// to the device in byte pieces on copy_stream, and tx-range chunk k is hashed
// (leaves, roots) and its signatures verified against the fresh ids on ctx->stream
// as soon as the arena prefix it reads is in, so the PCIe upload of the (large)
// arena overlaps the kernels and the host-side staging.  Any layout works; a
// component-ordered arena (what the JVM producer writes) makes the prefixes grow
// evenly.  Verdicts land in verdict_d at their absolute signature positions.
cg_status hip_ok(cg_ctx* ctx, hipError_t e, const char* what);

cg_status tx_pipeline(cg_ctx* ctx, int mode, size_t n_tx, const uint8_t* arena, size_t arena_bytes,
                      const uint64_t* comp_off, const uint32_t* comp_len, const uint32_t* comp_start,
                      const uint32_t* sig_start, const uint8_t* scheme_id, const uint8_t* pk, size_t pk_stride,
                      const uint8_t* sig, size_t sig_stride, const uint32_t* sig_len, TxDev& d, uint8_t* verdict_d,
                      std::vector<hipEvent_t>& ev, std::vector<cg_batch*>& batches) {
  // chunks: enough that the upload of the last one (after which only its kernels
  // remain) is short, few enough that each chunk's signature subsets still fill the
  // device (CORDA_AMD_TX_CHUNKS / CORDA_AMD_TX_MIN_CHUNK override, for tuning and tests)
  size_t kmax = 6, min_chunk = 65536;
  const cg::Options& o = ctx->opts;
  if (o.has(cg::OPT_TX_CHUNKS)) kmax = std::max(1, o.i(cg::OPT_TX_CHUNKS, 6));
  if (o.has(cg::OPT_TX_MIN_CHUNK)) min_chunk = std::max(1, o.i(cg::OPT_TX_MIN_CHUNK, 65536));
  const size_t K = std::max<size_t>(1, std::min<size_t>(kmax, n_tx / min_chunk));
  // The last chunk's kernels run after the last upload, unhidden: it gets `tail` of
  // a regular chunk's transactions (CORDA_AMD_TX_TAIL, default 1 = even split).
  double tail = 1.0;
  if (o.has(cg::OPT_TX_TAIL)) tail = std::min(1.0, std::max(0.1, o.d(cg::OPT_TX_TAIL, 1.0)));
  std::vector<size_t> tb(K + 1);
  const double wsum = (double)(K - 1) + tail;
  for (size_t k = 0; k <= K; ++k)
    tb[k] = k == K ? n_tx : (size_t)((double)n_tx * (double)k / wsum);
  // The row buffers come from the block cache: every block in it is idle here (the
  // API calls that freed them ended with a stream sync; compute_txids only enqueued
  // work on live blocks).
  const size_t n_sig = sig_start[n_tx];
  cg_status st;
  if (n_sig && ((st = dalloc(ctx, &d.raw_pk, n_sig * pk_stride, "alloc pk rows")) != CG_OK ||
                (st = dalloc(ctx, &d.raw_sig, n_sig * sig_stride, "alloc sig rows")) != CG_OK ||
                (sig_len && (st = dalloc(ctx, &d.raw_sl, n_sig, "alloc sig_len rows")) != CG_OK)))
    return st;
  ev.assign(2 * K + 1, nullptr);  // ev[k]: chunk k uploaded; ev[K + k]: its ids; ev[2K]: metadata staged
  for (hipEvent_t& e : ev) CG_TRY(ctx, hipEventCreateWithFlags(&e, hipEventDisableTiming), "tx pipeline event");
  // Chunk k's upload on copy_stream = the arena bytes its components reach beyond
  // what earlier chunks uploaded (a prefix; a component-ordered arena — what the JVM
  // producer writes — makes the pieces even), then its signature rows; event ev[k].
  // Uploads are enqueued chunk by chunk as the host scans the components, so the
  // copy engine starts at once and chunk k's kernels wait for exactly its own bytes.
  uint64_t up_to = 0;
  auto enqueue_upload = [&](size_t k) -> cg_status {
    const uint64_t from = up_to;
    for (uint32_t c = comp_start[tb[k]]; c < comp_start[tb[k + 1]]; ++c)
      up_to = std::max<uint64_t>(up_to, clamped_end(comp_off[c], comp_len[c], arena_bytes));
    if (up_to > from) {
      Timed t(ctx, "h2d_arena", up_to - from, ctx->copy_stream);
      CG_TRY(ctx, hipMemcpyAsync(d.arena + from, arena + from, up_to - from, hipMemcpyHostToDevice, ctx->copy_stream),
             "upload tx arena");
    }
    const size_t s0 = sig_start[tb[k]], s1 = sig_start[tb[k + 1]];
    if (s1 > s0) {
      Timed t(ctx, "h2d_rows", (s1 - s0) * (pk_stride + sig_stride), ctx->copy_stream);
      CG_TRY(ctx, hipMemcpyAsync(d.raw_pk + s0 * pk_stride, pk + s0 * pk_stride, (s1 - s0) * pk_stride,
                                 hipMemcpyHostToDevice, ctx->copy_stream), "upload pk rows");
      CG_TRY(ctx, hipMemcpyAsync(d.raw_sig + s0 * sig_stride, sig + s0 * sig_stride, (s1 - s0) * sig_stride,
                                 hipMemcpyHostToDevice, ctx->copy_stream), "upload sig rows");
      if (sig_len)
        CG_TRY(ctx, hipMemcpyAsync(d.raw_sl + s0, sig_len + s0, (s1 - s0) * 4, hipMemcpyHostToDevice, ctx->copy_stream),
               "upload sig_len rows");
    }
    CG_TRY(ctx, hipEventRecord(ev[k], ctx->copy_stream), "tx pipeline record");
    return CG_OK;
  };
  // Two chunks' uploads in flight before the first kernels are enqueued; chunk k + 2's
  // upload is enqueued with chunk k's kernels, so the copy engine never waits for the
  // host.
  if ((st = enqueue_upload(0)) != CG_OK) return st;
  if (K > 1 && (st = enqueue_upload(1)) != CG_OK) return st;
  // No host sync until the end: each chunk's staging goes out without one (index
  // vectors through pinned staging), its verdicts land in place, the ECDSA streams
  // run on across chunks and are joined once, and the batches live until the
  // caller's final sync.  The scratch buffers are sized for the largest chunk first,
  // so no chunk regrows (and frees) one that earlier chunks' kernels still use.
  uint32_t max_cnt[3] = {0, 0, 0};
  for (size_t k = 0; k < K; ++k) {
    uint32_t cnt[3] = {0, 0, 0};
    for (size_t i = sig_start[tb[k]]; i < sig_start[tb[k + 1]]; ++i) {
      const uint8_t sc = scheme_id ? scheme_id[i] : CG_SCHEME_EDDSA_ED25519_SHA512;
      cnt[sc == CG_SCHEME_EDDSA_ED25519_SHA512 ? 0 : sc == CG_SCHEME_ECDSA_SECP256K1_SHA256 ? 1 : 2] +=
          sc == CG_SCHEME_EDDSA_ED25519_SHA512 || sc == CG_SCHEME_ECDSA_SECP256K1_SHA256 ||
          sc == CG_SCHEME_ECDSA_SECP256R1_SHA256;
    }
    for (int c = 0; c < 3; ++c) max_cnt[c] = std::max(max_cnt[c], cnt[c]);
  }
  if (max_cnt[0] && (st = ensure_ed_scratch(ctx, max_cnt[0])) != CG_OK) return st;
  for (int c = 0; c < 2; ++c) {
    uint32_t chunk = 0;
    if (max_cnt[1 + c] &&
        (st = ecdsa_scratch_retry(ctx, c == 0 ? CG_SCHEME_ECDSA_SECP256K1_SHA256 : CG_SCHEME_ECDSA_SECP256R1_SHA256,
                                  max_cnt[1 + c], &chunk)) != CG_OK)
      return st;
  }
  const size_t pin_need = 4 * n_sig + 3 * 256 * K;
  if (ctx->pin_cap < pin_need) {
    if (ctx->pin) (void)hipHostFree(ctx->pin);  // idle: every earlier call ended with a sync
    ctx->pin = nullptr;
    ctx->pin_cap = 0;
    if (hipHostMalloc((void**)&ctx->pin, pin_need, hipHostMallocDefault) == hipSuccess) ctx->pin_cap = pin_need;
    else (void)hipGetLastError();  // no staging: the chunks sync instead
  }
  ctx->pin_used = 0;
  ctx->pin_active = true;
  struct PinOff {
    cg_ctx* c;
    ~PinOff() { c->pin_active = false; }
  } pin_off{ctx};
  // With four hardware queues both curves would share ec_stream[0], and the ECDSA
  // stream (~37 ms of kernels per 1 M transactions) became the step's critical path
  // once the Ed25519 kernels got faster (timeline r02x).  The second curve then runs
  // on hash_stream: chunk k's R1 work queues behind chunk k's Merkle ids and ahead of
  // chunk k+1's, which only start after chunk k+1's upload (~6 ms later) anyway.
  struct CurveStream {
    cg_ctx* c;
    hipStream_t saved;
    ~CurveStream() { c->ec_stream[1] = saved; }
  } curve_stream{ctx, ctx->ec_stream[1]};
  if (ctx->ec_stream[1] == ctx->ec_stream[0] && ctx->opts.on(cg::OPT_TX_CURVE_ON_HASH, true))
    ctx->ec_stream[1] = ctx->hash_stream;
  // Merkle ids on hash_stream (after compute_txids' metadata uploads and tx_index on
  // ctx->stream), so chunk k+1's hashing runs beside chunk k's signature kernels; the
  // signature kernels of chunk k wait for its ids (the ECDSA fork inherits that).
  CG_TRY(ctx, hipEventRecord(ev[2 * K], ctx->stream), "tx pipeline record");
  CG_TRY(ctx, hipStreamWaitEvent(ctx->hash_stream, ev[2 * K], 0), "tx pipeline wait");
  for (size_t k = 0; k < K; ++k) {
    CG_TRY(ctx, hipStreamWaitEvent(ctx->hash_stream, ev[k], 0), "tx pipeline wait");
    if ((st = hash_txs(ctx, d, arena_bytes, comp_start, tb[k], tb[k + 1], ctx->hash_stream)) != CG_OK) return st;
    CG_TRY(ctx, hipEventRecord(ev[K + k], ctx->hash_stream), "tx pipeline record");
    // (before the staging, which waits on the host when the key-reuse count runs)
    if (k + 2 < K && (st = enqueue_upload(k + 2)) != CG_OK) return st;
    const size_t s0 = sig_start[tb[k]], s1 = sig_start[tb[k + 1]];
    if (s1 > s0) {
      MsgSrc m;
      m.dev = d.ids;
      m.bytes = 32 * n_tx;
      m.off_dev = d.sig_moff + s0;
      m.len_dev = d.sig_mlen + s0;
      m.pk_dev = d.raw_pk + s0 * pk_stride;
      m.sig_dev = d.raw_sig + s0 * sig_stride;
      m.sl_dev = sig_len ? d.raw_sl + s0 : nullptr;
      m.raw_ready = ev[k];
      m.verdict_dev = verdict_d + s0;
      m.async = true;
      m.index_base = s0;
      cg_batch* b = nullptr;
      st = create_batch(ctx, s1 - s0, scheme_id ? scheme_id + s0 : nullptr, pk + s0 * pk_stride, pk_stride,
                        sig + s0 * sig_stride, sig_stride, sig_len ? sig_len + s0 : nullptr, m, &b);
      if (b) batches.push_back(b);  // freed by the caller after its final sync
      if (st == CG_OK) st = hip_ok(ctx, hipStreamWaitEvent(ctx->stream, ev[K + k], 0), "tx pipeline wait");
      if (st == CG_OK) st = launch_verify(ctx, b, mode, /*join_streams=*/false);
      if (st != CG_OK) return st;
    }
  }
  // ids of chunks without signatures, and the first_bad / ids readers, follow ctx->stream
  CG_TRY(ctx, hipEventRecord(ev[2 * K], ctx->hash_stream), "tx pipeline record");
  CG_TRY(ctx, hipStreamWaitEvent(ctx->stream, ev[2 * K], 0), "tx pipeline wait");
  return join_ecdsa_streams(ctx);
}

cg_status hip_ok(cg_ctx* ctx, hipError_t e, const char* what) {
  return e == hipSuccess ? CG_OK : hip_fail(ctx, e, what);
}

cg_status read_err_flag(cg_ctx* ctx) {
  uint32_t flag = 0;
  CG_TRY(ctx, hipMemcpyAsync(&flag, ctx->err_flag, 4, hipMemcpyDeviceToHost, ctx->stream), "read error flag");
  CG_TRY(ctx, hipStreamSynchronize(ctx->stream), "sync error flag");
  if (flag) return fail(ctx, CG_E_INVALID_ARGUMENT, "component out of arena bounds");
  return CG_OK;
}

uint32_t composite_scan(size_t n, const uint32_t* prog_start, const int32_t* prog, size_t n_sig, uint8_t* out);

// One cg_tx_verify_batch-style run: ids, every signature's verdict and the
// per-tx first failing signature, all left in device memory.
struct TxRun {
  TxDev d;
  uint8_t* verdict_d = nullptr;
  int32_t* fb_d = nullptr;
  std::vector<hipEvent_t> ev;
  std::vector<cg_batch*> batches;  // the pipeline's chunk batches (verdicts are slices of verdict_d)
  bool any_empty = false;
  size_t n_sig = 0;
  void release(cg_ctx* ctx) {
    for (hipStream_t s : {ctx->copy_stream, ctx->hash_stream, ctx->ec_stream[0], ctx->ec_stream[1], ctx->stream})
      (void)hipStreamSynchronize(s);
    for (cg_batch* b : batches) batch_free(ctx, b);
    batches.clear();
    for (hipEvent_t e : ev)
      if (e) (void)hipEventDestroy(e);
    ev.clear();
    dfree(ctx, fb_d);
    dfree(ctx, verdict_d);
    fb_d = nullptr;
    verdict_d = nullptr;
    d.release(ctx);
  }
};

cg_status tx_run(cg_ctx* ctx, int mode, size_t n_tx, const uint8_t* arena, size_t arena_bytes,
                 const uint64_t* comp_off, const uint32_t* comp_len, const uint32_t* comp_start, const uint8_t* salts,
                 const uint32_t* sig_start, const uint8_t* scheme_id, const uint8_t* pk, size_t pk_stride,
                 const uint8_t* sig, size_t sig_stride, const uint32_t* sig_len, TxRun& r) {
  cg_status st = compute_txids(ctx, n_tx, arena, arena_bytes, comp_off, comp_len, comp_start, salts, sig_start, r.d,
                               &r.any_empty, /*upload_arena=*/false);
  if (st != CG_OK) return st;
  r.n_sig = sig_start[n_tx];
  if (r.n_sig && (st = dalloc(ctx, &r.verdict_d, r.n_sig, "alloc tx verdicts")) != CG_OK) return st;
  st = tx_pipeline(ctx, mode, n_tx, arena, arena_bytes, comp_off, comp_len, comp_start, sig_start, scheme_id, pk,
                   pk_stride, sig, sig_stride, sig_len, r.d, r.verdict_d, r.ev, r.batches);
  if (st != CG_OK) return st;
  if ((st = dalloc(ctx, &r.fb_d, n_tx, "alloc first_bad")) != CG_OK) return st;
  CG_TRY(ctx, cg::launch_first_bad(r.verdict_d, r.d.sig_start, (uint32_t)n_tx, r.fb_d, ctx->stream), "first_bad");
  return CG_OK;
}

// A tx with no component has no id: CG_TX_NO_COMPONENTS (MerkleTreeException).
cg_status finish_empty_txs(cg_ctx* ctx, size_t n_tx, const uint32_t* comp_start, bool any_empty, int32_t* out) {
  if (!any_empty) return CG_OK;
  for (size_t t = 0; t < n_tx; ++t)
    if (comp_start[t + 1] == comp_start[t]) out[t] = CG_TX_NO_COMPONENTS;
  return fail(ctx, CG_E_MERKLE_EMPTY, "Cannot calculate Merkle root on empty hash list.");
}

}  // namespace

extern "C" {

cg_status cg_txid_batch(cg_ctx* ctx, size_t n_tx, const uint8_t* arena, size_t arena_bytes,
                        const uint64_t* comp_off, const uint32_t* comp_len, const uint32_t* comp_start,
                        const uint8_t* salts, uint8_t* ids_out) {
  CG_API_BEGIN
  if (!ctx) return CG_E_INVALID_ARGUMENT;
  if (n_tx == 0) return CG_OK;
  if (!ids_out) return fail(ctx, CG_E_INVALID_ARGUMENT, "null ids_out");
  if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, CG_E_DEVICE, "hipSetDevice");
  TxDev d;
  bool any_empty = false;
  cg_status st = compute_txids(ctx, n_tx, arena, arena_bytes, comp_off, comp_len, comp_start, salts, nullptr, d,
                               &any_empty);
  if (st == CG_OK) {
    hipError_t e = hipMemcpyAsync(ids_out, d.ids, 32 * n_tx, hipMemcpyDeviceToHost, ctx->stream);
    if (e != hipSuccess) st = hip_fail(ctx, e, "download ids");
  }
  if (st == CG_OK) st = read_err_flag(ctx);
  (void)hipStreamSynchronize(ctx->stream);
  d.release(ctx);
  collect_timings(ctx);
  if (st == CG_OK && any_empty)
    return fail(ctx, CG_E_MERKLE_EMPTY, "Cannot calculate Merkle root on empty hash list.");
  return st;
  CG_API_END(ctx)
}

cg_status cg_tx_verify_batch(cg_ctx* ctx, int mode, size_t n_tx, const uint8_t* arena, size_t arena_bytes,
                             const uint64_t* comp_off, const uint32_t* comp_len, const uint32_t* comp_start,
                             const uint8_t* salts, const uint32_t* sig_start, const uint8_t* scheme_id,
                             const uint8_t* pk, size_t pk_stride, const uint8_t* sig, size_t sig_stride,
                             const uint32_t* sig_len, int32_t* first_bad_out, uint8_t* verdict_out,
                             uint8_t* ids_out) {
  CG_API_BEGIN
  if (!ctx) return CG_E_INVALID_ARGUMENT;
  if (n_tx == 0) return CG_OK;
  if (!sig_start || !first_bad_out) return fail(ctx, CG_E_INVALID_ARGUMENT, "null pointer");
  if (mode != CG_MODE_IS_VALID && mode != CG_MODE_DO_VERIFY) return fail(ctx, CG_E_INVALID_ARGUMENT, "bad mode");
  if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, CG_E_DEVICE, "hipSetDevice");
  TxRun r;
  cg_status st = tx_run(ctx, mode, n_tx, arena, arena_bytes, comp_off, comp_len, comp_start, salts, sig_start,
                        scheme_id, pk, pk_stride, sig, sig_stride, sig_len, r);
  if (st == CG_OK) {
    hipError_t e = hipMemcpyAsync(first_bad_out, r.fb_d, 4 * n_tx, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess && verdict_out && r.verdict_d)
      e = hipMemcpyAsync(verdict_out, r.verdict_d, r.n_sig, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess && ids_out) e = hipMemcpyAsync(ids_out, r.d.ids, 32 * n_tx, hipMemcpyDeviceToHost, ctx->stream);
    if (e != hipSuccess) st = hip_fail(ctx, e, "first_bad");
  }
  if (st == CG_OK) st = read_err_flag(ctx);
  r.release(ctx);
  collect_timings(ctx);
  if (st != CG_OK) return st;
  return finish_empty_txs(ctx, n_tx, comp_start, r.any_empty, first_bad_out);
  CG_API_END(ctx)
}

cg_status cg_tx_verify_signatures_except(cg_ctx* ctx, int mode, size_t n_tx, const uint8_t* arena, size_t arena_bytes,
                                         const uint64_t* comp_off, const uint32_t* comp_len,
                                         const uint32_t* comp_start, const uint8_t* salts, const uint32_t* sig_start,
                                         const uint8_t* scheme_id, const uint8_t* pk, size_t pk_stride,
                                         const uint8_t* sig, size_t sig_stride, const uint32_t* sig_len,
                                         const uint32_t* req_start, const uint32_t* prog_start, const int32_t* prog,
                                         const uint8_t* allowed, int32_t* status_out, uint8_t* missing_out,
                                         uint8_t* ids_out) {
  CG_API_BEGIN
  if (!ctx) return CG_E_INVALID_ARGUMENT;
  if (n_tx == 0) return CG_OK;
  if (!sig_start || !status_out || !req_start || !prog_start) return fail(ctx, CG_E_INVALID_ARGUMENT, "null pointer");
  if (mode != CG_MODE_IS_VALID && mode != CG_MODE_DO_VERIFY) return fail(ctx, CG_E_INVALID_ARGUMENT, "bad mode");
  for (size_t t = 0; t < n_tx; ++t)
    if (req_start[t + 1] < req_start[t] || sig_start[t + 1] < sig_start[t])
      return fail(ctx, CG_E_INVALID_ARGUMENT, "req_start / sig_start not monotone");
  const size_t n_req = req_start[n_tx];
  for (size_t q = 0; q < n_req; ++q)
    if (prog_start[q + 1] < prog_start[q]) return fail(ctx, CG_E_INVALID_ARGUMENT, "prog_start not monotone");
  if (prog_start[n_req] && !prog) return fail(ctx, CG_E_INVALID_ARGUMENT, "null prog");
  // host pass: CompositeKey construction rules; leaf signature indices are within the tx
  std::vector<uint8_t> cstat(n_req ? n_req : 1, 0);
  uint32_t depth = 1;
  for (size_t t = 0; t < n_tx; ++t) {
    const uint32_t r0 = req_start[t], r1 = req_start[t + 1];
    if (r1 == r0) continue;
    const uint32_t dd = composite_scan(r1 - r0, prog_start + r0, prog, sig_start[t + 1] - sig_start[t],
                                       cstat.data() + r0);
    depth = std::max(depth, dd);
  }
  for (size_t q = 0; q < n_req; ++q)
    if (cstat[q] == cg::kCompositeInvalid)
      return fail(ctx, CG_E_INVALID_ARGUMENT, "required key " + std::to_string(q) +
                                                  " violates CompositeKey construction rules");
  if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, CG_E_DEVICE, "hipSetDevice");
  TxRun r;
  cg_status st = tx_run(ctx, mode, n_tx, arena, arena_bytes, comp_off, comp_len, comp_start, salts, sig_start,
                        scheme_id, pk, pk_stride, sig, sig_stride, sig_len, r);
  uint32_t *rs_d = nullptr, *ps_d = nullptr, *stack_d = nullptr;
  int32_t* prog_d = nullptr;
  uint8_t *allowed_d = nullptr, *ful_d = nullptr, *missing_d = nullptr;
  if (st == CG_OK && n_req) {
    if ((st = upload(ctx, &rs_d, req_start, n_tx + 1, "upload req_start")) == CG_OK &&
        (st = upload(ctx, &ps_d, prog_start, n_req + 1, "upload prog_start")) == CG_OK &&
        (st = upload(ctx, &prog_d, prog, 4 * (size_t)prog_start[n_req], "upload prog")) == CG_OK &&
        (st = (allowed ? upload(ctx, &allowed_d, allowed, n_req, "upload allowed") : CG_OK)) == CG_OK &&
        (st = upload(ctx, &ful_d, cstat.data(), n_req, "upload composite status")) == CG_OK &&
        (st = dalloc(ctx, &missing_d, n_req, "alloc missing")) == CG_OK &&
        (st = dalloc(ctx, &stack_d, (size_t)depth * n_req, "alloc composite stack")) == CG_OK) {
      hipError_t e;
      {
        Timed tm(ctx, "composite_eval", n_req);
        e = cg::launch_composite_eval(ps_d, prog_d, nullptr, nullptr, (uint32_t)n_req, stack_d, ful_d, ctx->stream);
      }
      if (e == hipSuccess)
        e = cg::launch_tx_missing(r.fb_d, rs_d, ful_d, allowed_d, (uint32_t)n_tx, missing_d, ctx->stream);
      if (e == hipSuccess && missing_out)
        e = hipMemcpyAsync(missing_out, missing_d, n_req, hipMemcpyDeviceToHost, ctx->stream);
      if (e != hipSuccess) st = hip_fail(ctx, e, "missing signatures");
    }
  } else if (st == CG_OK && missing_out && n_req) {
    std::memset(missing_out, 0, n_req);
  }
  if (st == CG_OK) {
    hipError_t e = hipMemcpyAsync(status_out, r.fb_d, 4 * n_tx, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess && ids_out) e = hipMemcpyAsync(ids_out, r.d.ids, 32 * n_tx, hipMemcpyDeviceToHost, ctx->stream);
    if (e != hipSuccess) st = hip_fail(ctx, e, "tx status");
  }
  if (st == CG_OK) st = read_err_flag(ctx);
  r.release(ctx);
  for (const void* p : {(const void*)rs_d, (const void*)ps_d, (const void*)stack_d, (const void*)prog_d,
                        (const void*)allowed_d, (const void*)ful_d, (const void*)missing_d})
    dfree(ctx, p);
  collect_timings(ctx);
  if (st != CG_OK) return st;
  return finish_empty_txs(ctx, n_tx, comp_start, r.any_empty, status_out);
  CG_API_END(ctx)
}

}  // extern "C"

namespace {

bool hash_less(const std::array<uint8_t, 32>& a, const std::array<uint8_t, 32>& b) { return a < b; }

// cg_ftx_verify_batch's device part as a pipeline over ftx-index chunks (the
// non-validating notary's whole crypto path is host bytes in, one status byte out;
// round 2 uploaded everything, then hashed: PCIe and kernels back to back).  Every
// chunk's rows — the arena prefix its components reach, their offsets / lengths /
// nonces, its node programs and roots — go out on copy_stream back to back.  Once a
// chunk's bytes are in, k_pmt_scan checks its node programs on the device (well-formed
// post-order tree, else MALFORMED in the status bytes; the deepest stack per wave) on
// ctx->stream, and the host waits once per chunk (hipEventSynchronize on ev_depth) for
// the per-wave depths, which size that chunk's evaluation stack; its leaf hashes and
// tree evaluation then run on ctx->stream beside the later chunks' copies.  Kernels
// index components and nodes absolutely (the chunk passes offset comp_start /
// node_start / roots / status pointers), so results land in place.
// CORDA_AMD_FTX_CHUNKS / _MIN_CHUNK override the split.
cg_status ftx_pipeline(cg_ctx* ctx, size_t n_ftx, const uint8_t* arena, size_t arena_bytes, const uint64_t* comp_off,
                       const uint32_t* comp_len, const uint32_t* comp_start, const uint8_t* nonces,
                       const uint32_t* node_start, const uint8_t* node_kind, const uint8_t* node_hash,
                       const uint8_t* root_hashes, uint8_t* result_out, size_t n_comp, size_t n_node, TxDev& d,
                       uint32_t*& nonces_d, uint32_t*& node_start_d, uint8_t*& kind_d, uint32_t*& node_hash_d,
                       uint32_t*& roots_d, uint8_t*& status_d, std::vector<uint32_t*>& stacks,
                       std::vector<hipEvent_t>& ev) {
  size_t kmax = 6, min_chunk = 65536;
  const cg::Options& o = ctx->opts;
  if (o.has(cg::OPT_FTX_CHUNKS)) kmax = std::max(1, o.i(cg::OPT_FTX_CHUNKS, 6));
  if (o.has(cg::OPT_FTX_MIN_CHUNK)) min_chunk = std::max(1, o.i(cg::OPT_FTX_MIN_CHUNK, 65536));
  const size_t K = std::max<size_t>(1, std::min<size_t>(kmax, n_ftx / min_chunk));
  // the last chunk's kernels run after the last byte: it gets `tail` of a regular chunk
  double tail = 0.5;
  if (o.has(cg::OPT_FTX_TAIL)) tail = std::min(1.0, std::max(0.1, o.d(cg::OPT_FTX_TAIL, 0.5)));
  std::vector<size_t> tb(K + 1);
  const double wsum = (double)(K - 1) + (K > 1 ? tail : 1.0);
  for (size_t k = 0; k <= K; ++k) tb[k] = k == K ? n_ftx : (size_t)((double)n_ftx * (double)k / wsum);
  cg_status st;
  if ((st = dalloc(ctx, &d.arena, arena_bytes + 16, "alloc ftx arena")) != CG_OK ||
      (st = dalloc(ctx, &d.comp_off, std::max<size_t>(n_comp, 1), "alloc comp_off")) != CG_OK ||
      (st = dalloc(ctx, &d.comp_len, std::max<size_t>(n_comp, 1), "alloc comp_len")) != CG_OK ||
      (st = dalloc(ctx, &d.comp_start, n_ftx + 1, "alloc comp_start")) != CG_OK ||
      (st = dalloc(ctx, &nonces_d, 8 * std::max<size_t>(n_comp, 1), "alloc nonces")) != CG_OK ||
      (st = dalloc(ctx, &d.comp_tx, std::max<size_t>(n_comp, 1), "alloc comp_tx")) != CG_OK ||
      (st = dalloc(ctx, &d.leaves, 8 * std::max<size_t>(n_comp, 1), "alloc leaves")) != CG_OK ||
      (st = dalloc(ctx, &node_start_d, n_ftx + 1, "alloc node_start")) != CG_OK ||
      (st = dalloc(ctx, &kind_d, std::max<size_t>(n_node, 1), "alloc node_kind")) != CG_OK ||
      (st = dalloc(ctx, &node_hash_d, 8 * std::max<size_t>(n_node, 1), "alloc node_hash")) != CG_OK ||
      (st = dalloc(ctx, &roots_d, 8 * n_ftx, "alloc roots")) != CG_OK ||
      (st = dalloc(ctx, &status_d, n_ftx, "alloc status")) != CG_OK)
    return st;
  // per-wave deepest stacks of each chunk's node programs come back through page-locked
  // memory (the evaluation stack is sized from their maximum)
  const size_t dw_words = ((n_ftx + 255) / 256) * 4 + 4 * K;
  uint32_t* depth_w_d = nullptr;
  if ((st = dalloc(ctx, &depth_w_d, dw_words, "alloc pmt depths")) != CG_OK) return st;
  stacks.push_back(depth_w_d);  // freed with the stacks
  if (ctx->pin_cap < dw_words * 4) {
    if (ctx->pin) (void)hipHostFree(ctx->pin);  // idle: every earlier call ended with a sync
    ctx->pin = nullptr;
    ctx->pin_cap = 0;
    if (hipHostMalloc((void**)&ctx->pin, dw_words * 4, hipHostMallocDefault) != hipSuccess) {
      (void)hipGetLastError();
      return fail(ctx, CG_E_OUT_OF_MEMORY, "page-locked staging for the pmt depths");
    }
    ctx->pin_cap = dw_words * 4;
  }
  uint32_t* depth_w_h = (uint32_t*)ctx->pin;
  ev.assign(K, nullptr);
  for (hipEvent_t& e : ev) CG_TRY(ctx, hipEventCreateWithFlags(&e, hipEventDisableTiming), "ftx pipeline event");
  CG_TRY(ctx, hipMemsetAsync(ctx->err_flag, 0, 4, ctx->stream), "clear error flag");
  CG_TRY(ctx, hipMemsetAsync(d.arena + arena_bytes, 0, 16, ctx->copy_stream), "pad ftx arena");
  std::vector<uint32_t> depth(K, 1);
  uint64_t up_to = 0;
  hipStream_t cs = ctx->copy_stream;
  auto put = [&](void* dst, const void* src, size_t bytes, hipStream_t q, const char* what) -> cg_status {
    if (bytes) CG_TRY(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, q), what);
    return CG_OK;
  };
  // 1. every chunk's bulk rows on copy_stream, back to back (the host work in between is
  //    one pass over the chunk's component offsets); event ev[k]
  for (size_t k = 0; k < K; ++k) {
    const size_t t0 = tb[k], t1 = tb[k + 1];
    for (size_t t = t0; t < t1; ++t)
      if (comp_start[t + 1] < comp_start[t] || node_start[t + 1] < node_start[t])
        return fail(ctx, CG_E_INVALID_ARGUMENT, "comp_start / node_start not monotone");
    const size_t c0 = comp_start[t0], c1 = comp_start[t1], j0 = node_start[t0], j1 = node_start[t1];
    if (c1 > n_comp || j1 > n_node)  // (a later decrease: the buffers were sized from the last entries)
      return fail(ctx, CG_E_INVALID_ARGUMENT, "comp_start / node_start not monotone");
    const uint64_t from = up_to;
    for (size_t c = c0; c < c1; ++c)
      up_to = std::max<uint64_t>(up_to, clamped_end(comp_off[c], comp_len[c], arena_bytes));
    Timed t(ctx, "h2d_ftx", (up_to - from) + (c1 - c0) * 44 + (j1 - j0) * 33 + (t1 - t0) * 40, cs);
    if ((st = put(d.arena + from, arena + from, up_to - from, cs, "upload ftx arena")) != CG_OK ||
        (st = put(d.comp_off + c0, comp_off + c0, (c1 - c0) * 8, cs, "upload comp_off")) != CG_OK ||
        (st = put(d.comp_len + c0, comp_len + c0, (c1 - c0) * 4, cs, "upload comp_len")) != CG_OK ||
        (st = put(d.comp_start + t0, comp_start + t0, (t1 - t0 + 1) * 4, cs, "upload comp_start")) != CG_OK ||
        (st = put(nonces_d + 8 * c0, nonces + 32 * c0, (c1 - c0) * 32, cs, "upload nonces")) != CG_OK ||
        (st = put(node_start_d + t0, node_start + t0, (t1 - t0 + 1) * 4, cs, "upload node_start")) != CG_OK ||
        (st = put(kind_d + j0, node_kind + j0, j1 - j0, cs, "upload node_kind")) != CG_OK ||
        (st = put(node_hash_d + 8 * j0, node_hash + 32 * j0, (j1 - j0) * 32, cs, "upload node_hash")) != CG_OK ||
        (st = put(roots_d + 8 * t0, root_hashes + 32 * t0, (t1 - t0) * 32, cs, "upload roots")) != CG_OK)
      return st;
    CG_TRY(ctx, hipEventRecord(ev[k], cs), "ftx pipeline record");
  }
  // 2. per chunk: its node programs checked on the device (k_pmt_scan: status, per-wave
  //    deepest stack) as soon as its rows are in, the depths read back (the host waits
  //    for this chunk's copy, not for later ones), then its leaf and tree kernels
  hipEvent_t ev_depth = nullptr;
  struct EvFree {
    hipEvent_t& e;
    ~EvFree() {
      if (e) (void)hipEventDestroy(e);
    }
  } ev_depth_free{ev_depth};
  CG_TRY(ctx, hipEventCreateWithFlags(&ev_depth, hipEventDisableTiming), "ftx pipeline event");
  size_t dw_off = 0;
  for (size_t k = 0; k < K; ++k) {
    const size_t t0 = tb[k], t1 = tb[k + 1], nk = t1 - t0;
    const uint32_t c0 = comp_start[t0], c1 = comp_start[t1];
    const size_t nw = ((nk + 255) / 256) * 4;
    CG_TRY(ctx, hipStreamWaitEvent(ctx->stream, ev[k], 0), "ftx pipeline wait");
    {
      Timed tm(ctx, "pmt_scan", nk);
      CG_TRY(ctx, cg::launch_pmt_scan(node_start_d + t0, kind_d, (uint32_t)nk, status_d + t0, depth_w_d + dw_off,
                                      ctx->stream),
             "launch pmt scan");
    }
    CG_TRY(ctx, hipMemcpyAsync(depth_w_h + dw_off, depth_w_d + dw_off, nw * 4, hipMemcpyDeviceToHost, ctx->stream),
           "download pmt depths");
    CG_TRY(ctx, hipEventRecord(ev_depth, ctx->stream), "ftx pipeline record");
    CG_TRY(ctx, hipEventSynchronize(ev_depth), "ftx pipeline depths");
    depth[k] = 1;
    for (size_t w = 0; w < nw; ++w) depth[k] = std::max(depth[k], depth_w_h[dw_off + w]);
    dw_off += nw;
    uint32_t* stack = nullptr;
    if ((st = dalloc(ctx, &stack, (size_t)8 * depth[k] * std::max<size_t>(nk, 1), "alloc pmt stack")) != CG_OK) return st;
    stacks.push_back(stack);
    CG_TRY(ctx, cg::launch_tx_index(d.comp_start + t0, nullptr, (uint32_t)nk, d.comp_tx, nullptr, nullptr, ctx->stream),
           "launch tx index");
    {
      Timed tm(ctx, "merkle_leaf", c1 - c0);
      CG_TRY(ctx,
             cg::launch_merkle_leaf(d.arena, arena_bytes, d.comp_off, d.comp_len, d.comp_start + t0, d.comp_tx, nullptr,
                                    nonces_d, c0, c1, d.leaves, ctx->err_flag, ctx->stream),
             "launch merkle leaf");
    }
    {
      Timed tm(ctx, "pmt_eval", nk);
      CG_TRY(ctx,
             cg::launch_pmt_eval(node_start_d + t0, kind_d, node_hash_d, d.comp_start + t0, d.leaves, roots_d + 8 * t0,
                                 (uint32_t)nk, stack, status_d + t0, ctx->stream),
             "launch pmt eval");
    }
  }
  CG_TRY(ctx, hipMemcpyAsync(result_out, status_d, n_ftx, hipMemcpyDeviceToHost, ctx->stream), "download ftx status");
  return CG_OK;
}

}  // namespace

extern "C" {

cg_status cg_ftx_verify_batch(cg_ctx* ctx, size_t n_ftx, const uint8_t* arena, size_t arena_bytes,
                              const uint64_t* comp_off, const uint32_t* comp_len, const uint32_t* comp_start,
                              const uint8_t* nonces, const uint32_t* node_start, const uint8_t* node_kind,
                              const uint8_t* node_hash, const uint8_t* root_hashes, uint8_t* result_out) {
  CG_API_BEGIN
  if (!ctx) return CG_E_INVALID_ARGUMENT;
  if (n_ftx == 0) return CG_OK;
  if (n_ftx > 0xFFFFFFF0ull) return fail(ctx, CG_E_INVALID_ARGUMENT, "too many transactions");
  if (!comp_start || !node_start || !root_hashes || !result_out || (node_start[n_ftx] && (!node_kind || !node_hash)) ||
      (comp_start[n_ftx] && (!comp_off || !comp_len || !arena || !nonces)))
    return fail(ctx, CG_E_INVALID_ARGUMENT, "null pointer");
  // (comp_start / node_start monotonicity is checked chunk by chunk in ftx_pipeline,
  // before any kernel runs, beside the earlier chunks' copies)
  if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, CG_E_DEVICE, "hipSetDevice");
  const size_t n_comp = comp_start[n_ftx], n_node = node_start[n_ftx];
  TxDev d;
  uint32_t *nonces_d = nullptr, *node_start_d = nullptr, *node_hash_d = nullptr, *roots_d = nullptr;
  uint8_t *kind_d = nullptr, *status_d = nullptr;
  std::vector<uint32_t*> stacks;
  std::vector<hipEvent_t> ev;
  cg_status st = ftx_pipeline(ctx, n_ftx, arena, arena_bytes, comp_off, comp_len, comp_start, nonces, node_start,
                              node_kind, node_hash, root_hashes, result_out, n_comp, n_node, d, nonces_d,
                              node_start_d, kind_d, node_hash_d, roots_d, status_d, stacks, ev);
  if (st == CG_OK) st = read_err_flag(ctx);
  // txs whose root matched but whose included-leaf multiset is too large for one lane:
  // compare sorted hash lists here (the hashes were computed on the device)
  std::vector<uint32_t> big;
  if (st == CG_OK)
    for (size_t t = 0; t < n_ftx; ++t)
      if (result_out[t] == cg::kPmtHostCheck) big.push_back((uint32_t)t);
  for (uint32_t t : big) {
    const uint32_t c0 = comp_start[t], k = comp_start[t + 1] - c0;
    std::vector<uint32_t> lv(8 * (size_t)k);
    hipError_t e = hipMemcpy(lv.data(), d.leaves + (size_t)8 * c0, 32 * (size_t)k, hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
      st = hip_fail(ctx, e, "download leaves");
      break;
    }
    std::vector<std::array<uint8_t, 32>> a, b;
    for (uint32_t c = 0; c < k; ++c) {
      std::array<uint8_t, 32> h;
      for (int q = 0; q < 8; ++q)
        for (int y = 0; y < 4; ++y) h[4 * q + y] = (uint8_t)(lv[8 * (size_t)c + q] >> (24 - 8 * y));  // big-endian words
      a.push_back(h);
    }
    for (uint32_t j = node_start[t]; j < node_start[t + 1]; ++j)
      if (node_kind[j] == cg::kPmtIncluded) {
        std::array<uint8_t, 32> h;
        memcpy(h.data(), node_hash + 32 * (size_t)j, 32);
        b.push_back(h);
      }
    std::sort(a.begin(), a.end(), hash_less);
    std::sort(b.begin(), b.end(), hash_less);
    result_out[t] = a == b ? cg::kPmtTrue : cg::kPmtFalse;
  }
  (void)hipStreamSynchronize(ctx->stream);
  (void)hipStreamSynchronize(ctx->copy_stream);
  (void)hipStreamSynchronize(ctx->hash_stream);
  for (const void* p : {(const void*)nonces_d, (const void*)node_start_d, (const void*)node_hash_d,
                        (const void*)roots_d, (const void*)kind_d, (const void*)status_d})
    dfree(ctx, p);
  for (uint32_t* p : stacks) dfree(ctx, p);
  for (hipEvent_t e : ev)
    if (e) (void)hipEventDestroy(e);
  d.release(ctx);
  collect_timings(ctx);
  return st;
  CG_API_END(ctx)
}

}  // extern "C"

namespace {

// Host pass over the composite-key programs: the construction-time constraints of
// CompositeKey (CompositeKey.kt:73-85, 139-144: arity >= 2, weights > 0, threshold
// > 0 and <= the children's total weight, totals that fit an Int) and the stack
// discipline of a single tree.  Returns the deepest stack; bad programs get
// kCompositeInvalid.
uint32_t composite_scan(size_t n, const uint32_t* prog_start, const int32_t* prog, size_t n_sig, uint8_t* out) {
  uint32_t max_depth = 1;
  std::vector<int64_t> st;
  for (size_t q = 0; q < n; ++q) {
    st.clear();
    bool bad = prog_start[q + 1] == prog_start[q];
    for (uint32_t o = prog_start[q]; o < prog_start[q + 1] && !bad; ++o) {
      const int32_t* op = prog + 4 * (size_t)o;
      if (op[2] <= 0) {
        bad = true;
      } else if (op[0] == cg::kCompositeLeaf) {
        bad = op[1] < -1 || (op[1] >= 0 && (size_t)op[1] >= n_sig);
        st.push_back(op[2]);
      } else if (op[0] == cg::kCompositeNode && op[1] >= 2 && (size_t)op[1] <= st.size()) {
        int64_t total = 0;
        for (int32_t c = 0; c < op[1]; ++c) {
          total += st.back();
          st.pop_back();
        }
        bad = total > INT32_MAX || op[3] <= 0 || op[3] > total;
        st.push_back(op[2]);
      } else {
        bad = true;
      }
      if (st.size() > max_depth) max_depth = (uint32_t)st.size();
    }
    out[q] = (bad || st.size() != 1) ? cg::kCompositeInvalid : 0;
  }
  return max_depth;
}

}  // namespace

extern "C" {

cg_status cg_composite_eval_batch(cg_ctx* ctx, size_t n_q, const uint32_t* prog_start, const int32_t* prog,
                                  size_t n_sig, const uint32_t* sig_start, const uint8_t* verdicts, uint8_t* out) {
  CG_API_BEGIN
  if (!ctx) return CG_E_INVALID_ARGUMENT;
  if (n_q == 0) return CG_OK;
  if (n_q > 0xFFFFFFF0ull) return fail(ctx, CG_E_INVALID_ARGUMENT, "too many queries");
  if (!prog_start || !sig_start || !out || (prog_start[n_q] && !prog) || false)
    return fail(ctx, CG_E_INVALID_ARGUMENT, "null pointer");
  for (size_t q = 0; q < n_q; ++q)
    if (prog_start[q + 1] < prog_start[q] || sig_start[q + 1] < sig_start[q] || sig_start[q + 1] > n_sig)
      return fail(ctx, CG_E_INVALID_ARGUMENT, "prog_start / sig_start not monotone or out of range");
  if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, CG_E_DEVICE, "hipSetDevice");
  const uint32_t depth = composite_scan(n_q, prog_start, prog, n_sig, out);
  const size_t n_ops = prog_start[n_q];
  uint32_t *ps_d = nullptr, *ss_d = nullptr, *stack_d = nullptr;
  int32_t* prog_d = nullptr;
  uint8_t *ver_d = nullptr, *out_d = nullptr;
  cg_status st;
  if ((st = upload(ctx, &ps_d, prog_start, n_q + 1, "upload prog_start")) == CG_OK &&
      (st = upload(ctx, &prog_d, prog, 4 * n_ops, "upload prog")) == CG_OK &&
      (st = upload(ctx, &ss_d, sig_start, n_q + 1, "upload sig_start")) == CG_OK &&
      (!verdicts || !n_sig || (st = upload(ctx, &ver_d, verdicts, n_sig, "upload verdicts")) == CG_OK) &&
      (st = upload(ctx, &out_d, out, n_q, "upload status")) == CG_OK &&
      (st = dalloc(ctx, &stack_d, (size_t)depth * n_q, "alloc composite stack")) == CG_OK) {
    hipError_t e;
    {
      Timed tm(ctx, "composite_eval", n_q);
      e = cg::launch_composite_eval(ps_d, prog_d, ss_d, ver_d, (uint32_t)n_q, stack_d, out_d, ctx->stream);
    }
    if (e == hipSuccess) e = hipMemcpyAsync(out, out_d, n_q, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) st = hip_fail(ctx, e, "composite eval");
  }
  (void)hipStreamSynchronize(ctx->stream);
  for (const void* p : {(const void*)ps_d, (const void*)prog_d, (const void*)ss_d, (const void*)ver_d,
                        (const void*)out_d, (const void*)stack_d})
    dfree(ctx, p);
  collect_timings(ctx);
  return st;
  CG_API_END(ctx)
}

}  // extern "C"
