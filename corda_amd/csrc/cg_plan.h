// Host-side plan of libcordagpu: the run-time options of a context and the choices a
// host-buffer verify (cg_verify_batch) makes from its shape — copy-bound or compute-bound,
// chunk bounds, latency lanes, early / split points, async arena, grouped MSM — as pure
// functions of (call shape, options).  No HIP, no context: cordagpu.cpp calls them, and
// the host build (tests/native/cg_host.cpp) runs them in the CPU suite and under
// ASan / UBSan (tests/test_plan.py), at every boundary the GPU plan tests cross.
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace cg {

// ------------------------------------------------------------------ constants
constexpr uint32_t kEdChunk = 1u << 21;  // Ed25519 scratch chunk (elements)
// cg_batch_verify of a large Ed25519 subset: pieces on two streams (launch_verify);
// CORDA_AMD_ED_SPLIT overrides the count, pieces stay >= kEdSplitMin elements
constexpr uint32_t kEdSplitMin = 65536;
constexpr uint32_t kEdSplitDefault = 1;  // r03d A/B: 2 or 4 pieces measured no faster (95-96 M/s either way)
// Ed25519 pieces up to this size run in the latency mode (two lanes per signature):
// r04f/r04g sweeps (host-buffer verify p50, 1 KB messages): 16,384 1.13 -> 1.02 ms,
// 32,768 1.51 -> 1.37 ms with it, 65,536 2.21 -> 2.36 ms (slower: two waves per SIMD
// already), so the crossover lies between 32k and 64k signatures
constexpr uint32_t kEdPairMaxDefault = 40000;
// ... for a one-chunk host-buffer call, by its bytes per element (verify_copy_bound):
// latency mode only up to where it beats the balanced path with split points (r05z: 32 B
// ids 24,576 0.84 vs 0.81 ms, 40,000 0.97 vs 0.83; 1 KB 32,768 1.21 vs 1.33, 40,000 1.65
// vs 1.49)
constexpr uint32_t kEdPairMaxCopyBound = 32768;
constexpr uint32_t kEdPairMaxCompute = 20480;
// ... and up to this size with four lanes per signature (the scalars' 64-bit halves
// over 2^64-multiple tables: ~64 doublings per lane instead of ~128)
constexpr uint32_t kEdQuadMaxDefault = 32768;
// ... and up to this size with eight (32-bit parts over 2^(32 u)-multiple tables: ~32
// doublings per lane): r04ap, 1 KB messages, 2,048-6,144 signatures -0.012..0.015 ms
// against four lanes, 8,192 +0.07 ms — past ~7,280 signatures the eight-lane points
// blocks and the hash blocks no longer get a CU each (ed_spread_lds)
constexpr uint32_t kEdOctMaxDefault = 7168;
// grouped balanced MSM (cg_ed25519_bucket) from this many signatures per piece (round 6;
// the bucket kernels need at least 3,072)
constexpr uint32_t kEdBucketMinDefault = 16384;
constexpr uint32_t kEdBucketMinFloor = 4096;
// Early points: a one-chunk verify of an all-Ed25519 in-order batch on the balanced path
// uploads its key and signature rows in up to CORDA_AMD_EARLY_POINTS (default 4) parts of
// at least kEarlyPartMin signatures, and each part's points kernel starts on copy_stream,
// reading the raw rows, as soon as that part has landed (2^18 x 32 B: rows copy ~0.55 ms,
// then the points kernel ~0.63 ms, both ahead of the MSM; r05g: 4 parts 3.24 -> 2.92 ms).
// Smaller parts lose: a points kernel of 32,768 signatures takes as long as one of 65,536,
// and the extra pageable copies cost ~0.1 ms (r05g: 65,536 in two parts 0.98 -> 1.10 ms).
constexpr uint32_t kEarlyPartMin = 65536;
// Async arena: a one-chunk call's deferred arena (and offsets / lengths) of at least
// kAsyncArenaMin bytes goes up from the upload thread while the calling thread copies the
// key and signature rows, instead of after them — below the early-points sizes, whose row
// parts it would slow (r05x: 65,536 x 1 KB 2.19 -> 2.11 ms, 16,384 x 1 KB 0.79 -> 0.77;
// but 4,096 x 1 KB 0.47 -> 0.56, the thread hand-off, and 2^17-2^18 x 32 B +0.05-0.15).
constexpr size_t kAsyncArenaMin = (size_t)8 << 20;
// From kBoundsBesideMin elements the arena-bounds pass runs on the upload thread
// (cordagpu.cpp BoundsBeside), so the thread is awake and an arena from 1 MB goes up from
// it too, with no hand-off wait (r06v, 32 B ids: 40,001 0.857 -> 0.83 ms, 65,536 0.945 ->
// 0.90; 100,000 equal).
constexpr size_t kBoundsBesideMin = 32768;
constexpr size_t kAsyncArenaSmallMin = (size_t)1 << 20;
// The async arena's copies run on hash_stream from the upload thread with no wait on the
// split pieces' fork: it must never coexist with a split (> 1 piece) prepared batch, which
// needs at least 2 * kEdSplitMin Ed25519 elements (advisor r05).
static_assert(kEarlyPartMin <= kEdSplitMin,
              "async arena (n < 2 kEarlyPartMin) must stay below the split pieces (n >= 2 kEdSplitMin)");

// ------------------------------------------------------------------ options
// Run-time options of a context: every CORDA_AMD_* knob is read from the
// environment ONCE, at cg_open, into the context; cg_set_option(ctx, key, value) changes
// one per context (value NULL: unset, the library default).  No call path reads the
// environment.  None of them changes a verdict.
enum Opt : int {
  OPT_KEY_REUSE,
  OPT_ED_PAIR_MAX,
  OPT_ED_QUAD_MAX,
  OPT_ED_OCT_MAX,
  OPT_ED_SPREAD_LDS,
  OPT_ED_OVERLAP,
  OPT_ED_SPLIT,
  OPT_ED_BUCKET_MIN,
  OPT_EARLY_POINTS,
  OPT_SPLIT_POINTS,
  OPT_ASYNC_ARENA,
  OPT_ARENA_BESIDE,
  OPT_VERIFY_POLICY,
  OPT_VERIFY_CHUNKS,
  OPT_VERIFY_MIN_CHUNK,
  OPT_VERIFY_HEAD,
  OPT_VERIFY_TAIL,
  OPT_VERIFY_LANES,
  OPT_VERIFY_SERIAL,
  OPT_VERIFY_UPLOAD_THREAD,
  OPT_VERIFY_AHEAD,
  OPT_VERIFY_RING,
  OPT_VERIFY_ONE_DMA,
  OPT_VERIFY_SLICE_KB,
  OPT_RING_MAX_MB,
  OPT_COPY_THREADS,
  OPT_TX_CHUNKS,
  OPT_TX_MIN_CHUNK,
  OPT_TX_TAIL,
  OPT_TX_CURVE_ON_HASH,
  OPT_FTX_CHUNKS,
  OPT_FTX_MIN_CHUNK,
  OPT_FTX_TAIL,
  OPT_TIMELINE,
  OPT_COUNT
};
inline const char* opt_name(int o) {
  static const char* const k[OPT_COUNT] = {
      "CORDA_AMD_KEY_REUSE",         "CORDA_AMD_ED_PAIR_MAX",       "CORDA_AMD_ED_QUAD_MAX",
      "CORDA_AMD_ED_OCT_MAX",        "CORDA_AMD_ED_SPREAD_LDS",     "CORDA_AMD_ED_OVERLAP",
      "CORDA_AMD_ED_SPLIT",          "CORDA_AMD_ED_BUCKET_MIN",     "CORDA_AMD_EARLY_POINTS",
      "CORDA_AMD_SPLIT_POINTS",      "CORDA_AMD_ASYNC_ARENA",       "CORDA_AMD_ARENA_BESIDE",
      "CORDA_AMD_VERIFY_POLICY",     "CORDA_AMD_VERIFY_CHUNKS",     "CORDA_AMD_VERIFY_MIN_CHUNK",
      "CORDA_AMD_VERIFY_HEAD",       "CORDA_AMD_VERIFY_TAIL",       "CORDA_AMD_VERIFY_LANES",
      "CORDA_AMD_VERIFY_SERIAL",     "CORDA_AMD_VERIFY_UPLOAD_THREAD", "CORDA_AMD_VERIFY_AHEAD",
      "CORDA_AMD_VERIFY_RING",       "CORDA_AMD_VERIFY_ONE_DMA",    "CORDA_AMD_VERIFY_SLICE_KB",
      "CORDA_AMD_RING_MAX_MB",       "CORDA_AMD_COPY_THREADS",      "CORDA_AMD_TX_CHUNKS",
      "CORDA_AMD_TX_MIN_CHUNK",      "CORDA_AMD_TX_TAIL",           "CORDA_AMD_TX_CURVE_ON_HASH",
      "CORDA_AMD_FTX_CHUNKS",        "CORDA_AMD_FTX_MIN_CHUNK",     "CORDA_AMD_FTX_TAIL",
      "CORDA_AMD_TIMELINE"};
  return o >= 0 && o < OPT_COUNT ? k[o] : nullptr;
}

struct Options {
  bool set[OPT_COUNT] = {};
  std::string val[OPT_COUNT];

  static int find(const char* key) {  // -1: not an option
    for (int o = 0; key && o < OPT_COUNT; ++o)
      if (std::strcmp(key, opt_name(o)) == 0) return o;
    return -1;
  }
  void assign(int o, const char* v) {
    set[o] = v != nullptr;
    val[o] = v ? v : "";
  }
  // the snapshot cg_open takes (the only getenv of the options)
  void from_env() {
    for (int o = 0; o < OPT_COUNT; ++o) assign(o, std::getenv(opt_name(o)));
  }
  // "KEY=VALUE;KEY=VALUE" (tests of the host build); returns false on an unknown key
  bool parse(const char* spec) {
    std::string s = spec ? spec : "";
    size_t a = 0;
    while (a < s.size()) {
      size_t z = s.find(';', a);
      if (z == std::string::npos) z = s.size();
      const std::string kv = s.substr(a, z - a);
      a = z + 1;
      if (kv.empty()) continue;
      const size_t eq = kv.find('=');
      const int o = find(kv.substr(0, eq).c_str());
      if (o < 0) return false;
      assign(o, eq == std::string::npos ? "" : kv.c_str() + eq + 1);
    }
    return true;
  }
  bool has(Opt o) const { return set[o]; }
  const char* str(Opt o) const { return set[o] ? val[o].c_str() : nullptr; }
  int i(Opt o, int def) const { return set[o] ? std::atoi(val[o].c_str()) : def; }
  double d(Opt o, double def) const { return set[o] ? std::atof(val[o].c_str()) : def; }
  bool on(Opt o, bool def) const { return set[o] ? std::atoi(val[o].c_str()) != 0 : def; }
};

// ------------------------------------------------------------------ knob readers
// CORDA_AMD_KEY_REUSE: 0 never, 1 always, unset / other: automatic (-1)
inline int key_reuse_forced(const Options& o) {
  const char* e = o.str(OPT_KEY_REUSE);
  return e && (e[0] == '0' || e[0] == '1') ? e[0] - '0' : -1;
}
// Latency mode (two / four / eight lanes per signature) for Ed25519 pieces of at most this
// many signatures on the balanced path; CORDA_AMD_ED_PAIR_MAX overrides (0: never).
// call_default: the batch's own threshold (a one-chunk host-buffer call's, by its bytes
// per element).
inline uint32_t ed_pair_max(const Options& o, uint32_t call_default = 0) {
  return o.has(OPT_ED_PAIR_MAX) ? (uint32_t)std::max(0, o.i(OPT_ED_PAIR_MAX, 0))
                                : call_default ? call_default : kEdPairMaxDefault;
}
inline uint32_t ed_quad_max(const Options& o) { return (uint32_t)std::max(0, o.i(OPT_ED_QUAD_MAX, (int)kEdQuadMaxDefault)); }
inline uint32_t ed_oct_max(const Options& o) { return (uint32_t)std::max(0, o.i(OPT_ED_OCT_MAX, (int)kEdOctMaxDefault)); }
// Balanced MSM pieces of at least this many signatures run over lanes grouped by digit
// count; CORDA_AMD_ED_BUCKET_MIN overrides (0: never; values below 4,096 mean 4,096).
inline uint32_t ed_bucket_min(const Options& o) {
  const int v = o.i(OPT_ED_BUCKET_MIN, (int)kEdBucketMinDefault);
  return v > 0 ? std::max<uint32_t>((uint32_t)v, kEdBucketMinFloor) : UINT32_MAX;
}
inline bool ed_overlap_enabled(const Options& o) { return o.on(OPT_ED_OVERLAP, true); }
inline bool async_arena_enabled(const Options& o) { return o.on(OPT_ASYNC_ARENA, true); }
inline bool split_points_enabled(const Options& o) { return o.on(OPT_SPLIT_POINTS, true); }
inline uint32_t early_points_parts(const Options& o) {
  return o.has(OPT_EARLY_POINTS) ? (uint32_t)std::min(8, std::max(0, o.i(OPT_EARLY_POINTS, 4))) : 4u;
}

// Lanes per signature of an Ed25519 piece of `cnt` signatures on the balanced path
// (launch_verify): 1 above pair_max, else 8 / 4 / 2 by the oct / quad thresholds — when
// the piece's scratch region has room for its tables (four lanes: 2 cnt slots, eight: 4
// cnt) and it is one piece.
inline uint32_t ed_lanes(uint32_t cnt, uint32_t pair_max, const Options& o, bool quad_room = true,
                         bool oct_room = true) {
  if (cnt > pair_max) return 1;
  const bool quad = cnt <= std::min(pair_max, ed_quad_max(o)) && quad_room;
  const bool oct = quad && cnt <= ed_oct_max(o) && oct_room;
  return oct ? 8 : quad ? 4 : 2;
}

// A host-buffer call is copy-bound when its bytes take longer over PCIe than its
// Ed25519 kernels take on the device: ~50 GB/s against ~9.5 ns per verify (105 M/s), i.e.
// above ~475 bytes per element (1 KB messages: 1,132 B; 32 B tx ids: 140 B).  A
// compute-bound call gains nothing from chunking its copies: its chunks' kernels, which
// the pipeline runs two at a time, each pay a serial chain and the host staging of the
// first chunk delays the first kernel.  CORDA_AMD_VERIFY_POLICY=0 restores the copy-bound
// chunking for every call (A/B).
inline bool verify_copy_bound(size_t n, size_t msg_bytes, size_t row_bytes, const Options& o) {
  if (o.has(OPT_VERIFY_POLICY) && o.i(OPT_VERIFY_POLICY, 1) == 0) return true;
  return n && (double)msg_bytes / (double)n + (double)row_bytes > 475.0;
}

// Chunk boundaries of an n-element host batch: K = n / min_chunk chunks (at most kmax),
// 64-aligned (whole waves); the first is `head` and the last `tail` times a regular one (a
// small first chunk starts the kernels early, a small last one shortens what runs after
// the last byte).  CORDA_AMD_VERIFY_CHUNKS / _MIN_CHUNK / _HEAD / _TAIL override.
inline std::vector<size_t> verify_chunk_bounds(size_t n, bool copy_bound, const Options& o) {
  // head 0.25: the host stages the first chunk's pageable bytes before any DMA can start
  // (r04d spans: 0.37 ms at 0.5); tail 0.25: the last chunk — the only one whose kernels
  // run after the last byte — runs in the four-lane latency mode for 2^18-element calls
  // (r05 sweeps, 2^18 x 1 KB: 6.89-6.91 ms against 6.98-7.05 at 0.4)
  const size_t kmax = o.has(OPT_VERIFY_CHUNKS) ? (size_t)std::max(1, o.i(OPT_VERIFY_CHUNKS, 8)) : 8;
  const size_t min_chunk = o.has(OPT_VERIFY_MIN_CHUNK) ? (size_t)std::max(1, o.i(OPT_VERIFY_MIN_CHUNK, 32768)) : 32768;
  const double head = o.has(OPT_VERIFY_HEAD) ? std::min(2.0, std::max(0.05, o.d(OPT_VERIFY_HEAD, 0.25))) : 0.25;
  const double tail = o.has(OPT_VERIFY_TAIL) ? std::min(2.0, std::max(0.05, o.d(OPT_VERIFY_TAIL, 0.25))) : 0.25;
  // below 2^17 elements one chunk is fastest (r03b sweep, 65,536 x 1 KB pageable: 2.38 ms
  // as one chunk, 2.70 ms as two: every chunk adds a serial ~0.7 ms kernel chain); a
  // compute-bound call runs as one chunk up to 2^20 elements (r05 sweeps, 32 B ids)
  const bool tuned = o.has(OPT_VERIFY_MIN_CHUNK) || o.has(OPT_VERIFY_CHUNKS);
  const size_t whole = tuned ? 0 : (size_t)1 << (copy_bound ? 17 : 20);
  const size_t K = n < whole ? 1 : std::max<size_t>(1, std::min<size_t>(kmax, n / min_chunk));
  std::vector<size_t> b(K + 1, 0);
  std::vector<double> w(K, 1.0);
  if (K > 1) {
    w[0] = head;
    w[K - 1] = tail;
  }
  double wsum = 0;
  for (double x : w) wsum += x;
  double acc = 0;
  for (size_t k = 1; k < K; ++k) {
    acc += w[k - 1];
    b[k] = std::min(n, (size_t)((double)n * acc / wsum) / 64 * 64);
  }
  b[K] = n;
  for (size_t k = 1; k <= K; ++k) b[k] = std::max(b[k], b[k - 1]);
  return b;
}

// ------------------------------------------------------------------ the plan
// Shape of a cg_verify_batch call (what the host knows before any copy).
struct VerifyShape {
  size_t n = 0;                 // elements
  size_t n_ed = 0;              // Ed25519 elements among them
  size_t msg_bytes = 0;         // message arena bytes
  size_t pk_stride = 0, sig_stride = 0;
  bool sig_len = false;         // the caller passes signature lengths
  bool ecdsa = false;           // some element is ECDSA
  bool ed_in_order = false;     // every element Ed25519, in order, none flagged KEY_INVALID
  int keys_repeat = -1;         // the host key sample (key_sample_suggests_reuse): 1 / 0, -1 not taken
};

struct VerifyPlan {
  bool copy_bound = false;
  std::vector<size_t> chunks;   // boundaries: 2 entries = one chunk (stage, then verify)
  // one-chunk calls (chunks.size() == 2); the pipeline plans its chunks as it goes
  uint32_t pair_max = 0;        // latency-mode threshold of the call
  bool defer_arena = false;     // the message arena goes up from launch_verify, beside the points kernel
  bool defer_meta = false;      // ... and its offsets / lengths with it
  bool async_arena = false;     // ... issued by the upload thread beside the row copies
  bool rows_direct = false;     // the points kernels read the caller's raw rows
  bool needs_key_sample = false;  // early / split points hinge on keys_repeat, which was not given
  uint32_t early_parts = 0;     // row upload parts with a points kernel each (> 1: early points)
  bool split_points = false;    // the key half of the points phase beside the signature rows' copy
  bool key_dedupe = false;      // staged with the device key dedupe (key-reuse path if keys repeat)
  uint32_t lanes = 1;           // Ed25519 lanes per signature (balanced path; 1 when key_dedupe finds reuse too)
  bool grouped_msm = false;     // balanced MSM over lanes grouped by digit count
};

// One-chunk plan of a call.  Two choices depend on the host key sample
// (key_sample_suggests_reuse: do the keys repeat?) — early / split points (only for
// distinct keys) and the device key dedupe (only for repeating ones); when the shape
// does not say (keys_repeat -1) and a choice hinges on it, needs_key_sample is set and
// the caller plans again with the sample's answer, so the sample is taken at most once
// and only when it matters.  lanes / grouped_msm are the balanced path's: a dedupe that
// finds keys repeating n / n_keys >= 8 times runs the key-reuse kernels instead.
inline VerifyPlan plan_verify(const VerifyShape& s, const Options& o) {
  VerifyPlan p;
  p.copy_bound = verify_copy_bound(s.n, s.msg_bytes, 12 + s.pk_stride + s.sig_stride + (s.sig_len ? 4 : 0), o);
  p.chunks = verify_chunk_bounds(s.n, p.copy_bound, o);
  if (p.chunks.size() != 2) return p;
  p.pair_max = p.copy_bound ? kEdPairMaxCopyBound : kEdPairMaxCompute;
  const uint32_t pair_max = ed_pair_max(o, p.pair_max);
  const int forced = key_reuse_forced(o);
  p.defer_arena = s.msg_bytes && !s.ecdsa && s.n_ed;
  p.defer_meta = p.defer_arena && s.ed_in_order;
  p.async_arena = p.defer_arena &&
                  (s.msg_bytes >= kAsyncArenaMin || (s.msg_bytes >= kAsyncArenaSmallMin && s.n >= kBoundsBesideMin)) &&
                  s.n < 2 * (size_t)kEarlyPartMin &&
                  async_arena_enabled(o) && !o.has(OPT_ED_SPLIT);
  p.rows_direct = s.ed_in_order && s.pk_stride % 4 == 0 && s.sig_stride % 4 == 0;
  if (p.rows_direct && s.n > pair_max && s.n <= kEdChunk && ed_overlap_enabled(o) && !o.has(OPT_ED_SPLIT)) {
    if (forced == 0 || (forced < 0 && s.keys_repeat == 0)) {
      p.early_parts = std::min<uint32_t>(early_points_parts(o), (uint32_t)(s.n / kEarlyPartMin));
      p.split_points = p.early_parts <= 1 && split_points_enabled(o);
    } else if (forced < 0 && s.keys_repeat < 0) {
      p.needs_key_sample = true;
    }
  }
  if (forced == 1) {
    p.key_dedupe = true;
  } else if (forced < 0 && s.n_ed >= 64 && s.n_ed > pair_max) {
    if (s.keys_repeat < 0) p.needs_key_sample = true;
    p.key_dedupe = s.keys_repeat == 1;
  }
  const uint32_t ne = (uint32_t)std::min<size_t>(s.n_ed, UINT32_MAX);
  p.lanes = forced == 1 ? 1 : ed_lanes(ne, pair_max, o);
  p.grouped_msm = p.lanes == 1 && forced != 1 && ne >= ed_bucket_min(o);
  return p;
}

}  // namespace cg
