// K1: Ed25519 (EDDSA_ED25519_SHA512) batch verification kernels for gfx950
// (phases of cg_ed25519.h, one lane per signature in each):
//
//   cg_ed25519_hash     SHA-512 challenge, scalars, half-size reduction, digits —
//                       integer/hash work, no field arithmetic beyond Abyte
//   cg_ed25519_points   decode A and R (two square roots), tables k*(-A) and k*R
//                       (k = 1..8) written to HBM scratch; independent of the hash
//                       kernel (its own verdict word pstat), so the two may run side
//                       by side
//   cg_ed25519_msm      [b]B + [c0](-A) + [c1](+-R) over ~132 shared bit positions
//                       (4-bit windows for A/R, kBWin-bit windows over the shared
//                       tables B and 2^128 B in HBM), identity test -> verdict
//   cg_ed25519_btab_build  the shared tables (context creation)
//
// Integer VALU work only (no MFMA): field products are v_mad_i64_i32.
// Device layout (SoA, word-major, `cap` = batch capacity, i = element):
//   pk[w*cap+i] (8 words), sig[w*cap+i] (16 words: R then S), sig_len[i],
//   msg_off[i] (u64, into the arena), msg_len[i]; scratch (`scap` = chunk):
//   status[i] (verdict | digit count << 8 | R sign << 16), digits[w*scap+i]
//   (24 words), and the per-signature tables entries 0..7 = k*(-A), 8..15 = k*R for
//   k = 1..8 (cached points packed to 32 words = one 128-byte line)
//   lane-contiguous: table[(i*17 + e)*32 + w] (one pad entry: CG_ED_TAB_PAD), 2,176 B per
//   lane; a zero digit reads one shared identity entry.  (Round 3 measured a
//   quad-major layout across lanes — each wave load one contiguous 1 KB run — slower:
//   msm 7.11 -> 8.35 ms, points 2.47 -> 3.9 ms per 1 M, an entry's quads 16 MB apart.)
#include "cg_ed25519.h"
#include "cg_kernels.h"

using namespace cg;

namespace {

// Occupancy target of the MSM kernel (waves per SIMD).
#ifndef CG_MSM_WAVES
#define CG_MSM_WAVES 2
#endif
// the same for the key-reuse MSM
#ifndef CG_MSM_R_WAVES
#define CG_MSM_R_WAVES 2
#endif

// A table entry is its four coordinates as canonical 255-bit values (8 words each):
// 128 B = one cache line per entry (round 3: against 160 B of limbs over two or three
// lines, MSM -2 %); the points kernel canonicalises on store, the MSM unpacks
// (floor-shaped limbs).  The lane tables keep k = 1..8 only (16 entries, 2 KB per lane);
// a zero digit reads one shared identity entry (L1 / L2 resident) instead (+1 %).
constexpr int kTabLimbs = 32;  // words per cached point: 4 fe x 8 packed
constexpr int kSlotsPerPoint = kATabEntries - 1;
// CG_ED_TAB_PAD: unused entries after a lane's table, so the lane stride is not a
// power of two: at 16 entries = 2 KB every lane of a wave writes into the same L2
// channel and set, lines leave L2 before their eight 16-byte stores have merged and
// the points kernel wrote 3.4 KB per verify for its 2 KB of entries; 17 entries:
// 2.1 KB (r03k PMC).
#ifndef CG_ED_TAB_PAD
#define CG_ED_TAB_PAD 1
#endif
constexpr int kLaneEntries = 2 * kSlotsPerPoint + CG_ED_TAB_PAD;
constexpr int kBStride = 32;   // shared-table entry (precomputed point, 3 fe x 10 limbs) padded to one 128-byte line

// A lane's view of the per-signature tables (lane-contiguous: a lane's entries are
// consecutive lines; round 3 measured the quad-major alternative 17 % slower): entry
// k's quad q sits at base[k * kTabLimbs / 4 + q].
struct LaneTab {
  int4* base;
  CG_DEV int4* entry(uint32_t k) const { return base + (size_t)k * (kTabLimbs / 4); }
};
CG_DEV LaneTab lane_table(int32_t* table, uint32_t i, uint32_t scap) {
  (void)scap;
  return {reinterpret_cast<int4*>(table + (size_t)i * (kLaneEntries * kTabLimbs))};
}

// Occupancy target of the hash kernel (0: the compiler's choice, 3 waves / SIMD at 138
// VGPRs).  4 waves (128 VGPRs, 26 dwords spilled in the balanced path) hides more of
// the serial SHA-512 rounds' latency: hash 1.355 -> 1.31 ms per 10 M chunk-set, config 2
// +0.8 % (profiles/r04o_ab.txt, 3 interleaved reps).
#ifndef CG_HASH_WAVES
#define CG_HASH_WAVES 4
#endif
#if CG_HASH_WAVES
#define CG_HASH_ATTR __attribute__((amdgpu_waves_per_eu(CG_HASH_WAVES, 8)))
#else
#define CG_HASH_ATTR
#endif
// Wave priority of the hash kernel (it runs beside the points kernel, CG_WAVE_PRIO): 2,
// one above the points kernel — the hash is the longer of the two chains before the
// MSM in small calls (4,096 x 1 KB host verify 0.658 -> 0.630 ms, r04s), config 2 equal
// (r04t).
#ifndef CG_HASH_PRIO
#define CG_HASH_PRIO 2
#endif
template <bool REUSE>
__global__ __launch_bounds__(256) CG_HASH_ATTR void cg_ed25519_hash(const uint32_t* __restrict__ pk, const uint32_t* __restrict__ sig,
                                                       const uint32_t* __restrict__ sig_len,
                                                       const uint8_t* __restrict__ arena,
                                                       const uint64_t* __restrict__ msg_off,
                                                       const uint32_t* __restrict__ msg_len, uint32_t n, uint32_t cap,
                                                       uint32_t scap, uint32_t mode, uint32_t* __restrict__ status,
                                                       uint32_t* __restrict__ digits, uint32_t full_mod,
                                                       uint32_t index_base) {
  CG_WAVE_PRIO(CG_HASH_PRIO);
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t pkw[8], rw[8], dig[kDigitWords], ndig, rneg;
  CG_UNROLL for (int w = 0; w < 8; ++w) pkw[w] = pk[(size_t)w * cap + i];
  CG_UNROLL for (int w = 0; w < 8; ++w) rw[w] = sig[(size_t)w * cap + i];
  const bool force_full = full_mod != 0 && (index_base + i) % full_mod == 0;  // cg_set_debug test hook
  // S (signature words 8..15) is loaded after the half-size reduction (ed25519_hash_stage_r)
  const uint32_t pre = ed25519_hash_stage_r<false, REUSE>(
      pkw, rw, [&](uint32_t sw[8]) CG_LINLINE {
        CG_UNROLL for (int w = 0; w < 8; ++w) sw[w] = sig[(size_t)(8 + w) * cap + i];
      },
      sig_len[i], arena + msg_off[i], msg_len[i], mode, dig, ndig, rneg, force_full);
  status[i] = pre | ndig << 8 | rneg << 16;
  if (pre != V_COMPUTE) return;
  CG_UNROLL for (int w = 0; w < kDigitWords; ++w) digits[(size_t)w * scap + i] = dig[w];
}

// The shared identity entry (1, 1, 1, 0) in the table's entry format.
__device__ __attribute__((aligned(128))) const int4 g_ident_entry[kTabLimbs / 4] = {
    {1, 0, 0, 0}, {0, 0, 0, 0}, {1, 0, 0, 0}, {0, 0, 0, 0}, {1, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};

CG_DEV void store_cached(int4* dst, const ge_cached& c) {
  uint32_t w[4][8];
  fe_tobytes(w[0], c.YplusX);
  fe_tobytes(w[1], c.YminusX);
  fe_tobytes(w[2], c.Z);
  fe_tobytes(w[3], c.T2d);
  CG_UNROLL for (int f = 0; f < 4; ++f)
    CG_UNROLL for (int h = 0; h < 2; ++h)
      dst[2 * f + h] = make_int4((int)w[f][4 * h], (int)w[f][4 * h + 1], (int)w[f][4 * h + 2], (int)w[f][4 * h + 3]);
}

// A table entry in its storage form (the MSM fetches the A entry of a window before
// the window's doublings and unpacks it after them: 32 packed words live across the
// doublings instead of 40 limbs).
struct RawEntry {
  int4 q[kTabLimbs / 4];
};
CG_DEV void unpack_entry(const RawEntry& r, ge_cached& c) {
  uint32_t w[4][8];
  CG_UNROLL for (int f = 0; f < 4; ++f)
    CG_UNROLL for (int h = 0; h < 2; ++h) {
      const int4 x = r.q[2 * f + h];
      w[f][4 * h] = (uint32_t)x.x;
      w[f][4 * h + 1] = (uint32_t)x.y;
      w[f][4 * h + 2] = (uint32_t)x.z;
      w[f][4 * h + 3] = (uint32_t)x.w;
    }
  fe_frombytes(c.YplusX, w[0]);
  fe_frombytes(c.YminusX, w[1]);
  fe_frombytes(c.Z, w[2]);
  fe_frombytes(c.T2d, w[3]);
}

// Entry k (0..8) of point p (0: -A, 1: R; a per-signature table holding R only uses
// p = 0) of a lane's table: stored at k - 1 (k = 0 reads the shared identity entry).
CG_DEV void store_slot(const LaneTab& lt, int p, int k, const ge_cached& c) {
  if (k == 0) return;
  store_cached(lt.entry(p * kSlotsPerPoint + k - 1), c);
}
// Lane-table entries are read through the global address space: the select between a
// lane's entry and the shared identity entry left a generic pointer, and the MSM issued
// flat loads (r06bb: global loads, msm 6.50-6.77 -> 6.41-6.54 ms, config 2 +1 %; the same
// loads marked nontemporal measured 9 % slower).
CG_DEV int4 gload(const int4* p, int q) {
  typedef int v4i __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(1))) const v4i* gv4p;
  const v4i t = ((gv4p)p)[q];
  return make_int4(t.x, t.y, t.z, t.w);
}
CG_DEV void fetch_slot(const LaneTab& lt, int p, uint32_t k, RawEntry& r) {
  const int4* src = k ? lt.entry(p * kSlotsPerPoint + k - 1) : g_ident_entry;
  CG_UNROLL for (int q = 0; q < kTabLimbs / 4; ++q) r.q[q] = gload(src, q);
}
CG_DEV void load_entry(const int4* src, ge_cached& c) {
  RawEntry r;
  CG_UNROLL for (int q = 0; q < kTabLimbs / 4; ++q) r.q[q] = gload(src, q);
  unpack_entry(r, c);
}
CG_DEV void load_slot(const LaneTab& lt, int p, uint32_t k, ge_cached& c) {
  load_entry(k ? lt.entry(p * kSlotsPerPoint + k - 1) : g_ident_entry, c);
}

#ifndef CG_POINTS_WAVES
#define CG_POINTS_WAVES 2
#endif
// Inputs: word w of element i at pk[i * pk_es + w * pk_ws] (and sig likewise): the staged
// SoA arrays (es 1, ws cap) or the raw rows of a one-chunk call (es = row stride in words,
// ws 1), which lets the kernel start before the staging kernels (Ed25519Dev::pk_rows).
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(CG_POINTS_WAVES, 8))) void cg_ed25519_points(
    const uint32_t* __restrict__ pk, const uint32_t* __restrict__ sig, uint32_t n, uint32_t pk_es, uint32_t pk_ws,
    uint32_t sig_es, uint32_t sig_ws, uint32_t scap, uint32_t* __restrict__ pstat, int32_t* __restrict__ table) {
  CG_WAVE_PRIO(1);
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t pkw[8], rw[8];
  CG_UNROLL for (int w = 0; w < 8; ++w) {
    pkw[w] = pk[(size_t)i * pk_es + (size_t)w * pk_ws];
    rw[w] = sig[(size_t)i * sig_es + (size_t)w * sig_ws];
  }
  // independent of the hash kernel (it may run beside it): the points verdict alone
  // (KEY_INVALID / REJECT for a bad R / COMPUTE); the MSM merges it with the hash's
  ge_p3 negA, R;
  const uint32_t v = ed25519_points_stage(pkw, rw, V_COMPUTE, negA, R);
  pstat[i] = v;
  if (v != V_COMPUTE) return;
  const LaneTab lt = lane_table(table, i, scap);
  ed25519_build_table(negA, [&](int k, const ge_cached& c) { store_slot(lt, 0, k, c); });
  ed25519_build_table(R, [&](int k, const ge_cached& c) { store_slot(lt, 1, k, c); });
}

// The points phase in two halves (one-chunk host-buffer calls: the key rows land before
// the signature rows, so the A half runs beside the signatures' copy): HALF 0 decodes -A
// into point 0 of lane slot i and writes pstat[i] (KEY_INVALID / COMPUTE); HALF 1, ordered
// after it on the same stream, decodes R (strict) into point 1 unless the key already
// failed and writes REJECT / COMPUTE — together the verdict and tables of
// ed25519_points_stage.  rows: word w of element i at rows[i * es + w].
template <int HALF>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(CG_POINTS_WAVES, 8))) void cg_ed25519_points_half(
    const uint32_t* __restrict__ rows, uint32_t n, uint32_t es, uint32_t scap, uint32_t* __restrict__ pstat,
    int32_t* __restrict__ table) {
  CG_WAVE_PRIO(1);
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (HALF == 1 && pstat[i] != V_COMPUTE) return;
  uint32_t w[8];
  CG_UNROLL for (int k = 0; k < 8; ++k) w[k] = rows[(size_t)i * es + k];
  ge_p3 P;
  uint32_t ok = ge_frombytes_i2p(P, w);
  if (HALF == 1) {
    ok = ok && ge_strict_check(P, w);
  } else {
    fe_neg_p(P.X, P.X);  // -A kept floor-shaped, as ed25519_points_stage
    fe_neg_p(P.T, P.T);
  }
  pstat[i] = ok ? V_COMPUTE : HALF ? V_REJECT : V_KEY_INVALID;
  if (!ok) return;
  const LaneTab lt = lane_table(table, i, scap);
  ed25519_build_table(P, [&](int k, const ge_cached& c) { store_slot(lt, HALF, k, c); });
}

// Key-reuse path, once per distinct key and verify call: decode A and build its
// four tables k * 2^(64 t) (-A) (lane-contiguous, kKeyEntries entries per key).
constexpr int kKeyEntries = 4 * kATabEntries;
CG_DEV int4* key_table(int32_t* ktab, uint32_t j) {
  return reinterpret_cast<int4*>(ktab + (size_t)j * (kKeyEntries * kTabLimbs));
}
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(CG_POINTS_WAVES, 8))) void cg_ed25519_keyprep(
    const uint32_t* __restrict__ pk, uint32_t cap, const uint32_t* __restrict__ key_first, uint32_t n_keys,
    int32_t* __restrict__ ktab, uint32_t* __restrict__ kstat) {
  // the longest chain of the key-reuse path (decode + 192 doublings per key, few
  // blocks) and the points / MSM kernels wait for it: above the hash kernel beside it
  CG_WAVE_PRIO(3);
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_keys) return;
  const uint32_t e = key_first[j];
  uint32_t pkw[8];
  CG_UNROLL for (int w = 0; w < 8; ++w) pkw[w] = pk[(size_t)w * cap + e];
  int4* kt = key_table(ktab, j);
  kstat[j] = ed25519_key_tables(pkw, [&](int t, int k, const ge_cached& c) CG_LINLINE {
    store_cached(kt + (t * kATabEntries + k) * (kTabLimbs / 4), c);
  });
}

// Key-reuse path, per signature: decode R only (the key's verdict comes from its
// distinct-key slot) and build k*R in the lane table.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(CG_POINTS_WAVES, 8))) void cg_ed25519_points_r(
    const uint32_t* __restrict__ sig, uint32_t n, uint32_t cap, uint32_t scap, const uint32_t* __restrict__ key_index,
    const uint32_t* __restrict__ kstat, uint32_t* __restrict__ pstat, int32_t* __restrict__ table) {
  CG_WAVE_PRIO(1);
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t rw[8];
  CG_UNROLL for (int w = 0; w < 8; ++w) rw[w] = sig[(size_t)w * cap + i];
  ge_p3 R;
  const uint32_t v = ed25519_points_stage_r(rw, V_COMPUTE, kstat[key_index[i]], R);
  pstat[i] = v;
  if (v != V_COMPUTE) return;
  const LaneTab lt = lane_table(table, i, scap);
  ed25519_build_table(R, [&](int k, const ge_cached& c) { store_slot(lt, 0, k, c); });
}

// The shared B tables: entry k of table s = k * 2^(32 s) B in affine form, s = 0..7,
// one lane per entry (8 * (2^(kBWin-1) + 1) lanes), at context creation.
__global__ __launch_bounds__(256) void cg_ed25519_btab_build(int32_t* __restrict__ btab) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= kBTables * (uint32_t)kBTabEntries) return;
  ge_precomp e;
  ed25519_btab_entry(e, i / kBTabEntries, i % kBTabEntries);  // table s = k * 2^(32 s) B
  int32_t* o = btab + (size_t)i * kBStride;
  CG_UNROLL for (int l = 0; l < 10; ++l) {
    o[l] = e.yplusx.v[l];
    o[10 + l] = e.yminusx.v[l];
    o[20 + l] = e.xy2d.v[l];
  }
  o[30] = o[31] = 0;
}

// The element's verdict from the hash phase's status word and the points phase's
// verdict (ed25519_points_stage precedence: KEY_INVALID first, then the hash phase's
// pre-verdict, then a bad R); V_COMPUTE: the MSM decides.
CG_DEV uint32_t ed_merge_verdict(uint32_t st, uint32_t pv) {
  const uint32_t vh = ed_status_verdict(st);
  return pv == V_KEY_INVALID ? pv : vh != V_COMPUTE ? vh : pv;
}

CG_DEV uint32_t wave_max(uint32_t v) {
  CG_UNROLL for (int o = 32; o >= 1; o >>= 1) {
    const uint32_t u = (uint32_t)__shfl_xor((int)v, o, 64);
    v = u > v ? u : v;
  }
  return v;
}

CG_DEV void load_bentry(const int32_t* btab_g, uint32_t t, uint32_t k, ge_precomp& p) {
  // one 128-byte line per entry: eight 16-byte loads (L2 / MALL resident table)
  const int4* b = reinterpret_cast<const int4*>(btab_g + ((size_t)t * kBTabEntries + k) * kBStride);
  int32_t v[kBStride];
  CG_UNROLL for (int q = 0; q < kBStride / 4; ++q) {
    const int4 x = b[q];
    v[4 * q] = x.x;
    v[4 * q + 1] = x.y;
    v[4 * q + 2] = x.z;
    v[4 * q + 3] = x.w;
  }
  CG_UNROLL for (int l = 0; l < 10; ++l) {
    p.yplusx.v[l] = v[l];
    p.yminusx.v[l] = v[10 + l];
    p.xy2d.v[l] = v[20 + l];
  }
}

// Staging of the lane-table entries in the MSM loop (ed25519_msm's loadX / unpackX): the
// A entry's packed words are fetched before a window's doublings and held across them;
// the R entry is loaded just before its addition.  (Round 4 also staged them through
// LDS by LDS-DMA — 3 waves / SIMD without spills — and measured no gain; removed.)
struct LateSlot {
  uint32_t k;
};

CG_DEV uint32_t msm_lane(uint32_t ndig, const uint32_t* dig, uint32_t scap, uint32_t rneg, const LaneTab& lt,
                         const int32_t* btab_g) {
  auto getDig = [&](int w) CG_LINLINE { return dig[(size_t)w * scap]; };
  auto getB = [&](uint32_t t, uint32_t k, ge_precomp& p) CG_LINLINE { load_bentry(btab_g, t, k, p); };
  auto loadA = [&](uint32_t k, RawEntry& r) CG_LINLINE { fetch_slot(lt, 0, k, r); };
  auto unpackA = [&](const RawEntry& r, ge_cached& c) CG_LINLINE { unpack_entry(r, c); };
  auto loadR = [&](uint32_t k, LateSlot& r) CG_LINLINE { r.k = k; };
  auto unpackR = [&](LateSlot& r, ge_cached& c) CG_LINLINE { load_slot(lt, 1, r.k, c); };
  return ed25519_msm<RawEntry, LateSlot>(ndig, getDig, rneg, loadA, unpackA, loadR, unpackR, getB);
}

// Lane j of a grouped MSM (order != null): the classes' lanes back to back (class 0, the
// longest, dispatched first), from the counts the bucket kernel left; past the last class
// the lane has nothing to do (its verdict, if any, the bucket kernel wrote).
CG_DEV uint32_t grouped_lane(uint32_t j, const uint32_t* __restrict__ order, const uint32_t* __restrict__ count,
                             uint32_t scap, bool& in) {
  const uint32_t n0 = count[3], n01 = n0 + count[7], all = n01 + count[11];  // cg_ed25519_bucket_scatter
  in = j < all;
  const size_t k = j < n0 ? j : j < n01 ? (size_t)scap + (j - n0) : 2 * (size_t)scap + (j - n01);
  return in ? order[k] : 0u;
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(CG_MSM_WAVES, CG_MSM_WAVES))) void cg_ed25519_msm(
    const uint32_t* __restrict__ status, const uint32_t* __restrict__ pstat, const uint32_t* __restrict__ digits,
    const int32_t* __restrict__ table, const int32_t* __restrict__ btab_g, uint32_t n, uint32_t scap,
    const uint32_t* __restrict__ order, const uint32_t* __restrict__ order_count,
    const uint32_t* __restrict__ out_index, uint8_t* __restrict__ verdict) {
  CG_WAVE_PRIO(0);
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  bool in = j < n;
  const uint32_t i = order ? grouped_lane(j, order, order_count, scap, in) : j;
  const uint32_t st = in ? status[i] : 0u;
  const uint32_t v = in ? ed_merge_verdict(st, pstat[i]) : 0u;
  const bool live = in && v == V_COMPUTE;
  // every lane of the wave walks the same bit positions: the longest scalar sets the length
  const uint32_t ndig = wave_max(live ? ed_status_ndig(st) : 0u);
  if (!in) return;
  const uint32_t dst = out_index ? out_index[i] : i;
  if (!live) {
    verdict[dst] = (uint8_t)v;
    return;
  }
  const uint32_t* dig = digits + i;
  const LaneTab lt = lane_table(const_cast<int32_t*>(table), i, scap);
  const uint32_t ok = msm_lane(ndig, dig, scap, ed_status_rneg(st), lt, btab_g);
  verdict[dst] = ok ? (uint8_t)V_ACCEPT : (uint8_t)V_REJECT;
}

// Lanes grouped by digit count for the balanced MSM (round 6).  The MSM's loop length is
// the wave's largest digit count; in index order ~23 % of waves hold one of the 0.4 % of
// lanes with 34 digits and none runs fewer than 33 (32 for 34 % of lanes): grouping cuts
// the windows per lane from 33.2 to 32.7 (profiles/r06_digit_hist.json).  Two passes
// over 1,024-lane blocks, no atomics (a first version appended every wave's lanes with
// one atomicAdd per wave and class on three words: +0.6 ms per 1 M, r06a), and the order
// within a class is the index order:
//   cg_ed25519_bucket_count    lanes the MSM need not run (hash or points verdict final)
//                              get their verdict; the block's class sizes -> blk[4 b + c]
//   cg_ed25519_bucket_scatter  block b sums the sizes of blocks < b (at most a few
//                              thousand words), places its live lanes in their classes;
//                              the last block writes the class totals to blk[4 c + 3]
// Class of a lane: 0 >= 34 digits, 1: 33, 2: 32, 3: not live.
constexpr uint32_t kBucketBlock = 1024;
CG_DEV uint32_t bucket_class(const uint32_t* __restrict__ status, const uint32_t* __restrict__ pstat, uint32_t i,
                             uint32_t n, uint32_t& v) {
  const bool in = i < n;
  const uint32_t st = in ? status[i] : 0u;
  v = in ? ed_merge_verdict(st, pstat[i]) : 0u;
  const uint32_t nd = ed_status_ndig(st);
  return !(in && v == V_COMPUTE) ? 3u : nd >= 34u ? 0u : nd == 33u ? 1u : 2u;
}

__global__ __launch_bounds__(kBucketBlock) void cg_ed25519_bucket_count(const uint32_t* __restrict__ status,
                                                                        const uint32_t* __restrict__ pstat, uint32_t n,
                                                                        uint32_t* __restrict__ blk,
                                                                        const uint32_t* __restrict__ out_index,
                                                                        uint8_t* __restrict__ verdict) {
  CG_WAVE_PRIO(1);
  __shared__ uint32_t part[kBucketBlock / 64][3];
  const uint32_t i = blockIdx.x * kBucketBlock + threadIdx.x, wv = threadIdx.x / 64;
  uint32_t v;
  const uint32_t cls = bucket_class(status, pstat, i, n, v);
  if (i < n && cls == 3u) verdict[out_index ? out_index[i] : i] = (uint8_t)v;
  CG_UNROLL for (uint32_t c = 0; c < 3; ++c) {
    const uint32_t k = (uint32_t)__popcll(__ballot(cls == c));
    if ((threadIdx.x & 63u) == 0) part[wv][c] = k;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    uint32_t t = 0;
    CG_UNROLL for (uint32_t w = 0; w < kBucketBlock / 64; ++w) t += part[w][threadIdx.x];
    blk[4 * blockIdx.x + threadIdx.x] = t;
  }
}

__global__ __launch_bounds__(kBucketBlock) void cg_ed25519_bucket_scatter(const uint32_t* __restrict__ status,
                                                                          const uint32_t* __restrict__ pstat,
                                                                          uint32_t n, uint32_t scap,
                                                                          uint32_t* __restrict__ blk,
                                                                          uint32_t* __restrict__ order) {
  CG_WAVE_PRIO(1);
  __shared__ uint32_t part[kBucketBlock / 64][3];
  __shared__ uint32_t base[3];
  const uint32_t b = blockIdx.x, wv = threadIdx.x / 64, lane = threadIdx.x & 63u;
  // this block's class offsets: the sizes of the blocks before it (the last block also
  // adds its own: the totals the MSM reads)
  const uint32_t upto = b + 1 == gridDim.x ? b + 1 : b;
  uint32_t s[3] = {0, 0, 0};
  for (uint32_t k = threadIdx.x; k < upto; k += kBucketBlock)
    CG_UNROLL for (uint32_t c = 0; c < 3; ++c) s[c] += blk[4 * k + c];
  CG_UNROLL for (uint32_t c = 0; c < 3; ++c) {
    CG_UNROLL for (int o = 32; o >= 1; o >>= 1) s[c] += (uint32_t)__shfl_xor((int)s[c], o, 64);
    if (lane == 0) part[wv][c] = s[c];
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    uint32_t t = 0;
    CG_UNROLL for (uint32_t w = 0; w < kBucketBlock / 64; ++w) t += part[w][threadIdx.x];
    if (b + 1 == gridDim.x) {  // totals, then back to this block's own offsets
      blk[4 * threadIdx.x + 3] = t;
      t -= blk[4 * b + threadIdx.x];
    }
    base[threadIdx.x] = t;
  }
  __syncthreads();
  const uint32_t i = b * kBucketBlock + threadIdx.x;
  uint32_t v;
  const uint32_t cls = bucket_class(status, pstat, i, n, v);
  const uint64_t below = lane ? (~0ull >> (64u - lane)) : 0ull;
  uint64_t m[3];
  CG_UNROLL for (uint32_t c = 0; c < 3; ++c) {
    m[c] = __ballot(cls == c);
    if (lane == 0) part[wv][c] = (uint32_t)__popcll(m[c]);
  }
  __syncthreads();
  if (cls < 3u) {
    uint32_t off = base[cls];
    for (uint32_t w = 0; w < wv; ++w) off += part[w][cls];
    order[(size_t)cls * scap + off + (uint32_t)__popcll(m[cls] & below)] = i;
  }
}

// ---------------------------------------------------------------- latency mode
// Small batches (a notary's request queue: ValidatingNotaryFlow.kt:34-40) leave most
// SIMDs idle and each signature's dependent chain sets the call's time, so the points
// and MSM phases run with LANES = 2 or 4 lanes per signature (lanes LANES i + q):
//   cg_ed25519_points_lanes  lane q decodes one point — half h = q (LANES 2) or q / 2
//                            (LANES 4): h = 0 A -> -A, KEY_INVALID when it has no root;
//                            h = 1 R, strict, REJECT — takes it to 2^64 P in the odd
//                            lanes of LANES 4 (64 doublings), and builds its eight
//                            table entries; its verdict byte goes to byte q of pstat[i]
//                            (the lanes store different bytes of the word).  Tables:
//                            LANES 2 in lane slot i (points -A, R), LANES 4 in slots
//                            2i (-A, 2^64 (-A)) and 2i + 1 (R, 2^64 R): 2n slots.
//   cg_ed25519_msm_lanes     lane q runs ed25519_msm_lane<LANES> (LANES 2: q = 0
//                            [c0](-A) + [b_lo]B, q = 1 [c1](+-R) + [b_hi] 2^128 B; LANES
//                            4 each of those over the scalars' 64-bit halves) over the
//                            shared window positions; the partial sums meet through
//                            lane swaps (ed25519_lane_sum, ed25519_pair_combine), lane 0
//                            writes the verdict
// Per signature ~1.4x (2 lanes) / ~1.7x (4 lanes) the MSM work of cg_ed25519_msm, on a
// chain ~30 % / ~60 % shorter.
#ifndef CG_PAIR_WAVES
#define CG_PAIR_WAVES 2
#endif
// Lane q of signature i: its half h, part u, and where its table lives (scratch slot,
// point 0 / 1 of the slot): LANES 2 slot i, point h; LANES 4 / 8 slot P i + (P / 2) h +
// u / 2, point u % 2 (P = LANES / 2: the signature's 2 P tables in P slots).
template <int LANES>
struct LaneOf {
  static constexpr uint32_t P = LANES / 2;
  uint32_t h, u, slot;
  int point;
  CG_DEV LaneOf(uint32_t i, uint32_t q) : h(q / P), u(q % P) {
    slot = LANES == 2 ? i : P * i + (P / 2) * h + u / 2;
    point = LANES == 2 ? (int)h : (int)(u & 1);
  }
};

template <int LANES>
// Inputs: word k of element i at pk[i * pk_es + k * pk_ws] (and sig likewise): the staged
// SoA arrays (es 1, ws cap) or the raw rows (es = the row stride in words, ws 1).
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(CG_POINTS_WAVES, 8))) void cg_ed25519_points_lanes(
    const uint32_t* __restrict__ pk, const uint32_t* __restrict__ sig, uint32_t n, uint32_t pk_es, uint32_t pk_ws,
    uint32_t sig_es, uint32_t sig_ws, uint32_t scap, uint32_t* __restrict__ pstat, int32_t* __restrict__ table) {
  CG_WAVE_PRIO(1);
  const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t i = l / LANES, q = l % LANES;
  const LaneOf<LANES> lo(i, q);
  if (i >= n) return;
  const uint32_t* src = lo.h ? sig + (size_t)i * sig_es : pk + (size_t)i * pk_es;  // R: words 0..7 of the signature
  const uint32_t ws = lo.h ? sig_ws : pk_ws;
  uint32_t w[8];
  CG_UNROLL for (int k = 0; k < 8; ++k) w[k] = src[(size_t)k * ws];
  ge_p3 P;
  uint32_t ok = ge_frombytes_i2p(P, w);
  if (lo.h) {
    ok = ok && ge_strict_check(P, w);
  } else {
    fe_neg_p(P.X, P.X);  // -A kept floor-shaped, as ed25519_points_stage
    fe_neg_p(P.T, P.T);
  }
  // verdict bytes: LANES 2 / 4 byte q (A in bytes 0 (and 1), R in byte 1 / 2 (and 3));
  // LANES 8 only the part-0 lanes, bytes 0 and 2
  if (LANES != 8 || lo.u == 0)
    reinterpret_cast<uint8_t*>(pstat)[4 * (size_t)i + (LANES == 8 ? 2 * lo.h : q)] =
        (uint8_t)(ok ? V_COMPUTE : lo.h ? V_REJECT : V_KEY_INVALID);
  if (!ok) return;
  if (lo.u) ge_p3_dbl_n(P, 4 * (32 / LaneOf<LANES>::P) * lo.u);  // 2^(4 u D) P
  const LaneTab lt = lane_table(table, lo.slot, scap);
  ed25519_build_table(P, [&](int k, const ge_cached& c) { store_slot(lt, lo.point, k, c); });
}

template <int LANES>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(CG_PAIR_WAVES, CG_PAIR_WAVES))) void cg_ed25519_msm_lanes(
    const uint32_t* __restrict__ status, const uint32_t* __restrict__ pstat, const uint32_t* __restrict__ digits,
    const int32_t* __restrict__ table, const int32_t* __restrict__ btab_g, uint32_t n, uint32_t scap,
    const uint32_t* __restrict__ out_index, uint8_t* __restrict__ verdict) {
  CG_WAVE_PRIO(0);
  const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t i = l / LANES, q = l % LANES;
  const LaneOf<LANES> lo(i, q);
  const bool in = i < n;
  const uint32_t st = in ? status[i] : 0u;
  const uint32_t pw = in ? pstat[i] : 0u;
  // ed25519_points_stage precedence: A's KEY_INVALID first, then (after the hash
  // phase's verdict, ed_merge_verdict) R's REJECT (byte 1 / byte 2 for LANES 2 / 4, 8)
  const uint32_t pa = pw & 0xff, pr = (pw >> (LANES == 2 ? 8 : 16)) & 0xff;
  const uint32_t v = in ? ed_merge_verdict(st, pa != V_COMPUTE ? pa : pr) : 0u;
  const bool live = in && v == V_COMPUTE;
  const uint32_t ndig = wave_max(live ? ed_status_ndig(st) : 0u);
  if (!in) return;
  const uint32_t dst = out_index ? out_index[i] : i;
  if (!live) {  // every lane of a signature takes the same branch
    if (q == 0) verdict[dst] = (uint8_t)v;
    return;
  }
  const uint32_t* dig = digits + i;
  const LaneTab lt = lane_table(const_cast<int32_t*>(table), lo.slot, scap);
  ge_p1p1 t;
  ed25519_msm_lane<RawEntry, LANES>(
      t, ndig, q, [&](int w) CG_LINLINE { return dig[(size_t)w * scap]; }, lo.h ? ed_status_rneg(st) : 0u,
      [&](uint32_t k, RawEntry& r) CG_LINLINE { fetch_slot(lt, lo.point, k, r); },
      [&](const RawEntry& r, ge_cached& c) CG_LINLINE { unpack_entry(r, c); },
      [&](uint32_t tb, uint32_t k, ge_precomp& p) CG_LINLINE { load_bentry(btab_g, tb, k, p); });
  // the partial sums meet in log2(LANES) swaps, the last one with the identity test
  CG_UNROLL for (int m = 1; m < LANES / 2; m *= 2)
    ed25519_lane_sum(t, [&](fe& x) CG_LINLINE {
      CG_UNROLL for (int k = 0; k < 10; ++k) x.v[k] = __shfl_xor(x.v[k], m, 64);
    });
  const uint32_t ok = ed25519_pair_combine(t, [&](fe& x) CG_LINLINE {
    CG_UNROLL for (int k = 0; k < 10; ++k) x.v[k] = __shfl_xor(x.v[k], LANES / 2, 64);
  });
  if (q == 0) verdict[dst] = ok ? (uint8_t)V_ACCEPT : (uint8_t)V_REJECT;
}

CG_DEV uint32_t wave_or(uint32_t v) { return __ballot(v != 0) != 0ull; }

// MSM of the key-reuse split (cg_ed25519.h ed25519_msm_reuse): per-key A tables,
// per-lane R table, four shared B tables; 60 doublings.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(CG_MSM_R_WAVES, CG_MSM_R_WAVES))) void cg_ed25519_msm_r(
    const uint32_t* __restrict__ status, const uint32_t* __restrict__ pstat, const uint32_t* __restrict__ digits,
    const int32_t* __restrict__ table, const int32_t* __restrict__ ktab, const uint32_t* __restrict__ key_index,
    const int32_t* __restrict__ btab_g, uint32_t n, uint32_t scap, const uint32_t* __restrict__ out_index,
    uint8_t* __restrict__ verdict) {
  CG_WAVE_PRIO(0);
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t st = i < n ? status[i] : 0u;
  const uint32_t v = i < n ? ed_merge_verdict(st, pstat[i]) : 0u;
  const bool live = i < n && v == V_COMPUTE;
  // wave-uniform loop shape: the most chunk-3 windows and a 17th c1 digit in any lane
  const uint32_t shape = live ? ed_status_ndig(st) : 0u;
  const uint32_t c3w = wave_max(shape & 31u), win17 = wave_or(shape >> 5);
  if (i >= n) return;
  const uint32_t dst = out_index ? out_index[i] : i;
  if (!live) {
    verdict[dst] = (uint8_t)v;
    return;
  }
  uint32_t dig[kDigitWords];
  CG_UNROLL for (int w = 0; w < kDigitWords; ++w) dig[w] = digits[(size_t)w * scap + i];
  const LaneTab lt = lane_table(const_cast<int32_t*>(table), i, scap);
  const int4* kt = key_table(const_cast<int32_t*>(ktab), key_index[i]);
  const uint32_t ok = ed25519_msm_reuse(
      c3w, win17, dig, ed_status_rneg(st),
      [&](uint32_t t, uint32_t k, ge_cached& c) CG_LINLINE {
        load_entry(kt + (t * kATabEntries + k) * (kTabLimbs / 4), c);
      },
      [&](uint32_t k, ge_cached& c) CG_LINLINE { load_slot(lt, 0, k, c); },
      [&](uint32_t t, uint32_t k, ge_precomp& p) CG_LINLINE { load_bentry(btab_g, t, k, p); });
  verdict[dst] = ok ? (uint8_t)V_ACCEPT : (uint8_t)V_REJECT;
}

}  // namespace

namespace cg {

size_t ed25519_table_bytes(uint32_t scap) { return (size_t)kLaneEntries * kTabLimbs * scap * sizeof(int32_t); }
size_t ed25519_table_offset(uint32_t lanes) {  // int32 offset of lane `lanes` (the base of a sub-range's view)
  return (size_t)kLaneEntries * kTabLimbs * lanes;
}
size_t ed25519_digit_words() { return kDigitWords; }
size_t ed25519_btab_words() { return (size_t)kBTables * kBTabEntries * kBStride; }
size_t ed25519_key_table_bytes(uint32_t n_keys) { return (size_t)kKeyEntries * kTabLimbs * n_keys * sizeof(int32_t); }

hipError_t launch_ed25519_btab_build(int32_t* btab, hipStream_t s) {
  const uint32_t n = kBTables * kBTabEntries;
  hipLaunchKernelGGL(cg_ed25519_btab_build, dim3((n + 255) / 256), dim3(256), 0, s, btab);
  return hipGetLastError();
}

hipError_t launch_ed25519_hash(const Ed25519Dev& d, uint32_t n, uint32_t mode, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (d.key_index)
    hipLaunchKernelGGL(cg_ed25519_hash<true>, dim3((n + 255) / 256), dim3(256), 0, s, d.pk, d.sig, d.sig_len, d.arena,
                       d.msg_off, d.msg_len, n, d.cap, d.scap, mode, d.status, d.digits, d.full_mod, d.index_base);
  else
    hipLaunchKernelGGL(cg_ed25519_hash<false>, dim3((n + 255) / 256), dim3(256), d.spread_lds_hash, s, d.pk, d.sig, d.sig_len,
                       d.arena, d.msg_off, d.msg_len, n, d.cap, d.scap, mode, d.status, d.digits, d.full_mod,
                       d.index_base);
  return hipGetLastError();
}

hipError_t launch_ed25519_keyprep(const Ed25519Dev& d, const uint32_t* key_first, uint32_t n_keys, hipStream_t s) {
  if (n_keys == 0) return hipSuccess;
  hipLaunchKernelGGL(cg_ed25519_keyprep, dim3((n_keys + 255) / 256), dim3(256), 0, s, d.pk, d.cap, key_first, n_keys,
                     const_cast<int32_t*>(d.ktab), const_cast<uint32_t*>(d.kstat));
  return hipGetLastError();
}

hipError_t launch_ed25519_points_half(const Ed25519Dev& d, int half, uint32_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (half == 0)
    hipLaunchKernelGGL(cg_ed25519_points_half<0>, dim3((n + 255) / 256), dim3(256), 0, s, d.pk_rows, n,
                       d.pk_row_words, d.scap, d.pstat, d.table);
  else
    hipLaunchKernelGGL(cg_ed25519_points_half<1>, dim3((n + 255) / 256), dim3(256), 0, s, d.sig_rows, n,
                       d.sig_row_words, d.scap, d.pstat, d.table);
  return hipGetLastError();
}

hipError_t launch_ed25519_points(const Ed25519Dev& d, uint32_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (d.key_index)
    hipLaunchKernelGGL(cg_ed25519_points_r, dim3((n + 255) / 256), dim3(256), 0, s, d.sig, n, d.cap, d.scap,
                       d.key_index, d.kstat, d.pstat, d.table);
  else if (d.pk_rows && d.sig_rows)
    hipLaunchKernelGGL(cg_ed25519_points, dim3((n + 255) / 256), dim3(256), 0, s, d.pk_rows, d.sig_rows, n,
                       d.pk_row_words, 1u, d.sig_row_words, 1u, d.scap, d.pstat, d.table);
  else
    hipLaunchKernelGGL(cg_ed25519_points, dim3((n + 255) / 256), dim3(256), 0, s, d.pk, d.sig, n, 1u, d.cap, 1u, d.cap,
                       d.scap, d.pstat, d.table);
  return hipGetLastError();
}

hipError_t launch_ed25519_points_lanes(const Ed25519Dev& d, uint32_t n, uint32_t lanes, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (lanes != 2 && lanes != 4 && lanes != 8) return hipErrorInvalidValue;
  // four / eight lanes: tables in scratch slots [0, lanes / 2 n) of this view (the caller sized scap for it)
  if (lanes > 2 && (uint64_t)lanes / 2 * n > d.scap) return hipErrorInvalidValue;
  const dim3 grid((uint32_t)(((uint64_t)lanes * n + 255) / 256));
  const bool rows = d.pk_rows && d.sig_rows;
  const uint32_t* pk = rows ? d.pk_rows : d.pk;
  const uint32_t* sig = rows ? d.sig_rows : d.sig;
  const uint32_t pk_es = rows ? d.pk_row_words : 1u, pk_ws = rows ? 1u : d.cap;
  const uint32_t sig_es = rows ? d.sig_row_words : 1u, sig_ws = rows ? 1u : d.cap;
  if (lanes == 8)
    hipLaunchKernelGGL(cg_ed25519_points_lanes<8>, grid, dim3(256), d.spread_lds, s, pk, sig, n, pk_es, pk_ws, sig_es,
                       sig_ws, d.scap, d.pstat, d.table);
  else if (lanes == 4)
    hipLaunchKernelGGL(cg_ed25519_points_lanes<4>, grid, dim3(256), d.spread_lds, s, pk, sig, n, pk_es, pk_ws, sig_es,
                       sig_ws, d.scap, d.pstat, d.table);
  else
    hipLaunchKernelGGL(cg_ed25519_points_lanes<2>, grid, dim3(256), d.spread_lds, s, pk, sig, n, pk_es, pk_ws, sig_es,
                       sig_ws, d.scap, d.pstat, d.table);
  return hipGetLastError();
}

hipError_t launch_ed25519_msm_lanes(const Ed25519Dev& d, uint32_t n, uint32_t lanes, const uint32_t* out_index,
                                    uint8_t* verdict, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (lanes != 2 && lanes != 4 && lanes != 8) return hipErrorInvalidValue;
  if (lanes > 2 && (uint64_t)lanes / 2 * n > d.scap) return hipErrorInvalidValue;
  const dim3 grid((uint32_t)(((uint64_t)lanes * n + 255) / 256));
  if (lanes == 8)
    hipLaunchKernelGGL(cg_ed25519_msm_lanes<8>, grid, dim3(256), 0, s, d.status, d.pstat, d.digits, d.table, d.btab, n,
                       d.scap, out_index, verdict);
  else if (lanes == 4)
    hipLaunchKernelGGL(cg_ed25519_msm_lanes<4>, grid, dim3(256), 0, s, d.status, d.pstat, d.digits, d.table, d.btab, n,
                       d.scap, out_index, verdict);
  else
    hipLaunchKernelGGL(cg_ed25519_msm_lanes<2>, grid, dim3(256), 0, s, d.status, d.pstat, d.digits, d.table, d.btab, n,
                       d.scap, out_index, verdict);
  return hipGetLastError();
}

hipError_t launch_ed25519_msm(const Ed25519Dev& d, uint32_t n, const uint32_t* out_index, uint8_t* verdict,
                              hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (d.key_index)
    hipLaunchKernelGGL(cg_ed25519_msm_r, dim3((n + 255) / 256), dim3(256), 0, s, d.status, d.pstat, d.digits, d.table,
                       d.ktab, d.key_index, d.btab, n, d.scap, out_index, verdict);
  else
    hipLaunchKernelGGL(cg_ed25519_msm, dim3((n + 255) / 256), dim3(256), 0, s, d.status, d.pstat, d.digits, d.table,
                       d.btab, n, d.scap, d.order, d.order_count, out_index, verdict);
  return hipGetLastError();
}

hipError_t launch_ed25519_bucket(const Ed25519Dev& d, uint32_t n, const uint32_t* out_index, uint8_t* verdict,
                                 hipStream_t s) {
  // the class totals live in the 4th words of the first three block entries
  if (!d.order || !d.order_count || d.key_index || n < 3 * kBucketBlock) return hipErrorInvalidValue;
  const dim3 grid((n + kBucketBlock - 1) / kBucketBlock);
  hipLaunchKernelGGL(cg_ed25519_bucket_count, grid, dim3(kBucketBlock), 0, s, d.status, d.pstat, n, d.order_count,
                     out_index, verdict);
  hipLaunchKernelGGL(cg_ed25519_bucket_scatter, grid, dim3(kBucketBlock), 0, s, d.status, d.pstat, n, d.scap,
                     d.order_count, d.order);
  return hipGetLastError();
}

}  // namespace cg
