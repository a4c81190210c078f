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
//  * no CPU fallback: without a gfx950 device cg_open fails.
#include "cordagpu.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>
#include <cstdio>
#include <cstring>
#include <map>
#include <new>
#include <string>
#include <vector>

#include "cg_kernels.h"
#include "cg_ecdsa_api.h"
#include "cg_merkle_api.h"

namespace {

constexpr uint32_t kEdChunk = 1u << 21;  // Ed25519 scratch chunk (elements)

struct Stat {
  double ms = 0;
  uint64_t launches = 0;
  uint64_t items = 0;
};

}  // namespace

struct cg_ctx {
  int device = -1;
  hipStream_t stream = nullptr;
  std::string err;
  int32_t* btab = nullptr;
  // Ed25519 chunk scratch
  uint32_t ed_scap = 0;
  uint32_t* ed_status = nullptr;
  uint32_t* ed_digits = nullptr;
  int32_t* ed_table = nullptr;
  bool profiling = false;
  std::map<std::string, Stat> stats;
  std::vector<std::pair<std::string, std::pair<hipEvent_t, hipEvent_t>>> pending;
  std::vector<hipEvent_t> event_pool;
  cg::EcdsaConsts* ec = nullptr;
};

namespace {

struct DevMem {
  void* p = nullptr;
  size_t bytes = 0;
};

cg_status fail(cg_ctx* ctx, cg_status code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  return code;
}

cg_status hip_fail(cg_ctx* ctx, hipError_t e, const char* what) {
  std::string m = std::string(what) + ": " + hipGetErrorString(e);
  (void)hipGetLastError();
  return fail(ctx, e == hipErrorOutOfMemory ? CG_E_OUT_OF_MEMORY : CG_E_DEVICE, m);
}

#define CG_TRY(ctx, expr, what)                      \
  do {                                               \
    hipError_t e_ = (expr);                          \
    if (e_ != hipSuccess) return hip_fail(ctx, e_, what); \
  } while (0)

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

// RAII timing scope around one kernel launch on the context stream.
struct Timed {
  cg_ctx* ctx;
  const char* name;
  uint64_t items;
  hipEvent_t a = nullptr, b = nullptr;
  Timed(cg_ctx* c, const char* n, uint64_t it) : ctx(c), name(n), items(it) {
    if (ctx->profiling) {
      a = take_event(ctx);
      b = take_event(ctx);
      if (a) (void)hipEventRecord(a, ctx->stream);
    }
  }
  ~Timed() {
    if (ctx->profiling && a && b) {
      (void)hipEventRecord(b, ctx->stream);
      ctx->pending.push_back({name, {a, b}});
      ctx->stats[name].items += items;
    }
  }
};

void collect_timings(cg_ctx* ctx) {
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

template <typename T>
cg_status dalloc(cg_ctx* ctx, T** p, size_t count, const char* what) {
  *p = nullptr;
  if (count == 0) count = 1;
  hipError_t e = hipMalloc((void**)p, count * sizeof(T));
  if (e != hipSuccess) return hip_fail(ctx, e, what);
  return CG_OK;
}

void dfree(void* p) {
  if (p) (void)hipFree(p);
}

cg_status ensure_ed_scratch(cg_ctx* ctx, uint32_t need) {
  const uint32_t want = std::min(need, kEdChunk);
  if (ctx->ed_scap >= want) return CG_OK;
  dfree(ctx->ed_status);
  dfree(ctx->ed_digits);
  dfree(ctx->ed_table);
  ctx->ed_status = nullptr;
  ctx->ed_digits = nullptr;
  ctx->ed_table = nullptr;
  ctx->ed_scap = 0;
  cg_status st;
  if ((st = dalloc(ctx, &ctx->ed_status, want, "alloc ed25519 status")) != CG_OK) return st;
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
  uint32_t* bitmap = nullptr;   // [ceil(n/32)]
  uint8_t* arena = nullptr;     // message arena (+16 pad)
  bool arena_owned = true;
  uint64_t* msg_off_all = nullptr;
  uint32_t* msg_len_all = nullptr;
  // Ed25519 subset
  uint32_t n_ed = 0;
  uint32_t* ed_index = nullptr;  // null when the subset is the whole batch in order
  uint32_t* ed_pk = nullptr;
  uint32_t* ed_sig = nullptr;
  uint32_t* ed_sig_len = nullptr;
  uint64_t* ed_msg_off = nullptr;
  uint32_t* ed_msg_len = nullptr;
  // ECDSA subsets (K1, R1)
  cg::EcdsaBatch ec[2];
};

namespace {

void batch_free(cg_batch* b) {
  if (!b) return;
  dfree(b->verdict);
  dfree(b->bitmap);
  if (b->arena_owned) dfree(b->arena);
  dfree(b->msg_off_all);
  dfree(b->msg_len_all);
  dfree(b->ed_index);
  dfree(b->ed_pk);
  dfree(b->ed_sig);
  dfree(b->ed_sig_len);
  dfree(b->ed_msg_off);
  dfree(b->ed_msg_len);
  for (auto& e : b->ec) cg::ecdsa_batch_free(e);
  delete b;
}

cg_status check_inputs(cg_ctx* ctx, size_t n, const uint8_t* scheme_id, const uint8_t* pk, size_t pk_stride,
                       const uint8_t* sig, size_t sig_stride, const uint32_t* sig_len, const uint8_t* msg,
                       size_t msg_bytes, const uint64_t* msg_off, const uint32_t* msg_len) {
  if (!ctx) return CG_E_INVALID_ARGUMENT;
  if (n > 0xFFFFFFF0ull) return fail(ctx, CG_E_INVALID_ARGUMENT, "batch larger than 2^32 - 16 elements");
  if (n == 0) return CG_OK;
  if (!pk || !sig || !msg_off || !msg_len) return fail(ctx, CG_E_INVALID_ARGUMENT, "null input pointer");
  if (msg_bytes > 0 && !msg) return fail(ctx, CG_E_INVALID_ARGUMENT, "null message arena");
  bool has_ed = false, has_ec = false;
  for (size_t i = 0; i < n; ++i) {
    const uint8_t s = scheme_id ? scheme_id[i] : CG_SCHEME_EDDSA_ED25519_SHA512;
    if (s == CG_SCHEME_EDDSA_ED25519_SHA512) has_ed = true;
    if (s == CG_SCHEME_ECDSA_SECP256K1_SHA256 || s == CG_SCHEME_ECDSA_SECP256R1_SHA256) {
      has_ec = true;
      const uint32_t l = sig_len ? sig_len[i] : (uint32_t)sig_stride;
      if (l > sig_stride)
        return fail(ctx, CG_E_INVALID_ARGUMENT, "ECDSA signature longer than sig_stride at element " + std::to_string(i));
    }
    if ((uint64_t)msg_off[i] + msg_len[i] > msg_bytes)
      return fail(ctx, CG_E_INVALID_ARGUMENT, "message out of arena bounds at element " + std::to_string(i));
  }
  if (has_ed && (pk_stride < 32 || sig_stride < 64))
    return fail(ctx, CG_E_INVALID_ARGUMENT, "Ed25519 needs pk_stride >= 32 and sig_stride >= 64");
  if (has_ec && pk_stride < 64) return fail(ctx, CG_E_INVALID_ARGUMENT, "ECDSA needs pk_stride >= 64");
  return CG_OK;
}

template <typename T>
cg_status upload(cg_ctx* ctx, T** dst, const T* src, size_t count, const char* what) {
  cg_status st = dalloc(ctx, dst, count, what);
  if (st != CG_OK) return st;
  if (count) CG_TRY(ctx, hipMemcpyAsync(*dst, src, count * sizeof(T), hipMemcpyHostToDevice, ctx->stream), what);
  return CG_OK;
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
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
    delete ctx;
    return CG_E_DEVICE;
  }
  static int32_t bt[cg::kEdBaseTableWords];
  static std::once_flag bt_once;
  std::call_once(bt_once, [] { cg::ed25519_base_table_words(bt); });
  if (dalloc(ctx, &ctx->btab, cg::kEdBaseTableWords, "alloc base table") != CG_OK ||
      hipMemcpy(ctx->btab, bt, sizeof bt, hipMemcpyHostToDevice) != hipSuccess) {
    cg_close(ctx);
    return CG_E_DEVICE;
  }
  if (cg::ecdsa_consts_create(&ctx->ec) != hipSuccess) {
    cg_close(ctx);
    return CG_E_DEVICE;
  }
  *out = ctx;
  return CG_OK;
}

void cg_close(cg_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  collect_timings(ctx);
  dfree(ctx->btab);
  dfree(ctx->ed_status);
  dfree(ctx->ed_digits);
  dfree(ctx->ed_table);
  cg::ecdsa_consts_free(ctx->ec);
  for (hipEvent_t e : ctx->event_pool) (void)hipEventDestroy(e);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

const char* cg_last_error(const cg_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

}  // extern "C"

namespace {

// Stages a batch; the message arena comes from host memory (msg) or, for the
// signed-transaction path, from a device buffer the library owns (msg_dev: the
// recomputed ids), which the batch then references without owning.
cg_status create_batch(cg_ctx* ctx, size_t n, const uint8_t* scheme_id, const uint8_t* pk, size_t pk_stride,
                       const uint8_t* sig, size_t sig_stride, const uint32_t* sig_len, const uint8_t* msg,
                       uint8_t* msg_dev, size_t msg_bytes, const uint64_t* msg_off, const uint32_t* msg_len,
                       cg_batch** out) {
  if (!out) return fail(ctx, CG_E_INVALID_ARGUMENT, "null out");
  *out = nullptr;
  cg_status st = check_inputs(ctx, n, scheme_id, pk, pk_stride, sig, sig_stride, sig_len,
                              msg_dev ? (const uint8_t*)msg_dev : msg, msg_bytes, msg_off, msg_len);
  if (st != CG_OK) return st;
  if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, CG_E_DEVICE, "hipSetDevice");
  cg_batch* b = new (std::nothrow) cg_batch();
  if (!b) return fail(ctx, CG_E_OUT_OF_MEMORY, "host alloc");
  b->n = n;
  auto bail = [&](cg_status s) {
    (void)hipStreamSynchronize(ctx->stream);
    batch_free(b);
    return s;
  };
  // host-side partition by scheme
  std::vector<uint32_t> idx[3];  // 0: ed25519, 1: K1, 2: R1
  bool ed_identity = true;
  for (size_t i = 0; i < n; ++i) {
    const uint8_t s = scheme_id ? scheme_id[i] : CG_SCHEME_EDDSA_ED25519_SHA512;
    if (s == CG_SCHEME_EDDSA_ED25519_SHA512) {
      if (idx[0].size() != i) ed_identity = false;
      idx[0].push_back((uint32_t)i);
    } else if (s == CG_SCHEME_ECDSA_SECP256K1_SHA256) {
      idx[1].push_back((uint32_t)i);
    } else if (s == CG_SCHEME_ECDSA_SECP256R1_SHA256) {
      idx[2].push_back((uint32_t)i);
    }
  }
  if (idx[0].size() != n) ed_identity = false;
  const size_t nwords = (n + 31) / 32;
  if ((st = dalloc(ctx, &b->verdict, n, "alloc verdict")) != CG_OK) return bail(st);
  if ((st = dalloc(ctx, &b->bitmap, nwords, "alloc bitmap")) != CG_OK) return bail(st);
  // raw element-major inputs (temporary) + arena (kept)
  uint8_t *pk_raw = nullptr, *sig_raw = nullptr;
  uint32_t* sl_raw = nullptr;
  if (msg_dev) {
    b->arena = msg_dev;  // caller-owned device arena (padded by the caller)
    b->arena_owned = false;
  } else {
    if ((st = dalloc(ctx, &b->arena, msg_bytes + 16, "alloc arena")) != CG_OK) return bail(st);
    if (msg_bytes)
      CG_TRY(ctx, hipMemcpyAsync(b->arena, msg, msg_bytes, hipMemcpyHostToDevice, ctx->stream), "upload arena");
    CG_TRY(ctx, hipMemsetAsync(b->arena + msg_bytes, 0, 16, ctx->stream), "pad arena");
  }
  if ((st = upload(ctx, &b->msg_off_all, msg_off, n, "upload msg_off")) != CG_OK) return bail(st);
  if ((st = upload(ctx, &b->msg_len_all, msg_len, n, "upload msg_len")) != CG_OK) return bail(st);
  if ((st = upload(ctx, &pk_raw, pk, n * pk_stride, "upload pk")) != CG_OK) return bail(st);
  if ((st = upload(ctx, &sig_raw, sig, n * sig_stride, "upload sig")) != CG_OK) {
    dfree(pk_raw);
    return bail(st);
  }
  if (sig_len && (st = upload(ctx, &sl_raw, sig_len, n, "upload sig_len")) != CG_OK) {
    dfree(pk_raw);
    dfree(sig_raw);
    return bail(st);
  }
  auto cleanup_raw = [&]() {
    (void)hipStreamSynchronize(ctx->stream);
    dfree(pk_raw);
    dfree(sig_raw);
    dfree(sl_raw);
  };
  {
    Timed t(ctx, "stage", n);
    // Ed25519 subset -> SoA
    const uint32_t ne = (uint32_t)idx[0].size();
    b->n_ed = ne;
    if (ne) {
      if (!ed_identity && (st = upload(ctx, &b->ed_index, idx[0].data(), ne, "upload ed index")) != CG_OK) {
        cleanup_raw();
        return bail(st);
      }
      if ((st = dalloc(ctx, &b->ed_pk, (size_t)8 * ne, "alloc ed pk")) != CG_OK ||
          (st = dalloc(ctx, &b->ed_sig, (size_t)16 * ne, "alloc ed sig")) != CG_OK ||
          (st = dalloc(ctx, &b->ed_sig_len, ne, "alloc ed sig_len")) != CG_OK ||
          (st = dalloc(ctx, &b->ed_msg_off, ne, "alloc ed msg_off")) != CG_OK ||
          (st = dalloc(ctx, &b->ed_msg_len, ne, "alloc ed msg_len")) != CG_OK) {
        cleanup_raw();
        return bail(st);
      }
      hipError_t e = cg::launch_gather_words(pk_raw, pk_stride, 0, 8, b->ed_index, ne, ne, b->ed_pk, ctx->stream);
      if (e == hipSuccess)
        e = cg::launch_gather_words(sig_raw, sig_stride, 0, 16, b->ed_index, ne, ne, b->ed_sig, ctx->stream);
      if (e == hipSuccess)
        e = cg::launch_gather_u32(sl_raw, b->ed_index, ne, b->ed_sig_len, (uint32_t)sig_stride, ctx->stream);
      if (e == hipSuccess) e = cg::launch_gather_u64(b->msg_off_all, b->ed_index, ne, b->ed_msg_off, ctx->stream);
      if (e == hipSuccess) e = cg::launch_gather_u32(b->msg_len_all, b->ed_index, ne, b->ed_msg_len, 0, ctx->stream);
      if (e != hipSuccess) {
        cleanup_raw();
        return bail(hip_fail(ctx, e, "stage ed25519"));
      }
    }
    for (int c = 0; c < 2; ++c) {
      const std::vector<uint32_t>& ix = idx[1 + c];
      if (ix.empty()) continue;
      hipError_t e = cg::ecdsa_batch_stage(b->ec[c], c == 0 ? CG_SCHEME_ECDSA_SECP256K1_SHA256
                                                           : CG_SCHEME_ECDSA_SECP256R1_SHA256,
                                           ix.data(), (uint32_t)ix.size(), pk_raw, pk_stride, sig_raw, sig_stride,
                                           sl_raw, b->msg_off_all, b->msg_len_all, ctx->stream);
      if (e != hipSuccess) {
        cleanup_raw();
        return bail(hip_fail(ctx, e, "stage ecdsa"));
      }
    }
  }
  cleanup_raw();
  hipError_t e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) return bail(hip_fail(ctx, e, "stage sync"));
  collect_timings(ctx);
  *out = b;
  return CG_OK;
}

}  // namespace

extern "C" {

cg_status cg_batch_create(cg_ctx* ctx, size_t n, const uint8_t* scheme_id, const uint8_t* pk, size_t pk_stride,
                          const uint8_t* sig, size_t sig_stride, const uint32_t* sig_len, const uint8_t* msg,
                          size_t msg_bytes, const uint64_t* msg_off, const uint32_t* msg_len, cg_batch** out) {
  return create_batch(ctx, n, scheme_id, pk, pk_stride, sig, sig_stride, sig_len, msg, nullptr, msg_bytes, msg_off,
                      msg_len, out);
}

cg_status cg_batch_verify(cg_ctx* ctx, cg_batch* b, int mode, uint8_t* verdict_out, uint32_t* accept_bitmap_out,
                          void* device_bitmap_out) {
  if (!ctx || !b) return fail(ctx, CG_E_INVALID_ARGUMENT, "null context or batch");
  if (mode != CG_MODE_IS_VALID && mode != CG_MODE_DO_VERIFY) return fail(ctx, CG_E_INVALID_ARGUMENT, "bad mode");
  if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, CG_E_DEVICE, "hipSetDevice");
  const size_t n = b->n;
  if (n == 0) return CG_OK;
  cg_status st;
  // elements of unsupported schemes keep this value
  CG_TRY(ctx, hipMemsetAsync(b->verdict, CG_UNSUPPORTED, n, ctx->stream), "init verdict");
  if (b->n_ed) {
    if ((st = ensure_ed_scratch(ctx, b->n_ed)) != CG_OK) return st;
    for (uint32_t base = 0; base < b->n_ed; base += ctx->ed_scap) {
      const uint32_t cnt = std::min(ctx->ed_scap, b->n_ed - base);
      cg::Ed25519Dev d;
      d.cap = b->n_ed;
      d.scap = ctx->ed_scap;
      d.pk = b->ed_pk + base;
      d.sig = b->ed_sig + base;
      d.sig_len = b->ed_sig_len + base;
      d.arena = b->arena;
      d.msg_off = b->ed_msg_off + base;
      d.msg_len = b->ed_msg_len + base;
      d.status = ctx->ed_status;
      d.digits = ctx->ed_digits;
      d.table = ctx->ed_table;
      d.btab = ctx->btab;
      {
        Timed t(ctx, "ed25519_prep", cnt);
        CG_TRY(ctx, cg::launch_ed25519_prep(d, cnt, (uint32_t)mode, ctx->stream), "launch ed25519_prep");
      }
      {
        Timed t(ctx, "ed25519_msm", cnt);
        CG_TRY(ctx,
               cg::launch_ed25519_msm(d, cnt, b->ed_index ? b->ed_index + base : nullptr,
                                      b->ed_index ? b->verdict : b->verdict + base, ctx->stream),
               "launch ed25519_msm");
      }
    }
  }
  for (int c = 0; c < 2; ++c) {
    if (!b->ec[c].n) continue;
    const cg::EcdsaBatch& eb = b->ec[c];
    const char* prep_name = eb.scheme == 2 ? "ecdsa_k1_prep" : "ecdsa_r1_prep";
    const char* msm_name = eb.scheme == 2 ? "ecdsa_k1_msm" : "ecdsa_r1_msm";
    uint32_t chunk = 0;
    CG_TRY(ctx, cg::ecdsa_scratch(ctx->ec, eb.n, &chunk), "alloc ecdsa scratch");
    for (uint32_t base = 0; base < eb.n; base += chunk) {
      const uint32_t cnt = std::min(chunk, eb.n - base);
      {
        Timed t(ctx, prep_name, cnt);
        CG_TRY(ctx, cg::ecdsa_launch_prep(eb, ctx->ec, base, cnt, b->arena, (uint32_t)mode, ctx->stream),
               "launch ecdsa prep");
      }
      {
        Timed t(ctx, msm_name, cnt);
        CG_TRY(ctx, cg::ecdsa_launch_msm(eb, ctx->ec, base, cnt, b->verdict, ctx->stream), "launch ecdsa msm");
      }
    }
  }
  CG_TRY(ctx, cg::launch_verdict_bitmap(b->verdict, (uint32_t)n, b->bitmap, ctx->stream), "launch bitmap");
  const size_t nwords = (n + 31) / 32;
  if (device_bitmap_out)
    CG_TRY(ctx, hipMemcpyAsync(device_bitmap_out, b->bitmap, nwords * 4, hipMemcpyDeviceToDevice, ctx->stream),
           "copy device bitmap");
  if (verdict_out)
    CG_TRY(ctx, hipMemcpyAsync(verdict_out, b->verdict, n, hipMemcpyDeviceToHost, ctx->stream), "download verdict");
  if (accept_bitmap_out)
    CG_TRY(ctx, hipMemcpyAsync(accept_bitmap_out, b->bitmap, nwords * 4, hipMemcpyDeviceToHost, ctx->stream),
           "download bitmap");
  CG_TRY(ctx, hipStreamSynchronize(ctx->stream), "verify sync");
  collect_timings(ctx);
  return CG_OK;
}

size_t cg_batch_size(const cg_batch* b) { return b ? b->n : 0; }

void cg_batch_destroy(cg_ctx* ctx, cg_batch* b) {
  if (ctx) {
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
  }
  batch_free(b);
}

cg_status cg_verify_batch(cg_ctx* ctx, size_t n, int mode, const uint8_t* scheme_id, const uint8_t* pk,
                          size_t pk_stride, const uint8_t* sig, size_t sig_stride, const uint32_t* sig_len,
                          const uint8_t* msg, size_t msg_bytes, const uint64_t* msg_off, const uint32_t* msg_len,
                          uint8_t* verdict_out, uint32_t* accept_bitmap_out) {
  if (!ctx) return CG_E_INVALID_ARGUMENT;
  if (n && !verdict_out) return fail(ctx, CG_E_INVALID_ARGUMENT, "null verdict_out");
  if (n == 0) return CG_OK;
  cg_batch* b = nullptr;
  cg_status st = cg_batch_create(ctx, n, scheme_id, pk, pk_stride, sig, sig_stride, sig_len, msg, msg_bytes, msg_off,
                                 msg_len, &b);
  if (st != CG_OK) return st;
  st = cg_batch_verify(ctx, b, mode, verdict_out, accept_bitmap_out, nullptr);
  cg_batch_destroy(ctx, b);
  return st;
}

cg_status cg_der_parse_batch(cg_ctx* ctx, size_t n, const uint8_t* scheme_id, const uint8_t* sig,
                             size_t sig_stride, const uint32_t* sig_len, uint8_t* rs_out, uint8_t* status_out) {
  if (!ctx) return CG_E_INVALID_ARGUMENT;
  if (n == 0) return CG_OK;
  if (!sig || !rs_out || !status_out) return fail(ctx, CG_E_INVALID_ARGUMENT, "null pointer");
  if (n > 0xFFFFFFF0ull) return fail(ctx, CG_E_INVALID_ARGUMENT, "batch too large");
  for (size_t i = 0; sig_len && i < n; ++i)
    if (sig_len[i] > sig_stride) return fail(ctx, CG_E_INVALID_ARGUMENT, "signature longer than sig_stride");
  if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, CG_E_DEVICE, "hipSetDevice");
  std::vector<uint32_t> idx[2];
  for (size_t i = 0; i < n; ++i)
    idx[(scheme_id && scheme_id[i] == CG_SCHEME_ECDSA_SECP256K1_SHA256) ? 0 : 1].push_back((uint32_t)i);
  uint8_t* sig_d = nullptr;
  uint32_t *sl_d = nullptr, *rs_d = nullptr, *st_d = nullptr, *ix_d = nullptr;
  cg_status st = CG_OK;
  auto cleanup = [&]() {
    (void)hipStreamSynchronize(ctx->stream);
    dfree(sig_d); dfree(sl_d); dfree(rs_d); dfree(st_d); dfree(ix_d);
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
}

cg_status cg_set_profiling(cg_ctx* ctx, int enable) {
  if (!ctx) return CG_E_INVALID_ARGUMENT;
  ctx->profiling = enable != 0;
  return CG_OK;
}

cg_status cg_kernel_stats(cg_ctx* ctx, const char* kernel, double* total_ms, uint64_t* launches, uint64_t* items) {
  if (!ctx || !kernel) return CG_E_INVALID_ARGUMENT;
  collect_timings(ctx);
  auto it = ctx->stats.find(kernel);
  const Stat s = it == ctx->stats.end() ? Stat() : it->second;
  if (total_ms) *total_ms = s.ms;
  if (launches) *launches = s.launches;
  if (items) *items = s.items;
  return CG_OK;
}

cg_status cg_reset_stats(cg_ctx* ctx) {
  if (!ctx) return CG_E_INVALID_ARGUMENT;
  collect_timings(ctx);
  ctx->stats.clear();
  return CG_OK;
}

}  // extern "C"

namespace {

// Device buffers of one tx-id computation (K5 + K6).
struct TxIds {
  uint8_t* arena = nullptr;
  uint64_t *slot = nullptr, *leaf_pos = nullptr, *tree_base = nullptr;
  uint32_t *len = nullptr, *comp_tx = nullptr, *comp_idx = nullptr, *is_salt = nullptr, *salts = nullptr,
           *comp_start = nullptr, *leaves = nullptr;
  uint8_t* ids = nullptr;  // 32 B per tx (+16 pad): digest byte order
  void release() {
    for (void* p : {(void*)arena, (void*)slot, (void*)leaf_pos, (void*)tree_base, (void*)len, (void*)comp_tx,
                    (void*)comp_idx, (void*)is_salt, (void*)salts, (void*)comp_start, (void*)leaves, (void*)ids})
      dfree(p);
    *this = TxIds();
  }
};

cg_status compute_txids(cg_ctx* ctx, size_t n_tx, const uint8_t* arena, size_t arena_bytes, const uint64_t* comp_off,
                        const uint32_t* comp_len, const uint32_t* comp_start, const uint8_t* salts, TxIds& d,
                        bool* any_empty) {
  if (n_tx > 0xFFFFFFF0ull) return fail(ctx, CG_E_INVALID_ARGUMENT, "too many transactions");
  if (!comp_start || !salts || (comp_start[n_tx] && (!comp_off || !comp_len || !arena)))
    return fail(ctx, CG_E_INVALID_ARGUMENT, "null pointer");
  const size_t n_comp = comp_start[n_tx];
  if (n_comp > 0xFFFFFFF0ull) return fail(ctx, CG_E_INVALID_ARGUMENT, "too many components");
  // host-side layout: aligned slots with 32 spare bytes for the nonce; trees padded to 2^k
  std::vector<uint64_t> slot(n_comp), leaf_pos(n_comp), tree_base(n_tx + 1);
  std::vector<uint32_t> comp_tx(n_comp), comp_idx(n_comp), is_salt(n_comp);
  uint64_t pos = 0, leaves = 0;
  *any_empty = false;
  for (size_t t = 0; t < n_tx; ++t) {
    if (comp_start[t + 1] < comp_start[t]) return fail(ctx, CG_E_INVALID_ARGUMENT, "comp_start not monotone");
    const uint32_t k = comp_start[t + 1] - comp_start[t];
    if (k == 0) *any_empty = true;
    uint32_t kp = 1;
    while (kp < k) kp <<= 1;
    tree_base[t] = leaves;
    leaves += k ? kp : 1;
    for (uint32_t i = 0; i < k; ++i) {
      const size_t c = comp_start[t] + i;
      if (comp_off[c] + comp_len[c] > arena_bytes)
        return fail(ctx, CG_E_INVALID_ARGUMENT, "component out of arena bounds");
      slot[c] = pos;
      pos += ((uint64_t)comp_len[c] + 32 + 3) & ~3ull;
      comp_tx[c] = (uint32_t)t;
      comp_idx[c] = i;
      is_salt[c] = i == k - 1;
      leaf_pos[c] = tree_base[t] + i;
    }
  }
  std::vector<uint8_t> slotted(pos + 16, 0);
  for (size_t c = 0; c < n_comp; ++c) std::memcpy(slotted.data() + slot[c], arena + comp_off[c], comp_len[c]);
  cg_status st;
  if ((st = upload(ctx, &d.arena, slotted.data(), slotted.size(), "upload tx arena")) != CG_OK ||
      (st = upload(ctx, &d.slot, slot.data(), n_comp, "upload slots")) != CG_OK ||
      (st = upload(ctx, &d.leaf_pos, leaf_pos.data(), n_comp, "upload leaf_pos")) != CG_OK ||
      (st = upload(ctx, &d.tree_base, tree_base.data(), n_tx, "upload tree_base")) != CG_OK ||
      (st = upload(ctx, &d.len, comp_len, n_comp, "upload comp_len")) != CG_OK ||
      (st = upload(ctx, &d.comp_tx, comp_tx.data(), n_comp, "upload comp_tx")) != CG_OK ||
      (st = upload(ctx, &d.comp_idx, comp_idx.data(), n_comp, "upload comp_idx")) != CG_OK ||
      (st = upload(ctx, &d.is_salt, is_salt.data(), n_comp, "upload is_salt")) != CG_OK ||
      (st = upload(ctx, &d.salts, (const uint32_t*)salts, 8 * n_tx, "upload salts")) != CG_OK ||
      (st = upload(ctx, &d.comp_start, comp_start, n_tx + 1, "upload comp_start")) != CG_OK ||
      (st = dalloc(ctx, &d.leaves, 8 * leaves, "alloc leaves")) != CG_OK ||
      (st = dalloc(ctx, &d.ids, 32 * n_tx + 16, "alloc ids")) != CG_OK) {
    (void)hipStreamSynchronize(ctx->stream);
    return st;
  }
  CG_TRY(ctx, hipMemsetAsync(d.leaves, 0, 32 * leaves, ctx->stream), "zero leaves");
  CG_TRY(ctx, hipMemsetAsync(d.ids, 0, 32 * n_tx + 16, ctx->stream), "zero ids");
  {
    Timed t(ctx, "merkle_leaf", n_comp);
    CG_TRY(ctx, cg::launch_merkle_nonce(d.arena, d.slot, d.len, d.comp_tx, d.comp_idx, d.is_salt, d.salts,
                                        (uint32_t)n_comp, ctx->stream), "launch merkle_nonce");
    CG_TRY(ctx, cg::launch_merkle_leaf(d.arena, d.slot, d.len, d.is_salt, d.leaf_pos, (uint32_t)n_comp, d.leaves,
                                       ctx->stream), "launch merkle_leaf");
  }
  {
    Timed t(ctx, "merkle_tree", n_tx);
    CG_TRY(ctx, cg::launch_merkle_tree(d.leaves, d.tree_base, d.comp_start, (uint32_t)n_tx, (uint32_t*)d.ids,
                                       ctx->stream), "launch merkle_tree");
  }
  // the host staging vectors die here: wait for the uploads that read them
  CG_TRY(ctx, hipStreamSynchronize(ctx->stream), "txid sync");
  return CG_OK;
}

}  // namespace

extern "C" {

cg_status cg_txid_batch(cg_ctx* ctx, size_t n_tx, const uint8_t* arena, size_t arena_bytes,
                        const uint64_t* comp_off, const uint32_t* comp_len, const uint32_t* comp_start,
                        const uint8_t* salts, uint8_t* ids_out) {
  if (!ctx) return CG_E_INVALID_ARGUMENT;
  if (n_tx == 0) return CG_OK;
  if (!ids_out) return fail(ctx, CG_E_INVALID_ARGUMENT, "null ids_out");
  if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, CG_E_DEVICE, "hipSetDevice");
  TxIds d;
  bool any_empty = false;
  cg_status st = compute_txids(ctx, n_tx, arena, arena_bytes, comp_off, comp_len, comp_start, salts, d, &any_empty);
  if (st == CG_OK) {
    hipError_t e = hipMemcpyAsync(ids_out, d.ids, 32 * n_tx, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) st = hip_fail(ctx, e, "download ids");
  }
  d.release();
  collect_timings(ctx);
  if (st == CG_OK && any_empty)
    return fail(ctx, CG_E_MERKLE_EMPTY, "Cannot calculate Merkle root on empty hash list.");
  return st;
}

cg_status cg_tx_verify_batch(cg_ctx* ctx, int mode, size_t n_tx, const uint8_t* arena, size_t arena_bytes,
                             const uint64_t* comp_off, const uint32_t* comp_len, const uint32_t* comp_start,
                             const uint8_t* salts, const uint32_t* sig_start, const uint8_t* scheme_id,
                             const uint8_t* pk, size_t pk_stride, const uint8_t* sig, size_t sig_stride,
                             const uint32_t* sig_len, int32_t* first_bad_out, uint8_t* verdict_out,
                             uint8_t* ids_out) {
  if (!ctx) return CG_E_INVALID_ARGUMENT;
  if (n_tx == 0) return CG_OK;
  if (!sig_start || !first_bad_out) return fail(ctx, CG_E_INVALID_ARGUMENT, "null pointer");
  if (mode != CG_MODE_IS_VALID && mode != CG_MODE_DO_VERIFY) return fail(ctx, CG_E_INVALID_ARGUMENT, "bad mode");
  if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, CG_E_DEVICE, "hipSetDevice");
  TxIds d;
  bool any_empty = false;
  cg_status st = compute_txids(ctx, n_tx, arena, arena_bytes, comp_off, comp_len, comp_start, salts, d, &any_empty);
  if (st != CG_OK) {
    d.release();
    return st;
  }
  const size_t n_sig = sig_start[n_tx];
  std::vector<uint64_t> moff(n_sig);
  std::vector<uint32_t> mlen(n_sig, 32);
  for (size_t t = 0; t < n_tx; ++t) {
    if (sig_start[t + 1] < sig_start[t]) {
      d.release();
      return fail(ctx, CG_E_INVALID_ARGUMENT, "sig_start not monotone");
    }
    for (uint32_t s = sig_start[t]; s < sig_start[t + 1]; ++s) moff[s] = 32 * (uint64_t)t;
  }
  cg_batch* b = nullptr;
  if (n_sig) {
    st = create_batch(ctx, n_sig, scheme_id, pk, pk_stride, sig, sig_stride, sig_len, nullptr, d.ids, 32 * n_tx,
                      moff.data(), mlen.data(), &b);
    if (st == CG_OK) st = cg_batch_verify(ctx, b, mode, verdict_out, nullptr, nullptr);
  }
  uint32_t* ss_d = nullptr;
  int32_t* fb_d = nullptr;
  if (st == CG_OK && (st = upload(ctx, &ss_d, sig_start, n_tx + 1, "upload sig_start")) == CG_OK &&
      (st = dalloc(ctx, &fb_d, n_tx, "alloc first_bad")) == CG_OK) {
    uint8_t* verdict_dev = b ? b->verdict : nullptr;
    hipError_t e = cg::launch_first_bad(verdict_dev, ss_d, (uint32_t)n_tx, fb_d, ctx->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(first_bad_out, fb_d, 4 * n_tx, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess && ids_out) e = hipMemcpyAsync(ids_out, d.ids, 32 * n_tx, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) st = hip_fail(ctx, e, "first_bad");
  }
  (void)hipStreamSynchronize(ctx->stream);
  dfree(ss_d);
  dfree(fb_d);
  if (b) cg_batch_destroy(ctx, b);
  // a tx with no component has no id: report it as -3 (MerkleTreeException)
  if (st == CG_OK && any_empty) {
    for (size_t t = 0; t < n_tx; ++t)
      if (comp_start[t + 1] == comp_start[t]) first_bad_out[t] = -3;
  }
  d.release();
  collect_timings(ctx);
  if (st == CG_OK && any_empty)
    return fail(ctx, CG_E_MERKLE_EMPTY, "Cannot calculate Merkle root on empty hash list.");
  return st;
}

}  // extern "C"
