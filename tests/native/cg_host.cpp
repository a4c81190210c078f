// Host build of the device Ed25519 pipeline (the exact cg_*.h code the HIP
// kernels compile), used only by tests/test_native_host.py to check the device
// algorithm — limb bounds, carries, scalar recodings, window arithmetic — against
// the CPU oracle on millions of cases without a GPU.  Not part of the product.
#include <stdint.h>
#include <string.h>

#include "cg_ed25519.h"

using namespace cg;

extern "C" {

// out = canonical(a * b mod p); a, b: 8 LE words (bit 255 ignored, i2p style).
void cgh_fe_mul(const uint32_t* a, const uint32_t* b, uint32_t* out) {
  fe x, y, z;
  fe_frombytes(x, a);
  fe_frombytes(y, b);
  fe_mul(z, x, y);
  fe_tobytes(out, z);
}

void cgh_fe_sq(const uint32_t* a, uint32_t* out) {
  fe x, z;
  fe_frombytes(x, a);
  fe_sq(z, x);
  fe_tobytes(out, z);
}

void cgh_fe_invert(const uint32_t* a, uint32_t* out) {
  fe x, z;
  fe_frombytes(x, a);
  fe_invert(z, x);
  fe_tobytes(out, z);
}

void cgh_sc_reduce512(const uint32_t* x, uint32_t* out) { sc_reduce512(out, x); }

uint32_t cgh_slide_drop(const uint32_t* s) { return slide_drops_carry(s); }

void cgh_effective_s(const uint32_t* s, uint32_t* out) { sc_effective_s(out, s); }

void cgh_recode16(const uint32_t* k, uint32_t* out) { sc_recode16(out, k); }

void cgh_sha512_ed25519(const uint32_t* r, const uint32_t* ab, const uint8_t* msg, uint32_t n, uint32_t* out) {
  sha512_ed25519(out, r, ab, msg, n);
}

int cgh_abyte(const uint32_t* pk, uint32_t* out) {
  ge_p3 A;
  if (!ge_frombytes_i2p(A, pk)) return -1;
  ed25519_abyte(out, A);
  return 0;
}

static ge_precomp g_btab[9];
static int g_init;

int cgh_ed25519_verify(const uint8_t* pk_bytes, const uint8_t* sig_bytes, uint32_t sig_len, const uint8_t* msg,
                       uint32_t msg_len, uint32_t mode) {
  if (!g_init) {
    ed25519_base_table(g_btab);
    g_init = 1;
  }
  uint32_t pk[8], sig[16] = {0};
  memcpy(pk, pk_bytes, 32);
  memcpy(sig, sig_bytes, sig_len < 64 ? sig_len : 64);
  ge_p3 negA;
  uint32_t hd[8], sd[8];
  const uint32_t pre = ed25519_prep(pk, sig, sig_len, msg, msg_len, mode, negA, hd, sd);
  if (pre != V_COMPUTE) return (int)pre;
  ge_cached tab[9];
  ed25519_build_table(negA, [&](int k, const ge_cached& c) { tab[k] = c; });
  uint32_t rc[8];
  ed25519_msm(
      rc, hd, sd, [&](uint32_t k, ge_cached& c) { c = tab[k]; }, [&](uint32_t k, ge_precomp& p) { p = g_btab[k]; });
  return memcmp(rc, sig, 32) == 0 ? (int)V_ACCEPT : (int)V_REJECT;
}
}
