// Sanitizer driver (TEST INFRASTRUCTURE ONLY): the host build of the device arithmetic
// (cg_host.cpp, the very cg_*.h code the HIP kernels compile) and the C oracle, both
// compiled with -fsanitize=address,undefined into one executable (no preloading: the
// program itself is instrumented), fed cases on stdin by tests/test_sanitizers.py.
// Every line is one command with hex fields ("-" = empty); every answer is one line.
//
//   E pk sig msg          Ed25519: oracle (isValid, doVerify), host (both modes), the
//                         (h, 1) fallback and padded-digit runs, the 2/4/8-lane latency
//                         splits, the key-reuse path (plain, wide, wide + fallback)
//   C scheme q sig msg    ECDSA: oracle and host in both modes, K4 DER status + r, s
//   F a b                 GF(2^255-19) a*b, a^2, a^-1 (8 LE words each)
//   P scheme a b          radix-2^26 Montgomery field of the curve: ops 0..4
//   S x                   sc_reduce512 of 16 LE words
//   H h                   half-size scalars (TB 128 and the key-reuse TB 192)
//   J scheme u1 u2 qx qy  joint multiplication u1 G + u2 Q (GLV on secp256k1)
//   T msg tail            SHA-256(msg || tail) as the Merkle leaf kernel streams it
//   Q n n_ed bytes pks sgs sl ec ord keys opts
//                         cg_verify_batch's host plan (cg_plan.h) for that shape and options
//                         ("-" = none): its 13 fields and the chunk boundaries
//   X                     negative control: a deliberate heap overread (must be reported)
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../oracle/c/oracle.h"

extern "C" {
void cgh_fe_mul(const uint32_t* a, const uint32_t* b, uint32_t* out);
void cgh_fe_sq(const uint32_t* a, uint32_t* out);
void cgh_fe_invert(const uint32_t* a, uint32_t* out);
void cgh_sc_reduce512(const uint32_t* x, uint32_t* out);
int cgh_half_scalars(const uint32_t* h, uint32_t* c0, uint32_t* c1, uint32_t* c1neg);
int cgh_half_scalars_reuse(const uint32_t* h, uint32_t* c0, uint32_t* c1, uint32_t* c1neg);
int cgh_ed25519_verify_nd(const uint8_t* pk, const uint8_t* sig, uint32_t sig_len, const uint8_t* msg,
                          uint32_t msg_len, uint32_t mode, uint32_t force_ndig, uint32_t full_length);
int cgh_ed25519_verify_pair(const uint8_t* pk, const uint8_t* sig, uint32_t sig_len, const uint8_t* msg,
                            uint32_t msg_len, uint32_t mode, uint32_t force_ndig);
int cgh_ed25519_verify_quad(const uint8_t* pk, const uint8_t* sig, uint32_t sig_len, const uint8_t* msg,
                            uint32_t msg_len, uint32_t mode, uint32_t force_ndig);
int cgh_ed25519_verify_oct(const uint8_t* pk, const uint8_t* sig, uint32_t sig_len, const uint8_t* msg,
                           uint32_t msg_len, uint32_t mode, uint32_t force_ndig);
int cgh_ed25519_verify_reuse(const uint8_t* pk, const uint8_t* sig, uint32_t sig_len, const uint8_t* msg,
                             uint32_t msg_len, uint32_t mode, uint32_t wide, uint32_t full_length);
int cgh_ecdsa_verify(int scheme, const uint8_t* q_be, const uint8_t* sig, uint32_t sig_len, const uint8_t* msg,
                     uint32_t msg_len, uint32_t mode);
uint32_t cgh_der_parse(int scheme, const uint8_t* sig, uint32_t n, uint32_t* r, uint32_t* s);
void cgh_f26_op(int scheme, int op, const uint32_t* a, const uint32_t* b, uint32_t* out);
int cgh_ecdsa_joint(int scheme, const uint32_t* u1, const uint32_t* u2, const uint32_t* qx, const uint32_t* qy,
                    uint32_t* out, uint32_t force_nd);
void cgh_sha256_tail(const uint8_t* msg, uint32_t n, const uint8_t* tail, uint32_t tail_n, uint8_t* out);
int cgh_plan_verify(uint64_t n, uint64_t n_ed, uint64_t msg_bytes, uint64_t pk_stride, uint64_t sig_stride, int sig_len,
                    int ecdsa, int ed_in_order, int keys_repeat, const char* opts, uint64_t* out, uint64_t* bounds,
                    int max_bounds);
}

namespace {

// Exactly-sized heap copies, so ASan sees any read past a field's end.
std::vector<uint8_t> unhex(const std::string& s) {
  std::vector<uint8_t> out;
  if (s == "-") return out;
  for (size_t i = 0; i + 1 < s.size(); i += 2) out.push_back((uint8_t)std::stoul(s.substr(i, 2), nullptr, 16));
  return out;
}

std::vector<uint32_t> words(const std::string& s, size_t n) {  // n LE words from little-endian hex bytes
  std::vector<uint8_t> b = unhex(s);
  b.resize(4 * n, 0);
  std::vector<uint32_t> w(n);
  memcpy(w.data(), b.data(), 4 * n);
  return w;
}

void put_words(const uint32_t* w, size_t n) {
  printf(" ");
  const uint8_t* b = reinterpret_cast<const uint8_t*>(w);
  for (size_t i = 0; i < 4 * n; ++i) printf("%02x", b[i]);
}

// A heap buffer of exactly the field's bytes plus `pad` (never a null pointer, so an
// empty field is a zero-length argument, not a null one).  Messages get the 16 bytes
// the device arena carries after the last message (cordagpu.cpp: "padded by 16 B so
// tail loads stay in bounds"); keys and signatures get none.
struct Buf {
  std::vector<uint8_t> v;
  uint8_t* p;
  Buf(const std::string& s, size_t pad = 0) : v(unhex(s)), p(new uint8_t[v.size() + pad + (v.empty() && !pad)]()) {
    if (!v.empty()) memcpy(p, v.data(), v.size());
  }
  ~Buf() { delete[] p; }
  uint32_t n() const { return (uint32_t)v.size(); }
};

void cmd_ed(char* f[]) {
  Buf pk(f[1]), sig(f[2]), msg(f[3], 16);
  if (pk.n() != 32) {
    printf("E skip\n");
    return;
  }
  const uint32_t ns = sig.n(), nm = msg.n();
  printf("E");
  for (int mode = 0; mode < 2; ++mode) printf(" %d", oracle_ed25519_verify(pk.p, sig.p, ns, msg.p, nm, mode));
  for (int mode = 0; mode < 2; ++mode) printf(" %d", cgh_ed25519_verify_nd(pk.p, sig.p, ns, msg.p, nm, mode, 0, 0));
  printf(" %d %d", cgh_ed25519_verify_nd(pk.p, sig.p, ns, msg.p, nm, 0, 0, 1),
         cgh_ed25519_verify_nd(pk.p, sig.p, ns, msg.p, nm, 0, 64, 0));
  printf(" %d %d %d", cgh_ed25519_verify_pair(pk.p, sig.p, ns, msg.p, nm, 0, 0),
         cgh_ed25519_verify_quad(pk.p, sig.p, ns, msg.p, nm, 0, 0),
         cgh_ed25519_verify_oct(pk.p, sig.p, ns, msg.p, nm, 1, 64));
  printf(" %d %d %d\n", cgh_ed25519_verify_reuse(pk.p, sig.p, ns, msg.p, nm, 0, 0, 0),
         cgh_ed25519_verify_reuse(pk.p, sig.p, ns, msg.p, nm, 0, 1, 0),
         cgh_ed25519_verify_reuse(pk.p, sig.p, ns, msg.p, nm, 1, 1, 1));
}

void cmd_ec(char* f[]) {
  const int scheme = atoi(f[1]);
  Buf q(f[2]), sig(f[3]), msg(f[4], 16);
  if (q.n() != 64) {
    printf("C skip\n");
    return;
  }
  printf("C");
  for (int mode = 0; mode < 2; ++mode)
    printf(" %d", oracle_ecdsa_verify(scheme, q.p, sig.p, sig.n(), msg.p, msg.n(), mode));
  for (int mode = 0; mode < 2; ++mode)
    printf(" %d", cgh_ecdsa_verify(scheme, q.p, sig.p, sig.n(), msg.p, msg.n(), mode));
  uint32_t r[8] = {0}, s[8] = {0};
  printf(" %u", cgh_der_parse(scheme, sig.p, sig.n(), r, s));
  put_words(r, 8);
  put_words(s, 8);
  printf("\n");
}

}  // namespace

int main() {
  oracle_ed25519_init();
  static char line[1 << 22];
  while (fgets(line, sizeof line, stdin)) {
    char* f[12] = {nullptr};
    int nf = 0;
    for (char* t = strtok(line, " \n"); t && nf < 12; t = strtok(nullptr, " \n")) f[nf++] = t;
    if (nf == 0) continue;
    switch (f[0][0]) {
      case 'E':
        cmd_ed(f);
        break;
      case 'C':
        cmd_ec(f);
        break;
      case 'F': {
        std::vector<uint32_t> a = words(f[1], 8), b = words(f[2], 8), o(8);
        printf("F");
        cgh_fe_mul(a.data(), b.data(), o.data());
        put_words(o.data(), 8);
        cgh_fe_sq(a.data(), o.data());
        put_words(o.data(), 8);
        cgh_fe_invert(a.data(), o.data());
        put_words(o.data(), 8);
        printf("\n");
        break;
      }
      case 'P': {
        const int scheme = atoi(f[1]);
        std::vector<uint32_t> a = words(f[2], 8), b = words(f[3], 8), o(8);
        printf("P");
        for (int op = 0; op < 5; ++op) {
          cgh_f26_op(scheme, op, a.data(), b.data(), o.data());
          put_words(o.data(), 8);
        }
        printf("\n");
        break;
      }
      case 'S': {
        std::vector<uint32_t> x = words(f[1], 16), o(8);
        cgh_sc_reduce512(x.data(), o.data());
        printf("S");
        put_words(o.data(), 8);
        printf("\n");
        break;
      }
      case 'H': {
        std::vector<uint32_t> h = words(f[1], 8), c0(8), c1(8);
        uint32_t neg = 0;
        printf("H %d", cgh_half_scalars(h.data(), c0.data(), c1.data(), &neg));
        put_words(c0.data(), 8);
        put_words(c1.data(), 8);
        printf(" %u", neg);
        printf(" %d", cgh_half_scalars_reuse(h.data(), c0.data(), c1.data(), &neg));
        put_words(c0.data(), 8);
        put_words(c1.data(), 8);
        printf(" %u\n", neg);
        break;
      }
      case 'J': {
        const int scheme = atoi(f[1]);
        std::vector<uint32_t> u1 = words(f[2], 8), u2 = words(f[3], 8), qx = words(f[4], 8), qy = words(f[5], 8),
                              o(16);
        printf("J %d", cgh_ecdsa_joint(scheme, u1.data(), u2.data(), qx.data(), qy.data(), o.data(), 0));
        put_words(o.data(), 16);
        printf("\n");
        break;
      }
      case 'T': {
        Buf msg(f[1], 16), tail(f[2]);  // (the leaf kernel's arena is padded too)
        uint8_t out[32];
        cgh_sha256_tail(msg.p, msg.n(), tail.p, tail.n(), out);
        printf("T ");
        for (int i = 0; i < 32; ++i) printf("%02x", out[i]);
        printf("\n");
        break;
      }
      case 'Q': {  // host plan: n n_ed bytes pk_stride sig_stride sig_len ecdsa in_order keys_repeat opts
        if (nf < 10) {
          printf("Q skip\n");
          break;
        }
        uint64_t out[13] = {0}, bounds[16] = {0};
        const char* opts = nf > 10 && strcmp(f[10], "-") ? f[10] : "";
        const int nb = cgh_plan_verify(strtoull(f[1], nullptr, 10), strtoull(f[2], nullptr, 10),
                                       strtoull(f[3], nullptr, 10), strtoull(f[4], nullptr, 10),
                                       strtoull(f[5], nullptr, 10), atoi(f[6]), atoi(f[7]), atoi(f[8]), atoi(f[9]),
                                       opts, out, bounds, 16);
        printf("Q %d", nb);
        for (int i = 0; i < 13; ++i) printf(" %llu", (unsigned long long)out[i]);
        for (int i = 0; i < nb && i < 16; ++i) printf(" %llu", (unsigned long long)bounds[i]);
        printf("\n");
        break;
      }
      case 'X': {  // negative control for the tests: a 31-byte key buffer read as a 32-byte key
        uint8_t* k = new uint8_t[31]();
        uint8_t ab[32];
        printf("X %d\n", oracle_ed25519_abyte(k, ab));
        delete[] k;
        break;
      }
      default:
        printf("?\n");
    }
    fflush(stdout);
  }
  return 0;
}
