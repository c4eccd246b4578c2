// HOST INSTRUMENTATION BUILD of the BLS (BN254) kernel code -- test tooling
// only, never loaded by the product (tests/test_bls_hostcheck.py).
//
// Compiles indy-plenum_amd/csrc/pv_bn254.h with g++ so that the exact per-lane
// schedule the HIP kernels run (line precomputation, fixed-Q Miller loop,
// Scott final exponentiation, hash-to-G1, sigma decoding) can be compared with
// the independent C oracle (oracle/bn254_oracle.c) on the CPU, with every
// multiply's signed column sums checked against 2^63 and the Fp
// multiplications counted (the roofline's algorithmic work).
#include <stdint.h>
#include <stdio.h>
#include <string.h>

static uint64_t g_cnt[2];
static int g_bad = 0;
static double g_max_col = 0;   // log2 of the largest |column sum| seen
// the operand contract of bn::mul (pv_bn254.h f2mul): every limb below 2^30 and
// at least one operand with every limb below 2^29 -- then NO arrangement of such
// limbs can push a column past 2^62.3, whatever the values seen here
static int g_disc_bad = 0;

#define PV_HD static inline
#define PV_BN_COUNT(kind) (++g_cnt[kind])
static void bn_check_mul(const int32_t* a, const int32_t* b);
#define PV_BN_CHECK_MUL(a, b) bn_check_mul((a).l, (b).l)

#include "../../indy-plenum_amd/csrc/pv_bn254.h"
#include "../../indy-plenum_amd/csrc/pv_bn254_pair.h"
#include "../../indy-plenum_amd/csrc/pv_sha256.h"

#include <math.h>

// |a_i| |b_j| summed per column (upper bound of the signed sum) + the
// reduction products m_i p_j (< 2^28 * 2^28) + the carry in: < 2^63
static void bn_check_mul(const int32_t* a, const int32_t* b) {
  int64_t ma = 0, mb = 0;
  for (int i = 0; i < bn::NL; ++i) {
    const int64_t x = a[i] < 0 ? -(int64_t)a[i] : a[i], y = b[i] < 0 ? -(int64_t)b[i] : b[i];
    ma = x > ma ? x : ma;
    mb = y > mb ? y : mb;
  }
  if (ma >= (1ll << 30) || mb >= (1ll << 30) || (ma >= (1ll << 29) && mb >= (1ll << 29))) {
    if (!g_disc_bad) fprintf(stderr, "bn254 operand contract violated: max limbs 2^%.2f, 2^%.2f\n", log2((double)ma), log2((double)mb));
    g_disc_bad = 1;
  }
  for (int k = 0; k < 2 * bn::NL - 1; ++k) {
    unsigned __int128 s = (unsigned __int128)1 << 36;   // carry
    for (int i = 0; i < bn::NL; ++i) {
      const int j = k - i;
      if (j < 0 || j >= bn::NL) continue;
      const int64_t x = a[i] < 0 ? -(int64_t)a[i] : a[i], y = b[j] < 0 ? -(int64_t)b[j] : b[j];
      s += (unsigned __int128)(x * y);
      s += (unsigned __int128)1 << 56;   // m_i p_j
    }
    const double l = log2((double)s);
    if (l > g_max_col) g_max_col = l;
    if (s >> 63) {
      if (!g_bad) fprintf(stderr, "bn254 column bound violated: column %d, 2^%.2f\n", k, l);
      g_bad = 1;
    }
  }
}

using namespace bn;

extern "C" {

int bnc_bad(void) { return g_bad; }
int bnc_disc_bad(void) { return g_disc_bad; }
double bnc_max_col(void) { return g_max_col; }
void bnc_counts(uint64_t* out) {
  out[0] = g_cnt[0];
  out[1] = g_cnt[1];
}
void bnc_reset(void) {
  g_cnt[0] = g_cnt[1] = 0;
  g_bad = 0;
  g_disc_bad = 0;
  g_max_col = 0;
}

// the 69 lines of a G2 point (N_LINES x LINE_WORDS words); returns the status
int bnc_g2_lines(const uint8_t* b128, uint32_t* out) {
  g2a q;
  const int st = g2_decode(b128, q);
  if (st == 0) g2_lines(out, q);
  return st;
}

// H(m) as the 128-byte G1 representation
void bnc_hash_to_g1(const uint8_t* m, uint64_t n, uint8_t* out) {
  uint8_t buf[4096 + 64];
  memcpy(buf, m, n);
  memset(buf + n, 0, 64);
  uint32_t d[8];
  pv::sha256_msg(d, buf, n, 0, 0);
  fp x, y;
  hash_to_g1(reinterpret_cast<const uint8_t*>(d), x, y);
  memset(out, 0, 128);
  out[0] = 4;
  to_be32(out + 1, from_mont(x));
  to_be32(out + 33, from_mont(y));
}

void bnc_sign(const uint8_t* sk, const uint8_t* m, uint64_t n, uint8_t* out) {
  uint8_t h[128];
  bnc_hash_to_g1(m, n, h);
  const fp hx = to_mont(from_be32(h + 1)), hy = to_mont(from_be32(h + 33));
  g1_sign(out, hx, hy, sk);
}

// the whole check on the kernel's schedule (message <= 4096 bytes)
int bnc_verify(const uint8_t* sig128, const uint8_t* m, uint64_t n, const uint8_t* pk128, const uint8_t* gen128) {
  static uint32_t gl[N_LINES * LINE_WORDS], pl[N_LINES * LINE_WORDS];
  if (bnc_g2_lines(gen128, gl) != 0) return -1;
  g2a q;
  const int st = g2_decode(pk128, q);
  if (st == 0) g2_lines(pl, q);
  else memset(pl, 0, sizeof pl);
  uint8_t h[128];
  bnc_hash_to_g1(m, n, h);
  const fp hx = to_mont(from_be32(h + 1)), hy = to_mont(from_be32(h + 33));
  fp xqh, yqh;
  line_point(hx, hy, true, xqh, yqh);
  if (st != 0) xqh = yqh = fzero();
  fp xs, ys;
  bool s_inf;
  g1_decode(sig128, xs, ys, s_inf);
  return bls_check(xs, ys, s_inf, xqh, yqh, st == 1, gl, pl) ? 1 : 0;
}

// the same check on the lane-pair kernel's schedule (pv_bn254_pair.h, both
// lanes emulated; the slot is the check's LDS Fp12)
int bnc_verify_pair(const uint8_t* sig128, const uint8_t* m, uint64_t n, const uint8_t* pk128, const uint8_t* gen128) {
  static uint32_t gl[N_LINES * LINE_WORDS], pl[N_LINES * LINE_WORDS];
  if (bnc_g2_lines(gen128, gl) != 0) return -1;
  g2a q;
  const int st = g2_decode(pk128, q);
  if (st == 0) g2_lines(pl, q);
  else memset(pl, 0, sizeof pl);
  uint8_t h[128];
  bnc_hash_to_g1(m, n, h);
  const fp hx = to_mont(from_be32(h + 1)), hy = to_mont(from_be32(h + 33));
  fp xqh, yqh;
  line_point(hx, hy, true, xqh, yqh);
  if (st != 0) xqh = yqh = fzero();
  fp xs, ys;
  bool s_inf;
  g1_decode(sig128, xs, ys, s_inf);
  uint32_t slot[12 * NL];
  const pslot<1> S{slot};
  return bls_check_pair(S, xs, ys, s_inf, xqh, yqh, st == 1, gl, pl) ? 1 : 0;
}

// ... and on the lane-QUAD kernel's schedule (k_bls_verify_quad: one pairing's
// Miller loop per lane pair, the pairs' values multiplied, one final exponentiation)
int bnc_verify_quad(const uint8_t* sig128, const uint8_t* m, uint64_t n, const uint8_t* pk128, const uint8_t* gen128) {
  static uint32_t gl[N_LINES * LINE_WORDS], pl[N_LINES * LINE_WORDS];
  if (bnc_g2_lines(gen128, gl) != 0) return -1;
  g2a q;
  const int st = g2_decode(pk128, q);
  if (st == 0) g2_lines(pl, q);
  else memset(pl, 0, sizeof pl);
  uint8_t h[128];
  bnc_hash_to_g1(m, n, h);
  const fp hx = to_mont(from_be32(h + 1)), hy = to_mont(from_be32(h + 33));
  fp xqh, yqh;
  line_point(hx, hy, true, xqh, yqh);
  if (st != 0) xqh = yqh = fzero();
  fp xs, ys, xq = fzero(), yq = fzero();
  bool s_inf;
  g1_decode(sig128, xs, ys, s_inf);
  if (!s_inf) line_point(xs, ys, false, xq, yq);
  p1 qa[2], qb[2];
  for (int j = 0; j < PL; ++j) {
    qa[0].e[j] = qa[1].e[j] = fsel(prole(j), yq, xq);
    qb[0].e[j] = qb[1].e[j] = fsel(prole(j), yqh, xqh);
  }
  uint32_t sa[12 * NL], sb[12 * NL];
  const p6 fa = miller_pair<1, true>(pslot<1>{sa}, gl, nullptr, qa);
  const p6 fb = miller_pair<1, true>(pslot<1>{sb}, pl, nullptr, qb);
  const bool one = pr_is_one(pr_final_exp(pslot<1>{sa}, pr_mul(fa, fb)));
  if (s_inf || st == 1) return (s_inf && st == 1) ? 1 : 0;
  return one ? 1 : 0;
}

// the pair kernel's final exponentiation as a step program (pr_final_exp_fx, the
// product streaming x from the slot) against the chain of calls (the same
// template at level 1, which on the host runs the pair operations), limb by
// limb, on the quad schedule's Miller product of this check: 1 = identical
int bnc_fe_prog_vs_chain(const uint8_t* sig128, const uint8_t* m, uint64_t n, const uint8_t* pk128,
                         const uint8_t* gen128) {
  static uint32_t gl[N_LINES * LINE_WORDS], pl[N_LINES * LINE_WORDS];
  if (bnc_g2_lines(gen128, gl) != 0) return -1;
  g2a q;
  if (g2_decode(pk128, q) != 0) return -1;
  g2_lines(pl, q);
  uint8_t h[128];
  bnc_hash_to_g1(m, n, h);
  const fp hx = to_mont(from_be32(h + 1)), hy = to_mont(from_be32(h + 33));
  fp xqh, yqh, xs, ys, xq = fzero(), yq = fzero();
  line_point(hx, hy, true, xqh, yqh);
  bool s_inf;
  g1_decode(sig128, xs, ys, s_inf);
  if (s_inf) return -1;
  line_point(xs, ys, false, xq, yq);
  p1 qa[2], qb[2];
  for (int j = 0; j < PL; ++j) {
    qa[0].e[j] = qa[1].e[j] = fsel(prole(j), yq, xq);
    qb[0].e[j] = qb[1].e[j] = fsel(prole(j), yqh, xqh);
  }
  uint32_t sa[12 * NL], sb[12 * NL];
  const p6 fa = miller_pair<1, true>(pslot<1>{sa}, gl, nullptr, qa);
  const p6 fb = miller_pair<1, true>(pslot<1>{sb}, pl, nullptr, qb);
  const p6 f = pr_mul(fa, fb);
  const p6 r0 = pr_final_exp<1, 0>(pslot<1>{sa}, f);
  const p6 r1 = pr_final_exp<1, 1>(pslot<1>{sb}, f);
  return memcmp(&r0, &r1, sizeof r0) == 0 ? 1 : 0;
}

// the Fp multiplies / squarings of ONE check as k_bls_verify runs it (sigma
// decoding + bls_check; the lines and H(m) are per key / per message and are
// prepared before the counters are reset): out = {mul, sqr}
int bnc_check_counts(const uint8_t* sig128, const uint8_t* m, uint64_t n, const uint8_t* pk128, const uint8_t* gen128,
                     uint64_t* out) {
  static uint32_t gl[N_LINES * LINE_WORDS], pl[N_LINES * LINE_WORDS];
  if (bnc_g2_lines(gen128, gl) != 0 || bnc_g2_lines(pk128, pl) != 0) return -1;
  uint8_t h[128];
  bnc_hash_to_g1(m, n, h);
  const fp hx = to_mont(from_be32(h + 1)), hy = to_mont(from_be32(h + 33));
  fp xqh, yqh;
  line_point(hx, hy, true, xqh, yqh);
  g_cnt[0] = g_cnt[1] = 0;
  fp xs, ys;
  bool s_inf;
  g1_decode(sig128, xs, ys, s_inf);
  const int ok = bls_check(xs, ys, s_inf, xqh, yqh, false, gl, pl) ? 1 : 0;
  out[0] = g_cnt[0];
  out[1] = g_cnt[1];
  return ok;
}

// e(P, Q) on the kernel's schedule, 12 canonical 32-byte big-endian values
// in the order a.c0.a a.c0.b a.c1.a ... b.c2.b
void bnc_pairing(const uint8_t* g1b, const uint8_t* g2b, uint8_t* out) {
  static uint32_t ql[N_LINES * LINE_WORDS];
  bnc_g2_lines(g2b, ql);
  fp x, y;
  bool inf;
  g1_decode(g1b, x, y, inf);
  fp xq[1], yq[1];
  line_point(x, y, false, xq[0], yq[0]);
  const uint32_t* L[1] = {ql};
  const fp12 f = final_exp(miller_fixed<1>(L, xq, yq));
  const fp2* c[6] = {&f.a.c0, &f.a.c1, &f.a.c2, &f.b.c0, &f.b.c1, &f.b.c2};
  for (int j = 0; j < 6; ++j) {
    to_be32(out + 64 * j, from_mont(c[j]->a));
    to_be32(out + 64 * j + 32, from_mont(c[j]->b));
  }
}

static void put12(uint8_t* out, const fp12& f) {
  const fp2* c[6] = {&f.a.c0, &f.a.c1, &f.a.c2, &f.b.c0, &f.b.c1, &f.b.c2};
  for (int j = 0; j < 6; ++j) {
    to_be32(out + 64 * j, from_mont(c[j]->a));
    to_be32(out + 64 * j + 32, from_mont(c[j]->b));
  }
}
static fp12 get12(const uint8_t* in) {
  fp12 f;
  fp2* c[6] = {&f.a.c0, &f.a.c1, &f.a.c2, &f.b.c0, &f.b.c1, &f.b.c2};
  for (int j = 0; j < 6; ++j) {
    c[j]->a = to_mont(from_be32(in + 64 * j));
    c[j]->b = to_mont(from_be32(in + 64 * j + 32));
  }
  return f;
}
// debugging stages: the Miller value (kernel lines), f12 ops on canonical inputs
void bnc_miller(const uint8_t* g1b, const uint8_t* g2b, uint8_t* out) {
  static uint32_t ql[N_LINES * LINE_WORDS];
  bnc_g2_lines(g2b, ql);
  fp x, y;
  bool inf;
  g1_decode(g1b, x, y, inf);
  fp xq[1], yq[1];
  line_point(x, y, false, xq[0], yq[0]);
  const uint32_t* L[1] = {ql};
  put12(out, miller_fixed<1>(L, xq, yq));
}
void bnc_f12(int op, const uint8_t* a, const uint8_t* b, uint8_t* out) {
  const fp12 x = get12(a), y = get12(b);
  fp12 r;
  switch (op) {
    case 0: r = f12mul(x, y); break;
    case 1: r = f12sqr(x); break;
    case 2: r = f12inv(x); break;
    case 3: r = f12frob1(x); break;
    case 4: r = f12frob2(x); break;
    case 5: r = f12frob3(x); break;
    case 6: r = cyc_sqr(x); break;
    case 7: r = final_exp(x); break;
    case 8: r = cyc_pow_u(x); break;
    default: r = x;
  }
  put12(out, r);
}

// field self-test: a * b, a^2, a^-1 of plain 32-byte inputs, canonical plain outputs
void bnc_field(const uint8_t* a32, const uint8_t* b32, uint8_t* prod, uint8_t* sq, uint8_t* iv) {
  const fp a = to_mont(from_be32(a32)), b = to_mont(from_be32(b32));
  to_be32(prod, from_mont(mul(a, b)));
  to_be32(sq, from_mont(sqr(a)));
  to_be32(iv, from_mont(inv(a)));
}

}  // extern "C"
