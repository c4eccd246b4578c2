/* ORACLE (test infrastructure only -- never linked into the product):
 * plain-C restatement of the BLS signature check Plenum runs on every COMMIT,
 *
 *   BlsCryptoVerifierIndyCrypto.verify_sig(signature, message, pk)
 *     (crypto/bls/indy_crypto/bls_crypto_indy_crypto.py:73-82)
 *   -> python-ursa 0.1.1 Bls.verify(sig, msg, vk, gen)
 *        == ( e(sigma, g) == e(H(msg), pk) )
 *
 * over Milagro AMCL's BN254 (the curve python-ursa's `pair_amcl` backend uses:
 * u = -0x4080000000000001, E: y^2 = x^3 + 2, D-type sextic twist
 * E': y^2 = x^3 + 2/(1+i) over Fp2 = Fp[i]/(i^2+1)).
 *
 * PARITY UNPINNED: ursa (and AMCL) are not in /root/reference nor installed
 * anywhere here, and the reference holds no BLS signature, key or pairing
 * vector.  What IS pinned: the reference's one BLS constant, the G2 generator
 * (bls_crypto_indy_crypto.py:19), decodes under the encoding below to a point
 * of order r on exactly this twist (tests/test_bls_oracle.py), which fixes the
 * curve, the twist type and the G2 byte layout.  The rest restates ursa/AMCL's
 * published algorithms:
 *   - H(m) = PointG1::from_hash(SHA-256(m)): x = digest mod p, y =
 *     (x^3+2)^((p+1)/4) when x^3+2 is a non-zero square, else x += 1 and retry;
 *   - sigma: 128-byte representation, AMCL ECP::frombytes (0x04|x|y, or
 *     0x02/0x03|x compressed); x or y >= p, other prefixes or points off the
 *     curve decode to the point at infinity O;
 *   - pk / g: 128 bytes x.a|x.b|y.a|y.b (ECP2::frombytes), coordinates taken
 *     mod p, off-twist points decode to O;
 *   - e(O, Q) = e(P, O) = 1.
 *
 * The pairing here is written for obviousness and independence from the
 * kernel (csrc/pv_bn254.h): 4 x 64-bit Montgomery limbs, affine Miller loop on
 * the twist with unnormalised lines y_P + B' x_P w + C' v w, generic Fp12
 * multiplications, both pairings of the check computed separately and
 * compared (as ursa does), final exponentiation as f^((p^6-1)(p^2+1)) then a
 * 4-base multi-exponentiation of the hard part lambda = sum lambda_i p^i. */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef struct { uint64_t v[4]; } fp;      /* Montgomery form, fully reduced */
typedef struct { fp a, b; } fp2;           /* a + b i */
typedef struct { fp2 c[3]; } fp6;          /* c0 + c1 v + c2 v^2 */
typedef struct { fp6 a, b; } fp12;         /* a + b w */

/* p = 0x2523648240000001 ba344d8000000008 6121000000000013 a700000000000013, little-endian words */
static const uint64_t P[4] = {0xa700000000000013ull, 0x6121000000000013ull, 0xba344d8000000008ull, 0x2523648240000001ull};
static uint64_t N0;            /* -p^-1 mod 2^64 */
static fp R2, ONE, ZERO;       /* R^2 mod p (plain), 1 and 0 in Montgomery form */
static int inited;

/* ------------------------------------------------------------------ Fp */
static int geq_p(const uint64_t a[4]) {
  for (int i = 3; i >= 0; --i) {
    if (a[i] != P[i]) return a[i] > P[i];
  }
  return 1;
}

static void sub_p(uint64_t a[4]) {
  uint64_t br = 0;
  for (int i = 0; i < 4; ++i) {
    u128 t = (u128)a[i] - P[i] - br;
    a[i] = (uint64_t)t;
    br = (uint64_t)(t >> 64) & 1;
  }
}

static void fp_add(fp *r, const fp *x, const fp *y) {
  uint64_t c = 0, t[4];
  for (int i = 0; i < 4; ++i) {
    u128 s = (u128)x->v[i] + y->v[i] + c;
    t[i] = (uint64_t)s;
    c = (uint64_t)(s >> 64);
  }
  if (c || geq_p(t)) sub_p(t);
  memcpy(r->v, t, 32);
}

static void fp_sub(fp *r, const fp *x, const fp *y) {
  uint64_t br = 0, t[4];
  for (int i = 0; i < 4; ++i) {
    u128 s = (u128)x->v[i] - y->v[i] - br;
    t[i] = (uint64_t)s;
    br = (uint64_t)(s >> 64) & 1;
  }
  if (br) {
    uint64_t c = 0;
    for (int i = 0; i < 4; ++i) {
      u128 s = (u128)t[i] + P[i] + c;
      t[i] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
  }
  memcpy(r->v, t, 32);
}

static void fp_neg(fp *r, const fp *x) { fp_sub(r, &ZERO, x); }

/* CIOS Montgomery multiplication, R = 2^256 */
static void fp_mul(fp *r, const fp *x, const fp *y) {
  uint64_t t[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; ++i) {
    uint64_t c = 0;
    for (int j = 0; j < 4; ++j) {
      u128 s = (u128)x->v[j] * y->v[i] + t[j] + c;
      t[j] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
    u128 s = (u128)t[4] + c;
    t[4] = (uint64_t)s;
    t[5] = (uint64_t)(s >> 64);
    uint64_t m = t[0] * N0;
    s = (u128)m * P[0] + t[0];
    c = (uint64_t)(s >> 64);
    for (int j = 1; j < 4; ++j) {
      s = (u128)m * P[j] + t[j] + c;
      t[j - 1] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
    s = (u128)t[4] + c;
    t[3] = (uint64_t)s;
    t[4] = t[5] + (uint64_t)(s >> 64);
  }
  if (t[4] || geq_p(t)) sub_p(t);
  memcpy(r->v, t, 32);
}

static int fp_eq(const fp *x, const fp *y) { return !memcmp(x->v, y->v, 32); }
static int fp_iszero(const fp *x) { return fp_eq(x, &ZERO); }

/* big-endian 32 bytes -> plain integer words; returns 1 if < p */
static int words_be(uint64_t w[4], const uint8_t b[32]) {
  for (int i = 0; i < 4; ++i) {
    uint64_t x = 0;
    for (int k = 0; k < 8; ++k) x = x << 8 | b[8 * (3 - i) + k];
    w[i] = x;
  }
  return !geq_p(w);
}

static void fp_from_words(fp *r, const uint64_t w[4]) {   /* w < p, plain -> Montgomery */
  fp t;
  memcpy(t.v, w, 32);
  fp_mul(r, &t, &R2);
}

/* any 256-bit big-endian integer, reduced mod p (FP::new_big) */
static void fp_from_be_mod(fp *r, const uint8_t b[32]) {
  uint64_t w[4];
  words_be(w, b);
  while (geq_p(w)) sub_p(w);
  fp_from_words(r, w);
}

static void fp_to_be(uint8_t b[32], const fp *x) {
  fp one_plain = {{1, 0, 0, 0}}, t;
  fp_mul(&t, x, &one_plain);
  for (int i = 0; i < 4; ++i)
    for (int k = 0; k < 8; ++k) b[8 * (3 - i) + k] = (uint8_t)(t.v[i] >> (56 - 8 * k));
}

static void fp_from_u64(fp *r, uint64_t x) {
  uint64_t w[4] = {x, 0, 0, 0};
  fp_from_words(r, w);
}

/* x^e, e as little-endian 64-bit words */
static void fp_pow(fp *r, const fp *x, const uint64_t *e, int nw) {
  fp acc = ONE, b = *x;
  for (int i = 0; i < nw; ++i)
    for (int k = 0; k < 64; ++k) {
      if ((e[i] >> k) & 1) fp_mul(&acc, &acc, &b);
      fp_mul(&b, &b, &b);
    }
  *r = acc;
}

static uint64_t E_PM2[4], E_SQRT[4], E_LEG[4];   /* p-2, (p+1)/4, (p-1)/2 */

static void fp_inv(fp *r, const fp *x) { fp_pow(r, x, E_PM2, 4); }
static int fp_is_square(const fp *x) {            /* Legendre(x) == 1 */
  fp t;
  fp_pow(&t, x, E_LEG, 4);
  return fp_eq(&t, &ONE);
}

/* ------------------------------------------------------------------ Fp2 */
static void f2_add(fp2 *r, const fp2 *x, const fp2 *y) { fp_add(&r->a, &x->a, &y->a); fp_add(&r->b, &x->b, &y->b); }
static void f2_sub(fp2 *r, const fp2 *x, const fp2 *y) { fp_sub(&r->a, &x->a, &y->a); fp_sub(&r->b, &x->b, &y->b); }
static void f2_neg(fp2 *r, const fp2 *x) { fp_neg(&r->a, &x->a); fp_neg(&r->b, &x->b); }
static void f2_conj(fp2 *r, const fp2 *x) { r->a = x->a; fp_neg(&r->b, &x->b); }
static void f2_mul(fp2 *r, const fp2 *x, const fp2 *y) {
  fp t0, t1, t2, t3;
  fp_mul(&t0, &x->a, &y->a);
  fp_mul(&t1, &x->b, &y->b);
  fp_mul(&t2, &x->a, &y->b);
  fp_mul(&t3, &x->b, &y->a);
  fp_sub(&r->a, &t0, &t1);
  fp_add(&r->b, &t2, &t3);
}
static void f2_mul_fp(fp2 *r, const fp2 *x, const fp *s) { fp_mul(&r->a, &x->a, s); fp_mul(&r->b, &x->b, s); }
static void f2_mul_xi(fp2 *r, const fp2 *x) {   /* (a + b i)(1 + i) = (a - b) + (a + b) i */
  fp t;
  fp_sub(&t, &x->a, &x->b);
  fp_add(&r->b, &x->a, &x->b);
  r->a = t;
}
static void f2_inv(fp2 *r, const fp2 *x) {
  fp t0, t1;
  fp_mul(&t0, &x->a, &x->a);
  fp_mul(&t1, &x->b, &x->b);
  fp_add(&t0, &t0, &t1);
  fp_inv(&t0, &t0);
  fp_mul(&r->a, &x->a, &t0);
  fp_mul(&t1, &x->b, &t0);
  fp_neg(&r->b, &t1);
}
static int f2_eq(const fp2 *x, const fp2 *y) { return fp_eq(&x->a, &y->a) && fp_eq(&x->b, &y->b); }
static int f2_iszero(const fp2 *x) { return fp_iszero(&x->a) && fp_iszero(&x->b); }
static void f2_pow(fp2 *r, const fp2 *x, const uint64_t *e, int nw) {
  fp2 acc = {ONE, ZERO}, b = *x;
  for (int i = 0; i < nw; ++i)
    for (int k = 0; k < 64; ++k) {
      if ((e[i] >> k) & 1) f2_mul(&acc, &acc, &b);
      f2_mul(&b, &b, &b);
    }
  *r = acc;
}

/* ------------------------------------------------------------------ Fp6 / Fp12 */
static void f6_add(fp6 *r, const fp6 *x, const fp6 *y) { for (int k = 0; k < 3; ++k) f2_add(&r->c[k], &x->c[k], &y->c[k]); }
static void f6_sub(fp6 *r, const fp6 *x, const fp6 *y) { for (int k = 0; k < 3; ++k) f2_sub(&r->c[k], &x->c[k], &y->c[k]); }
static void f6_neg(fp6 *r, const fp6 *x) { for (int k = 0; k < 3; ++k) f2_neg(&r->c[k], &x->c[k]); }
static void f6_mul(fp6 *r, const fp6 *x, const fp6 *y) {   /* schoolbook, v^3 = xi */
  fp2 t[5], u;
  for (int k = 0; k < 5; ++k) memset(&t[k], 0, sizeof(fp2)), t[k].a = ZERO, t[k].b = ZERO;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      f2_mul(&u, &x->c[i], &y->c[j]);
      f2_add(&t[i + j], &t[i + j], &u);
    }
  f2_mul_xi(&u, &t[3]);
  f2_add(&r->c[0], &t[0], &u);
  f2_mul_xi(&u, &t[4]);
  f2_add(&r->c[1], &t[1], &u);
  r->c[2] = t[2];
}
static void f6_mul_v(fp6 *r, const fp6 *x) {
  fp2 t;
  f2_mul_xi(&t, &x->c[2]);
  r->c[2] = x->c[1];
  r->c[1] = x->c[0];
  r->c[0] = t;
}
static void f6_inv(fp6 *r, const fp6 *x) {
  fp2 t0, t1, t2, u, d;
  f2_mul(&t0, &x->c[0], &x->c[0]);
  f2_mul(&u, &x->c[1], &x->c[2]);
  f2_mul_xi(&u, &u);
  f2_sub(&t0, &t0, &u);
  f2_mul(&t1, &x->c[2], &x->c[2]);
  f2_mul_xi(&t1, &t1);
  f2_mul(&u, &x->c[0], &x->c[1]);
  f2_sub(&t1, &t1, &u);
  f2_mul(&t2, &x->c[1], &x->c[1]);
  f2_mul(&u, &x->c[0], &x->c[2]);
  f2_sub(&t2, &t2, &u);
  f2_mul(&d, &x->c[0], &t0);
  f2_mul(&u, &x->c[2], &t1);
  f2_mul_xi(&u, &u);
  f2_add(&d, &d, &u);
  f2_mul(&u, &x->c[1], &t2);
  f2_mul_xi(&u, &u);
  f2_add(&d, &d, &u);
  f2_inv(&d, &d);
  f2_mul(&r->c[0], &t0, &d);
  f2_mul(&r->c[1], &t1, &d);
  f2_mul(&r->c[2], &t2, &d);
}
static int f6_eq(const fp6 *x, const fp6 *y) {
  return f2_eq(&x->c[0], &y->c[0]) && f2_eq(&x->c[1], &y->c[1]) && f2_eq(&x->c[2], &y->c[2]);
}

static void f12_one(fp12 *r) {
  memset(r, 0, sizeof *r);
  for (int k = 0; k < 3; ++k) r->a.c[k].a = r->a.c[k].b = r->b.c[k].a = r->b.c[k].b = ZERO;
  r->a.c[0].a = ONE;
}
static void f12_mul(fp12 *r, const fp12 *x, const fp12 *y) {
  fp6 t0, t1, t2, t3;
  f6_mul(&t0, &x->a, &y->a);
  f6_mul(&t1, &x->b, &y->b);
  f6_mul(&t2, &x->a, &y->b);
  f6_mul(&t3, &x->b, &y->a);
  f6_mul_v(&t1, &t1);
  f6_add(&r->a, &t0, &t1);
  f6_add(&r->b, &t2, &t3);
}
static void f12_conj(fp12 *r, const fp12 *x) { r->a = x->a; f6_neg(&r->b, &x->b); }
static void f12_inv(fp12 *r, const fp12 *x) {
  fp6 t0, t1;
  f6_mul(&t0, &x->a, &x->a);
  f6_mul(&t1, &x->b, &x->b);
  f6_mul_v(&t1, &t1);
  f6_sub(&t0, &t0, &t1);
  f6_inv(&t0, &t0);
  f6_mul(&r->a, &x->a, &t0);
  f6_mul(&t1, &x->b, &t0);
  f6_neg(&r->b, &t1);
}
static int f12_eq(const fp12 *x, const fp12 *y) { return f6_eq(&x->a, &y->a) && f6_eq(&x->b, &y->b); }

/* Frobenius: x = sum_e c_e w^e (e = 2j + k for v^j w^k), x^p = sum conj(c_e) gamma_e w^e,
 * gamma_e = xi^(e (p-1)/6) */
static fp2 GAMMA[6];
static void f12_frob(fp12 *r, const fp12 *x) {
  fp2 c[6];
  for (int j = 0; j < 3; ++j) {
    c[2 * j] = x->a.c[j];
    c[2 * j + 1] = x->b.c[j];
  }
  for (int e = 0; e < 6; ++e) {
    f2_conj(&c[e], &c[e]);
    f2_mul(&c[e], &c[e], &GAMMA[e]);
  }
  for (int j = 0; j < 3; ++j) {
    r->a.c[j] = c[2 * j];
    r->b.c[j] = c[2 * j + 1];
  }
}

/* ------------------------------------------------------------------ curves */
typedef struct { fp x, y; int inf; } g1;
typedef struct { fp2 x, y; int inf; } g2;
static fp B1;        /* 2 */
static fp2 BT;       /* 2 / (1 + i) */

static int g1_on_curve(const fp *x, const fp *y) {
  fp l, r;
  fp_mul(&l, y, y);
  fp_mul(&r, x, x);
  fp_mul(&r, &r, x);
  fp_add(&r, &r, &B1);
  return fp_eq(&l, &r);
}

static int g2_on_curve(const fp2 *x, const fp2 *y) {
  fp2 l, r;
  f2_mul(&l, y, y);
  f2_mul(&r, x, x);
  f2_mul(&r, &r, x);
  f2_add(&r, &r, &BT);
  return f2_eq(&l, &r);
}

static void g1_add(g1 *r, const g1 *p, const g1 *q) {   /* affine, handles every case */
  if (p->inf) { *r = *q; return; }
  if (q->inf) { *r = *p; return; }
  fp lam, t, u;
  if (fp_eq(&p->x, &q->x)) {
    fp_add(&t, &p->y, &q->y);
    if (fp_iszero(&t)) { r->inf = 1; return; }
    fp_mul(&t, &p->x, &p->x);
    fp_add(&u, &t, &t);
    fp_add(&t, &u, &t);
    fp_add(&u, &p->y, &p->y);
  } else {
    fp_sub(&t, &q->y, &p->y);
    fp_sub(&u, &q->x, &p->x);
  }
  fp_inv(&u, &u);
  fp_mul(&lam, &t, &u);
  g1 o;
  fp_mul(&o.x, &lam, &lam);
  fp_sub(&o.x, &o.x, &p->x);
  fp_sub(&o.x, &o.x, &q->x);
  fp_sub(&t, &p->x, &o.x);
  fp_mul(&t, &lam, &t);
  fp_sub(&o.y, &t, &p->y);
  o.inf = 0;
  *r = o;
}

/* lam_out (the slope) is set to 0 when the line is vertical (q == -p) or a
 * point is O; the Miller loop never takes that case for points of G2 */
static void g2_add(g2 *r, const g2 *p, const g2 *q, fp2 *lam_out) {
  if (lam_out) lam_out->a = lam_out->b = ZERO;
  if (p->inf) { *r = *q; return; }
  if (q->inf) { *r = *p; return; }
  fp2 lam, t, u;
  if (f2_eq(&p->x, &q->x)) {
    f2_add(&t, &p->y, &q->y);
    if (f2_iszero(&t)) { r->inf = 1; return; }
    f2_mul(&t, &p->x, &p->x);
    f2_add(&u, &t, &t);
    f2_add(&t, &u, &t);
    f2_add(&u, &p->y, &p->y);
  } else {
    f2_sub(&t, &q->y, &p->y);
    f2_sub(&u, &q->x, &p->x);
  }
  f2_inv(&u, &u);
  f2_mul(&lam, &t, &u);
  if (lam_out) *lam_out = lam;
  g2 o;
  f2_mul(&o.x, &lam, &lam);
  f2_sub(&o.x, &o.x, &p->x);
  f2_sub(&o.x, &o.x, &q->x);
  f2_sub(&t, &p->x, &o.x);
  f2_mul(&t, &lam, &t);
  f2_sub(&o.y, &t, &p->y);
  o.inf = 0;
  *r = o;
}

/* k as 32-byte big-endian scalar */
static void g1_mul(g1 *r, const g1 *p, const uint8_t k[32]) {
  g1 acc;
  acc.inf = 1;
  for (int i = 0; i < 256; ++i) {
    g1_add(&acc, &acc, &acc);
    if ((k[i >> 3] >> (7 - (i & 7))) & 1) g1_add(&acc, &acc, p);
  }
  *r = acc;
}

static void g2_mul(g2 *r, const g2 *p, const uint8_t k[32]) {
  g2 acc;
  acc.inf = 1;
  for (int i = 0; i < 256; ++i) {
    g2_add(&acc, &acc, &acc, 0);
    if ((k[i >> 3] >> (7 - (i & 7))) & 1) g2_add(&acc, &acc, p, 0);
  }
  *r = acc;
}

/* ------------------------------------------------------------------ SHA-256 */
static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

static uint32_t ror(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

static void sha256_block(uint32_t h[8], const uint8_t *p) {
  uint32_t w[64];
  for (int i = 0; i < 16; ++i) w[i] = (uint32_t)p[4 * i] << 24 | p[4 * i + 1] << 16 | p[4 * i + 2] << 8 | p[4 * i + 3];
  for (int i = 16; i < 64; ++i) {
    uint32_t s0 = ror(w[i - 15], 7) ^ ror(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = ror(w[i - 2], 17) ^ ror(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], k = h[7];
  for (int i = 0; i < 64; ++i) {
    uint32_t t1 = k + (ror(e, 6) ^ ror(e, 11) ^ ror(e, 25)) + ((e & f) ^ (~e & g)) + K256[i] + w[i];
    uint32_t t2 = (ror(a, 2) ^ ror(a, 13) ^ ror(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    k = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += k;
}

static void sha256(const uint8_t *m, uint64_t n, uint8_t out[32]) {
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  uint64_t i = 0;
  for (; i + 64 <= n; i += 64) sha256_block(h, m + i);
  uint8_t buf[128];
  uint64_t rem = n - i;
  memcpy(buf, m + i, rem);
  buf[rem] = 0x80;
  uint64_t tot = rem + 9 <= 64 ? 64 : 128;
  memset(buf + rem + 1, 0, tot - rem - 1);
  for (int k = 0; k < 8; ++k) buf[tot - 1 - k] = (uint8_t)((n * 8) >> (8 * k));
  sha256_block(h, buf);
  if (tot == 128) sha256_block(h, buf + 64);
  for (int k = 0; k < 8; ++k) {
    out[4 * k] = h[k] >> 24; out[4 * k + 1] = h[k] >> 16; out[4 * k + 2] = h[k] >> 8; out[4 * k + 3] = h[k];
  }
}

/* ------------------------------------------------------------------ init */
static void init(void) {
  if (inited) return;
  /* N0 = -p^-1 mod 2^64 (Newton) */
  uint64_t x = 1;
  for (int i = 0; i < 7; ++i) x *= 2 - P[0] * x;
  N0 = (uint64_t)0 - x;
  /* R2 = 2^512 mod p by doubling (plain integers; add mod p is representation-free) */
  fp t = {{1, 0, 0, 0}};
  memset(&ZERO, 0, sizeof ZERO);
  for (int i = 0; i < 512; ++i) fp_add(&t, &t, &t);
  R2 = t;
  fp_from_u64(&ONE, 1);
  fp_from_u64(&B1, 2);
  /* exponents */
  memcpy(E_PM2, P, 32);
  E_PM2[0] -= 2;
  /* (p+1)/4 and (p-1)/2 */
  uint64_t pp1[4], c = 1;
  for (int i = 0; i < 4; ++i) {
    u128 s = (u128)P[i] + c;
    pp1[i] = (uint64_t)s;
    c = (uint64_t)(s >> 64);
  }
  for (int i = 0; i < 4; ++i) E_SQRT[i] = (pp1[i] >> 2) | (i < 3 ? pp1[i + 1] << 62 : 0);
  for (int i = 0; i < 4; ++i) E_LEG[i] = (P[i] >> 1) | (i < 3 ? P[i + 1] << 63 : 0);
  /* twist constant 2/(1+i) */
  fp2 xi = {ONE, ONE}, two = {B1, ZERO};
  f2_inv(&BT, &xi);
  f2_mul(&BT, &BT, &two);
  /* Frobenius gammas: xi^((p-1)/6 * e) */
  uint64_t e6[4];
  {
    uint64_t pm1[4];
    memcpy(pm1, P, 32);
    pm1[0] -= 1;
    /* divide by 6: long division on 64-bit words */
    u128 rem = 0;
    for (int i = 3; i >= 0; --i) {
      u128 cur = (rem << 64) | pm1[i];
      e6[i] = (uint64_t)(cur / 6);
      rem = cur % 6;
    }
  }
  fp2 g1c;
  f2_pow(&g1c, &xi, e6, 4);
  GAMMA[0].a = ONE;
  GAMMA[0].b = ZERO;
  for (int e = 1; e < 6; ++e) f2_mul(&GAMMA[e], &GAMMA[e - 1], &g1c);
  inited = 1;
}

/* hard part lambda = (p^4 - p^2 + 1)/r = l0 + l1 p + l2 p^2 + l3 p^3 with
 * l3 = 1, l2 = 6u^2 + 1, l1 = -36u^3 - 18u^2 - 12u + 1, l0 = -36u^3 - 30u^2 - 18u - 2
 * (all positive for u = -0x4080000000000001; checked in tests/_bn254_py.py) */
static const uint64_t LAM[4][4] = {
    {0xa100000000000016ull, 0xf393800000000010ull, 0x9366c48000000004ull, 0},
    {0x2a0000000000001full, 0xb696800000000015ull, 0x9366c48000000005ull, 0},
    {0x0600000000000007ull, 0x6181800000000003ull, 0, 0},
    {1, 0, 0, 0}};

/* ------------------------------------------------------------------ pairing */
static const uint64_t ATE = 0x8300000000000004ull;   /* |6u + 2| = 0x1_8300000000000004: bit 64 + these */
static int ate_bit(int i) { return i == 64 ? 1 : (int)((ATE >> i) & 1); }

/* line through T and S (both on the twist, affine, T == S: tangent) evaluated
 * at P: y_P + B' x_P w + C' v w, B' = -lambda, C' = lambda x_T - y_T; T <- T + S */
static void line_step(fp12 *l, g2 *T, const g2 *S, const g1 *p) {
  fp2 lam, t;
  g2 T0 = *T;
  g2_add(T, &T0, S, &lam);
  f12_one(l);
  l->a.c[0].a = p->y;
  fp2 bx;
  f2_mul_fp(&bx, &lam, &p->x);
  f2_neg(&l->b.c[0], &bx);
  f2_mul(&t, &lam, &T0.x);
  f2_sub(&l->b.c[1], &t, &T0.y);
}

static void g2_frob(g2 *r, const g2 *q) {     /* (conj(x) xi^((p-1)/3), conj(y) xi^((p-1)/2)) */
  f2_conj(&r->x, &q->x);
  f2_mul(&r->x, &r->x, &GAMMA[2]);
  f2_conj(&r->y, &q->y);
  f2_mul(&r->y, &r->y, &GAMMA[3]);
  r->inf = q->inf;
}

static void miller(fp12 *f, const g1 *p, const g2 *q) {
  f12_one(f);
  if (p->inf || q->inf) return;
  g2 T = *q;
  fp12 l;
  for (int i = 63; i >= 0; --i) {
    f12_mul(f, f, f);
    line_step(&l, &T, &T, p);
    f12_mul(f, f, &l);
    if (ate_bit(i)) {
      line_step(&l, &T, q, p);
      f12_mul(f, f, &l);
    }
  }
  /* 6u + 2 < 0 */
  f12_conj(f, f);
  f2_neg(&T.y, &T.y);
  g2 q1, q2;
  g2_frob(&q1, q);
  g2_frob(&q2, &q1);
  f2_neg(&q2.y, &q2.y);
  line_step(&l, &T, &q1, p);
  f12_mul(f, f, &l);
  line_step(&l, &T, &q2, p);
  f12_mul(f, f, &l);
}

static void final_exp(fp12 *r, const fp12 *f) {
  fp12 t, u;
  f12_inv(&t, f);
  f12_conj(&u, f);
  f12_mul(&t, &u, &t);            /* f^(p^6 - 1) */
  f12_frob(&u, &t);
  f12_frob(&u, &u);
  f12_mul(&t, &u, &t);            /* ^(p^2 + 1) */
  /* multi-exponentiation: prod_i (t^(p^i))^(lambda_i) */
  fp12 base[4];
  base[0] = t;
  for (int i = 1; i < 4; ++i) f12_frob(&base[i], &base[i - 1]);
  fp12 acc;
  f12_one(&acc);
  for (int bit = 191; bit >= 0; --bit) {
    f12_mul(&acc, &acc, &acc);
    for (int i = 0; i < 4; ++i)
      if ((LAM[i][bit >> 6] >> (bit & 63)) & 1) f12_mul(&acc, &acc, &base[i]);
  }
  *r = acc;
}

static void pairing(fp12 *r, const g1 *p, const g2 *q) {
  fp12 f;
  miller(&f, p, q);
  final_exp(r, &f);
}

/* ------------------------------------------------------------------ encodings */
static int g1_decode(g1 *p, const uint8_t *b, uint64_t len) {   /* 0: bad length (verify -> False) */
  if (len != 128) return 0;
  p->inf = 1;
  uint64_t w[4];
  if (!words_be(w, b + 1)) return 1;
  fp_from_words(&p->x, w);
  if (b[0] == 4) {
    if (!words_be(w, b + 33)) return 1;
    fp_from_words(&p->y, w);
    p->inf = !g1_on_curve(&p->x, &p->y);
  } else if (b[0] == 2 || b[0] == 3) {
    fp rhs;
    fp_mul(&rhs, &p->x, &p->x);
    fp_mul(&rhs, &rhs, &p->x);
    fp_add(&rhs, &rhs, &B1);
    if (!fp_is_square(&rhs)) return 1;
    fp_pow(&p->y, &rhs, E_SQRT, 4);
    uint8_t yb[32];
    fp_to_be(yb, &p->y);
    if ((yb[31] & 1) != (b[0] & 1)) fp_neg(&p->y, &p->y);
    p->inf = 0;
  }
  return 1;
}

static void g2_decode(g2 *q, const uint8_t b[128]) {
  fp_from_be_mod(&q->x.a, b);
  fp_from_be_mod(&q->x.b, b + 32);
  fp_from_be_mod(&q->y.a, b + 64);
  fp_from_be_mod(&q->y.b, b + 96);
  q->inf = !g2_on_curve(&q->x, &q->y);
}

static void g1_encode(uint8_t b[128], const g1 *p) {
  memset(b, 0, 128);
  if (p->inf) return;
  b[0] = 4;
  fp_to_be(b + 1, &p->x);
  fp_to_be(b + 33, &p->y);
}

static void g2_encode(uint8_t b[128], const g2 *q) {
  memset(b, 0, 128);
  if (q->inf) return;
  fp_to_be(b, &q->x.a);
  fp_to_be(b + 32, &q->x.b);
  fp_to_be(b + 64, &q->y.a);
  fp_to_be(b + 96, &q->y.b);
}

static void hash_to_g1(g1 *h, const uint8_t *m, uint64_t n) {
  uint8_t d[32];
  sha256(m, n, d);
  for (;;) {
    fp rhs;
    fp_from_be_mod(&h->x, d);
    fp_mul(&rhs, &h->x, &h->x);
    fp_mul(&rhs, &rhs, &h->x);
    fp_add(&rhs, &rhs, &B1);
    if (fp_is_square(&rhs)) {
      fp_pow(&h->y, &rhs, E_SQRT, 4);
      h->inf = 0;
      return;
    }
    for (int k = 31; k >= 0 && ++d[k] == 0; --k) {
    }
  }
}

/* ------------------------------------------------------------------ exported */
int bls_oracle_verify(const uint8_t *sig, uint64_t sig_len, const uint8_t *msg, uint64_t mlen, const uint8_t pk[128],
                      const uint8_t gen[128]) {
  init();
  g1 s, h;
  g2 g, q;
  if (!g1_decode(&s, sig, sig_len)) return 0;
  g2_decode(&g, gen);
  g2_decode(&q, pk);
  hash_to_g1(&h, msg, mlen);
  fp12 e1, e2;
  pairing(&e1, &s, &g);
  pairing(&e2, &h, &q);
  return f12_eq(&e1, &e2);
}

/* e(P, Q) as 12 x 32-byte big-endian Fp values in the order
 * a.c0.a a.c0.b a.c1.a ... b.c2.b (tests cross-check with tests/_bn254_py.py) */
void bls_oracle_pairing(const uint8_t g1b[128], const uint8_t g2b[128], uint8_t out[384]) {
  init();
  g1 p;
  g2 q;
  g1_decode(&p, g1b, 128);
  g2_decode(&q, g2b);
  fp12 e;
  pairing(&e, &p, &q);
  const fp6 *h[2] = {&e.a, &e.b};
  for (int k = 0; k < 2; ++k)
    for (int j = 0; j < 3; ++j) {
      fp_to_be(out + 192 * k + 64 * j, &h[k]->c[j].a);
      fp_to_be(out + 192 * k + 64 * j + 32, &h[k]->c[j].b);
    }
}

void bls_oracle_hash_to_g1(const uint8_t *msg, uint64_t mlen, uint8_t out[128]) {
  init();
  g1 h;
  hash_to_g1(&h, msg, mlen);
  g1_encode(out, &h);
}

/* sk: 32-byte big-endian scalar; sign: sk * H(m) (ursa Bls::sign), pubkey: sk * g */
void bls_oracle_sign(const uint8_t sk[32], const uint8_t *msg, uint64_t mlen, uint8_t out[128]) {
  init();
  g1 h, s;
  hash_to_g1(&h, msg, mlen);
  g1_mul(&s, &h, sk);
  g1_encode(out, &s);
}

void bls_oracle_pubkey(const uint8_t sk[32], const uint8_t gen[128], uint8_t out[128]) {
  init();
  g2 g, q;
  g2_decode(&g, gen);
  g2_mul(&q, &g, sk);
  g2_encode(out, &q);
}

/* 1 if the 128-byte G2 encoding decodes to a point P != O with r P = O */
int bls_oracle_g2_in_subgroup(const uint8_t b[128]) {
  init();
  static const uint8_t RB[32] = {0x25, 0x23, 0x64, 0x82, 0x40, 0x00, 0x00, 0x01, 0xba, 0x34, 0x4d,
                                 0x80, 0x00, 0x00, 0x00, 0x07, 0xff, 0x9f, 0x80, 0x00, 0x00, 0x00,
                                 0x00, 0x10, 0xa1, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x0d};
  g2 q, t;
  g2_decode(&q, b);
  if (q.inf) return 0;
  g2_mul(&t, &q, RB);
  return t.inf;
}

/* ursa Bls::verify_multi_sig (crypto/bls/indy_crypto/bls_crypto_indy_crypto.py:84-97):
 * e(sigma, g) == e(H(msg), pk_0 + ... + pk_{k-1}), the keys decoded as keys are
 * (off the twist = O) and summed from O. */
int bls_oracle_verify_multi(const uint8_t *sig, uint64_t sig_len, const uint8_t *msg, uint64_t mlen,
                            const uint8_t *pks, uint64_t k, const uint8_t gen[128]) {
  init();
  g1 s, h;
  g2 g, agg, q;
  if (!g1_decode(&s, sig, sig_len)) return 0;
  g2_decode(&g, gen);
  agg.inf = 1;
  for (uint64_t t = 0; t < k; ++t) {
    g2_decode(&q, pks + 128 * t);
    g2_add(&agg, &agg, &q, 0);
  }
  hash_to_g1(&h, msg, mlen);
  fp12 e1, e2;
  pairing(&e1, &s, &g);
  pairing(&e2, &h, &agg);
  return f12_eq(&e1, &e2);
}

/* 128-byte representation of the sum of k G2 keys (O: 128 zero bytes) */
void bls_oracle_aggregate_keys(const uint8_t *pks, uint64_t k, uint8_t out[128]) {
  init();
  g2 agg, q;
  agg.inf = 1;
  for (uint64_t t = 0; t < k; ++t) {
    g2_decode(&q, pks + 128 * t);
    g2_add(&agg, &agg, &q, 0);
  }
  g2_encode(out, &agg);
}

/* ursa MultiSignature::new (:99-102): the sum of k signatures' G1 points (each
 * decoded as sigma is: 128 bytes, O when it does not decode), as ECP::tobytes
 * writes it: 0x04|x|y, and O as 0x04|0|1 (AMCL's affine (0, 1) of infinity). */
void bls_oracle_aggregate_sigs(const uint8_t *sigs, uint64_t k, uint8_t out[128]) {
  init();
  g1 agg, s;
  agg.inf = 1;
  for (uint64_t t = 0; t < k; ++t) {
    g1_decode(&s, sigs + 128 * t, 128);
    g1_add(&agg, &agg, &s);
  }
  g1_encode(out, &agg);
  if (agg.inf) {
    out[0] = 4;
    out[64] = 1;
  }
}

/* batch: check j = (sig j, message msg_idx[j] of blob/off, key key_idx[j] of keys), threads workers */
typedef struct {
  const uint8_t *sigs, *blob, *keys, *gen;
  const uint64_t *off, *sig_len;
  const uint32_t *msg_idx, *key_idx;
  uint8_t *out;
  uint64_t lo, hi;
} bjob;

static void *bworker(void *arg) {
  bjob *j = (bjob *)arg;
  for (uint64_t i = j->lo; i < j->hi; ++i) {
    const uint32_t m = j->msg_idx[i];
    j->out[i] = (uint8_t)bls_oracle_verify(j->sigs + 128 * i, j->sig_len ? j->sig_len[i] : 128, j->blob + j->off[m],
                                           j->off[m + 1] - j->off[m], j->keys + 128 * (uint64_t)j->key_idx[i], j->gen);
  }
  return 0;
}

void bls_oracle_verify_batch(const uint8_t *sigs, const uint64_t *sig_len, const uint8_t *blob, const uint64_t *off,
                             const uint32_t *msg_idx, const uint32_t *key_idx, const uint8_t *keys,
                             const uint8_t *gen, uint64_t n, uint8_t *out, int threads) {
  init();
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t th[256];
  bjob jobs[256];
  for (int t = 0; t < threads; ++t) {
    jobs[t] = (bjob){sigs, blob, keys, gen, off, sig_len, msg_idx, key_idx, out, n * t / threads, n * (t + 1) / threads};
    pthread_create(&th[t], 0, bworker, &jobs[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], 0);
}
