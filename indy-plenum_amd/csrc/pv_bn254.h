// BN254 (Milagro AMCL's curve -- the one python-ursa 0.1.1's BLS uses) for the
// batch BLS COMMIT check, one check per lane.  SURVEY.md §8 row f4:
//   BlsBftReplicaPlenum._validate_signature (plenum/bls/bls_bft_replica_plenum.py:194-213)
//   -> BlsCryptoVerifierIndyCrypto.verify_sig (crypto/bls/indy_crypto/bls_crypto_indy_crypto.py:73-82)
//   -> ursa Bls.verify: e(sigma, g) == e(H(m), pk).
// Here: e(sigma, g) * e(-H(m), pk) == 1 as ONE product of Miller loops with
// ONE final exponentiation (both G2 arguments are fixed -- the group generator
// and the node's key -- so their lines are precomputed once per key set).
//
// Field: GF(p), p = 0x2523648240000001ba344d80000000086121000000000013a700000000000013
// (254 bits), 10 signed 32-bit limbs of 28 bits, Montgomery form with R = 2^280.
// Products are 64-bit column sums of v_mad_i64_i32 (product scanning, one
// carry per column).  Values are SIGNED: a - b is a limbwise subtraction and a
// multiply of any two operands of magnitude < 2^266 returns a value in
// (-p/2, 3p/2), so sums and differences feed multiplies without reductions;
// only equality tests and encodings reduce to [0, p) (canon).
//
// Limb discipline (host bound-checking build: tools/hostcheck checks every
// multiply's column sums against 2^63):
//   normalised : limbs 0..8 in [0, 2^28), limb 9 signed (mul / sqr / norm outputs)
//   lazy       : |limbs| < 2^29 (one add or sub of two normalised values)
//   mul / sqr take lazy operands: a column sums 10 products < 2^58 and 8
//   reduction products < 2^56: < 2^62.
// Tower: Fp2 = Fp[i]/(i^2+1), Fp6 = Fp2[v]/(v^3 - xi), Fp12 = Fp6[w]/(w^2 - v),
// xi = 1 + i (tests/_bn254_py.py is the readable restatement of every formula).
#pragma once
#include <stdint.h>
#include "pv_bn254_consts.h"

#ifndef PV_HD
#define PV_HD __host__ __device__ __forceinline__
#endif
// the heavy building blocks (Fp6 / Fp12 products, squarings, Frobenius maps,
// exponentiations, point steps) are out-of-line functions: fully inlined, one
// check is ~10^6 instructions and hipcc takes most of an hour
#ifndef PV_BN_CALL
#if defined(__HIPCC__)
#define PV_BN_CALL __device__ __noinline__
#else
#define PV_BN_CALL static __attribute__((noinline))
#endif
#endif
#ifndef PV_BN_CHECK_MUL
#define PV_BN_CHECK_MUL(a, b)
#endif
#ifndef PV_BN_COUNT
#define PV_BN_COUNT(kind)
#endif

namespace bn {

static constexpr int32_t M28 = (1 << 28) - 1;
static constexpr int NL = 10;

struct fp {
  int32_t l[NL];
};
struct fp2 {
  fp a, b;
};
struct fp6 {
  fp2 c0, c1, c2;
};
struct fp12 {
  fp6 a, b;
};

PV_HD fp cst(const uint32_t* c) {
  fp r;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.l[i] = (int32_t)c[i];
  return r;
}
PV_HD fp fzero() {
  fp r;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.l[i] = 0;
  return r;
}
PV_HD fp fone() { return cst(ONE_M); }

// ------------------------------------------------------------------ Fp
// Montgomery product a b / 2^280 (mod p): signed column sums, the reduction
// multiples m_k in [0, 2^28) (p's zero limbs 1 and 3 skipped)
PV_HD fp mul(const fp& a, const fp& b) {
  PV_BN_CHECK_MUL(a, b);
  PV_BN_COUNT(0);
  int32_t m[NL];
  fp r;
  int64_t carry = 0;
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    int64_t acc = carry;
#pragma unroll
    for (int i = 0; i <= k; ++i) acc += (int64_t)a.l[i] * b.l[k - i];
#pragma unroll
    for (int i = 0; i < k; ++i)
      if (P_L[k - i]) acc += (int64_t)m[i] * (int32_t)P_L[k - i];
    m[k] = (int32_t)(((uint32_t)acc * NP) & (uint32_t)M28);
    acc += (int64_t)m[k] * (int32_t)P_L[0];
    carry = acc >> 28;
  }
#pragma unroll
  for (int k = NL; k < 2 * NL - 1; ++k) {
    int64_t acc = carry;
#pragma unroll
    for (int i = k - NL + 1; i < NL; ++i) acc += (int64_t)a.l[i] * b.l[k - i];
#pragma unroll
    for (int i = k - NL + 1; i < NL; ++i)
      if (P_L[k - i]) acc += (int64_t)m[i] * (int32_t)P_L[k - i];
    r.l[k - NL] = (int32_t)(acc & M28);
    carry = acc >> 28;
  }
  r.l[NL - 1] = (int32_t)carry;
  return r;
}

// squaring: the cross products once, through one pre-doubled operand
PV_HD fp sqr(const fp& a) {
  PV_BN_CHECK_MUL(a, a);
  PV_BN_COUNT(1);
  int32_t m[NL], d[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) d[i] = a.l[i] * 2;   // |d| < 2^30
  fp r;
  int64_t carry = 0;
#pragma unroll
  for (int k = 0; k < 2 * NL - 1; ++k) {
    int64_t acc = carry;
#pragma unroll
    for (int i = (k < NL ? 0 : k - NL + 1); 2 * i < k; ++i) acc += (int64_t)a.l[i] * d[k - i];
    if ((k & 1) == 0) acc += (int64_t)a.l[k / 2] * a.l[k / 2];
    if (k < NL) {
#pragma unroll
      for (int i = 0; i < k; ++i)
        if (P_L[k - i]) acc += (int64_t)m[i] * (int32_t)P_L[k - i];
      m[k] = (int32_t)(((uint32_t)acc * NP) & (uint32_t)M28);
      acc += (int64_t)m[k] * (int32_t)P_L[0];
    } else {
#pragma unroll
      for (int i = k - NL + 1; i < NL; ++i)
        if (P_L[k - i]) acc += (int64_t)m[i] * (int32_t)P_L[k - i];
      r.l[k - NL] = (int32_t)(acc & M28);
    }
    carry = acc >> 28;
  }
  r.l[NL - 1] = (int32_t)carry;
  return r;
}

// signed carry propagation: limbs 0..8 to [0, 2^28), limb 9 takes the sign
PV_HD fp norm(const fp& a) {
  fp r;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < NL - 1; ++i) {
    const int32_t v = a.l[i] + c;
    r.l[i] = v & M28;
    c = v >> 28;
  }
  r.l[NL - 1] = a.l[NL - 1] + c;
  return r;
}

// lazy (limbwise)
PV_HD fp add(const fp& a, const fp& b) {
  fp r;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.l[i] = a.l[i] + b.l[i];
  return r;
}
PV_HD fp sub(const fp& a, const fp& b) {
  fp r;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.l[i] = a.l[i] - b.l[i];
  return r;
}
PV_HD fp neg(const fp& b) {
  fp r;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.l[i] = -b.l[i];
  return r;
}
// normalised sums / differences
PV_HD fp addn(const fp& a, const fp& b) { return norm(add(a, b)); }
PV_HD fp subn(const fp& a, const fp& b) { return norm(sub(a, b)); }
PV_HD fp negn(const fp& a) { return norm(neg(a)); }
PV_HD fp dbl(const fp& a) { return norm(add(a, a)); }

// a normalised value of any magnitude < 2^282 -> the same residue with
// magnitude < 3p: subtract q p, q = floor(top limb * 2^252 / p) estimated as
// (top * floor(2^284 / p)) >> 32.  For the few add/sub chains that feed back
// into themselves without a multiply (the twist point of the line
// precomputation, Granger-Scott squarings), which otherwise double per step.
PV_HD fp reduce(const fp& a) {
  const int64_t q = ((int64_t)a.l[NL - 1] * QC) >> 32;
  fp r;
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int64_t v = (int64_t)a.l[i] - q * (int64_t)P_L[i] + c;
    if (i < NL - 1) {
      r.l[i] = (int32_t)(v & M28);
      c = v >> 28;
    } else {
      r.l[i] = (int32_t)v;
    }
  }
  return r;
}

// a normalised value in (-p, 2p) -> [0, p)
PV_HD fp fold(const fp& t) {
  fp lo, hi;   // t + p, t - p
  int32_t c0 = 0, c1 = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int32_t x = t.l[i] + (int32_t)P_L[i] + c0;
    const int32_t y = t.l[i] - (int32_t)P_L[i] + c1;
    lo.l[i] = i < NL - 1 ? (x & M28) : x;
    hi.l[i] = i < NL - 1 ? (y & M28) : y;
    c0 = x >> 28;
    c1 = y >> 28;
  }
  const bool neg_t = t.l[NL - 1] < 0;
  const bool ge_p = hi.l[NL - 1] >= 0;
  fp r;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.l[i] = neg_t ? lo.l[i] : (ge_p ? hi.l[i] : t.l[i]);
  return r;
}
// the canonical Montgomery representative of a (any operand a multiply takes)
PV_HD fp canon(const fp& a) { return fold(mul(a, cst(ONE_M))); }
PV_HD bool is_zero(const fp& a) {
  const fp c = canon(a);
  int32_t d = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) d |= c.l[i];
  return d == 0;
}
PV_HD bool eq(const fp& a, const fp& b) { return is_zero(sub(a, b)); }

// plain integer (limbs, value < 2^280) -> Montgomery form
PV_HD fp to_mont(const fp& x) { return mul(x, cst(R2_L)); }
// Montgomery -> plain canonical integer in [0, p)
PV_HD fp from_mont(const fp& a) {
  fp one = fzero();
  one.l[0] = 1;
  return fold(mul(a, one));
}

// 32-byte big-endian integer -> plain limbs (value < 2^256)
PV_HD fp from_be32(const uint8_t* b) {
  fp r = fzero();
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    const int bit = 8 * (31 - k);
    const int32_t v = b[k];
    r.l[bit / 28] |= (v << (bit % 28)) & M28;
    if (bit % 28 > 20) r.l[bit / 28 + 1] |= v >> (28 - bit % 28);
  }
  return r;
}
PV_HD void to_be32(uint8_t* b, const fp& x) {   // x plain, canonical
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    const int bit = 8 * (31 - k);
    uint32_t v = (uint32_t)x.l[bit / 28] >> (bit % 28);
    if (bit % 28 > 20 && bit / 28 + 1 < NL) v |= (uint32_t)x.l[bit / 28 + 1] << (28 - bit % 28);
    b[k] = (uint8_t)v;
  }
}
// plain non-negative limbs < p ?
PV_HD bool lt_p(const fp& x) {
  int32_t br = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int32_t t = x.l[i] - (int32_t)P_L[i] + br;
    br = t >> 28;
  }
  return br < 0;
}

// x^e for a fixed 256-bit exponent (little-endian words, uniform branches)
PV_BN_CALL fp pow_fixed(const fp& x, const uint64_t* e) {
  fp acc = fone(), b = x;
  for (int w = 0; w < 4; ++w) {
    const uint64_t ew = e[w];
    for (int k = 0; k < 64; ++k) {
      if ((ew >> k) & 1) acc = mul(acc, b);
      if (w < 3 || (ew >> k) > 1) b = sqr(b);
    }
  }
  return acc;
}
PV_HD fp inv(const fp& x) { return pow_fixed(x, E_PM2); }

// ------------------------------------------------------------------ Fp2
PV_HD fp2 f2(const fp& a, const fp& b) { return fp2{a, b}; }
PV_HD fp2 f2zero() { return fp2{fzero(), fzero()}; }
PV_HD fp2 f2one() { return fp2{fone(), fzero()}; }
PV_HD fp2 f2cst(const uint32_t* a, const uint32_t* b) { return fp2{cst(a), cst(b)}; }
PV_HD fp2 f2add(const fp2& x, const fp2& y) { return fp2{addn(x.a, y.a), addn(x.b, y.b)}; }
PV_HD fp2 f2sub(const fp2& x, const fp2& y) { return fp2{subn(x.a, y.a), subn(x.b, y.b)}; }
PV_HD fp2 f2neg(const fp2& x) { return fp2{negn(x.a), negn(x.b)}; }
PV_HD fp2 f2conj(const fp2& x) { return fp2{x.a, negn(x.b)}; }
PV_HD fp2 f2dbl(const fp2& x) { return fp2{dbl(x.a), dbl(x.b)}; }
// (a + b i)(c + d i), Karatsuba; operands lazy or normalised
PV_HD fp2 f2mul(const fp2& x, const fp2& y) {
  const fp t0 = mul(x.a, y.a), t1 = mul(x.b, y.b);
  const fp t2 = mul(add(x.a, x.b), add(y.a, y.b));
  return fp2{subn(t0, t1), subn(sub(t2, t0), t1)};
}
PV_HD fp2 f2sqr(const fp2& x) {   // (a+b)(a-b), 2ab
  const fp t = mul(x.a, x.b);
  return fp2{mul(add(x.a, x.b), sub(x.a, x.b)), dbl(t)};
}
PV_HD fp2 f2mulfp(const fp2& x, const fp& s) { return fp2{mul(x.a, s), mul(x.b, s)}; }
PV_HD fp2 f2mulxi(const fp2& x) { return fp2{subn(x.a, x.b), addn(x.a, x.b)}; }   // (a + bi)(1 + i)
PV_HD fp2 f2reduce(const fp2& x) { return fp2{reduce(x.a), reduce(x.b)}; }
PV_HD bool f2eq(const fp2& x, const fp2& y) { return eq(x.a, y.a) && eq(x.b, y.b); }
PV_HD bool f2is_zero(const fp2& x) { return is_zero(x.a) && is_zero(x.b); }
PV_HD fp2 f2inv(const fp2& x) {
  const fp t = inv(addn(sqr(x.a), sqr(x.b)));
  return fp2{mul(x.a, t), negn(mul(x.b, t))};
}

// ------------------------------------------------------------------ Fp6
PV_HD fp6 f6zero() { return fp6{f2zero(), f2zero(), f2zero()}; }
PV_HD fp6 f6one() { return fp6{f2one(), f2zero(), f2zero()}; }
PV_HD fp6 f6add(const fp6& x, const fp6& y) { return fp6{f2add(x.c0, y.c0), f2add(x.c1, y.c1), f2add(x.c2, y.c2)}; }
PV_HD fp6 f6sub(const fp6& x, const fp6& y) { return fp6{f2sub(x.c0, y.c0), f2sub(x.c1, y.c1), f2sub(x.c2, y.c2)}; }
PV_HD fp6 f6neg(const fp6& x) { return fp6{f2neg(x.c0), f2neg(x.c1), f2neg(x.c2)}; }
PV_HD fp6 f6mulv(const fp6& x) { return fp6{f2mulxi(x.c2), x.c0, x.c1}; }
// lazy Fp2 helpers (limbwise, no carry pass) for sums of normalised values
// that are normalised once at the end: |limb| stays below 2^31
PV_HD fp2 f2addL(const fp2& x, const fp2& y) { return fp2{add(x.a, y.a), add(x.b, y.b)}; }
PV_HD fp2 f2subL(const fp2& x, const fp2& y) { return fp2{sub(x.a, y.a), sub(x.b, y.b)}; }
PV_HD fp2 f2mulxiL(const fp2& x) { return fp2{sub(x.a, x.b), add(x.a, x.b)}; }
PV_HD fp2 f2norm(const fp2& x) { return fp2{norm(x.a), norm(x.b)}; }

// Karatsuba over Fp2 (6 Fp2 products); each output coefficient is one lazy
// combination of normalised products (|limb| < 7 * 2^28) and one carry pass
PV_HD fp6 f6mul_i(const fp6& a, const fp6& b) {
  const fp2 v0 = f2mul(a.c0, b.c0), v1 = f2mul(a.c1, b.c1), v2 = f2mul(a.c2, b.c2);
  const fp2 s12 = f2mul(f2addL(a.c1, a.c2), f2addL(b.c1, b.c2));
  const fp2 s01 = f2mul(f2addL(a.c0, a.c1), f2addL(b.c0, b.c1));
  const fp2 s02 = f2mul(f2addL(a.c0, a.c2), f2addL(b.c0, b.c2));
  fp6 r;
  r.c0 = f2norm(f2addL(f2mulxiL(f2subL(f2subL(s12, v1), v2)), v0));
  r.c1 = f2norm(f2addL(f2subL(f2subL(s01, v0), v1), f2mulxiL(v2)));
  r.c2 = f2norm(f2addL(f2subL(f2subL(s02, v0), v2), v1));
  return r;
}
PV_BN_CALL fp6 f6mul(const fp6& a, const fp6& b) { return f6mul_i(a, b); }
// x * (b0 + b1 v): 5 Fp2 products
PV_HD fp6 f6mul01(const fp6& x, const fp2& b0, const fp2& b1) {
  const fp2 t0 = f2mul(x.c0, b0), t1 = f2mul(x.c1, b1), t2 = f2mul(x.c2, b0), t3 = f2mul(x.c2, b1);
  const fp2 m = f2mul(f2addL(x.c0, x.c1), f2addL(b0, b1));
  fp6 r;
  r.c0 = f2norm(f2addL(t0, f2mulxiL(t3)));
  r.c1 = f2norm(f2subL(f2subL(m, t0), t1));
  r.c2 = f2norm(f2addL(t1, t2));
  return r;
}
PV_BN_CALL fp6 f6inv(const fp6& x) {
  const fp2 t0 = f2sub(f2sqr(x.c0), f2mulxi(f2mul(x.c1, x.c2)));
  const fp2 t1 = f2sub(f2mulxi(f2sqr(x.c2)), f2mul(x.c0, x.c1));
  const fp2 t2 = f2sub(f2sqr(x.c1), f2mul(x.c0, x.c2));
  const fp2 d = f2inv(f2add(f2add(f2mul(x.c0, t0), f2mulxi(f2mul(x.c2, t1))), f2mulxi(f2mul(x.c1, t2))));
  return fp6{f2mul(t0, d), f2mul(t1, d), f2mul(t2, d)};
}

// ------------------------------------------------------------------ Fp12
PV_HD fp12 f12one() { return fp12{f6one(), f6zero()}; }
PV_HD fp12 f12conj(const fp12& x) { return fp12{x.a, f6neg(x.b)}; }
PV_BN_CALL fp12 f12mul(const fp12& x, const fp12& y) {   // Karatsuba: 3 Fp6 products
  const fp6 t0 = f6mul(x.a, y.a), t1 = f6mul(x.b, y.b);
  const fp6 s = f6mul(f6add(x.a, x.b), f6add(y.a, y.b));
  fp12 r;
  r.a.c0 = f2norm(f2addL(t0.c0, f2mulxiL(t1.c2)));
  r.a.c1 = f2norm(f2addL(t0.c1, t1.c0));
  r.a.c2 = f2norm(f2addL(t0.c2, t1.c1));
  r.b.c0 = f2norm(f2subL(f2subL(s.c0, t0.c0), t1.c0));
  r.b.c1 = f2norm(f2subL(f2subL(s.c1, t0.c1), t1.c1));
  r.b.c2 = f2norm(f2subL(f2subL(s.c2, t0.c2), t1.c2));
  return r;
}
PV_HD fp12 f12sqr_i(const fp12& x) {   // complex squaring: 2 Fp6 products
  const fp6 t = f6mul_i(x.a, x.b);
  const fp6 s = f6mul_i(f6add(x.a, x.b), f6add(x.a, f6mulv(x.b)));
  fp12 r;   // (s - t - v t) + 2t w
  r.a.c0 = f2norm(f2subL(f2subL(s.c0, t.c0), f2mulxiL(t.c2)));
  r.a.c1 = f2norm(f2subL(f2subL(s.c1, t.c1), t.c0));
  r.a.c2 = f2norm(f2subL(f2subL(s.c2, t.c2), t.c1));
  r.b = fp6{f2dbl(t.c0), f2dbl(t.c1), f2dbl(t.c2)};
  return r;
}
PV_BN_CALL fp12 f12sqr(const fp12& x) { return f12sqr_i(x); }
PV_BN_CALL fp12 f12inv(const fp12& x) {
  const fp6 d = f6inv(f6sub(f6mul(x.a, x.a), f6mulv(f6mul(x.b, x.b))));
  return fp12{f6mul(x.a, d), f6neg(f6mul(x.b, d))};
}
// f * (1 + (b0 + b1 v) w): the normalised line (5 + 5 Fp2 products)
PV_HD fp12 f12mul_line_i(const fp12& f, const fp2& b0, const fp2& b1) {
  const fp6 t = f6mul01(f.b, b0, b1);
  const fp6 s = f6mul01(f.a, b0, b1);
  fp12 r;   // (f.a + v t) + (f.b + s) w, one carry pass per coefficient
  r.a.c0 = f2norm(f2addL(f.a.c0, f2mulxiL(t.c2)));
  r.a.c1 = f2norm(f2addL(f.a.c1, t.c0));
  r.a.c2 = f2norm(f2addL(f.a.c2, t.c1));
  r.b = f6add(f.b, s);
  return r;
}
PV_BN_CALL fp12 f12mul_line(const fp12& f, const fp2& b0, const fp2& b1) { return f12mul_line_i(f, b0, b1); }
PV_HD bool f12is_one(const fp12& x) {
  bool ok = eq(x.a.c0.a, fone()) && is_zero(x.a.c0.b);
  ok = ok && f2is_zero(x.a.c1) && f2is_zero(x.a.c2);
  ok = ok && f2is_zero(x.b.c0) && f2is_zero(x.b.c1) && f2is_zero(x.b.c2);
  return ok;
}

// Frobenius x -> x^(p^n): coefficient of w^e (e = 2j + k for v^j w^k) becomes
// conj^n(c_e) * xi^(e (p^n - 1)/6)
PV_HD fp2 frob_c(const fp2& c, int n, const uint32_t* ga, const uint32_t* gb) {
  const fp2 x = (n & 1) ? f2conj(c) : c;
  return f2mul(x, f2cst(ga, gb));
}
PV_BN_CALL fp12 f12frob1(const fp12& x) {
  fp12 r;
  r.a.c0 = f2conj(x.a.c0);
  r.b.c0 = frob_c(x.b.c0, 1, G1_1_A, G1_1_B);
  r.a.c1 = frob_c(x.a.c1, 1, G1_2_A, G1_2_B);
  r.b.c1 = frob_c(x.b.c1, 1, G1_3_A, G1_3_B);
  r.a.c2 = frob_c(x.a.c2, 1, G1_4_A, G1_4_B);
  r.b.c2 = frob_c(x.b.c2, 1, G1_5_A, G1_5_B);
  return r;
}
PV_BN_CALL fp12 f12frob2(const fp12& x) {   // gamma_{2,e} in Fp
  fp12 r;
  r.a.c0 = x.a.c0;
  r.b.c0 = f2mulfp(x.b.c0, cst(G2_1_A));
  r.a.c1 = f2mulfp(x.a.c1, cst(G2_2_A));
  r.b.c1 = f2mulfp(x.b.c1, cst(G2_3_A));
  r.a.c2 = f2mulfp(x.a.c2, cst(G2_4_A));
  r.b.c2 = f2mulfp(x.b.c2, cst(G2_5_A));
  return r;
}
PV_BN_CALL fp12 f12frob3(const fp12& x) {
  fp12 r;
  r.a.c0 = f2conj(x.a.c0);
  r.b.c0 = frob_c(x.b.c0, 3, G3_1_A, G3_1_B);
  r.a.c1 = frob_c(x.a.c1, 3, G3_2_A, G3_2_B);
  r.b.c1 = frob_c(x.b.c1, 3, G3_3_A, G3_3_B);
  r.a.c2 = frob_c(x.a.c2, 3, G3_4_A, G3_4_B);
  r.b.c2 = frob_c(x.b.c2, 3, G3_5_A, G3_5_B);
  return r;
}

// Granger-Scott squaring in the cyclotomic subgroup (after the easy part):
// x = A + B w + C w^2 over Fp4 = Fp2[s]/(s^2 - xi), s = w^3:
// A = (a.c0, b.c1), B = (b.c0, a.c2), C = (a.c1, b.c2)
PV_HD void fp4_sqr(fp2& t0, fp2& t1, const fp2& z0, const fp2& z1) {   // (z0 + z1 s)^2
  const fp2 tmp = f2mul(z0, z1);
  const fp2 s = f2mul(fp2{add(z0.a, z1.a), add(z0.b, z1.b)}, f2add(f2mulxi(z1), z0));
  t0 = f2sub(f2sub(s, tmp), f2mulxi(tmp));
  t1 = f2dbl(tmp);
}
PV_HD fp2 three_minus_two(const fp2& t, const fp2& z) {   // 3t - 2z
  const fp2 d = f2sub(t, z);
  return f2add(f2dbl(d), t);
}
PV_HD fp2 three_plus_two(const fp2& t, const fp2& z) {    // 3t + 2z
  const fp2 d = f2add(t, z);
  return f2add(f2dbl(d), t);
}
PV_HD fp12 cyc_sqr_i(const fp12& x) {
  fp2 t0, t1, t2, t3, t4, t5;
  fp4_sqr(t0, t1, x.a.c0, x.b.c1);
  fp4_sqr(t2, t3, x.b.c0, x.a.c2);
  fp4_sqr(t4, t5, x.a.c1, x.b.c2);
  fp12 r;
  r.a.c0 = three_minus_two(t0, x.a.c0);
  r.b.c1 = three_plus_two(t1, x.b.c1);
  r.b.c0 = three_plus_two(f2mulxi(t5), x.b.c0);
  r.a.c2 = three_minus_two(t4, x.a.c2);
  r.a.c1 = three_minus_two(t2, x.a.c1);
  r.b.c2 = three_plus_two(t3, x.b.c2);
  return r;
}
PV_BN_CALL fp12 cyc_sqr(const fp12& x) { return cyc_sqr_i(x); }
// x^u (u = -0x4080000000000001) in the cyclotomic subgroup: x^(2^62 + 2^55 + 1), conjugated
// (the squarings' 3t -/+ 2z feed the input back unreduced: values double per
// squaring, so every fourth one is followed by a reduction)
PV_HD fp6 f6reduce(const fp6& x) { return fp6{f2reduce(x.c0), f2reduce(x.c1), f2reduce(x.c2)}; }
PV_BN_CALL fp12 f12reduce(const fp12& x) { return fp12{f6reduce(x.a), f6reduce(x.b)}; }
PV_BN_CALL fp12 cyc_pow_u(const fp12& x) {
  fp12 t = x;
  for (int i = 0; i < 7; ++i) {
    t = cyc_sqr_i(t);
    if ((i & 3) == 3) t = f12reduce(t);
  }
  t = f12mul(t, x);                  // x^(2^7 + 1)
  for (int i = 0; i < 55; ++i) {
    t = cyc_sqr_i(t);
    if ((i & 3) == 3) t = f12reduce(t);
  }
  t = f12mul(t, x);                  // x^(2^62 + 2^55 + 1)
  return f12conj(t);
}

// f^((p^12 - 1)/r): easy part, then Scott et al.'s hard-part chain
PV_BN_CALL fp12 final_exp(const fp12& f0) {
  fp12 f = f12mul(f12conj(f0), f12inv(f0));   // ^(p^6 - 1)
  f = f12mul(f12frob2(f), f);                // ^(p^2 + 1)
  const fp12 fu = cyc_pow_u(f);
  const fp12 fu2 = cyc_pow_u(fu);
  const fp12 fu3 = cyc_pow_u(fu2);
  const fp12 y6 = f12conj(f12mul(fu3, f12frob1(fu3)));
  fp12 t0 = cyc_sqr(y6);
  t0 = f12mul(t0, f12conj(f12mul(fu, f12frob1(fu2))));   // y4
  const fp12 y5 = f12conj(fu2);
  t0 = f12mul(t0, y5);
  fp12 t1 = f12mul(f12mul(f12conj(f12frob1(fu)), y5), t0);   // y3 y5 t0
  t0 = f12mul(t0, f12frob2(fu2));                             // y2
  t1 = f12mul(cyc_sqr(t1), t0);
  t1 = cyc_sqr(t1);
  t0 = f12mul(t1, f12conj(f));                                  // y1
  const fp12 y0 = f12mul(f12mul(f12frob1(f), f12frob2(f)), f12frob3(f));
  t1 = f12mul(t1, y0);
  return f12mul(cyc_sqr(t0), t1);
}

// ------------------------------------------------------------------ lines of a fixed G2 point
// Optimal ate, |6u + 2| = 2^64 + ATE_LO; the line sequence of one G2 point Q
// (consumption order): for bit i = 63..0 the doubling line, then for set bits
// (63, 57, 56, 2) the addition line; after the loop (6u + 2 < 0: f conjugated,
// T negated) the lines with pi(Q) and -pi^2(Q).
static constexpr int N_LINES = 70;
static constexpr int LINE_WORDS = 4 * NL;   // B'.a B'.b C'.a C'.b
// a line on the twist through T and S (affine): l = y_P + B' x_P w + C' v w,
// B' = -lambda, C' = lambda x_T - y_T; T <- T + S (T != -S)
struct g2a {
  fp2 x, y;
};
PV_BN_CALL void line_affine(uint32_t* out, g2a& T, const g2a& S, bool dbl_step) {
  fp2 lam;
  if (dbl_step) {
    const fp2 x2 = f2sqr(T.x);
    lam = f2mul(f2add(f2dbl(x2), x2), f2inv(f2dbl(T.y)));
  } else {
    lam = f2mul(f2sub(S.y, T.y), f2inv(f2sub(S.x, T.x)));
  }
  const fp2 B = f2neg(lam);
  const fp2 C = f2sub(f2mul(lam, T.x), T.y);
  const fp2 x3 = f2sub(f2sub(f2sqr(lam), T.x), S.x);
  const fp2 y3 = f2sub(f2mul(lam, f2sub(T.x, x3)), T.y);
  T.x = f2reduce(x3);   // x3 = lambda^2 - 2 x_T feeds back: reduce
  T.y = f2reduce(y3);
  const fp* v[4] = {&B.a, &B.b, &C.a, &C.b};
  for (int j = 0; j < 4; ++j)
    for (int i = 0; i < NL; ++i) out[j * NL + i] = v[j]->l[i];
}
PV_HD bool ate_bit(int i) { return (ATE_LO >> i) & 1; }

PV_BN_CALL void g2_lines(uint32_t* out, const g2a& Q) {
  g2a T = Q;
  int k = 0;
  for (int i = 63; i >= 0; --i) {
    line_affine(out + LINE_WORDS * k++, T, T, true);
    if (ate_bit(i)) line_affine(out + LINE_WORDS * k++, T, Q, false);
  }
  T.y = f2neg(T.y);
  const g2a Q1 = {f2mul(f2conj(Q.x), f2cst(FX1_A, FX1_B)), f2mul(f2conj(Q.y), f2cst(FY1_A, FY1_B))};
  line_affine(out + LINE_WORDS * k++, T, Q1, false);
  const g2a Q2 = {f2mul(Q.x, f2cst(FX2_A, FX2_B)), f2neg(f2mul(Q.y, f2cst(FY2_A, FY2_B)))};
  line_affine(out + LINE_WORDS * k++, T, Q2, false);
}

PV_HD fp2 ld_f2(const uint32_t* w) {
  fp2 r;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    r.a.l[i] = w[i];
    r.b.l[i] = w[NL + i];
  }
  return r;
}

// the Miller loop of prod_t e(P_t, Q_t) over fixed-Q lines, P_t given as
// (xq, yq) = (x/y, 1/y) (a point at infinity as (0, 0): its lines become 1)
template <int T_>
PV_HD fp12 miller_fixed(const uint32_t* const lines[T_], const fp* xq, const fp* yq) {
  fp12 f = f12one();
  int k = 0;
  for (int i = 63; i >= 0; --i) {
    if (i != 63) f = f12sqr(f);
#pragma unroll
    for (int t = 0; t < T_; ++t) {
      const uint32_t* L = lines[t] + LINE_WORDS * k;
      f = f12mul_line(f, f2mulfp(ld_f2(L), xq[t]), f2mulfp(ld_f2(L + 2 * NL), yq[t]));
    }
    ++k;
    if (ate_bit(i)) {
#pragma unroll
      for (int t = 0; t < T_; ++t) {
        const uint32_t* L = lines[t] + LINE_WORDS * k;
        f = f12mul_line(f, f2mulfp(ld_f2(L), xq[t]), f2mulfp(ld_f2(L + 2 * NL), yq[t]));
      }
      ++k;
    }
  }
  f = f12conj(f);
  for (int j = 0; j < 2; ++j, ++k) {
#pragma unroll
    for (int t = 0; t < T_; ++t) {
      const uint32_t* L = lines[t] + LINE_WORDS * k;
      f = f12mul_line(f, f2mulfp(ld_f2(L), xq[t]), f2mulfp(ld_f2(L + 2 * NL), yq[t]));
    }
  }
  return f;
}

// the kernel's Miller product of two pairings: ONE out-of-line function whose
// loop body (squaring + the two lines) is inlined, so f stays in registers
// across the 68 steps (as calls, f went through the stack at every one)
PV_HD fp12 line2_i(const fp12& f, const uint32_t* Lg, const uint32_t* Lp, const fp* xq, const fp* yq) {
  fp12 r = f12mul_line_i(f, f2mulfp(ld_f2(Lg), xq[0]), f2mulfp(ld_f2(Lg + 2 * NL), yq[0]));
  return f12mul_line_i(r, f2mulfp(ld_f2(Lp), xq[1]), f2mulfp(ld_f2(Lp + 2 * NL), yq[1]));
}
PV_BN_CALL fp12 miller2(const uint32_t* g_lines, const uint32_t* pk_lines, const fp* xq, const fp* yq) {
  fp12 f = f12one();
  int k = 0;
  // steps: bit i = 63..0 doubling (squaring first, except for f = 1), then an
  // addition step for the set bits; 2 Frobenius steps after the conjugation
  for (int i = 63; i >= 0; --i) {
    for (int add = 0; add < 2; ++add) {
      if (add && !ate_bit(i)) break;
      if (!add && i != 63) f = f12sqr_i(f);
      f = line2_i(f, g_lines + LINE_WORDS * k, pk_lines + LINE_WORDS * k, xq, yq);
      ++k;
    }
  }
  f = f12conj(f);
  for (int j = 0; j < 2; ++j, ++k) f = line2_i(f, g_lines + LINE_WORDS * k, pk_lines + LINE_WORDS * k, xq, yq);
  return f;
}

// ------------------------------------------------------------------ G1 / G2 points
// y^2 == x^3 + 2 (Montgomery coordinates)
PV_HD bool g1_on_curve(const fp& x, const fp& y) { return eq(sqr(y), addn(mul(sqr(x), x), cst(TWO_M))); }
PV_HD bool g2_on_curve(const fp2& x, const fp2& y) {
  return f2eq(f2sqr(y), f2add(f2mul(f2sqr(x), x), f2cst(BTW_A, BTW_B)));
}

// square root for p = 3 mod 4 (AMCL FP::sqrt): a^((p+1)/4); ok = it squares back to a != 0
PV_HD fp sqrt_fp(const fp& a, bool& ok) {
  const fp y = pow_fixed(a, E_SQRT);
  ok = eq(sqr(y), a) && !is_zero(a);
  return y;
}

// Jacobian G1 (a = 0), for the batch signer (bench / test data)
struct g1j {
  fp x, y, z;
};
PV_BN_CALL g1j g1j_dbl(const g1j& p) {   // dbl-2009-l
  const fp A = sqr(p.x), B = sqr(p.y), C = sqr(B);
  const fp D = dbl(subn(subn(sqr(addn(p.x, B)), A), C));
  const fp E = addn(dbl(A), A), F = sqr(E);
  g1j r;
  r.x = subn(F, dbl(D));
  r.y = subn(mul(E, subn(D, r.x)), dbl(dbl(dbl(C))));
  r.z = dbl(mul(p.y, p.z));
  return r;
}
// p + q with q affine (madd-2007-bl); p may be the point at infinity (z = 0)
PV_BN_CALL g1j g1j_madd(const g1j& p, const fp& qx, const fp& qy, bool p_inf) {
  if (p_inf) return g1j{qx, qy, fone()};
  const fp Z1Z1 = sqr(p.z), U2 = mul(qx, Z1Z1), S2 = mul(qy, mul(p.z, Z1Z1));
  const fp H = subn(U2, p.x), HH = sqr(H), I = dbl(dbl(HH)), J = mul(H, I);
  const fp rr = dbl(subn(S2, p.y)), V = mul(p.x, I);
  g1j r;
  r.x = subn(subn(sqr(rr), J), dbl(V));
  r.y = subn(mul(rr, subn(V, r.x)), dbl(mul(p.y, J)));
  r.z = subn(subn(sqr(addn(p.z, H)), Z1Z1), HH);
  return r;
}

// Jacobian G2 doubling / mixed addition over Fp2 (subgroup check)
struct g2j {
  fp2 x, y, z;
};
PV_BN_CALL g2j g2j_dbl(const g2j& p) {
  const fp2 A = f2sqr(p.x), B = f2sqr(p.y), C = f2sqr(B);
  const fp2 D = f2dbl(f2sub(f2sub(f2sqr(f2add(p.x, B)), A), C));
  const fp2 E = f2add(f2dbl(A), A), F = f2sqr(E);
  g2j r;
  r.x = f2sub(F, f2dbl(D));
  r.y = f2sub(f2mul(E, f2sub(D, r.x)), f2dbl(f2dbl(f2dbl(C))));
  r.z = f2dbl(f2mul(p.y, p.z));
  return r;
}
// full Jacobian addition with every exceptional case (doubling, inverse, infinity)
PV_BN_CALL g2j g2j_add(const g2j& p, const g2j& q) {
  if (f2is_zero(p.z)) return q;
  if (f2is_zero(q.z)) return p;
  const fp2 Z1Z1 = f2sqr(p.z), Z2Z2 = f2sqr(q.z);
  const fp2 U1 = f2mul(p.x, Z2Z2), U2 = f2mul(q.x, Z1Z1);
  const fp2 S1 = f2mul(p.y, f2mul(q.z, Z2Z2)), S2 = f2mul(q.y, f2mul(p.z, Z1Z1));
  if (f2eq(U1, U2)) {
    if (f2eq(S1, S2)) return g2j_dbl(p);
    return g2j{f2one(), f2one(), f2zero()};
  }
  const fp2 H = f2sub(U2, U1), I = f2sqr(f2dbl(H)), J = f2mul(H, I);
  const fp2 rr = f2dbl(f2sub(S2, S1)), V = f2mul(U1, I);
  g2j r;
  r.x = f2sub(f2sub(f2sqr(rr), J), f2dbl(V));
  r.y = f2sub(f2mul(rr, f2sub(V, r.x)), f2dbl(f2mul(S1, J)));
  r.z = f2mul(f2sub(f2sub(f2sqr(f2add(p.z, q.z)), Z1Z1), Z2Z2), H);
  return r;
}
// r * Q == O  (Q affine, not O)
PV_BN_CALL bool g2_in_subgroup(const g2a& q) {
  g2j acc{f2one(), f2one(), f2zero()};
  const g2j Q{q.x, q.y, f2one()};
  for (int w = 3; w >= 0; --w)
    for (int k = 63; k >= 0; --k) {
      acc = g2j_dbl(acc);
      if ((E_R[w] >> k) & 1) acc = g2j_add(acc, Q);
    }
  return f2is_zero(acc.z);
}


// ------------------------------------------------------------------ the BLS check, per lane
// H(m) = ursa PointG1::from_hash(SHA-256(m)) (AMCL ECP::new_big): x = the digest
// as a big-endian integer taken mod p; y = (x^3 + 2)^((p+1)/4) when x^3 + 2 is
// a non-zero square, else the integer is incremented and the map retried.
PV_HD void hash_to_g1(const uint8_t digest[32], fp& x, fp& y) {
  fp xi = from_be32(digest);
  for (;;) {
    x = to_mont(xi);
    const fp rhs = addn(mul(sqr(x), x), cst(TWO_M));
    bool ok;
    y = sqrt_fp(rhs, ok);
    if (ok) return;
    xi.l[0] += 1;
    xi = norm(xi);
  }
}

// sigma from its 128-byte representation (AMCL ECP::frombytes): 0x04|x|y, or
// 0x02/0x03|x with y's parity; x or y >= p, another prefix, a point off the
// curve or a non-square x^3 + 2 decode to the point at infinity (inf = true)
PV_HD void g1_decode(const uint8_t* b, fp& x, fp& y, bool& inf) {
  inf = true;
  x = fzero();
  y = fzero();
  const fp xp = from_be32(b + 1);
  if (!lt_p(xp)) return;
  x = to_mont(xp);
  if (b[0] == 4) {
    const fp yp = from_be32(b + 33);
    if (!lt_p(yp)) return;
    y = to_mont(yp);
    inf = !g1_on_curve(x, y);
  } else if (b[0] == 2 || b[0] == 3) {
    bool ok;
    y = sqrt_fp(addn(mul(sqr(x), x), cst(TWO_M)), ok);
    if (!ok) return;
    if ((from_mont(y).l[0] & 1) != (b[0] & 1)) y = negn(y);
    inf = false;
  }
}

// G2 from 128 bytes (ECP2::frombytes): x.a|x.b|y.a|y.b big-endian, each taken
// mod p; status 0 = a point of G2 (order r), 1 = off the twist (-> O),
// 2 = on the twist but outside the order-r subgroup
PV_HD int g2_decode(const uint8_t* b, g2a& q, bool check_subgroup = true) {
  q.x = fp2{to_mont(from_be32(b)), to_mont(from_be32(b + 32))};
  q.y = fp2{to_mont(from_be32(b + 64)), to_mont(from_be32(b + 96))};
  if (!g2_on_curve(q.x, q.y)) return 1;
  if (check_subgroup && !g2_in_subgroup(q)) return 2;
  return 0;
}

// (x/y, 1/y) of P (or of -P), the form the normalised lines take
PV_HD void line_point(const fp& x, const fp& y, bool negate, fp& xq, fp& yq) {
  fp yi = inv(y);
  if (negate) yi = negn(yi);
  xq = mul(x, yi);
  yq = yi;
}

// the check: e(sigma, g) == e(H, pk) <=> e(sigma, g) e(-H, pk) == 1 for sigma
// and H in G1 (cofactor 1) and g, pk in G2.  sigma = O or pk = O make their
// pairing 1: the check then holds iff both are O.
PV_HD bool bls_check(const fp& xs, const fp& ys, bool s_inf, const fp& xqh, const fp& yqh, bool pk_inf,
                     const uint32_t* g_lines, const uint32_t* pk_lines) {
  fp xq[2], yq[2];
  if (s_inf) {
    xq[0] = fzero();
    yq[0] = fzero();
  } else {
    line_point(xs, ys, false, xq[0], yq[0]);
  }
  xq[1] = xqh;
  yq[1] = yqh;
  const fp12 f = final_exp(miller2(g_lines, pk_lines, xq, yq));
  if (s_inf || pk_inf) return s_inf && pk_inf;
  return f12is_one(f);
}

// sigma = sk H (ursa Bls::sign) as its 128-byte representation; sk: 32-byte
// big-endian scalar (bench / test data generation)
PV_HD void g1_sign(uint8_t* out, const fp& hx, const fp& hy, const uint8_t* sk) {
  g1j acc{fone(), fone(), fzero()};
  bool inf = true;
  for (int k = 0; k < 256; ++k) {
    if (!inf) acc = g1j_dbl(acc);
    if ((sk[k >> 3] >> (7 - (k & 7))) & 1) {
      acc = g1j_madd(acc, hx, hy, inf);
      inf = false;
    }
  }
  for (int k = 0; k < 128; ++k) out[k] = 0;
  if (inf || is_zero(acc.z)) return;
  const fp zi = inv(acc.z), zi2 = sqr(zi);
  out[0] = 4;
  to_be32(out + 1, from_mont(mul(acc.x, zi2)));
  to_be32(out + 33, from_mont(mul(acc.y, mul(zi2, zi))));
}

}  // namespace bn
