// Half-size scalars for the cofactorless verification equation
// (Pornin 2020, "Optimized lattice basis reduction in dimension 2, and fast
// Schnorr and EdDSA signature verification", restated for libsodium's exact
// verdicts).
//
// libsodium 1.0.18 accepts iff encode(R') == R (32 bytes) with
// R' = S*B - h*A.  Decoding R to a point P_R
// succeeds exactly for the canonical encodings (y < p, on the curve, and
// x != 0 or sign bit 0 -- x == 0 encodings are on the small-order blocklist
// anyway), so encode(R') == R  <=>  P_R decodes and R' == P_R.  The group
// E(F_p) is cyclic of order 8L; for an ODD d with 0 < d < L,
//     R' == P_R  <=>  d (R' - P_R) == O
//                <=>  (d S mod L) B + c (-A) + d (-P_R) == O
// whenever c == d h (mod 8L): then c A == (d h) A for every curve point A,
// including mixed-order keys, and B has order L.  So the verdict stays
// bit-identical while the variable-base scalars c and d are ~128 bits
// instead of 253: half the doublings.
//
// (c, d) comes from Euclid's algorithm on (8L, h), which walks the lattice
// {(c, d) : c == d h (mod 8L)}: a_i = (r_i, t_i) with r_i == t_i h, r_i
// decreasing, |t_i| increasing, sign(t_i) = (-1)^(i+1).  At the first r_i <
// 2^128, |t_i| <= 8L / r_{i-1} < 2^128.  If t_i is even, a_{i-1} - k a_i
// (t_{i-1} is odd: consecutive t are coprime) with the smallest k that brings
// the r part under the window bound is used.  Signatures for which no vector
// fits 132-bit signed-digit windows (or with a quotient >= 2^32 on the way)
// are DEFERRED to the full-length path: ~0.2 % of random h (tools/lattice_sim
// statistics in DESIGN.md §4); the verdict never depends on which path runs.
#pragma once
#include <stdint.h>
#include <math.h>
#include "pv_scalar.h"

namespace pv {

// |c|, d < HS_MAX so that c + 0x88..8 (33 nibbles) < 2^132: 33 signed radix-16
// digits in [-8, 8), i.e. 32 windows of 4 doublings.
constexpr int HS_WORDS = 5;   // 160-bit |c|, d (plus the digit offset)
constexpr int HS_T = 6;       // |t| during the reduction (< 2^161 after the last step)
constexpr uint32_t HS_NONE = 0, HS_HALF = 1, HS_DEFER = 2;

// 8L = the order of E(F_p), 8 little-endian words
PV_HD uint32_t sc_8L(int i) {
  const uint32_t v[8] = {0xe7ae9f68u, 0xc09318d2u, 0x17bce6b2u, 0xa6f7cef5u, 0u, 0u, 0u, 0x80000000u};
  return v[i];
}

// value of 8 words as a double (relative error < 2^-50: all terms positive)
PV_HD double words_to_f64(const uint32_t r[8]) {
  double x = (double)r[7];
#pragma unroll
  for (int k = 6; k >= 0; --k) x = x * 4294967296.0 + (double)r[k];
  return x;
}

PV_HD bool ge2_128(const uint32_t r[8]) { return (r[4] | r[5] | r[6] | r[7]) != 0; }

// a >= b (8 words)
PV_HD bool ge8(const uint32_t a[8], const uint32_t b[8]) {
  bool gt = false, decided = false;
#pragma unroll
  for (int k = 7; k >= 0; --k) {
    if (!decided && a[k] != b[k]) {
      gt = a[k] > b[k];
      decided = true;
    }
  }
  return !decided || gt;
}

PV_HD void add8(uint32_t a[8], const uint32_t b[8]) {
#if defined(__HIP_DEVICE_COMPILE__)
  unsigned c = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) a[k] = __builtin_addc(a[k], b[k], c, &c);
#else
  uint64_t c = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    c += (uint64_t)a[k] + b[k];
    a[k] = (uint32_t)c;
    c >>= 32;
  }
#endif
}

PV_HD void sub8(uint32_t a[8], const uint32_t b[8]) {
#if defined(__HIP_DEVICE_COMPILE__)
  unsigned bw = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) a[k] = __builtin_subc(a[k], b[k], bw, &bw);
#else
  uint32_t br = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint64_t d = (uint64_t)a[k] - b[k] - br;
    a[k] = (uint32_t)d;
    br = (uint32_t)(d >> 63);
  }
#endif
}

// a -= q b over 8 words; returns true iff the exact result is negative (then a
// holds it mod 2^256; callers know it lies in (-b, 0))
PV_HD bool submul8(uint32_t a[8], const uint32_t b[8], uint32_t q) {
#if defined(__HIP_DEVICE_COMPILE__)
  // device: the eight products q b_k are independent (one v_mad_u64_u32 each);
  // their low words and the previous product's high word leave a[k] through two
  // borrow chains (v_subb_co_u32 with carry in/out) instead of 64-bit sign tricks
  uint32_t lo[8], hi[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint64_t p = (uint64_t)q * b[k];
    lo[k] = (uint32_t)p;
    hi[k] = (uint32_t)(p >> 32);
  }
  unsigned b1 = 0, b2 = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    unsigned o1, o2;
    const uint32_t t = __builtin_subc(a[k], lo[k], b1, &o1);
    a[k] = __builtin_subc(t, k ? hi[k - 1] : 0u, b2, &o2);
    b1 = o1;
    b2 = o2;
  }
  return (hi[7] | b1 | b2) != 0;
#else
  uint64_t pc = 0;
  uint32_t br = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint64_t p = (uint64_t)q * b[k] + pc;
    pc = p >> 32;
    const uint64_t d = (uint64_t)a[k] - (uint32_t)p - br;
    a[k] = (uint32_t)d;
    br = (uint32_t)(d >> 63);
  }
  return (pc + br) != 0;
#endif
}

// t += q u (HS_T words; no overflow by the bounds above)
PV_HD void addmul_t(uint32_t t[HS_T], const uint32_t u[HS_T], uint32_t q) {
#if defined(__HIP_DEVICE_COMPILE__)
  // independent products, their low and (shifted) high words added by two carry chains
  uint32_t lo[HS_T], hi[HS_T];
#pragma unroll
  for (int k = 0; k < HS_T; ++k) {
    const uint64_t p = (uint64_t)q * u[k];
    lo[k] = (uint32_t)p;
    hi[k] = (uint32_t)(p >> 32);
  }
  unsigned c1 = 0, c2 = 0;
#pragma unroll
  for (int k = 0; k < HS_T; ++k) {
    const uint32_t x = __builtin_addc(t[k], lo[k], c1, &c1);
    t[k] = __builtin_addc(x, k ? hi[k - 1] : 0u, c2, &c2);
  }
#else
  uint64_t c = 0;
#pragma unroll
  for (int k = 0; k < HS_T; ++k) {
    const uint64_t p = (uint64_t)q * u[k] + t[k] + c;
    t[k] = (uint32_t)p;
    c = p >> 32;
  }
#endif
}

PV_HD void add_t(uint32_t t[HS_T], const uint32_t u[HS_T]) {
#if defined(__HIP_DEVICE_COMPILE__)
  unsigned cc = 0;
#pragma unroll
  for (int k = 0; k < HS_T; ++k) t[k] = __builtin_addc(t[k], u[k], cc, &cc);
#else
  uint64_t c = 0;
#pragma unroll
  for (int k = 0; k < HS_T; ++k) {
    c += (uint64_t)t[k] + u[k];
    t[k] = (uint32_t)c;
    c >>= 32;
  }
#endif
}

PV_HD void sub_t(uint32_t t[HS_T], const uint32_t u[HS_T]) {
#if defined(__HIP_DEVICE_COMPILE__)
  unsigned bw = 0;
#pragma unroll
  for (int k = 0; k < HS_T; ++k) t[k] = __builtin_subc(t[k], u[k], bw, &bw);
#else
  uint32_t br = 0;
#pragma unroll
  for (int k = 0; k < HS_T; ++k) {
    const uint64_t d = (uint64_t)t[k] - u[k] - br;
    t[k] = (uint32_t)d;
    br = (uint32_t)(d >> 63);
  }
#endif
}

// One exact Euclid step (ra >= rb > 0): q = floor(ra / rb),
// (ra, ta) <- (ra - q rb, ta + q tb).  q is estimated in float64 (within one
// of the true quotient while q < 2^32) and fixed by one conditional add or
// subtract of rb.  false: quotient too large for one 32-bit step (deferred).
// floor(a / b) within one: the device takes the hardware reciprocal and two
// Newton steps (relative error ~2^-50, so below 2^-18 absolute while the
// quotient is < 2^32) instead of the correctly rounded division sequence; the
// callers correct the quotient by one either way
PV_HD double quot_est(double a, double b) {
#if defined(__HIP_DEVICE_COMPILE__)
  double r = __builtin_amdgcn_rcp(b);
  r = fma(r, fma(-b, r, 1.0), r);
  r = fma(r, fma(-b, r, 1.0), r);
  return floor(a * r);
#else
  return floor(a / b);
#endif
}

PV_HD bool euclid_step(uint32_t ra[8], uint32_t ta[HS_T], const uint32_t rb[8], const uint32_t tb[HS_T]) {
  const double qd = quot_est(words_to_f64(ra), words_to_f64(rb));
  if (!(qd < 4294967294.0)) return false;
  const uint32_t q = (uint32_t)qd;
  if (submul8(ra, rb, q)) {          // over-estimate by one
    add8(ra, rb);
    addmul_t(ta, tb, q);
    sub_t(ta, tb);
  } else {
    addmul_t(ta, tb, q);
    if (ge8(ra, rb)) {               // under-estimate by one
      sub8(ra, rb);
      add_t(ta, tb);
    }
  }
  return true;
}

// v (nw words) + 0x88..8 (33 nibbles) < 2^132: v fits the signed-digit windows
PV_HD bool fits132(const uint32_t* v, int nw) {
  uint32_t hi = 0;
  for (int k = HS_WORDS; k < nw; ++k) hi |= v[k];
  if (hi) return false;
  uint64_t c = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) c = ((uint64_t)v[k] + 0x88888888u + c) >> 32;
  return (uint64_t)v[4] + 8u + c < 16u;
}

// h (< L, 8 words) -> |c|, d (HS_WORDS words each) with c == d h (mod 8L),
// d odd and positive, |c|, d within the 132-bit windows; c_neg = sign of c.
// Returns HS_HALF, or HS_DEFER when no such pair was found (see header).
PV_HD uint32_t half_scalars(uint32_t c[HS_WORDS], uint32_t d[HS_WORDS], bool& c_neg, const uint32_t h[8]) {
  uint32_t ra[8], rb[8], ta[HS_T], tb[HS_T];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    ra[k] = sc_8L(k);
    rb[k] = h[k];
  }
#pragma unroll
  for (int k = 0; k < HS_T; ++k) ta[k] = tb[k] = 0;
  tb[0] = 1;
  // a_{i-1} = (ra, ta), a_i = (rb, tb); odd = parity of i.  Two steps per trip
  // so the roles alternate without swapping registers; the exit swaps once.
  uint32_t odd = 1;
  int trips = 0;
#pragma unroll 1
  for (;;) {
    if (!ge2_128(rb)) break;
    if (++trips > 96 || !euclid_step(ra, ta, rb, tb)) return HS_DEFER;  // ra <- r_{i+1}
    odd ^= 1u;
    if (!ge2_128(ra)) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t x = ra[k];
        ra[k] = rb[k];
        rb[k] = x;
      }
#pragma unroll
      for (int k = 0; k < HS_T; ++k) {
        const uint32_t x = ta[k];
        ta[k] = tb[k];
        tb[k] = x;
      }
      break;
    }
    if (!euclid_step(rb, tb, ra, ta)) return HS_DEFER;                   // rb <- r_{i+1}
    odd ^= 1u;
  }
  if (tb[0] & 1u) {
    // a_i itself: r_i < 2^128, |t_i| < 2^128; t_i < 0 iff i even
    c_neg = odd == 0;
#pragma unroll
    for (int k = 0; k < HS_WORDS; ++k) {
      c[k] = rb[k];
      d[k] = tb[k];
    }
    return HS_HALF;
  }
  // t_i even: a_{i-1} - k a_i for the smallest k >= 0 with r <= bound
  // (t_{i-1} odd, opposite sign to t_i, so |t| = |t_{i-1}| + k |t_i|)
  if (!fits132(ra, 8)) {
    if ((rb[0] | rb[1] | rb[2] | rb[3]) == 0) return HS_DEFER;   // r_i = 0 (cannot happen)
    // k ~ (ra - target) / rb rounded up, target 2.5e39 just under the bound
    // 0x77..78 (33 nibbles) = 2.54e39; one more subtraction if it fell short
    const double kd = ceil((words_to_f64(ra) - 2.5e39) / words_to_f64(rb));
    if (!(kd < 4294967294.0)) return HS_DEFER;
    const uint32_t k = kd > 0.0 ? (uint32_t)kd : 0u;
    if (submul8(ra, rb, k)) return HS_DEFER;
    addmul_t(ta, tb, k);
    if (!fits132(ra, 8)) {
      sub8(ra, rb);
      add_t(ta, tb);
    }
    if (!fits132(ra, 8)) return HS_DEFER;
  }
  if (!fits132(ta, HS_T)) return HS_DEFER;
  c_neg = odd == 1;
#pragma unroll
  for (int k = 0; k < HS_WORDS; ++k) {
    c[k] = ra[k];
    d[k] = ta[k];
  }
  return HS_HALF;
}

// v + 0x88..8 (33 nibbles), in place: the offset form whose nibble w minus 8
// is signed digit w (callers guarantee fits132)
PV_HD void hs_offset(uint32_t v[HS_WORDS]) {
  uint64_t c = 0;
#pragma unroll
  for (int k = 0; k < HS_WORDS; ++k) {
    c += (uint64_t)v[k] + (k < 4 ? 0x88888888u : 0x8u);
    v[k] = (uint32_t)c;
    c >>= 32;
  }
}

// s' = d * S mod L (d: HS_WORDS words, S: 8 words)
PV_HD void sc_mul_small(uint32_t out[8], const uint32_t d[HS_WORDS], const uint32_t S[8]) {
  uint32_t x[16];
  uint64_t carry = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    uint64_t acc = carry & 0xffffffffu;
    uint64_t acchi = carry >> 32;
#pragma unroll
    for (int i = 0; i < HS_WORDS; ++i) {
      const int j = k - i;
      if (j >= 0 && j < 8) {
        const uint64_t p = mul32x32(d[i], S[j]);
        acc += p & 0xffffffffu;
        acchi += p >> 32;
      }
    }
    acchi += acc >> 32;
    x[k] = (uint32_t)acc;
    carry = acchi;
  }
  sc_reduce64(out, x);
}

}  // namespace pv
