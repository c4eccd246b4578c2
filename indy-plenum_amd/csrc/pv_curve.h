// Edwards25519 group operations for the batch verifier (twisted Edwards,
// a = -1, extended coordinates).  Complete unified formulas, so the identity
// and torsion points need no special cases: that is what lets every lane of a
// wavefront run the SAME fixed-window schedule (no data-dependent branches).
//
// Point forms (as in the libsodium/ref10 family the reference binds):
//   p2     (X:Y:Z)                       x = X/Z, y = Y/Z
//   p3     (X:Y:Z:T)                     T = XY/Z
//   p1p1   completed ((X:Z),(Y:T))       x = X/Z, y = Y/T
//   cached (Y+X, Y-X, 2Z, 2dT)           projective table entry ("2Z" keeps
//                                        the add's D term TIGHT)
//   niels  (y+x, y-x, 2dxy)              affine table entry (base-point table)
#pragma once
#include "pv_field.h"

namespace pv {

struct ge_p2 { fe X, Y, Z; };
struct ge_p3 { fe X, Y, Z, T; };
struct ge_p1p1 { fe X, Y, Z, T; };
struct ge_cached { fe YpX, YmX, Z2, T2d; };
struct ge_niels { fe ypx, ymx, xy2d; };

PV_HD void ge_p3_0(ge_p3& h) { fe_0(h.X); fe_1(h.Y); fe_1(h.Z); fe_0(h.T); }

// PV_FUSE selects where independent products go through the fused forms
// (fe_mul2 / fe_sq2: two column chains interleaved in one asm block,
// pv_field.h): bit 0 the doubling's squarings, bit 1 the p1p1 conversions,
// bit 2 the table-entry additions (pv_verify_core.h).  Same values either way.
#ifndef PV_FUSE
#define PV_FUSE 0
#endif
// Operand roles (f = the 2f_odd side, g = the 19g side) are chosen so the
// prepared operands are shared: T is g of X*T and Z*T (19T once), Z is f of
// Z*T and Z*Y (2Z_odd once), as X is f of X*T and X*Y in the p3 form.
PV_HD void ge_p1p1_to_p2(ge_p2& r, const ge_p1p1& p) {
#if PV_FUSE & 2
  fe_mul2(r.X, p.X, p.T, r.Y, p.Z, p.Y);
#else
  fe_mul(r.X, p.X, p.T);
  fe_mul(r.Y, p.Z, p.Y);
#endif
  fe_mul(r.Z, p.Z, p.T);
}

PV_HD void ge_p1p1_to_p3(ge_p3& r, const ge_p1p1& p) {
#if PV_FUSE & 2
  fe_mul2(r.X, p.X, p.T, r.Y, p.Z, p.Y);
  fe_mul2(r.Z, p.Z, p.T, r.T, p.X, p.Y);
#else
  fe_mul(r.X, p.X, p.T);
  fe_mul(r.Y, p.Z, p.Y);
  fe_mul(r.Z, p.Z, p.T);
  fe_mul(r.T, p.X, p.Y);
#endif
}

// dbl-2008-hwcd (a = -1) from p2:  r.X = 2XY, r.Y = Y^2+X^2, r.Z = Y^2-X^2, r.T = 2Z^2-(Y^2-X^2)
PV_HD void ge_p2_dbl(ge_p1p1& r, const ge_p2& p) {
  fe xx, yy, zz2, xy2, t;
  fe_add(t, p.X, p.Y);         // LOOSE
#if PV_FUSE & 1
  fe_sq2(xx, p.X, yy, p.Y);
  fe_sq2(zz2, p.Z, xy2, t);    // Z^2, (X+Y)^2
  fe_add(zz2, zz2, zz2);       // 2Z^2
#else
  fe_sq(xx, p.X);
  fe_sq(yy, p.Y);
  fe_sq2x(zz2, p.Z);           // 2Z^2 in one squaring (p.Z TIGHT)
  fe_sq(xy2, t);               // (X+Y)^2
#endif
  fe_add(r.Y, yy, xx);         // LOOSE
  fe_sub(r.Z, yy, xx);         // LOOSE
  fe_sub4(r.X, xy2, r.Y);      // (X+Y)^2 - X^2 - Y^2 = 2XY, even limbs < 2^28.4:
                               // only ever the FIRST operand of r.X*r.T / r.X*r.Y
                               // (second operand TIGHT / LOOSE), so no carry needed
  fe_sub4(r.T, zz2, r.Z);      // even limbs <= 2^28.4, odd <= 2^27.4
  fe_carry_even(r.T);          // T is the 19x operand of X*T and Z*T: 19 T_j < 2^32
}

PV_HD void ge_p3_dbl(ge_p1p1& r, const ge_p3& p) {
  ge_p2 q;
  fe_copy(q.X, p.X);
  fe_copy(q.Y, p.Y);
  fe_copy(q.Z, p.Z);
  ge_p2_dbl(r, q);
}

PV_HD void ge_p3_to_cached(ge_cached& r, const ge_p3& p) {
  fe d2;
  fe_const_d2(d2);
  fe_add(r.YpX, p.Y, p.X);
  fe_sub(r.YmX, p.Y, p.X);
  fe_add(r.Z2, p.Z, p.Z);
  fe_mul(r.T2d, p.T, d2);
}

PV_HD void ge_cached_identity(ge_cached& r) {
  fe_1(r.YpX);
  fe_1(r.YmX);
  fe_0(r.Z2);
  r.Z2.v[0] = 2;
  fe_0(r.T2d);
}

// r = p + s*q   (s = sign: false add, true subtract), q cached.  Branch-free.
PV_HD void ge_add_cached(ge_p1p1& r, const ge_p3& p, const ge_cached& q, bool neg) {
  fe ypx1, ymx1, a, b, c, d, qa, qb;
  fe_add(ypx1, p.Y, p.X);
  fe_sub(ymx1, p.Y, p.X);
  fe_cmov(qa, q.YpX, q.YmX, neg);
  fe_cmov(qb, q.YmX, q.YpX, neg);
  fe_mul(a, ypx1, qa);
  fe_mul(b, ymx1, qb);
  fe_mul(c, q.T2d, p.T);
  fe_mul(d, p.Z, q.Z2);        // TIGHT 2*Z1*Z2
  fe_sub(r.X, a, b);
  fe_add(r.Y, a, b);
  fe e, f;
  fe_add(e, d, c);
  fe_sub(f, d, c);
  fe_cmov(r.Z, e, f, neg);
  fe_cmov(r.T, f, e, neg);
}

// r = p + s*q, q affine niels (base-point table)
PV_HD void ge_madd(ge_p1p1& r, const ge_p3& p, const ge_niels& q, bool neg) {
  fe ypx1, ymx1, a, b, c, d, qa, qb;
  fe_add(ypx1, p.Y, p.X);
  fe_sub(ymx1, p.Y, p.X);
  fe_cmov(qa, q.ypx, q.ymx, neg);
  fe_cmov(qb, q.ymx, q.ypx, neg);
  fe_mul(a, ypx1, qa);
  fe_mul(b, ymx1, qb);
  fe_mul(c, q.xy2d, p.T);
  fe_add(d, p.Z, p.Z);
  fe_carry(d);                 // TIGHT so that d - c stays LOOSE
  fe_sub(r.X, a, b);
  fe_add(r.Y, a, b);
  fe e, f;
  fe_add(e, d, c);
  fe_sub(f, d, c);
  fe_cmov(r.Z, e, f, neg);
  fe_cmov(r.T, f, e, neg);
}

// Decompress s and NEGATE (returns -P, x chosen with parity != sign bit).
// Restates ge25519_frombytes_negate_vartime's contract (SURVEY.md App. C.2
// step 4): fails iff (y^2-1)/(dy^2+1) has no square root; x == 0 with the
// sign bit set is accepted (libsodium 1.0.18).
// -P from its encoding in two phases: phase a forms y, u = y^2 - 1,
// v = d y^2 + 1, z = u v^7 and the first half of z's (p-5)/8 power chain
// (z^(2^50-1), z^(2^100-1)); phase b finishes the chain and the square-root
// checks.  The operations and their order are exactly fe_pow22523's.  (Rounds
// 3-4 ran the phases on either side of a block barrier in the keyed latency
// kernel; round 5 measured moving the split (profiles/r05_root_split.jsonl) and
// then replaced the barrier by LDS flags, so the chain now runs in one piece.)
struct NegDecode {
  fe Y, u, v, v3, z, a, b;
};

PV_HD void neg_decode_a(NegDecode& st, const uint32_t s[8]) {
  fe one, d;
  fe_const_d(d);
  fe_1(one);
  fe_frombytes_w(st.Y, s);
  fe_sq(st.u, st.Y);
  fe_mul(st.v, st.u, d);
  fe_sub(st.u, st.u, one);
  fe_carry(st.u);              // y^2 - 1, TIGHT
  fe_add(st.v, st.v, one);     // d y^2 + 1, LOOSE
  fe_sq(st.v3, st.v);
  fe_mul(st.v3, st.v3, st.v);  // v^3
  fe_sq(st.z, st.v3);
  fe_mul(st.z, st.z, st.v);
  fe_mul(st.z, st.z, st.u);    // u v^7
  fe z2, z9, t, c;             // fe_pow_2_250_1, up to 2^100 - 1
  fe_sq(z2, st.z);
  fe_sqn(t, z2, 2);
  fe_mul(z9, t, st.z);
  fe_mul(c, z9, z2);           // z^11
  fe_sq(t, c);
  fe_mul(st.a, t, z9);                       // 2^5 - 1
  fe_sqn(t, st.a, 5);   fe_mul(st.b, t, st.a);  // 2^10 - 1
  fe_sqn(t, st.b, 10);  fe_mul(c, t, st.b);     // 2^20 - 1
  fe_sqn(t, c, 20);     fe_mul(t, t, c);        // 2^40 - 1
  fe_sqn(t, t, 10);     fe_mul(st.a, t, st.b);  // 2^50 - 1
  fe_sqn(t, st.a, 50);  fe_mul(st.b, t, st.a);  // 2^100 - 1
}

PV_HD bool neg_decode_b(ge_p3& h, NegDecode& st, const uint32_t s[8]) {
  fe t;
  fe_sqn(t, st.b, 100); fe_mul(t, t, st.b);     // 2^200 - 1
  fe_sqn(t, t, 50);     fe_mul(t, t, st.a);     // 2^250 - 1
  fe_sqn(t, t, 2);
  fe_mul(h.X, t, st.z);        // z^((p-5)/8)
  fe_copy(h.Y, st.Y);
  fe_1(h.Z);
  fe vxx, chk;
  fe_mul(h.X, h.X, st.v3);
  fe_mul(h.X, h.X, st.u);      // u v^3 (u v^7)^((p-5)/8)
  fe_sq(vxx, h.X);
  fe_mul(vxx, vxx, st.v);
  fe_sub(chk, vxx, st.u);
  bool ok = true;
  if (!fe_iszero(chk)) {
    fe_add(chk, vxx, st.u);
    if (!fe_iszero(chk)) ok = false;
    fe sqrtm1;
    fe_const_sqrtm1(sqrtm1);
    fe_mul(h.X, h.X, sqrtm1);
  }
  const uint32_t sign = s[7] >> 31;
  fe nx;
  fe_neg(nx, h.X);
  fe_carry(nx);
  fe_cmov(h.X, h.X, nx, fe_isnegative(h.X) == sign);
  fe_mul(h.T, h.X, h.Y);
  return ok;
}

PV_HD bool ge_frombytes_negate(ge_p3& h, const uint32_t s[8]) {
  NegDecode st;
  neg_decode_a(st, s);
  return neg_decode_b(h, st, s);
}

// canonical encoding of a p2 point as 8 LE words (y | sign(x) << 255)
PV_HD void ge_p2_tobytes(uint32_t w[8], const ge_p2& p) {
  fe zi, x, y;
  fe_invert(zi, p.Z);
  fe_mul(x, p.X, zi);
  fe_mul(y, p.Y, zi);
  fe_tobytes_w(w, y);
  w[7] ^= fe_isnegative(x) << 31;
}

PV_HD void ge_p3_tobytes(uint32_t w[8], const ge_p3& p) {
  ge_p2 q;
  fe_copy(q.X, p.X);
  fe_copy(q.Y, p.Y);
  fe_copy(q.Z, p.Z);
  ge_p2_tobytes(w, q);
}

// small-order encodings refused by libsodium 1.0.18,
// compared with bit 255 cleared
PV_HD bool has_small_order(const uint32_t s[8]) {
  const uint32_t bl[7][8] = {
      {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u},
      {1u, 0u, 0u, 0u, 0u, 0u, 0u, 0u},
      {0x8f95e826u, 0xb027b2c2u, 0x89f4c345u, 0xf098eff2u, 0x05acdfd5u, 0x3933c6d3u, 0x880238b1u, 0x05fc536du},
      {0x706a17c7u, 0x4fd84d3du, 0x760b3cbau, 0x0f67100du, 0xfa53202au, 0xc6cc392cu, 0x77fdc74eu, 0x7a03ac92u},
      {0xffffffecu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0x7fffffffu},
      {0xffffffedu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0x7fffffffu},
      {0xffffffeeu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0x7fffffffu},
  };
  bool any = false;
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    uint32_t diff = 0;
#pragma unroll
    for (int i = 0; i < 7; ++i) diff |= s[i] ^ bl[k][i];
    diff |= (s[7] & 0x7fffffffu) ^ bl[k][7];
    any = any || diff == 0;
  }
  return any;
}

// y (bit 255 cleared) < p  (ge25519_is_canonical, App. C.2 step 3)
PV_HD bool y_is_canonical(const uint32_t s[8]) {
  uint32_t all1 = s[1] & s[2] & s[3] & s[4] & s[5] & s[6];
  const bool top = (s[7] & 0x7fffffffu) == 0x7fffffffu && all1 == 0xffffffffu;
  return !(top && s[0] >= 0xffffffedu);
}

}  // namespace pv
