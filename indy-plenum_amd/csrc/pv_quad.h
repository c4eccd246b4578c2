// Lane-quad group arithmetic for the latency kernel (k_verify_quad).
//
// Plenum verifies at most 100 client or 1,000 node messages per Looper pass
// (stp_core/config.py:32-33), so a pass's batch is a few waves: its latency is
// one lane's serial chain, not the chip's throughput.  Here one POINT lives on
// four lanes of a quad, lane l holding coordinate l of (X, Y, Z, T).  The
// extended-coordinate formulas (dbl-2008-hwcd, add-2008-hwcd-3; a = -1) have
// four independent products per stage, so a doubling is ONE squaring + ONE
// multiply per lane and an addition TWO multiplies per lane (Hisil, Wong,
// Carter, Dawson 2008, "Twisted Edwards curves revisited", §5 parallel forms),
// instead of 4 sq + 4 mul and 8 mul on one lane.  The operand exchanges
// between the stages are DPP quad_perm moves (full-rate VALU, no LDS).
//
// Every lane of a quad runs the same instruction stream (lane roles are
// selected with per-lane values, never with branches), and all field values
// are the ones the one-lane formulas of pv_curve.h compute, with the same
// operand bounds (tools/hostcheck runs this file on the host with the bound
// checks, emulating a quad with QL = 4 lanes in lockstep).
//
// Table entries (cached form) are stored per quad as 4 coordinates in ADD
// ORDER (Y-X, Y+X, 2dT, 2Z): in the addition's first stage lane l multiplies
// [Y1-X1, Y1+X1, T1, Z1][l] by entry coordinate l (lanes 0 and 1 swapped for a
// negative digit), so each lane reads 40 bytes of an entry.
#pragma once
#include "pv_verify_core.h"

namespace pv {

#if defined(__HIP_DEVICE_COMPILE__)
constexpr int QL = 1;   // one lane = one coordinate
#else
constexpr int QL = 4;   // host emulation: the four lanes of a quad in lockstep
#endif

// one coordinate per lane (device) / the quad's four coordinates (host)
struct qfe {
  fe l[QL];
};

// A lane's role in its quad as all-ones / all-zero masks, computed once per
// kernel: every role-dependent value is formed with bit-selects (bitsel is
// one v_bitop3_b32) and integer ops.  Plain `l == k ? a : b` chains on the
// lane index were turned by the compiler into a switch, i.e. divergent branch
// regions per limb.
struct QRole {
  uint32_t l;                      // index in the quad
  uint32_t is0, is1, is2, is3;     // l == k
  uint32_t lt2, ge2;               // l < 2, l >= 2
};
PV_HD QRole qrole_of(uint32_t l) {
  QRole r;
  r.l = l;
  r.is0 = 0u - (uint32_t)(l == 0);
  r.is1 = 0u - (uint32_t)(l == 1);
  r.is2 = 0u - (uint32_t)(l == 2);
  r.is3 = 0u - (uint32_t)(l == 3);
  r.lt2 = 0u - (uint32_t)(l < 2);
  r.ge2 = ~r.lt2;
  return r;
}
// role of element j: the lane's own on the device, lane j of the emulated quad on the host
PV_HD QRole qrole(int j, const QRole& r) { return QL == 1 ? r : qrole_of((uint32_t)j); }

constexpr int QTAB_WORDS = 9 * 40;   // entries 0..8, 4 coordinates each

// lane l of the quad reads lane P_l's value (quad_perm DPP)
template <int P0, int P1, int P2, int P3>
PV_HD void q_perm(qfe& out, const qfe& in) {
#if defined(__HIP_DEVICE_COMPILE__)
  constexpr int ctrl = P0 | (P1 << 2) | (P2 << 4) | (P3 << 6);
#pragma unroll
  for (int i = 0; i < 10; ++i)
    out.l[0].v[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)in.l[0].v[i], ctrl, 0xf, 0xf, false);
#else
  const qfe t = in;
  const int p[4] = {P0, P1, P2, P3};
  for (int j = 0; j < 4; ++j) out.l[j] = t.l[p[j]];
#endif
}
template <int K>
PV_HD void q_bcast(qfe& out, const qfe& in) {
  q_perm<K, K, K, K>(out, in);
}

PV_HD void q_mul(qfe& h, const qfe& f, const qfe& g) {
#pragma unroll
  for (int j = 0; j < QL; ++j) fe_mul(h.l[j], f.l[j], g.l[j]);
}
PV_HD void q_sq(qfe& h, const qfe& f) {
#pragma unroll
  for (int j = 0; j < QL; ++j) fe_sq(h.l[j], f.l[j]);
}

// limb i of 2p
PV_HD uint32_t p2_limb(int i) { return i == 0 ? P2_0 : ((i & 1) ? P2_O : P2_E); }

// x or -x (two's complement) by mask
PV_HD uint32_t cneg(uint32_t x, uint32_t m) { return (x ^ m) - m; }

// ------------------------------------------------------------ lane roles
// coordinate l of the p3 point P
PV_HD void role_coord(fe& out, const ge_p3& P, const QRole& r) {
#pragma unroll
  for (int i = 0; i < 10; ++i)
    out.v[i] = bitsel(r.is0, P.X.v[i], bitsel(r.is1, P.Y.v[i], bitsel(r.is2, P.Z.v[i], P.T.v[i])));
}

// identity: p3 (0, 1, 1, 0); cached in add order (Y-X, Y+X, 2dT, 2Z) = (1, 1, 0, 2)
PV_HD void role_p3_identity(fe& out, const QRole& r) {
  fe_0(out);
  out.v[0] = (r.is1 | r.is2) & 1u;
}
PV_HD void role_cached_identity(fe& out, const QRole& r) {
  fe_0(out);
  out.v[0] = (r.lt2 & 1u) | (r.is3 & 2u);
}

// first-stage operand of an addition / cached conversion:
// [Y - X + 2p, Y + X, T, Z][l] from x = X, y = Y (broadcast) and zt = the
// quad's (., ., T, Z)
PV_HD void role_add_op(fe& op, const fe& x, const fe& y, const fe& zt, const QRole& r) {
#pragma unroll
  for (int i = 0; i < 10; ++i) op.v[i] = bitsel(r.lt2, y.v[i] + bitsel(r.is0, p2_limb(i) - x.v[i], x.v[i]), zt.v[i]);
}

// second stage of an addition.  own/oth = this lane's first-stage product and
// its pair partner's (lanes 0 <-> 1: A = (Y1-X1)(Y2-X2), B = (Y1+X1)(Y2+X2);
// lanes 2 <-> 3: C = T1 2dT2, D = Z1 2Z2).  With C' = -C for a negative digit:
//   rX = B - A, rY = B + A, rZ = D + C', rT = D - C'   (ge_add_entry's p1p1)
PV_HD void role_add_u(fe& u, const fe& own, const fe& oth, bool neg, const QRole& r) {
  const uint32_t nm = 0u - (uint32_t)neg;
  const uint32_t nb = r.is0 | (r.is2 & nm) | (r.is3 & ~nm);
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t x = bitsel(r.is3, own.v[i], oth.v[i]);
    const uint32_t y = bitsel(r.is3, oth.v[i], own.v[i]);
    u.v[i] = x + bitsel(nb, p2_limb(i) - y, y);
  }
}

// second stage of a doubling from the squares s = [X^2, Y^2, Z^2, (X+Y)^2]:
//   lane 0: rY = Y^2 + X^2            lane 1: rZ = Y^2 - X^2
//   lane 2: rT = 2Z^2 - rZ            lane 3: rX = (X+Y)^2 - rY
// (ge_p2_dbl's p1p1; every lane carried to TIGHT)
PV_HD void role_dbl_u(fe& u, const fe& own, const fe& s0, const fe& s1, const QRole& r) {
  const uint32_t n0 = r.is1 | r.is3, n1 = r.ge2, sh = r.is2 & 1u;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t p2 = p2_limb(i);
    const uint32_t k = (p2 & (r.is1 | r.is2)) | ((2u * p2) & r.is3);
    const uint32_t o = (own.v[i] << sh) & r.ge2;
    u.v[i] = k + o + cneg(s0.v[i], n0) + cneg(s1.v[i], n1);
  }
  fe_carry(u);
}

// per-lane factor of the cached conversion: [1, 1, 2d, 2][l]
PV_HD void role_cached_factor(fe& k, const QRole& r) {
  fe d2;
  fe_const_d2(d2);
#pragma unroll
  for (int i = 0; i < 10; ++i) k.v[i] = bitsel(r.is2, d2.v[i], i == 0 ? ((r.lt2 & 1u) | (r.is3 & 2u)) : 0u);
}

// ------------------------------------------------------------ quad ops
// P = 2P  (p3 -> p3: [X^2, Y^2, Z^2, (X+Y)^2], then [rX rT, rY rZ, rZ rT, rX rY])
PV_HD void q_dbl(qfe& P, const QRole& q) {
  qfe x, y, s;
  q_bcast<0>(x, P);
  q_bcast<1>(y, P);
#pragma unroll
  for (int j = 0; j < QL; ++j) {
    const QRole r = qrole(j, q);
#pragma unroll
    for (int i = 0; i < 10; ++i) s.l[j].v[i] = bitsel(r.is3, x.l[j].v[i] + y.l[j].v[i], P.l[j].v[i]);   // X + Y: LOOSE
  }
  q_sq(s, s);
  qfe s0, s1, u;
  q_bcast<0>(s0, s);
  q_bcast<1>(s1, s);
#pragma unroll
  for (int j = 0; j < QL; ++j) role_dbl_u(u.l[j], s.l[j], s0.l[j], s1.l[j], qrole(j, q));   // [rY, rZ, rT, rX]
  qfe a, b;
  q_perm<3, 0, 1, 3>(a, u);   // [rX, rY, rZ, rX]
  q_perm<2, 1, 2, 0>(b, u);   // [rT, rZ, rT, rY]
  q_mul(P, a, b);
}

// first stage of an addition: [A, B, C, D] = [Y1-X1, Y1+X1, T1, Z1] * e
PV_HD void q_add_stage1(qfe& prod, const qfe& P, const qfe& e, const QRole& q) {
  qfe x, y, zt;
  q_bcast<0>(x, P);
  q_bcast<1>(y, P);
  q_perm<0, 1, 3, 2>(zt, P);
#pragma unroll
  for (int j = 0; j < QL; ++j) role_add_op(prod.l[j], x.l[j], y.l[j], zt.l[j], qrole(j, q));
  q_mul(prod, prod, e);
}

// second-stage sums [rX, rY, rZ, rT] of an addition (the p1p1 result)
PV_HD void q_add_stage2(qfe& u, const qfe& prod, bool neg, const QRole& q) {
  qfe o;
  q_perm<1, 0, 3, 2>(o, prod);
#pragma unroll
  for (int j = 0; j < QL; ++j) role_add_u(u.l[j], prod.l[j], o.l[j], neg, qrole(j, q));
}

// P = P + (neg ? -E : E); e = E's coordinates in add order (lanes 0/1 already
// swapped for neg, q_load_cached / q_load_niels)
PV_HD void q_add(qfe& P, const qfe& e, bool neg, const QRole& q) {
  qfe prod, u;
  q_add_stage1(prod, P, e, q);
  q_add_stage2(u, prod, neg, q);
  qfe a, b;
  q_perm<0, 1, 2, 0>(a, u);   // [rX, rY, rZ, rX]
  q_perm<3, 2, 3, 1>(b, u);   // [rT, rZ, rT, rY]
  q_mul(P, a, b);
}

// cached form of P in add order: [Y-X, Y+X, 2dT, 2Z] (one product per lane)
PV_HD void q_to_cached(qfe& e, const qfe& P, const QRole& q) {
  qfe x, y, zt, op, k;
  q_bcast<0>(x, P);
  q_bcast<1>(y, P);
  q_perm<0, 1, 3, 2>(zt, P);
#pragma unroll
  for (int j = 0; j < QL; ++j) {
    role_add_op(op.l[j], x.l[j], y.l[j], zt.l[j], qrole(j, q));
    role_cached_factor(k.l[j], qrole(j, q));
  }
  q_mul(e, op, k);
}

// entry k of a quad table; a negative digit swaps Y-X / Y+X (lanes 0, 1)
PV_HD void q_load_cached(qfe& e, const uint32_t* ent, bool neg, const QRole& q) {
#pragma unroll
  for (int j = 0; j < QL; ++j) {
    const QRole r = qrole(j, q);
    const uint32_t c = r.l ^ ((uint32_t)neg & r.lt2);
    load_fe(e.l[j], ent + 10 * c);
  }
}
PV_HD void q_store_cached(uint32_t* ent, const qfe& e, const QRole& q) {
#pragma unroll
  for (int j = 0; j < QL; ++j) store_fe(ent + 10 * qrole(j, q).l, e.l[j]);
}

// affine base-point entry (y+x, y-x, 2dxy at words 0, 10, 20) in add order
// (y-x, y+x, 2dxy, 2): the D product of the affine addition is Z1 * 2
PV_HD void q_load_niels(qfe& e, const uint32_t* ent, bool neg, const QRole& q) {
#pragma unroll
  for (int j = 0; j < QL; ++j) {
    const QRole r = qrole(j, q);
    const uint32_t c = bitsel(r.lt2, r.l ^ 1u ^ (uint32_t)neg, 2u);
    fe t;
    load_fe(t, ent + 10 * c);
#pragma unroll
    for (int i = 0; i < 10; ++i) e.l[j].v[i] = bitsel(r.is3, i == 0 ? 2u : 0u, t.v[i]);
  }
}

// ------------------------------------------------------------ one side
// signed digit of window w: nibble w of the offset words, minus 8
PV_HD int q_digit(const uint32_t dw[8], int w) { return (int)((pick8(dw, w >> 3) >> (4 * (w & 7))) & 15u) - 8; }

// One side of the quad verdict (the lane-pair split of k_curve_lat, each
// side now on a quad):
//   side 0: Q = c (-A) + b B,         c = the signed |c| (33 windows) or h (deferred: 64)
//   side 1: Q = k (-R) + b (2^128 B), k = d or, deferred, 1
// with b = s'_lo / s'_hi (S_lo / S_hi when deferred), so that
// Q0 + Q1 = s' B + c (-A) + d (-R) (half-size) or S B - h A - R (deferred):
// the identity iff libsodium accepts (pv_lattice.h).  The sign of c is folded
// into the digits (c (-A) = |c| (+A): every digit of side 0 negated), so the
// point and its table do not depend on the scalar stage: q_side_table runs
// before the record exists (k_verify_quad overlaps it with the hash).

// decode side's point (-A, or -R with canonical y) and write its cached
// multiples 0..8 to the quad table `tab` (QTAB_WORDS, each lane its
// coordinate); Q = the point.  false = does not decode.
// Q = -P for the 32-byte encoding at `enc` (every lane of the quad decodes the
// point: the chain is serial anyway); canon: also require y < p (R's rule).
// false = does not decode.
PV_HD bool q_decode_neg(qfe& Q, const uint8_t* enc_bytes, bool canon, const QRole& q) {
  bool ok = true;
#pragma unroll
  for (int j = 0; j < QL; ++j) {
    uint32_t enc[8];
    load8(enc, enc_bytes);
    ge_p3 P;
    const bool dec = ge_frombytes_negate(P, enc);
    ok = dec && (!canon || y_is_canonical(enc));
    role_coord(Q.l[j], P, qrole(j, q));
  }
  return ok;
}

PV_HD bool q_side_table(qfe& Q, const uint8_t* pk, const uint8_t* sig, int side, uint32_t* tab, const QRole& q) {
  const bool ok = q_decode_neg(Q, side ? sig : pk, side != 0, q);
  qfe e1, e, acc;
  q_to_cached(e1, Q, q);
#pragma unroll
  for (int j = 0; j < QL; ++j) {
    role_cached_identity(e.l[j], qrole(j, q));
    store_fe(tab + 10 * qrole(j, q).l, e.l[j]);
  }
  q_store_cached(tab + 40, e1, q);
  acc = Q;
#pragma unroll 1
  for (int k = 2; k <= 8; ++k) {
    q_add(acc, e1, false, q);
    q_to_cached(e, acc, q);
    q_store_cached(tab + 40 * k, e, q);
  }
  return ok;
}

// Horner over the side's windows from its record (tab from q_side_table,
// bt = the side's radix-2^16 base-point table): Q = the side's sum
PV_HD void q_side_msm(qfe& Q, const uint32_t* rec, int side, const uint32_t* tab, const uint32_t* bt,
                      const QRole& q) {
  const uint32_t flags = rec[HREC_FLAGS];
  const bool defer = (flags & 0xffu) == HS_DEFER;
  const bool cneg = side == 0 && (flags & 0x100u);   // c < 0: side 0's digits negated
  // digit words: side 0 = |c| (words 0..4) or h (0..7); side 1 = d (5..9) or 1,
  // aligned so that the top window's word sits in dw[7] (half-size records
  // start at window 32 = word 4); the words then shift up one per 8 windows
  // (static indices only: a dynamic pick would put the array in scratch)
  const bool full0 = defer && side == 0;
  uint32_t dw[8], sw[4];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int src = full0 ? k : k - 3;   // word of the scalar held in dw[k]
    uint32_t r = 0;
    if (src >= 0) {
      const uint32_t one = src == 0 ? 0x88888889u : (src < 4 ? 0x88888888u : 8u);
      r = side == 0 ? rec[HREC_C + src] : (defer ? one : rec[HREC_D + (src < 5 ? src : 4)]);
    }
    dw[k] = r;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) sw[k] = rec[HREC_S + 4 * side + k];
  const int top = full0 ? 63 : 32;
  qfe acc, e;
#pragma unroll
  for (int j = 0; j < QL; ++j) role_p3_identity(acc.l[j], qrole(j, q));
  int dg = (int)((dw[7] >> (4 * (top & 7))) & 15u) - 8;
  bool ng = (dg < 0) != cneg;
  q_load_cached(e, tab + 40 * (dg < 0 ? -dg : dg), ng, q);
  q_add(acc, e, ng, q);
#pragma unroll 1
  for (int w = top - 1; w >= 0; --w) {
    if ((w & 7) == 7) {
#pragma unroll
      for (int k = 7; k > 0; --k) dw[k] = dw[k - 1];
    }
    // this window's entries are fetched before its doublings
    dg = (int)((dw[7] >> (4 * (w & 7))) & 15u) - 8;
    ng = (dg < 0) != cneg;
    q_load_cached(e, tab + 40 * (dg < 0 ? -dg : dg), ng, q);
    const bool bwin = (w & 3) == 0 && w < 32;
    int db = 0;
    qfe eb;
    if (bwin) {
      const uint32_t m1 = 0u - ((uint32_t)(w >> 3) & 1u), m2 = 0u - ((uint32_t)(w >> 4) & 1u);
      const uint32_t sword = bitsel(m2, bitsel(m1, sw[3], sw[2]), bitsel(m1, sw[1], sw[0]));
      db = (int)((sword >> (16 * ((w >> 2) & 1))) & 0xffffu) - 32768;
      q_load_niels(eb, bt + (db < 0 ? -db : db) * BT_WORDS, db < 0, q);
    }
#pragma unroll 1
    for (int k = 0; k < 4; ++k) q_dbl(acc, q);
    q_add(acc, e, ng, q);
    if (bwin) q_add(acc, eb, db < 0, q);
  }
  Q = acc;
}

PV_HD bool q_side(qfe& Q, const uint8_t* pk, const uint8_t* sig, const uint32_t* rec, int side, uint32_t* tab,
                  const uint32_t* bt, const QRole& q) {
  const bool ok = q_side_table(Q, pk, sig, side, tab, q);
  q_side_msm(Q, rec, side, tab, bt, q);
  return ok;
}

// Q0 + E1 == O for side 0's point Q0 and side 1's point in cached add order
// (every lane of the quad computes the same answer)
PV_HD bool q_sum_is_identity(const qfe& Q0, const qfe& e1, const QRole& q) {
  qfe prod, u, a, b, c, d;
  q_add_stage1(prod, Q0, e1, q);
  q_add_stage2(u, prod, false, q);   // [rX, rY, rZ, rT]
  q_bcast<0>(a, u);
  q_bcast<1>(b, u);
  q_bcast<2>(c, u);
  q_bcast<3>(d, u);
  bool id = true;
#pragma unroll
  for (int j = 0; j < QL; ++j) {
    ge_p1p1 t;
    fe_copy(t.X, a.l[j]);
    fe_copy(t.Y, b.l[j]);
    fe_copy(t.Z, c.l[j]);
    fe_copy(t.T, d.l[j]);
    id = p1p1_is_identity(t);
  }
  return id;
}

// ------------------------------------------------------- prepared keys
// Latency verdict of a signature whose key is in the device key cache
// (k_verify_quad_keyed): -A is never decompressed.  The key's 8-way comb
// tables (key_prepare: k 2^(32 q) (-A), affine niels) and the radix-2^16
// chunk tables of B give R' = h(-A) + S B in 28 doublings and 80 affine adds
// (double_scalarmult_comb's schedule), split over the signature's KQ_SIDES
// lane quads: side s adds the key tables and the base-point chunks
// q = (8 / KQ_SIDES) s ..  + 8 / KQ_SIDES - 1, so with four sides a lane runs
// 28 (sq + mul) + 20 x 2 mul (two sides: 28 (sq + mul) + 40 x 2 mul; eight,
// the small-call form: 28 (sq + mul) + 10 x 2 mul).  The sides' points are
// then summed over a tree of exchanges (the kernel's shfl_xor 4, 8, 16;
// hc_verify_keyed_quad on the host).  libsodium accepts iff
// encode(R') == R, i.e. iff R decodes with a canonical y and R' + (-R) = O (the
// identity test of the half-size path, pv_lattice.h): -R is decoded while the
// scalar wave hashes, and side 0 tests the sides' total plus -R for O.
//
// record (LDS): h + the radix-16 digit offsets (8 words), pre-check verdict
constexpr int KQ_H = 0, KQ_OK = 8, KQ_WORDS = 9;
constexpr int KQ_SIDES = 4;   // lane quads per signature in k_verify_quad_keyed (8 per block)
constexpr int KQ_SIDES_SMALL = 8;   // ... in its small-call form (4 signatures per block)

PV_HD void keyed_record(uint32_t* rec, bool pre, const uint32_t dig[16]) {
  uint32_t hh[8];
  if (pre) {
    sc_reduce64(hh, dig);            // h = SHA-512(R||A||M) mod L (App. C.2 step 5)
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) hh[k] = 0;
  }
  sc_add_pattern(hh, hh, 0x88888888u);
#pragma unroll
  for (int k = 0; k < 8; ++k) rec[KQ_H + k] = hh[k];
  rec[KQ_OK] = pre ? 1u : 0u;
}

// SHA-512(R || A || M) as k_verify_quad_keyed's hash wave forms it (round 5):
// the message schedules of the first KQ_SCHED_BLOCKS blocks are computed first,
// one lane per (signature, block) of the wave (keyed_sched_block, all blocks'
// loads in flight at once), and the hashing lane runs only their 80 rounds
// (keyed_hash); later blocks are scheduled inline as in hash_one.  The same
// words as hash_one: the schedule is sha512_compress's, split in two.
constexpr int KQ_SCHED_BLOCKS = 4;   // messages up to 431 bytes
PV_HD void keyed_sched_block(uint64_t* kw, int stride, const uint8_t* sig, const uint8_t* pk, const uint8_t* m,
                             uint64_t mlen, uint64_t b) {
  uint64_t w[16];
  hram_block(w, sig, pk, m, mlen, b, hram_blocks(mlen));
  sha512_schedule_kw(kw, stride, w);
}
// kw + b * bstride: block b's K_t + W_t at stride `stride` (b < KQ_SCHED_BLOCKS)
PV_HD bool keyed_hash(uint32_t dig[16], const uint64_t* kw, int stride, int bstride, const uint8_t* sig,
                      const uint8_t* pk, const uint8_t* m, uint64_t mlen) {
  if (!precheck(pk, sig)) return false;
  uint64_t h[8], w[16];
  sha512_init(h);
  const uint64_t nb = hram_blocks(mlen);
  for (uint64_t b = 0; b < nb; ++b) {
    if (b < (uint64_t)KQ_SCHED_BLOCKS) {
      sha512_compress_kw(h, kw + b * (uint64_t)bstride, stride);
    } else {
      hram_block(w, sig, pk, m, mlen, b, nb);
      sha512_compress(h, w);
    }
  }
  sha512_digest_words(dig, h);
  return true;
}

// S's share of the comb, which needs no hash: with the signed radix-2^16
// digits of S (offset form), side s sums its chunks q = (8 / SIDES) s .. of the
// high halves (added at window 4, i.e. doubled 16 times) and of the low halves
// (added last) into two points, returned in cached add order.  Runs while the
// scalar wave hashes.
template <int SIDES = KQ_SIDES>
PV_HD void q_comb_base(qfe& e_hi, qfe& e_lo, const uint8_t* sig, int side, const uint32_t* bw, const QRole& q) {
  constexpr int KQ_TPS = 8 / SIDES;   // comb tables (and base-point chunks) per side
  uint32_t sp[8];
  load8(sp, sig + 32);
  sc_add_pattern(sp, sp, HALF_S_PATTERN);
  const uint32_t* bws = bw + (uint64_t)(KQ_TPS * side) * BW_TABLE;
  qfe ph, pl, eh[KQ_TPS], el[KQ_TPS];
#pragma unroll
  for (int k = 0; k < KQ_TPS; ++k) {
    const uint32_t wd = pick8(sp, KQ_TPS * side + k);
    const int dh = (int)(wd >> 16) - 32768, dl = (int)(wd & 0xffffu) - 32768;
    const uint32_t* t = bws + (uint64_t)k * BW_TABLE;
    q_load_niels(eh[k], t + (uint64_t)(dh < 0 ? -dh : dh) * BT_WORDS, dh < 0, q);
    q_load_niels(el[k], t + (uint64_t)(dl < 0 ? -dl : dl) * BT_WORDS, dl < 0, q);
  }
#pragma unroll
  for (int j = 0; j < QL; ++j) {
    role_p3_identity(ph.l[j], qrole(j, q));
    role_p3_identity(pl.l[j], qrole(j, q));
  }
#pragma unroll
  for (int k = 0; k < KQ_TPS; ++k) {
    const uint32_t wd = pick8(sp, KQ_TPS * side + k);
    q_add(ph, eh[k], (wd >> 16) < 32768u, q);
    q_add(pl, el[k], (wd & 0xffffu) < 32768u, q);
  }
  q_to_cached(e_hi, ph, q);
  q_to_cached(e_lo, pl, q);
}

// h's share of the comb on side s: the key tables q = (8 / SIDES) s .. (kt = the
// key's 8 comb tables), 8 windows of 4 doublings; the base-point sums of
// q_comb_base join at window 4 (e_hi) and after the last window (e_lo).  Each
// window's key entries are fetched before its doublings.
template <int SIDES = KQ_SIDES>
PV_HD void q_comb_side(qfe& acc, const uint32_t* rec, int side, const uint32_t* kt, const qfe& e_hi, const qfe& e_lo,
                       const QRole& q) {
  constexpr int KQ_TPS = 8 / SIDES;
  uint32_t hp[KQ_TPS];
#pragma unroll
  for (int k = 0; k < KQ_TPS; ++k) hp[k] = rec[KQ_H + KQ_TPS * side + k];
  const uint32_t* kts = kt + KQ_TPS * side * KT_TABLE;
#pragma unroll
  for (int j = 0; j < QL; ++j) role_p3_identity(acc.l[j], qrole(j, q));
#pragma unroll 1
  for (int w = 7; w >= 0; --w) {
    qfe ek[KQ_TPS];
    int dk[KQ_TPS];
#pragma unroll
    for (int k = 0; k < KQ_TPS; ++k) {
      dk[k] = (int)((hp[k] >> (4 * w)) & 15u) - 8;
      q_load_niels(ek[k], kts + k * KT_TABLE + (dk[k] < 0 ? -dk[k] : dk[k]) * KT_ENTRY, dk[k] < 0, q);
    }
    if (w != 7) {
#pragma unroll 1
      for (int k = 0; k < 4; ++k) q_dbl(acc, q);
    }
#pragma unroll
    for (int k = 0; k < KQ_TPS; ++k) q_add(acc, ek[k], dk[k] < 0, q);
    if (w == 4) q_add(acc, e_hi, false, q);
  }
  q_add(acc, e_lo, false, q);
}

// -R of the keyed verdict as k_verify_quad_keyed's decoding lane leaves it:
// 40 words in cached add order + the decode verdict (canonical y, on the curve)
PV_HD void keyed_neg_r(uint32_t* o, const uint8_t* sig) {
  uint32_t enc[8];
  load8(enc, sig);
  ge_p3 P;
  const bool ok = ge_frombytes_negate(P, enc) && y_is_canonical(enc);
  ge_cached c;
  ge_p3_to_cached(c, P);
  fe_carry(c.YmX);
  fe_carry(c.YpX);
  fe_carry(c.Z2);
  store_fe(o, c.YmX);
  store_fe(o + 10, c.YpX);
  store_fe(o + 20, c.T2d);
  store_fe(o + 30, c.Z2);
  o[40] = ok ? 1u : 0u;
}

}  // namespace pv
