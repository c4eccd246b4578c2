// One BLS COMMIT check over a lane PAIR (the kernel
// pvbls::k_bls_verify_pair).  The same check as bls_check (pv_bn254.h) --
// e(sigma, g) e(-H(m), pk) == 1 over the precomputed lines, one final
// exponentiation -- with every Fp12 split in halves between the two lanes:
//   role h = 0 computes and writes the a-half (the Fp6 coefficient of w^0),
//   role h = 1 the b-half (the coefficient of w),
// and each lane's work per step is ONE Fp6 product of the complex squaring, ONE
// sparse Fp6 product per line, three of the six Fp2 products of a cyclotomic
// squaring, two of the four Fp6 products of an Fp12 product.  Half the work per
// lane and half the registers: the kernel runs at 2 waves per SIMD (256
// registers) where the one-lane check needs 512.
//
// The two lanes run the same instruction stream; a role only selects operands
// (v_cndmask), never a branch, and the halves cross between the lanes with
// quad_perm DPP moves (v_mov_dpp [1,0,3,2]) -- always in pair-uniform control
// flow, so both lanes of a pair are active at every exchange.  The Miller
// accumulator and the cyclotomic powers live in LDS, one Fp12 per check shared
// by the pair (pslot); the final exponentiation's other values are halves in
// registers (p6).
//
// The host build (tools/hostcheck/bn254check.cpp) compiles the same code with
// both lanes of a pair emulated in one thread (PL = 2: element j plays role j,
// an exchange swaps the elements), so the column-sum bound checker and the C
// oracle cover exactly the formulas the kernel runs.
#pragma once
#include "pv_bn254.h"

// the final exponentiation's Fp12-half operations (out of line by default)
#ifndef PV_FE_CALL
#define PV_FE_CALL PV_BN_CALL
#endif
#ifndef PV_FE_DCALL
#define PV_FE_DCALL __device__ __noinline__
#endif
#ifndef PV_FE_F6MUL
#define PV_FE_F6MUL f6mul
#endif
// member functions (PV_HD may be `static inline` in the host checker)
#if defined(__HIPCC__)
#define PV_MD __host__ __device__ __forceinline__
#else
#define PV_MD inline
#endif

namespace bn {

#if defined(__HIP_DEVICE_COMPILE__)
constexpr int PL = 1;   // pair lanes held by one thread
#else
constexpr int PL = 2;
#endif

PV_HD int prole(int j) {
#if defined(__HIP_DEVICE_COMPILE__)
  (void)j;
  return (int)(threadIdx.x & 1);
#else
  return j;
#endif
}

struct p1 {
  fp e[PL];
};
struct p2 {
  fp2 e[PL];
};
struct p6 {
  fp6 e[PL];
};

#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ fp px_fp(const fp& x) {   // the partner lane's x
  fp r;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.l[i] = __builtin_amdgcn_mov_dpp(x.l[i], 0xB1, 0xf, 0xf, false);
  return r;
}
__device__ __forceinline__ fp2 px_fp2(const fp2& x) { return fp2{px_fp(x.a), px_fp(x.b)}; }
#endif
PV_HD p2 pswap(const p2& x) {
  p2 r;
#if defined(__HIP_DEVICE_COMPILE__)
  r.e[0] = px_fp2(x.e[0]);
#else
  r.e[0] = x.e[1];
  r.e[1] = x.e[0];
#endif
  return r;
}
PV_HD p6 pswap(const p6& x) {
  p6 r;
#if defined(__HIP_DEVICE_COMPILE__)
  r.e[0] = fp6{px_fp2(x.e[0].c0), px_fp2(x.e[0].c1), px_fp2(x.e[0].c2)};
#else
  r.e[0] = x.e[1];
  r.e[1] = x.e[0];
#endif
  return r;
}
// both lanes' flags ANDed
PV_HD bool pand(const bool (&ok)[PL]) {
#if defined(__HIP_DEVICE_COMPILE__)
  const int o = __builtin_amdgcn_mov_dpp((int)ok[0], 0xB1, 0xf, 0xf, false);
  return ok[0] && o;
#else
  return ok[0] && ok[1];
#endif
}

PV_HD void mp_fence() {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" ::: "memory");
#endif
}

// pin an Fp2 product's limbs in 32-bit registers: left alone, the compiler sinks
// a product's final column masks / carries to the (distant) uses and keeps the
// 64-bit column sums alive instead -- twice the registers -- which spilled the
// Miller loop to scratch at every line
PV_HD fp2 pin(fp2 x) {
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
  for (int i = 0; i < NL; ++i) asm volatile("" : "+v"(x.a.l[i]), "+v"(x.b.l[i]));
#endif
  return x;
}

// lazy (limbwise) helpers
PV_HD fp2 f2negL(const fp2& x) { return fp2{neg(x.a), neg(x.b)}; }
// role selects of values computed on both lanes (function arguments: both are
// evaluated, so the choice is a v_cndmask, never a divergent branch)
PV_HD fp fsel(bool h, const fp& x, const fp& y) { return h ? x : y; }
PV_HD fp2 f2sel(bool h, const fp2& x, const fp2& y) { return h ? x : y; }
PV_HD fp6 f6sel(bool h, const fp6& x, const fp6& y) { return h ? x : y; }

// the pair kernel's block: 128 checks, f of check c at word w -> mp_buf[w * 128 + c]
constexpr int MP_CHECKS = 128;
#if defined(__HIP_DEVICE_COMPILE__)
__shared__ uint32_t mp_buf[12 * NL * MP_CHECKS];
#endif

// one check's Fp12 in LDS, shared by its pair: word w at mp_buf[w * ST + c] on
// the device (indexed from the __shared__ array itself, so that every access is
// a ds_read / ds_write, never a flat access through a generic pointer), at
// p[w * ST] on the host (coefficient e = a.c0 a.c1 a.c2 b.c0 b.c1 b.c2 = 0..5,
// each fp2 as a then b)
//
// Banks: ds_read_b32 / ds_write_b32 conflict within a 32-lane half (16 checks),
// bank = dword address mod 32, and ST = 128 puts every word of check c on bank
// c.  The lanes of a pair often touch different halves of their Fp12 in one
// instruction (role 0 the b-half, role 1 the a-half), so the b-half of check c
// is stored in column c ^ 16: the two roles then always use disjoint banks.
template <int ST>
struct pslot {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t c;
  PV_MD uint32_t& at(int w, int e) const { return mp_buf[w * ST + (c ^ (e >= 3 ? 16u : 0u))]; }
#else
  uint32_t* p;
  PV_MD uint32_t& at(int w, int) const { return p[w * ST]; }
#endif
  PV_MD fp2 ld(int e) const {
    fp2 r;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      r.a.l[i] = (int32_t)at(2 * e * NL + i, e);
      r.b.l[i] = (int32_t)at((2 * e + 1) * NL + i, e);
    }
    return r;
  }
  PV_MD void st(int e, const fp2& x) const {
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      at(2 * e * NL + i, e) = (uint32_t)x.a.l[i];
      at((2 * e + 1) * NL + i, e) = (uint32_t)x.b.l[i];
    }
  }
  PV_MD fp6 ld6(int half) const { return fp6{ld(3 * half), ld(3 * half + 1), ld(3 * half + 2)}; }
  PV_MD void st6(int half, const fp6& x) const {
    st(3 * half, x.c0);
    st(3 * half + 1, x.c1);
    st(3 * half + 2, x.c2);
  }
};

// x (the Fp6 half `half` of the slot) * (b0 + b1 v), each Fp2 of x fetched when
// its product starts: f6mul01's five products folded into lazy output sums as
// they are formed (c0 = t0 + xi t3, c1 = m - t0 - t1, c2 = t1 + t2; |limb| <
// 3 * 2^28); the sum's product first, then b1's two, then b0's
template <int ST>
PV_HD fp6 mp_f6mul01(pslot<ST> S, int half, const fp2& b0, const fp2& b1) {
  const int X = 3 * half;
  fp2 c0, c1, c2;
  c1 = pin(f2mul(f2addL(S.ld(X), S.ld(X + 1)), f2add(b0, b1)));
  mp_fence();
  {
    const fp2 t1 = pin(f2mul(S.ld(X + 1), b1));
    c1 = f2subL(c1, t1);
    c2 = t1;
  }
  mp_fence();
  c0 = f2mulxiL(pin(f2mul(S.ld(X + 2), b1)));
  mp_fence();
  {
    const fp2 t0 = pin(f2mul(S.ld(X), b0));
    c0 = f2addL(c0, t0);
    c1 = f2subL(c1, t0);
  }
  mp_fence();
  c2 = f2addL(c2, pin(f2mul(S.ld(X + 2), b0)));
  return fp6{f2norm(c0), f2norm(c1), f2norm(c2)};
}

// f6mul_i(x, y) with each Fp2 product folded into the three lazy output sums as
// it is formed (|limb| < 7 * 2^28 as in f6mul_i) instead of holding all six
PV_HD fp6 f6mul_fold(const fp6& x, const fp6& y) {
  fp2 c0, c1, c2;
  {
    const fp2 v0 = pin(f2mul(x.c0, y.c0));
    c0 = v0;
    c1 = f2negL(v0);
    c2 = f2negL(v0);
  }
  {
    const fp2 v1 = pin(f2mul(x.c1, y.c1));
    c0 = f2subL(c0, f2mulxiL(v1));
    c1 = f2subL(c1, v1);
    c2 = f2addL(c2, v1);
  }
  {
    const fp2 v2 = pin(f2mul(x.c2, y.c2));
    const fp2 xv2 = f2mulxiL(v2);
    c0 = f2subL(c0, xv2);
    c1 = f2addL(c1, xv2);
    c2 = f2subL(c2, v2);
  }
  c0 = f2addL(c0, f2mulxiL(pin(f2mul(f2addL(x.c1, x.c2), f2add(y.c1, y.c2)))));
  c1 = f2addL(c1, pin(f2mul(f2addL(x.c0, x.c1), f2add(y.c0, y.c1))));
  c2 = f2addL(c2, pin(f2mul(f2addL(x.c0, x.c2), f2add(y.c0, y.c2))));
  return fp6{f2norm(c0), f2norm(c1), f2norm(c2)};
}

#if defined(__HIP_DEVICE_COMPILE__)
// ------------------------------------------------------------------ lane groups above the pair
// k_bls_verify_quad runs a check over a lane QUAD (two pairs, qrole = lane bit 1),
// k_bls_verify_oct over an OCTET (two quads, orole = lane bit 2); the other
// pair's value of the same role crosses with quad_perm [2,3,0,1], the other
// quad's with ds_swizzle (xor 4), both in group-uniform control flow
__device__ __forceinline__ fp qx_fp(const fp& x) {
  fp r;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.l[i] = __builtin_amdgcn_mov_dpp(x.l[i], 0x4E, 0xf, 0xf, false);
  return r;
}
__device__ __forceinline__ fp2 qx_fp2(const fp2& x) { return fp2{qx_fp(x.a), qx_fp(x.b)}; }
__device__ __forceinline__ p6 pqswap(const p6& x) {
  const fp6& c = x.e[0];
  p6 r;
  r.e[0] = fp6{qx_fp2(c.c0), qx_fp2(c.c1), qx_fp2(c.c2)};
  return r;
}
__device__ __forceinline__ bool qrole() { return (threadIdx.x >> 1) & 1; }
__device__ __forceinline__ fp ox_fp(const fp& x) {
  fp r;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.l[i] = __builtin_amdgcn_ds_swizzle(x.l[i], 0x101F);   // and 0x1f, xor 4
  return r;
}
__device__ __forceinline__ fp2 ox_fp2(const fp2& x) { return fp2{ox_fp(x.a), ox_fp(x.b)}; }
__device__ __forceinline__ bool orole() { return (threadIdx.x >> 2) & 1; }
template <int LV>
__device__ __forceinline__ fp2 sx_fp2(const fp2& x) { return LV == 1 ? qx_fp2(x) : ox_fp2(x); }
template <int LV>
__device__ __forceinline__ bool srole() { return LV == 1 ? qrole() : orole(); }

// f6mul_i's sums from the split products: the half g = 0 of the group level LV
// holds the diagonal p = v0, v1, v2, the half g = 1 the Karatsuba sums s12, s01, s02
template <int LV>
__device__ __forceinline__ fp6 f6_sums(const fp2& p0, const fp2& p1, const fp2& p2) {
  const bool g = srole<LV>();
  const fp2 o0 = sx_fp2<LV>(p0), o1 = sx_fp2<LV>(p1), o2 = sx_fp2<LV>(p2);
  const fp2 v0 = f2sel(g, o0, p0), v1 = f2sel(g, o1, p1), v2 = f2sel(g, o2, p2);
  const fp2 s12 = f2sel(g, p0, o0), s01 = f2sel(g, p1, o1), s02 = f2sel(g, p2, o2);
  fp6 r;
  r.c0 = f2norm(f2addL(f2mulxiL(f2subL(f2subL(s12, v1), v2)), v0));
  r.c1 = f2norm(f2addL(f2subL(f2subL(s01, v0), v1), f2mulxiL(v2)));
  r.c2 = f2norm(f2addL(f2subL(f2subL(s02, v0), v2), v1));
  return r;
}
// f6mul_i(x, y) with its six Fp2 products split over the level-LV halves
template <int LV>
__device__ __forceinline__ fp6 f6mul_s(const fp6& x, const fp6& y) {
  const bool g = srole<LV>();
  const fp2 p0 = pin(f2mul(f2sel(g, f2addL(x.c1, x.c2), x.c0), f2sel(g, f2add(y.c1, y.c2), y.c0)));
  const fp2 p1 = pin(f2mul(f2sel(g, f2addL(x.c0, x.c1), x.c1), f2sel(g, f2add(y.c0, y.c1), y.c1)));
  const fp2 p2 = pin(f2mul(f2sel(g, f2addL(x.c0, x.c2), x.c2), f2sel(g, f2add(y.c0, y.c2), y.c2)));
  return f6_sums<LV>(p0, p1, p2);
}
__device__ __forceinline__ fp6 f6mul_q(const fp6& x, const fp6& y) { return f6mul_s<1>(x, y); }
// the octet's Fp6 product split four ways: pair m's three products (as f6mul_q)
// with the first on quad g = 0, the third on g = 1, the second on both
__device__ __forceinline__ fp6 f6mul_o4(const fp6& x, const fp6& y) {
  const bool m = qrole(), g = orole();
  const fp2 xa0 = f2sel(m, f2addL(x.c1, x.c2), x.c0), ya0 = f2sel(m, f2add(y.c1, y.c2), y.c0);
  const fp2 xa2 = f2sel(m, f2addL(x.c0, x.c2), x.c2), ya2 = f2sel(m, f2add(y.c0, y.c2), y.c2);
  const fp2 pa = pin(f2mul(f2sel(g, xa2, xa0), f2sel(g, ya2, ya0)));
  const fp2 p1 = pin(f2mul(f2sel(m, f2addL(x.c0, x.c1), x.c1), f2sel(m, f2add(y.c0, y.c1), y.c1)));
  const fp2 oa = ox_fp2(pa);
  return f6_sums<1>(f2sel(g, oa, pa), p1, f2sel(g, pa, oa));
}
// mp_f6mul01 split over the octet's quads: g = 0 forms m and t1, g = 1 t0 and t2,
// both t3; the same sums (c0 = t0 + xi t3, c1 = m - t0 - t1, c2 = t1 + t2)
template <int ST>
__device__ __forceinline__ fp6 mo_f6mul01(pslot<ST> S, int half, const fp2& b0, const fp2& b1) {
  const int X = 3 * half;
  const bool g = orole();
  const fp2 pa = pin(f2mul(f2sel(g, S.ld(X), f2addL(S.ld(X), S.ld(X + 1))), f2sel(g, b0, f2add(b0, b1))));
  mp_fence();
  const fp2 pb = pin(f2mul(S.ld(g ? X + 2 : X + 1), f2sel(g, b0, b1)));
  mp_fence();
  const fp2 t3 = pin(f2mul(S.ld(X + 2), b1));
  const fp2 oa = ox_fp2(pa), ob = ox_fp2(pb);
  const fp2 m = f2sel(g, oa, pa), t0 = f2sel(g, pa, oa), t1 = f2sel(g, ob, pb), t2 = f2sel(g, pb, ob);
  return fp6{f2norm(f2addL(f2mulxiL(t3), t0)), f2norm(f2subL(f2subL(m, t1), t0)), f2norm(f2addL(t1, t2))};
}
#endif

// f = f (1 + (b0 + b1 v) w), f12mul_line_i split: role 0 forms v (f.b l) and
// writes f.a + v f.b l, role 1 forms f.a l and writes f.b + f.a l.  The line's
// coefficients b0 = B' x_P (role 0) and b1 = C' y_P (role 1) are exchanged;
// q holds each role's coordinate of P (x_P for role 0, y_P for role 1).
template <int ST, bool OCT = false>
PV_HD void mp_line(pslot<ST> S, const uint32_t* L, const p1& q) {
  p2 c;
#pragma unroll
  for (int j = 0; j < PL; ++j) c.e[j] = pin(f2mulfp(ld_f2(L + 2 * NL * prole(j)), q.e[j]));
  const p2 o = pswap(c);
  p6 P;
#pragma unroll
  for (int j = 0; j < PL; ++j) {
    const int h = prole(j);
    const fp2 b0 = f2sel(h, o.e[j], c.e[j]), b1 = f2sel(h, c.e[j], o.e[j]);
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (OCT) P.e[j] = mo_f6mul01(S, 1 - h, b0, b1); else
#endif
    P.e[j] = mp_f6mul01(S, 1 - h, b0, b1);
  }
  mp_fence();
#pragma unroll
  for (int j = 0; j < PL; ++j) {
    const int h = prole(j), E = 3 * h;
    const fp6& t = P.e[j];
    const fp2 q0 = f2sel(h, t.c0, f2mulxiL(t.c2)), q1 = f2sel(h, t.c1, t.c0), q2 = f2sel(h, t.c2, t.c1);
    S.st(E, f2norm(f2addL(S.ld(E), q0)));
    S.st(E + 1, f2norm(f2addL(S.ld(E + 1), q1)));
    S.st(E + 2, f2norm(f2addL(S.ld(E + 2), q2)));
  }
  mp_fence();
}

// f = f^2 (f12sqr_i's complex squaring split): role 0 forms s = (a + b)(a + v b),
// role 1 t = a b; t crosses to role 0, which writes s - t - v t, role 1 writes
// 2t (as p - (-p) - 0, the same integer as f2dbl)
template <int ST, bool OCT = false>
PV_HD fp6 mp_sqr_prod(pslot<ST> S, int h) {
  fp6 x, y;
  {
    const fp6 a = S.ld6(0), b = S.ld6(1);
    x = f6sel(h, a, f6add(a, b));
    y = f6sel(h, b, f6add(a, f6mulv(b)));
  }
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (OCT) return f6mul_s<2>(x, y);   // the octet's quads split the six products
#endif
  return f6mul_fold(x, y);
}
template <int ST, bool OCT = false>
PV_HD void mp_sqr(pslot<ST> S) {
  p6 P;
#pragma unroll
  for (int j = 0; j < PL; ++j) P.e[j] = mp_sqr_prod<ST, OCT>(S, prole(j));
  mp_fence();
  const p6 Q = pswap(P);
#pragma unroll
  for (int j = 0; j < PL; ++j) {
    const int h = prole(j);
    const fp6& p = P.e[j];
    const fp6& q = Q.e[j];
    const fp2 z = f2zero();
    const fp2 a0 = f2sel(h, f2negL(p.c0), q.c0), a1 = f2sel(h, f2negL(p.c1), q.c1), a2 = f2sel(h, f2negL(p.c2), q.c2);
    const fp2 c0 = f2sel(h, z, f2mulxiL(q.c2)), c1 = f2sel(h, z, q.c0), c2 = f2sel(h, z, q.c1);
    S.st6(h, fp6{f2norm(f2subL(f2subL(p.c0, a0), c0)), f2norm(f2subL(f2subL(p.c1, a1), c1)),
                 f2norm(f2subL(f2subL(p.c2, a2), c2))});
  }
  mp_fence();
}

// cyc_sqr_i split: of each Fp4 pair (z0, z1) -- A = (a.c0, b.c1), B = (b.c0,
// a.c2), C = (a.c1, b.c2) -- role 0 forms s = (z0 + z1)(xi z1 + z0), role 1
// tmp = z0 z1; tmp crosses to role 0.  Role 0 writes a.c0, a.c1, a.c2 =
// 3 t0 - 2 z (t0 = s - tmp - xi tmp of A, B, C), role 1 writes b.c1, b.c2,
// b.c0 = 3 t1 + 2 z (t1 = 2 tmp of A, B and xi 2 tmp of C).  Every sum is formed
// limbwise (|limb| < 2^31) and carried once: the same integers as fp4_sqr /
// three_minus_two / three_plus_two, so the same normalised limbs.
template <int ST>
PV_HD void mp_cyc_sqr(pslot<ST> S) {
  constexpr int Z0[3] = {0, 3, 1}, Z1[3] = {4, 2, 5}, O0[3] = {0, 1, 2}, O1[3] = {4, 5, 3};
  p2 P[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
#pragma unroll
    for (int j = 0; j < PL; ++j) {
      const int h = prole(j);
      const fp2 z0 = S.ld(Z0[k]), z1 = S.ld(Z1[k]);
      const fp2 x = f2sel(h, z0, f2addL(z0, z1));                    // lazy factor
      const fp2 y = f2sel(h, z1, f2norm(f2addL(f2mulxiL(z1), z0)));   // normalised factor
      P[k].e[j] = pin(f2mul(x, y));
    }
    mp_fence();
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const p2 Q = pswap(P[k]);
#pragma unroll
    for (int j = 0; j < PL; ++j) {
      const int h = prole(j);
      const fp2& p = P[k].e[j];
      // u = a - b - c: role 0 s - tmp - xi tmp, role 1 2 tmp = a - (-a) - 0 (a = xi tmp for C)
      const fp2 a = k == 2 ? f2sel(h, f2mulxiL(p), p) : p;
      const fp2 u = f2norm(f2subL(f2subL(a, f2sel(h, f2negL(a), Q.e[j])), f2sel(h, f2zero(), f2mulxiL(Q.e[j]))));
      const int e = h ? O1[k] : O0[k];
      const fp2 zz = S.ld(e);
      const fp2 zs = f2sel(h, zz, f2negL(zz));   // 3u - 2z (role 0) / 3u + 2z (role 1)
      S.st(e, f2norm(f2addL(f2addL(f2addL(u, u), u), f2addL(zs, zs))));
    }
  }
  mp_fence();
}
template <int ST>
PV_HD void mp_reduce(pslot<ST> S) {
#pragma unroll
  for (int j = 0; j < PL; ++j) {
    const int h = prole(j);
#pragma unroll 1
    for (int k = 0; k < 3; ++k) S.st(3 * h + k, f2reduce(S.ld(3 * h + k)));
  }
  mp_fence();
}
template <int ST>
PV_HD void mp_put(pslot<ST> S, const p6& x) {
#pragma unroll
  for (int j = 0; j < PL; ++j) S.st6(prole(j), x.e[j]);
  mp_fence();
}
template <int ST>
PV_HD p6 mp_get(pslot<ST> S) {
  p6 r;
#pragma unroll
  for (int j = 0; j < PL; ++j) r.e[j] = S.ld6(prole(j));
  return r;
}

// ------------------------------------------------------------------ Fp12 halves (p6)
// x y, f12mul's Karatsuba split: role 0 forms t0 = x.a y.a, role 1 t1 = x.b y.b
// (one Fp6 product each, from the lane's own halves); the third product s =
// (x.a + x.b)(y.a + y.b) is split at the Fp2 level -- role 0 forms its v0, v1,
// v2, role 1 its s12, s01, s02.  Role 0 writes t0 + v t1, role 1 s - t0 - t1:
// the same sums as f12mul, so the same limbs.
// the sums of pr_mul from the lane's own-half product t and the three Fp2
// products m of s (role 0 v0, v1, v2; role 1 s12, s01, s02)
PV_HD p6 pr_mul_tail(const p6& t, const p2 (&m)[3]) {
  const p6 to = pswap(t);
  const p2 mo[3] = {pswap(m[0]), pswap(m[1]), pswap(m[2])};
  p6 r;
#pragma unroll
  for (int j = 0; j < PL; ++j) {
    const int h = prole(j);
    const fp6& t0 = h ? to.e[j] : t.e[j];
    const fp6& t1 = h ? t.e[j] : to.e[j];
    // s (role 1's view: v's from role 0)
    const fp2 &v0 = mo[0].e[j], &v1 = mo[1].e[j], &v2 = mo[2].e[j];
    const fp2 &s12 = m[0].e[j], &s01 = m[1].e[j], &s02 = m[2].e[j];
    const fp2 sc0 = f2norm(f2addL(f2mulxiL(f2subL(f2subL(s12, v1), v2)), v0));
    const fp2 sc1 = f2norm(f2addL(f2subL(f2subL(s01, v0), v1), f2mulxiL(v2)));
    const fp2 sc2 = f2norm(f2addL(f2subL(f2subL(s02, v0), v2), v1));
    const fp6 rb{f2norm(f2subL(f2subL(sc0, t0.c0), t1.c0)), f2norm(f2subL(f2subL(sc1, t0.c1), t1.c1)),
                 f2norm(f2subL(f2subL(sc2, t0.c2), t1.c2))};
    const fp6 ra{f2norm(f2addL(t0.c0, f2mulxiL(t1.c2))), f2norm(f2addL(t0.c1, t1.c0)), f2norm(f2addL(t0.c2, t1.c1))};
    r.e[j] = f6sel(h, rb, ra);
  }
  return r;
}
PV_FE_CALL p6 pr_mul(const p6& x, const p6& y) {
  p6 t;   // the out-of-line product first: nothing else is live across the call
#pragma unroll
  for (int j = 0; j < PL; ++j) t.e[j] = PV_FE_F6MUL(x.e[j], y.e[j]);
  p2 m[3];
  {
    const p6 xo = pswap(x), yo = pswap(y);
#pragma unroll
    for (int j = 0; j < PL; ++j) {
      const int h = prole(j);
      const fp6 X = f6add(x.e[j], xo.e[j]), Y = f6add(y.e[j], yo.e[j]);
      // role 0: X_k Y_k (k = 0, 1, 2); role 1: (X_a + X_b)(Y_a + Y_b) for (a, b) = (1, 2), (0, 1), (0, 2)
      m[0].e[j] = f2mul(f2sel(h, f2addL(X.c1, X.c2), X.c0), f2sel(h, f2add(Y.c1, Y.c2), Y.c0));
      m[1].e[j] = f2mul(f2sel(h, f2addL(X.c0, X.c1), X.c1), f2sel(h, f2add(Y.c0, Y.c1), Y.c1));
      m[2].e[j] = f2mul(f2sel(h, f2addL(X.c0, X.c2), X.c2), f2sel(h, f2add(Y.c0, Y.c2), Y.c2));
    }
  }
  return pr_mul_tail(t, m);
}
PV_HD p6 pr_conj(const p6& x) {
  p6 r;
#pragma unroll
  for (int j = 0; j < PL; ++j) r.e[j] = f6sel(prole(j), f6neg(x.e[j]), x.e[j]);
  return r;
}
// 1 / x = (a - b w) / (a^2 - v b^2): role 0 squares a, role 1 b; both invert
// the same Fp6 norm
PV_FE_CALL p6 pr_inv(const p6& x) {
  p6 sq;
#pragma unroll
  for (int j = 0; j < PL; ++j) sq.e[j] = PV_FE_F6MUL(x.e[j], x.e[j]);
  const p6 so = pswap(sq);
  p6 r;
#pragma unroll
  for (int j = 0; j < PL; ++j) {
    const int h = prole(j);
    const fp6 d = f6inv(f6sub(f6sel(h, so.e[j], sq.e[j]), f6mulv(f6sel(h, sq.e[j], so.e[j]))));
    const fp6 m = PV_FE_F6MUL(x.e[j], d);
    r.e[j] = f6sel(h, f6neg(m), m);
  }
  return r;
}
// Frobenius maps on the lane's own coefficients (f12frob1/2/3): role 0 holds
// w^0, w^2, w^4 (gamma_{n,0} = 1, gamma_{n,2}, gamma_{n,4}), role 1 w^1, w^3,
// w^5 -- one multiply per coefficient with the role's constant (role 0 times
// the Montgomery one for w^0)
PV_HD p6 pr_frob_odd(const p6& x, int n, const uint32_t* const (&g)[10]) {
  p6 r;
#pragma unroll
  for (int j = 0; j < PL; ++j) {
    const int h = prole(j);
    const fp6& c = x.e[j];
    const fp2 one = f2one();
    r.e[j].c0 = f2mul(f2conj(c.c0), f2sel(h, f2cst(g[0], g[1]), one));
    r.e[j].c1 = f2mul(f2conj(c.c1), f2sel(h, f2cst(g[4], g[5]), f2cst(g[2], g[3])));
    r.e[j].c2 = f2mul(f2conj(c.c2), f2sel(h, f2cst(g[8], g[9]), f2cst(g[6], g[7])));
  }
  (void)n;
  return r;
}
PV_FE_CALL p6 pr_frob1(const p6& x) {
  const uint32_t* const g[10] = {G1_1_A, G1_1_B, G1_2_A, G1_2_B, G1_3_A, G1_3_B, G1_4_A, G1_4_B, G1_5_A, G1_5_B};
  return pr_frob_odd(x, 1, g);
}
PV_FE_CALL p6 pr_frob3(const p6& x) {
  const uint32_t* const g[10] = {G3_1_A, G3_1_B, G3_2_A, G3_2_B, G3_3_A, G3_3_B, G3_4_A, G3_4_B, G3_5_A, G3_5_B};
  return pr_frob_odd(x, 3, g);
}
PV_FE_CALL p6 pr_frob2(const p6& x) {
  p6 r;
#pragma unroll
  for (int j = 0; j < PL; ++j) {
    const int h = prole(j);
    const fp6& c = x.e[j];
    r.e[j].c0 = f2mulfp(c.c0, fsel(h, cst(G2_1_A), fone()));
    r.e[j].c1 = f2mulfp(c.c1, fsel(h, cst(G2_3_A), cst(G2_2_A)));
    r.e[j].c2 = f2mulfp(c.c2, fsel(h, cst(G2_5_A), cst(G2_4_A)));
  }
  return r;
}
PV_HD bool pr_is_one(const p6& x) {
  bool ok[PL];
#pragma unroll
  for (int j = 0; j < PL; ++j) {
    const fp6& c = x.e[j];
    const bool rest = f2is_zero(c.c1) && f2is_zero(c.c2) && is_zero(c.c0.b);
    ok[j] = rest && (prole(j) ? is_zero(c.c0.a) : eq(c.c0.a, fone()));
  }
  return pand(ok);
}

// ------------------------------------------------------------------ lane-QUAD final exponentiation
// In k_bls_verify_quad the two lane pairs of a check (qrole g = 0 / 1) hold the
// SAME Fp12 halves after the Miller product -- bit-identical, since both pairs
// form the same sums of the same products -- and split the Fp2 products of each
// final-exponentiation step between them, exchanging results with quad_perm
// [2,3,0,1] DPP moves:
//   an Fp6 product (f6mul_q): g = 0 forms the diagonal v0, v1, v2, g = 1 the
//   three Karatsuba sums s12, s01, s02 -- 3 products in sequence instead of 6;
//   an Fp12 product (pr_mul_q): that split for the lane's half product t, m0 of
//   the third product on g = 0, m1 on g = 1, m2 on both -- 5 instead of 9;
//   a cyclotomic squaring (mq_cyc_sqr): the Fp4 squaring k = g, then k = 2 on
//   both pairs -- 2 instead of 3 -- on the quad's shared LDS slot (the even
//   pair's), each pair writing its own k's coefficients and g = 0 those of k = 2.
// Every sum is the pair version's (the same integers, so the same limbs).  The
// host build has no quad: there pmul / pcyc / preduce / pinv are the pair ops.
#if defined(__HIP_DEVICE_COMPILE__)
PV_FE_DCALL p6 pr_mul_q(const p6& x, const p6& y) {
  const int h = prole(0);
  const bool g = qrole();
  p6 t;
  t.e[0] = f6mul_q(x.e[0], y.e[0]);
  p2 m[3];
  {
    const p6 xo = pswap(x), yo = pswap(y);
    const fp6 X = f6add(x.e[0], xo.e[0]), Y = f6add(y.e[0], yo.e[0]);
    const fp2 a0 = f2sel(h, f2addL(X.c1, X.c2), X.c0), b0 = f2sel(h, f2add(Y.c1, Y.c2), Y.c0);
    const fp2 a1 = f2sel(h, f2addL(X.c0, X.c1), X.c1), b1 = f2sel(h, f2add(Y.c0, Y.c1), Y.c1);
    const fp2 ma = pin(f2mul(f2sel(g, a1, a0), f2sel(g, b1, b0)));   // m0 (g = 0) / m1 (g = 1)
    m[2].e[0] = pin(f2mul(f2sel(h, f2addL(X.c0, X.c2), X.c2), f2sel(h, f2add(Y.c0, Y.c2), Y.c2)));
    const fp2 mo = qx_fp2(ma);
    m[0].e[0] = f2sel(g, mo, ma);
    m[1].e[0] = f2sel(g, ma, mo);
  }
  return pr_mul_tail(t, m);
}
// pr_inv with its two Fp6 products split (the Fp6 inverse runs on both pairs)
PV_FE_DCALL p6 pr_inv_q(const p6& x) {
  p6 sq;
  sq.e[0] = f6mul_q(x.e[0], x.e[0]);
  const p6 so = pswap(sq);
  const int h = prole(0);
  const fp6 d = f6inv(f6sub(f6sel(h, so.e[0], sq.e[0]), f6mulv(f6sel(h, sq.e[0], so.e[0]))));
  const fp6 m = f6mul_q(x.e[0], d);
  p6 r;
  r.e[0] = f6sel(h, f6neg(m), m);
  return r;
}
// mp_cyc_sqr over the quad's shared slot: Fp4 squarings k = g and k = 2.  Every
// read of the slot precedes every write (the pairs read coefficients the other
// pair writes).
template <int ST>
__device__ __forceinline__ void mq_cyc_sqr(pslot<ST> S) {
  const int h = prole(0);
  const bool g = qrole();
  // Z0 = {0, 3, 1}, Z1 = {4, 2, 5}; outputs O0 = {0, 1, 2} (role 0), O1 = {4, 5, 3} (role 1)
  fp2 pa, p2v;
  {
    const fp2 z0 = S.ld(g ? 3 : 0), z1 = S.ld(g ? 2 : 4);
    pa = pin(f2mul(f2sel(h, z0, f2addL(z0, z1)), f2sel(h, z1, f2norm(f2addL(f2mulxiL(z1), z0)))));
  }
  mp_fence();
  {
    const fp2 z0 = S.ld(1), z1 = S.ld(5);
    p2v = pin(f2mul(f2sel(h, z0, f2addL(z0, z1)), f2sel(h, z1, f2norm(f2addL(f2mulxiL(z1), z0)))));
  }
  const int ea = h ? (g ? 5 : 4) : (g ? 1 : 0), e2 = h ? 3 : 2;
  const fp2 za = S.ld(ea), z2 = S.ld(e2);
  mp_fence();
  fp2 outa, out2;
  {
    const fp2 q = px_fp2(pa);
    const fp2 u = f2norm(f2subL(f2subL(pa, f2sel(h, f2negL(pa), q)), f2sel(h, f2zero(), f2mulxiL(q))));
    const fp2 zs = f2sel(h, za, f2negL(za));
    outa = f2norm(f2addL(f2addL(f2addL(u, u), u), f2addL(zs, zs)));
  }
  {
    const fp2 q = px_fp2(p2v);
    const fp2 a = f2sel(h, f2mulxiL(p2v), p2v);
    const fp2 u = f2norm(f2subL(f2subL(a, f2sel(h, f2negL(a), q)), f2sel(h, f2zero(), f2mulxiL(q))));
    const fp2 zs = f2sel(h, z2, f2negL(z2));
    out2 = f2norm(f2addL(f2addL(f2addL(u, u), u), f2addL(zs, zs)));
  }
  S.st(ea, outa);
  if (!g) S.st(e2, out2);
  mp_fence();
}
// mp_reduce over the quad: components g and 2 of the lane's half
template <int ST>
__device__ __forceinline__ void mq_reduce(pslot<ST> S) {
  const int h = prole(0);
  const bool g = qrole();
  const int ea = 3 * h + (int)g, e2 = 3 * h + 2;
  const fp2 ra = f2reduce(S.ld(ea)), r2 = f2reduce(S.ld(e2));
  mp_fence();
  S.st(ea, ra);
  if (!g) S.st(e2, r2);
  mp_fence();
}
// ---- the octet (k_bls_verify_oct): the quad's split, each pair's share split
// again between the two quads (orole g)
// x y: of pair m's five products (its three of t, its m-product ma, and m2) quad
// g = 0 forms t's first and second and m2, g = 1 t's third, ma and m2
PV_FE_DCALL p6 pr_mul_o(const p6& x, const p6& y) {
  const int h = prole(0);
  const bool m = qrole(), g = orole();
  const fp6 &xs = x.e[0], &ys = y.e[0];
  p6 t;
  p2 mm[3];
  {
    const p6 xo = pswap(x), yo = pswap(y);
    const fp6 X = f6add(xs, xo.e[0]), Y = f6add(ys, yo.e[0]);
    const fp2 t0x = f2sel(m, f2addL(xs.c1, xs.c2), xs.c0), t0y = f2sel(m, f2add(ys.c1, ys.c2), ys.c0);
    const fp2 t1x = f2sel(m, f2addL(xs.c0, xs.c1), xs.c1), t1y = f2sel(m, f2add(ys.c0, ys.c1), ys.c1);
    const fp2 t2x = f2sel(m, f2addL(xs.c0, xs.c2), xs.c2), t2y = f2sel(m, f2add(ys.c0, ys.c2), ys.c2);
    const fp2 a0 = f2sel(h, f2addL(X.c1, X.c2), X.c0), b0 = f2sel(h, f2add(Y.c1, Y.c2), Y.c0);
    const fp2 a1 = f2sel(h, f2addL(X.c0, X.c1), X.c1), b1 = f2sel(h, f2add(Y.c0, Y.c1), Y.c1);
    const fp2 max = f2sel(m, a1, a0), may = f2sel(m, b1, b0);   // m0 (pair 0) / m1 (pair 1)
    const fp2 pa = pin(f2mul(f2sel(g, t2x, t0x), f2sel(g, t2y, t0y)));   // t0 / t2
    const fp2 pb = pin(f2mul(f2sel(g, max, t1x), f2sel(g, may, t1y)));   // t1 / ma
    mm[2].e[0] = pin(f2mul(f2sel(h, f2addL(X.c0, X.c2), X.c2), f2sel(h, f2add(Y.c0, Y.c2), Y.c2)));
    const fp2 oa = ox_fp2(pa), ob = ox_fp2(pb);
    t.e[0] = f6_sums<1>(f2sel(g, oa, pa), f2sel(g, ob, pb), f2sel(g, pa, oa));
    const fp2 ma = f2sel(g, pb, ob);
    const fp2 mo = qx_fp2(ma);
    mm[0].e[0] = f2sel(m, mo, ma);
    mm[1].e[0] = f2sel(m, ma, mo);
  }
  return pr_mul_tail(t, mm);
}
PV_FE_DCALL p6 pr_inv_o(const p6& x) {
  p6 sq;
  sq.e[0] = f6mul_o4(x.e[0], x.e[0]);
  const p6 so = pswap(sq);
  const int h = prole(0);
  const fp6 d = f6inv(f6sub(f6sel(h, so.e[0], sq.e[0]), f6mulv(f6sel(h, sq.e[0], so.e[0]))));
  const fp6 m = f6mul_o4(x.e[0], d);
  p6 r;
  r.e[0] = f6sel(h, f6neg(m), m);
  return r;
}
// mp_cyc_sqr over the octet's shared slot: quad g = 0 squares the Fp4 pair k = m,
// g = 1 the pair k = 2 (written by pair 0 of that quad); every read before every write
template <int ST>
__device__ __forceinline__ void mo_cyc_sqr(pslot<ST> S) {
  const int h = prole(0);
  const bool m = qrole(), g = orole();
  const fp2 z0 = S.ld(g ? 1 : (m ? 3 : 0)), z1 = S.ld(g ? 5 : (m ? 2 : 4));
  const fp2 p = pin(f2mul(f2sel(h, z0, f2addL(z0, z1)), f2sel(h, z1, f2norm(f2addL(f2mulxiL(z1), z0)))));
  const int e = g ? (h ? 3 : 2) : (h ? (m ? 5 : 4) : (m ? 1 : 0));
  const fp2 zz = S.ld(e);
  mp_fence();
  const fp2 q = px_fp2(p);
  const fp2 a = f2sel(g, f2sel(h, f2mulxiL(p), p), p);
  const fp2 u = f2norm(f2subL(f2subL(a, f2sel(h, f2negL(a), q)), f2sel(h, f2zero(), f2mulxiL(q))));
  const fp2 zs = f2sel(h, zz, f2negL(zz));
  const fp2 out = f2norm(f2addL(f2addL(f2addL(u, u), u), f2addL(zs, zs)));
  if (!(g && m)) S.st(e, out);
  mp_fence();
}
template <int ST>
__device__ __forceinline__ void mo_reduce(pslot<ST> S) {
  const int h = prole(0);
  const bool m = qrole(), g = orole();
  const int e = 3 * h + (g ? 2 : (int)m);
  const fp2 r = f2reduce(S.ld(e));
  mp_fence();
  if (!(g && m)) S.st(e, r);
  mp_fence();
}
#endif
// the final exponentiation's operations at group level LV (0 pair, 1 quad, 2 octet)
template <int LV>
PV_HD p6 pmul(const p6& x, const p6& y) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (LV == 1) return pr_mul_q(x, y);
  if constexpr (LV == 2) return pr_mul_o(x, y);
#endif
  return pr_mul(x, y);
}
template <int LV>
PV_HD p6 pinv(const p6& x) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (LV == 1) return pr_inv_q(x);
  if constexpr (LV == 2) return pr_inv_o(x);
#endif
  return pr_inv(x);
}
template <int LV, int ST>
PV_HD void pcyc(pslot<ST> S) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (LV == 1) return mq_cyc_sqr(S);
  if constexpr (LV == 2) return mo_cyc_sqr(S);
#endif
  mp_cyc_sqr(S);
}
template <int LV, int ST>
PV_HD void preduce(pslot<ST> S) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (LV == 1) return mq_reduce(S);
  if constexpr (LV == 2) return mo_reduce(S);
#endif
  mp_reduce(S);
}

// x^u in the cyclotomic subgroup (cyc_pow_u's chain) with the power in the slot
template <int ST, int LV = 0>
PV_BN_CALL p6 pr_pow_u(pslot<ST> S, const p6& x) {
  mp_put(S, x);
  for (int i = 0; i < 7; ++i) {
    pcyc<LV>(S);
    if ((i & 3) == 3) preduce<LV>(S);
  }
  mp_put(S, pmul<LV>(mp_get(S), x));   // x^(2^7 + 1)
  for (int i = 0; i < 55; ++i) {
    pcyc<LV>(S);
    if ((i & 3) == 3) preduce<LV>(S);
  }
  return pr_conj(pmul<LV>(mp_get(S), x));   // x^(2^62 + 2^55 + 1), conjugated
}
template <int ST, int LV = 0>
PV_BN_CALL p6 pr_cyc_sqr(pslot<ST> S, const p6& x) {
  mp_put(S, x);
  pcyc<LV>(S);
  return mp_get(S);
}

// ---- the pair kernel's final exponentiation as a step program (round 6,
// VERDICT r5 item 2).  Out of line, every Fp12-half product, inverse and
// Frobenius map of the chain below is a call that saves and restores the
// callee-saved VGPRs it uses (145 KB of scratch traffic per check,
// profiles/r04_bls_pmc.json); round 5 inlined them into one loop and the
// product's working set -- x, y, their swapped halves, t, the three Fp2
// products, ~360 VGPRs -- spilled (238 KB).  Here the loop holds ONE copy of
// each operation and the product streams its first operand from the check's
// LDS slot (both halves: the lane's own for t, both for the Karatsuba sums, so
// no swapped copy of x is ever held), the second operand's partner half crosses
// one Fp2 at a time, and the result's sums take the partner's products one Fp2
// at a time: the product needs y, t and m (~180 VGPRs) instead of ~360.
// The chain's long-lived values (f, f^u, f^u^2, t0, t1) are parked in a private
// array (FX_SLOTS halves).  A step: acc = post(op(pre_a(X_a), pre_b(X_b))), X =
// acc (FX_ACC) or a parked slot, pre = the Frobenius map n (bits 0-1) then a
// conjugation (bit 2); op FX_MUL the product, FX_INV the inverse of X_a, FX_CYC n
// cyclotomic squarings of X_a in the LDS slot (n in the b field, a reduction
// after every fourth: pr_pow_u's schedule); post = conjugation; then acc may be
// parked.  The operands and their order are final_exp's (the chain below), and
// every product forms pr_mul's sums, so every value has the same limbs.
// PV_FE_PROG = 0 builds the chain of calls (A/B).
#ifndef PV_FE_PROG
#define PV_FE_PROG 1
#endif
#ifndef PV_FX_YHOLD
#define PV_FX_YHOLD 0   // 1: the three Y = y + y' held through the m products (A/B)
#endif
constexpr uint32_t FX_MUL = 0, FX_INV = 1, FX_CYC = 2;
constexpr uint32_t FX_ACC = 7, FX_NONE = 15;
constexpr int FX_SLOTS = 5;   // 0 f (f0 before step 2), 1 f^u, 2 f^u^2, 3 t0, 4 t1
constexpr uint32_t FX_CONJ = 4, FX_F1 = 1, FX_F2 = 2, FX_F3 = 3;
constexpr uint32_t fx(uint32_t op, uint32_t a, uint32_t pa, uint32_t b, uint32_t pb, uint32_t post, uint32_t park) {
  return op | a << 4 | pa << 8 | b << 12 | pb << 20 | post << 24 | park << 28;
}
constexpr uint32_t fx_mul(uint32_t a, uint32_t pa, uint32_t b, uint32_t pb, uint32_t post = 0,
                          uint32_t park = FX_NONE) {
  return fx(FX_MUL, a, pa, b, pb, post, park);
}
constexpr uint32_t fx_cyc(uint32_t a, uint32_t n, uint32_t park = FX_NONE) { return fx(FX_CYC, a, 0, n, 0, 0, park); }
constexpr int FX_STEPS = 32;
constexpr uint32_t FX_PROG[FX_STEPS] = {
    fx(FX_INV, FX_ACC, 0, 0, 0, 0, FX_NONE),              //  0 1 / f0
    fx_mul(0, FX_CONJ, FX_ACC, 0),                        //  1 conj(f0) / f0
    fx_mul(FX_ACC, FX_F2, FX_ACC, 0, 0, 0),               //  2 f = frob2(f) f
    fx_cyc(FX_ACC, 7), fx_mul(FX_ACC, 0, 0, 0),           //  3, 4 pow_u(f)
    fx_cyc(FX_ACC, 55), fx_mul(FX_ACC, 0, 0, 0, 1, 1),    //  5, 6 -> fu
    fx_cyc(FX_ACC, 7), fx_mul(FX_ACC, 0, 1, 0),           //  7, 8 pow_u(fu)
    fx_cyc(FX_ACC, 55), fx_mul(FX_ACC, 0, 1, 0, 1, 2),    //  9, 10 -> fu2
    fx_cyc(FX_ACC, 7), fx_mul(FX_ACC, 0, 2, 0),           // 11, 12 pow_u(fu2)
    fx_cyc(FX_ACC, 55), fx_mul(FX_ACC, 0, 2, 0, 1),       // 13, 14 -> fu3
    fx_mul(FX_ACC, 0, FX_ACC, FX_F1, 1),                  // 15 y6 = conj(fu3 frob1(fu3))
    fx_cyc(FX_ACC, 1, 3),                                 // 16 t0 = cyc_sqr(y6)
    fx_mul(1, 0, 2, FX_F1, 1),                            // 17 conj(fu frob1(fu2))
    fx_mul(3, 0, FX_ACC, 0),                              // 18 t0 = t0 (17)
    fx_mul(FX_ACC, 0, 2, FX_CONJ, 0, 3),                  // 19 t0 = t0 y5, y5 = conj(fu2)
    fx_mul(1, FX_F1 | FX_CONJ, 2, FX_CONJ),               // 20 conj(frob1(fu)) y5
    fx_mul(FX_ACC, 0, 3, 0, 0, 4),                        // 21 t1 = (20) t0
    fx_mul(3, 0, 2, FX_F2, 0, 3),                         // 22 t0 = t0 frob2(fu2)
    fx_cyc(4, 1), fx_mul(FX_ACC, 0, 3, 0),                // 23, 24 t1 = cyc_sqr(t1) t0
    fx_cyc(FX_ACC, 1, 4),                                 // 25 t1 = cyc_sqr(t1)
    fx_mul(FX_ACC, 0, 0, FX_CONJ, 0, 3),                  // 26 t0 = t1 conj(f)
    fx_mul(0, FX_F1, 0, FX_F2),                           // 27 frob1(f) frob2(f)
    fx_mul(FX_ACC, 0, 0, FX_F3),                          // 28 y0 = (27) frob3(f)
    fx_mul(4, 0, FX_ACC, 0, 0, 4),                        // 29 t1 = t1 y0
    fx_cyc(3, 1), fx_mul(FX_ACC, 0, 4, 0),                // 30, 31 cyc_sqr(t0) t1
};
static_assert(FX_PROG[FX_STEPS - 1] == fx_mul(FX_ACC, 0, 4, 0), "program length");
#if defined(__HIPCC__)
// the device copy the kernel reads with a lane-indexed vector load
__device__ const uint32_t FX_PROG_DEV[FX_STEPS] = {
    FX_PROG[0], FX_PROG[1], FX_PROG[2], FX_PROG[3], FX_PROG[4], FX_PROG[5], FX_PROG[6], FX_PROG[7],
    FX_PROG[8], FX_PROG[9], FX_PROG[10], FX_PROG[11], FX_PROG[12], FX_PROG[13], FX_PROG[14], FX_PROG[15],
    FX_PROG[16], FX_PROG[17], FX_PROG[18], FX_PROG[19], FX_PROG[20], FX_PROG[21], FX_PROG[22], FX_PROG[23],
    FX_PROG[24], FX_PROG[25], FX_PROG[26], FX_PROG[27], FX_PROG[28], FX_PROG[29], FX_PROG[30], FX_PROG[31]};
#endif

// limbwise role select (v_cndmask per limb): a select of whole structs can be
// lowered to a select of their addresses, which puts both in scratch
PV_HD fp2 f2pick(bool h, const fp2& x, const fp2& y) {
  fp2 r;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    r.a.l[i] = h ? x.a.l[i] : y.a.l[i];
    r.b.l[i] = h ? x.b.l[i] : y.b.l[i];
  }
  return r;
}

// coefficient k of a lane's Fp6 half (k a compile-time constant after unrolling)
PV_HD const fp2& f6c(const fp6& x, int k) { return k == 0 ? x.c0 : (k == 1 ? x.c1 : x.c2); }
PV_HD p2 p6c(const p6& x, int k) {
  p2 r;
#pragma unroll
  for (int j = 0; j < PL; ++j) r.e[j] = f6c(x.e[j], k);
  return r;
}

// gamma_{n,e} (the Frobenius map n's constant of the coefficient of w^e, e =
// 2k + role; e = 0: the Montgomery one) as (a, b) limb pointers.  Indexed with
// compile-time k only (the callers unroll k), so every constant is an immediate:
// the check kernels read no data through the scalar cache beyond their kernel
// arguments (tests/test_isa_guards.py), and n, a wave-uniform runtime value,
// selects between immediates, never between addresses.
PV_BN_CONST uint32_t FX_ZERO[NL] = {};
PV_BN_CONST const uint32_t* FX_GP[3][6][2] = {
    {{ONE_M, FX_ZERO}, {G1_1_A, G1_1_B}, {G1_2_A, G1_2_B}, {G1_3_A, G1_3_B}, {G1_4_A, G1_4_B}, {G1_5_A, G1_5_B}},
    {{ONE_M, FX_ZERO}, {G2_1_A, FX_ZERO}, {G2_2_A, FX_ZERO}, {G2_3_A, FX_ZERO}, {G2_4_A, FX_ZERO}, {G2_5_A, FX_ZERO}},
    {{ONE_M, FX_ZERO}, {G3_1_A, G3_1_B}, {G3_2_A, G3_2_B}, {G3_3_A, G3_3_B}, {G3_4_A, G3_4_B}, {G3_5_A, G3_5_B}},
};
PV_HD fp fx_cst_sel(bool c, const uint32_t* x, const uint32_t* y) {   // c ? x : y, limbwise
  fp r;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.l[i] = (int32_t)(c ? x[i] : y[i]);
  return r;
}
// coefficient k of the Frobenius map n (0..3) of a lane's half, then a
// conjugation (bit 2): pr_frob2 / pr_frob_odd / pr_conj one coefficient at a
// time (the same multiplies by the same constants, so the same limbs)
template <int K>
PV_HD p2 fx_pre_c(const p2& x, uint32_t pre) {
  const uint32_t n = pre & 3u;
  p2 r = x;
  if (n == 2) {
#pragma unroll
    for (int j = 0; j < PL; ++j) {
      const fp g = fx_cst_sel(prole(j), FX_GP[1][2 * K + 1][0], FX_GP[1][2 * K][0]);
      r.e[j] = f2mulfp(x.e[j], g);
    }
  } else if (n != 0) {
    const bool one = n == 1;
#pragma unroll
    for (int j = 0; j < PL; ++j) {
      const int e = 2 * K + prole(j);
      // (e is role-dependent: both roles' constants as immediates, then selects)
      const fp2 g1{fx_cst_sel(one, FX_GP[0][2 * K + 1][0], FX_GP[2][2 * K + 1][0]),
                   fx_cst_sel(one, FX_GP[0][2 * K + 1][1], FX_GP[2][2 * K + 1][1])};
      const fp2 g0{fx_cst_sel(one, FX_GP[0][2 * K][0], FX_GP[2][2 * K][0]),
                   fx_cst_sel(one, FX_GP[0][2 * K][1], FX_GP[2][2 * K][1])};
      (void)e;
      r.e[j] = f2mul(f2conj(x.e[j]), f2pick(prole(j), g1, g0));
    }
  }
  if (pre & FX_CONJ) {
#pragma unroll
    for (int j = 0; j < PL; ++j) r.e[j] = f2pick(prole(j), f2neg(r.e[j]), r.e[j]);
  }
  return r;
}
PV_HD int fx_slot(uint32_t a) { return a < (uint32_t)FX_SLOTS ? (int)a : 0; }
// The parked halves: fx_park[3 * slot + k] holds coefficient k of each lane's
// half (PL of them on the host).  The slot index is wave-uniform (it comes from
// FX_PROG): made scalar, every access is a scalar base + constant offset, and no
// per-slot copy of the operand code is generated.
PV_HD uint32_t fx_uni(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_readfirstlane(x);
#else
  return x;
#endif
}
PV_HD p2 fx_park_c(const p2 (&park)[3 * FX_SLOTS], uint32_t x, int k) { return park[3 * fx_uni(fx_slot(x)) + k]; }
PV_HD void fx_park_st(p2 (&park)[3 * FX_SLOTS], uint32_t x, const p6& v) {
  const uint32_t u = fx_uni(x);
  if (u >= (uint32_t)FX_SLOTS) return;
#pragma unroll
  for (int k = 0; k < 3; ++k) park[3 * u + k] = p6c(v, k);
}


// x y with x (both halves) in the slot S and y the lanes' halves in registers:
// pr_mul's products and sums.  Role 0 forms t0 = x.a y.a, role 1 t1 = x.b y.b
// (f6mul_i's products on the lane's own half of x, read from the slot when each
// product starts, folded into three lazy sums as f6mul_fold does); the third
// product's Fp2 products m (role 0 X_k Y_k, role 1 the Karatsuba sums) from X =
// x.a + x.b (both halves from the slot) and Y = y + y' (the partner's half of y
// crossing one Fp2 at a time).  Then pr_mul_tail's sums, with the partner's m
// and t crossing one Fp2 at a time.
template <int ST>
PV_HD void pr_mul_s(pslot<ST> S, const p6& y, bool conj) {
  p2 m[3];
  {
#if PV_FX_YHOLD
    p2 Y[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const p2 yk = p6c(y, k), yo = pswap(yk);
#pragma unroll
      for (int j = 0; j < PL; ++j) Y[k].e[j] = f2add(yk.e[j], yo.e[j]);
    }
    mp_fence();
    auto Yk = [&](int k, int j) -> fp2 { return Y[k].e[j]; };
#else
    // Y_k = y_k + y'_k formed where each product needs it (the partner's Fp2
    // crossing again): no three Y's held through the m products
    auto Yk = [&](int k, int j) -> fp2 {
      const p2 yk = p6c(y, k), yo = pswap(yk);
      return f2add(yk.e[j], yo.e[j]);
    };
#endif
    // (a, b) of role 1's Karatsuba factor of m_k; role 0 takes X_k Y_k
    constexpr int KA[3] = {1, 0, 0}, KB[3] = {2, 1, 2};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
#pragma unroll
      for (int j = 0; j < PL; ++j) {
        const int h = prole(j);
        const fp2 Xa = f2add(S.ld(KA[k]), S.ld(3 + KA[k])), Xb = f2add(S.ld(KB[k]), S.ld(3 + KB[k]));
        const fp2 Xk = f2add(S.ld(k), S.ld(3 + k));
        m[k].e[j] = pin(f2mul(f2pick(h, f2addL(Xa, Xb), Xk), f2pick(h, f2add(Yk(KA[k], j), Yk(KB[k], j)), Yk(k, j))));
      }
      mp_fence();
    }
  }
  p6 t;
#pragma unroll
  for (int j = 0; j < PL; ++j) {
    const int X = 3 * prole(j);
    const fp6& b = y.e[j];
    fp2 c0, c1, c2;
    {
      const fp2 v0 = pin(f2mul(S.ld(X), b.c0));
      c0 = v0;
      c1 = f2negL(v0);
      c2 = f2negL(v0);
    }
    mp_fence();
    {
      const fp2 v1 = pin(f2mul(S.ld(X + 1), b.c1));
      c0 = f2subL(c0, f2mulxiL(v1));
      c1 = f2subL(c1, v1);
      c2 = f2addL(c2, v1);
    }
    mp_fence();
    {
      const fp2 v2 = pin(f2mul(S.ld(X + 2), b.c2));
      const fp2 xv2 = f2mulxiL(v2);
      c0 = f2subL(c0, xv2);
      c1 = f2addL(c1, xv2);
      c2 = f2subL(c2, v2);
    }
    mp_fence();
    c0 = f2addL(c0, f2mulxiL(pin(f2mul(f2addL(S.ld(X + 1), S.ld(X + 2)), f2add(b.c1, b.c2)))));
    mp_fence();
    c1 = f2addL(c1, pin(f2mul(f2addL(S.ld(X), S.ld(X + 1)), f2add(b.c0, b.c1))));
    mp_fence();
    c2 = f2addL(c2, pin(f2mul(f2addL(S.ld(X), S.ld(X + 2)), f2add(b.c0, b.c2))));
    t.e[j] = fp6{f2norm(c0), f2norm(c1), f2norm(c2)};
  }
  mp_fence();
  // pr_mul_tail: role 0 writes t0 + v t1, role 1 s - t0 - t1 (s from the m's)
  p2 sc[3];
  {
    const p2 mo[3] = {pswap(m[0]), pswap(m[1]), pswap(m[2])};
#pragma unroll
    for (int j = 0; j < PL; ++j) {
      const fp2 &v0 = mo[0].e[j], &v1 = mo[1].e[j], &v2 = mo[2].e[j];
      const fp2 &s12 = m[0].e[j], &s01 = m[1].e[j], &s02 = m[2].e[j];
      sc[0].e[j] = f2norm(f2addL(f2mulxiL(f2subL(f2subL(s12, v1), v2)), v0));
      sc[1].e[j] = f2norm(f2addL(f2subL(f2subL(s01, v0), v1), f2mulxiL(v2)));
      sc[2].e[j] = f2norm(f2addL(f2subL(f2subL(s02, v0), v2), v1));
    }
  }
  // every read of x is done: the result overwrites it, each lane its own half
  mp_fence();
  // role 0: ra_k = t0_k + (xi t1_2 | t1_0 | t1_1); role 1: rb_k = sc_k - t0_k - t1_k
  constexpr int RT[3] = {2, 0, 1};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const p2 tk = p6c(t, k), tko = pswap(tk);
    const p2 tr = p6c(t, RT[k]), tro = pswap(tr);
#pragma unroll
    for (int j = 0; j < PL; ++j) {
      const int h = prole(j);
      // (value selects: a select of references puts both operands in memory)
      const fp2 t0k = f2pick(h, tko.e[j], tk.e[j]);
      const fp2 t1k = f2pick(h, tk.e[j], tko.e[j]);
      const fp2 rb = f2norm(f2subL(f2subL(sc[k].e[j], t0k), t1k));
      const fp2 t1r = tro.e[j];   // role 0's partner (role 1) t1 at RT[k]
      const fp2 ra = f2norm(f2addL(tk.e[j], k == 0 ? f2mulxiL(t1r) : t1r));
      fp2 v = f2pick(h, rb, ra);
      if (conj) v = f2pick(h, f2neg(v), v);   // pr_conj: role 1's half negated
      S.st(3 * h + k, v);
    }
  }
  mp_fence();
}

// 1 / x with both Fp6 products inlined (the step program's one copy)
PV_HD p6 pr_inv_i(const p6& x) {
  p6 sq;
#pragma unroll
  for (int j = 0; j < PL; ++j) sq.e[j] = f6mul_fold(x.e[j], x.e[j]);
  const p6 so = pswap(sq);
  p6 r;
#pragma unroll
  for (int j = 0; j < PL; ++j) {
    const int h = prole(j);
    const fp6 d = f6inv(f6sub(f6sel(h, so.e[j], sq.e[j]), f6mulv(f6sel(h, sq.e[j], so.e[j]))));
    const fp6 m = f6mul_fold(x.e[j], d);
    r.e[j] = f6sel(h, f6neg(m), m);
  }
  return r;
}

// The accumulator lives in the check's LDS slot (each lane its own half), never
// in registers across steps.  Operand X into the slot with its pre-map, one Fp2
// at a time: a parked half copied in, or acc mapped in place.
template <int ST, int K>
PV_HD void fx_put_c(pslot<ST> S, const p2 (&park)[3 * FX_SLOTS], uint32_t x, uint32_t pre) {
  p2 c;
  if (x == FX_ACC) {
#pragma unroll
    for (int j = 0; j < PL; ++j) c.e[j] = S.ld(3 * prole(j) + K);
  } else {
    c = fx_park_c(park, x, K);
  }
  c = fx_pre_c<K>(c, pre);
#pragma unroll
  for (int j = 0; j < PL; ++j) S.st(3 * prole(j) + K, c.e[j]);
  mp_fence();
}
template <int ST>
PV_HD void fx_put(pslot<ST> S, const p2 (&park)[3 * FX_SLOTS], uint32_t x, uint32_t pre) {
  if (x == FX_ACC && pre == 0) return;
  fx_put_c<ST, 0>(S, park, x, pre);
  fx_put_c<ST, 1>(S, park, x, pre);
  fx_put_c<ST, 2>(S, park, x, pre);
}
// operand X with its pre-map in registers (acc read from the slot)
template <int ST, int K>
PV_HD p2 fx_get_c(pslot<ST> S, const p2 (&park)[3 * FX_SLOTS], uint32_t x, uint32_t pre) {
  p2 c;
  if (x == FX_ACC) {
#pragma unroll
    for (int j = 0; j < PL; ++j) c.e[j] = S.ld(3 * prole(j) + K);
  } else {
    c = fx_park_c(park, x, K);
  }
  return fx_pre_c<K>(c, pre);
}
template <int ST>
PV_HD p6 fx_get(pslot<ST> S, const p2 (&park)[3 * FX_SLOTS], uint32_t x, uint32_t pre) {
  const p2 c0 = fx_get_c<ST, 0>(S, park, x, pre), c1 = fx_get_c<ST, 1>(S, park, x, pre),
           c2 = fx_get_c<ST, 2>(S, park, x, pre);
  p6 r;
#pragma unroll
  for (int j = 0; j < PL; ++j) r.e[j] = fp6{c0.e[j], c1.e[j], c2.e[j]};
  mp_fence();
  return r;
}

// final_exp(f0) on halves as FX_PROG: one loop, one copy of each operation.
// Inlined into the pair kernel (one call site): as a call it saved and restored
// the callee-saved VGPRs it uses on every check.
#ifndef PV_FX_CALL
#define PV_FX_CALL PV_HD
#endif
template <int ST>
PV_FX_CALL p6 pr_final_exp_fx(pslot<ST> S, const p6& f0) {
  p2 park[3 * FX_SLOTS];
  fx_park_st(park, 0, f0);
  mp_put(S, f0);
#if defined(__HIP_DEVICE_COMPILE__)
  // the program's words, word s in lane s of one VGPR (a lane-indexed vector
  // load), read back with v_readlane: no scalar-cache load of the table
  static_assert(FX_STEPS <= 64, "one word per lane");
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t progv = FX_PROG_DEV[lane < (uint32_t)FX_STEPS ? lane : 0u];
#endif
#pragma unroll 1
  for (int s = 0; s < FX_STEPS; ++s) {
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t w = (uint32_t)__builtin_amdgcn_readlane((int)progv, s);
#else
    const uint32_t w = FX_PROG[s];
#endif
    const uint32_t op = w & 15u, a = (w >> 4) & 15u, b = (w >> 12) & 255u;
    const bool post = (w >> 24) & 1u;
    if (op == FX_MUL) {
      // B first: it may be the accumulator the slot is about to receive A over
      const p6 B = fx_get(S, park, b, (w >> 20) & 15u);
      fx_put(S, park, a, (w >> 8) & 15u);
      pr_mul_s(S, B, post);
    } else {
      if (op == FX_INV) {
        static_assert(FX_PROG[0] == fx(FX_INV, FX_ACC, 0, 0, 0, 0, FX_NONE), "the inverse takes acc, unmapped");
        mp_put(S, pr_inv_i(mp_get(S)));
      } else {
        fx_put(S, park, a, (w >> 8) & 15u);
#pragma unroll 1
        for (uint32_t i = 0; i < b; ++i) {
          mp_cyc_sqr(S);
          if ((i & 3) == 3) mp_reduce(S);
        }
      }
      if (post) mp_put(S, pr_conj(mp_get(S)));
    }
    const uint32_t pk = w >> 28;
    if (pk < (uint32_t)FX_SLOTS) fx_park_st(park, pk, mp_get(S));   // (pk: an SGPR; uniform branch)
  }
  return mp_get(S);
}

// final_exp's chain on halves
template <int ST, int LV = 0>
PV_BN_CALL p6 pr_final_exp_chain(pslot<ST> S, const p6& f0) {
  p6 f = pmul<LV>(pr_conj(f0), pinv<LV>(f0));   // ^(p^6 - 1)
  f = pmul<LV>(pr_frob2(f), f);              // ^(p^2 + 1)
  const p6 fu = pr_pow_u<ST, LV>(S, f);
  const p6 fu2 = pr_pow_u<ST, LV>(S, fu);
  const p6 fu3 = pr_pow_u<ST, LV>(S, fu2);
  const p6 y6 = pr_conj(pmul<LV>(fu3, pr_frob1(fu3)));
  p6 t0 = pr_cyc_sqr<ST, LV>(S, y6);
  t0 = pmul<LV>(t0, pr_conj(pmul<LV>(fu, pr_frob1(fu2))));   // y4
  const p6 y5 = pr_conj(fu2);
  t0 = pmul<LV>(t0, y5);
  p6 t1 = pmul<LV>(pmul<LV>(pr_conj(pr_frob1(fu)), y5), t0);
  t0 = pmul<LV>(t0, pr_frob2(fu2));
  t1 = pmul<LV>(pr_cyc_sqr<ST, LV>(S, t1), t0);
  t1 = pr_cyc_sqr<ST, LV>(S, t1);
  t0 = pmul<LV>(t1, pr_conj(f));
  const p6 y0 = pmul<LV>(pmul<LV>(pr_frob1(f), pr_frob2(f)), pr_frob3(f));
  t1 = pmul<LV>(t1, y0);
  return pmul<LV>(pr_cyc_sqr<ST, LV>(S, t0), t1);
}
// the pair kernel (LV 0) runs the step program, the quad / octet the chain
template <int ST, int LV = 0>
PV_HD p6 pr_final_exp(pslot<ST> S, const p6& f0) {
  if constexpr (LV == 0 && PV_FE_PROG) return pr_final_exp_fx<ST>(S, f0);
  return pr_final_exp_chain<ST, LV>(S, f0);
}

#if defined(__HIPCC__)
// this lane's check slot (lanes 2c and 2c + 1 share check c of the block)
__device__ __forceinline__ pslot<MP_CHECKS> mp_slot() {
#if defined(__HIP_DEVICE_COMPILE__)
  return pslot<MP_CHECKS>{threadIdx.x >> 1};
#else
  return pslot<MP_CHECKS>{nullptr};
#endif
}
#endif

// the two-pairing Miller product into the slot (miller2's steps); returns f's halves
// (q: the lane's coordinate of each G1 point, x/y for role 0 and 1/y for role 1).
// Inlined into the kernel (one call site): as an out-of-line function its
// wave-uniform arguments (the line pointers) lived in VGPRs and went through
// scratch at every step.
// QUAD (the small-batch kernel, one check over four lanes): each lane pair runs
// ONE pairing's Miller loop -- pair 0 over the generator's lines with sigma's
// point, pair 1 over the key's lines with -H's -- with its point in q[0]; on the
// host the caller passes that pairing's lines as g_lines.
// OCT (k_bls_verify_oct, one check over eight lanes): QUAD's schedule with each
// step's Fp2 products split between the octet's two quads (mp_sqr / mp_line's
// OCT forms), both quads on the same slot.
template <int ST, bool QUAD = false, bool OCT = false>
PV_HD p6 miller_pair(pslot<ST> S, const uint32_t* g_lines, const uint32_t* pk_lines, const p1 (&q)[2]) {
#pragma unroll
  for (int j = 0; j < PL; ++j) S.st6(prole(j), prole(j) ? f6zero() : f6one());
  mp_fence();
#if defined(__HIP_DEVICE_COMPILE__)
  // the step's two lines staged per wave in LDS (one key per wave), one step ahead
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
  uint32_t pg = 0, pp = 0;
  auto fetch = [&](int kk) {
    if (ln < LINE_WORDS && kk < N_LINES) {
      pg = g_lines[LINE_WORDS * kk + ln];
      pp = pk_lines[LINE_WORDS * kk + ln];
    }
  };
  auto stash = [&](int kk) {
    if (ln < LINE_WORDS && kk < N_LINES) {
      mf_lines[wv][kk & 1][0][ln] = pg;
      mf_lines[wv][kk & 1][1][ln] = pp;
    }
    mp_fence();
    __builtin_amdgcn_wave_barrier();
  };
  const int own = QUAD ? (int)((threadIdx.x >> 1) & 1) : 0;   // the pair's pairing (QUAD)
  auto Lg = [&](int kk) -> const uint32_t* { return mf_lines[wv][kk & 1][own]; };
  auto Lp = [&](int kk) -> const uint32_t* { return mf_lines[wv][kk & 1][1]; };
  fetch(0);
  stash(0);
#else
  auto fetch = [](int) {};
  auto stash = [](int) {};
  auto Lg = [&](int kk) -> const uint32_t* { return g_lines + LINE_WORDS * kk; };
  auto Lp = [&](int kk) -> const uint32_t* { return pk_lines + LINE_WORDS * kk; };
#endif
  int k = 0;
  for (int i = 63; i >= 0; --i) {
    for (int add = 0; add < 2; ++add) {
      if (add && !ate_bit(i)) break;
      fetch(k + 1);
      if (!add && i != 63) mp_sqr<ST, OCT>(S);
      mp_line<ST, OCT>(S, Lg(k), q[0]);
      if (!QUAD) mp_line(S, Lp(k), q[1]);
      stash(k + 1);
      ++k;
    }
  }
  mp_put(S, pr_conj(mp_get(S)));
  for (int j = 0; j < 2; ++j, ++k) {
    fetch(k + 1);
    mp_line<ST, OCT>(S, Lg(k), q[0]);
    if (!QUAD) mp_line(S, Lp(k), q[1]);
    stash(k + 1);
  }
  return mp_get(S);
}

// the check over the pair from each lane's coordinates of sigma's and -H(m)'s
// line points (q[0], q[1]; a point at infinity as 0); both lanes return the verdict
template <int ST>
PV_HD bool bls_check_pair_q(pslot<ST> S, const p1 (&q)[2], bool s_inf, bool pk_inf, const uint32_t* g_lines,
                            const uint32_t* pk_lines) {
  const bool one = pr_is_one(pr_final_exp(S, miller_pair(S, g_lines, pk_lines, q)));
  if (s_inf || pk_inf) return s_inf && pk_inf;
  return one;
}
#if defined(__HIPCC__)
// the check over a lane QUAD (small batches): the two pairs' Miller values are
// multiplied (each pair forms the same product) and both run the final
// exponentiation in lockstep; q[0] = the pair's own point coordinate
__device__ __forceinline__ bool bls_check_quad_q(pslot<MP_CHECKS> S, const p1 (&q)[2], bool s_inf, bool pk_inf,
                                                 const uint32_t* g_lines, const uint32_t* pk_lines) {
#if defined(__HIP_DEVICE_COMPILE__)
  const p6 f = miller_pair<MP_CHECKS, true>(S, g_lines, pk_lines, q);
  // both pairs multiply sigma's value (pair 0's) by -H's (pair 1's) in that order,
  // so that both hold the same limbs from here on
  const p6 o = pqswap(f);
  const bool g = qrole();
  const p6 fs = g ? o : f, fh = g ? f : o;
  const pslot<MP_CHECKS> Sq{S.c & ~1u};   // the even pair's slot, shared by the quad
  const bool one = pr_is_one(pr_final_exp<MP_CHECKS, 1>(Sq, pr_mul_q(fs, fh)));
  if (s_inf || pk_inf) return s_inf && pk_inf;
  return one;
#else
  return false;
#endif
}
#endif
#if defined(__HIPCC__)
// the check over a lane OCTET (k_bls_verify_oct, the smallest calls): the quad
// schedule with every step's products split between the octet's quads; the
// Miller slots are per (check, pairing), shared by the two quads
__device__ __forceinline__ bool bls_check_oct_q(const p1 (&q)[2], bool s_inf, bool pk_inf, const uint32_t* g_lines,
                                                const uint32_t* pk_lines) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t col = ((threadIdx.x >> 3) << 1) | ((threadIdx.x >> 1) & 1u);
  const p6 f = miller_pair<MP_CHECKS, true, true>(pslot<MP_CHECKS>{col}, g_lines, pk_lines, q);
  const p6 o = pqswap(f);
  const bool m = qrole();
  const p6 fs = m ? o : f, fh = m ? f : o;
  const pslot<MP_CHECKS> Sq{col & ~1u};   // the octet's shared slot
  const bool one = pr_is_one(pr_final_exp<MP_CHECKS, 2>(Sq, pr_mul_o(fs, fh)));
  if (s_inf || pk_inf) return s_inf && pk_inf;
  return one;
#else
  return false;
#endif
}
#endif
// bls_check's arguments (host checker)
template <int ST>
PV_HD bool bls_check_pair(pslot<ST> S, const fp& xs, const fp& ys, bool s_inf, const fp& xqh, const fp& yqh,
                          bool pk_inf, const uint32_t* g_lines, const uint32_t* pk_lines) {
  fp xq = fzero(), yq = fzero();
  if (!s_inf) line_point(xs, ys, false, xq, yq);
  p1 q[2];
#pragma unroll
  for (int j = 0; j < PL; ++j) {
    q[0].e[j] = fsel(prole(j), yq, xq);
    q[1].e[j] = fsel(prole(j), yqh, xqh);
  }
  return bls_check_pair_q(S, q, s_inf, pk_inf, g_lines, pk_lines);
}

}  // namespace bn
