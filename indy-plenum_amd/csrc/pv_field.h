// GF(2^255 - 19) arithmetic for the batch verifier, one field element per lane.
//
// Representation: 10 unsigned 32-bit limbs in radix 2^25.5 (limb i has weight
// 2^ceil(25.5 i): 0,26,51,77,102,128,153,179,204,230).  Products are formed
// with v_mad_u64_u32 (32x32 -> 64-bit multiply-accumulate), which measures
// ~45 lane-ops/clk/CU on gfx950 (profiles/r01_int_rates.json) and is the
// instruction the roofline is priced in.  MFMA is not used: this is modular
// 255-bit arithmetic, not a dense contraction.
//
// Bound discipline (checked on every multiply by the host bound-checking
// build, tests/test_hostcheck.py):
//   TIGHT  : even limbs <= 2^26 + 2^10, odd limbs <= 2^25 + 2^18   (mul/sq output)
//   LOOSE  : even limbs <= 2^27.7,      odd limbs <= 2^26.7        (safe for any mul/sq)
//   tight+tight, tight+tight+tight and tight + 2p - tight are LOOSE.
//   fe_mul(h, f, g) also accepts f up to ~2^28.3 (even) when g is LOOSE: the
//   exact limits are 2f < 2^32, 19g < 2^32 and column sums < 2^64.
//
// Restates the field layer libsodium 1.0.18 uses under crypto_sign_open
// (SURVEY.md Appendix C); the verdict only depends on exact field results, so
// any exact representation is parity-equivalent.
#pragma once
#include <stdint.h>
#include "pv_madchains.h"

#ifndef PV_HD
#define PV_HD __host__ __device__ __forceinline__
#endif
#ifndef PV_COUNT
#define PV_COUNT(kind)
#endif
// Host bound-checking hooks (tools/hostcheck): the exact conditions for a
// multiply to be exact are 2 f_i < 2^32, 19 g_j < 2^32 and every 64-bit
// column sum < 2^64 (checked on the actual operands).
#ifndef PV_CHECK_MUL
#define PV_CHECK_MUL(f, g)
#endif
#ifndef PV_CHECK_SQ
#define PV_CHECK_SQ(f)
#endif
#ifndef PV_CHECK_SQ2X
#define PV_CHECK_SQ2X(f)
#endif
// Optional scheduling fence after every field multiply (-DPV_FE_FENCE_ON):
// keeps the scheduler from interleaving consecutive multiplies.  Off by
// default since the column-asm multiply (below): with each column one asm
// block the interleaving is limited anyway, and the fence-free build measured
// equal on C2 and 1-3 % faster on the keyed C3 curve
// (profiles/r02_ab_colasm_c2.json, r02_ab_colasm_c3.json).
#ifndef PV_FE_FENCE
#if defined(__HIP_DEVICE_COMPILE__) && defined(PV_FE_FENCE_ON)
#define PV_FE_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define PV_FE_FENCE()
#endif
#endif

namespace pv {

static constexpr uint32_t M26 = (1u << 26) - 1;
static constexpr uint32_t M25 = (1u << 25) - 1;

struct fe {
  uint32_t v[10];
};

PV_HD uint64_t mul32x32(uint32_t a, uint32_t b) { return (uint64_t)a * (uint64_t)b; }

// 2x of a limb.  -DPV_TWICE_ADD forces v_add_u32 (asm) instead of the
// compiler's v_lshlrev_b32: the isolated issue rates suggest it should be
// cheaper (profiles/r01_int_cycles.json), but the doubling chain measured 2 %
// slower with it (profiles/r02_fe_ilp_twice.txt), so the default is the shift.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(PV_FE_NOASM) && defined(PV_TWICE_ADD)
__device__ __forceinline__ uint32_t twice(uint32_t x) {
  uint32_t y;
  asm("v_add_u32 %0, %1, %1" : "=v"(y) : "v"(x));
  return y;
}
#else
PV_HD uint32_t twice(uint32_t x) { return 2u * x; }
#endif

// Column sums as v_mad_u64_u32 chains whose first addend is the incoming
// carry.  As plain C++ the compiler reassociates every column (starts it from
// 0 and adds the carry with a trailing v_lshl_add_u64: one extra half-rate
// 64-bit op per column, 10 per multiply).  A whole column is ONE asm block:
// an asm statement cannot be reassociated, and the gfx950 hazard recognizer,
// which assumes an inline-asm result feeding another inline asm needs a wait
// state (dst-sel forwarding), then sees one asm block per column instead of
// one per product (a per-product asm statement cost an s_nop 0 per MAD).
// Dependent v_mad_u64_u32 need no wait states between them (the compiler's
// own chains are back to back).  Host builds (tools/hostcheck) and
// -DPV_FE_NOASM use the plain expressions: the same sums.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(PV_FE_NOASM)
#define PV_ASM_FN __device__ __forceinline__
PV_ASM_FN uint64_t mad10(uint64_t c, uint32_t a0, uint32_t b0, uint32_t a1, uint32_t b1, uint32_t a2, uint32_t b2, uint32_t a3, uint32_t b3, uint32_t a4, uint32_t b4, uint32_t a5, uint32_t b5, uint32_t a6, uint32_t b6, uint32_t a7, uint32_t b7, uint32_t a8, uint32_t b8, uint32_t a9, uint32_t b9) {
  uint64_t d;
  asm("v_mad_u64_u32 %0, vcc, %1, %2, %0\n"
      "v_mad_u64_u32 %0, vcc, %3, %4, %0\n"
      "v_mad_u64_u32 %0, vcc, %5, %6, %0\n"
      "v_mad_u64_u32 %0, vcc, %7, %8, %0\n"
      "v_mad_u64_u32 %0, vcc, %9, %10, %0\n"
      "v_mad_u64_u32 %0, vcc, %11, %12, %0\n"
      "v_mad_u64_u32 %0, vcc, %13, %14, %0\n"
      "v_mad_u64_u32 %0, vcc, %15, %16, %0\n"
      "v_mad_u64_u32 %0, vcc, %17, %18, %0\n"
      "v_mad_u64_u32 %0, vcc, %19, %20, %0\n"
      : "=v"(d)
      : "v"(a0), "v"(b0), "v"(a1), "v"(b1), "v"(a2), "v"(b2), "v"(a3), "v"(b3), "v"(a4), "v"(b4), "v"(a5), "v"(b5), "v"(a6), "v"(b6), "v"(a7), "v"(b7), "v"(a8), "v"(b8), "v"(a9), "v"(b9), "0"(c)
      : "vcc");
  return d;
}
PV_ASM_FN uint64_t mad10z(uint32_t a0, uint32_t b0, uint32_t a1, uint32_t b1, uint32_t a2, uint32_t b2, uint32_t a3, uint32_t b3, uint32_t a4, uint32_t b4, uint32_t a5, uint32_t b5, uint32_t a6, uint32_t b6, uint32_t a7, uint32_t b7, uint32_t a8, uint32_t b8, uint32_t a9, uint32_t b9) {
  uint64_t d;
  asm("v_mad_u64_u32 %0, vcc, %1, %2, 0\n"
      "v_mad_u64_u32 %0, vcc, %3, %4, %0\n"
      "v_mad_u64_u32 %0, vcc, %5, %6, %0\n"
      "v_mad_u64_u32 %0, vcc, %7, %8, %0\n"
      "v_mad_u64_u32 %0, vcc, %9, %10, %0\n"
      "v_mad_u64_u32 %0, vcc, %11, %12, %0\n"
      "v_mad_u64_u32 %0, vcc, %13, %14, %0\n"
      "v_mad_u64_u32 %0, vcc, %15, %16, %0\n"
      "v_mad_u64_u32 %0, vcc, %17, %18, %0\n"
      "v_mad_u64_u32 %0, vcc, %19, %20, %0\n"
      : "=&v"(d)
      : "v"(a0), "v"(b0), "v"(a1), "v"(b1), "v"(a2), "v"(b2), "v"(a3), "v"(b3), "v"(a4), "v"(b4), "v"(a5), "v"(b5), "v"(a6), "v"(b6), "v"(a7), "v"(b7), "v"(a8), "v"(b8), "v"(a9), "v"(b9)
      : "vcc");
  return d;
}
PV_ASM_FN uint64_t mad6(uint64_t c, uint32_t a0, uint32_t b0, uint32_t a1, uint32_t b1, uint32_t a2, uint32_t b2, uint32_t a3, uint32_t b3, uint32_t a4, uint32_t b4, uint32_t a5, uint32_t b5) {
  uint64_t d;
  asm("v_mad_u64_u32 %0, vcc, %1, %2, %0\n"
      "v_mad_u64_u32 %0, vcc, %3, %4, %0\n"
      "v_mad_u64_u32 %0, vcc, %5, %6, %0\n"
      "v_mad_u64_u32 %0, vcc, %7, %8, %0\n"
      "v_mad_u64_u32 %0, vcc, %9, %10, %0\n"
      "v_mad_u64_u32 %0, vcc, %11, %12, %0\n"
      : "=v"(d)
      : "v"(a0), "v"(b0), "v"(a1), "v"(b1), "v"(a2), "v"(b2), "v"(a3), "v"(b3), "v"(a4), "v"(b4), "v"(a5), "v"(b5), "0"(c)
      : "vcc");
  return d;
}
PV_ASM_FN uint64_t mad6z(uint32_t a0, uint32_t b0, uint32_t a1, uint32_t b1, uint32_t a2, uint32_t b2, uint32_t a3, uint32_t b3, uint32_t a4, uint32_t b4, uint32_t a5, uint32_t b5) {
  uint64_t d;
  asm("v_mad_u64_u32 %0, vcc, %1, %2, 0\n"
      "v_mad_u64_u32 %0, vcc, %3, %4, %0\n"
      "v_mad_u64_u32 %0, vcc, %5, %6, %0\n"
      "v_mad_u64_u32 %0, vcc, %7, %8, %0\n"
      "v_mad_u64_u32 %0, vcc, %9, %10, %0\n"
      "v_mad_u64_u32 %0, vcc, %11, %12, %0\n"
      : "=&v"(d)
      : "v"(a0), "v"(b0), "v"(a1), "v"(b1), "v"(a2), "v"(b2), "v"(a3), "v"(b3), "v"(a4), "v"(b4), "v"(a5), "v"(b5)
      : "vcc");
  return d;
}
PV_ASM_FN uint64_t mad5(uint64_t c, uint32_t a0, uint32_t b0, uint32_t a1, uint32_t b1, uint32_t a2, uint32_t b2, uint32_t a3, uint32_t b3, uint32_t a4, uint32_t b4) {
  uint64_t d;
  asm("v_mad_u64_u32 %0, vcc, %1, %2, %0\n"
      "v_mad_u64_u32 %0, vcc, %3, %4, %0\n"
      "v_mad_u64_u32 %0, vcc, %5, %6, %0\n"
      "v_mad_u64_u32 %0, vcc, %7, %8, %0\n"
      "v_mad_u64_u32 %0, vcc, %9, %10, %0\n"
      : "=v"(d)
      : "v"(a0), "v"(b0), "v"(a1), "v"(b1), "v"(a2), "v"(b2), "v"(a3), "v"(b3), "v"(a4), "v"(b4), "0"(c)
      : "vcc");
  return d;
}
PV_ASM_FN uint64_t mad5z(uint32_t a0, uint32_t b0, uint32_t a1, uint32_t b1, uint32_t a2, uint32_t b2, uint32_t a3, uint32_t b3, uint32_t a4, uint32_t b4) {
  uint64_t d;
  asm("v_mad_u64_u32 %0, vcc, %1, %2, 0\n"
      "v_mad_u64_u32 %0, vcc, %3, %4, %0\n"
      "v_mad_u64_u32 %0, vcc, %5, %6, %0\n"
      "v_mad_u64_u32 %0, vcc, %7, %8, %0\n"
      "v_mad_u64_u32 %0, vcc, %9, %10, %0\n"
      : "=&v"(d)
      : "v"(a0), "v"(b0), "v"(a1), "v"(b1), "v"(a2), "v"(b2), "v"(a3), "v"(b3), "v"(a4), "v"(b4)
      : "vcc");
  return d;
}
#undef PV_ASM_FN
#else
#define PV_MADN_PLAIN 1
#endif

// column of n products a[0]b[0] + ... + a[n-1]b[n-1] (+ carry unless first)
template <int N>
PV_HD uint64_t column(const uint32_t a[N], const uint32_t b[N], uint64_t carry, bool first) {
#if defined(PV_MADN_PLAIN)
  uint64_t acc = first ? 0 : carry;
#pragma unroll
  for (int i = 0; i < N; ++i) acc += mul32x32(a[i], b[i]);
  return acc;
#else
  if constexpr (N == 10) {
    if (first) return mad10z(a[0], b[0], a[1], b[1], a[2], b[2], a[3], b[3], a[4], b[4], a[5], b[5], a[6], b[6], a[7],
                             b[7], a[8], b[8], a[9], b[9]);
    return mad10(carry, a[0], b[0], a[1], b[1], a[2], b[2], a[3], b[3], a[4], b[4], a[5], b[5], a[6], b[6], a[7], b[7],
                 a[8], b[8], a[9], b[9]);
  } else if constexpr (N == 6) {
    if (first) return mad6z(a[0], b[0], a[1], b[1], a[2], b[2], a[3], b[3], a[4], b[4], a[5], b[5]);
    return mad6(carry, a[0], b[0], a[1], b[1], a[2], b[2], a[3], b[3], a[4], b[4], a[5], b[5]);
  } else {
    static_assert(N == 5, "column widths of fe_mul / fe_sq");
    if (first) return mad5z(a[0], b[0], a[1], b[1], a[2], b[2], a[3], b[3], a[4], b[4]);
    return mad5(carry, a[0], b[0], a[1], b[1], a[2], b[2], a[3], b[3], a[4], b[4]);
  }
#endif
}

PV_HD void fe_0(fe& h) {
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = 0;
}
PV_HD void fe_1(fe& h) {
  fe_0(h);
  h.v[0] = 1;
}
PV_HD void fe_copy(fe& h, const fe& f) {
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = f.v[i];
}

// 64-bit column sums -> TIGHT limbs.  Two interleaved carry chains (0..4 and
// 4..9) keep the dependency depth short; final wrap multiplies by 19 because
// 2^255 == 19 (mod p).
PV_HD void fe_carry_wide(fe& out, uint64_t h[10]) {
  uint64_t c;
  c = h[0] >> 26; h[1] += c; h[0] &= M26;
  c = h[4] >> 26; h[5] += c; h[4] &= M26;
  c = h[1] >> 25; h[2] += c; h[1] &= M25;
  c = h[5] >> 25; h[6] += c; h[5] &= M25;
  c = h[2] >> 26; h[3] += c; h[2] &= M26;
  c = h[6] >> 26; h[7] += c; h[6] &= M26;
  c = h[3] >> 25; h[4] += c; h[3] &= M25;
  c = h[7] >> 25; h[8] += c; h[7] &= M25;
  c = h[4] >> 26; h[5] += c; h[4] &= M26;
  c = h[8] >> 26; h[9] += c; h[8] &= M26;
  c = h[9] >> 25; h[0] += c * 19; h[9] &= M25;
  c = h[0] >> 26; h[1] += c; h[0] &= M26;
#pragma unroll
  for (int i = 0; i < 10; ++i) out.v[i] = (uint32_t)h[i];
}

// Columns are produced in order k = 0..9 and each column's accumulation
// STARTS from the previous column's carry, so the carry add rides inside a
// v_mad_u64_u32 addend instead of costing a separate 64-bit add; one wrap
// (x19) and one last carry into limb 1 finish the reduction.  Output TIGHT:
// even limbs < 2^26, odd < 2^25 + 2^17.  (tools/ubench/fe_bench.hip measured
// this +3-5 % over interleaved ref10-order carries on gfx950.)
PV_HD void fe_finish_columns(fe& h, uint64_t carry_out_of_9, uint32_t out[10]) {
  const uint64_t t = (uint64_t)out[0] + carry_out_of_9 * 19u;
  out[0] = (uint32_t)t & M26;
  out[1] += (uint32_t)(t >> 26);
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = out[i];
}

// h = f * g.  Column k collects f_i g_j with i + j = k (weight doubles when i
// and j are both odd) and, wrapped, 19 f_i g_j with i + j = k + 10.
PV_HD void fe_mul(fe& h, const fe& f, const fe& g) {
  PV_COUNT(mul);
  PV_CHECK_MUL(f, g);
  uint32_t g19[10], f2[10];
#pragma unroll
  for (int j = 1; j < 10; ++j) g19[j] = 19u * g.v[j];
#pragma unroll
  for (int i = 1; i < 10; i += 2) f2[i] = twice(f.v[i]);
  uint64_t carry = 0;
  uint32_t out[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    uint32_t a[10], b[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      const int j = (k - i + 10) % 10;
      const bool oo = (i & 1) && (j & 1);
      a[i] = oo ? f2[i] : f.v[i];
      b[i] = i + j >= 10 ? g19[j] : g.v[j];
    }
    const uint64_t acc = column<10>(a, b, carry, k == 0);
    carry = acc >> ((k & 1) ? 25 : 26);
    out[k] = (uint32_t)acc & ((k & 1) ? M25 : M26);
  }
  fe_finish_columns(h, carry, out);
  PV_FE_FENCE();
}

// Squaring operands.  Product (i, j), i <= j, of MULT * f^2 carries the
// coefficient c = MULT * (i == j ? 1 : 2) * (i, j both odd ? 2 : 1) *
// (i + j >= 10 ? 19 : 1) and is formed as (m_i f_i)(m_j f_j) with m_i m_j = c
// from a set of PREPARED multiples, the smallest set that covers all 55
// products (exhaustive search, tools/sq_prep_search.py):
//   MULT 1: 13 values  2f_0..7, 19f_6, 19f_8, 38f_5, 38f_7, 38f_9
//           (against 20 for 2f_0..9, 19f_5..9, 4f_odd); odd limbs <= 2^26.75,
//           even <= 2^27.75 (LOOSE inputs qualify);
//   MULT 2: 16 values  2f_0..7, 4f_0, 4f_1, 4f_3, 38f_6, 38f_8, 76f_5, 76f_7,
//           76f_9 -- 2 f^2 in one squaring (ge_p2_dbl's 2Z^2) instead of a
//           squaring + 10 adds; TIGHT inputs only (76 f_odd < 2^32).
// The host build checks every operand and column bound.
template <int MULT>
constexpr bool sq_avail(int i, int m) {
  if (MULT == 1)
    return m == 1 || (m == 2 && i < 8) || (m == 19 && (i == 6 || i == 8)) || (m == 38 && (i == 5 || i == 7 || i == 9));
  return m == 1 || (m == 2 && i < 8) || (m == 4 && (i == 0 || i == 1 || i == 3)) || (m == 38 && (i == 6 || i == 8)) ||
         (m == 76 && (i == 5 || i == 7 || i == 9));
}
template <int MULT>
constexpr int sq_coef(int i, int j) {
  return MULT * (i == j ? 1 : 2) * ((i & 1) && (j & 1) ? 2 : 1) * (i + j >= 10 ? 19 : 1);
}
// the multiple of f_i (first) / f_j (second) used for product (i, j)
template <int MULT>
constexpr int sq_pick(int i, int j, bool second) {
  const int ms[6] = {1, 2, 4, 19, 38, 76};
  for (int a = 0; a < 6; ++a)
    for (int b = 0; b < 6; ++b)
      if (ms[a] * ms[b] == sq_coef<MULT>(i, j) && sq_avail<MULT>(i, ms[a]) && sq_avail<MULT>(j, ms[b]))
        return second ? ms[b] : ms[a];
  return 0;
}
template <int MULT>
constexpr bool sq_plan_ok() {
  for (int i = 0; i < 10; ++i)
    for (int j = i; j < 10; ++j)
      if (sq_pick<MULT>(i, j, false) * sq_pick<MULT>(i, j, true) != sq_coef<MULT>(i, j)) return false;
  return true;
}
static_assert(sq_plan_ok<1>() && sq_plan_ok<2>(), "every squaring product needs a prepared operand pair");
struct sq_ops {
  uint32_t f[10], f2[10], f4[10], f19[10], f38[10], f76[10];
};
PV_HD uint32_t sq_get(const sq_ops& o, int m, int i) {
  return m == 1 ? o.f[i] : m == 2 ? o.f2[i] : m == 4 ? o.f4[i] : m == 19 ? o.f19[i] : m == 38 ? o.f38[i] : o.f76[i];
}
// every multiple of every limb; the ones a plan does not read are dead code
PV_HD void sq_prepare(sq_ops& o, const fe& f) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    o.f[i] = f.v[i];
    o.f2[i] = twice(f.v[i]);
    o.f4[i] = twice(o.f2[i]);
    o.f19[i] = 19u * f.v[i];
    o.f38[i] = 38u * f.v[i];
    o.f76[i] = 76u * f.v[i];
  }
}
// column k of MULT f^2: (as, bs) with 6 products (k even) or 5 (k odd)
template <int MULT>
PV_HD void sq_column(const sq_ops& o, int k, uint32_t as[6], uint32_t bs[6]) {
  int t = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
#pragma unroll
    for (int j = i; j < 10; ++j) {
      if ((i + j) % 10 != k) continue;
      as[t] = sq_get(o, sq_pick<MULT>(i, j, false), i);
      bs[t] = sq_get(o, sq_pick<MULT>(i, j, true), j);
      ++t;
    }
  }
}

// h = MULT f^2 with the symmetric cross terms folded (55 products instead of 100).
template <int MULT>
PV_HD void fe_sq_t(fe& h, const fe& f) {
  sq_ops o;
  sq_prepare(o, f);
  uint64_t carry = 0;
  uint32_t out[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    uint32_t as[6], bs[6];
    sq_column<MULT>(o, k, as, bs);
    // column k has 6 products when k is even, 5 when odd
    const uint64_t acc = (k & 1) ? column<5>(as, bs, carry, false) : column<6>(as, bs, carry, k == 0);
    carry = acc >> ((k & 1) ? 25 : 26);
    out[k] = (uint32_t)acc & ((k & 1) ? M25 : M26);
  }
  fe_finish_columns(h, carry, out);
  PV_FE_FENCE();
}
PV_HD void fe_sq(fe& h, const fe& f) {
  PV_COUNT(sq);
  PV_CHECK_SQ(f);
  fe_sq_t<1>(h, f);
}
// h = 2 f^2 (f TIGHT)
PV_HD void fe_sq2x(fe& h, const fe& f) {
  PV_COUNT(sq);
  PV_CHECK_SQ2X(f);
  fe_sq_t<2>(h, f);
}

// ---- two / three independent products at once (k_curve_half's hot loop).
// Same column sums, carries and bounds as fe_mul / fe_sq; on the device each
// column of the C products is ONE asm block with the C v_mad_u64_u32 chains
// interleaved instruction by instruction (pv_madchains.h), so a wave always
// has C independent MADs to issue instead of one serial chain.
template <int C>
PV_HD void fe_mul_n(fe* const h[C], const fe* const f[C], const fe* const g[C]) {
#if defined(PV_MADN_PLAIN)
#pragma unroll
  for (int c = 0; c < C; ++c) fe_mul(*h[c], *f[c], *g[c]);
#else
  uint32_t g19[C][10], f2[C][10];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    PV_COUNT(mul);
#pragma unroll
    for (int j = 1; j < 10; ++j) g19[c][j] = 19u * g[c]->v[j];
#pragma unroll
    for (int i = 1; i < 10; i += 2) f2[c][i] = twice(f[c]->v[i]);
  }
  uint64_t carry[C];
  uint32_t out[C][10];
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    uint32_t a[C][10], b[C][10];
#pragma unroll
    for (int c = 0; c < C; ++c) {
#pragma unroll
      for (int i = 0; i < 10; ++i) {
        const int j = (k - i + 10) % 10;
        const bool oo = (i & 1) && (j & 1);
        a[c][i] = oo ? f2[c][i] : f[c]->v[i];
        b[c][i] = i + j >= 10 ? g19[c][j] : g[c]->v[j];
      }
    }
    uint64_t acc[C];
    if constexpr (C == 2) {
      if (k == 0) madc10x2z(acc[0], acc[1], a[0], b[0], a[1], b[1]);
      else madc10x2(acc[0], acc[1], a[0], b[0], a[1], b[1], carry[0], carry[1]);
    } else {
      static_assert(C == 3, "fe_mul_n: 2 or 3 products");
      if (k == 0) madc10x3z(acc[0], acc[1], acc[2], a[0], b[0], a[1], b[1], a[2], b[2]);
      else madc10x3(acc[0], acc[1], acc[2], a[0], b[0], a[1], b[1], a[2], b[2], carry[0], carry[1], carry[2]);
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
      carry[c] = acc[c] >> ((k & 1) ? 25 : 26);
      out[c][k] = (uint32_t)acc[c] & ((k & 1) ? M25 : M26);
    }
  }
#pragma unroll
  for (int c = 0; c < C; ++c) fe_finish_columns(*h[c], carry[c], out[c]);
#endif
}

template <int C>
PV_HD void fe_sq_n(fe* const h[C], const fe* const f[C]) {
#if defined(PV_MADN_PLAIN)
#pragma unroll
  for (int c = 0; c < C; ++c) fe_sq(*h[c], *f[c]);
#else
  sq_ops o[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    PV_COUNT(sq);
    sq_prepare(o[c], *f[c]);
  }
  uint64_t carry[C];
  uint32_t out[C][10];
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    uint32_t as[C][6], bs[C][6];
#pragma unroll
    for (int c = 0; c < C; ++c) sq_column<1>(o[c], k, as[c], bs[c]);
    uint64_t acc[C];
    if constexpr (C == 2) {
      if (k & 1) madc5x2(acc[0], acc[1], as[0], bs[0], as[1], bs[1], carry[0], carry[1]);
      else if (k == 0) madc6x2z(acc[0], acc[1], as[0], bs[0], as[1], bs[1]);
      else madc6x2(acc[0], acc[1], as[0], bs[0], as[1], bs[1], carry[0], carry[1]);
    } else {
      static_assert(C == 3, "fe_sq_n: 2 or 3 squares");
      if (k & 1) madc5x3(acc[0], acc[1], acc[2], as[0], bs[0], as[1], bs[1], as[2], bs[2], carry[0], carry[1], carry[2]);
      else if (k == 0) madc6x3z(acc[0], acc[1], acc[2], as[0], bs[0], as[1], bs[1], as[2], bs[2]);
      else madc6x3(acc[0], acc[1], acc[2], as[0], bs[0], as[1], bs[1], as[2], bs[2], carry[0], carry[1], carry[2]);
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
      carry[c] = acc[c] >> ((k & 1) ? 25 : 26);
      out[c][k] = (uint32_t)acc[c] & ((k & 1) ? M25 : M26);
    }
  }
#pragma unroll
  for (int c = 0; c < C; ++c) fe_finish_columns(*h[c], carry[c], out[c]);
#endif
}

PV_HD void fe_mul2(fe& h0, const fe& f0, const fe& g0, fe& h1, const fe& f1, const fe& g1) {
  PV_CHECK_MUL(f0, g0);
  PV_CHECK_MUL(f1, g1);
  fe* const h[2] = {&h0, &h1};
  const fe* const f[2] = {&f0, &f1};
  const fe* const g[2] = {&g0, &g1};
  fe_mul_n<2>(h, f, g);
  PV_FE_FENCE();
}
PV_HD void fe_mul3(fe& h0, const fe& f0, const fe& g0, fe& h1, const fe& f1, const fe& g1, fe& h2, const fe& f2,
                   const fe& g2) {
  PV_CHECK_MUL(f0, g0);
  PV_CHECK_MUL(f1, g1);
  PV_CHECK_MUL(f2, g2);
  fe* const h[3] = {&h0, &h1, &h2};
  const fe* const f[3] = {&f0, &f1, &f2};
  const fe* const g[3] = {&g0, &g1, &g2};
  fe_mul_n<3>(h, f, g);
  PV_FE_FENCE();
}
PV_HD void fe_sq2(fe& h0, const fe& f0, fe& h1, const fe& f1) {
  PV_CHECK_SQ(f0);
  PV_CHECK_SQ(f1);
  fe* const h[2] = {&h0, &h1};
  const fe* const f[2] = {&f0, &f1};
  fe_sq_n<2>(h, f);
  PV_FE_FENCE();
}

// ---- latency forms (a wave alone on its SIMD: the latency kernels).
// The carry-seeded columns of fe_mul / fe_sq are ONE dependent chain per
// product (column k starts from column k-1's carry), which suits the
// throughput kernels: two waves per SIMD hide each other's latency and every
// saved instruction counts.  A wave ALONE issues a dependent v_mad_u64_u32
// every ~10 cycles but independent ones every ~5.5
// (profiles/r05_lane_exec.json: mad_dep vs mad_ind4).  Here every column
// starts from zero, two columns' chains are interleaved in one asm block, and
// the carries run afterwards in the same order -- acc_k = C_k + carry_{k-1},
// limb_k = acc_k & mask, carry_k = acc_k >> 25/26, then the x19 wrap -- so
// acc_k, and hence every limb, is bit-identical to fe_mul / fe_sq_t's (the
// same bounds hold; the host build runs the seeded forms).
// MEASURED SLOWER on a lone wave (profiles/r05_fe_lat.json: fe_sq_l 506 vs
// fe_sq 454 cycles, fe_mul_l 671 vs 654 -- the split columns issue more
// instructions, and a lone wave is issue-bound): no
// kernel uses them; tools/ubench/fe_lat.hip keeps the comparison reproducible.
#if defined(PV_MADN_PLAIN)
PV_HD void fe_mul_l(fe& h, const fe& f, const fe& g) { fe_mul(h, f, g); }
template <int MULT>
PV_HD void fe_sq_lt(fe& h, const fe& f) {
  if (MULT == 1) fe_sq(h, f);
  else fe_sq2x(h, f);
}
#else
PV_HD void fe_carry_columns(fe& h, const uint64_t col[10]) {
  uint64_t carry = 0;
  uint32_t out[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    const uint64_t acc = k == 0 ? col[0] : col[k] + carry;
    carry = acc >> ((k & 1) ? 25 : 26);
    out[k] = (uint32_t)acc & ((k & 1) ? M25 : M26);
  }
  fe_finish_columns(h, carry, out);
}
PV_HD void fe_mul_l(fe& h, const fe& f, const fe& g) {
  PV_COUNT(mul);
  uint32_t g19[10], f2[10];
#pragma unroll
  for (int j = 1; j < 10; ++j) g19[j] = 19u * g.v[j];
#pragma unroll
  for (int i = 1; i < 10; i += 2) f2[i] = twice(f.v[i]);
  uint64_t col[10];
#pragma unroll
  for (int k = 0; k < 10; k += 2) {
    uint32_t a[2][10], b[2][10];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
#pragma unroll
      for (int i = 0; i < 10; ++i) {
        const int j = (k + c - i + 10) % 10;
        const bool oo = (i & 1) && (j & 1);
        a[c][i] = oo ? f2[i] : f.v[i];
        b[c][i] = i + j >= 10 ? g19[j] : g.v[j];
      }
    }
    madc10x2z(col[k], col[k + 1], a[0], b[0], a[1], b[1]);
  }
  fe_carry_columns(h, col);
  PV_FE_FENCE();
}
template <int MULT>
PV_HD void fe_sq_lt(fe& h, const fe& f) {
  PV_COUNT(sq);
  sq_ops o;
  sq_prepare(o, f);
  uint64_t col[10];
  uint32_t as[10][6], bs[10][6];
#pragma unroll
  for (int k = 0; k < 10; ++k) sq_column<MULT>(o, k, as[k], bs[k]);
  // pairs of equal width, in carry order: (0,2) (1,3) (4,6) (5,7) (8,9)
  madc6x2z(col[0], col[2], as[0], bs[0], as[2], bs[2]);
  madc5x2z(col[1], col[3], as[1], bs[1], as[3], bs[3]);
  madc6x2z(col[4], col[6], as[4], bs[4], as[6], bs[6]);
  madc5x2z(col[5], col[7], as[5], bs[5], as[7], bs[7]);
  madc6_5z(col[8], col[9], as[8], bs[8], as[9], bs[9]);
  fe_carry_columns(h, col);
  PV_FE_FENCE();
}
#endif
PV_HD void fe_sq_l(fe& h, const fe& f) {
  PV_CHECK_SQ(f);
  fe_sq_lt<1>(h, f);
}
PV_HD void fe_sq2x_l(fe& h, const fe& f) {
  PV_CHECK_SQ2X(f);
  fe_sq_lt<2>(h, f);
}
PV_HD void fe_sqn_l(fe& h, const fe& f, int n) {
  fe_sq_l(h, f);
#pragma unroll 1
  for (int i = 1; i < n; ++i) fe_sq_l(h, h);
}

PV_HD void fe_sqn(fe& h, const fe& f, int n) {
  fe_sq(h, f);
#pragma unroll 1
  for (int i = 1; i < n; ++i) fe_sq(h, h);
}

PV_HD void fe_add(fe& h, const fe& f, const fe& g) {
  PV_COUNT(add);
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = f.v[i] + g.v[i];
}

// 2p in radix 2^25.5
static constexpr uint32_t P2_0 = 2u * ((1u << 26) - 19);
static constexpr uint32_t P2_E = 2u * ((1u << 26) - 1);
static constexpr uint32_t P2_O = 2u * ((1u << 25) - 1);

// h = f - g + 2p ; g must be TIGHT.  LOOSE result when f is TIGHT.
PV_HD void fe_sub(fe& h, const fe& f, const fe& g) {
  PV_COUNT(sub);
  h.v[0] = f.v[0] + P2_0 - g.v[0];
#pragma unroll
  for (int i = 1; i < 10; ++i) h.v[i] = f.v[i] + ((i & 1) ? P2_O : P2_E) - g.v[i];
}

// h = f - g + 4p ; g may be LOOSE up to 2^28 / 2^27.  Result needs fe_carry.
PV_HD void fe_sub4(fe& h, const fe& f, const fe& g) {
  PV_COUNT(sub);
  h.v[0] = f.v[0] + 2u * P2_0 - g.v[0];
#pragma unroll
  for (int i = 1; i < 10; ++i) h.v[i] = f.v[i] + 2u * ((i & 1) ? P2_O : P2_E) - g.v[i];
}

// -f = 2p - f (f TIGHT) -> LOOSE
PV_HD void fe_neg(fe& h, const fe& f) {
  PV_COUNT(sub);
  h.v[0] = P2_0 - f.v[0];
#pragma unroll
  for (int i = 1; i < 10; ++i) h.v[i] = ((i & 1) ? P2_O : P2_E) - f.v[i];
}

// one carry pass over 32-bit limbs (inputs up to ~2^31): -> TIGHT
PV_HD void fe_carry(fe& h) {
  PV_COUNT(carry);
  uint32_t c;
  c = h.v[0] >> 26; h.v[0] &= M26; h.v[1] += c;
  c = h.v[1] >> 25; h.v[1] &= M25; h.v[2] += c;
  c = h.v[2] >> 26; h.v[2] &= M26; h.v[3] += c;
  c = h.v[3] >> 25; h.v[3] &= M25; h.v[4] += c;
  c = h.v[4] >> 26; h.v[4] &= M26; h.v[5] += c;
  c = h.v[5] >> 25; h.v[5] &= M25; h.v[6] += c;
  c = h.v[6] >> 26; h.v[6] &= M26; h.v[7] += c;
  c = h.v[7] >> 25; h.v[7] &= M25; h.v[8] += c;
  c = h.v[8] >> 26; h.v[8] &= M26; h.v[9] += c;
  c = h.v[9] >> 25; h.v[9] &= M25; h.v[0] += 19u * c;
}

// carries out of the EVEN limbs only (into the odd limb above; no wrap):
// 15 ops instead of 30, five independent chains.  Even limbs -> < 2^26, odd
// limbs grow by < 2^(max even - 26).  Enough where only the even limbs exceed
// an operand bound (ge_p2_dbl's T: even <= 2^28.6, odd <= 2^27.6 before,
// odd <= 2^27.6 + 6 after, so 19 T_j < 2^32 for every j).
PV_HD void fe_carry_even(fe& h) {
  PV_COUNT(carry_even);
#pragma unroll
  for (int i = 0; i < 10; i += 2) {
    const uint32_t c = h.v[i] >> 26;
    h.v[i] &= M26;
    h.v[i + 1] += c;
  }
}

// conditional select: h = c ? g : f  (lane-local, branch-free)
PV_HD void fe_cmov(fe& h, const fe& f, const fe& g, bool c) {
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = c ? g.v[i] : f.v[i];
}

// 32-byte little-endian (as 8 words) -> limbs; bit 255 dropped (value < 2^255, TIGHT)
PV_HD void fe_frombytes_w(fe& h, const uint32_t w[8]) {
  h.v[0] = w[0] & M26;
  h.v[1] = ((w[0] >> 26) | (w[1] << 6)) & M25;
  h.v[2] = ((w[1] >> 19) | (w[2] << 13)) & M26;
  h.v[3] = ((w[2] >> 13) | (w[3] << 19)) & M25;
  h.v[4] = (w[3] >> 6) & M26;
  h.v[5] = w[4] & M25;
  h.v[6] = ((w[4] >> 25) | (w[5] << 7)) & M26;
  h.v[7] = ((w[5] >> 19) | (w[6] << 13)) & M25;
  h.v[8] = ((w[6] >> 12) | (w[7] << 20)) & M26;
  h.v[9] = (w[7] >> 6) & M25;
}

// canonical (fully reduced mod p) little-endian words.  Accepts any limbs a
// single fe_carry pass brings to TIGHT (value then < 2p).
PV_HD void fe_tobytes_w(uint32_t w[8], const fe& f) {
  fe h;
  fe_copy(h, f);
  fe_carry(h);
  fe_carry(h);
  // q = [h >= p] = carry out of h + 19 at bit 255
  uint32_t q = (h.v[0] + 19u) >> 26;
  q = (h.v[1] + q) >> 25;
  q = (h.v[2] + q) >> 26;
  q = (h.v[3] + q) >> 25;
  q = (h.v[4] + q) >> 26;
  q = (h.v[5] + q) >> 25;
  q = (h.v[6] + q) >> 26;
  q = (h.v[7] + q) >> 25;
  q = (h.v[8] + q) >> 26;
  q = (h.v[9] + q) >> 25;
  h.v[0] += 19u * q;
  uint32_t c;
  c = h.v[0] >> 26; h.v[0] &= M26; h.v[1] += c;
  c = h.v[1] >> 25; h.v[1] &= M25; h.v[2] += c;
  c = h.v[2] >> 26; h.v[2] &= M26; h.v[3] += c;
  c = h.v[3] >> 25; h.v[3] &= M25; h.v[4] += c;
  c = h.v[4] >> 26; h.v[4] &= M26; h.v[5] += c;
  c = h.v[5] >> 25; h.v[5] &= M25; h.v[6] += c;
  c = h.v[6] >> 26; h.v[6] &= M26; h.v[7] += c;
  c = h.v[7] >> 25; h.v[7] &= M25; h.v[8] += c;
  c = h.v[8] >> 26; h.v[8] &= M26; h.v[9] += c;
  h.v[9] &= M25;  // the dropped carry is q * 2^255
  w[0] = h.v[0] | (h.v[1] << 26);
  w[1] = (h.v[1] >> 6) | (h.v[2] << 19);
  w[2] = (h.v[2] >> 13) | (h.v[3] << 13);
  w[3] = (h.v[3] >> 19) | (h.v[4] << 6);
  w[4] = h.v[5] | (h.v[6] << 25);
  w[5] = (h.v[6] >> 7) | (h.v[7] << 19);
  w[6] = (h.v[7] >> 13) | (h.v[8] << 12);
  w[7] = (h.v[8] >> 20) | (h.v[9] << 6);
}

PV_HD bool fe_iszero(const fe& f) {
  uint32_t w[8];
  fe_tobytes_w(w, f);
  uint32_t d = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) d |= w[i];
  return d == 0;
}

PV_HD uint32_t fe_isnegative(const fe& f) {
  uint32_t w[8];
  fe_tobytes_w(w, f);
  return w[0] & 1u;
}

// z^(2^250 - 1) and z^11, the common prefix of the inversion and sqrt chains
PV_HD void fe_pow_2_250_1(fe& out, fe& z11, const fe& z) {
  fe z2, z9, t, a, b, c;
  fe_sq(z2, z);
  fe_sqn(t, z2, 2);
  fe_mul(z9, t, z);
  fe_mul(z11, z9, z2);
  fe_sq(t, z11);
  fe_mul(a, t, z9);                    // 2^5 - 1
  fe_sqn(t, a, 5);    fe_mul(b, t, a); // 2^10 - 1
  fe_sqn(t, b, 10);   fe_mul(c, t, b); // 2^20 - 1
  fe_sqn(t, c, 20);   fe_mul(t, t, c); // 2^40 - 1
  fe_sqn(t, t, 10);   fe_mul(a, t, b); // 2^50 - 1
  fe_sqn(t, a, 50);   fe_mul(b, t, a); // 2^100 - 1
  fe_sqn(t, b, 100);  fe_mul(t, t, b); // 2^200 - 1
  fe_sqn(t, t, 50);   fe_mul(out, t, a); // 2^250 - 1
}

// z^(p-2)
PV_HD void fe_invert(fe& h, const fe& z) {
  fe t, z11;
  fe_pow_2_250_1(t, z11, z);
  fe_sqn(t, t, 5);
  fe_mul(h, t, z11);
}

// z^((p-5)/8)
PV_HD void fe_pow22523(fe& h, const fe& z) {
  fe t, z11;
  fe_pow_2_250_1(t, z11, z);
  fe_sqn(t, t, 2);
  fe_mul(h, t, z);
}

// curve constants as TIGHT limbs (values checked against the oracle in tests)
PV_HD void fe_const_d(fe& h) {  // d = -121665/121666
  const uint32_t v[10] = {56195235u, 13857412u, 51736253u, 6949390u, 114729u,
                          24766616u, 60832955u, 30306712u, 48412415u, 21499315u};
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = v[i];
}
PV_HD void fe_const_d2(fe& h) {  // 2d
  const uint32_t v[10] = {45281625u, 27714825u, 36363642u, 13898781u, 229458u,
                          15978800u, 54557047u, 27058993u, 29715967u, 9444199u};
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = v[i];
}
PV_HD void fe_const_sqrtm1(fe& h) {  // 2^((p-1)/4)
  const uint32_t v[10] = {34513072u, 25610706u, 9377949u, 3500415u, 12389472u,
                          33281959u, 41962654u, 31548777u, 326685u, 11406482u};
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = v[i];
}

}  // namespace pv
