// Scalars modulo L = 2^252 + 27742317777372353535851937790883648493.
//
//  * sc_reduce64   : 512-bit SHA-512 output -> h mod L  (Barrett, HAC 14.42,
//                    b = 2^32, k = 8).  Restates sc25519_reduce, step 5 of
//                    SURVEY.md Appendix C.2.
//  * sc_is_canonical: S < L  (step 1 of Appendix C.2)
//  * sc_muladd     : (a*b + c) mod L for the batch signer (fixture/bench data)
//
// Words are little-endian uint32.
#pragma once
#include <stdint.h>
#include "pv_field.h"

namespace pv {

// L as 8 little-endian words
PV_HD uint32_t sc_L(int i) {
  const uint32_t L[8] = {0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu, 0u, 0u, 0u, 0x10000000u};
  return L[i];
}

// S < L, strictly (S as 8 LE words)
PV_HD bool sc_is_canonical(const uint32_t s[8]) {
  // lexicographic compare from the top word
  bool lt = false, decided = false;
#pragma unroll
  for (int i = 7; i >= 0; --i) {
    const uint32_t l = sc_L(i);
    if (!decided && s[i] != l) {
      lt = s[i] < l;
      decided = true;
    }
  }
  return decided && lt;
}

// r (9 words) >= L ? r - L : r     (r < 2^288)
PV_HD void sc_cond_sub_L(uint32_t r[9]) {
  uint32_t t[9];
  uint64_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const uint64_t li = i < 8 ? sc_L(i) : 0u;
    const uint64_t d = (uint64_t)r[i] - li - borrow;
    t[i] = (uint32_t)d;
    borrow = (d >> 63) & 1u;
  }
  const bool ge = borrow == 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) r[i] = ge ? t[i] : r[i];
}

// x: 16 LE words (< 2^512)  ->  out: 8 LE words, x mod L
PV_HD void sc_reduce64(uint32_t out[8], const uint32_t x[16]) {
  PV_COUNT(sc);
  // mu = floor(2^512 / L), 9 words
  const uint32_t mu[9] = {0x0a2c131bu, 0xed9ce5a3u, 0x086329a7u, 0x2106215du, 0xffffffebu,
                          0xffffffffu, 0xffffffffu, 0xffffffffu, 0x0000000fu};
  // q1 = x >> 224 (words 7..15), q3 = (q1 * mu) >> 288 : only product words 9..17 needed,
  // but carries from lower columns matter, so accumulate all columns >= 7 exactly and
  // words < 7 for their carries.
  uint32_t q2[18];
  uint64_t carry = 0;
  // column-wise product of q1 (9 words) and mu (9 words)
#pragma unroll
  for (int k = 0; k < 18; ++k) {
    uint64_t lo = carry & 0xffffffffu, hi = carry >> 32;  // 96-bit accumulator (hi:lo as 32+64)
    uint64_t acc = lo;
    uint64_t acchi = hi;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const int j = k - i;
      if (j >= 0 && j < 9) {
        const uint64_t p = mul32x32(x[7 + i], mu[j]);
        acc += p & 0xffffffffu;
        acchi += p >> 32;
      }
    }
    acchi += acc >> 32;
    q2[k] = (uint32_t)acc;
    carry = acchi;
  }
  const uint32_t* q3 = q2 + 9;  // 9 words
  // r2 = (q3 * L) mod 2^288
  uint32_t r2[9];
  carry = 0;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    uint64_t acc = carry & 0xffffffffu;
    uint64_t acchi = carry >> 32;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const int j = k - i;
      if (j >= 0 && j < 8) {
        const uint64_t p = mul32x32(q3[i], sc_L(j));
        acc += p & 0xffffffffu;
        acchi += p >> 32;
      }
    }
    acchi += acc >> 32;
    r2[k] = (uint32_t)acc;
    carry = acchi;
  }
  // r = (x mod 2^288) - r2 (mod 2^288)
  uint32_t r[9];
  uint64_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const uint64_t d = (uint64_t)x[i] - r2[i] - borrow;
    r[i] = (uint32_t)d;
    borrow = (d >> 63) & 1u;
  }
  sc_cond_sub_L(r);
  sc_cond_sub_L(r);
#pragma unroll
  for (int i = 0; i < 8; ++i) out[i] = r[i];
}

// out = (a * b + c) mod L  (all 8-word scalars < 2^256)
PV_HD void sc_muladd(uint32_t out[8], const uint32_t a[8], const uint32_t b[8], const uint32_t c[8]) {
  uint32_t x[16];
  uint64_t carry = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    uint64_t acc = (carry & 0xffffffffu) + (k < 8 ? c[k] : 0u);
    uint64_t acchi = carry >> 32;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int j = k - i;
      if (j >= 0 && j < 8) {
        const uint64_t p = mul32x32(a[i], b[j]);
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

// 256-bit add of a constant word pattern (recoding offset); s < 2^253 so no overflow
PV_HD void sc_add_pattern(uint32_t out[8], const uint32_t s[8], uint32_t pattern) {
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    c += (uint64_t)s[i] + pattern;
    out[i] = (uint32_t)c;
    c >>= 32;
  }
}

}  // namespace pv
