// Per-signature algorithms shared by the HIP kernels (pv_kernels.hip) and the
// host instrumentation build (tools/hostcheck: bound checks, op counts, gdb).
// Everything here is lane-local; the kernels only add indexing, LDS staging
// and the wavefront ballot.
//
//   hash_one   : SURVEY.md App. C.2 steps 1-3 and 5
//   curve_one  : steps 4, 6, 7
//   sign_one   : crypto_sign_seed_keypair + crypto_sign_detached (batch signer)
#pragma once
#include <stdint.h>
#include "pv_field.h"
#include "pv_scalar.h"
#include "pv_curve.h"
#include "pv_sha512.h"

namespace pv {

constexpr int BT_ENTRIES = 129;   // niels k*B, k = 0..128
constexpr int BT_WORDS = 32;      // 3 fe (30 words) padded to 32
constexpr int AT_ENTRY = 40;      // cached entry words
constexpr int AT_WORDS = 9 * 40;  // k*(-A), k = 0..8

PV_HD void load8(uint32_t w[8], const uint8_t* p) {
  const uint32_t* q = reinterpret_cast<const uint32_t*>(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = q[i];
}
PV_HD void store8(uint8_t* p, const uint32_t w[8]) {
  uint32_t* q = reinterpret_cast<uint32_t*>(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) q[i] = w[i];
}

// a[k] for a wave-uniform k without dynamic register indexing (7 selects)
PV_HD uint32_t pick8(const uint32_t a[8], int k) {
  uint32_t r = a[0];
#pragma unroll
  for (int j = 1; j < 8; ++j) r = (k == j) ? a[j] : r;
  return r;
}

PV_HD uint64_t bswap64(uint64_t x) {
  return ((uint64_t)bswap32((uint32_t)x) << 32) | bswap32((uint32_t)(x >> 32));
}

// 8 bytes of M at byte q, little-endian packed; bytes past mlen are zero and
// byte mlen is the 0x80 pad.  Reads 3 aligned words (callers guarantee >= 16
// readable bytes after the last message).
PV_HD uint64_t msg_bytes8(const uint8_t* m, uint64_t mlen, uint64_t q) {
  uint64_t v = 0;
  if (q < mlen) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(m + q);
    const uint32_t* wp = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
    const uint32_t s = (uint32_t)(a & 3u) * 8u;
    const uint32_t w0 = wp[0], w1 = wp[1], w2 = wp[2];
    const uint32_t lo = (uint32_t)((((uint64_t)w1 << 32) | w0) >> s);
    const uint32_t hi = (uint32_t)((((uint64_t)w2 << 32) | w1) >> s);
    v = ((uint64_t)hi << 32) | lo;
  }
  const uint64_t rem = mlen > q ? mlen - q : 0;
  if (rem < 8) {
    const uint64_t keep = rem == 0 ? 0 : ((1ull << (8 * rem)) - 1);
    v &= keep;
    if (q <= mlen) v |= 0x80ull << (8 * rem);
  }
  return v;
}

// SHA-512(prefix || M); prefix = pre_words64 * 8 bytes held as LE words
PV_HD void sha512_prefixed(uint32_t out[16], const uint32_t* pre, int pre_words64, const uint8_t* m, uint64_t mlen) {
  uint64_t h[8], w[16];
  sha512_init(h);
  const uint64_t total = (uint64_t)pre_words64 * 8 + mlen;
  const uint64_t nblocks = (total + 17 + 127) / 128;
  for (uint64_t b = 0; b < nblocks; ++b) {
    const bool last = b + 1 == nblocks;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint64_t g = b * 16 + j;
      uint64_t word;
      if (g < (uint64_t)pre_words64) {
        word = be64_from_le32(pre[2 * g], pre[2 * g + 1]);
      } else {
        word = bswap64(msg_bytes8(m, mlen, (g - pre_words64) * 8));
      }
      if (last && j == 14) word = 0;
      if (last && j == 15) word = total * 8;
      w[j] = word;
    }
    sha512_compress(h, w);
  }
  sha512_digest_words(out, h);
}

// ------------------------------------------------------------------ hash
// pre-checks + h = SHA-512(R||A||M) mod L.  Returns the pre-check verdict.
PV_HD bool hash_one(uint32_t h[8], const uint8_t* pk, const uint8_t* sig, const uint8_t* m, uint64_t mlen) {
  uint32_t ra[16], sw[8];
  load8(ra, sig);
  load8(sw, sig + 32);
  load8(ra + 8, pk);
  const bool ok = sc_is_canonical(sw) && !has_small_order(ra) && y_is_canonical(ra + 8) && !has_small_order(ra + 8);
#pragma unroll
  for (int k = 0; k < 8; ++k) h[k] = 0;
  if (ok) {
    uint32_t dig[16];
    sha512_prefixed(dig, ra, 8, m, mlen);
    sc_reduce64(h, dig);
  }
  return ok;
}

// ------------------------------------------------------------ table access
PV_HD void store_fe(uint32_t* p, const fe& f) {
#pragma unroll
  for (int i = 0; i < 10; ++i) p[i] = f.v[i];
}
PV_HD void load_fe(fe& f, const uint32_t* p) {
#pragma unroll
  for (int i = 0; i < 10; ++i) f.v[i] = p[i];
}
PV_HD void store_cached(uint32_t* p, const ge_cached& c) {
  store_fe(p, c.YpX);
  store_fe(p + 10, c.YmX);
  store_fe(p + 20, c.Z2);
  store_fe(p + 30, c.T2d);
}
PV_HD void load_cached(ge_cached& c, const uint32_t* p) {
  load_fe(c.YpX, p);
  load_fe(c.YmX, p + 10);
  load_fe(c.Z2, p + 20);
  load_fe(c.T2d, p + 30);
}
PV_HD void load_niels(ge_niels& q, const uint32_t* p) {
  load_fe(q.ypx, p);
  load_fe(q.ymx, p + 10);
  load_fe(q.xy2d, p + 20);
}

// -------------------------------------------------------- base-point table
PV_HD void ge_basepoint(ge_p3& B) {
  const uint32_t enc[8] = {0x66666658u, 0x66666666u, 0x66666666u, 0x66666666u,
                           0x66666666u, 0x66666666u, 0x66666666u, 0x66666666u};
  ge_p3 nb;
  ge_frombytes_negate(nb, enc);  // -B
  fe_copy(B.Y, nb.Y);
  fe_copy(B.Z, nb.Z);
  fe_neg(B.X, nb.X); fe_carry(B.X);
  fe_neg(B.T, nb.T); fe_carry(B.T);
}

// niels form of k*B (k <= 255), written as 32 words
PV_HD void btable_entry(uint32_t* p, int k) {
  ge_p3 B, acc;
  ge_basepoint(B);
  ge_cached cb;
  ge_p3_to_cached(cb, B);
  ge_p3_0(acc);
  for (int bit = 7; bit >= 0; --bit) {
    ge_p1p1 t;
    ge_p3_dbl(t, acc);
    ge_p1p1_to_p3(acc, t);
    if ((k >> bit) & 1) {
      ge_add_cached(t, acc, cb, false);
      ge_p1p1_to_p3(acc, t);
    }
  }
  fe zi, x, y, d2, ypx, ymx, xy2d;
  fe_invert(zi, acc.Z);
  fe_mul(x, acc.X, zi);
  fe_mul(y, acc.Y, zi);
  fe_const_d2(d2);
  fe_add(ypx, y, x); fe_carry(ypx);
  fe_sub(ymx, y, x); fe_carry(ymx);
  fe_mul(xy2d, x, y);
  fe_mul(xy2d, xy2d, d2);
  store_fe(p, ypx);
  store_fe(p + 10, ymx);
  store_fe(p + 20, xy2d);
  p[30] = 0;
  p[31] = 0;
}

// ----------------------------------------------------------------- curve
// cached multiples 0..8 of P into a per-lane table (9 x 40 words)
PV_HD void build_atab(uint32_t* atab, const ge_p3& P) {
  ge_cached c1, c;
  ge_cached_identity(c);
  store_cached(atab, c);
  ge_p3_to_cached(c1, P);
  store_cached(atab + AT_ENTRY, c1);
  ge_p3 prev = P;
  ge_p1p1 t;
#pragma unroll 1
  for (int k = 2; k <= 8; ++k) {
    ge_add_cached(t, prev, c1, false);
    ge_p1p1_to_p3(prev, t);
    ge_p3_to_cached(c, prev);
    store_cached(atab + AT_ENTRY * k, c);
  }
}

// R' = hh*(-A) + ss*B.  hh + 0x88..88 gives radix-16 digits (nibble - 8) in
// [-8, 8); ss + 0x8080..80 gives radix-256 digits (byte - 128) in [-128, 128);
// hh, ss < 2^253 so neither addition overflows 2^256.  Horner from the top:
// per window 4 doublings, one A add, and a B add on even windows.
PV_HD void double_scalarmult(ge_p2& out, const uint32_t hh[8], const uint32_t ss[8], const uint32_t* atab,
                             const uint32_t* btab) {
  uint32_t hp[8], sp[8];
  sc_add_pattern(hp, hh, 0x88888888u);
  sc_add_pattern(sp, ss, 0x80808080u);
  ge_p3 acc;
  ge_p3_0(acc);
  ge_p1p1 t;
  ge_p2 r2;
  {
    const int dA = (int)(hp[7] >> 28) - 8;
    ge_cached c;
    load_cached(c, atab + (dA < 0 ? -dA : dA) * AT_ENTRY);
    ge_add_cached(t, acc, c, dA < 0);
    ge_p1p1_to_p2(r2, t);
  }
#pragma unroll 1
  for (int i = 62; i >= 0; --i) {
#pragma unroll 1
    for (int k = 0; k < 3; ++k) {
      ge_p2_dbl(t, r2);
      ge_p1p1_to_p2(r2, t);
    }
    ge_p2_dbl(t, r2);
    ge_p1p1_to_p3(acc, t);
    const uint32_t hw = pick8(hp, i >> 3);
    const int dA = (int)((hw >> (4 * (i & 7))) & 15u) - 8;
    {
      ge_cached c;
      load_cached(c, atab + (dA < 0 ? -dA : dA) * AT_ENTRY);
      ge_add_cached(t, acc, c, dA < 0);
    }
    if ((i & 1) == 0) {
      const uint32_t sw = pick8(sp, i >> 3);
      const int dB = (int)((sw >> (8 * ((i >> 1) & 3))) & 255u) - 128;
      ge_p1p1_to_p3(acc, t);
      ge_niels q;
      load_niels(q, btab + (dB < 0 ? -dB : dB) * BT_WORDS);
      ge_madd(t, acc, q, dB < 0);
    }
    ge_p1p1_to_p2(r2, t);
  }
  out = r2;
}

// decompress A, R' = h(-A) + S B, encode(R') == R.  `atab` is this lane's
// 360-word scratch; `btab` the base-point table (LDS in the kernel).
PV_HD bool curve_one(const uint8_t* pk, const uint8_t* sig, const uint32_t hh[8], uint32_t* atab,
                     const uint32_t* btab) {
  uint32_t A[8], R[8], S[8];
  load8(A, pk);
  load8(R, sig);
  load8(S, sig + 32);
  ge_p3 negA;
  if (!ge_frombytes_negate(negA, A)) return false;
  build_atab(atab, negA);
  ge_p2 rp;
  double_scalarmult(rp, hh, S, atab, btab);
  uint32_t enc[8];
  ge_p2_tobytes(enc, rp);
  uint32_t diff = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) diff |= enc[k] ^ R[k];
  return diff == 0;
}

// ------------------------------------------------------------ batch signer
// fixed-base k*B for k < 2^253, radix-256 signed digits, 8 doublings per digit
PV_HD void scalarmult_base(ge_p3& out, const uint32_t k[8], const uint32_t* btab) {
  uint32_t kp[8];
  sc_add_pattern(kp, k, 0x80808080u);
  ge_p3 acc;
  ge_p3_0(acc);
  ge_p1p1 t;
  ge_p2 r2;
#pragma unroll 1
  for (int j = 31; j >= 0; --j) {
    if (j != 31) {
      fe_copy(r2.X, acc.X);
      fe_copy(r2.Y, acc.Y);
      fe_copy(r2.Z, acc.Z);
#pragma unroll 1
      for (int d = 0; d < 7; ++d) {
        ge_p2_dbl(t, r2);
        ge_p1p1_to_p2(r2, t);
      }
      ge_p2_dbl(t, r2);
      ge_p1p1_to_p3(acc, t);
    }
    const uint32_t w = pick8(kp, j >> 2);
    const int dB = (int)((w >> (8 * (j & 3))) & 255u) - 128;
    ge_niels q;
    load_niels(q, btab + (dB < 0 ? -dB : dB) * BT_WORDS);
    ge_madd(t, acc, q, dB < 0);
    ge_p1p1_to_p3(acc, t);
  }
  out = acc;
}

// keypair(seed) and detached signature over M (RFC 8032 / crypto_sign_detached)
PV_HD void sign_one(uint8_t pk_out[32], uint8_t sig_out[64], const uint8_t seed_b[32], const uint8_t* m, uint64_t mlen,
                    const uint32_t* btab) {
  uint32_t seed[8], az[16];
  load8(seed, seed_b);
  sha512_short(az, seed, 32);
  az[0] &= 0xfffffff8u;
  az[7] &= 0x7fffffffu;
  az[7] |= 0x40000000u;
  uint32_t wide[16], ared[8];
#pragma unroll
  for (int k = 0; k < 16; ++k) wide[k] = k < 8 ? az[k] : 0u;
  sc_reduce64(ared, wide);  // a mod L: a*B unchanged (B has order L)
  ge_p3 A;
  scalarmult_base(A, ared, btab);
  uint32_t pkw[8];
  ge_p3_tobytes(pkw, A);
  uint32_t dig[16], r[8];
  sha512_prefixed(dig, az + 8, 4, m, mlen);
  sc_reduce64(r, dig);
  ge_p3 Rp;
  scalarmult_base(Rp, r, btab);
  uint32_t ra[16];
  ge_p3_tobytes(ra, Rp);
#pragma unroll
  for (int k = 0; k < 8; ++k) ra[8 + k] = pkw[k];
  uint32_t kk[8];
  sha512_prefixed(dig, ra, 8, m, mlen);
  sc_reduce64(kk, dig);
  uint32_t S[8];
  sc_muladd(S, kk, az, r);
  store8(pk_out, pkw);
  store8(sig_out, ra);
  store8(sig_out + 32, S);
}

// ------------------------------------------------------ synthetic workload
// SHA-512 input tag || cfg || u64le(i) [|| u64le(c)]  (plenum_gpu/synth.py)
PV_HD int put_tag(uint32_t w[16], const char* tag, int taglen, uint32_t cfg, uint64_t i, bool with_c, uint64_t c) {
  uint8_t b[64];
  int n = 0;
  for (int k = 0; k < taglen; ++k) b[n++] = (uint8_t)tag[k];
  b[n++] = (uint8_t)cfg;
  for (int k = 0; k < 8; ++k) b[n++] = (uint8_t)(i >> (8 * k));
  if (with_c)
    for (int k = 0; k < 8; ++k) b[n++] = (uint8_t)(c >> (8 * k));
  for (int k = n; k < 64; ++k) b[k] = 0;
  for (int k = 0; k < 16; ++k)
    w[k] = (uint32_t)b[4 * k] | ((uint32_t)b[4 * k + 1] << 8) | ((uint32_t)b[4 * k + 2] << 16) |
           ((uint32_t)b[4 * k + 3] << 24);
  return n;
}

}  // namespace pv
