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
#include "pv_lattice.h"

namespace pv {

constexpr int BT_ENTRIES = 129;   // niels k*B, k = 0..128
constexpr int BT_WORDS = 32;      // 3 fe (30 words) padded to 32
#ifndef PV_HALF_PREFETCH
#define PV_HALF_PREFETCH 1
#endif
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
// libsodium 1.0.18 pre-checks on (R, A, S)
PV_HD bool precheck(const uint8_t* pk, const uint8_t* sig) {
  uint32_t r[8], a[8], sw[8];
  load8(r, sig);
  load8(sw, sig + 32);
  load8(a, pk);
  return sc_is_canonical(sw) && !has_small_order(r) && y_is_canonical(a) && !has_small_order(a);
}

// SHA-512 compressions of R || A || M
PV_HD uint64_t hram_blocks(uint64_t mlen) { return (64 + mlen + 17 + 127) / 128; }

PV_HD uint32_t funnel32(uint32_t hi, uint32_t lo, uint32_t sh) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbit(hi, lo, sh);
#else
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> sh);
#endif
}

// message byte offset of block `blk` of R || A || M (block 0 holds R || A and M[0, 64))
PV_HD uint64_t hram_q(uint64_t blk) { return blk == 0 ? 0 : 128 * blk - 64; }

// Raw aligned words covering message bytes [q, q + 128), fetched as 4-word
// groups: group g is loaded iff its first word holds a message byte, so a
// group reads at most 15 bytes past the message end (the blob guarantees 16
// readable bytes after the last message) and each lane issues <= 9 dwordx4
// loads instead of 33 guarded dword loads.  Block 0 only needs words 0..16
// (M[0, 64) behind R || A).  Words past the message are masked by
// msg_assemble.  The pointer keeps the blob's address space (global loads).
#ifndef PV_FETCH_WORDS
constexpr int MSG_Y = 36;
PV_HD void msg_fetch(uint32_t y[MSG_Y], const uint8_t* m, uint64_t mlen, uint64_t q, bool first) {
  const int64_t rem = (int64_t)mlen - (int64_t)q;
  const uint32_t mis = (uint32_t)((reinterpret_cast<uintptr_t>(m) + q) & 3u);
  const uint32_t* wp = reinterpret_cast<const uint32_t*>(m + q - mis);
#pragma unroll
  for (int g = 0; g < 9; ++g) {
    const bool ld = (int64_t)(16 * g) - (int64_t)mis < rem && (!first || g < 5);
    uint32_t a = 0, b = 0, c = 0, d = 0;
    if (ld) {
      a = wp[4 * g];
      b = wp[4 * g + 1];
      c = wp[4 * g + 2];
      d = wp[4 * g + 3];
    }
    y[4 * g] = a;
    y[4 * g + 1] = b;
    y[4 * g + 2] = c;
    y[4 * g + 3] = d;
  }
}
#else
// (A/B baseline) one guarded dword load per word that holds a message byte
constexpr int MSG_Y = 33;
PV_HD void msg_fetch(uint32_t y[MSG_Y], const uint8_t* m, uint64_t mlen, uint64_t q, bool) {
  const int64_t rem = (int64_t)mlen - (int64_t)q;
  const uintptr_t base = reinterpret_cast<uintptr_t>(m) + q;
  const uint32_t mis = (uint32_t)(base & 3u);
  const uint32_t* wp = reinterpret_cast<const uint32_t*>(base - mis);
#pragma unroll
  for (int k = 0; k < 33; ++k) y[k] = (int64_t)(4 * k) - (int64_t)mis < rem ? wp[k] : 0u;
}
#endif

// 32 little-endian words = message bytes [q, q + 128) with SHA padding applied:
// bytes past mlen are zero and byte mlen is 0x80 (funnel shift of the raw words)
// (a & m) | (b & ~m) as one v_bitop3_b32 (an intrinsic the compiler cannot
// turn back into a select of addresses)
PV_HD uint32_t bitsel(uint32_t m, uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(m, a, b, 0xca);
#else
  return (a & m) | (b & ~m);
#endif
}

#ifndef PV_FETCH_WORDS
// groups [g0, g1) of msg_fetch's window only (the same guards): k_hash loads
// the window's first groups one compression ahead (PV_HASH_PF)
PV_HD void msg_fetch_part(uint32_t* y, const uint8_t* m, uint64_t mlen, uint64_t q, bool first, int g0, int g1) {
  const int64_t rem = (int64_t)mlen - (int64_t)q;
  const uint32_t mis = (uint32_t)((reinterpret_cast<uintptr_t>(m) + q) & 3u);
  const uint32_t* wp = reinterpret_cast<const uint32_t*>(m + q - mis);
#pragma unroll
  for (int g = 0; g < 9; ++g) {
    if (g < g0 || g >= g1) continue;
    const bool ld = (int64_t)(16 * g) - (int64_t)mis < rem && (!first || g < 5);
    uint32_t a = 0, b = 0, c = 0, d = 0;
    if (ld) {
      a = wp[4 * g];
      b = wp[4 * g + 1];
      c = wp[4 * g + 2];
      d = wp[4 * g + 3];
    }
    y[4 * (g - g0)] = a;
    y[4 * (g - g0) + 1] = b;
    y[4 * (g - g0) + 2] = c;
    y[4 * (g - g0) + 3] = d;
  }
}
#endif

PV_HD void msg_assemble(uint32_t x[32], const uint32_t y[MSG_Y], const uint8_t* m, uint64_t mlen, uint64_t q) {
  const int64_t rem64 = (int64_t)mlen - (int64_t)q;
  // rem clamped to [-1, 132] (every word full above 128, all zero below 0)
  const int32_t rem = rem64 < 0 ? -1 : (rem64 > 132 ? 132 : (int32_t)rem64);
  const uint32_t mis = (uint32_t)((reinterpret_cast<uintptr_t>(m) + q) & 3u);
  // the one word holding byte `rem` keeps its low rem % 4 bytes and takes the
  // 0x80 pad byte; masks are the same for every k, so each word costs one
  // and-or and two compare-selects (branch-free: no divergent stores)
  const uint32_t rb = 8u * ((uint32_t)rem & 3u);
  const uint32_t keep = (1u << rb) - 1u, pad = 0x80u << rb;
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    const uint32_t v = funnel32(y[k + 1], y[k], 8u * mis);
    const uint32_t t = (v & keep) | pad;
    x[k] = rem >= 4 * k + 4 ? v : (rem >= 4 * k ? t : 0u);
  }
}

// block `blk` of R || A || M as 16 big-endian 64-bit words from the raw message
// words of hram_q(blk) (R, A read from sig/pk on block 0; length words on the last)
// R || A as 16 LE words (block 0's prefix), loaded ahead by the caller
PV_HD void hram_assemble_ra(uint64_t w[16], const uint32_t y[MSG_Y], const uint32_t ra[16], const uint8_t* m,
                            uint64_t mlen, uint64_t blk, uint64_t nblk) {
  const bool first = blk == 0, last = blk + 1 == nblk;
  uint32_t x[32];
  msg_assemble(x, y, m, mlen, hram_q(blk));
  // per-word bitwise selects at static indices: a `?:` between two elements
  // of x is folded by the compiler into ONE load at a computed index, which
  // forces x into private memory (scratch) -- the opaque bit-select keeps the
  // block in registers
  const uint32_t fm = first ? 0xffffffffu : 0u;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    w[j] = be64_from_le32(bitsel(fm, ra[2 * j], x[2 * j]), bitsel(fm, ra[2 * j + 1], x[2 * j + 1]));
    w[8 + j] = be64_from_le32(bitsel(fm, x[2 * j], x[16 + 2 * j]), bitsel(fm, x[2 * j + 1], x[16 + 2 * j + 1]));
  }
  w[14] = last ? 0 : w[14];
  w[15] = last ? (64 + mlen) * 8 : w[15];
}

PV_HD void hram_assemble(uint64_t w[16], const uint32_t y[MSG_Y], const uint8_t* sig, const uint8_t* pk,
                         const uint8_t* m, uint64_t mlen, uint64_t blk, uint64_t nblk) {
  uint32_t ra[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) ra[j] = 0;
  if (blk == 0) {
    load8(ra, sig);
    load8(ra + 8, pk);
  }
  hram_assemble_ra(w, y, ra, m, mlen, blk, nblk);
}

PV_HD void hram_block(uint64_t w[16], const uint8_t* sig, const uint8_t* pk, const uint8_t* m, uint64_t mlen,
                      uint64_t blk, uint64_t nblk) {
  uint32_t y[MSG_Y];
  msg_fetch(y, m, mlen, hram_q(blk), blk == 0);
  hram_assemble(w, y, sig, pk, m, mlen, blk, nblk);
}

// pre-checks + digest = SHA-512(R||A||M) as 16 LE words (reduced mod L by the
// curve stage).  Returns the pre-check verdict; the digest is only written
// when it passes.
PV_HD bool hash_one(uint32_t dig[16], const uint8_t* pk, const uint8_t* sig, const uint8_t* m, uint64_t mlen) {
  if (!precheck(pk, sig)) return false;
  uint64_t h[8], w[16];
  sha512_init(h);
  const uint64_t nb = hram_blocks(mlen);
  for (uint64_t b = 0; b < nb; ++b) {
    hram_block(w, sig, pk, m, mlen, b, nb);
    sha512_compress(h, w);
  }
  sha512_digest_words(dig, h);
  return true;
}

// ------------------------------------------------------------ table access
// Per-lane tables (cached multiples of -A / -R) take a word stride S: S = 1
// is a lane-contiguous table; S = 64 interleaves the 64 lanes of a wavefront
// word by word ([word][lane]), so one load instruction of the wave reads 256
// contiguous bytes instead of touching 64 scattered cache lines.
template <int S = 1>
PV_HD void store_fe(uint32_t* p, const fe& f) {
#pragma unroll
  for (int i = 0; i < 10; ++i) p[i * S] = f.v[i];
}
template <int S = 1>
PV_HD void load_fe(fe& f, const uint32_t* p) {
#pragma unroll
  for (int i = 0; i < 10; ++i) f.v[i] = p[i * S];
}
template <int S = 1>
PV_HD void store_cached(uint32_t* p, const ge_cached& c) {
  store_fe<S>(p, c.YpX);
  store_fe<S>(p + 10 * S, c.YmX);
  store_fe<S>(p + 20 * S, c.Z2);
  store_fe<S>(p + 30 * S, c.T2d);
}
template <int S = 1>
PV_HD void load_cached(ge_cached& c, const uint32_t* p) {
  load_fe<S>(c.YpX, p);
  load_fe<S>(c.YmX, p + 10 * S);
  load_fe<S>(c.Z2, p + 20 * S);
  load_fe<S>(c.T2d, p + 30 * S);
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

// niels form of k * 2^(32 q) * B (k <= 255, q = 0..7), written as 32 words.
// Table q = 0 serves the generic kernels (q = 4, 2^128 B, the half-size one);
// the comb kernel of prepared keys uses all eight (B_q = 2^(32 q) B, so
// S*B = sum_q S_q B_q with the 32-bit words S_q).
PV_HD void btable_entry(uint32_t* p, int k, int q = 0, int nbits = 8) {
  ge_p3 B, acc;
  ge_basepoint(B);
#pragma unroll 1
  for (int d = 0; d < 32 * q; ++d) {
    ge_p1p1 t;
    ge_p3_dbl(t, B);
    ge_p1p1_to_p3(B, t);
  }
  ge_cached cb;
  ge_p3_to_cached(cb, B);
  ge_p3_0(acc);
  for (int bit = nbits - 1; bit >= 0; --bit) {
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

// ------------------------------------------- table-operand point additions
// r = p + s*Q with Q read straight from a table entry (`q`), one field element
// at a time right before the multiply that consumes it.  The sign is applied
// by choosing WHICH of Y+X / Y-X to load and negating the C term, so no
// 10-limb copies are made: this keeps the hot loop inside 3 waves/SIMD of
// registers.  Same formulas as ge_add_cached / ge_madd (add-2008-hwcd-3).
template <int S = 1>
PV_HD void ge_add_cached_at(ge_p1p1& r, const ge_p3& p, const uint32_t* q, bool neg) {
  fe c, d, a, b, u, g;
  load_fe<S>(g, q + 30 * S);             // 2d*T2
  fe_mul(c, g, p.T);
  load_fe<S>(g, q + 20 * S);             // 2*Z2
  fe_mul(d, p.Z, g);
  fe_add(u, p.Y, p.X);
  load_fe<S>(g, q + (neg ? 10 * S : 0)); // Y2+X2 (Y2-X2 for -Q)
  fe_mul(a, u, g);
  fe_sub(u, p.Y, p.X);
  load_fe<S>(g, q + (neg ? 0 : 10 * S));
  fe_mul(b, u, g);
  fe_sub(r.X, a, b);
  fe_add(r.Y, a, b);
  fe_neg(u, c);                   // -Q: C -> -C
  fe_cmov(c, c, u, neg);
  fe_add(r.Z, d, c);
  fe_sub(r.T, d, c);
}

PV_HD void ge_madd_at(ge_p1p1& r, const ge_p3& p, const uint32_t* q, bool neg) {
  fe c, d, a, b, u, g;
  load_fe(g, q + 20);             // 2d*x2*y2
  fe_mul(c, g, p.T);
  fe_add(d, p.Z, p.Z);
  fe_carry(d);
  fe_add(u, p.Y, p.X);
  load_fe(g, q + (neg ? 10 : 0)); // y2+x2 (y2-x2 for -Q)
  fe_mul(a, u, g);
  fe_sub(u, p.Y, p.X);
  load_fe(g, q + (neg ? 0 : 10));
  fe_mul(b, u, g);
  fe_sub(r.X, a, b);
  fe_add(r.Y, a, b);
  fe_neg(u, c);
  fe_cmov(c, c, u, neg);
  fe_add(r.Z, d, c);
  fe_sub(r.T, d, c);
}

// Register-operand form of ge_add_cached_at for software-pipelined table
// reads: the entry is fetched (already sign-swapped) into registers well
// before the add that consumes it, so its global-memory latency runs under
// the doublings / the previous add instead of stalling the wave.
struct ge_entry { fe a, b, z2, t2d; };

template <int S = 1>
PV_HD void load_entry(ge_entry& e, const uint32_t* q, bool neg) {
  load_fe<S>(e.a, q + (neg ? 10 * S : 0));   // Y2+X2 (Y2-X2 for -Q)
  load_fe<S>(e.b, q + (neg ? 0 : 10 * S));
  load_fe<S>(e.z2, q + 20 * S);
  load_fe<S>(e.t2d, q + 30 * S);
}

// same operation sequence (and operand bounds) as ge_add_cached_at
PV_HD void ge_add_entry(ge_p1p1& r, const ge_p3& p, const ge_entry& e, bool neg) {
  fe c, d, a, b, u, v;
#if PV_FUSE & 4
  fe_mul2(c, e.t2d, p.T, d, p.Z, e.z2);
  fe_add(u, p.Y, p.X);
  fe_sub(v, p.Y, p.X);
#if PV_FUSE & 4
  fe_mul2(a, u, e.a, b, v, e.b);
#else
  fe_mul(a, u, e.a);
  fe_mul(b, v, e.b);
#endif
#else
  fe_mul(c, e.t2d, p.T);
  fe_mul(d, p.Z, e.z2);
  fe_add(u, p.Y, p.X);
  fe_mul(a, u, e.a);
  fe_sub(v, p.Y, p.X);
  fe_mul(b, v, e.b);
#endif
  fe_sub(r.X, a, b);
  fe_add(r.Y, a, b);
  fe_neg(u, c);
  fe_cmov(c, c, u, neg);
  fe_add(r.Z, d, c);
  fe_sub(r.T, d, c);
}

// affine (niels) entry in registers, sign-swapped at load: same operation
// sequence and bounds as ge_madd_at
struct ge_nentry { fe a, b, c; };

PV_HD void load_nentry(ge_nentry& e, const uint32_t* q, bool neg) {
  load_fe(e.a, q + (neg ? 10 : 0));   // y2+x2 (y2-x2 for -Q)
  load_fe(e.b, q + (neg ? 0 : 10));
  load_fe(e.c, q + 20);               // 2d*x2*y2
}

PV_HD void ge_madd_entry(ge_p1p1& r, const ge_p3& p, const ge_nentry& e, bool neg) {
  fe c, d, a, b, u, v;
  fe_mul(c, e.c, p.T);
  fe_add(d, p.Z, p.Z);
  fe_carry(d);
  fe_add(u, p.Y, p.X);
  fe_sub(v, p.Y, p.X);
#if PV_FUSE & 4
  fe_mul2(a, u, e.a, b, v, e.b);
#else
  fe_mul(a, u, e.a);
  fe_mul(b, v, e.b);
#endif
  fe_sub(r.X, a, b);
  fe_add(r.Y, a, b);
  fe_neg(u, c);
  fe_cmov(c, c, u, neg);
  fe_add(r.Z, d, c);
  fe_sub(r.T, d, c);
}

// ----------------------------------------------------------------- curve
// cached multiples 0..8 of P into a per-lane table (9 x 40 words)
template <int LS = 1>
PV_HD void build_atab(uint32_t* atab, const ge_p3& P) {
  ge_cached c;
  ge_cached_identity(c);
  store_cached<LS>(atab, c);
  ge_p3_to_cached(c, P);
  store_cached<LS>(atab + AT_ENTRY * LS, c);
  ge_p3 prev = P;
#pragma unroll 1
  for (int k = 2; k <= 8; ++k) {
    // re-read 1*P from the table instead of keeping it live (register budget)
    ge_cached c1;
    load_cached<LS>(c1, atab + AT_ENTRY * LS);
    ge_p1p1 t;
    ge_add_cached(t, prev, c1, false);
    ge_p1p1_to_p3(prev, t);
    ge_p3_to_cached(c, prev);
    store_cached<LS>(atab + AT_ENTRY * k * LS, c);
  }
}

// R' = hh*(-A) + ss*B.  hh + 0x88..88 gives radix-16 digits (nibble - 8) in
// [-8, 8); ss + 0x8080..80 gives radix-256 digits (byte - 128) in [-128, 128);
// hh, ss < 2^253 so neither addition overflows 2^256.  Horner from the top:
// per window 4 doublings, one A add, and a B add on even windows.
template <int LS = 1>
PV_HD void double_scalarmult(ge_p2& out, const uint32_t hh[8], const uint32_t ss[8], const uint32_t* atab,
                             const uint32_t* btab) {
  uint32_t hp[8], sp[8];
  sc_add_pattern(hp, hh, 0x88888888u);
  sc_add_pattern(sp, ss, 0x80808080u);
  ge_p3 acc;
  ge_p3_0(acc);
  ge_p1p1 t;
  ge_p2 r2;
  // Digits are consumed from the top word down.  The current words sit in
  // hw/sw; at each 8-window boundary the arrays shift by one word with static
  // indices only (a wave-uniform dynamic index would make the compiler spill
  // hp/sp to scratch).
  uint32_t hw = hp[7], sw = sp[7];
  {
    const int dA = (int)(hw >> 28) - 8;
    ge_add_cached_at<LS>(t, acc, atab + (dA < 0 ? -dA : dA) * AT_ENTRY * LS, dA < 0);
    ge_p1p1_to_p2(r2, t);
  }
#pragma unroll 1
  for (int i = 62; i >= 0; --i) {
    if ((i & 7) == 7) {
#pragma unroll
      for (int k = 7; k > 0; --k) {
        hp[k] = hp[k - 1];
        sp[k] = sp[k - 1];
      }
      hw = hp[7];
      sw = sp[7];
    }
#pragma unroll 1
    for (int k = 0; k < 3; ++k) {
      ge_p2_dbl(t, r2);
      ge_p1p1_to_p2(r2, t);
    }
    ge_p2_dbl(t, r2);
    ge_p1p1_to_p3(acc, t);
    const int dA = (int)((hw >> (4 * (i & 7))) & 15u) - 8;
    ge_add_cached_at<LS>(t, acc, atab + (dA < 0 ? -dA : dA) * AT_ENTRY * LS, dA < 0);
    if ((i & 1) == 0) {
      const int dB = (int)((sw >> (8 * ((i >> 1) & 3))) & 255u) - 128;
      ge_p1p1_to_p3(acc, t);
      ge_madd_at(t, acc, btab + (dB < 0 ? -dB : dB) * BT_WORDS, dB < 0);
    }
    ge_p1p1_to_p2(r2, t);
  }
  out = r2;
}

// decompress A and compute R' = h(-A) + S B (projective, not yet encoded).
// `atab` is this lane's table scratch; `btab` the base-point table (LDS in the
// kernel).  Inputs are loaded right where they are consumed so that no
// 32-byte value stays live across the whole verification (register budget of
// the hot loop).  false = rejected before the final comparison.
template <int LS = 1>
PV_HD bool curve_point(ge_p2& rp, const uint8_t* pk, const uint8_t* sig, const uint32_t* dig_src, uint32_t* atab,
                       const uint32_t* btab) {
  ge_p3 negA;
  {
    uint32_t A[8];
    load8(A, pk);
    if (!ge_frombytes_negate(negA, A)) return false;
  }
  build_atab<LS>(atab, negA);
  uint32_t hh[8], S[8];
  {
    uint32_t dig[16];
    load8(dig, reinterpret_cast<const uint8_t*>(dig_src));
    load8(dig + 8, reinterpret_cast<const uint8_t*>(dig_src + 8));
    sc_reduce64(hh, dig);  // h = SHA-512(R||A||M) mod L (App. C.2 step 5)
  }
  load8(S, sig + 32);
  double_scalarmult<LS>(rp, hh, S, atab, btab);
  return true;
}

// ------------------------------------------------------------- key cache
// A verifying key prepared once and shared by every signature under it, as an
// 8-way comb over the 32-bit words of the scalar: A_q = 2^(32 q) * (-A) for
// q = 0..7, each with its 9 multiples k * A_q (k = 0..8) in AFFINE niels form
// (y+x, y-x, 2dxy; 32 words per entry, all 64 non-trivial points normalised
// with one shared inversion).  With the base-point tables B_q = 2^(32 q) B,
//   h*(-A) = sum_q h_q A_q,   S*B = sum_q S_q B_q   (h_q, S_q = word q)
// and the double-scalar multiplication needs 28 doublings instead of 253 (the
// 4-way comb of 64-bit quarters needed 60).  The group element
// R' = h(-A) + S B is the same, so the verdict (encode(R') == R) is
// bit-identical.  Status word: 1 = A canonical,
// not small order, decompresses (steps 2-4).
constexpr int COMB_Q = 8;
constexpr int BT_CHUNKS = 8;            // base-point tables 2^(32 q) B, q = 0..7
constexpr int BT_TABLE = BT_ENTRIES * BT_WORDS;
// s' = d S mod L in the curve stage: signed radix-2^16 digits in offset form
// (+0x8000 per 16-bit digit, one 256-bit add: the carry out of the low 128
// bits lands in the high half), digit i of the low half from the table of B,
// of the high half from the table of 2^128 B, both with 2^15 + 1 affine
// entries k * P.  The device holds BW_CHUNKS such tables, k * 2^(32 q) * B for
// q = 0..7 (33.5 MB, read from L2/MALL): chunks 0 and 4 serve the half-size
// path, all eight the comb of prepared keys.
constexpr uint32_t HALF_S_PATTERN = 0x80008000u;
constexpr int BW_ENTRIES = (1 << 15) + 1;
constexpr int BW_TABLE = BW_ENTRIES * BT_WORDS;
constexpr int BW_CHUNKS = 8;
constexpr int KT_ENTRY = 32;
constexpr int KT_TABLE = 9 * KT_ENTRY;
constexpr int KEY_STATUS = COMB_Q * KT_TABLE;
constexpr int KEY_WORDS = KEY_STATUS + 32;   // status word + padding: every key starts on a 128-byte line
// per-key scratch: the projective entries (X, Y, Z of the 8 * COMB_Q multiples)
// and the prefix products of their shared inversion.  Private to key_prepare,
// so k_keys lays it out lane-interleaved ([word][lane] per 64 keys: every
// scratch load and store of a wave is one contiguous 256-byte row); only the
// final affine entries go to the key-major table the curve kernel reads.
// PV_KEYS_XYP = 1 (A/B): the prefix products folded into X and Y, see key_prepare
#ifndef PV_KEYS_XYP
#define PV_KEYS_XYP 0
#endif
constexpr int KS_XYZ = 0;
constexpr int KS_PREFIX = 8 * COMB_Q * 30;
constexpr int KEY_SCRATCH = KS_PREFIX + 8 * COMB_Q * 10;

PV_HD void store_xyz(uint32_t* p, const ge_p3& q) {
  store_fe(p, q.X);
  store_fe(p + 10, q.Y);
  store_fe(p + 20, q.Z);
}

// one 32-word affine entry (a, b, c at words 0, 10, 20; words 30-31 zero) as
// eight 16-byte stores: the table is key-major, so each store instruction of a
// wave touches 64 cache lines -- 8 wide stores instead of 30 narrow ones
PV_HD void store_entry32(uint32_t* slot, const fe& a, const fe& b, const fe& c) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t w[32];
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    w[i] = a.v[i];
    w[10 + i] = b.v[i];
    w[20 + i] = c.v[i];
  }
  w[30] = w[31] = 0;
  uint4* d = reinterpret_cast<uint4*>(slot);
#pragma unroll
  for (int i = 0; i < 8; ++i) d[i] = make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]);
#else
  store_fe(slot, a);
  store_fe(slot + 10, b);
  store_fe(slot + 20, c);
  slot[30] = slot[31] = 0;
#endif
}

// kt: KEY_WORDS words (key-major); scr: KEY_SCRATCH words of this key's
// scratch, word w at scr[w * LS] (LS = 64 on the device: lane-interleaved)
template <int LS = 1>
PV_HD void key_prepare(uint32_t* kt, uint32_t* scr, const uint8_t* pk) {
  uint32_t A[8];
  load8(A, pk);
  ge_p3 P;
  const bool ok = y_is_canonical(A) && !has_small_order(A) && ge_frombytes_negate(P, A);
  // (only the words the comb reads are written: entries' words 30-31 and the
  // words after the status are padding)
  kt[KEY_STATUS] = ok ? 1u : 0u;
  if (!ok) return;
  // projective multiples k * A_q (X, Y, Z) into the scratch, entry e = 8 q + k - 1
  auto xyz = [&](int e) { return scr + (KS_XYZ + 30 * e) * LS; };
  auto pre = [&](int e) { return scr + (KS_PREFIX + 10 * e) * LS; };
  fe zacc;
#pragma unroll 1
  for (int q = 0; q < COMB_Q; ++q) {
    ge_cached c1;
    ge_p3_to_cached(c1, P);
    ge_p3 Q = P;
#if PV_KEYS_XYP
    // (A/B) X P_(e-1), Y P_(e-1), Z per entry: 30 scratch words instead of
    // 40, one more multiply per entry (backward: x = X' acc, y = Y' acc)
    auto put = [&](int e, const ge_p3& R) {
      if (e == 0) {
        store_fe<LS>(xyz(e), R.X);
        store_fe<LS>(xyz(e) + 10 * LS, R.Y);
        fe_copy(zacc, R.Z);
      } else {
        fe t;
        fe_mul(t, R.X, zacc);
        store_fe<LS>(xyz(e), t);
        fe_mul(t, R.Y, zacc);
        store_fe<LS>(xyz(e) + 10 * LS, t);
        fe_mul(zacc, zacc, R.Z);
      }
      store_fe<LS>(xyz(e) + 20 * LS, R.Z);
    };
    put(8 * q, Q);
#pragma unroll 1
    for (int k = 2; k <= 8; ++k) {
      ge_p1p1 t;
      ge_add_cached(t, Q, c1, false);
      ge_p1p1_to_p3(Q, t);
      put(8 * q + k - 1, Q);
    }
#else
    store_fe<LS>(xyz(8 * q), Q.X);
    store_fe<LS>(xyz(8 * q) + 10 * LS, Q.Y);
    store_fe<LS>(xyz(8 * q) + 20 * LS, Q.Z);
    // prefix products of the Z's for the shared inversion, formed while each
    // Z is in registers
    if (q == 0) fe_copy(zacc, Q.Z);
    else fe_mul(zacc, zacc, Q.Z);
    store_fe<LS>(pre(8 * q), zacc);
#pragma unroll 1
    for (int k = 2; k <= 8; ++k) {
      ge_p1p1 t;
      ge_add_cached(t, Q, c1, false);
      ge_p1p1_to_p3(Q, t);
      const int e = 8 * q + k - 1;
      store_fe<LS>(xyz(e), Q.X);
      store_fe<LS>(xyz(e) + 10 * LS, Q.Y);
      store_fe<LS>(xyz(e) + 20 * LS, Q.Z);
      fe_mul(zacc, zacc, Q.Z);
      store_fe<LS>(pre(e), zacc);
    }
#endif
    if (q + 1 < COMB_Q) {  // A_{q+1} = 2^32 A_q = 2^29 (8 A_q)
      ge_p1p1 t;
      ge_p2 r;
      fe_copy(r.X, Q.X);
      fe_copy(r.Y, Q.Y);
      fe_copy(r.Z, Q.Z);
#pragma unroll 1
      for (int d = 0; d < 28; ++d) {
        ge_p2_dbl(t, r);
        ge_p1p1_to_p2(r, t);
      }
      ge_p2_dbl(t, r);
      ge_p1p1_to_p3(P, t);
    }
  }
  // one inversion for all 8 * COMB_Q Z's (Montgomery's trick; prefix
  // products in scr).  Backward pass with the next entry's operands (X, Y, Z
  // of entry e - 1, prefix e - 2) fetched one iteration ahead.
  constexpr int NE = 8 * COMB_Q;
  fe acc, u, z, x, y, un, zn, xn, yn;
  fe_invert(acc, zacc);
  fe d2;
  fe_const_d2(d2);
#if !PV_KEYS_XYP
  load_fe<LS>(un, pre(NE - 2));
#endif
  load_fe<LS>(xn, xyz(NE - 1));
  load_fe<LS>(yn, xyz(NE - 1) + 10 * LS);
  load_fe<LS>(zn, xyz(NE - 1) + 20 * LS);
#pragma unroll 1
  for (int e = NE - 1; e >= 0; --e) {
    uint32_t* slot = kt + (e >> 3) * KT_TABLE + ((e & 7) + 1) * KT_ENTRY;
    fe_copy(u, un);
    fe_copy(z, zn);
    fe_copy(x, xn);
    fe_copy(y, yn);
    if (e > 0) {
#if !PV_KEYS_XYP
      if (e > 1) load_fe<LS>(un, pre(e - 2));
#endif
      load_fe<LS>(xn, xyz(e - 1));
      load_fe<LS>(yn, xyz(e - 1) + 10 * LS);
      load_fe<LS>(zn, xyz(e - 1) + 20 * LS);
    }
#if PV_KEYS_XYP
    // acc = (Z_0 ... Z_e)^-1 and X' = X P_(e-1): x = X' acc = X / Z_e
    fe_mul(x, x, acc);
    fe_mul(y, y, acc);
    if (e > 0) fe_mul(acc, acc, z);  // (Z_0 ... Z_{e-1})^-1
#else
    fe zi;
    if (e > 0) {
      fe_mul(zi, acc, u);            // Z_e^-1
      fe_mul(acc, acc, z);           // (Z_0 ... Z_{e-1})^-1
    } else {
      fe_copy(zi, acc);
    }
    fe_mul(x, x, zi);
    fe_mul(y, y, zi);
#endif
    fe ypx, ymx;
    fe_add(ypx, y, x); fe_carry(ypx);
    fe_sub(ymx, y, x); fe_carry(ymx);
    fe_mul(u, x, y);
    fe_mul(u, u, d2);
    store_entry32(slot, ypx, ymx, u);
  }
  // identity entries (k = 0): y+x = 1, y-x = 1, 2dxy = 0
  fe one, zero;
  fe_1(one);
  fe_0(zero);
#pragma unroll 1
  for (int q = 0; q < COMB_Q; ++q) store_entry32(kt + q * KT_TABLE, one, one, zero);
}

// R' = hh*(-A) + ss*B from a prepared key (8 comb tables in kt) and the eight
// radix-2^16 base-point chunk tables bw + q * BW_TABLE (k * 2^(32 q) * B).
// Windows w = 7..0 (4 doublings apart): per window one affine add per chunk q
// with the signed radix-16 digit 8q + w of hh, and on windows 4 and 0 one per
// chunk with the signed radix-2^16 digit 2q + w/4 of ss (16 base-point adds;
// radix 256 needed 32).  Every table entry is fetched one add ahead into
// ping-pong registers.  The chunk loops are not unrolled (code size); the
// digit words rotate through static indices.
//
// The 16 offset digit words (h, S) live in `dg` (word k at dg[k * DS]): the
// kernel passes a lane-interleaved LDS array (DS = the block size), so they
// hold no registers through the comb (the keyed kernel sits at 256 VGPRs);
// DS = 1 is a plain local array (host build).
template <int DS = 1>
PV_HD void double_scalarmult_comb(ge_p2& out, const uint32_t hh[8], const uint32_t ss[8], const uint32_t* kt,
                                  const uint32_t* bw, uint32_t* dg) {
  {
    uint32_t hp[8], sp[8];
    sc_add_pattern(hp, hh, 0x88888888u);
    sc_add_pattern(sp, ss, HALF_S_PATTERN);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      dg[k * DS] = hp[k];
      dg[(8 + k) * DS] = sp[k];
    }
  }
  ge_p3 acc;
  ge_p3_0(acc);
  ge_p1p1 t;
  ge_p2 r2;
  ge_nentry ea, eb;
  int dA = (int)((dg[0] >> 28) & 15u) - 8;
  load_nentry(ea, kt + (dA < 0 ? -dA : dA) * KT_ENTRY, dA < 0);
#pragma unroll 1
  for (int w = 7; w >= 0; --w) {
    if (w != 7) {
#pragma unroll 1
      for (int k = 0; k < 3; ++k) {
        ge_p2_dbl(t, r2);
        ge_p1p1_to_p2(r2, t);
      }
      ge_p2_dbl(t, r2);
      ge_p1p1_to_p3(acc, t);
    }
    const int sh4 = 4 * w;
    const bool bwin = (w & 3) == 0;
    // two key adds per trip, ping-ponging the register entries: the entry of
    // the next add (chunk q + 1; chunk 0 of window w - 1 after the last one)
    // is in flight during the current add
#pragma unroll 1
    for (int q = 0; q < COMB_Q; q += 2) {
      {
        const int dn = (int)((dg[(q + 1) * DS] >> sh4) & 15u) - 8;
        load_nentry(eb, kt + (q + 1) * KT_TABLE + (dn < 0 ? -dn : dn) * KT_ENTRY, dn < 0);
        ge_madd_entry(t, acc, ea, dA < 0);
        ge_p1p1_to_p3(acc, t);
        dA = dn;
      }
      {
        const bool last = q + 2 >= COMB_Q;
        const bool more = !last || w > 0;
        const int dn = (int)((dg[(last ? 0 : q + 2) * DS] >> ((last ? sh4 - 4 : sh4) & 31)) & 15u) - 8;
        if (more) load_nentry(ea, kt + (last ? 0 : q + 2) * KT_TABLE + (dn < 0 ? -dn : dn) * KT_ENTRY, dn < 0);
        ge_madd_entry(t, acc, eb, dA < 0);
        if (!last || bwin) ge_p1p1_to_p3(acc, t);
        else ge_p1p1_to_p2(r2, t);          // a doubling comes next: no T needed
        dA = dn;
      }
    }
    if (bwin) {
      const int sh16 = 4 * w;   // w = 4: high half of each word, w = 0: low half
      ge_nentry ba, bb;
      int db = (int)((dg[8 * DS] >> sh16) & 0xffffu) - 32768;
      load_nentry(ba, bw + (db < 0 ? -db : db) * BT_WORDS, db < 0);
#pragma unroll 1
      for (int q = 0; q < COMB_Q; q += 2) {
        const int d1 = (int)((dg[(8 + q + 1) * DS] >> sh16) & 0xffffu) - 32768;
        load_nentry(bb, bw + (q + 1) * BW_TABLE + (d1 < 0 ? -d1 : d1) * BT_WORDS, d1 < 0);
        ge_madd_entry(t, acc, ba, db < 0);
        ge_p1p1_to_p3(acc, t);
        const bool last = q + 2 >= COMB_Q;
        const int d2 = last ? 0 : (int)((dg[(8 + q + 2) * DS] >> sh16) & 0xffffu) - 32768;
        if (!last) load_nentry(ba, bw + (q + 2) * BW_TABLE + (d2 < 0 ? -d2 : d2) * BT_WORDS, d2 < 0);
        ge_madd_entry(t, acc, bb, d1 < 0);
        if (!last) ge_p1p1_to_p3(acc, t);
        else ge_p1p1_to_p2(r2, t);
        db = d2;
      }
    }
  }
  out = r2;
}

// ------------------------------------------------- wide comb (node keys)
// The same 8-way comb with radix-256 windows: table q holds k * A_q for
// k = 0..128 (129 affine entries, 132 KB per key), the signed digits are the
// bytes of h + 0x80..80 minus 128, and a verify needs 3 x 8 = 24 doublings
// and 32 key adds (+ the 16 base-point adds) instead of 28 and 64.  For keys
// that sign many messages per preparation -- a pool's node keys (C3) -- where
// the 16x larger preparation is amortised; the 9-entry format stays the
// default for key pools (C4) and the latency kernels.
constexpr int KW_ENT = 129;
constexpr int KW_TABLE = KW_ENT * KT_ENTRY;          // 4128 words
constexpr int KEYW_STATUS = COMB_Q * KW_TABLE;       // 33024
constexpr int KEYW_WORDS = KEYW_STATUS + 32;         // 132224 B per key (128-byte multiple)
// k_keys_wide spreads a table over KW_SLICES lanes: lane (q, s) builds the
// multiples k = KW_SLICE s + 1 .. KW_SLICE (s + 1) of A_q (its projective
// points and the prefix products of their shared inversion in scratch, word w
// at scr[w * LS]).  Every lane of a table redoes the 32 q doublings of A_q:
// the chain (224 doublings for q = 7) bounds the kernel's latency either way,
// and redoing it costs no barrier and no exchange between lanes.
constexpr int KW_SLICES = 16;
constexpr int KW_SLICE = 128 / KW_SLICES;            // 8 multiples per lane
constexpr int KWS_PREFIX = KW_SLICE * 30;
constexpr int KEYW_SCRATCH = KWS_PREFIX + KW_SLICE * 10;

PV_HD void ge_p3_cmov(ge_p3& h, const ge_p3& f, const ge_p3& g, bool c) {
  fe_cmov(h.X, f.X, g.X, c);
  fe_cmov(h.Y, f.Y, g.Y, c);
  fe_cmov(h.Z, f.Z, g.Z, c);
  fe_cmov(h.T, f.T, g.T, c);
}

// slice s of table q of a wide prepared key (kt = the key's KEYW_WORDS words);
// lane (0, 0) also writes the status word (1 = A canonical, not small order,
// decodes) and lane (q, 0) the identity entry k = 0 of table q
template <int LS = 1>
PV_HD void key_prepare_wide_slice(uint32_t* kt, uint32_t* scr, const uint8_t* pk, int q, int s) {
  uint32_t A[8];
  load8(A, pk);
  ge_p3 P;
  const bool ok = y_is_canonical(A) && !has_small_order(A) && ge_frombytes_negate(P, A);
  if (q == 0 && s == 0) kt[KEYW_STATUS] = ok ? 1u : 0u;
  if (!ok) return;
  ge_p1p1 t;
  if (q > 0) {   // A_q = 2^(32 q) (-A)
    ge_p2 r;
    fe_copy(r.X, P.X);
    fe_copy(r.Y, P.Y);
    fe_copy(r.Z, P.Z);
#pragma unroll 1
    for (int d = 0; d + 1 < 32 * q; ++d) {
      ge_p2_dbl(t, r);
      ge_p1p1_to_p2(r, t);
    }
    ge_p2_dbl(t, r);
    ge_p1p1_to_p3(P, t);
  }
  ge_cached c1;
  ge_p3_to_cached(c1, P);
  // Q = (KW_SLICE s + 1) A_q = s (8 A_q) + A_q: 4-bit ladder over s, MSB first
  // (the extended-coordinate formulas are complete: the identity and equal
  // operands need no special case)
  ge_p3 P8 = P, Q, T;
#pragma unroll 1
  for (int d = 0; d < 3; ++d) {
    ge_p3_dbl(t, P8);
    ge_p1p1_to_p3(P8, t);
  }
  ge_cached c8;
  ge_p3_to_cached(c8, P8);
  ge_p3_0(Q);
#pragma unroll 1
  for (int b = 3; b >= 0; --b) {
    ge_p3_dbl(t, Q);
    ge_p1p1_to_p3(Q, t);
    ge_add_cached(t, Q, c8, false);
    ge_p1p1_to_p3(T, t);
    ge_p3_cmov(Q, Q, T, (s >> b) & 1);
  }
  ge_add_cached(t, Q, c1, false);
  ge_p1p1_to_p3(Q, t);
  auto xyz = [&](int e) { return scr + 30 * e * LS; };
  auto pre = [&](int e) { return scr + (KWS_PREFIX + 10 * e) * LS; };
  store_fe<LS>(xyz(0), Q.X);
  store_fe<LS>(xyz(0) + 10 * LS, Q.Y);
  store_fe<LS>(xyz(0) + 20 * LS, Q.Z);
  fe zacc;
  fe_copy(zacc, Q.Z);
  store_fe<LS>(pre(0), zacc);
#pragma unroll 1
  for (int e = 1; e < KW_SLICE; ++e) {   // entry e = (KW_SLICE s + e + 1) A_q
    ge_add_cached(t, Q, c1, false);
    ge_p1p1_to_p3(Q, t);
    store_fe<LS>(xyz(e), Q.X);
    store_fe<LS>(xyz(e) + 10 * LS, Q.Y);
    store_fe<LS>(xyz(e) + 20 * LS, Q.Z);
    fe_mul(zacc, zacc, Q.Z);
    store_fe<LS>(pre(e), zacc);
  }
  // one inversion for the slice's Z's, backward pass (key_prepare's)
  uint32_t* tab = kt + q * KW_TABLE + (KW_SLICE * s + 1) * KT_ENTRY;
  fe acc, u, z, x, y, d2;
  fe_invert(acc, zacc);
  fe_const_d2(d2);
#pragma unroll 1
  for (int e = KW_SLICE - 1; e >= 0; --e) {
    load_fe<LS>(x, xyz(e));
    load_fe<LS>(y, xyz(e) + 10 * LS);
    fe zi;
    if (e > 0) {
      load_fe<LS>(u, pre(e - 1));
      load_fe<LS>(z, xyz(e) + 20 * LS);
      fe_mul(zi, acc, u);            // Z_e^-1
      fe_mul(acc, acc, z);           // (Z_0 ... Z_{e-1})^-1
    } else {
      fe_copy(zi, acc);
    }
    fe_mul(x, x, zi);
    fe_mul(y, y, zi);
    fe ypx, ymx;
    fe_add(ypx, y, x); fe_carry(ypx);
    fe_sub(ymx, y, x); fe_carry(ymx);
    fe_mul(u, x, y);
    fe_mul(u, u, d2);
    store_entry32(tab + e * KT_ENTRY, ypx, ymx, u);
  }
  if (s == 0) {
    fe one, zero;
    fe_1(one);
    fe_0(zero);
    store_entry32(kt + q * KW_TABLE, one, one, zero);   // k = 0: the identity
  }
}

// R' = hh (-A) + ss B from a wide prepared key: windows w = 3..0 (bytes), 8
// doublings apart; per window one affine add per table q with the signed
// digit of byte w of word q, and on windows 2 and 0 the radix-2^16 base-point
// digits of ss (high / low halves) as in double_scalarmult_comb.  Entries are
// fetched one add ahead; the digit words live in dg (word k at dg[k * DS]).
template <int DS = 1>
PV_HD void double_scalarmult_comb_wide(ge_p2& out, const uint32_t hh[8], const uint32_t ss[8], const uint32_t* kt,
                                       const uint32_t* bw, uint32_t* dg) {
  {
    uint32_t hp[8], sp[8];
    sc_add_pattern(hp, hh, 0x80808080u);
    sc_add_pattern(sp, ss, HALF_S_PATTERN);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      dg[k * DS] = hp[k];
      dg[(8 + k) * DS] = sp[k];
    }
  }
  ge_p3 acc;
  ge_p3_0(acc);
  ge_p1p1 t;
  ge_p2 r2;
  ge_nentry ea, eb;
  int dA = (int)((dg[0] >> 24) & 255u) - 128;
  load_nentry(ea, kt + (dA < 0 ? -dA : dA) * KT_ENTRY, dA < 0);
#pragma unroll 1
  for (int w = 3; w >= 0; --w) {
    if (w != 3) {
#pragma unroll 1
      for (int k = 0; k < 7; ++k) {
        ge_p2_dbl(t, r2);
        ge_p1p1_to_p2(r2, t);
      }
      ge_p2_dbl(t, r2);
      ge_p1p1_to_p3(acc, t);
    }
    const int sh8 = 8 * w;
    const bool bwin = (w & 1) == 0;
#pragma unroll 1
    for (int q = 0; q < COMB_Q; q += 2) {
      {
        const int dn = (int)((dg[(q + 1) * DS] >> sh8) & 255u) - 128;
        load_nentry(eb, kt + (q + 1) * KW_TABLE + (dn < 0 ? -dn : dn) * KT_ENTRY, dn < 0);
        ge_madd_entry(t, acc, ea, dA < 0);
        ge_p1p1_to_p3(acc, t);
        dA = dn;
      }
      {
        const bool last = q + 2 >= COMB_Q;
        const bool more = !last || w > 0;
        const int dn = (int)((dg[(last ? 0 : q + 2) * DS] >> ((last ? sh8 - 8 : sh8) & 31)) & 255u) - 128;
        if (more) load_nentry(ea, kt + (last ? 0 : q + 2) * KW_TABLE + (dn < 0 ? -dn : dn) * KT_ENTRY, dn < 0);
        ge_madd_entry(t, acc, eb, dA < 0);
        if (!last || bwin) ge_p1p1_to_p3(acc, t);
        else ge_p1p1_to_p2(r2, t);          // a doubling comes next: no T needed
        dA = dn;
      }
    }
    if (bwin) {
      const int sh16 = 8 * w;   // w = 2: high half of each word, w = 0: low half
      ge_nentry ba, bb;
      int db = (int)((dg[8 * DS] >> sh16) & 0xffffu) - 32768;
      load_nentry(ba, bw + (db < 0 ? -db : db) * BT_WORDS, db < 0);
#pragma unroll 1
      for (int q = 0; q < COMB_Q; q += 2) {
        const int d1 = (int)((dg[(8 + q + 1) * DS] >> sh16) & 0xffffu) - 32768;
        load_nentry(bb, bw + (q + 1) * BW_TABLE + (d1 < 0 ? -d1 : d1) * BT_WORDS, d1 < 0);
        ge_madd_entry(t, acc, ba, db < 0);
        ge_p1p1_to_p3(acc, t);
        const bool last = q + 2 >= COMB_Q;
        const int d2 = last ? 0 : (int)((dg[(8 + q + 2) * DS] >> sh16) & 0xffffu) - 32768;
        if (!last) load_nentry(ba, bw + (q + 2) * BW_TABLE + (d2 < 0 ? -d2 : d2) * BT_WORDS, d2 < 0);
        ge_madd_entry(t, acc, bb, d1 < 0);
        if (!last) ge_p1p1_to_p3(acc, t);
        else ge_p1p1_to_p2(r2, t);
        db = d2;
      }
    }
  }
  out = r2;
}

// key formats of prepared keys: 0 = the 9-entry comb (KEY_WORDS), 1 = wide (KEYW_WORDS)
template <int KF>
PV_HD constexpr int key_words() { return KF ? KEYW_WORDS : KEY_WORDS; }

// R' = h(-A) + S B with -A's comb tables taken from a prepared key
template <int DS = 1, int KF = 0>
PV_HD bool curve_point_keyed(ge_p2& rp, const uint32_t* kt, const uint8_t* sig, const uint32_t* dig_src,
                             const uint32_t* bw, uint32_t* dg) {
  if (!kt[KF ? KEYW_STATUS : KEY_STATUS]) return false;
  uint32_t hh[8], S[8];
  {
    uint32_t dig[16];
    load8(dig, reinterpret_cast<const uint8_t*>(dig_src));
    load8(dig + 8, reinterpret_cast<const uint8_t*>(dig_src + 8));
    sc_reduce64(hh, dig);
  }
  load8(S, sig + 32);
  if constexpr (KF != 0) double_scalarmult_comb_wide<DS>(rp, hh, S, kt, bw, dg);
  else double_scalarmult_comb<DS>(rp, hh, S, kt, bw, dg);
  return true;
}

// Signatures one lane finishes together: their final Z^-1 share ONE field
// inversion (Montgomery's trick: 3(K-1) multiplies + 1 inversion instead of
// K inversions).
#ifndef PV_CURVE_K
#define PV_CURVE_K 8
#endif
constexpr int CURVE_K = PV_CURVE_K;
constexpr int PT_WORDS = 40;                        // X, Y, Z, prefix product
constexpr int LANE_WORDS = AT_WORDS + CURVE_K * PT_WORDS;

// in place over K entries of (X, Y, Z, P): Z_k <- Z_k^-1 (all Z_k != 0)
PV_HD void batch_invert_z(uint32_t* pts, int K) {
  fe acc, z, t;
  load_fe(acc, pts + 20);
  store_fe(pts + 30, acc);
#pragma unroll 1
  for (int k = 1; k < K; ++k) {
    load_fe(z, pts + PT_WORDS * k + 20);
    fe_mul(acc, acc, z);
    store_fe(pts + PT_WORDS * k + 30, acc);
  }
  fe_invert(acc, acc);                              // (Z_0 ... Z_{K-1})^-1
#pragma unroll 1
  for (int k = K - 1; k > 0; --k) {
    load_fe(t, pts + PT_WORDS * (k - 1) + 30);      // Z_0 ... Z_{k-1}
    load_fe(z, pts + PT_WORDS * k + 20);
    fe_mul(t, acc, t);                              // Z_k^-1
    fe_mul(acc, acc, z);                            // (Z_0 ... Z_{k-1})^-1
    store_fe(pts + PT_WORDS * k + 20, t);
  }
  store_fe(pts + 20, acc);
}

// One lane's group of CURVE_K signatures i0, i0 + stride, ...: returns the
// accepted bitmask.  Rejected or absent entries carry Z = 1 through the
// shared inversion.  scratch = LANE_WORDS words owned by this lane.
// KEYED: signature i uses prepared key kidx[i] (comb tables in ktab; btab
// then holds the even chunk tables 0, 2, 4, 6 and bg all eight).
template <bool KEYED, int DS = 1, int KF = 0>
PV_HD uint32_t curve_group(const uint8_t* pk, const uint8_t* sig, const uint32_t* h, const uint8_t* pre, uint64_t i0,
                           uint64_t stride, uint64_t n, uint32_t* scratch, const uint32_t* btab,
                           const uint32_t* ktab = nullptr, const uint32_t* kidx = nullptr,
                           const uint32_t* bg = nullptr, uint32_t* dg = nullptr) {
  uint32_t dloc[DS == 1 ? 16 : 1];   // host build: the comb's digit words
  if (DS == 1) dg = dloc;
  uint32_t* pts = scratch + AT_WORDS;
  uint32_t live = 0;
#pragma unroll 1
  for (int k = 0; k < CURVE_K; ++k) {
    const uint64_t i = i0 + (uint64_t)k * stride;
    ge_p2 rp;
    bool ok = false;
    if (i < n && pre[i]) {
      if constexpr (KEYED)
        ok = curve_point_keyed<DS, KF>(rp, ktab + (uint64_t)kidx[i] * key_words<KF>(), sig + 64 * i, h + 16 * i, bg,
                                       dg);
      else
        ok = curve_point(rp, pk + 32 * i, sig + 64 * i, h + 16 * i, scratch, btab);
    }
    if (!ok) {
      fe_0(rp.X);
      fe_0(rp.Y);
      fe_1(rp.Z);
    }
    store_fe(pts + PT_WORDS * k, rp.X);
    store_fe(pts + PT_WORDS * k + 10, rp.Y);
    store_fe(pts + PT_WORDS * k + 20, rp.Z);
    live |= (ok ? 1u : 0u) << k;
  }
  batch_invert_z(pts, CURVE_K);
  uint32_t accepted = 0;
#pragma unroll 1
  for (int k = 0; k < CURVE_K; ++k) {
    if (!((live >> k) & 1u)) continue;
    const uint64_t i = i0 + (uint64_t)k * stride;
    fe zi, x, y;
    load_fe(zi, pts + PT_WORDS * k + 20);
    load_fe(x, pts + PT_WORDS * k);
    fe_mul(x, x, zi);
    load_fe(y, pts + PT_WORDS * k + 10);
    fe_mul(y, y, zi);
    uint32_t enc[8], R[8];
    fe_tobytes_w(enc, y);
    enc[7] ^= fe_isnegative(x) << 31;
    load8(R, sig + 64 * i);
    uint32_t diff = 0;
#pragma unroll
    for (int w = 0; w < 8; ++w) diff |= enc[w] ^ R[w];
    accepted |= (diff == 0 ? 1u : 0u) << k;
  }
  return accepted;
}

// ------------------------------------------------- half-size scalar path
// Per-signature record written by the lattice stage (k_lattice) and read by
// the curve stage: |c|, d in their signed-digit offset form (33 nibbles),
// s' = d S mod L in radix-256 offset form, and a status word
// (HS_NONE: rejected before the curve, HS_HALF, HS_DEFER) | c_neg << 8.
constexpr int HREC_WORDS = 20;
constexpr int HREC_C = 0, HREC_D = 5, HREC_S = 10, HREC_FLAGS = 18;
constexpr int HREC_H = 0;   // deferred records: h's 64 offset nibbles over words 0..7 (S at HREC_S)
constexpr int HALF_LANE_WORDS = 2 * AT_WORDS;   // tables of +-A and -R

// pre = the hash stage's pre-check verdict; dig = SHA-512(R||A||M)
PV_HD uint32_t lattice_one(uint32_t* rec, bool pre, const uint32_t* dig, const uint8_t* sig, bool force_full) {
  uint32_t st = HS_NONE;
  bool c_neg = false;
  if (pre) {
    st = HS_DEFER;
    uint32_t h[8];
    {
      uint32_t x[16];
      load8(x, reinterpret_cast<const uint8_t*>(dig));
      load8(x + 8, reinterpret_cast<const uint8_t*>(dig + 8));
      sc_reduce64(h, x);  // h = SHA-512(R||A||M) mod L (App. C.2 step 5)
    }
    if (!force_full) {
      uint32_t c[HS_WORDS], d[HS_WORDS];
      st = half_scalars(c, d, c_neg, h);
      if (st == HS_HALF) {
        uint32_t S[8], sp[8];
        load8(S, sig + 32);
        sc_mul_small(sp, d, S);
        sc_add_pattern(sp, sp, HALF_S_PATTERN);
        hs_offset(c);
        hs_offset(d);
#pragma unroll
        for (int k = 0; k < HS_WORDS; ++k) {
          rec[HREC_C + k] = c[k];
          rec[HREC_D + k] = d[k];
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) rec[HREC_S + k] = sp[k];
      }
    }
    if (st == HS_DEFER) {
      // full-length record (the lane-quad kernel's deferred form): h in signed
      // radix-16 offset form (64 nibbles over words 0..7) and S in the signed
      // radix-2^16 offset form of s'.  k_curve_half re-reads the digest instead.
      uint32_t S[8], hp[8];
      load8(S, sig + 32);
      sc_add_pattern(hp, h, 0x88888888u);
      sc_add_pattern(S, S, HALF_S_PATTERN);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        rec[HREC_H + k] = hp[k];
        rec[HREC_S + k] = S[k];
      }
    }
  }
  rec[HREC_FLAGS] = st | (c_neg ? 0x100u : 0u);
  return st;
}

// Q = s' B + c (+-A) + d (-R) over 33 radix-16 windows (c, d) with the
// signed radix-2^16 digits of s' split over the tables of B (low 128 bits)
// and 2^128 B (high 128 bits), both added on every fourth window (8 pairs of
// affine adds instead of 16 with radix 256).  Horner from the top: per window
// 4 doublings, one add from each per-lane table.  Leaves the last sum in
// p1p1 form.
template <int LS = 1>
PV_HD void msm_half(ge_p1p1& t, const uint32_t* rec, const uint32_t* atab, const uint32_t* rtab, const uint32_t* blo,
                    const uint32_t* bhi) {
  // digit words: the current group (windows 8g .. 8g + 7 of |c|, d and the
  // 16-bit digits of s' halves) in registers and the next lower group loaded
  // one group ahead from the record -- not all 16 words live through the loop
  // (register pressure: the kernel sits at 256 VGPRs)
  uint32_t cw = rec[HREC_C + 3], dw = rec[HREC_D + 3], lw = rec[HREC_S + 3], hw = rec[HREC_S + 7];
  uint32_t cn = rec[HREC_C + 2], dn = rec[HREC_D + 2], ln = rec[HREC_S + 2], hn = rec[HREC_S + 6];
  ge_p3 acc;
  ge_p2 r2;
  ge_p3_0(acc);
  {
    const int dA = (int)(rec[HREC_C + 4] & 15u) - 8;
    ge_add_cached_at<LS>(t, acc, atab + (dA < 0 ? -dA : dA) * AT_ENTRY * LS, dA < 0);
    ge_p1p1_to_p3(acc, t);
    const int dR = (int)(rec[HREC_D + 4] & 15u) - 8;
    ge_add_cached_at<LS>(t, acc, rtab + (dR < 0 ? -dR : dR) * AT_ENTRY * LS, dR < 0);
    ge_p1p1_to_p2(r2, t);
  }
#if PV_HALF_PREFETCH
  // software pipeline: the +-A entry of window w is loaded before its four
  // doublings, the -R entry before the +-A add
  ge_entry ea, er;
  int dA = (int)((cw >> 28) & 15u) - 8;
  load_entry<LS>(ea, atab + (dA < 0 ? -dA : dA) * AT_ENTRY * LS, dA < 0);
#endif
#pragma unroll 1
  for (int w = 31; w >= 0; --w) {
    if ((w & 7) == 7 && w != 31) {
      // next lower digit group; the one after it is fetched now
      cw = cn;
      dw = dn;
      lw = ln;
      hw = hn;
      const int g = (w >> 3) - 1;
      if (g >= 0) {
        cn = rec[HREC_C + g];
        dn = rec[HREC_D + g];
        ln = rec[HREC_S + g];
        hn = rec[HREC_S + 4 + g];
      }
    }
#pragma unroll 1
    for (int k = 0; k < 3; ++k) {
      ge_p2_dbl(t, r2);
      ge_p1p1_to_p2(r2, t);
    }
    ge_p2_dbl(t, r2);
    ge_p1p1_to_p3(acc, t);
    const int sh4 = 4 * (w & 7);
#if PV_HALF_PREFETCH
    const int dR = (int)((dw >> sh4) & 15u) - 8;
    load_entry<LS>(er, rtab + (dR < 0 ? -dR : dR) * AT_ENTRY * LS, dR < 0);
    ge_add_entry(t, acc, ea, dA < 0);
    ge_p1p1_to_p3(acc, t);
    // base-point windows (w % 4 == 0): 16-bit digit w / 4 of each half of s';
    // the low entry is in flight during the -R add, the high one during the
    // low madd
    const bool bwin = (w & 3) == 0;
    const int sh16 = 16 * ((w >> 2) & 1);
    const int dL = (int)((lw >> sh16) & 0xffffu) - 32768;
    const int dH = (int)((hw >> sh16) & 0xffffu) - 32768;
    ge_nentry eb;
    if (bwin) load_nentry(eb, blo + (dL < 0 ? -dL : dL) * BT_WORDS, dL < 0);
    ge_add_entry(t, acc, er, dR < 0);
    if (bwin) {
      ge_p1p1_to_p3(acc, t);
      ge_nentry ec;
      load_nentry(ec, bhi + (dH < 0 ? -dH : dH) * BT_WORDS, dH < 0);
      ge_madd_entry(t, acc, eb, dL < 0);
      ge_p1p1_to_p3(acc, t);
      ge_madd_entry(t, acc, ec, dH < 0);
    }
#else
    const int dA = (int)((cw >> sh4) & 15u) - 8;
    ge_add_cached_at<LS>(t, acc, atab + (dA < 0 ? -dA : dA) * AT_ENTRY * LS, dA < 0);
    ge_p1p1_to_p3(acc, t);
    const int dR = (int)((dw >> sh4) & 15u) - 8;
    ge_add_cached_at<LS>(t, acc, rtab + (dR < 0 ? -dR : dR) * AT_ENTRY * LS, dR < 0);
    if ((w & 3) == 0) {
      // base-point digits: 16-bit digit w / 4 of each half of s' (the
      // entries come from L2/MALL: each load is issued one step ahead)
      const int sh16 = 16 * ((w >> 2) & 1);
      const int dL = (int)((lw >> sh16) & 0xffffu) - 32768;
      const int dH = (int)((hw >> sh16) & 0xffffu) - 32768;
      ge_nentry eb;
      load_nentry(eb, blo + (dL < 0 ? -dL : dL) * BT_WORDS, dL < 0);
      ge_p1p1_to_p3(acc, t);
      ge_nentry ec;
      load_nentry(ec, bhi + (dH < 0 ? -dH : dH) * BT_WORDS, dH < 0);
      ge_madd_entry(t, acc, eb, dL < 0);
      ge_p1p1_to_p3(acc, t);
      ge_madd_entry(t, acc, ec, dH < 0);
    }
#endif
    if (w == 0) break;
#if PV_HALF_PREFETCH
    {
      // digit of window w - 1: its word is the next group's when w - 1 starts one
      const uint32_t nw = ((w - 1) & 7) == 7 ? cn : cw;
      dA = (int)((nw >> (4 * ((w - 1) & 7))) & 15u) - 8;
      load_entry<LS>(ea, atab + (dA < 0 ? -dA : dA) * AT_ENTRY * LS, dA < 0);
    }
#endif
    ge_p1p1_to_p2(r2, t);
  }
}

// p1p1 ((X:Z),(Y:T)) is the identity iff x = 0 and y = 1, i.e. X == 0 and Y == T
PV_HD bool p1p1_is_identity(const ge_p1p1& p) {
  fe u;
  fe_sub4(u, p.Y, p.T);
  fe_carry(u);
  return fe_iszero(p.X) && fe_iszero(u);
}

// The half-size verdict for a HS_HALF record (see pv_lattice.h):
// accept iff -A and -R decode and s' B + c (-A) + d (-R) == O.  R's y must be
// canonical (a non-canonical R never equals an encoding libsodium computes).
// scratch = HALF_LANE_WORDS words of this lane (word stride LS); blo/bhi =
// tables of B, 2^128 B.
template <int LS = 1>
PV_HD bool curve_half(const uint8_t* pk, const uint8_t* sig, const uint32_t* rec, uint32_t* scratch,
                      const uint32_t* blo, const uint32_t* bhi) {
  ge_p3 P;
  {
    uint32_t A[8];
    load8(A, pk);
    if (!ge_frombytes_negate(P, A)) return false;  // -A (A canonical: hash-stage pre-check)
  }
  if (rec[HREC_FLAGS] & 0x100u) {                // c < 0: c (-A) = |c| A
    fe_neg(P.X, P.X);
    fe_carry(P.X);
    fe_neg(P.T, P.T);
    fe_carry(P.T);
  }
  build_atab<LS>(scratch, P);
  {
    uint32_t R[8];
    load8(R, sig);
    if (!y_is_canonical(R) || !ge_frombytes_negate(P, R)) return false;  // -R
  }
  build_atab<LS>(scratch + AT_WORDS * LS, P);
  ge_p1p1 t;
  msm_half<LS>(t, rec, scratch, scratch + AT_WORDS * LS, blo, bhi);
  return p1p1_is_identity(t);
}

// ------------------------------------------------ latency mode (small batches)
// One signature on a lane PAIR (k_curve_lat): side 0 holds -A (+A when c < 0)
// and computes Q0 = |c| (+-A) + s'_lo B, side 1 holds -R and computes
// Q1 = d (-R) + s'_hi (2^128 B) -- each over its own 9-entry table and the
// same 33 radix-16 windows as msm_half -- and the pair then tests Q0 + Q1 == O.
// It is msm_half's sum regrouped, so the verdict is identical; the chain one
// lane runs shrinks from two decompressions, two tables and 66 + 16 adds to
// one decompression, one table and 33 + 8 adds (the 128 doublings remain).

// -A / +A (side 0, c's sign from the record) or -R (side 1, canonical y
// required); false = rejected
PV_HD bool side_point(ge_p3& P, const uint8_t* pk, const uint8_t* sig, const uint32_t* rec, int side) {
  uint32_t e[8];
  load8(e, side ? sig : pk);
  bool ok = side ? y_is_canonical(e) : true;
  ok = ok && ge_frombytes_negate(P, e);
  const bool flip = side == 0 && (rec[HREC_FLAGS] & 0x100u);  // c < 0: c (-A) = |c| A
  fe u;
  fe_neg(u, P.X);
  fe_carry(u);
  fe_cmov(P.X, P.X, u, flip);
  fe_neg(u, P.T);
  fe_carry(u);
  fe_cmov(P.T, P.T, u, flip);
  return ok;
}

// Horner over this side's digits: 33 windows of 4 doublings, one add from the
// lane's table per window, and on every fourth window one affine add with the
// side's 16-bit digit of s' (low half from the table of B, high half from
// 2^128 B).  Leaves the last sum in p1p1 form (same window schedule as msm_half).
template <int LS = 1>
PV_HD void msm_side(ge_p1p1& t, const uint32_t* rec, const uint32_t* tab, const uint32_t* bt, int side) {
  uint32_t dp[4], sp[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    dp[k] = side ? rec[HREC_D + k] : rec[HREC_C + k];
    sp[k] = rec[HREC_S + 4 * side + k];
  }
  ge_p3 acc;
  ge_p2 r2;
  ge_p3_0(acc);
  {
    const int d0 = (int)((side ? rec[HREC_D + 4] : rec[HREC_C + 4]) & 15u) - 8;
    ge_add_cached_at<LS>(t, acc, tab + (d0 < 0 ? -d0 : d0) * AT_ENTRY * LS, d0 < 0);
    ge_p1p1_to_p2(r2, t);
  }
  uint32_t dw = dp[3], sw = sp[3];
  ge_entry ea;
  int dA = (int)((dw >> 28) & 15u) - 8;
  load_entry<LS>(ea, tab + (dA < 0 ? -dA : dA) * AT_ENTRY * LS, dA < 0);
#pragma unroll 1
  for (int w = 31; w >= 0; --w) {
    if ((w & 7) == 7 && w != 31) {
#pragma unroll
      for (int k = 3; k > 0; --k) {
        dp[k] = dp[k - 1];
        sp[k] = sp[k - 1];
      }
      dw = dp[3];
      sw = sp[3];
    }
#pragma unroll 1
    for (int k = 0; k < 3; ++k) {
      ge_p2_dbl(t, r2);
      ge_p1p1_to_p2(r2, t);
    }
    ge_p2_dbl(t, r2);
    ge_p1p1_to_p3(acc, t);
    const bool bwin = (w & 3) == 0;
    const int sh16 = 16 * ((w >> 2) & 1);
    const int dB = (int)((sw >> sh16) & 0xffffu) - 32768;
    ge_nentry eb;
    if (bwin) load_nentry(eb, bt + (dB < 0 ? -dB : dB) * BT_WORDS, dB < 0);
    ge_add_entry(t, acc, ea, dA < 0);
    if (bwin) {
      ge_p1p1_to_p3(acc, t);
      ge_madd_entry(t, acc, eb, dB < 0);
    }
    if (w == 0) break;
    {
      const uint32_t nw = ((w - 1) & 7) == 7 ? dp[2] : dw;
      dA = (int)((nw >> (4 * ((w - 1) & 7))) & 15u) - 8;
      load_entry<LS>(ea, tab + (dA < 0 ? -dA : dA) * AT_ENTRY * LS, dA < 0);
    }
    ge_p1p1_to_p2(r2, t);
  }
}

// Full-length verdict of one signature (deferred records): R' = h(-A) + S B,
// encode, compare.  scratch = AT_WORDS words (stride LS); btab = table of B.
template <int LS = 1>
PV_HD bool verify_full_one(const uint8_t* pk, const uint8_t* sig, const uint32_t* dig, uint32_t* scratch,
                           const uint32_t* btab) {
  ge_p2 rp;
  if (!curve_point<LS>(rp, pk, sig, dig, scratch, btab)) return false;
  uint32_t enc[8], R[8];
  ge_p2_tobytes(enc, rp);
  load8(R, sig);
  uint32_t diff = 0;
#pragma unroll
  for (int w = 0; w < 8; ++w) diff |= enc[w] ^ R[w];
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
