// SHA-512 (FIPS 180-4) compression for one lane.  64-bit words are lowered by
// the compiler to 32-bit VALU pairs (v_alignbit_b32 for rotates, v_add_co /
// v_addc_co for adds).  The message schedule is a rolling 16-word window, so
// the state is 8 + 16 64-bit values per lane.
//
// Used for h = SHA-512(R || A || M), and by the
// batch signer for SHA-512(seed) and the nonce.
#pragma once
#include <stdint.h>
#include "pv_field.h"

#ifndef PV_SHA_ASM_ADD
#define PV_SHA_ASM_ADD 1
#endif

namespace pv {

// first 64 bits of the fractional parts of the cube roots of the first 80
// primes; device copy in constant memory (read with scalar loads: the round
// index is wave-uniform)
#if defined(__HIPCC__)
__constant__ uint64_t PV_SHA512_K[80] = {
      0x428a2f98d728ae22ull, 0x7137449123ef65cdull, 0xb5c0fbcfec4d3b2full, 0xe9b5dba58189dbbcull,
      0x3956c25bf348b538ull, 0x59f111f1b605d019ull, 0x923f82a4af194f9bull, 0xab1c5ed5da6d8118ull,
      0xd807aa98a3030242ull, 0x12835b0145706fbeull, 0x243185be4ee4b28cull, 0x550c7dc3d5ffb4e2ull,
      0x72be5d74f27b896full, 0x80deb1fe3b1696b1ull, 0x9bdc06a725c71235ull, 0xc19bf174cf692694ull,
      0xe49b69c19ef14ad2ull, 0xefbe4786384f25e3ull, 0x0fc19dc68b8cd5b5ull, 0x240ca1cc77ac9c65ull,
      0x2de92c6f592b0275ull, 0x4a7484aa6ea6e483ull, 0x5cb0a9dcbd41fbd4ull, 0x76f988da831153b5ull,
      0x983e5152ee66dfabull, 0xa831c66d2db43210ull, 0xb00327c898fb213full, 0xbf597fc7beef0ee4ull,
      0xc6e00bf33da88fc2ull, 0xd5a79147930aa725ull, 0x06ca6351e003826full, 0x142929670a0e6e70ull,
      0x27b70a8546d22ffcull, 0x2e1b21385c26c926ull, 0x4d2c6dfc5ac42aedull, 0x53380d139d95b3dfull,
      0x650a73548baf63deull, 0x766a0abb3c77b2a8ull, 0x81c2c92e47edaee6ull, 0x92722c851482353bull,
      0xa2bfe8a14cf10364ull, 0xa81a664bbc423001ull, 0xc24b8b70d0f89791ull, 0xc76c51a30654be30ull,
      0xd192e819d6ef5218ull, 0xd69906245565a910ull, 0xf40e35855771202aull, 0x106aa07032bbd1b8ull,
      0x19a4c116b8d2d0c8ull, 0x1e376c085141ab53ull, 0x2748774cdf8eeb99ull, 0x34b0bcb5e19b48a8ull,
      0x391c0cb3c5c95a63ull, 0x4ed8aa4ae3418acbull, 0x5b9cca4f7763e373ull, 0x682e6ff3d6b2b8a3ull,
      0x748f82ee5defb2fcull, 0x78a5636f43172f60ull, 0x84c87814a1f0ab72ull, 0x8cc702081a6439ecull,
      0x90befffa23631e28ull, 0xa4506cebde82bde9ull, 0xbef9a3f7b2c67915ull, 0xc67178f2e372532bull,
      0xca273eceea26619cull, 0xd186b8c721c0c207ull, 0xeada7dd6cde0eb1eull, 0xf57d4f7fee6ed178ull,
      0x06f067aa72176fbaull, 0x0a637dc5a2c898a6ull, 0x113f9804bef90daeull, 0x1b710b35131c471bull,
      0x28db77f523047d84ull, 0x32caab7b40c72493ull, 0x3c9ebe0a15c9bebcull, 0x431d67c49c100d4cull,
      0x4cc5d4becb3e42b6ull, 0x597f299cfc657e2aull, 0x5fcb6fab3ad6faecull, 0x6c44198c4a475817ull,
};
#else
static const uint64_t PV_SHA512_K[80] = {
      0x428a2f98d728ae22ull, 0x7137449123ef65cdull, 0xb5c0fbcfec4d3b2full, 0xe9b5dba58189dbbcull,
      0x3956c25bf348b538ull, 0x59f111f1b605d019ull, 0x923f82a4af194f9bull, 0xab1c5ed5da6d8118ull,
      0xd807aa98a3030242ull, 0x12835b0145706fbeull, 0x243185be4ee4b28cull, 0x550c7dc3d5ffb4e2ull,
      0x72be5d74f27b896full, 0x80deb1fe3b1696b1ull, 0x9bdc06a725c71235ull, 0xc19bf174cf692694ull,
      0xe49b69c19ef14ad2ull, 0xefbe4786384f25e3ull, 0x0fc19dc68b8cd5b5ull, 0x240ca1cc77ac9c65ull,
      0x2de92c6f592b0275ull, 0x4a7484aa6ea6e483ull, 0x5cb0a9dcbd41fbd4ull, 0x76f988da831153b5ull,
      0x983e5152ee66dfabull, 0xa831c66d2db43210ull, 0xb00327c898fb213full, 0xbf597fc7beef0ee4ull,
      0xc6e00bf33da88fc2ull, 0xd5a79147930aa725ull, 0x06ca6351e003826full, 0x142929670a0e6e70ull,
      0x27b70a8546d22ffcull, 0x2e1b21385c26c926ull, 0x4d2c6dfc5ac42aedull, 0x53380d139d95b3dfull,
      0x650a73548baf63deull, 0x766a0abb3c77b2a8ull, 0x81c2c92e47edaee6ull, 0x92722c851482353bull,
      0xa2bfe8a14cf10364ull, 0xa81a664bbc423001ull, 0xc24b8b70d0f89791ull, 0xc76c51a30654be30ull,
      0xd192e819d6ef5218ull, 0xd69906245565a910ull, 0xf40e35855771202aull, 0x106aa07032bbd1b8ull,
      0x19a4c116b8d2d0c8ull, 0x1e376c085141ab53ull, 0x2748774cdf8eeb99ull, 0x34b0bcb5e19b48a8ull,
      0x391c0cb3c5c95a63ull, 0x4ed8aa4ae3418acbull, 0x5b9cca4f7763e373ull, 0x682e6ff3d6b2b8a3ull,
      0x748f82ee5defb2fcull, 0x78a5636f43172f60ull, 0x84c87814a1f0ab72ull, 0x8cc702081a6439ecull,
      0x90befffa23631e28ull, 0xa4506cebde82bde9ull, 0xbef9a3f7b2c67915ull, 0xc67178f2e372532bull,
      0xca273eceea26619cull, 0xd186b8c721c0c207ull, 0xeada7dd6cde0eb1eull, 0xf57d4f7fee6ed178ull,
      0x06f067aa72176fbaull, 0x0a637dc5a2c898a6ull, 0x113f9804bef90daeull, 0x1b710b35131c471bull,
      0x28db77f523047d84ull, 0x32caab7b40c72493ull, 0x3c9ebe0a15c9bebcull, 0x431d67c49c100d4cull,
      0x4cc5d4becb3e42b6ull, 0x597f299cfc657e2aull, 0x5fcb6fab3ad6faecull, 0x6c44198c4a475817ull,
};
#endif

PV_HD void sha512_init(uint64_t h[8]) {
  h[0] = 0x6a09e667f3bcc908ull; h[1] = 0xbb67ae8584caa73bull;
  h[2] = 0x3c6ef372fe94f82bull; h[3] = 0xa54ff53a5f1d36f1ull;
  h[4] = 0x510e527fade682d1ull; h[5] = 0x9b05688c2b3e6c1full;
  h[6] = 0x1f83d9abfb41bd6bull; h[7] = 0x5be0cd19137e2179ull;
}

// 64-bit rotate / shift on the two 32-bit halves: one v_alignbit_b32 per half
// (n is a compile-time constant in the unrolled rounds, so the branch folds)
PV_HD uint64_t rotr64(uint64_t x, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  uint32_t rl, rh;
  if (n < 32) {
    rl = __builtin_amdgcn_alignbit(hi, lo, n);
    rh = __builtin_amdgcn_alignbit(lo, hi, n);
  } else {
    rl = __builtin_amdgcn_alignbit(lo, hi, n - 32);
    rh = __builtin_amdgcn_alignbit(hi, lo, n - 32);
  }
  return ((uint64_t)rh << 32) | rl;
#else
  return (x >> n) | (x << (64 - n));
#endif
}

PV_HD uint64_t shr64(uint64_t x, int n) {  // n < 32
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  return ((uint64_t)(hi >> n) << 32) | __builtin_amdgcn_alignbit(hi, lo, n);
#else
  return x >> n;
#endif
}

// 3-input bitwise functions on both halves: one v_bitop3_b32 per half on
// gfx950 (truth tables in the f(0xf0, 0xcc, 0xaa) convention: xor3 0x96,
// choose 0xca, majority 0xe8)
#if defined(__HIP_DEVICE_COMPILE__)
#define PV_BITOP3_64(a, b, c, T)                                                                        \
  ((((uint64_t)(uint32_t)__builtin_amdgcn_bitop3_b32((uint32_t)((a) >> 32), (uint32_t)((b) >> 32),     \
                                                     (uint32_t)((c) >> 32), (T)))                       \
    << 32) |                                                                                            \
   (uint64_t)(uint32_t)__builtin_amdgcn_bitop3_b32((uint32_t)(a), (uint32_t)(b), (uint32_t)(c), (T)))
PV_HD uint64_t xor3_64(uint64_t a, uint64_t b, uint64_t c) { return PV_BITOP3_64(a, b, c, 0x96); }
PV_HD uint64_t ch64(uint64_t e, uint64_t f, uint64_t g) { return PV_BITOP3_64(e, f, g, 0xca); }
PV_HD uint64_t maj64(uint64_t a, uint64_t b, uint64_t c) { return PV_BITOP3_64(a, b, c, 0xe8); }
#else
PV_HD uint64_t xor3_64(uint64_t a, uint64_t b, uint64_t c) { return a ^ b ^ c; }
PV_HD uint64_t ch64(uint64_t e, uint64_t f, uint64_t g) { return (e & f) | (~e & g); }
PV_HD uint64_t maj64(uint64_t a, uint64_t b, uint64_t c) { return (a & b) | (a & c) | (b & c); }
#endif

// 64-bit add as ONE v_lshl_add_u64 on the two register pairs.  Plain `+` on
// values assembled from 32-bit halves (rotates, bit functions) is split by
// the compiler into a zero-extended low add plus a 32-bit high add and moves
// of a zero register (3 extra instructions per round).
PV_HD uint64_t add64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__) && PV_SHA_ASM_ADD
  uint64_t r;
  asm("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
#else
  return a + b;
#endif
}

// one compression; w[16] holds the block as big-endian-decoded 64-bit words
// (it is overwritten by the schedule).  Per round: 6 alignbit + 2 bitop3 per
// Sigma, 2 bitop3 for Ch, 2 for Maj, 7 64-bit adds.
PV_HD void sha512_round(uint64_t& a, uint64_t& b, uint64_t& c, uint64_t& d, uint64_t& e, uint64_t& f, uint64_t& g,
                        uint64_t& k, uint64_t kw) {
  const uint64_t S1 = xor3_64(rotr64(e, 14), rotr64(e, 18), rotr64(e, 41));
  const uint64_t t1 = add64(add64(add64(k, kw), ch64(e, f, g)), S1);
  const uint64_t S0 = xor3_64(rotr64(a, 28), rotr64(a, 34), rotr64(a, 39));
  const uint64_t t2 = add64(S0, maj64(a, b, c));
  k = g; g = f; f = e; e = add64(d, t1); d = c; c = b; b = a; a = add64(t1, t2);
}

PV_HD void sha512_compress(uint64_t h[8], uint64_t w[16]) {
  PV_COUNT(sha);
  uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], k = h[7];
#pragma clang loop unroll(full)
  for (int j = 0; j < 16; ++j) sha512_round(a, b, c, d, e, f, g, k, PV_SHA512_K[j] + w[j]);
  // rounds 16..79: 4 passes of 16 with the rolling schedule at static indices
  // (kept as a loop: the fully unrolled 80 rounds overflow the instruction cache)
#pragma unroll 1
  for (int r = 16; r < 80; r += 16) {
#pragma clang loop unroll(full)
    for (int j = 0; j < 16; ++j) {
      const uint64_t w15 = w[(j + 1) & 15], w2 = w[(j + 14) & 15];
      const uint64_t s0 = xor3_64(rotr64(w15, 1), rotr64(w15, 8), shr64(w15, 7));
      const uint64_t s1 = xor3_64(rotr64(w2, 19), rotr64(w2, 61), shr64(w2, 6));
      w[j] = add64(add64(add64(w[j], w[(j + 9) & 15]), s0), s1);
      sha512_round(a, b, c, d, e, f, g, k, PV_SHA512_K[r + j] + w[j]);
    }
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += k;
}

// The compression split in two (k_verify_quad_keyed's hash wave: one lane per
// message block computes that block's schedule, the hashing lane then runs
// only the 80 rounds).  kw[t * stride] = K_t + W_t for t < 80 from the block's
// 16 big-endian words; the same sums as sha512_compress's rolling schedule.
PV_HD void sha512_schedule_kw(uint64_t* kw, int stride, const uint64_t w0[16]) {
  uint64_t w[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    w[j] = w0[j];
    kw[j * stride] = PV_SHA512_K[j] + w[j];
  }
#pragma unroll 1
  for (int r = 16; r < 80; r += 16) {
#pragma clang loop unroll(full)
    for (int j = 0; j < 16; ++j) {
      const uint64_t w15 = w[(j + 1) & 15], w2 = w[(j + 14) & 15];
      const uint64_t s0 = xor3_64(rotr64(w15, 1), rotr64(w15, 8), shr64(w15, 7));
      const uint64_t s1 = xor3_64(rotr64(w2, 19), rotr64(w2, 61), shr64(w2, 6));
      w[j] = add64(add64(add64(w[j], w[(j + 9) & 15]), s0), s1);
      kw[(r + j) * stride] = PV_SHA512_K[r + j] + w[j];
    }
  }
}
PV_HD void sha512_compress_kw(uint64_t h[8], const uint64_t* kw, int stride) {
  PV_COUNT(sha);
  uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], k = h[7];
#pragma unroll 1
  for (int r = 0; r < 80; r += 16) {
#pragma clang loop unroll(full)
    for (int j = 0; j < 16; ++j) sha512_round(a, b, c, d, e, f, g, k, kw[(r + j) * stride]);
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += k;
}

PV_HD uint32_t bswap32(uint32_t x) {
  return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
}

// little-endian byte words (as loaded from memory) -> big-endian 64-bit word
PV_HD uint64_t be64_from_le32(uint32_t lo, uint32_t hi) {
  return ((uint64_t)bswap32(lo) << 32) | bswap32(hi);
}

// 64-byte digest h[8] -> 16 little-endian words (digest byte order)
PV_HD void sha512_digest_words(uint32_t out[16], const uint64_t h[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    out[2 * i] = bswap32((uint32_t)(h[i] >> 32));
    out[2 * i + 1] = bswap32((uint32_t)h[i]);
  }
}

// SHA-512 of a short, register-resident message of n32 little-endian words
// (n32 * 4 < 112 bytes) : one block.  Used for seeds and fixed-size inputs.
PV_HD void sha512_short(uint32_t out[16], const uint32_t* m, int nbytes) {
  uint64_t h[8], w[16];
  sha512_init(h);
#pragma unroll
  for (int i = 0; i < 16; ++i) w[i] = 0;
  for (int i = 0; i < 14; ++i) {
    const int b0 = 8 * i;
    uint32_t lo = 0, hi = 0;
    if (b0 < nbytes) lo = m[2 * i];
    if (b0 + 4 < nbytes) hi = m[2 * i + 1];
    // mask partial words
    if (b0 + 4 > nbytes && b0 < nbytes) lo &= (1u << (8 * (nbytes - b0))) - 1u;
    if (b0 + 8 > nbytes && b0 + 4 < nbytes) hi &= (1u << (8 * (nbytes - b0 - 4))) - 1u;
    // padding byte 0x80 at position nbytes
    if (nbytes >= b0 && nbytes < b0 + 4) lo |= 0x80u << (8 * (nbytes - b0));
    if (nbytes >= b0 + 4 && nbytes < b0 + 8) hi |= 0x80u << (8 * (nbytes - b0 - 4));
    w[i] = be64_from_le32(lo, hi);
  }
  w[15] = (uint64_t)nbytes * 8u;
  sha512_compress(h, w);
  sha512_digest_words(out, h);
}

}  // namespace pv
