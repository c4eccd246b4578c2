// SHA-256 (FIPS 180-4) for one lane, native 32-bit words: rotates are
// v_alignbit_b32(x, x, n), Ch / Maj / 3-way XOR one v_bitop3_b32 each on gfx950.
//
// Used for SURVEY.md §8 row f3: request digests (Request.key =
// sha256(serialize_msg_for_signing(signingState)), plenum/common/request.py:82-90)
// and the ledger's Merkle tree hashing (ledger/tree_hasher.py:4-30: leaf =
// SHA-256(0x00 || data), node = SHA-256(0x01 || left || right)).
#pragma once
#include <stdint.h>
#include "pv_field.h"

namespace pv {

#if defined(__HIPCC__)
__constant__ uint32_t PV_SHA256_K[64] = {
#else
static const uint32_t PV_SHA256_K[64] = {
#endif
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u,
};

PV_HD uint32_t rotr32(uint32_t x, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbit(x, x, n);
#else
  return (x >> n) | (x << (32 - n));
#endif
}

#if defined(__HIP_DEVICE_COMPILE__)
PV_HD uint32_t xor3_32(uint32_t a, uint32_t b, uint32_t c) { return (uint32_t)__builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }
PV_HD uint32_t ch32(uint32_t e, uint32_t f, uint32_t g) { return (uint32_t)__builtin_amdgcn_bitop3_b32(e, f, g, 0xca); }
PV_HD uint32_t maj32(uint32_t a, uint32_t b, uint32_t c) { return (uint32_t)__builtin_amdgcn_bitop3_b32(a, b, c, 0xe8); }
#else
PV_HD uint32_t xor3_32(uint32_t a, uint32_t b, uint32_t c) { return a ^ b ^ c; }
PV_HD uint32_t ch32(uint32_t e, uint32_t f, uint32_t g) { return (e & f) | (~e & g); }
PV_HD uint32_t maj32(uint32_t a, uint32_t b, uint32_t c) { return (a & b) | (a & c) | (b & c); }
#endif

PV_HD void sha256_init(uint32_t h[8]) {
  h[0] = 0x6a09e667u; h[1] = 0xbb67ae85u; h[2] = 0x3c6ef372u; h[3] = 0xa54ff53au;
  h[4] = 0x510e527fu; h[5] = 0x9b05688cu; h[6] = 0x1f83d9abu; h[7] = 0x5be0cd19u;
}

PV_HD void sha256_round(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d, uint32_t& e, uint32_t& f, uint32_t& g,
                        uint32_t& k, uint32_t kw) {
  const uint32_t t1 = k + xor3_32(rotr32(e, 6), rotr32(e, 11), rotr32(e, 25)) + ch32(e, f, g) + kw;
  const uint32_t t2 = xor3_32(rotr32(a, 2), rotr32(a, 13), rotr32(a, 22)) + maj32(a, b, c);
  k = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
}

// one compression; w[16] = the block as big-endian-decoded words (overwritten)
PV_HD void sha256_compress(uint32_t h[8], uint32_t w[16]) {
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], k = h[7];
#pragma clang loop unroll(full)
  for (int j = 0; j < 16; ++j) sha256_round(a, b, c, d, e, f, g, k, PV_SHA256_K[j] + w[j]);
#pragma unroll 1
  for (int r = 16; r < 64; r += 16) {
#pragma clang loop unroll(full)
    for (int j = 0; j < 16; ++j) {
      const uint32_t w15 = w[(j + 1) & 15], w2 = w[(j + 14) & 15];
      const uint32_t s0 = xor3_32(rotr32(w15, 7), rotr32(w15, 18), w15 >> 3);
      const uint32_t s1 = xor3_32(rotr32(w2, 17), rotr32(w2, 19), w2 >> 10);
      w[j] = w[j] + s0 + w[(j + 9) & 15] + s1;
      sha256_round(a, b, c, d, e, f, g, k, PV_SHA256_K[r + j] + w[j]);
    }
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += k;
}

PV_HD uint32_t bswap32_(uint32_t x) {
  return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
}

PV_HD uint32_t funnel32_(uint32_t hi, uint32_t lo, uint32_t sh) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbit(hi, lo, sh);
#else
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> sh);
#endif
}

// SHA-256 blocks of (prefix || M), plen = 0 or 1 prefix bytes
PV_HD uint64_t sha256_blocks(uint64_t mlen, uint32_t plen) { return (plen + mlen + 9 + 63) / 64; }

// block `blk` of (prefix || M) as 16 big-endian words, SHA padding and length
// applied, from the aligned-word window of its first data byte.
// PV_SHA256_GROUPS = 1: the window is fetched as 4-word groups (group g is
// loaded iff its first word holds a message byte: at most 5 dwordx4 loads per
// lane and block instead of 17 guarded dword loads, each of which touches one
// cache line per lane; a group reads at most 15 bytes past the message end, so
// the blob needs >= 16 readable bytes after the last message), and the padding
// is branch-free 32-bit selects (the clamped terminator position, as
// msg_assemble of pv_verify_core.h); 0 = the per-word form (A/B baseline).
#ifndef PV_SHA256_GROUPS
#define PV_SHA256_GROUPS 1
#endif
#if PV_SHA256_GROUPS
constexpr int SHA256_Y = 20;
PV_HD void sha256_window(uint32_t y[SHA256_Y], const uint8_t* m, uint64_t mlen, uint32_t plen, uint64_t blk) {
  const bool pre = plen != 0 && blk == 0;
  const uint64_t q = pre ? 0 : 64 * blk - plen;        // first data byte of the window
  const int64_t rem = (int64_t)mlen - (int64_t)q;
  const uintptr_t base = reinterpret_cast<uintptr_t>(m) + q;
  const uint32_t mis = (uint32_t)(base & 3u);
  const uint32_t* wp = reinterpret_cast<const uint32_t*>(m + q - mis);
#pragma unroll
  for (int g = 0; g < 5; ++g) {
    uint32_t a = 0, b = 0, c = 0, d = 0;
    if ((int64_t)(16 * g) - (int64_t)mis < rem) {
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
PV_HD void sha256_assemble(uint32_t w[16], const uint32_t y[SHA256_Y], const uint8_t* m, uint64_t mlen, uint32_t plen,
                           uint32_t prefix, uint64_t blk, uint64_t nblk) {
  const bool pre = plen != 0 && blk == 0;
  const uint64_t q = pre ? 0 : 64 * blk - plen;
  const uint32_t mis = (uint32_t)((reinterpret_cast<uintptr_t>(m) + q) & 3u);
  uint32_t d[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) d[k] = funnel32_(y[k + 1], y[k], 8u * mis);
  if (pre) {  // shift the data one byte up and put the prefix in byte 0
#pragma unroll
    for (int k = 15; k > 0; --k) d[k] = funnel32_(d[k], d[k - 1], 24u);
    d[0] = (d[0] << 8) | (prefix & 0xffu);
  }
  // terminator position in this block, clamped to [-1, 68]: words below it
  // are data, the word holding it keeps its low t % 4 bytes and takes 0x80,
  // words above it are zero
  const int64_t t64 = (int64_t)(plen + mlen) - (int64_t)(64 * blk);
  const int32_t t = t64 < 0 ? -1 : (t64 > 68 ? 68 : (int32_t)t64);
  const uint32_t rb = 8u * ((uint32_t)t & 3u);
  const uint32_t keep = (1u << rb) - 1u, pad = 0x80u << rb;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint32_t v = d[k];
    const uint32_t tv = (v & keep) | pad;
    w[k] = bswap32_(t >= 4 * k + 4 ? v : (t >= 4 * k ? tv : 0u));
  }
  if (blk + 1 == nblk) {
    const uint64_t bits = (plen + mlen) * 8;
    w[14] = (uint32_t)(bits >> 32);
    w[15] = (uint32_t)bits;
  }
}
#else
constexpr int SHA256_Y = 17;
// the aligned-word window of block blk of (prefix || M): 17 words from the
// aligned-down first data byte, zero past the message (no load issued there)
PV_HD void sha256_window(uint32_t y[SHA256_Y], const uint8_t* m, uint64_t mlen, uint32_t plen, uint64_t blk) {
  const bool pre = plen != 0 && blk == 0;
  const uint64_t q = pre ? 0 : 64 * blk - plen;        // first data byte of the window
  const int64_t rem = (int64_t)mlen - (int64_t)q;
  const uintptr_t base = reinterpret_cast<uintptr_t>(m) + q;
  const uint32_t mis = (uint32_t)(base & 3u);
  const uint32_t* wp = reinterpret_cast<const uint32_t*>(base - mis);
#pragma unroll
  for (int k = 0; k < 17; ++k) y[k] = (int64_t)(4 * k) - (int64_t)mis < rem ? wp[k] : 0u;
}
// block blk's 16 big-endian words from its window: funnel shift by the
// misalignment, the prefix byte, the 0x80 terminator and the bit length
PV_HD void sha256_assemble(uint32_t w[16], const uint32_t y[SHA256_Y], const uint8_t* m, uint64_t mlen, uint32_t plen,
                           uint32_t prefix, uint64_t blk, uint64_t nblk) {
  const bool pre = plen != 0 && blk == 0;
  const uint64_t q = pre ? 0 : 64 * blk - plen;
  const uint32_t mis = (uint32_t)((reinterpret_cast<uintptr_t>(m) + q) & 3u);
  uint32_t d[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) d[k] = funnel32_(y[k + 1], y[k], 8u * mis);
  if (pre) {  // shift the data one byte up and put the prefix in byte 0
#pragma unroll
    for (int k = 15; k > 0; --k) d[k] = (d[k] << 8) | (d[k - 1] >> 24);
    d[0] = (d[0] << 8) | (prefix & 0xffu);
  }
  const int64_t t = (int64_t)(plen + mlen) - (int64_t)(64 * blk);   // terminator position in this block
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int64_t r = t - 4 * k;
    uint32_t v = d[k];
    if (r < 4) {
      const uint32_t keep = r <= 0 ? 0u : (1u << (8 * (uint32_t)r)) - 1u;
      v = (v & keep) | ((r >= 0) ? (0x80u << (8 * (uint32_t)r)) : 0u);
    }
    w[k] = bswap32_(v);
  }
  if (blk + 1 == nblk) {
    const uint64_t bits = (plen + mlen) * 8;
    w[14] = (uint32_t)(bits >> 32);
    w[15] = (uint32_t)bits;
  }
}
#endif
PV_HD void sha256_block(uint32_t w[16], const uint8_t* m, uint64_t mlen, uint32_t plen, uint32_t prefix, uint64_t blk,
                        uint64_t nblk) {
  uint32_t y[SHA256_Y];
  sha256_window(y, m, mlen, plen, blk);
  sha256_assemble(w, y, m, mlen, plen, prefix, blk, nblk);
}

// digest of (prefix || M) as 8 little-endian words (digest byte order)
PV_HD void sha256_msg(uint32_t out[8], const uint8_t* m, uint64_t mlen, uint32_t plen, uint32_t prefix) {
  uint32_t h[8], w[16];
  sha256_init(h);
  const uint64_t nb = sha256_blocks(mlen, plen);
  for (uint64_t b = 0; b < nb; ++b) {
    sha256_block(w, m, mlen, plen, prefix, b, nb);
    sha256_compress(h, w);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) out[i] = bswap32_(h[i]);
}

// Merkle interior node SHA-256(0x01 || left || right) of two 32-byte hashes
// given as 16 little-endian words (left then right)
PV_HD void sha256_node(uint32_t out[8], const uint32_t lr[16]) {
  uint32_t h[8], w[16];
  sha256_init(h);
  // block 0: 0x01, lr bytes 0..62; block 1: lr byte 63, 0x80, zeros, length 520 bits
#pragma unroll
  for (int k = 0; k < 16; ++k) w[k] = bswap32_((lr[k] << 8) | (k ? lr[k - 1] >> 24 : 0x01u));
  sha256_compress(h, w);
#pragma unroll
  for (int k = 0; k < 16; ++k) w[k] = 0;
  w[0] = bswap32_((lr[15] >> 24) | (0x80u << 8));
  w[15] = 65 * 8;
  sha256_compress(h, w);
#pragma unroll
  for (int i = 0; i < 8; ++i) out[i] = bswap32_(h[i]);
}

}  // namespace pv
