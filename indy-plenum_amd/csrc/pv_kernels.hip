// HIP kernels for gfx950 (MI355X): batch Ed25519 verification with
// libsodium-1.0.18 verdict semantics, batch keygen/sign, n-f quorum tally.
//
// Verify = two launches, one lane per signature:
//   k_hash  : pre-checks (S < L, R/A not small order, A canonical) and
//             h = SHA-512(R || A || M) mod L                  
//   k_curve : -A = decompress(A), R' = h(-A) + S B by a FIXED signed-digit
//             schedule (A: radix 16, 9-entry per-lane table in scratch;
//             B: radix 256, 129-entry niels table in LDS), then
//             encode(R') == R                                 (steps 4, 6, 7)
// Every lane runs the same window schedule (digit 0 adds the identity), so
// a wavefront never diverges inside the scalar multiplication.
#include <hip/hip_runtime.h>
#include "pv_field.h"
#include "pv_scalar.h"
#include "pv_curve.h"
#include "pv_sha512.h"
#include "pv_kernels.h"

namespace pv {

// ------------------------------------------------------------------ loads
__device__ __forceinline__ void load8(uint32_t w[8], const uint8_t* p) {
  const uint4 a = *reinterpret_cast<const uint4*>(p);
  const uint4 b = *reinterpret_cast<const uint4*>(p + 16);
  w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
  w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
}
__device__ __forceinline__ void store8(uint8_t* p, const uint32_t w[8]) {
  *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
  *reinterpret_cast<uint4*>(p + 16) = make_uint4(w[4], w[5], w[6], w[7]);
}

PV_HD uint32_t pick8(const uint32_t a[8], int k) {
  uint32_t r = a[0];
#pragma unroll
  for (int j = 1; j < 8; ++j) r = (k == j) ? a[j] : r;
  return r;
}

// 8 message bytes starting at byte q of M (q < mlen), little-endian packed;
// bytes past mlen are zero, byte mlen is the 0x80 pad.  Reads 3 aligned words
// (the blob is allocated with >= 16 bytes of tail padding).
__device__ __forceinline__ uint64_t msg_bytes8(const uint8_t* m, uint64_t mlen, uint64_t q) {
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
  const uint64_t rem = mlen > q ? mlen - q : 0;  // bytes of M left
  if (rem < 8) {
    const uint64_t keep = rem == 0 ? 0 : ((1ull << (8 * rem)) - 1);
    v &= keep;
    if (q <= mlen) v |= 0x80ull << (8 * rem);  // pad byte lands in this word
  }
  return v;
}

PV_HD uint64_t bswap64(uint64_t x) {
  return ((uint64_t)bswap32((uint32_t)x) << 32) | bswap32((uint32_t)(x >> 32));
}

// SHA-512(prefix || M): prefix is 32 or 64 bytes held as LE words.
__device__ void sha512_prefixed(uint32_t out[16], const uint32_t* pre, int pre_words64, const uint8_t* m,
                                uint64_t mlen) {
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
        const uint64_t q = (g - pre_words64) * 8;
        word = (q <= mlen + 7) ? bswap64(msg_bytes8(m, mlen, q)) : 0;
        if (q > mlen) word = 0;
      }
      if (last && j == 14) word = 0;
      if (last && j == 15) word = total * 8;
      w[j] = word;
    }
    sha512_compress(h, w);
  }
  sha512_digest_words(out, h);
}

// ------------------------------------------------------------- hash kernel
__global__ __launch_bounds__(HASH_BLOCK) void k_hash(const uint8_t* __restrict__ pk, const uint8_t* __restrict__ sig,
                                                      const uint8_t* __restrict__ blob,
                                                      const uint64_t* __restrict__ off, uint64_t n,
                                                      uint32_t* __restrict__ hout, uint8_t* __restrict__ pre) {
  const uint64_t i = (uint64_t)blockIdx.x * HASH_BLOCK + threadIdx.x;
  if (i >= n) return;
  uint32_t ra[16];  // R (8 words) || A (8 words)
  uint32_t sw[8];
  load8(ra, sig + 64 * i);
  load8(sw, sig + 64 * i + 32);
  load8(ra + 8, pk + 32 * i);
  const bool ok = sc_is_canonical(sw) && !has_small_order(ra) && y_is_canonical(ra + 8) && !has_small_order(ra + 8);
  pre[i] = ok ? 1 : 0;
  uint32_t h[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (ok) {
    const uint64_t o = off[i];
    const uint64_t mlen = off[i + 1] - o;
    uint32_t dig[16];
    sha512_prefixed(dig, ra, 8, blob + o, mlen);
    sc_reduce64(h, dig);
  }
  store8(reinterpret_cast<uint8_t*>(hout + 8 * i), h);
}

hipError_t launch_hash(const uint8_t* pk, const uint8_t* sig, const uint8_t* blob, const uint64_t* off, uint64_t n,
                       uint32_t* h, uint8_t* pre, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t blocks = (n + HASH_BLOCK - 1) / HASH_BLOCK;
  hipLaunchKernelGGL(k_hash, dim3((uint32_t)blocks), dim3(HASH_BLOCK), 0, s, pk, sig, blob, off, n, h, pre);
  return hipGetLastError();
}

// ------------------------------------------------------------ table access
__device__ __forceinline__ void store_fe(uint32_t* p, const fe& f) {
  *reinterpret_cast<uint4*>(p) = make_uint4(f.v[0], f.v[1], f.v[2], f.v[3]);
  *reinterpret_cast<uint4*>(p + 4) = make_uint4(f.v[4], f.v[5], f.v[6], f.v[7]);
  *reinterpret_cast<uint2*>(p + 8) = make_uint2(f.v[8], f.v[9]);
}
__device__ __forceinline__ void load_fe(fe& f, const uint32_t* p) {
  const uint4 a = *reinterpret_cast<const uint4*>(p);
  const uint4 b = *reinterpret_cast<const uint4*>(p + 4);
  const uint2 c = *reinterpret_cast<const uint2*>(p + 8);
  f.v[0] = a.x; f.v[1] = a.y; f.v[2] = a.z; f.v[3] = a.w;
  f.v[4] = b.x; f.v[5] = b.y; f.v[6] = b.z; f.v[7] = b.w;
  f.v[8] = c.x; f.v[9] = c.y;
}
__device__ __forceinline__ void store_cached(uint32_t* p, const ge_cached& c) {
  store_fe(p, c.YpX);
  store_fe(p + 10, c.YmX);
  store_fe(p + 20, c.Z2);
  store_fe(p + 30, c.T2d);
}
__device__ __forceinline__ void load_cached(ge_cached& c, const uint32_t* p) {
  load_fe(c.YpX, p);
  load_fe(c.YmX, p + 10);
  load_fe(c.Z2, p + 20);
  load_fe(c.T2d, p + 30);
}
// niels entry in LDS (or global): 3 fe at word offsets 0, 10, 20 of a 32-word slot
__device__ __forceinline__ void load_niels(ge_niels& q, const uint32_t* p) {
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    q.ypx.v[k] = p[k];
    q.ymx.v[k] = p[10 + k];
    q.xy2d.v[k] = p[20 + k];
  }
}

// ---------------------------------------------------------- base-point table
__device__ void ge_basepoint(ge_p3& B) {
  // encoding of B: y = 4/5, x even: 0x58 0x66 ... 0x66
  uint32_t enc[8] = {0x66666658u, 0x66666666u, 0x66666666u, 0x66666666u,
                     0x66666666u, 0x66666666u, 0x66666666u, 0x66666666u};
  ge_p3 nb;
  ge_frombytes_negate(nb, enc);  // -B
  fe_copy(B.Y, nb.Y);
  fe_copy(B.Z, nb.Z);
  fe_neg(B.X, nb.X); fe_carry(B.X);
  fe_neg(B.T, nb.T); fe_carry(B.T);
}

__global__ void k_btable_init(uint32_t* btab) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= BTAB_ENTRIES) return;
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
  uint32_t* p = btab + k * BTAB_WORDS;
  for (int i = 0; i < 10; ++i) {
    p[i] = ypx.v[i];
    p[10 + i] = ymx.v[i];
    p[20 + i] = xy2d.v[i];
  }
  p[30] = 0;
  p[31] = 0;
}

hipError_t launch_btable_init(uint32_t* btab, hipStream_t s) {
  hipLaunchKernelGGL(k_btable_init, dim3(3), dim3(64), 0, s, btab);
  return hipGetLastError();
}

// ------------------------------------------------------------ curve kernel
// R' = hh*(-A) + ss*B with hh' = hh + 0x88..88 (radix-16 digits d-8) and
// ss' = ss + 0x8080..80 (radix-256 digits d-128).  Returns R' as p2.
__device__ void double_scalarmult(ge_p2& out, const uint32_t hh[8], const uint32_t ss[8], const uint32_t* atab,
                                  const uint32_t* btab_lds) {
  uint32_t hp[8], sp[8];
  sc_add_pattern(hp, hh, 0x88888888u);
  sc_add_pattern(sp, ss, 0x80808080u);
  ge_p3 acc;
  ge_p3_0(acc);
  ge_p1p1 t;
  ge_p2 r2;
  // window 63 (top): acc = d63 * (-A), no doublings
  {
    const int dA = (int)(hp[7] >> 28) - 8;
    ge_cached c;
    load_cached(c, atab + (dA < 0 ? -dA : dA) * 40);
    ge_add_cached(t, acc, c, dA < 0);
    ge_p1p1_to_p2(r2, t);
  }
#pragma unroll 1
  for (int i = 62; i >= 0; --i) {
    // 16 * acc
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
      load_cached(c, atab + (dA < 0 ? -dA : dA) * 40);
      ge_add_cached(t, acc, c, dA < 0);
    }
    if ((i & 1) == 0) {
      const uint32_t sw = pick8(sp, i >> 3);
      const int dB = (int)((sw >> (8 * ((i >> 1) & 3))) & 255u) - 128;
      ge_p1p1_to_p3(acc, t);
      ge_niels q;
      load_niels(q, btab_lds + (dB < 0 ? -dB : dB) * BTAB_WORDS);
      ge_madd(t, acc, q, dB < 0);
    }
    ge_p1p1_to_p2(r2, t);
  }
  out = r2;
}

// cached odd/even multiples 0..8 of P into a per-lane table
__device__ void build_atab(uint32_t* atab, const ge_p3& P) {
  ge_cached c1, c;
  ge_cached_identity(c);
  store_cached(atab, c);
  ge_p3_to_cached(c1, P);
  store_cached(atab + 40, c1);
  ge_p3 prev = P;  // k*P as p3
  ge_p1p1 t;
#pragma unroll 1
  for (int k = 2; k <= 8; ++k) {
    ge_add_cached(t, prev, c1, false);
    ge_p1p1_to_p3(prev, t);
    ge_p3_to_cached(c, prev);
    store_cached(atab + 40 * k, c);
  }
}

__global__ __launch_bounds__(CURVE_BLOCK) void k_curve(const uint8_t* __restrict__ pk, const uint8_t* __restrict__ sig,
                                                        const uint32_t* __restrict__ hin,
                                                        const uint8_t* __restrict__ pre,
                                                        const uint32_t* __restrict__ btab_g,
                                                        uint32_t* __restrict__ scratch, uint8_t* __restrict__ verdict,
                                                        uint64_t* __restrict__ bitmap, uint64_t n) {
  __shared__ uint32_t btab[BTAB_ENTRIES * BTAB_WORDS];
  for (int j = threadIdx.x; j < BTAB_ENTRIES * BTAB_WORDS; j += CURVE_BLOCK) btab[j] = btab_g[j];
  __syncthreads();
  const uint64_t nthreads = (uint64_t)gridDim.x * CURVE_BLOCK;
  const uint64_t gid = (uint64_t)blockIdx.x * CURVE_BLOCK + threadIdx.x;
  uint32_t* atab = scratch + gid * ATAB_WORDS;
  for (uint64_t base = 0; base < n; base += nthreads) {
    const uint64_t i = base + gid;
    bool ok = false;
    if (i < n && pre[i]) {
      uint32_t A[8], R[8], S[8], hh[8];
      load8(A, pk + 32 * i);
      load8(R, sig + 64 * i);
      load8(S, sig + 64 * i + 32);
      load8(hh, reinterpret_cast<const uint8_t*>(hin + 8 * i));
      ge_p3 negA;
      if (ge_frombytes_negate(negA, A)) {
        build_atab(atab, negA);
        ge_p2 rp;
        double_scalarmult(rp, hh, S, atab, btab);
        uint32_t enc[8];
        ge_p2_tobytes(enc, rp);
        uint32_t diff = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) diff |= enc[k] ^ R[k];
        ok = diff == 0;
      }
    }
    const uint64_t ball = __ballot(ok);
    if (i < n) {
      verdict[i] = ok ? 1 : 0;
      if ((threadIdx.x & 63) == 0) bitmap[i >> 6] = ball;
    }
  }
}

hipError_t curve_occupancy(int* blocks_per_cu) {
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, reinterpret_cast<const void*>(k_curve),
                                                      CURVE_BLOCK, 0);
}

hipError_t launch_curve(const uint8_t* pk, const uint8_t* sig, const uint32_t* h, const uint8_t* pre,
                        const uint32_t* btab, uint32_t* scratch, uint64_t scratch_lanes, uint8_t* verdict,
                        uint64_t* bitmap, uint64_t n, int blocks, hipStream_t s) {
  if (n == 0) return hipSuccess;
  uint64_t need = (n + CURVE_BLOCK - 1) / CURVE_BLOCK;
  uint64_t b = (uint64_t)blocks < need ? (uint64_t)blocks : need;
  if (b * CURVE_BLOCK > scratch_lanes) b = scratch_lanes / CURVE_BLOCK;
  if (b == 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_curve, dim3((uint32_t)b), dim3(CURVE_BLOCK), 0, s, pk, sig, h, pre, btab, scratch, verdict,
                     bitmap, n);
  return hipGetLastError();
}

// ------------------------------------------------------------- batch signer
// fixed-base k*B, k < 2^253 (reduced scalar), radix-256 signed digits
__device__ void scalarmult_base(ge_p3& out, const uint32_t k[8], const uint32_t* btab) {
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
    load_niels(q, btab + (dB < 0 ? -dB : dB) * BTAB_WORDS);
    ge_madd(t, acc, q, dB < 0);
    ge_p1p1_to_p3(acc, t);
  }
  out = acc;
}

__global__ __launch_bounds__(256) void k_sign(const uint8_t* __restrict__ seeds, const uint8_t* __restrict__ blob,
                                               const uint64_t* __restrict__ off, uint64_t n,
                                               const uint32_t* __restrict__ btab_g, uint8_t* __restrict__ pk_out,
                                               uint8_t* __restrict__ sig_out) {
  __shared__ uint32_t btab[BTAB_ENTRIES * BTAB_WORDS];
  for (int j = threadIdx.x; j < BTAB_ENTRIES * BTAB_WORDS; j += 256) btab[j] = btab_g[j];
  __syncthreads();
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  uint32_t seed[8], az[16];
  load8(seed, seeds + 32 * i);
  sha512_short(az, seed, 32);
  az[0] &= 0xfffffff8u;
  az[7] &= 0x7fffffffu;
  az[7] |= 0x40000000u;
  // A = a*B with a reduced mod L (B has order L)
  uint32_t wide[16], ared[8];
#pragma unroll
  for (int k = 0; k < 16; ++k) wide[k] = k < 8 ? az[k] : 0u;
  sc_reduce64(ared, wide);
  ge_p3 A;
  scalarmult_base(A, ared, btab);
  uint32_t pkw[8];
  ge_p3_tobytes(pkw, A);
  const uint64_t o = off[i];
  const uint64_t mlen = off[i + 1] - o;
  // r = SHA-512(prefix || M) mod L
  uint32_t dig[16], r[8];
  sha512_prefixed(dig, az + 8, 4, blob + o, mlen);
  sc_reduce64(r, dig);
  ge_p3 Rp;
  scalarmult_base(Rp, r, btab);
  uint32_t ra[16];
  ge_p3_tobytes(ra, Rp);
#pragma unroll
  for (int k = 0; k < 8; ++k) ra[8 + k] = pkw[k];
  uint32_t kk[8];
  sha512_prefixed(dig, ra, 8, blob + o, mlen);
  sc_reduce64(kk, dig);
  uint32_t S[8];
  sc_muladd(S, kk, az, r);
  store8(pk_out + 32 * i, pkw);
  store8(sig_out + 64 * i, ra);
  store8(sig_out + 64 * i + 32, S);
}

hipError_t launch_sign(const uint8_t* seeds, const uint8_t* blob, const uint64_t* off, uint64_t n,
                       const uint32_t* btab, uint8_t* pk_out, uint8_t* sig_out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(k_sign, dim3((uint32_t)blocks), dim3(256), 0, s, seeds, blob, off, n, btab, pk_out, sig_out);
  return hipGetLastError();
}

// ------------------------------------------------------------------- tally
// One wavefront per 3PC batch: lanes OR (1 << sender) of valid votes into the
// voter set (duplicates collapse), popcount, compare with the quorum.
// plenum/server/models.py:24-45,91-114 ; plenum/server/quorums.py:15-39
__global__ __launch_bounds__(256) void k_tally(const uint8_t* __restrict__ verdict, const uint32_t* __restrict__ sender,
                                                const uint64_t* __restrict__ batch_off, uint64_t n_batches,
                                                uint32_t n_nodes, uint32_t quorum, uint32_t* __restrict__ votes,
                                                uint8_t* __restrict__ reached) {
  const uint64_t b = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (b >= n_batches) return;
  const uint64_t s0 = batch_off[b], s1 = batch_off[b + 1];
  const uint32_t words = (n_nodes + 63) / 64;  // voter-set words; n_nodes <= 1024 (16 words)
  uint32_t count = 0;
  for (uint32_t w = 0; w < words; ++w) {
    uint64_t mine = 0;
    for (uint64_t m = s0 + lane; m < s1; m += 64) {
      const uint32_t snd = sender[m];
      if (verdict[m] && snd < n_nodes && (snd >> 6) == w) mine |= 1ull << (snd & 63);
    }
    // wave OR-reduction
#pragma unroll
    for (int sh = 1; sh < 64; sh <<= 1) {
      const uint32_t lo = __shfl_xor((uint32_t)mine, sh, 64);
      const uint32_t hi = __shfl_xor((uint32_t)(mine >> 32), sh, 64);
      mine |= ((uint64_t)hi << 32) | lo;
    }
    count += __popcll(mine);
  }
  if (lane == 0) {
    votes[b] = count;
    reached[b] = count >= quorum ? 1 : 0;
  }
}

hipError_t launch_tally(const uint8_t* verdict, const uint32_t* sender, const uint64_t* batch_off, uint64_t n_batches,
                        uint32_t n_nodes, uint32_t quorum, uint32_t* votes, uint8_t* reached, hipStream_t s) {
  if (n_batches == 0) return hipSuccess;
  const uint64_t blocks = (n_batches * 64 + 255) / 256;
  hipLaunchKernelGGL(k_tally, dim3((uint32_t)blocks), dim3(256), 0, s, verdict, sender, batch_off, n_batches, n_nodes,
                     quorum, votes, reached);
  return hipGetLastError();
}

// ------------------------------------------------------- synthetic workload
// tag || cfg || u64le(i) [|| u64le(c)] hashed with SHA-512 (single block);
// spec restated in plenum_gpu/synth.py, checked by tests/test_gpu_synth.py.
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

__global__ void k_synth(uint32_t cfg, uint64_t first, uint64_t n, uint32_t key_mod, uint32_t mlen,
                        uint64_t* __restrict__ off_out, uint8_t* __restrict__ seeds_out,
                        uint8_t* __restrict__ tamper_out) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j > n) return;
  off_out[j] = j * (uint64_t)mlen;
  if (j == n) return;
  const uint64_t i = first + j;
  uint32_t w[16], d[16];
  int nb = put_tag(w, "plenum-gpu/key", 14, cfg, key_mod ? i % key_mod : i, false, 0);
  sha512_short(d, w, nb);
  store8(seeds_out + 32 * j, d);
  nb = put_tag(w, "plenum-gpu/tamper", 17, cfg, i, false, 0);
  sha512_short(d, w, nb);
  tamper_out[j] = d[0] < 214748365u ? 1 : 0;
}

__global__ void k_synth_fill(uint32_t cfg, uint64_t first, uint64_t n, const uint64_t* __restrict__ off,
                             uint8_t* __restrict__ blob) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint64_t i = first + j;
  const uint64_t o = off[j], len = off[j + 1] - o;
  uint32_t w[16], d[16];
  for (uint64_t c = 0; c * 64 < len; ++c) {
    const int nb = put_tag(w, "plenum-gpu/msg", 14, cfg, i, true, c);
    sha512_short(d, w, nb);
    for (int k = 0; k < 64 && c * 64 + k < len; ++k) blob[o + c * 64 + k] = (uint8_t)(d[k >> 2] >> (8 * (k & 3)));
  }
}

__global__ void k_tamper(uint64_t first, uint64_t n, const uint8_t* __restrict__ tamper,
                         const uint64_t* __restrict__ off, uint8_t* __restrict__ blob, uint8_t* __restrict__ sig) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n || !tamper[j]) return;
  const uint64_t i = first + j;
  const uint64_t o = off[j], len = off[j + 1] - o;
  const uint8_t bit = (uint8_t)(1u << (i % 8));
  const uint64_t kind = i % 3;
  if (kind == 0 && len > 0) blob[o + (i / 3) % len] ^= bit;
  else if (kind == 1 || (kind == 0 && len == 0)) sig[64 * j + (i / 3) % 32] ^= bit;
  else sig[64 * j + 32 + (i / 3) % 16] ^= bit;
}

hipError_t launch_synth(uint32_t cfg, uint64_t first, uint64_t n, uint32_t key_mod, uint32_t mlen_fixed, uint32_t,
                        uint32_t, uint64_t* off_out, uint8_t* seeds_out, uint8_t* tamper_out, hipStream_t s) {
  const uint64_t blocks = (n + 1 + 255) / 256;
  hipLaunchKernelGGL(k_synth, dim3((uint32_t)blocks), dim3(256), 0, s, cfg, first, n, key_mod, mlen_fixed, off_out,
                     seeds_out, tamper_out);
  return hipGetLastError();
}

hipError_t launch_synth_fill(uint32_t cfg, uint64_t first, uint64_t n, const uint64_t* off, uint8_t* blob,
                             hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(k_synth_fill, dim3((uint32_t)blocks), dim3(256), 0, s, cfg, first, n, off, blob);
  return hipGetLastError();
}

hipError_t launch_tamper(uint64_t first, uint64_t n, const uint8_t* tamper, const uint64_t* off, uint8_t* blob,
                         uint8_t* sig, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(k_tamper, dim3((uint32_t)blocks), dim3(256), 0, s, first, n, tamper, off, blob, sig);
  return hipGetLastError();
}

}  // namespace pv
