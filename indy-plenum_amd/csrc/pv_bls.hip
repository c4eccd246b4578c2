// BLS COMMIT check on the GPU -- kernels and C-ABI
// (include/plenum_verify.h, "BLS COMMIT check").
//
// Reference path: every COMMIT's BLS signature is checked by
//   BlsBftReplicaPlenum.validate_commit -> _validate_signature
//     (plenum/bls/bls_bft_replica_plenum.py:55-75, 194-213)
//   -> BlsCryptoVerifierIndyCrypto.verify_sig (crypto/bls/indy_crypto/bls_crypto_indy_crypto.py:73-82)
//   -> python-ursa Bls.verify: e(sigma, g) == e(H(m), pk) over AMCL BN254.
// Here one lane runs one check as e(sigma, g) e(-H(m), pk) == 1: a product of
// two Miller loops over PRECOMPUTED lines of the fixed G2 arguments (the
// generator and the node keys, k_bls_lines) and one final exponentiation
// (csrc/pv_bn254.h).  Checks are grouped by key so that each wave reads ONE
// key's lines (wave-uniform addresses: one L2 line serves 64 lanes), and each
// distinct message is hashed to G1 once (k_bls_hash).
//
// PARITY UNPINNED: ursa / AMCL are absent here and the reference holds no BLS
// vector; the checker is oracle/bn254_oracle.c.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <atomic>
#include <mutex>
#include <vector>

#include "../../include/plenum_verify.h"
#include "pv_bn254.h"
#include "pv_bn254_pair.h"
#include "pv_sha256.h"

// a named namespace: profilers show the kernels as pvbls::k_bls_*
namespace pvbls {

using namespace bn;

constexpr int KEY_LINE_WORDS = N_LINES * LINE_WORDS;   // 2800 words per G2 point
constexpr int MSG_WORDS = 4 * NL;                        // x_H, y_H, xq(-H), yq(-H)
constexpr int BLS_BLOCK = 256;
#if defined(__HIP_DEVICE_COMPILE__) && !defined(PV_BN_MILLER_REGS)
static_assert(BLS_BLOCK == bn::MF_LANES && BLS_BLOCK == 2 * bn::MP_CHECKS,
              "the Miller loop's LDS accumulator is laid out per check block");
#endif
// the check kernel: one check per lane PAIR at 2 waves per SIMD
// (k_bls_verify_pair, pv_bn254_pair.h); -DPV_BLS_ONE_LANE builds the one-lane
// kernel k_bls_verify (512 registers, 1 wave per SIMD) for A/B timing
#ifdef PV_BLS_ONE_LANE
constexpr uint32_t BLS_WAVE_CHECKS = 64;   // checks per wave (= the key segments' padding)
#else
constexpr uint32_t BLS_WAVE_CHECKS = 32;
#endif
// calls of at most pv_tuning.bls_quad_max checks (default PV_BLS_QUAD_MAX) run
// one check per lane QUAD (k_bls_verify_quad: the two Miller loops on two lane
// pairs, the final exponentiation's products split over both, 16 checks per
// wave): a lone check's chain is ~30 % shorter, the total work larger (the
// Miller loop's squarings run on both pairs); from ~50k checks the pair kernel
// is faster (profiles/r04g_bls_latency_quad_threshold.jsonl)
#ifndef PV_BLS_QUAD_MAX
#define PV_BLS_QUAD_MAX 32768
#endif
std::atomic<uint64_t> g_quad_max{PV_BLS_QUAD_MAX};
void set_quad_max(uint64_t n) { g_quad_max.store(n); }
constexpr uint32_t BLS_QUAD_CHECKS = 16;
// calls of at most pv_tuning.bls_oct_max checks (default PV_BLS_OCT_MAX) run one
// check per lane OCTET (k_bls_verify_oct: the quad schedule with every step's
// products split between two quads, 8 checks per wave): the shortest chain, the
// most work per check
#ifndef PV_BLS_OCT_MAX
#define PV_BLS_OCT_MAX 4096
#endif
std::atomic<uint64_t> g_oct_max{PV_BLS_OCT_MAX};
void set_oct_max(uint64_t n) { g_oct_max.store(n); }
constexpr uint32_t BLS_OCT_CHECKS = 8;

__device__ __forceinline__ void st_fp(uint32_t* w, const fp& a) {
#pragma unroll
  for (int i = 0; i < NL; ++i) w[i] = (uint32_t)a.l[i];
}
__device__ __forceinline__ fp ld_fp(const uint32_t* w) {
  fp r;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.l[i] = (int32_t)w[i];
  return r;
}

// one lane per G2 point: status + the 70 lines of the generator (point 0) and the keys
__global__ __launch_bounds__(64) void k_bls_lines(const uint8_t* __restrict__ pts, uint32_t n, uint32_t* __restrict__ lines,
                                                  uint8_t* __restrict__ status) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  g2a q;
  const int st = g2_decode(pts + 128ull * i, q);
  status[i] = (uint8_t)st;
  uint32_t* out = lines + (uint64_t)KEY_LINE_WORDS * i;
  if (st == 0) {
    g2_lines(out, q);
  } else {
    for (int k = 0; k < KEY_LINE_WORDS; ++k) out[k] = 0;
  }
}

// one lane per distinct message: H(m) and (x/y, 1/y) of -H(m)
__device__ __forceinline__ void hash_one(const uint8_t* __restrict__ blob, const uint64_t* __restrict__ off, uint32_t i,
                                         uint32_t* __restrict__ tab) {
  uint32_t d[8];
  pv::sha256_msg(d, blob + off[i], off[i + 1] - off[i], 0, 0);
  fp x, y, xq, yq;
  hash_to_g1(reinterpret_cast<const uint8_t*>(d), x, y);
  line_point(x, y, true, xq, yq);
  uint32_t* t = tab + (uint64_t)MSG_WORDS * i;
  st_fp(t, x);
  st_fp(t + NL, y);
  st_fp(t + 2 * NL, xq);
  st_fp(t + 3 * NL, yq);
}
__global__ __launch_bounds__(64) void k_bls_hash(const uint8_t* __restrict__ blob, const uint64_t* __restrict__ off,
                                                 uint32_t n, uint32_t* __restrict__ tab) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) hash_one(blob, off, i, tab);
}

// grouping by key: count, padded segment starts (aligned to the checks per wave), scatter
// a check whose key index is out of range is never scheduled: its verdict stays 0
// Key sets of at most GROUP_LOCAL_KEYS keys (node keys: 4..100s) are counted per
// block in LDS first, GROUP_PER_THREAD checks per thread, so that a 25-key set
// takes one global atomic per key per 2,048 checks instead of one per check (2.5M
// atomics on 25 addresses serialised in L2: 2.7 ms each for count and scatter).
constexpr uint32_t GROUP_LOCAL_KEYS = 2048;
constexpr int GROUP_PER_THREAD = 8;
constexpr uint32_t GROUP_BLOCK = 256;
__global__ __launch_bounds__(GROUP_BLOCK) void k_bls_count(const uint32_t* __restrict__ key_idx, uint64_t n,
                                                           uint32_t nkeys, uint32_t* __restrict__ cnt) {
  __shared__ uint32_t lc[GROUP_LOCAL_KEYS];
  const uint64_t base = (uint64_t)blockIdx.x * GROUP_BLOCK * GROUP_PER_THREAD + threadIdx.x;
  if (nkeys > GROUP_LOCAL_KEYS) {   // block-uniform: global atomics per check
    for (int e = 0; e < GROUP_PER_THREAD; ++e) {
      const uint64_t i = base + (uint64_t)e * GROUP_BLOCK;
      if (i < n && key_idx[i] < nkeys) atomicAdd(cnt + key_idx[i], 1u);
    }
    return;
  }
  for (uint32_t k = threadIdx.x; k < nkeys; k += GROUP_BLOCK) lc[k] = 0;
  __syncthreads();
  for (int e = 0; e < GROUP_PER_THREAD; ++e) {
    const uint64_t i = base + (uint64_t)e * GROUP_BLOCK;
    if (i < n) {
      const uint32_t key = key_idx[i];
      if (key < nkeys) atomicAdd(&lc[key], 1u);
    }
  }
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < nkeys; k += GROUP_BLOCK)
    if (lc[k]) atomicAdd(cnt + k, lc[k]);
}

__global__ void k_bls_segments(const uint32_t* __restrict__ cnt, uint32_t k, uint32_t pad, uint32_t* __restrict__ seg,
                               uint32_t* __restrict__ total) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint32_t s = 0;
  for (uint32_t j = 0; j < k; ++j) {
    seg[j] = s;
    s += (cnt[j] + pad - 1) & ~(pad - 1);
  }
  *total = s;
}

// scatter: each check's rank within its block and key from an LDS atomic, one
// global atomic per key per block reserves the block's range of the key's segment
__global__ __launch_bounds__(GROUP_BLOCK) void k_bls_scatter(const uint32_t* __restrict__ key_idx, uint64_t n,
                                                             uint32_t nkeys, const uint32_t* __restrict__ seg,
                                                             uint32_t* __restrict__ cursor,
                                                             uint32_t* __restrict__ order) {
  __shared__ uint32_t lc[GROUP_LOCAL_KEYS];
  const uint64_t base = (uint64_t)blockIdx.x * GROUP_BLOCK * GROUP_PER_THREAD + threadIdx.x;
  if (nkeys > GROUP_LOCAL_KEYS) {   // block-uniform: global atomics per check
    for (int e = 0; e < GROUP_PER_THREAD; ++e) {
      const uint64_t i = base + (uint64_t)e * GROUP_BLOCK;
      if (i >= n) continue;
      const uint32_t key = key_idx[i];
      if (key < nkeys) order[seg[key] + atomicAdd(cursor + key, 1u)] = (uint32_t)i;
    }
    return;
  }
  for (uint32_t k = threadIdx.x; k < nkeys; k += GROUP_BLOCK) lc[k] = 0;
  __syncthreads();
  uint32_t key[GROUP_PER_THREAD], rank[GROUP_PER_THREAD];
#pragma unroll
  for (int e = 0; e < GROUP_PER_THREAD; ++e) {
    const uint64_t i = base + (uint64_t)e * GROUP_BLOCK;
    key[e] = i < n ? key_idx[i] : nkeys;
    rank[e] = key[e] < nkeys ? atomicAdd(&lc[key[e]], 1u) : 0u;
  }
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < nkeys; k += GROUP_BLOCK)
    if (lc[k]) lc[k] = seg[k] + atomicAdd(cursor + k, lc[k]);   // the block's first slot of key k
  __syncthreads();
#pragma unroll
  for (int e = 0; e < GROUP_PER_THREAD; ++e)
    if (key[e] < nkeys) order[lc[key[e]] + rank[e]] = (uint32_t)(base + (uint64_t)e * GROUP_BLOCK);
}

#ifdef PV_BLS_ONE_LANE
// one lane per check, one key per wave (slots of `order` padded to 64 per key;
// 0xffffffff = idle lane, which computes on the point at infinity and writes nothing)
__global__ __launch_bounds__(BLS_BLOCK, 1) void k_bls_verify(
    const uint8_t* __restrict__ sig, const uint32_t* __restrict__ msg_idx, const uint32_t* __restrict__ key_idx,
    const uint32_t* __restrict__ order, const uint32_t* __restrict__ total, const uint32_t* __restrict__ msgtab,
    const uint32_t* __restrict__ lines, const uint8_t* __restrict__ kstatus, uint32_t n_msgs,
    uint8_t* __restrict__ verdict) {
  const uint32_t slot = blockIdx.x * BLS_BLOCK + threadIdx.x;
  const uint32_t task0 = __builtin_amdgcn_readfirstlane(slot & ~63u);
  if (task0 >= *total) return;   // whole wave: past the last padded segment
  const uint32_t j = order[slot];
  const bool live = j != 0xffffffffu;
  // lane 0 of a task is always live (segments fill from their start)
  const uint32_t key = __builtin_amdgcn_readfirstlane(live ? key_idx[j] : 0u);
  const uint32_t* g_lines = lines;
  const uint32_t* pk_lines = lines + (uint64_t)KEY_LINE_WORDS * (1 + key);
  const uint8_t st = kstatus[1 + key];
  fp xs, ys, xqh = fzero(), yqh = fzero();
  bool s_inf = true;
  const bool msg_ok = live && msg_idx[j] < n_msgs;   // out of range: verdict 0
  if (live) {
    g1_decode(sig + 128ull * j, xs, ys, s_inf);
    const uint32_t* t = msgtab + (uint64_t)MSG_WORDS * (msg_ok ? msg_idx[j] : 0u);
    if (st == 0 && msg_ok) {
      xqh = ld_fp(t + 2 * NL);
      yqh = ld_fp(t + 3 * NL);
    }
  }
  const bool ok = bls_check(xs, ys, s_inf, xqh, yqh, st == 1, g_lines, pk_lines);
  if (live) verdict[j] = (st == 2 || !msg_ok) ? 0 : (uint8_t)ok;
}
#else
// sigma's line point per check, one lane per check (the pair kernel would run
// this chain -- decoding, one inversion -- on both lanes of a pair): word w of
// check i at prep[w * n + i], w = 0..9 x/y, 10..19 1/y, 20 = 1 if sigma decodes
// to the point at infinity
constexpr int SIGPREP_WORDS = 2 * NL + 1;
__device__ __forceinline__ void sigprep_one(const uint8_t* __restrict__ sig, uint64_t n, uint64_t i,
                                            uint32_t* __restrict__ prep) {
  fp xs, ys, xq = fzero(), yq = fzero();
  bool inf;
  g1_decode(sig + 128ull * i, xs, ys, inf);
  if (!inf) line_point(xs, ys, false, xq, yq);
#pragma unroll
  for (int w = 0; w < NL; ++w) {
    prep[w * n + i] = (uint32_t)xq.l[w];
    prep[(NL + w) * n + i] = (uint32_t)yq.l[w];
  }
  prep[2 * NL * n + i] = inf ? 1u : 0u;
}
__global__ __launch_bounds__(64) void k_bls_sigprep(const uint8_t* __restrict__ sig, uint64_t n,
                                                    uint32_t* __restrict__ prep) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) sigprep_one(sig, n, i, prep);
}
// a^(r ? E_ISQRT : E_SQRT) with the loop's branches uniform over a lane group
// whose lanes hold both r: a multiply runs where either exponent has a bit (67
// of 253 bits) and only lanes whose own exponent has it keep the product
__device__ __forceinline__ fp pow_root_pair(const fp& a, int r) {
  fp acc = fone(), b = a;
  for (int w = 0; w < 4; ++w) {
    const uint64_t es = E_SQRT[w], ei = E_ISQRT[w];
    for (int k = 0; k < 64; ++k) {
      const bool bs = (es >> k) & 1, bi = (ei >> k) & 1;
      if (bs || bi) {
        const fp t = mul(acc, b);
        if (r ? bi : bs) acc = t;
      }
      if (w < 3 || ((es | ei) >> k) > 1) b = sqr(b);
    }
  }
  return acc;
}
__device__ __forceinline__ fp shfl_fp(const fp& x, int src) {
  fp r;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.l[i] = __shfl(x.l[i], src);
  return r;
}

// small calls: H(m) over a group of 8 lanes per message.  Lane (c, r) = (lg >> 1,
// lg & 1) takes candidate xi + c (+ 4 per round) of hash_to_g1's increment map
// and forms, side by side, y = a^((p+1)/4) (r = 0) and a^((3p-5)/4) (r = 1; = 1/y
// when a = x^3 + 2 is a non-zero square, since the two exponents sum to p - 1):
// the lowest candidate whose a is a non-zero square is hash_to_g1's point (the
// same increment order), and -H's line point (x/y, 1/y) takes no inversion.  The
// serial hash_one runs ~2 square roots and an inversion one after another; this
// chain is one exponentiation.  Control flow is uniform over a group.
__device__ __forceinline__ void hash_group(const uint8_t* __restrict__ blob, const uint64_t* __restrict__ off,
                                           uint32_t i, uint32_t* __restrict__ tab) {
  const int lane = threadIdx.x & 63, lg = lane & 7, base = lane & ~7, r = lg & 1;
  uint32_t d[8];
  pv::sha256_msg(d, blob + off[i], off[i + 1] - off[i], 0, 0);
  fp xi = from_be32(reinterpret_cast<const uint8_t*>(d));
  xi.l[0] += lg >> 1;
  xi = norm(xi);
  for (;;) {
    const fp x = to_mont(xi);
    const fp a = addn(mul(sqr(x), x), cst(TWO_M));
    const fp e = pow_root_pair(a, r);
    const fp o = shfl_fp(e, lane ^ 1);
    const fp y = r ? o : e, yi = r ? e : o;
    const bool ok = eq(sqr(y), a) && !is_zero(a);
    const uint32_t gm = (uint32_t)(__ballot(ok) >> base) & 0xffu;
    if (gm) {
      if (lg == __builtin_ctz(gm)) {   // the winning candidate's r = 0 lane
        const fp yq = negn(yi), xq = mul(x, yq);
        uint32_t* t = tab + (uint64_t)MSG_WORDS * i;
        st_fp(t, x);
        st_fp(t + NL, y);
        st_fp(t + 2 * NL, xq);
        st_fp(t + 3 * NL, yq);
      }
      return;
    }
    xi.l[0] += 4;
    xi = norm(xi);
  }
}

// small calls: the message hashing (blocks [0, hb), 8 lanes per message) and
// sigma's prep (the blocks after, one lane per check) in ONE launch, so that the
// two chains run side by side
__global__ __launch_bounds__(64) void k_bls_prep(const uint8_t* __restrict__ blob, const uint64_t* __restrict__ off,
                                                 uint32_t n_msgs, uint32_t hb, uint32_t* __restrict__ tab,
                                                 const uint8_t* __restrict__ sig, uint64_t n,
                                                 uint32_t* __restrict__ prep) {
  if (blockIdx.x < hb) {
    const uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 3;
    if (i < n_msgs) hash_group(blob, off, (uint32_t)i, tab);
  } else {
    const uint64_t i = (uint64_t)(blockIdx.x - hb) * blockDim.x + threadIdx.x;
    if (i < n) sigprep_one(sig, n, i, prep);
  }
}

// one check per lane PAIR (lanes 2c, 2c + 1), one key per wave (slots of
// `order` padded to 32 per key; 0xffffffff = an idle pair, which computes on the
// point at infinity and writes nothing).  Control flow is pair-uniform: both
// lanes of a pair load the same check and take the same branches.
__global__ __launch_bounds__(BLS_BLOCK, 2) void k_bls_verify_pair(
    const uint8_t* __restrict__ sig, const uint32_t* __restrict__ msg_idx, const uint32_t* __restrict__ key_idx,
    const uint32_t* __restrict__ order, const uint32_t* __restrict__ total, const uint32_t* __restrict__ msgtab,
    const uint32_t* __restrict__ lines, const uint8_t* __restrict__ kstatus, uint32_t n_msgs,
    const uint32_t* __restrict__ prep, uint64_t n, uint8_t* __restrict__ verdict) {
  const uint32_t slot = (blockIdx.x * BLS_BLOCK + threadIdx.x) >> 1;
  const int h = threadIdx.x & 1;
  const uint32_t task0 = __builtin_amdgcn_readfirstlane(slot & ~(BLS_WAVE_CHECKS - 1));
  if (task0 >= *total) return;   // whole wave: past the last padded segment
  const uint32_t j = order[slot];
  const bool live = j != 0xffffffffu;
  // the first pair of a task is always live (segments fill from their start)
  const uint32_t key = __builtin_amdgcn_readfirstlane(live ? key_idx[j] : 0u);
  const uint32_t* g_lines = lines;
  const uint32_t* pk_lines = lines + (uint64_t)KEY_LINE_WORDS * (1 + key);
  const uint8_t st = kstatus[1 + key];
  // this lane's coordinate of each line point: x/y (role 0) or 1/y (role 1)
  p1 q[2] = {{fzero()}, {fzero()}};
  bool s_inf = true;
  const bool msg_ok = live && msg_idx[j] < n_msgs;   // out of range: verdict 0
  if (live) {
#pragma unroll
    for (int w = 0; w < NL; ++w) q[0].e[0].l[w] = (int32_t)prep[(h * NL + w) * n + j];
    s_inf = prep[2 * NL * n + j] != 0;
    const uint32_t* t = msgtab + (uint64_t)MSG_WORDS * (msg_ok ? msg_idx[j] : 0u);
    if (st == 0 && msg_ok) q[1].e[0] = ld_fp(t + (2 + h) * NL);
  }
  const bool ok = bls_check_pair_q(mp_slot(), q, s_inf, st == 1, g_lines, pk_lines);
  if (live && !h) verdict[j] = (st == 2 || !msg_ok) ? 0 : (uint8_t)ok;
}

// one check per lane QUAD (lanes 4c .. 4c + 3; small batches): lane pair 0 runs
// e(sigma, g)'s Miller loop, pair 1 e(-H, pk)'s, each on its own LDS slot; the
// product and the final exponentiation run on both pairs (bls_check_quad_q).
// 16 checks per wave, slots of `order` padded to 16 per key.
__global__ __launch_bounds__(BLS_BLOCK, 2) void k_bls_verify_quad(
    const uint8_t* __restrict__ sig, const uint32_t* __restrict__ msg_idx, const uint32_t* __restrict__ key_idx,
    const uint32_t* __restrict__ order, const uint32_t* __restrict__ total, const uint32_t* __restrict__ msgtab,
    const uint32_t* __restrict__ lines, const uint8_t* __restrict__ kstatus, uint32_t n_msgs,
    const uint32_t* __restrict__ prep, uint64_t n, uint8_t* __restrict__ verdict) {
  const uint32_t slot = (blockIdx.x * BLS_BLOCK + threadIdx.x) >> 2;
  const int h = threadIdx.x & 1, own = (threadIdx.x >> 1) & 1;
  const uint32_t task0 = __builtin_amdgcn_readfirstlane(slot & ~(BLS_QUAD_CHECKS - 1));
  if (task0 >= *total) return;
  const uint32_t j = order[slot];
  const bool live = j != 0xffffffffu;
  const uint32_t key = __builtin_amdgcn_readfirstlane(live ? key_idx[j] : 0u);
  const uint32_t* g_lines = lines;
  const uint32_t* pk_lines = lines + (uint64_t)KEY_LINE_WORDS * (1 + key);
  const uint8_t st = kstatus[1 + key];
  p1 q[2] = {{fzero()}, {fzero()}};   // q[0]: this pair's point (sigma for pair 0, -H for pair 1)
  bool s_inf = true;
  const bool msg_ok = live && msg_idx[j] < n_msgs;
  if (live) {
    s_inf = prep[2 * NL * n + j] != 0;
    if (own == 0) {
#pragma unroll
      for (int w = 0; w < NL; ++w) q[0].e[0].l[w] = (int32_t)prep[(h * NL + w) * n + j];
    } else if (st == 0 && msg_ok) {
      q[0].e[0] = ld_fp(msgtab + (uint64_t)MSG_WORDS * msg_idx[j] + (2 + h) * NL);
    }
  }
  const bool ok = bls_check_quad_q(mp_slot(), q, s_inf, st == 1, g_lines, pk_lines);
  if (live && (threadIdx.x & 3) == 0) verdict[j] = (st == 2 || !msg_ok) ? 0 : (uint8_t)ok;
}

// one check per lane OCTET (lanes 8c .. 8c + 7; the smallest calls): the quad
// kernel's roles (pair 0 e(sigma, g), pair 1 e(-H, pk)) in each of two quads,
// which split every step's Fp2 products between them (bls_check_oct_q).  8
// checks per wave, slots of `order` padded to 8 per key.
__global__ __launch_bounds__(BLS_BLOCK, 2) void k_bls_verify_oct(
    const uint8_t* __restrict__ sig, const uint32_t* __restrict__ msg_idx, const uint32_t* __restrict__ key_idx,
    const uint32_t* __restrict__ order, const uint32_t* __restrict__ total, const uint32_t* __restrict__ msgtab,
    const uint32_t* __restrict__ lines, const uint8_t* __restrict__ kstatus, uint32_t n_msgs,
    const uint32_t* __restrict__ prep, uint64_t n, uint8_t* __restrict__ verdict) {
  const uint32_t slot = (blockIdx.x * BLS_BLOCK + threadIdx.x) >> 3;
  const int h = threadIdx.x & 1, own = (threadIdx.x >> 1) & 1;
  const uint32_t task0 = __builtin_amdgcn_readfirstlane(slot & ~(BLS_OCT_CHECKS - 1));
  if (task0 >= *total) return;
  const uint32_t j = order[slot];
  const bool live = j != 0xffffffffu;
  const uint32_t key = __builtin_amdgcn_readfirstlane(live ? key_idx[j] : 0u);
  const uint32_t* g_lines = lines;
  const uint32_t* pk_lines = lines + (uint64_t)KEY_LINE_WORDS * (1 + key);
  const uint8_t st = kstatus[1 + key];
  p1 q[2] = {{fzero()}, {fzero()}};   // q[0]: this pair's point (sigma for pair 0, -H for pair 1)
  bool s_inf = true;
  const bool msg_ok = live && msg_idx[j] < n_msgs;
  if (live) {
    s_inf = prep[2 * NL * n + j] != 0;
    if (own == 0) {
#pragma unroll
      for (int w = 0; w < NL; ++w) q[0].e[0].l[w] = (int32_t)prep[(h * NL + w) * n + j];
    } else if (st == 0 && msg_ok) {
      q[0].e[0] = ld_fp(msgtab + (uint64_t)MSG_WORDS * msg_idx[j] + (2 + h) * NL);
    }
  }
  const bool ok = bls_check_oct_q(q, s_inf, st == 1, g_lines, pk_lines);
  if (live && (threadIdx.x & 7) == 0) verdict[j] = (st == 2 || !msg_ok) ? 0 : (uint8_t)ok;
}
#endif

// Bls::verify_multi_sig's aggregated key (ursa: PointG2::new_inf() + every
// ver_key.point): one lane per check sums its keys (each decoded as
// ECP2::frombytes: off the twist = O) and writes the sum's 128-byte affine
// representation at pts[1 + i]; O is written as 128 zero bytes, which decode off
// the twist (0 != 2/(1+i)), i.e. back to O.  k_bls_lines then prepares the sums
// like keys (status, subgroup check, lines).
__global__ __launch_bounds__(64) void k_bls_agg_g2(const uint8_t* __restrict__ pks, const uint64_t* __restrict__ set_off,
                                                   uint32_t m, uint8_t* __restrict__ pts) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  g2j acc{f2one(), f2one(), f2zero()};
  for (uint64_t t = set_off[i]; t < set_off[i + 1]; ++t) {
    g2a q;
    if (g2_decode(pks + 128ull * t, q, false) != 0) continue;
    acc = g2j_add(acc, g2j{q.x, q.y, f2one()});
  }
  uint8_t* out = pts + 128ull * (1 + i);
  for (int b = 0; b < 128; ++b) out[b] = 0;
  if (f2is_zero(acc.z)) return;
  const fp2 zi = f2inv(acc.z), zi2 = f2sqr(zi);
  const fp2 x = f2mul(acc.x, zi2), y = f2mul(acc.y, f2mul(zi2, zi));
  to_be32(out, from_mont(x.a));
  to_be32(out + 32, from_mont(x.b));
  to_be32(out + 64, from_mont(y.a));
  to_be32(out + 96, from_mont(y.b));
}

// MultiSignature::new (ursa: PointG1::new_inf() + every signature's point, each
// decoded as ECP::frombytes) -> its 128-byte representation (ECP::tobytes,
// uncompressed: 0x04|x|y; O as AMCL's (x, y) = (0, 1) of its infinity)
__global__ __launch_bounds__(64) void k_bls_agg_g1(const uint8_t* __restrict__ sigs, const uint64_t* __restrict__ set_off,
                                                   uint32_t m, uint8_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  g1j acc{fone(), fone(), fzero()};
  bool inf = true;
  for (uint64_t t = set_off[i]; t < set_off[i + 1]; ++t) {
    fp x, y;
    bool s_inf;
    g1_decode(sigs + 128ull * t, x, y, s_inf);
    if (!s_inf) acc = g1j_add_affine(acc, inf, x, y);
  }
  uint8_t* o = out + 128ull * i;
  for (int b = 0; b < 128; ++b) o[b] = 0;
  o[0] = 4;
  if (inf || is_zero(acc.z)) {
    o[64] = 1;
    return;
  }
  const fp zi = inv(acc.z), zi2 = sqr(zi);
  to_be32(o + 1, from_mont(mul(acc.x, zi2)));
  to_be32(o + 33, from_mont(mul(acc.y, mul(zi2, zi))));
}

// data generation: sig[j] = sk[key_idx[j]] * H(msg_idx[j])
__global__ __launch_bounds__(64) void k_bls_sign(const uint8_t* __restrict__ sks, const uint32_t* __restrict__ msgtab,
                                                 const uint32_t* __restrict__ msg_idx,
                                                 const uint32_t* __restrict__ key_idx, uint64_t n,
                                                 uint8_t* __restrict__ sig) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint32_t* t = msgtab + (uint64_t)MSG_WORDS * msg_idx[j];
  g1_sign(sig + 128 * j, ld_fp(t), ld_fp(t + NL), sks + 32ull * key_idx[j]);
}

// pk = sk * g (G2, one lane per key; bench / test data generation)
__global__ __launch_bounds__(64) void k_bls_pubkeys(const uint8_t* __restrict__ gen, const uint8_t* __restrict__ sks,
                                                    uint32_t k, uint8_t* __restrict__ pks) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= k) return;
  g2a g;
  g2_decode(gen, g, false);
  g2j acc{f2one(), f2one(), f2zero()};
  const g2j G{g.x, g.y, f2one()};
  const uint8_t* s = sks + 32ull * i;
  for (int b = 0; b < 256; ++b) {
    acc = g2j_dbl(acc);
    if ((s[b >> 3] >> (7 - (b & 7))) & 1) acc = g2j_add(acc, G);
  }
  uint8_t* out = pks + 128ull * i;
  for (int b = 0; b < 128; ++b) out[b] = 0;
  if (f2is_zero(acc.z)) return;
  const fp2 zi = f2inv(acc.z), zi2 = f2sqr(zi);
  const fp2 x = f2mul(acc.x, zi2), y = f2mul(acc.y, f2mul(zi2, zi));
  to_be32(out, from_mont(x.a));
  to_be32(out + 32, from_mont(x.b));
  to_be32(out + 64, from_mont(y.a));
  to_be32(out + 96, from_mont(y.b));
}

// ------------------------------------------------------------------ host side
thread_local char g_bls_err[512];

int bfail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_bls_err, sizeof g_bls_err, fmt, ap);
  va_end(ap);
  return code;
}

#define BLS_HIP(expr)                                                                                          \
  do {                                                                                                         \
    hipError_t e_ = (expr);                                                                                    \
    if (e_ != hipSuccess)                                                                                      \
      return bfail(e_ == hipErrorOutOfMemory ? PV_ENOMEM : PV_EIO, "%s failed: %s (%s:%d)", #expr,             \
                   hipGetErrorString(e_), __FILE__, __LINE__);                                                 \
  } while (0)

template <typename T>
struct Buf {
  T* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t n) {
    if (n <= cap && p) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    const size_t want = n < 64 ? 64 : n;
    const hipError_t e = hipMalloc(reinterpret_cast<void**>(&p), want * sizeof(T));
    if (e == hipSuccess) cap = want;
    return e;
  }
  // grow to >= n elements keeping the first `keep` (device copy on stream s,
  // synchronised): the incremental key set (pv_bls_add_keys)
  hipError_t grow_keep(size_t n, size_t keep, hipStream_t s) {
    if (n <= cap && p) return hipSuccess;
    size_t want = cap ? cap : 64;
    while (want < n) want *= 2;
    T* q = nullptr;
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&q), want * sizeof(T));
    if (e != hipSuccess) return e;
    if (keep && p) {
      e = hipMemcpyAsync(q, p, keep * sizeof(T), hipMemcpyDeviceToDevice, s);
      if (e == hipSuccess) e = hipStreamSynchronize(s);
      if (e != hipSuccess) {
        (void)hipFree(q);
        return e;
      }
    }
    if (p) (void)hipFree(p);
    p = q;
    cap = want;
    return hipSuccess;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

// a prepared set of G2 arguments: point 0 = the generator, points 1..nkeys the
// keys (or, for multi-signature checks, the per-check aggregated keys)
struct KeySet {
  uint32_t nkeys = 0;             // lines of 1 + nkeys points are valid (0: no set)
  bool gen_ok = false;            // point 0 (the generator) prepared: pv_bls_add_keys may append
  uint64_t points_prepared = 0;   // points k_bls_lines prepared for this set, cumulative (pv_bls_keyset_info)
  Buf<uint32_t> lines;
  Buf<uint8_t> kstatus, pts;
  void release() {
    nkeys = 0;
    gen_ok = false;
    lines.release();
    kstatus.release();
    pts.release();
  }
};

struct BlsDev {
  int ord = -1;
  hipStream_t stream = nullptr;
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  KeySet keys;                    // pv_bls_set_keys
  KeySet multi;                   // per call of pv_bls_verify_multi_batch
  // per-call workspaces
  Buf<uint32_t> msgtab, cnt, seg, cursor, order, total, midx, kidx, sigprep;
  Buf<uint8_t> sig, blob, verdict, sks, mpks;
  Buf<uint64_t> off, moff;
  float ms_hash = 0, ms_verify = 0;
};

std::mutex g_bls_mu;
std::vector<BlsDev> g_bls;

int bls_dev(int device, BlsDev** out) {
  for (auto& d : g_bls)
    if (d.ord == device) {
      *out = &d;
      return PV_OK;
    }
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count)
    return bfail(PV_ENODEV, "HIP device %d not available", device);
  g_bls.emplace_back();
  BlsDev& d = g_bls.back();
  d.ord = device;
  BLS_HIP(hipSetDevice(device));
  BLS_HIP(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
  for (auto& e : d.ev) BLS_HIP(hipEventCreate(&e));
  *out = &d;
  return PV_OK;
}

struct Guard {
  int prev = -1;
  Guard() { (void)hipGetDevice(&prev); }
  ~Guard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

unsigned blocks_for(uint64_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }

// grouping + verify on device buffers against key set `ks`, on stream s.
// Verdicts of checks the kernels skip (key index out of range) stay 0.
int enqueue_verify(BlsDev& d, const KeySet& ks, const uint8_t* sig, const uint8_t* blob, const uint64_t* off,
                   uint64_t n_msgs, const uint32_t* msg_idx, const uint32_t* key_idx, uint64_t n, uint8_t* verdict,
                   hipStream_t s) {
  if (!ks.nkeys) return bfail(PV_ENOTINIT, "no BLS key set on device %d (call pv_bls_set_keys)", d.ord);
  if (n > 0x7fffffffull - 64ull * ks.nkeys) return bfail(PV_EINVAL, "too many checks in one call");
  if (n_msgs > 0xffffffffull) return bfail(PV_EINVAL, "too many messages in one call");
#ifdef PV_BLS_ONE_LANE
  const uint32_t pad = BLS_WAVE_CHECKS;
#else
  const bool oct = n <= g_oct_max.load();
  const bool quad = !oct && n <= g_quad_max.load();
  const uint32_t pad = oct ? BLS_OCT_CHECKS : quad ? BLS_QUAD_CHECKS : BLS_WAVE_CHECKS;
#endif
  const uint64_t slots = ((n + pad - 1) / pad + ks.nkeys) * pad;
  BLS_HIP(d.msgtab.ensure(n_msgs * MSG_WORDS));
  BLS_HIP(d.cnt.ensure(ks.nkeys));
  BLS_HIP(d.cursor.ensure(ks.nkeys));
  BLS_HIP(d.seg.ensure(ks.nkeys));
  BLS_HIP(d.total.ensure(1));
  BLS_HIP(d.order.ensure(slots));
#ifndef PV_BLS_ONE_LANE
  BLS_HIP(d.sigprep.ensure(n * SIGPREP_WORDS));
#endif
  BLS_HIP(hipEventRecord(d.ev[0], s));
#ifndef PV_BLS_ONE_LANE
  if (quad || oct) {   // message hashing and sigma's prep in one launch (both timed as "hash")
    const uint32_t hb = blocks_for(8 * n_msgs, 64);
    if (n_msgs || n)
      hipLaunchKernelGGL(k_bls_prep, dim3(hb + blocks_for(n, 64)), dim3(64), 0, s, blob, off, (uint32_t)n_msgs, hb,
                         d.msgtab.p, sig, n, d.sigprep.p);
  } else
#endif
  if (n_msgs) hipLaunchKernelGGL(k_bls_hash, dim3(blocks_for(n_msgs, 64)), dim3(64), 0, s, blob, off, (uint32_t)n_msgs,
                                 d.msgtab.p);
  BLS_HIP(hipGetLastError());
  BLS_HIP(hipEventRecord(d.ev[1], s));
  BLS_HIP(hipMemsetAsync(verdict, 0, n, s));
  BLS_HIP(hipMemsetAsync(d.cnt.p, 0, ks.nkeys * 4, s));
  BLS_HIP(hipMemsetAsync(d.cursor.p, 0, ks.nkeys * 4, s));
  BLS_HIP(hipMemsetAsync(d.order.p, 0xff, slots * 4, s));
  const unsigned gblocks = blocks_for(n, GROUP_BLOCK * GROUP_PER_THREAD);
  if (gblocks)
    hipLaunchKernelGGL(k_bls_count, dim3(gblocks), dim3(GROUP_BLOCK), 0, s, key_idx, n, ks.nkeys, d.cnt.p);
  hipLaunchKernelGGL(k_bls_segments, dim3(1), dim3(64), 0, s, d.cnt.p, ks.nkeys, pad, d.seg.p, d.total.p);
  if (gblocks)
    hipLaunchKernelGGL(k_bls_scatter, dim3(gblocks), dim3(GROUP_BLOCK), 0, s, key_idx, n, ks.nkeys, d.seg.p,
                     d.cursor.p, d.order.p);
  BLS_HIP(hipGetLastError());
  BLS_HIP(hipEventRecord(d.ev[2], s));
#ifdef PV_BLS_ONE_LANE
  hipLaunchKernelGGL(k_bls_verify, dim3(blocks_for(slots, BLS_BLOCK)), dim3(BLS_BLOCK), 0, s, sig, msg_idx, key_idx,
                     d.order.p, d.total.p, d.msgtab.p, ks.lines.p, ks.kstatus.p, (uint32_t)n_msgs, verdict);
#else
  if (n && !quad && !oct) hipLaunchKernelGGL(k_bls_sigprep, dim3(blocks_for(n, 64)), dim3(64), 0, s, sig, n, d.sigprep.p);
  if (oct)
    hipLaunchKernelGGL(k_bls_verify_oct, dim3(blocks_for(8 * slots, BLS_BLOCK)), dim3(BLS_BLOCK), 0, s, sig, msg_idx,
                       key_idx, d.order.p, d.total.p, d.msgtab.p, ks.lines.p, ks.kstatus.p, (uint32_t)n_msgs,
                       d.sigprep.p, n, verdict);
  else if (quad)
    hipLaunchKernelGGL(k_bls_verify_quad, dim3(blocks_for(4 * slots, BLS_BLOCK)), dim3(BLS_BLOCK), 0, s, sig, msg_idx,
                       key_idx, d.order.p, d.total.p, d.msgtab.p, ks.lines.p, ks.kstatus.p, (uint32_t)n_msgs,
                       d.sigprep.p, n, verdict);
  else
    hipLaunchKernelGGL(k_bls_verify_pair, dim3(blocks_for(2 * slots, BLS_BLOCK)), dim3(BLS_BLOCK), 0, s, sig, msg_idx,
                       key_idx, d.order.p, d.total.p, d.msgtab.p, ks.lines.p, ks.kstatus.p, (uint32_t)n_msgs,
                       d.sigprep.p, n, verdict);
#endif
  BLS_HIP(hipGetLastError());
  BLS_HIP(hipEventRecord(d.ev[3], s));
  return PV_OK;
}

// host-side argument checks of the host-buffer entry points: offsets
// non-decreasing, message indices in range
int check_messages(const uint64_t* msg_off, uint64_t n_msgs, const uint32_t* msg_idx, uint64_t n) {
  for (uint64_t i = 0; i < n_msgs; ++i)
    if (msg_off[i + 1] < msg_off[i]) return bfail(PV_EINVAL, "msg_off not monotone at %llu", (unsigned long long)i);
  for (uint64_t j = 0; j < n; ++j)
    if (msg_idx[j] >= n_msgs) return bfail(PV_EINVAL, "msg_idx[%llu] = %u out of range", (unsigned long long)j, msg_idx[j]);
  return PV_OK;
}

// messages to the device workspace (offsets rebased to 0, 64 zero bytes of tail pad)
int upload_messages(BlsDev& d, const uint8_t* msg_blob, const uint64_t* msg_off, uint64_t n_msgs, hipStream_t s,
                    std::vector<uint64_t>& off) {
  const uint64_t b0 = msg_off[0], bytes = msg_off[n_msgs] - b0;
  BLS_HIP(d.blob.ensure(bytes + 64));
  BLS_HIP(d.off.ensure(n_msgs + 1));
  off.resize(n_msgs + 1);
  for (uint64_t i = 0; i <= n_msgs; ++i) off[i] = msg_off[i] - b0;
  if (bytes) BLS_HIP(hipMemcpyAsync(d.blob.p, msg_blob + b0, bytes, hipMemcpyHostToDevice, s));
  BLS_HIP(hipMemsetAsync(d.blob.p + bytes, 0, 64, s));
  BLS_HIP(hipMemcpyAsync(d.off.p, off.data(), (n_msgs + 1) * 8, hipMemcpyHostToDevice, s));
  return PV_OK;
}

int collect_times(BlsDev& d) {
  BLS_HIP(hipEventSynchronize(d.ev[3]));
  BLS_HIP(hipEventElapsedTime(&d.ms_hash, d.ev[0], d.ev[1]));
  BLS_HIP(hipEventElapsedTime(&d.ms_verify, d.ev[2], d.ev[3]));
  return PV_OK;
}

}  // namespace pvbls

using namespace pvbls;

extern "C" {

const char* pv_bls_last_error(void) { return g_bls_err; }

int pv_bls_set_keys(const uint8_t* gen, const uint8_t* pks, uint64_t k, uint8_t* status, int device) {
  std::lock_guard<std::mutex> lk(g_bls_mu);
  Guard gd;
  if (!gen || (k && !pks)) return bfail(PV_EINVAL, "null buffer");
  if (k > 65535) return bfail(PV_EINVAL, "at most 65535 keys per set (got %llu)", (unsigned long long)k);
  BlsDev* d = nullptr;
  if (int rc = bls_dev(device, &d)) return rc;
  // the old set is gone from here on: a failure below leaves NO set (verify ->
  // PV_ENOTINIT), never a key count over freed or half-written tables
  d->keys.nkeys = 0;
  d->keys.gen_ok = false;
  BLS_HIP(hipSetDevice(device));
  KeySet& ks = d->keys;
  const uint64_t np = k + 1;
  BLS_HIP(ks.pts.ensure(np * 128));
  BLS_HIP(ks.lines.ensure(np * KEY_LINE_WORDS));
  BLS_HIP(ks.kstatus.ensure(np));
  BLS_HIP(hipMemcpyAsync(ks.pts.p, gen, 128, hipMemcpyHostToDevice, d->stream));
  if (k) BLS_HIP(hipMemcpyAsync(ks.pts.p + 128, pks, k * 128, hipMemcpyHostToDevice, d->stream));
  hipLaunchKernelGGL(k_bls_lines, dim3(blocks_for(np, 64)), dim3(64), 0, d->stream, ks.pts.p, (uint32_t)np, ks.lines.p,
                     ks.kstatus.p);
  BLS_HIP(hipGetLastError());
  std::vector<uint8_t> st(np);
  BLS_HIP(hipMemcpyAsync(st.data(), ks.kstatus.p, np, hipMemcpyDeviceToHost, d->stream));
  BLS_HIP(hipStreamSynchronize(d->stream));
  if (st[0] != 0) return bfail(PV_EINVAL, "the generator is not a point of order r on the twist (status %d)", st[0]);
  ks.nkeys = (uint32_t)k;
  ks.gen_ok = true;
  ks.points_prepared += np;
  if (status) memcpy(status, st.data() + 1, k);
  return PV_OK;
}

int pv_bls_add_keys(const uint8_t* pks, uint64_t k, uint8_t* status, uint64_t* first, int device) {
  std::lock_guard<std::mutex> lk(g_bls_mu);
  Guard gd;
  if (k && !pks) return bfail(PV_EINVAL, "null buffer");
  BlsDev* d = nullptr;
  if (int rc = bls_dev(device, &d)) return rc;
  KeySet& ks = d->keys;
  if (!ks.gen_ok)
    return bfail(PV_ENOTINIT, "no BLS key set on device %d (call pv_bls_set_keys)", device);
  const uint64_t old = ks.nkeys;
  if (old > 65535 || k > 65535 - old)   // no wrap for any k
    return bfail(PV_EINVAL, "at most 65535 keys per set (%llu + %llu)", (unsigned long long)old,
                 (unsigned long long)k);
  if (first) *first = old;
  if (k == 0) return PV_OK;
  BLS_HIP(hipSetDevice(device));
  // the prepared points 0..old keep their lines; a failed growth leaves the set as it was
  const uint64_t np = old + 1 + k;
  BLS_HIP(ks.pts.grow_keep(np * 128, (old + 1) * 128, d->stream));
  BLS_HIP(ks.lines.grow_keep(np * KEY_LINE_WORDS, (old + 1) * KEY_LINE_WORDS, d->stream));
  BLS_HIP(ks.kstatus.grow_keep(np, old + 1, d->stream));
  BLS_HIP(hipMemcpyAsync(ks.pts.p + 128 * (old + 1), pks, k * 128, hipMemcpyHostToDevice, d->stream));
  hipLaunchKernelGGL(k_bls_lines, dim3(blocks_for(k, 64)), dim3(64), 0, d->stream, ks.pts.p + 128 * (old + 1),
                     (uint32_t)k, ks.lines.p + (uint64_t)KEY_LINE_WORDS * (old + 1), ks.kstatus.p + old + 1);
  BLS_HIP(hipGetLastError());
  std::vector<uint8_t> st(k);
  BLS_HIP(hipMemcpyAsync(st.data(), ks.kstatus.p + old + 1, k, hipMemcpyDeviceToHost, d->stream));
  BLS_HIP(hipStreamSynchronize(d->stream));
  ks.nkeys = (uint32_t)(old + k);
  ks.points_prepared += k;
  if (status) memcpy(status, st.data(), k);
  return PV_OK;
}

int pv_bls_keyset_info(int device, uint64_t* nkeys, uint64_t* points_prepared) {
  std::lock_guard<std::mutex> lk(g_bls_mu);
  for (auto& d : g_bls)
    if (d.ord == device) {
      if (nkeys) *nkeys = d.keys.nkeys;
      if (points_prepared) *points_prepared = d.keys.points_prepared;
      return PV_OK;
    }
  if (nkeys) *nkeys = 0;
  if (points_prepared) *points_prepared = 0;
  return PV_OK;
}

int pv_bls_verify_batch_device(const uint8_t* sig, const uint8_t* msg_blob, const uint64_t* msg_off, uint64_t n_msgs,
                               const uint32_t* msg_idx, const uint32_t* key_idx, uint64_t n, uint8_t* verdict,
                               int device, void* stream) {
  std::lock_guard<std::mutex> lk(g_bls_mu);
  Guard gd;
  BlsDev* d = nullptr;
  if (int rc = bls_dev(device, &d)) return rc;
  if (n == 0) return PV_OK;
  if (!sig || !msg_off || !msg_idx || !key_idx || !verdict || (n_msgs && !msg_blob)) return bfail(PV_EINVAL, "null buffer");
  BLS_HIP(hipSetDevice(device));
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : d->stream;
  if (int rc = enqueue_verify(*d, d->keys, sig, msg_blob, msg_off, n_msgs, msg_idx, key_idx, n, verdict, s)) return rc;
  BLS_HIP(hipStreamSynchronize(s));
  return collect_times(*d);
}

int pv_bls_verify_batch(const uint8_t* sig, const uint64_t* sig_len, const uint8_t* msg_blob, const uint64_t* msg_off,
                        uint64_t n_msgs, const uint32_t* msg_idx, const uint32_t* key_idx, uint64_t n,
                        uint8_t* verdict, int device) {
  std::lock_guard<std::mutex> lk(g_bls_mu);
  Guard gd;
  BlsDev* d = nullptr;
  if (int rc = bls_dev(device, &d)) return rc;
  if (n == 0) return PV_OK;
  if (!sig || !msg_off || !msg_idx || !key_idx || !verdict || (n_msgs && !msg_blob && msg_off[n_msgs] != msg_off[0]))
    return bfail(PV_EINVAL, "null buffer");
  if (!d->keys.nkeys) return bfail(PV_ENOTINIT, "no BLS key set on device %d (call pv_bls_set_keys)", device);
  // host-side argument checks: every index in range, offsets non-decreasing
  if (int rc = check_messages(msg_off, n_msgs, msg_idx, n)) return rc;
  for (uint64_t j = 0; j < n; ++j)
    if (key_idx[j] >= d->keys.nkeys)
      return bfail(PV_EINVAL, "key_idx[%llu] = %u out of range", (unsigned long long)j, key_idx[j]);
  BLS_HIP(hipSetDevice(device));
  BLS_HIP(d->sig.ensure(n * 128));
  BLS_HIP(d->midx.ensure(n));
  BLS_HIP(d->kidx.ensure(n));
  BLS_HIP(d->verdict.ensure(n));
  hipStream_t s = d->stream;
  std::vector<uint64_t> off;
  if (int rc = upload_messages(*d, msg_blob, msg_off, n_msgs, s, off)) return rc;
  BLS_HIP(hipMemcpyAsync(d->sig.p, sig, n * 128, hipMemcpyHostToDevice, s));
  BLS_HIP(hipMemcpyAsync(d->midx.p, msg_idx, n * 4, hipMemcpyHostToDevice, s));
  BLS_HIP(hipMemcpyAsync(d->kidx.p, key_idx, n * 4, hipMemcpyHostToDevice, s));
  if (int rc = enqueue_verify(*d, d->keys, d->sig.p, d->blob.p, d->off.p, n_msgs, d->midx.p, d->kidx.p, n,
                              d->verdict.p, s))
    return rc;
  BLS_HIP(hipMemcpyAsync(verdict, d->verdict.p, n, hipMemcpyDeviceToHost, s));
  BLS_HIP(hipStreamSynchronize(s));
  // a signature representation that is not 128 bytes does not decode:
  // bls_from_str returns None and verify_sig returns False
  if (sig_len)
    for (uint64_t j = 0; j < n; ++j)
      if (sig_len[j] != 128) verdict[j] = 0;
  return collect_times(*d);
}

int pv_bls_verify_multi_batch(const uint8_t* gen, const uint8_t* sig, const uint64_t* sig_len, const uint8_t* msg_blob,
                              const uint64_t* msg_off, uint64_t n_msgs, const uint32_t* msg_idx, const uint8_t* pks,
                              const uint64_t* pk_off, uint64_t n, uint8_t* verdict, int device) {
  std::lock_guard<std::mutex> lk(g_bls_mu);
  Guard gd;
  BlsDev* d = nullptr;
  if (int rc = bls_dev(device, &d)) return rc;
  if (n == 0) return PV_OK;
  if (!gen || !sig || !msg_off || !msg_idx || !pk_off || !verdict ||
      (n_msgs && !msg_blob && msg_off[n_msgs] != msg_off[0]))
    return bfail(PV_EINVAL, "null buffer");
  if (n > 65535) return bfail(PV_EINVAL, "at most 65535 multi-signature checks per call (got %llu)", (unsigned long long)n);
  if (int rc = check_messages(msg_off, n_msgs, msg_idx, n)) return rc;
  for (uint64_t j = 0; j < n; ++j)
    if (pk_off[j + 1] < pk_off[j]) return bfail(PV_EINVAL, "pk_off not monotone at %llu", (unsigned long long)j);
  const uint64_t p0 = pk_off[0], nk = pk_off[n] - p0;
  if (nk && !pks) return bfail(PV_EINVAL, "null buffer");
  BLS_HIP(hipSetDevice(device));
  KeySet& ks = d->multi;
  ks.nkeys = 0;
  const uint64_t np = n + 1;
  BLS_HIP(ks.pts.ensure(np * 128));
  BLS_HIP(ks.lines.ensure(np * KEY_LINE_WORDS));
  BLS_HIP(ks.kstatus.ensure(np));
  BLS_HIP(d->mpks.ensure(nk * 128));
  BLS_HIP(d->moff.ensure(np));
  BLS_HIP(d->sig.ensure(n * 128));
  BLS_HIP(d->midx.ensure(n));
  BLS_HIP(d->kidx.ensure(n));
  BLS_HIP(d->verdict.ensure(n));
  hipStream_t s = d->stream;
  std::vector<uint64_t> off, poff(np);
  std::vector<uint32_t> kid(n);
  for (uint64_t j = 0; j <= n; ++j) poff[j] = pk_off[j] - p0;
  for (uint64_t j = 0; j < n; ++j) kid[j] = (uint32_t)j;
  if (int rc = upload_messages(*d, msg_blob, msg_off, n_msgs, s, off)) return rc;
  BLS_HIP(hipMemcpyAsync(ks.pts.p, gen, 128, hipMemcpyHostToDevice, s));
  if (nk) BLS_HIP(hipMemcpyAsync(d->mpks.p, pks + 128 * p0, nk * 128, hipMemcpyHostToDevice, s));
  BLS_HIP(hipMemcpyAsync(d->moff.p, poff.data(), np * 8, hipMemcpyHostToDevice, s));
  BLS_HIP(hipMemcpyAsync(d->sig.p, sig, n * 128, hipMemcpyHostToDevice, s));
  BLS_HIP(hipMemcpyAsync(d->midx.p, msg_idx, n * 4, hipMemcpyHostToDevice, s));
  BLS_HIP(hipMemcpyAsync(d->kidx.p, kid.data(), n * 4, hipMemcpyHostToDevice, s));
  // the aggregated key of every check, then its lines (point 0: the generator)
  hipLaunchKernelGGL(k_bls_agg_g2, dim3(blocks_for(n, 64)), dim3(64), 0, s, d->mpks.p, d->moff.p, (uint32_t)n, ks.pts.p);
  hipLaunchKernelGGL(k_bls_lines, dim3(blocks_for(np, 64)), dim3(64), 0, s, ks.pts.p, (uint32_t)np, ks.lines.p,
                     ks.kstatus.p);
  BLS_HIP(hipGetLastError());
  ks.nkeys = (uint32_t)n;
  if (int rc = enqueue_verify(*d, ks, d->sig.p, d->blob.p, d->off.p, n_msgs, d->midx.p, d->kidx.p, n, d->verdict.p, s))
    return rc;
  uint8_t gst = 0xff;
  BLS_HIP(hipMemcpyAsync(verdict, d->verdict.p, n, hipMemcpyDeviceToHost, s));
  BLS_HIP(hipMemcpyAsync(&gst, ks.kstatus.p, 1, hipMemcpyDeviceToHost, s));
  BLS_HIP(hipStreamSynchronize(s));
  if (gst != 0) {
    memset(verdict, 0, n);
    return bfail(PV_EINVAL, "the generator is not a point of order r on the twist (status %d)", gst);
  }
  if (sig_len)
    for (uint64_t j = 0; j < n; ++j)
      if (sig_len[j] != 128) verdict[j] = 0;
  return collect_times(*d);
}

int pv_bls_aggregate_sigs(const uint8_t* sigs, const uint64_t* set_off, uint64_t m, uint8_t* out, int device) {
  std::lock_guard<std::mutex> lk(g_bls_mu);
  Guard gd;
  BlsDev* d = nullptr;
  if (int rc = bls_dev(device, &d)) return rc;
  if (m == 0) return PV_OK;
  if (!set_off || !out) return bfail(PV_EINVAL, "null buffer");
  if (m > 0xffffffffull) return bfail(PV_EINVAL, "too many sets");
  for (uint64_t j = 0; j < m; ++j)
    if (set_off[j + 1] < set_off[j]) return bfail(PV_EINVAL, "set_off not monotone at %llu", (unsigned long long)j);
  const uint64_t s0 = set_off[0], ns = set_off[m] - s0;
  if (ns && !sigs) return bfail(PV_EINVAL, "null buffer");
  BLS_HIP(hipSetDevice(device));
  hipStream_t s = d->stream;
  std::vector<uint64_t> so(m + 1);
  for (uint64_t j = 0; j <= m; ++j) so[j] = set_off[j] - s0;
  BLS_HIP(d->sig.ensure(ns * 128));
  BLS_HIP(d->moff.ensure(m + 1));
  BLS_HIP(d->blob.ensure(m * 128));
  if (ns) BLS_HIP(hipMemcpyAsync(d->sig.p, sigs + 128 * s0, ns * 128, hipMemcpyHostToDevice, s));
  BLS_HIP(hipMemcpyAsync(d->moff.p, so.data(), (m + 1) * 8, hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(k_bls_agg_g1, dim3(blocks_for(m, 64)), dim3(64), 0, s, d->sig.p, d->moff.p, (uint32_t)m, d->blob.p);
  BLS_HIP(hipGetLastError());
  BLS_HIP(hipMemcpyAsync(out, d->blob.p, m * 128, hipMemcpyDeviceToHost, s));
  BLS_HIP(hipStreamSynchronize(s));
  return PV_OK;
}

int pv_bls_sign_batch_device(const uint8_t* sks, const uint8_t* msg_blob, const uint64_t* msg_off, uint64_t n_msgs,
                             const uint32_t* msg_idx, const uint32_t* key_idx, uint64_t n, uint8_t* sig, int device,
                             void* stream) {
  std::lock_guard<std::mutex> lk(g_bls_mu);
  Guard gd;
  BlsDev* d = nullptr;
  if (int rc = bls_dev(device, &d)) return rc;
  if (n == 0) return PV_OK;
  if (!sks || !msg_off || !msg_idx || !key_idx || !sig || (n_msgs && !msg_blob)) return bfail(PV_EINVAL, "null buffer");
  BLS_HIP(hipSetDevice(device));
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : d->stream;
  BLS_HIP(d->msgtab.ensure(n_msgs * MSG_WORDS));
  hipLaunchKernelGGL(k_bls_hash, dim3(blocks_for(n_msgs, 64)), dim3(64), 0, s, msg_blob, msg_off, (uint32_t)n_msgs,
                     d->msgtab.p);
  hipLaunchKernelGGL(k_bls_sign, dim3(blocks_for(n, 64)), dim3(64), 0, s, sks, d->msgtab.p, msg_idx, key_idx, n, sig);
  BLS_HIP(hipGetLastError());
  BLS_HIP(hipStreamSynchronize(s));
  return PV_OK;
}

int pv_bls_sign_batch(const uint8_t* sks, uint64_t k, const uint8_t* msg_blob, const uint64_t* msg_off,
                      uint64_t n_msgs, const uint32_t* msg_idx, const uint32_t* key_idx, uint64_t n, uint8_t* sig,
                      int device) {
  if (n == 0) return PV_OK;
  if (!sks || !msg_off || !msg_idx || !key_idx || !sig) return bfail(PV_EINVAL, "null buffer");
  for (uint64_t i = 0; i < n_msgs; ++i)
    if (msg_off[i + 1] < msg_off[i]) return bfail(PV_EINVAL, "msg_off not monotone at %llu", (unsigned long long)i);
  for (uint64_t j = 0; j < n; ++j)
    if (msg_idx[j] >= n_msgs || key_idx[j] >= k) return bfail(PV_EINVAL, "index out of range at %llu", (unsigned long long)j);
  Guard gd;
  Buf<uint8_t> ks, bl, sg;
  Buf<uint64_t> of;
  Buf<uint32_t> mi, ki;
  const uint64_t b0 = msg_off[0], bytes = msg_off[n_msgs] - b0;
  std::vector<uint64_t> off(n_msgs + 1);
  for (uint64_t i = 0; i <= n_msgs; ++i) off[i] = msg_off[i] - b0;
  {
    std::lock_guard<std::mutex> lk(g_bls_mu);
    BlsDev* d = nullptr;
    if (int rc = bls_dev(device, &d)) return rc;
  }
  BLS_HIP(hipSetDevice(device));
  BLS_HIP(ks.ensure(k * 32));
  BLS_HIP(bl.ensure(bytes + 64));
  BLS_HIP(sg.ensure(n * 128));
  BLS_HIP(of.ensure(n_msgs + 1));
  BLS_HIP(mi.ensure(n));
  BLS_HIP(ki.ensure(n));
  BLS_HIP(hipMemcpy(ks.p, sks, k * 32, hipMemcpyHostToDevice));
  if (bytes) BLS_HIP(hipMemcpy(bl.p, msg_blob + b0, bytes, hipMemcpyHostToDevice));
  BLS_HIP(hipMemset(bl.p + bytes, 0, 64));
  BLS_HIP(hipMemcpy(of.p, off.data(), (n_msgs + 1) * 8, hipMemcpyHostToDevice));
  BLS_HIP(hipMemcpy(mi.p, msg_idx, n * 4, hipMemcpyHostToDevice));
  BLS_HIP(hipMemcpy(ki.p, key_idx, n * 4, hipMemcpyHostToDevice));
  int rc = pv_bls_sign_batch_device(ks.p, bl.p, of.p, n_msgs, mi.p, ki.p, n, sg.p, device, nullptr);
  if (rc == PV_OK) BLS_HIP(hipMemcpy(sig, sg.p, n * 128, hipMemcpyDeviceToHost));
  ks.release(); bl.release(); sg.release(); of.release(); mi.release(); ki.release();
  return rc;
}

int pv_bls_pubkeys(const uint8_t* gen, const uint8_t* sks, uint64_t k, uint8_t* pks, int device) {
  std::lock_guard<std::mutex> lk(g_bls_mu);
  Guard gd;
  BlsDev* d = nullptr;
  if (int rc = bls_dev(device, &d)) return rc;
  if (k == 0) return PV_OK;
  if (!gen || !sks || !pks) return bfail(PV_EINVAL, "null buffer");
  BLS_HIP(hipSetDevice(device));
  Buf<uint8_t> g, s, o;
  BLS_HIP(g.ensure(128));
  BLS_HIP(s.ensure(k * 32));
  BLS_HIP(o.ensure(k * 128));
  BLS_HIP(hipMemcpyAsync(g.p, gen, 128, hipMemcpyHostToDevice, d->stream));
  BLS_HIP(hipMemcpyAsync(s.p, sks, k * 32, hipMemcpyHostToDevice, d->stream));
  hipLaunchKernelGGL(k_bls_pubkeys, dim3(blocks_for(k, 64)), dim3(64), 0, d->stream, g.p, s.p, (uint32_t)k, o.p);
  BLS_HIP(hipGetLastError());
  BLS_HIP(hipMemcpyAsync(pks, o.p, k * 128, hipMemcpyDeviceToHost, d->stream));
  BLS_HIP(hipStreamSynchronize(d->stream));
  g.release();
  s.release();
  o.release();
  return PV_OK;
}

int pv_bls_kernel_ms(int device, float* hash_ms, float* verify_ms) {
  std::lock_guard<std::mutex> lk(g_bls_mu);
  for (auto& d : g_bls)
    if (d.ord == device) {
      if (hash_ms) *hash_ms = d.ms_hash;
      if (verify_ms) *verify_ms = d.ms_verify;
      return PV_OK;
    }
  return bfail(PV_ENOTINIT, "no BLS state on device %d", device);
}

void pv_bls_shutdown(void) {
  std::lock_guard<std::mutex> lk(g_bls_mu);
  Guard gd;
  for (auto& d : g_bls) {
    (void)hipSetDevice(d.ord);
    if (d.stream) (void)hipStreamSynchronize(d.stream);
    d.keys.release(); d.multi.release(); d.msgtab.release(); d.cnt.release(); d.seg.release();
    d.cursor.release(); d.order.release(); d.total.release(); d.midx.release(); d.kidx.release(); d.sig.release();
    d.blob.release(); d.verdict.release(); d.sks.release(); d.off.release(); d.mpks.release(); d.moff.release();
    for (auto& e : d.ev)
      if (e) (void)hipEventDestroy(e), e = nullptr;
    if (d.stream) (void)hipStreamDestroy(d.stream);
    d.stream = nullptr;
  }
  g_bls.clear();
}

}  // extern "C"
