// HOST INSTRUMENTATION BUILD of the kernel algorithms (test tooling only —
// never loaded by the product package, see tests/test_hostcheck.py).
//
// Compiles indy-plenum_amd/csrc/pv_verify_core.h with g++ so that the exact
// per-lane schedule the HIP kernels run can be
//   * bound-checked: every fe_mul/fe_sq input is asserted to be LOOSE,
//   * op-counted: field mul/sq/add/carry, SHA-512 blocks, scalar reductions
//     per verify (the roofline's algorithmic work),
//   * run under ASan/UBSan and gdb (no GPU needed).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t g_cnt[8];
enum { HC_mul, HC_sq, HC_add, HC_carry, HC_sha, HC_sc, HC_sub, HC_carry_even };
static int g_bad_bound = 0;

#define PV_HD static inline
#define PV_COUNT(kind) (++g_cnt[HC_##kind])
static void hc_bad(const char* what, int k, unsigned long long v) {
  if (!g_bad_bound) fprintf(stderr, "bound violation: %s [%d] = %llu\n", what, k, v);
  g_bad_bound = 1;
}
// exact exactness conditions of fe_mul(f, g): 2 f_i < 2^32 (odd i),
// 19 g_j < 2^32, every column sum (+ carry-in < 2^39) < 2^64
static void hc_check_mul(const uint32_t* f, const uint32_t* g) {
  for (int i = 1; i < 10; i += 2)
    if (2ull * f[i] >= (1ull << 32)) hc_bad("2f", i, f[i]);
  for (int j = 1; j < 10; ++j)
    if (19ull * g[j] >= (1ull << 32)) hc_bad("19g", j, g[j]);
  for (int k = 0; k < 10; ++k) {
    unsigned __int128 s = (unsigned __int128)1 << 39;
    for (int i = 0; i < 10; ++i) {
      const int j = (k - i + 10) % 10;
      unsigned __int128 t = (unsigned __int128)f[i] * g[j];
      if ((i & 1) && (j & 1)) t *= 2;
      if (i + j >= 10) t *= 19;
      s += t;
    }
    if (s >> 64) hc_bad("column", k, (unsigned long long)(s >> 64));
  }
}
// fe_sq(f): its prepared operands 2 f_0..7, 19 f_6, 19 f_8, 38 f_5, 38 f_7,
// 38 f_9 (pv_field.h sq_avail) and the columns of f*f
static void hc_check_sq(const uint32_t* f) {
  for (int i = 0; i < 8; ++i)
    if (2ull * f[i] >= (1ull << 32)) hc_bad("2f", i, f[i]);
  for (int j = 6; j < 10; j += 2)
    if (19ull * f[j] >= (1ull << 32)) hc_bad("19f", j, f[j]);
  for (int j = 5; j < 10; j += 2)
    if (38ull * f[j] >= (1ull << 32)) hc_bad("38f", j, f[j]);
  hc_check_mul(f, f);
}
// fe_sq2x(f) = 2 f^2: 2 f_0..7, 4 f_0,1,3, 38 f_6,8, 76 f_5,7,9 and twice the columns of f*f
static void hc_check_sq2x(const uint32_t* f) {
  for (int i = 0; i < 8; ++i)
    if (2ull * f[i] >= (1ull << 32)) hc_bad("2f", i, f[i]);
  static const int four[3] = {0, 1, 3};
  for (int i : four)
    if (4ull * f[i] >= (1ull << 32)) hc_bad("4f", i, f[i]);
  for (int j = 6; j < 10; j += 2)
    if (38ull * f[j] >= (1ull << 32)) hc_bad("38f", j, f[j]);
  for (int j = 5; j < 10; j += 2)
    if (76ull * f[j] >= (1ull << 32)) hc_bad("76f", j, f[j]);
  for (int k = 0; k < 10; ++k) {
    unsigned __int128 s = (unsigned __int128)1 << 39;
    for (int i = 0; i < 10; ++i) {
      const int j = (k - i + 10) % 10;
      unsigned __int128 t = (unsigned __int128)2 * f[i] * f[j];
      if ((i & 1) && (j & 1)) t *= 2;
      if (i + j >= 10) t *= 19;
      s += t;
    }
    if (s >> 64) hc_bad("column2x", k, (unsigned long long)(s >> 64));
  }
}
#define PV_CHECK_MUL(f, g) hc_check_mul((f).v, (g).v)
#define PV_CHECK_SQ2X(f) hc_check_sq2x((f).v)
#define PV_CHECK_SQ(f) hc_check_sq((f).v)

#include "../../indy-plenum_amd/csrc/pv_verify_core.h"
#include "../../indy-plenum_amd/csrc/pv_sha256.h"
#include "../../indy-plenum_amd/csrc/pv_quad.h"

using namespace pv;

static uint32_t g_btab[BT_CHUNKS * BT_TABLE];
static uint32_t g_btab_even[4 * BT_TABLE];   // chunks 0, 2, 4, 6 (the keyed kernel's LDS image)
static int g_btab_ready = 0;

// radix-2^16 chunk tables k * 2^(32 q) * B (the device builds each entry with
// btable_entry(.., 16); here: k*P = (k-1)*P + P and one batch inversion per
// table, the same points in affine niels form)
static uint32_t g_bw[BW_CHUNKS * BW_TABLE];

static void build_bw() {
  static ge_p3 pts[BW_ENTRIES];
  static fe pre[BW_ENTRIES];
  for (int t = 0; t < BW_CHUNKS; ++t) {
    ge_p3 P;
    ge_basepoint(P);
    for (int d = 0; d < 32 * t; ++d) {
      ge_p1p1 u;
      ge_p3_dbl(u, P);
      ge_p1p1_to_p3(P, u);
    }
    ge_cached cp;
    ge_p3_to_cached(cp, P);
    ge_p3_0(pts[0]);
    for (int k = 1; k < BW_ENTRIES; ++k) {
      ge_p1p1 u;
      ge_add_cached(u, pts[k - 1], cp, false);
      ge_p1p1_to_p3(pts[k], u);
    }
    fe acc;
    fe_copy(acc, pts[0].Z);
    fe_copy(pre[0], acc);
    for (int k = 1; k < BW_ENTRIES; ++k) {
      fe_mul(acc, acc, pts[k].Z);
      fe_copy(pre[k], acc);
    }
    fe_invert(acc, acc);
    fe d2;
    fe_const_d2(d2);
    for (int k = BW_ENTRIES - 1; k >= 0; --k) {
      fe zi, x, y, v;
      if (k > 0) {
        fe_mul(zi, acc, pre[k - 1]);
        fe_mul(acc, acc, pts[k].Z);
      } else {
        fe_copy(zi, acc);
      }
      fe_mul(x, pts[k].X, zi);
      fe_mul(y, pts[k].Y, zi);
      uint32_t* p = g_bw + (uint64_t)t * BW_TABLE + (uint64_t)k * BT_WORDS;
      fe_add(v, y, x); fe_carry(v);
      store_fe(p, v);
      fe_sub(v, y, x); fe_carry(v);
      store_fe(p + 10, v);
      fe_mul(v, x, y);
      fe_mul(v, v, d2);
      store_fe(p + 20, v);
      p[30] = 0;
      p[31] = 0;
    }
  }
}

static void ensure_btab() {
  if (g_btab_ready) return;
  for (int q = 0; q < BT_CHUNKS; ++q)
    for (int k = 0; k < BT_ENTRIES; ++k) btable_entry(g_btab + (q * BT_ENTRIES + k) * BT_WORDS, k, q);
  for (int t = 0; t < 4; ++t) memcpy(g_btab_even + t * BT_TABLE, g_btab + 2 * t * BT_TABLE, 4 * BT_TABLE);
  build_bw();
  g_btab_ready = 1;
}

extern "C" {

// verdicts with exactly the generic kernels' algorithm (k_hash, k_lattice,
// k_curve_half with its full-length tasks for deferred records); the message
// blob must have >= 16 readable bytes after the last message (same contract
// as the kernel).  force_full: every record deferred (PV_CURVE_MODE=full).
// n_deferred (may be NULL) receives the number of full-length verdicts.
void hc_verify_batch_mode(const uint8_t* pk, const uint8_t* sig, const uint8_t* blob, const uint64_t* off, uint64_t n,
                          uint8_t* verdict, int force_full, uint64_t* n_deferred) {
  ensure_btab();
  static uint32_t lane[HALF_LANE_WORDS];
  uint32_t rec[HREC_WORDS];
  uint64_t nd = 0;
  for (uint64_t i = 0; i < n; ++i) {
    uint32_t h[16];
    const bool pre = hash_one(h, pk + 32 * i, sig + 64 * i, blob + off[i], off[i + 1] - off[i]);
    const uint32_t st = lattice_one(rec, pre, h, sig + 64 * i, force_full != 0);
    bool ok = false;
    if (st == HS_HALF) {
      ok = curve_half(pk + 32 * i, sig + 64 * i, rec, lane, g_bw, g_bw + 4 * BW_TABLE);
    } else if (st == HS_DEFER) {
      ok = verify_full_one(pk + 32 * i, sig + 64 * i, h, lane, g_btab);
      ++nd;
    }
    verdict[i] = ok ? 1 : 0;
  }
  if (n_deferred) *n_deferred = nd;
}

// verdicts with the latency kernel's algorithm (k_verify_quad: each side of
// the lane-pair split on a lane QUAD, emulated here with the four lanes in
// lockstep; deferred records take the quad's full-length form)
void hc_verify_batch_quad(const uint8_t* pk, const uint8_t* sig, const uint8_t* blob, const uint64_t* off, uint64_t n,
                          uint8_t* verdict, int force_full, uint64_t* n_deferred) {
  ensure_btab();
  static uint32_t tab0[QTAB_WORDS], tab1[QTAB_WORDS];
  uint32_t rec[HREC_WORDS];
  uint64_t nd = 0;
  for (uint64_t i = 0; i < n; ++i) {
    uint32_t h[16];
    const bool pre = hash_one(h, pk + 32 * i, sig + 64 * i, blob + off[i], off[i + 1] - off[i]);
    const uint32_t st = lattice_one(rec, pre, h, sig + 64 * i, force_full != 0);
    bool ok = false;
    if (st == HS_HALF || st == HS_DEFER) {
      qfe Q0, Q1, e1;
      const QRole qr = qrole_of(0);   // (the emulation gives lane j role j)
      const bool ok0 = q_side(Q0, pk + 32 * i, sig + 64 * i, rec, 0, tab0, g_bw, qr);
      const bool ok1 = q_side(Q1, pk + 32 * i, sig + 64 * i, rec, 1, tab1, g_bw + 4 * BW_TABLE, qr);
      q_to_cached(e1, Q1, qr);
      ok = ok0 && ok1 && q_sum_is_identity(Q0, e1, qr);
      nd += st == HS_DEFER;
    }
    verdict[i] = ok ? 1 : 0;
  }
  if (n_deferred) *n_deferred = nd;
}

void hc_verify_batch(const uint8_t* pk, const uint8_t* sig, const uint8_t* blob, const uint64_t* off, uint64_t n,
                     uint8_t* verdict) {
  hc_verify_batch_mode(pk, sig, blob, off, n, verdict, 0, nullptr);
}

// half-size scalars of h (32 LE bytes, < L): |c|, d as 20 LE bytes each
// (plain values, no digit offset); returns HS_HALF / HS_DEFER
uint32_t hc_half_scalars(const uint8_t* h32, uint8_t* c20, uint8_t* d20, uint32_t* c_neg) {
  uint32_t h[8], c[HS_WORDS], d[HS_WORDS];
  memcpy(h, h32, 32);
  bool neg = false;
  const uint32_t st = half_scalars(c, d, neg, h);
  memcpy(c20, c, 4 * HS_WORDS);
  memcpy(d20, d, 4 * HS_WORDS);
  *c_neg = neg ? 1u : 0u;
  return st;
}

// s' = d * S mod L (d: 20 LE bytes, S: 32 LE bytes)
void hc_sc_mul_small(const uint8_t* d20, const uint8_t* s32, uint8_t* out32) {
  uint32_t d[HS_WORDS], S[8], r[8];
  memcpy(d, d20, 4 * HS_WORDS);
  memcpy(S, s32, 32);
  sc_mul_small(r, d, S);
  memcpy(out32, r, 32);
}

// the previous generic schedule: full-length scalars, CURVE_K signatures per
// lane sharing one inversion (the keyed kernel keeps this group structure)
void hc_verify_batch_grouped(const uint8_t* pk, const uint8_t* sig, const uint8_t* blob, const uint64_t* off,
                             uint64_t n, uint8_t* verdict) {
  ensure_btab();
  static uint32_t lane[LANE_WORDS];
  uint32_t* h = (uint32_t*)calloc(n ? n * 16 : 16, sizeof(uint32_t));
  uint8_t* pre = (uint8_t*)calloc(n ? n : 1, 1);
  for (uint64_t i = 0; i < n; ++i)
    pre[i] = hash_one(h + 16 * i, pk + 32 * i, sig + 64 * i, blob + off[i], off[i + 1] - off[i]);
  for (uint64_t i0 = 0; i0 < n; i0 += CURVE_K) {
    const uint32_t okm = curve_group<false>(pk, sig, h, pre, i0, 1, n, lane, g_btab);
    for (int k = 0; k < CURVE_K && i0 + k < n; ++k) verdict[i0 + k] = (okm >> k) & 1u;
  }
  free(h);
  free(pre);
}

// keyed variant: prepare each key of pk (k keys) once, signature i uses key kidx[i]
void hc_verify_keyed(const uint8_t* pk, uint64_t k, const uint32_t* kidx, const uint8_t* sig, const uint8_t* blob,
                     const uint64_t* off, uint64_t n, uint8_t* verdict) {
  ensure_btab();
  static uint32_t lane[LANE_WORDS];
  uint32_t* ktab = (uint32_t*)calloc(k ? k * KEY_WORDS : KEY_WORDS, sizeof(uint32_t));
  uint32_t* scr = (uint32_t*)calloc(KEY_SCRATCH, sizeof(uint32_t));
  for (uint64_t j = 0; j < k; ++j) key_prepare(ktab + j * KEY_WORDS, scr, pk + 32 * j);
  free(scr);
  uint32_t* h = (uint32_t*)calloc(n ? n * 16 : 16, sizeof(uint32_t));
  uint8_t* pre = (uint8_t*)calloc(n ? n : 1, 1);
  for (uint64_t i = 0; i < n; ++i)
    pre[i] = hash_one(h + 16 * i, pk + 32 * kidx[i], sig + 64 * i, blob + off[i], off[i + 1] - off[i]);
  for (uint64_t i0 = 0; i0 < n; i0 += CURVE_K) {
    const uint32_t okm = curve_group<true>(pk, sig, h, pre, i0, 1, n, lane, g_btab_even, ktab, kidx, g_bw);
    for (int q = 0; q < CURVE_K && i0 + q < n; ++q) verdict[i0 + q] = (okm >> q) & 1u;
  }
  free(ktab);
  free(h);
  free(pre);
}

// wide (radix-256) prepared keys: every table of every key on the host, then
// the keyed curve stage with the wide comb (k_curve<true, 1>'s algorithm)
void hc_verify_keyed_wide(const uint8_t* pk, uint64_t k, const uint32_t* kidx, const uint8_t* sig, const uint8_t* blob,
                          const uint64_t* off, uint64_t n, uint8_t* verdict) {
  ensure_btab();
  static uint32_t lane[LANE_WORDS];
  uint32_t* ktab = (uint32_t*)calloc(k ? k * KEYW_WORDS : KEYW_WORDS, sizeof(uint32_t));
  uint32_t* scr = (uint32_t*)calloc(KEYW_SCRATCH, sizeof(uint32_t));
  for (uint64_t j = 0; j < k; ++j)
    for (int q = 0; q < COMB_Q; ++q)
      for (int sl = 0; sl < KW_SLICES; ++sl) key_prepare_wide_slice(ktab + j * KEYW_WORDS, scr, pk + 32 * j, q, sl);
  free(scr);
  uint32_t* h = (uint32_t*)calloc(n ? n * 16 : 16, sizeof(uint32_t));
  uint8_t* pre = (uint8_t*)calloc(n ? n : 1, 1);
  for (uint64_t i = 0; i < n; ++i)
    pre[i] = hash_one(h + 16 * i, pk + 32 * kidx[i], sig + 64 * i, blob + off[i], off[i + 1] - off[i]);
  for (uint64_t i0 = 0; i0 < n; i0 += CURVE_K) {
    const uint32_t okm = curve_group<true, 1, 1>(pk, sig, h, pre, i0, 1, n, lane, g_btab_even, ktab, kidx, g_bw);
    for (int q = 0; q < CURVE_K && i0 + q < n; ++q) verdict[i0 + q] = (okm >> q) & 1u;
  }
  free(ktab);
  free(h);
  free(pre);
}

// keyed latency kernel (k_verify_quad_keyed): prepared keys, each of the
// SIDES sides' comb share on an emulated quad, the sides summed over the
// kernel's exchange tree (1 -> 0, 3 -> 2, ..., then 2 -> 0, ..., then SIDES / 2
// -> 0), the total plus -R tested for the identity on side 0
}  // extern "C" (a template below)
template <int SIDES>
static void verify_keyed_quad_t(const uint8_t* pk, uint64_t k, const uint32_t* kidx, const uint8_t* sig,
                                const uint8_t* blob, const uint64_t* off, uint64_t n, uint8_t* verdict) {
  ensure_btab();
  uint32_t* ktab = (uint32_t*)calloc(k ? k * KEY_WORDS : KEY_WORDS, sizeof(uint32_t));
  uint32_t* scr = (uint32_t*)calloc(KEY_SCRATCH, sizeof(uint32_t));
  for (uint64_t j = 0; j < k; ++j) key_prepare(ktab + j * KEY_WORDS, scr, pk + 32 * j);
  free(scr);
  const QRole qr = qrole_of(0);
  for (uint64_t i = 0; i < n; ++i) {
    uint32_t dig[16], rec[KQ_WORDS];
    // the hash wave's split: schedules of the first KQ_SCHED_BLOCKS blocks, then the rounds
    const uint64_t mlen = off[i + 1] - off[i];
    uint64_t kw[80 * KQ_SCHED_BLOCKS];
    for (uint64_t b = 0; b < (uint64_t)KQ_SCHED_BLOCKS && b < hram_blocks(mlen); ++b)
      keyed_sched_block(kw + b, KQ_SCHED_BLOCKS, sig + 64 * i, pk + 32 * kidx[i], blob + off[i], mlen, b);
    const bool pre = keyed_hash(dig, kw, KQ_SCHED_BLOCKS, 1, sig + 64 * i, pk + 32 * kidx[i], blob + off[i], mlen);
    keyed_record(rec, pre, dig);
    uint32_t nr[41];
    keyed_neg_r(nr, sig + 64 * i);
    qfe eR, Q[SIDES], x;
    q_load_cached(eR, nr, false, qr);
    const uint32_t* kt = ktab + (uint64_t)kidx[i] * KEY_WORDS;
    for (int s = 0; s < SIDES; ++s) {
      qfe hs, ls;
      q_comb_base<SIDES>(hs, ls, sig + 64 * i, s, g_bw, qr);
      q_comb_side<SIDES>(Q[s], rec, s, kt, hs, ls, qr);
    }
    for (int step = 1; step < SIDES; step <<= 1)   // the kernel's shfl_xor 4 (step 1), 8 (step 2) ...
      for (int s = 0; s < SIDES; s += 2 * step) {
        q_to_cached(x, Q[s + step], qr);
        q_add(Q[s], x, false, qr);
      }
    verdict[i] = (rec[KQ_OK] && kt[KEY_STATUS] && nr[40] && q_sum_is_identity(Q[0], eR, qr)) ? 1 : 0;
  }
  free(ktab);
}
extern "C" {
void hc_verify_keyed_quad(const uint8_t* pk, uint64_t k, const uint32_t* kidx, const uint8_t* sig,
                          const uint8_t* blob, const uint64_t* off, uint64_t n, uint8_t* verdict) {
  verify_keyed_quad_t<KQ_SIDES>(pk, k, kidx, sig, blob, off, n, verdict);
}
// the small-call form: 4 signatures per block, KQ_SIDES_SMALL comb sides each
void hc_verify_keyed_quad_small(const uint8_t* pk, uint64_t k, const uint32_t* kidx, const uint8_t* sig,
                                const uint8_t* blob, const uint64_t* off, uint64_t n, uint8_t* verdict) {
  verify_keyed_quad_t<KQ_SIDES_SMALL>(pk, k, kidx, sig, blob, off, n, verdict);
}

// SHA-256(prefix || M_i) with the kernels' block loader; prefix < 0 = none
void hc_sha256(const uint8_t* blob, const uint64_t* off, uint64_t n, int prefix, uint8_t* out) {
  for (uint64_t i = 0; i < n; ++i)
    sha256_msg(reinterpret_cast<uint32_t*>(out + 32 * i), blob + off[i], off[i + 1] - off[i], prefix < 0 ? 0 : 1,
               prefix < 0 ? 0 : (uint32_t)prefix);
}

// Merkle node SHA-256(0x01 || l || r) with the kernels' fixed-size path
void hc_sha256_node(const uint8_t* lr64, uint8_t* out) {
  uint32_t lr[16];
  memcpy(lr, lr64, 64);
  sha256_node(reinterpret_cast<uint32_t*>(out), lr);
}

void hc_sign_batch(const uint8_t* seeds, const uint8_t* blob, const uint64_t* off, uint64_t n, uint8_t* pk,
                   uint8_t* sig) {
  ensure_btab();
  for (uint64_t i = 0; i < n; ++i) sign_one(pk + 32 * i, sig + 64 * i, seeds + 32 * i, blob + off[i],
                                            off[i + 1] - off[i], g_btab);
}

void hc_btable(uint32_t* out) {
  ensure_btab();
  memcpy(out, g_btab, sizeof g_btab);
}

void hc_reset_counts(void) {
  memset(g_cnt, 0, sizeof g_cnt);
  g_bad_bound = 0;
}

// counts[0..7] = mul, sq, add, carry, sha blocks, scalar reductions, sub, even-limb carries
int hc_get_counts(uint64_t* counts) {
  for (int i = 0; i < 8; ++i) counts[i] = g_cnt[i];
  return g_bad_bound;
}

// field self-test helpers: c = a*b, c = a^2 from/to canonical 32-byte encodings
void hc_fe_mul(const uint8_t* a, const uint8_t* b, uint8_t* out) {
  uint32_t wa[8], wb[8], wo[8];
  load8(wa, a); load8(wb, b);
  fe fa, fb, fc;
  fe_frombytes_w(fa, wa); fe_frombytes_w(fb, wb);
  fe_mul(fc, fa, fb);
  fe_tobytes_w(wo, fc);
  store8(out, wo);
}
void hc_fe_sq(const uint8_t* a, uint8_t* out) {
  uint32_t wa[8], wo[8];
  load8(wa, a);
  fe fa, fc;
  fe_frombytes_w(fa, wa);
  fe_sq(fc, fa);
  fe_tobytes_w(wo, fc);
  store8(out, wo);
}
void hc_fe_invert(const uint8_t* a, uint8_t* out) {
  uint32_t wa[8], wo[8];
  load8(wa, a);
  fe fa, fc;
  fe_frombytes_w(fa, wa);
  fe_invert(fc, fa);
  fe_tobytes_w(wo, fc);
  store8(out, wo);
}
void hc_sc_reduce64(const uint8_t* in64, uint8_t* out32) {
  uint32_t x[16], r[8];
  memcpy(x, in64, 64);
  sc_reduce64(r, x);
  memcpy(out32, r, 32);
}
void hc_sc_muladd(const uint8_t* a, const uint8_t* b, const uint8_t* c, uint8_t* out) {
  uint32_t wa[8], wb[8], wc[8], wo[8];
  memcpy(wa, a, 32); memcpy(wb, b, 32); memcpy(wc, c, 32);
  sc_muladd(wo, wa, wb, wc);
  memcpy(out, wo, 32);
}

}  // extern "C"
