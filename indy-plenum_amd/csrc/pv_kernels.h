// Internal launch interface between the C-ABI layer (pv_api.cpp) and the HIP
// kernels (pv_kernels.hip).  All pointers are device pointers on the current
// device; every launch is asynchronous on `stream`.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pv {

// base-point table: 129 niels entries (k*B, k = 0..128), 32 words each
constexpr int BTAB_ENTRIES = 129;
constexpr int BTAB_WORDS = 32;
constexpr int BTAB_CHUNKS = 8;     // tables for 2^(32 q) B, q = 0..7 (comb kernel of prepared keys)
// per-lane scratch: A table (9 cached entries k*(-A), 40 words each) + the
// CURVE_K points awaiting the shared inversion (40 words each)
#ifndef PV_CURVE_K
#define PV_CURVE_K 8
#endif
constexpr int ATAB_WORDS = 9 * 40 + PV_CURVE_K * 40;
constexpr int CURVE_BLOCK = 256;
constexpr int HASH_BLOCK = 256;

struct DeviceCaps {
  int cu_count;
  int curve_blocks;  // persistent grid for the curve kernel
};

hipError_t launch_btable_init(uint32_t* btab, hipStream_t s);

// resident curve-kernel blocks per CU (occupancy query)
hipError_t curve_occupancy(int* blocks_per_cu, bool keyed = false);

// pre[i] = 1 iff S canonical, R/A not small order, A canonical;
// dig[i] (16 words) = SHA-512(R||A||M) when pre[i] (reduced mod L by the curve
// kernel).  Persistent grid of `blocks` blocks; `counter` is an 8-byte device
// word the launch resets (work queue).
hipError_t hash_occupancy(int* blocks_per_cu);
// kidx (may be NULL): signature i's key is pk[kidx[i]] (keyed batches)
// pre != null: k_precheck writes the pre-check verdicts first and k_hash skips
// the rejected signatures; pre == null: every signature is hashed (the
// half-size path checks in launch_lattice)
hipError_t launch_hash(const uint8_t* pk, const uint8_t* sig, const uint8_t* blob, const uint64_t* off, uint64_t n,
                       unsigned long long* counter, uint32_t* dig, uint8_t* pre, int blocks, hipStream_t s,
                       const uint32_t* kidx = nullptr);

// verdict[i] in {0,1}; bitmap[i/64] bit i%64 (bitmap must hold ceil(n/64) words);
// h = the hash kernel's digests (16 words per signature)
// ktab/kidx (may be NULL): keyed mode, signature i uses prepared key kidx[i]
hipError_t launch_curve(const uint8_t* pk, const uint8_t* sig, const uint32_t* h, const uint8_t* pre,
                        const uint32_t* btab, uint32_t* scratch, uint64_t scratch_lanes, uint8_t* verdict,
                        uint64_t* bitmap, uint64_t n, int blocks, hipStream_t s, const uint32_t* ktab = nullptr,
                        const uint32_t* kidx = nullptr, const uint32_t* bw = nullptr,
                        unsigned long long* tasks = nullptr,    // wave task queue counter (zeroed here)
                        bool wide = false);                     // ktab in the wide (radix-256) key format

// Half-size scalar path (generic batches, pv_lattice.h):
//   launch_lattice   pre-checks (-> pre) and h mod L -> (c, d, s') records
//                    (HSREC_WORDS words per signature), deferred indices ->
//                    dlist / *dcount; also
//                    zeroes *tasks and the bitmap (ceil(n/64) words) the curve
//                    kernel ORs into.  n < 2^32.
//   launch_curve_half  verdicts + bitmap; per-lane scratch HALF_SCRATCH_WORDS
//                    (tables of +-A and -R).
constexpr int HSREC_WORDS = 20;
constexpr int HALF_SCRATCH_WORDS = 2 * 9 * 40;
hipError_t curve_half_occupancy(int* blocks_per_cu);
// latency mode for small batches: lane pairs per signature, per-lane scratch
// ATAB_LAT_WORDS (one 9-entry table)
constexpr int ATAB_LAT_WORDS = 9 * 40;
hipError_t launch_curve_lat(const uint8_t* pk, const uint8_t* sig, const uint32_t* dig, const uint32_t* rec,
                            const uint32_t* btab, const uint32_t* bw, uint32_t* scratch, uint64_t scratch_lanes,
                            uint8_t* verdict, uint64_t* bitmap, uint64_t n, hipStream_t s);
// latency mode in one launch: pre-checks + hash + scalar stage (one wave) and
// the lane-quad curve stage (another) per block of 8 signatures; *dcount +=
// the deferred records (caller zeroes it); the bitmap needs no zeroing
hipError_t launch_verify_quad(const uint8_t* pk, const uint8_t* sig, const uint8_t* blob, const uint64_t* off, uint64_t n,
                              const uint32_t* bw, uint8_t* verdict, uint64_t* bitmap, unsigned long long* dcount,
                              bool force_full, hipStream_t s);
// host-buffer chunks: the whole half-size verify of a chunk in one persistent
// launch (pre-checks + hash + lattice + curve per 64-signature task; rec =
// HSREC_WORDS per signature, scratch as launch_curve_half); deferred records
// are appended to dlist as base + i (*dcount, zeroed by the caller) and left
// for launch_verify_quad_list, which verifies the listed indices (count read
// on the device; max_count bounds the grid) with the lane-quad kernel
hipError_t launch_chunk_half(const uint8_t* pk, const uint8_t* sig, const uint8_t* blob, const uint64_t* off,
                             uint64_t n, uint32_t* rec, const uint32_t* bw, uint32_t* scratch, uint64_t scratch_lanes,
                             uint8_t* verdict, uint32_t* dlist, unsigned long long* dcount, uint64_t base,
                             unsigned long long* tasks, int blocks, bool force_full, hipStream_t s);
hipError_t launch_verify_quad_list(const uint8_t* pk, const uint8_t* sig, const uint8_t* blob, const uint64_t* off,
                                   const uint32_t* list, const unsigned long long* lcount, uint64_t max_count,
                                   int blocks, const uint32_t* bw, uint8_t* verdict, bool force_full, hipStream_t s);
hipError_t launch_lattice(const uint8_t* pk, const uint8_t* sig, const uint32_t* dig, uint8_t* pre, uint64_t n,
                          uint32_t* rec, uint32_t* dlist, unsigned long long* dcount, unsigned long long* tasks,
                          uint64_t* bitmap, bool force_full, hipStream_t s);
// btab: the radix-256 base-point tables (deferred full-length tasks); bw:
// BWTAB_WORDS words, the radix-2^16 chunk tables k * 2^(32 q) * B, q = 0..7
// (launch_bw_init; chunks 0 and 4 serve the half-size path, all eight the
// keyed comb)
constexpr int BWTAB_ENTRIES = (1 << 15) + 1;
constexpr uint64_t BWTAB_WORDS = 8ull * BWTAB_ENTRIES * BTAB_WORDS;
hipError_t launch_bw_init(uint32_t* bw, hipStream_t s);
hipError_t launch_curve_half(const uint8_t* pk, const uint8_t* sig, const uint32_t* dig, const uint32_t* rec,
                             const uint32_t* btab, const uint32_t* bw, uint32_t* scratch, uint64_t scratch_lanes,
                             uint8_t* verdict, uint64_t* bitmap, uint64_t n, const uint32_t* dlist,
                             const unsigned long long* dcount, unsigned long long* tasks, int blocks, hipStream_t s);

// prepared keys: KEYTAB_WORDS words per key (8 comb tables of affine multiples
// k * 2^(32 q) * (-A) + status); KEYTAB_SCRATCH words of scratch per key
constexpr int KEYTAB_WORDS = 8 * 9 * 32 + 32;
constexpr int KEYTAB_SCRATCH = 64 * 40;   // projective entries + prefix products (lane-interleaved per 64 keys)
hipError_t launch_keys(const uint8_t* pk, uint64_t k, uint32_t* ktab, uint32_t* scr, hipStream_t s);
// wide key format (radix-256 comb, node keys): KEYTAB_WIDE_WORDS words per key,
// KEYTAB_WIDE_SCRATCH words of scratch per lane (KEYTAB_WIDE_LANES lanes per
// key: 16 per table, lane-interleaved per 64)
constexpr int KEYTAB_WIDE_WORDS = 8 * 129 * 32 + 32;
constexpr int KEYTAB_WIDE_LANES = 128;
constexpr int KEYTAB_WIDE_SCRATCH = 8 * 40;
hipError_t launch_keys_wide(const uint8_t* pk, uint64_t k, uint32_t* ktab, uint32_t* scr, hipStream_t s);
// latency mode for prepared keys (k_verify_quad_keyed): the whole verify of n
// signatures in one launch, signature e's key = ktab entry kidx[i] with i =
// list ? list[e] : e; the hashed key bytes are pk + 32 * (pk_by_key ? kidx[i] : i).
// Verdicts go to verdict[i]; bitmap (ceil(n/64) words, needs no zeroing) only
// without a list (may be NULL then too).  flag (host-mapped) / done (a device
// counter at 0): the last block writes seq to *flag when every verdict is out
// and re-arms *done (both NULL: no completion word)
hipError_t launch_verify_quad_keyed(const uint8_t* pk, bool pk_by_key, const uint8_t* sig, const uint8_t* blob,
                                    const uint64_t* off, uint64_t n, const uint32_t* list, const uint32_t* ktab,
                                    const uint32_t* kidx, const uint32_t* bw, uint8_t* verdict, uint64_t* bitmap,
                                    hipStream_t s, uint32_t* done = nullptr, uint32_t* flag = nullptr,
                                    uint32_t seq = 0);

// completion signal of a zero-copy host call: *flag = seq (system scope, after
// every earlier kernel of the stream), polled by the host instead of a stream
// synchronize (run_small)
hipError_t launch_signal(uint32_t* flag, uint32_t seq, hipStream_t s);

// keygen + sign: pk[i], sig[i] for seed[i] over M_i
hipError_t launch_sign(const uint8_t* seeds, const uint8_t* blob, const uint64_t* off, uint64_t n,
                       const uint32_t* btab, uint8_t* pk_out, uint8_t* sig_out, hipStream_t s);

// per-batch quorum tally over per-message verdicts + sender indices (*bad |= 1
// when a sender index is >= n_nodes), and over node-indexed voter bitmaps
hipError_t launch_tally(const uint8_t* verdict, const uint32_t* sender, const uint64_t* batch_off,
                        uint64_t n_batches, uint32_t n_nodes, uint32_t quorum, uint32_t* votes,
                        uint8_t* reached, uint32_t* bad, hipStream_t s);
hipError_t launch_tally_bits(const uint32_t* bits, const uint32_t* dup, uint64_t n_batches, uint32_t n_nodes,
                             uint32_t quorum, uint32_t* votes, uint8_t* reached, hipStream_t s);

// SHA-256 / Merkle: out (n x 8 words) = SHA-256(prefix || M_i)
// (plen 0 or 1 prefix bytes); one Merkle level m -> ceil(m/2) nodes
hipError_t sha256_occupancy(int* blocks_per_cu);
hipError_t launch_sha256(const uint8_t* blob, const uint64_t* off, uint64_t n, uint32_t plen, uint32_t prefix,
                         unsigned long long* counter, uint32_t* out, int blocks, hipStream_t s);
hipError_t launch_merkle_level(const uint32_t* in, uint64_t m, uint32_t* out, hipStream_t s);
// the remaining levels of m (2 <= m <= MERKLE_TAIL) nodes in one workgroup -> root
constexpr int MERKLE_TAIL = 256;
hipError_t launch_merkle_tail(const uint32_t* in, uint64_t m, uint32_t* root, hipStream_t s);

// deterministic synthetic workload; spec in plenum_gpu/synth.py.
// mode 0 FIXED (len = mlen_min), 1 RANGE (len uniform in [mlen_min, mlen_max]),
// 2 COMMIT (C3 3PC batches of n_nodes votes).
// off (n+1) <- exclusive prefix sum of message lengths; sums = scan_sums_words(n+1) words
uint64_t scan_sums_words(uint64_t m);
hipError_t launch_exclusive_scan(uint64_t* x, uint64_t m, uint64_t* sums, hipStream_t s);
hipError_t launch_synth_layout(uint32_t cfg, uint32_t mode, uint64_t first, uint64_t n, uint32_t mlen_min,
                               uint32_t mlen_max, uint32_t n_nodes, uint64_t* off, uint64_t* sums, hipStream_t s);
hipError_t launch_synth(uint32_t cfg, uint32_t mode, uint64_t first, uint64_t n, uint32_t key_mod, uint32_t n_nodes,
                        uint8_t* seeds_out, uint8_t* tamper_out, uint32_t* sender_out, hipStream_t s);
hipError_t launch_synth_fill(uint32_t cfg, uint32_t mode, uint64_t first, uint64_t n, uint32_t n_nodes,
                             const uint64_t* off, uint8_t* blob, hipStream_t s);
hipError_t launch_tamper(uint64_t first, uint64_t n, const uint8_t* tamper, const uint64_t* off, uint8_t* blob,
                         uint8_t* sig, hipStream_t s);

}  // namespace pv
