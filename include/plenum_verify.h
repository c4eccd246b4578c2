/*
 * plenum_verify.h — C ABI of the MI355X batch signature-verification and
 * vote-tally engine (libplenum_verify.so).
 *
 * Drop-in boundary for Plenum's request-authentication hot path.  Each entry
 * point names the reference interface it replaces:
 *
 *   pv_verify_batch  replaces N calls of libnacl.crypto_sign_open(sig||msg, pk)
 *                    made by stp_core/crypto/nacl_wrappers.py:86-108
 *                    (VerifyKey.verify) via Verifier.verify (:232-242) and
 *                    plenum/common/verifier.py:53-54 (DidVerifier.verify).
 *                    Native side of that call: libsodium 1.0.18
 *                    int crypto_sign_open(unsigned char *m, unsigned long long *mlen_p,
 *                                         const unsigned char *sm, unsigned long long smlen,
 *                                         const unsigned char *pk);
 *                    (/opt/conda/include/sodium/crypto_sign.h:67).  Verdicts are
 *                    bit-exact with crypto_sign_ed25519_verify_detached on
 *                    (sig[0:64], msg).  The sig||msg framing (smlen < 64 rejects,
 *                    a non-64-byte decoded signature shifts bytes into M) is the
 *                    caller's job, exactly as in the reference;
 *                    the Python glue (plenum_gpu.nacl_wrappers) does it.
 *   pv_tally         replaces the per-3PC-batch voter-set count of
 *                    plenum/server/models.py:16-114 (Commits/Prepares.addVote +
 *                    hasQuorum) with quorum values from plenum/server/quorums.py:15-39:
 *                    the SURVEY.md §8(b) contract (node-indexed voter bitmaps);
 *   pv_tally_votes   the same predicate built from per-message verdicts and sender
 *                    indices (the voter set is formed on the GPU; also the PROPAGATE
 *                    f+1 count of plenum/server/propagator.py:38-46).
 *   pv_sign_batch    batch counterpart of SigningKey(seed) + sign
 *                    (stp_core/crypto/nacl_wrappers.py:130-176; crypto_sign_seed_keypair
 *                    + crypto_sign_detached).  Used to generate fixtures/bench data.
 *
 * Conventions:
 *   - All host buffers are owned by the caller; nothing is retained after return.
 *   - Return 0 on success, a negative errno-style code on failure; no exceptions
 *     cross the ABI.  pv_last_error() describes the last failure (thread-local).
 *   - Calls are synchronous and thread-compatible (one caller thread at a time per
 *     device set), matching the single Looper thread (stp_core/loop/looper.py:64).
 *   - A verdict is a pure function of (pk, sig64, M).
 *   - msg_off has n+1 entries; message i is msg_blob[msg_off[i] : msg_off[i+1]].
 *
 * Device-pointer variants (*_device) take device pointers on `device` and an
 * optional hipStream_t (NULL = a library-owned stream) and return after the
 * work is enqueued AND complete (they synchronise the stream).  The message
 * blob passed to a device variant must have >= 16 readable bytes after the last
 * message (the hash kernel reads aligned words).
 */
#ifndef PLENUM_VERIFY_H
#define PLENUM_VERIFY_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PV_OK 0
#define PV_EINVAL (-22)   /* bad argument */
#define PV_ENODEV (-19)   /* no usable GPU in device_mask */
#define PV_ENOMEM (-12)   /* device allocation failed */
#define PV_EIO (-5)       /* HIP runtime / kernel failure */
#define PV_ENOTINIT (-77) /* pv_init not called */

/* flags for pv_verify_batch */
#define PV_FLAG_NONE 0u
/* Deduplicate verifying keys on the host and prepare each distinct key once
 * (decompressed -A and its cached multiples) when at least half of a shard's
 * signatures repeat a key (node COMMIT votes, many requests per client DID).
 * Verdicts are identical; only the work changes. */
#define PV_FLAG_DEDUP_KEYS 1u

/* words per prepared key (pv_keys_prepare_device): an 8-way comb of -A —
 * affine multiples k * 2^(32 q) * (-A), k = 0..8, q = 0..7, 32 words each —
 * + status word + padding to a multiple of 32 words (each key starts on a
 * 128-byte line, so no 128-byte entry straddles two cache lines) */
#define PV_KEY_WORDS 2336u

/* Initialise the engine on the GPUs in device_mask (bit d = HIP device d;
 * 0 = all visible devices).  Idempotent.  Builds the base-point tables
 * (radix 256, 132 KB; radix 2^16 chunk tables k * 2^(32 q) * B, 33.5 MB per
 * device). */
int pv_init(uint32_t device_mask);

/* Release every device resource.  Safe to call when not initialised. */
void pv_shutdown(void);

/* TEST ONLY (not part of the node-facing interface): pv_init(0) with k (2..8)
 * engine devices that all run on HIP device 0, so the multi-device paths of
 * pv_verify_batch (a worker thread per device, shard offsets, error
 * aggregation) run on a one-GPU box (tests/test_gpu_multidev.py).  Requires
 * that no device is initialised (PV_EINVAL otherwise); pv_shutdown ends it. */
int pv_test_init_dup(uint32_t k);

/* TEST ONLY: the spin budget (ns, default 20,000,000) a zero-copy small call
 * polls its completion word for before it falls back to hipStreamSynchronize;
 * 0 sends every such call through the fallback (tests/test_gpu_keycache.py).
 * PV_EINVAL for ns < 0. */
int pv_test_set_spin_ns(int64_t ns);

/* Human-readable description of the last error on this thread ("" if none). */
const char *pv_last_error(void);

/* Number of devices the engine is using (after pv_init), else 0. */
int pv_device_count(void);

/* Verify n signatures held in HOST memory.
 *   pk      n x 32 bytes
 *   sig     n x 64 bytes (R || S; the first 64 bytes of sig||msg)
 *   msg_blob, msg_off  messages (see conventions)
 *   verdict n bytes out, 1 = valid, 0 = invalid
 * The batch is split into contiguous shards over the devices in device_mask
 * (0 = every initialised device), each driven by its own host thread; a shard
 * runs as a pipeline of about 8 chunks: host threads gather chunk c into a
 * page-locked slot, its H2D runs on a copy stream, and its kernels run on one
 * of two compute streams (chunk c+1's grid fills chunk c's tail).  msg_off must
 * be non-decreasing (checked chunk by chunk before any kernel reads it:
 * PV_EINVAL).  Synchronous: returns after every verdict is in `verdict`. */
int pv_verify_batch(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg_blob, const uint64_t *msg_off,
                    uint64_t n, uint8_t *verdict, uint32_t device_mask, uint32_t flags);

/* Same with DEVICE pointers on `device`.  msg_off entries are offsets into
 * msg_blob.  bitmap (may be NULL) receives ceil(n/64) 64-bit words: bit i%64 of
 * word i/64 = verdict i (the layout all-gathered across ranks). */
int pv_verify_batch_device(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg_blob, const uint64_t *msg_off,
                           uint64_t n, uint8_t *verdict, uint64_t *bitmap, int device, void *stream);

/* Enqueue-only forms for pipelined device callers: the work is queued on
 * `stream` (NULL = the library stream of `slot`) with verify workspace `slot`
 * (0 or 1) and the call returns without waiting; the caller synchronises its
 * stream.  Two batches in flight at once must use different slots and
 * different output buffers (verdict, bitmap; for keys, ktab); work reusing a
 * slot must be ordered after that slot's previous batch (same stream, or an
 * event).  Inputs must be ready on `stream` (the caller orders its own writes).
 * A caller alternating two streams and two slots over consecutive batches lets
 * batch k + 1's hash stage run while batch k's curve grid drains.  bitmap is
 * required here. */
int pv_verify_batch_device_async(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg_blob,
                                 const uint64_t *msg_off, uint64_t n, uint8_t *verdict, uint64_t *bitmap, int device,
                                 void *stream, int slot);
int pv_verify_keyed_device_async(const uint32_t *ktab, const uint32_t *key_idx, const uint8_t *pk, const uint8_t *sig,
                                 const uint8_t *msg_blob, const uint64_t *msg_off, uint64_t n, uint8_t *verdict,
                                 uint64_t *bitmap, int device, void *stream, int slot);
int pv_keys_prepare_device_async(const uint8_t *pk, uint64_t k, uint32_t *ktab, int device, void *stream, int slot);

/* Verifying-key cache on the device.  pv_keys_prepare_device fills ktab
 * (k x PV_KEY_WORDS words) for the k 32-byte keys in pk; a key that libsodium
 * would refuse (non-canonical, small order, not on the curve) is marked so and
 * every signature under it is rejected.  The table is an 8-way comb, so a
 * keyed verification needs 28 doublings instead of 253.  pv_verify_keyed_device verifies n
 * signatures whose key is pk[key_idx[i]] (the same pk array the table was built
 * from: the hash still covers the key's bytes) — same verdicts as
 * pv_verify_batch_device on the gathered keys, without re-decompressing a key
 * per signature.  Replaces the per-call VerifyKey(key) construction of
 * stp_core/crypto/nacl_wrappers.py:71-81 for repeated keys. */
int pv_keys_prepare_device(const uint8_t *pk, uint64_t k, uint32_t *ktab, int device, void *stream);

int pv_verify_keyed_device(const uint32_t *ktab, const uint32_t *key_idx, const uint8_t *pk, const uint8_t *sig,
                           const uint8_t *msg_blob, const uint64_t *msg_off, uint64_t n, uint8_t *verdict,
                           uint64_t *bitmap, int device, void *stream);

/* Persistent verifying-key cache of host-buffer calls.  pv_keycache_add
 * prepares the comb tables of the k 32-byte keys in pk on every initialised
 * device (and on devices initialised later) and keeps them until
 * pv_keycache_clear / pv_shutdown; keys already cached are skipped.  A
 * pv_verify_batch shard of a Looper-pass size (<= the latency size) then looks
 * up every signature's key on the host: signatures under cached keys run the
 * keyed latency kernel (no decompression of A; the hashed key bytes are still
 * the caller's), the rest the generic one, in the same call.  Verdicts are
 * identical with or without the cache -- a key libsodium refuses is cached as
 * refused.  Fill it from the keys a node already knows: node keys, the client
 * DIDs of SimpleAuthNr.addIdr / getVerkey's NYM state lookups
 * (plenum/server/client_authn.py:145-168), replacing the per-call VerifyKey(key) of
 * stp_core/crypto/nacl_wrappers.py:71-81.  At most 2^32 - 2 keys. */
int pv_keycache_add(const uint8_t *pk, uint64_t k);
int pv_keycache_clear(void);
int pv_keycache_size(uint64_t *count);

/* Wide prepared keys (node keys): the same comb with radix-256 windows --
 * affine multiples k * 2^(32 q) * (-A), k = 0..128, q = 0..7 (129 entries of
 * 32 words per table) + status + padding, PV_KEY_WORDS_WIDE words (132 KB) per
 * key.  A verify then needs 24 doublings and 32 key adds instead of 28 and 64;
 * the preparation costs ~16x the default format's, so it pays for keys that
 * sign many messages per preparation (a pool's node keys, C3).  Same verdicts.
 * Preparation runs 128 lanes per key (16 slices of each of the 8 tables) and
 * holds 160 KB of device scratch per key while it runs (128 lanes x 320 words,
 * owned by the device context, grown to the largest k seen).  Async forms as
 * pv_*_device_async (slot 0 or 1, enqueue only). */
#define PV_KEY_WORDS_WIDE 33056u
int pv_keys_prepare_wide_device(const uint8_t *pk, uint64_t k, uint32_t *ktab, int device, void *stream);
int pv_keys_prepare_wide_device_async(const uint8_t *pk, uint64_t k, uint32_t *ktab, int device, void *stream,
                                      int slot);
int pv_verify_keyed_wide_device(const uint32_t *ktab, const uint32_t *key_idx, const uint8_t *pk, const uint8_t *sig,
                                const uint8_t *msg_blob, const uint64_t *msg_off, uint64_t n, uint8_t *verdict,
                                uint64_t *bitmap, int device, void *stream);
int pv_verify_keyed_wide_device_async(const uint32_t *ktab, const uint32_t *key_idx, const uint8_t *pk,
                                      const uint8_t *sig, const uint8_t *msg_blob, const uint64_t *msg_off, uint64_t n,
                                      uint8_t *verdict, uint64_t *bitmap, int device, void *stream, int slot);

/* Key preparation + keyed verification of one batch in one enqueue-only call
 * (slot / stream rules as pv_*_device_async): the k keys in pk are prepared
 * into ktab (wide = 0: the PV_KEY_WORDS format, 1: PV_KEY_WORDS_WIDE).  A key
 * grid of less than one wave per SIMD (e.g. a pool's 25 node keys in the wide
 * format) runs on the slot's own side stream, forked from `stream`, WHILE the
 * signatures' SHA-512 stage runs on `stream` (it reads only the key bytes
 * pk[key_idx[i]]), and the keyed curve kernel waits for both; a larger key
 * grid fills the GPU itself and runs before the hash stage on `stream`.  Same
 * verdicts and tables as
 * pv_keys_prepare[_wide]_device_async followed by
 * pv_verify_keyed[_wide]_device_async on the same stream, which run the two
 * stages one after the other.  n = 0 only prepares the keys.  As for every
 * keyed call, each key_idx[i] must be < k: the kernels do not bound-check it. */
int pv_verify_keys_device_async(const uint8_t *pk, uint64_t k, uint32_t *ktab, const uint32_t *key_idx,
                                const uint8_t *sig, const uint8_t *msg_blob, const uint64_t *msg_off, uint64_t n,
                                uint8_t *verdict, uint64_t *bitmap, uint32_t wide, int device, void *stream, int slot);

/* SHA-256 / Merkle tree hashing.
 *   pv_sha256_batch[_device]  digests[i] (32 bytes) = SHA-256(prefix || M_i); prefix -1 = none,
 *                             0..255 = that single byte.  Replaces the per-request
 *                             sha256(...).hexdigest() of Request.key / payload_digest
 *                             (plenum/common/request.py:82-90).
 *   pv_merkle_root[_device]   RFC 6962 Merkle Tree Hash of the leaves M_0..M_{n-1}, bit-identical
 *                             to ledger/tree_hasher.py TreeHasher.hash_full_tree (:55-86; leaf =
 *                             SHA-256(0x00 || M), node = SHA-256(0x01 || l || r), n = 0 ->
 *                             SHA-256("")); leaf_hashes (n x 32, may be NULL) receives the leaf
 *                             digests (TreeHasher.hash_leaf, :21-24).
 * Device variants: root is a 32-byte DEVICE buffer; the blob needs >= 16 readable bytes after
 * the last message. */
int pv_sha256_batch(const uint8_t *blob, const uint64_t *off, uint64_t n, int32_t prefix, uint8_t *digests);
int pv_sha256_batch_device(const uint8_t *blob, const uint64_t *off, uint64_t n, int32_t prefix, uint8_t *digests,
                           int device, void *stream);
int pv_merkle_root(const uint8_t *blob, const uint64_t *off, uint64_t n, uint8_t *root, uint8_t *leaf_hashes);
int pv_merkle_root_device(const uint8_t *blob, const uint64_t *off, uint64_t n, uint8_t *leaf_hashes, uint8_t *root,
                          int device, void *stream);

/* Per-batch quorum tally, SURVEY.md §8(b) form (HOST memory).
 *   verdict_bits  n_batches x W words, W = ceil(n_nodes / 32): bit j of word w of
 *                 batch b = node 32 w + j cast a valid vote in batch b (a voter SET:
 *                 a node's repeated votes are one bit, plenum/server/models.py:24-28)
 *   dup_mask      same shape, may be NULL: nodes whose votes must not count
 *                 (e.g. a sender the caller already counted elsewhere)
 *   reached       n_batches out: popcount(verdict_bits & ~dup_mask) >= quorum
 * Bits of nodes >= n_nodes are ignored. */
int pv_tally(const uint32_t *verdict_bits, const uint32_t *dup_mask, uint64_t n_batches, uint32_t n_nodes,
             uint32_t quorum, uint8_t *reached);

/* DEVICE buffers; votes (may be NULL) receives the per-batch counts. */
int pv_tally_device(const uint32_t *verdict_bits, const uint32_t *dup_mask, uint64_t n_batches, uint32_t n_nodes,
                    uint32_t quorum, uint8_t *reached, uint32_t *votes, int device, void *stream);

/* Per-batch quorum tally from per-message verdicts (HOST memory).
 *   verdict    n_msgs bytes (1 = vote counts)
 *   sender     n_msgs node indices (< n_nodes <= 1024; an index >= n_nodes is
 *              PV_EINVAL, never a silently dropped vote)
 *   batch_off  n_batches + 1 offsets into verdict/sender
 *   votes      n_batches out: distinct valid senders per batch
 *   reached    n_batches out: votes >= quorum
 * Duplicate senders count once (a voter SET, plenum/server/models.py:24-28). */
int pv_tally_votes(const uint8_t *verdict, const uint32_t *sender, const uint64_t *batch_off, uint64_t n_batches,
                   uint32_t n_nodes, uint32_t quorum, uint32_t *votes, uint8_t *reached);

int pv_tally_votes_device(const uint8_t *verdict, const uint32_t *sender, const uint64_t *batch_off,
                          uint64_t n_batches, uint32_t n_nodes, uint32_t quorum, uint32_t *votes, uint8_t *reached,
                          int device, void *stream);
/* Enqueue-only form for pipelined callers: the kernel ORs 1 into the DEVICE
 * word *bad when a sender index is >= n_nodes (the caller zeroes it and checks
 * it once its stream is synchronised -- such a vote is never counted). */
int pv_tally_votes_device_async(const uint8_t *verdict, const uint32_t *sender, const uint64_t *batch_off,
                                uint64_t n_batches, uint32_t n_nodes, uint32_t quorum, uint32_t *votes,
                                uint8_t *reached, uint32_t *bad, int device, void *stream);

/* Batch keygen + sign (HOST memory): pk_out[i], sig_out[i] for seed i over
 * message i.  Deterministic (RFC 8032 / crypto_sign_detached). */
int pv_sign_batch(const uint8_t *seeds, const uint8_t *msg_blob, const uint64_t *msg_off, uint64_t n,
                  uint8_t *pk_out, uint8_t *sig_out);

int pv_sign_batch_device(const uint8_t *seeds, const uint8_t *msg_blob, const uint64_t *msg_off, uint64_t n,
                         uint8_t *pk_out, uint8_t *sig_out, int device, void *stream);

/* Deterministic synthetic workload on the device (bench/tests; spec in
 * plenum_gpu/synth.py).  Two phases so that the caller can
 * size the message blob:
 *   pv_synth_layout_device  off[0..n] <- exclusive prefix sum of the message
 *                           lengths (off[n] = blob bytes)
 *   pv_synth_fill_device    messages, seeds, tamper flags (and for COMMIT the
 *                           sender node of every vote), then keygen + sign, then
 *                           the spec's single-bit tampering.
 * Modes: FIXED (C2: len = mlen_min), RANGE (C4: len uniform in [mlen_min,
 * mlen_max]), COMMIT (C3: signature i is node slot i % n_nodes's COMMIT vote
 * in 3PC batch i / n_nodes; M = "instId:0|op:COMMIT|ppSeqNo:<b+1>|viewNo:0").
 * key_mod (FIXED/RANGE): key index = i % key_mod (0 = distinct keys).
 * Buffers are device buffers the caller allocated: off (n+1), blob (off[n] + 16),
 * seeds (n*32), pk (n*32), sig (n*64), tamper (n), sender (n or NULL). */
#define PV_SYNTH_FIXED 0u
#define PV_SYNTH_RANGE 1u
#define PV_SYNTH_COMMIT 2u

int pv_synth_layout_device(uint32_t cfg, uint32_t mode, uint64_t first, uint64_t n, uint32_t mlen_min,
                           uint32_t mlen_max, uint32_t n_nodes, uint64_t *off, int device, void *stream);

int pv_synth_fill_device(uint32_t cfg, uint32_t mode, uint64_t first, uint64_t n, uint32_t key_mod,
                         uint32_t n_nodes, const uint64_t *off, uint8_t *blob, uint8_t *seeds, uint8_t *pk,
                         uint8_t *sig, uint8_t *tamper, uint32_t *sender, int device, void *stream);

/* FIXED-mode convenience (C2): layout + fill in one call; blob holds n*mlen + 16. */
int pv_synth_device(uint32_t cfg, uint64_t first, uint64_t n, uint32_t key_mod, uint32_t mlen, uint64_t *off,
                    uint8_t *blob, uint8_t *seeds, uint8_t *pk, uint8_t *sig, uint8_t *tamper, int device,
                    void *stream);

/* Time the verify kernels alone over `iters` launches on device-resident
 * inputs using HIP events on the launch stream; returns per-kernel average
 * milliseconds (hash, curve).  "hash" = k_hash plus, on the half-size path, the
 * scalar stage k_lattice; "curve" = the single curve kernel launch. */
int pv_time_verify_device(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg_blob, const uint64_t *msg_off,
                          uint64_t n, uint8_t *verdict, uint64_t *bitmap, int device, void *stream, int iters,
                          float *ms_hash, float *ms_curve);

/* ------------------------------------------------------------------------
 * Schedule tuning.  pv_init reads NO environment: a node runs the defaults
 * below unless its code calls pv_set_tuning.  None of these knobs changes a
 * verdict (tests/test_gpu_verify.py and test_gpu_device.py run the fixtures
 * through every setting); they exist for A/B timing (tools/) and tests.
 *
 *   curve_mode      curve stage of generic (non-keyed) batches:
 *     PV_CURVE_HALF     (default) half-size scalars: Euclid on (8L, h) gives
 *                       c == d h (mod 8L) with |c|, d < 2^131, d odd, and the
 *                       verdict is  s'B + c(-A) + d(-R) == O  (s' = dS mod L): the
 *                       same accept/reject as libsodium's encode(SB - hA) == R for
 *                       every input (derivation in indy-plenum_amd/csrc/pv_lattice.h);
 *                       the ~0.2 % of signatures whose h has no such (c, d) get the
 *                       full-length verdict in the same launch;
 *     PV_CURVE_FULL     every signature through the full-length verdict;
 *     PV_CURVE_GROUPED  the full-length kernel, 8 signatures per lane sharing one
 *                       inversion.
 *   lat_max         generic batches of at most this many signatures (per device
 *                   call / host-buffer shard) run the latency kernel: 8 lanes per
 *                   signature (lane-pair split, each side's point over a lane
 *                   QUAD, one coordinate per lane, DPP exchanges), so small
 *                   batches finish ~2x sooner.  Default 32768 (the measured
 *                   crossover with the throughput path is 32k-64k); 0 disables;
 *                   at most 2^20.
 *   lat_keyed_max   keyed batches (prepared keys, the key cache) of at most this
 *                   many signatures run the keyed latency kernel (the key's comb
 *                   over two lane quads per signature).  Default 8192; 0 disables.
 *   lat_kernel      PV_LAT_QUAD (default) or PV_LAT_PAIR (the lane-pair kernel, A/B).
 *   small_zc_max    host calls of at most this many signatures read their inputs
 *                   from, and write verdicts to, mapped page-locked memory (no
 *                   copies).  Default 2048; 0 = always copy.
 *   host_fused      host-buffer chunks of generic batches: 1 (default) = one
 *                   fused launch per chunk + one lane-quad pass over the deferred
 *                   records; 0 = hash, lattice, curve launches per chunk.
 *   host_staging    PV_STAGING_PINNED (default): each chunk is gathered by up to
 *                   host_copy_threads host threads into one of two page-locked
 *                   slots per device (at most host_pin_max_mb each) and DMA'd from
 *                   there; PV_STAGING_PAGEABLE: the caller's buffers go straight
 *                   to hipMemcpyAsync.  Switching to pageable releases the slots.
 *   host_chunks     a shard runs as leading ramp chunks (host_ramp, 2 host_ramp,
 *                   ... signatures below a regular chunk; host_ramp 0 = one first
 *                   chunk of host_first_pct % of a regular one) and then about
 *                   host_chunks equal chunks of >= 32768 signatures.
 *                   Defaults 8 (1..256), ramp 32768 (0 or 1024..2^20),
 *                   first_pct 50 (10..100), copy threads 8 (1..64), pin 512 MB
 *                   (16..4096).
 *   host_trace      1 = per-chunk host timings of pv_verify_batch on stderr.
 *   bls_quad_max    BLS calls (pv_bls_verify_*) of at most this many checks run
 *                   one check per lane quad (latency), larger ones one per lane
 *                   pair (throughput).  Default 32768 (0..2^20).
 *   bls_oct_max     BLS calls of at most this many checks run one check per lane
 *                   octet (the shortest chain; takes precedence over
 *                   bls_quad_max).  Default 4096 (0..2^20).
 *   reserved        must be 0.
 * (The test-only duplicate engine devices are not a tuning field: see
 * pv_test_init_dup below.)
 * pv_get_tuning fills *t with the current values (struct_size must be set to
 * sizeof(pv_tuning) by the caller); pv_set_tuning validates every field
 * (PV_EINVAL and nothing changes if one is out of range), keeps them for later
 * pv_init calls and applies them to every initialised device.
 * ---------------------------------------------------------------------- */
#define PV_CURVE_HALF 0u
#define PV_CURVE_FULL 1u
#define PV_CURVE_GROUPED 2u
#define PV_LAT_QUAD 0u
#define PV_LAT_PAIR 1u
#define PV_STAGING_PINNED 0u
#define PV_STAGING_PAGEABLE 1u
typedef struct pv_tuning {
  uint32_t struct_size;       /* sizeof(pv_tuning) */
  uint32_t curve_mode;
  uint64_t lat_max;
  uint64_t lat_keyed_max;
  uint64_t small_zc_max;
  uint32_t lat_kernel;
  uint32_t host_fused;
  uint32_t host_staging;
  uint32_t host_chunks;
  uint32_t host_first_pct;
  uint32_t host_copy_threads;
  uint64_t host_ramp;
  uint32_t host_pin_max_mb;
  uint32_t host_trace;
  uint32_t bls_quad_max;
  uint32_t bls_oct_max;
  uint32_t reserved;
} pv_tuning;
int pv_get_tuning(pv_tuning *t);
int pv_set_tuning(const pv_tuning *t);

/* mode (may be NULL) = the curve_mode of `device`; deferred (may be NULL) =
 * signatures of the last generic batch on this device that took the
 * full-length verdict (0 if none ran). */
int pv_curve_stats(int device, uint32_t *mode, uint64_t *deferred);

/* Live kernel timing of the verify calls themselves (bench.py's timed region):
 * enable = 1 resets and starts recording HIP events around the hash and curve
 * stages of every verify launch on `device` (on the launch stream, without
 * waiting for them: async launches stay in flight); enable = 0 stops, waits
 * for the recorded events and returns the summed milliseconds and the number
 * of launches. */
int pv_kernel_timing(int device, int enable, float *hash_ms, float *curve_ms, uint64_t *launches);

/* The SHA-512 part of the live "hash" interval: summed milliseconds from the
 * start of each timed verify launch to the end of its k_hash (the pre-checks +
 * SHA-512(R||A||M), without the half-size path's k_lattice), since the last
 * pv_kernel_timing(device, 1, ...).  bench.py's hash roofline. */
int pv_kernel_timing_sha(int device, float *sha_ms);

/* pv_time_verify_device for keyed batches. */
int pv_time_verify_keyed_device(const uint32_t *ktab, const uint32_t *key_idx, const uint8_t *pk, const uint8_t *sig,
                                const uint8_t *msg_blob, const uint64_t *msg_off, uint64_t n, uint8_t *verdict,
                                uint64_t *bitmap, int device, void *stream, int iters, float *ms_hash,
                                float *ms_curve);




/* ------------------------------------------------------------------------
 * BLS COMMIT check
 *
 *   pv_bls_verify_batch  replaces n calls of
 *                        BlsCryptoVerifierIndyCrypto.verify_sig(signature, message, bls_pk)
 *                        (crypto/bls/indy_crypto/bls_crypto_indy_crypto.py:73-82), made by
 *                        BlsBftReplicaPlenum._validate_signature for every COMMIT
 *                        (plenum/bls/bls_bft_replica_plenum.py:55-75, 194-213), i.e.
 *                        python-ursa 0.1.1 Bls.verify(sig, msg, vk, gen):
 *                        e(sigma, g) == e(H(msg), vk) over Milagro AMCL BN254.
 *   pv_bls_set_keys      the fixed G2 arguments of those checks: the group generator
 *                        (BlsGroupParamsLoaderIndyCrypto, bls_crypto_indy_crypto.py:15-20)
 *                        and the nodes' keys (bls_key_register.get_key_by_name);
 *                        replaces IndyCryptoBlsUtils.bls_from_str(v, VerKey) (:38-52)
 *                        + the pairing's G2 precomputation.
 *   pv_bls_sign_batch[_device], pv_bls_pubkeys
 *                        batch counterparts of Bls.sign / VerKey.new (data generation).
 *
 * PARITY UNPINNED: ursa / AMCL are not in the reference and not installed; the
 * reference holds no BLS vector.  Encodings (128-byte representations):
 *   sigma  0x04|x|y (uncompressed) or 0x02/0x03|x (compressed), big-endian, rest
 *          ignored; x or y >= p, another prefix, or a point off y^2 = x^3 + 2 is
 *          the point at infinity O (AMCL ECP::frombytes).  A representation that
 *          is not 128 bytes fails to decode: verdict 0 (sig_len).
 *   keys   x.a|x.b|y.a|y.b, big-endian, each taken mod p (ECP2::frombytes);
 *          off the twist y^2 = x^3 + 2/(1+i) = O.
 *   H(m)   SHA-256(m) as a big-endian integer mod p, try-and-increment on x,
 *          y = (x^3+2)^((p+1)/4) (ursa PointG1::from_hash / AMCL ECP::new_big).
 *   e(O, .) = e(., O) = 1: sigma = O or key = O verify iff both are O.
 * Errors of these entry points are reported by pv_bls_last_error().
 * ---------------------------------------------------------------------- */
#define PV_BLS_KEY_OK 0u          /* a point of order r on the twist */
#define PV_BLS_KEY_INFINITY 1u    /* off the twist: decodes to O */
#define PV_BLS_KEY_NOT_IN_G2 2u   /* on the twist outside the order-r subgroup: verdicts are 0 */

/* Prepare the generator (128 B) and k keys (k x 128 B) on HIP device `device`:
 * decode, subgroup check, the 70 optimal-ate lines of each point (kept on the
 * device; replaces the previous key set).  status (k bytes, may be NULL) gets
 * PV_BLS_KEY_*.  PV_EINVAL if the generator is not PV_BLS_KEY_OK. */
int pv_bls_set_keys(const uint8_t *gen, const uint8_t *pks, uint64_t k, uint8_t *status, int device);

/* Append k keys (k x 128 B) to the key set of pv_bls_set_keys on `device`
 * WITHOUT re-preparing the keys already there: one k_bls_lines launch over the
 * k new points (a node key added by a NODE txn, bls_key_register).  Their key
 * indices are *first .. *first + k - 1 (first may be NULL); status as in
 * pv_bls_set_keys.  PV_ENOTINIT without a set; PV_EINVAL past 65535 keys (the
 * set is left as it was on any error). */
int pv_bls_add_keys(const uint8_t *pks, uint64_t k, uint8_t *status, uint64_t *first, int device);

/* The key set on `device`: keys in it and the points k_bls_lines has prepared
 * for it so far (cumulative over pv_bls_set_keys / pv_bls_add_keys). */
int pv_bls_keyset_info(int device, uint64_t *nkeys, uint64_t *points_prepared);

/* n checks from HOST memory: check j = (sig[j] 128 B, message msg_idx[j] of
 * msg_blob/msg_off (n_msgs messages, msg_off has n_msgs+1 entries), key
 * key_idx[j] of the current key set) -> verdict[j] (1 = Bls.verify true).
 * sig_len (may be NULL): the decoded representation lengths; != 128 -> 0.
 * Every message is hashed once; checks are grouped by key on the device. */
int pv_bls_verify_batch(const uint8_t *sig, const uint64_t *sig_len, const uint8_t *msg_blob, const uint64_t *msg_off,
                        uint64_t n_msgs, const uint32_t *msg_idx, const uint32_t *key_idx, uint64_t n,
                        uint8_t *verdict, int device);
/* Same with DEVICE pointers (msg_blob needs >= 16 readable bytes past the last
 * message); synchronous on `stream` (NULL = library stream).  Indices are not
 * checked on the host here: a check whose key_idx is >= the key count or whose
 * msg_idx is >= n_msgs is skipped by the kernels and gets verdict 0. */
int pv_bls_verify_batch_device(const uint8_t *sig, const uint8_t *msg_blob, const uint64_t *msg_off, uint64_t n_msgs,
                               const uint32_t *msg_idx, const uint32_t *key_idx, uint64_t n, uint8_t *verdict,
                               int device, void *stream);
/* sig[j] = sk[key_idx[j]] * H(message msg_idx[j]) (uncompressed 128 B); sks: k x 32 B big-endian */
int pv_bls_sign_batch(const uint8_t *sks, uint64_t k, const uint8_t *msg_blob, const uint64_t *msg_off,
                      uint64_t n_msgs, const uint32_t *msg_idx, const uint32_t *key_idx, uint64_t n, uint8_t *sig,
                      int device);
int pv_bls_sign_batch_device(const uint8_t *sks, const uint8_t *msg_blob, const uint64_t *msg_off, uint64_t n_msgs,
                             const uint32_t *msg_idx, const uint32_t *key_idx, uint64_t n, uint8_t *sig, int device,
                             void *stream);
/* n multi-signature checks from HOST memory; replaces n calls of
 *   BlsCryptoVerifierIndyCrypto.verify_multi_sig(signature, message, pks)
 *   (crypto/bls/indy_crypto/bls_crypto_indy_crypto.py:84-97), made once per
 *   ledger of every PRE-PREPARE by BlsBftReplicaPlenum._validate_multi_sig
 *   (plenum/bls/bls_bft_replica_plenum.py:43-50, 212-225), i.e. python-ursa
 *   Bls.verify_multi_sig: e(sigma, g) == e(H(msg), sum of the keys).
 * Check j: sig[j] (128 B; sig_len as in pv_bls_verify_batch), message
 * msg_idx[j] of msg_blob/msg_off, keys pks[pk_off[j] .. pk_off[j+1]) (128 B each,
 * decoded as keys are; an empty set sums to O).  The sum is prepared like a key
 * (PV_BLS_KEY_NOT_IN_G2 -> verdict 0) together with the generator `gen`; the key
 * set of pv_bls_set_keys is not touched.  At most 65535 checks per call. */
int pv_bls_verify_multi_batch(const uint8_t *gen, const uint8_t *sig, const uint64_t *sig_len, const uint8_t *msg_blob,
                              const uint64_t *msg_off, uint64_t n_msgs, const uint32_t *msg_idx, const uint8_t *pks,
                              const uint64_t *pk_off, uint64_t n, uint8_t *verdict, int device);
/* m multi-signatures; replaces m calls of
 *   BlsCryptoVerifierIndyCrypto.create_multi_sig(signatures) (:99-102), made by
 *   BlsBftReplicaPlenum._calculate_single_multi_sig (bls_bft_replica_plenum.py:278-288),
 *   i.e. python-ursa MultiSignature.new: the sum of the signatures' G1 points.
 * Set j = sigs[set_off[j] .. set_off[j+1]) (128 B each, decoded as sigma is);
 * out[j] = the sum's 128-byte representation: 0x04|x|y, zero-padded; the point
 * at infinity as 0x04|0|1 (AMCL's affine (0, 1) of O). */
int pv_bls_aggregate_sigs(const uint8_t *sigs, const uint64_t *set_off, uint64_t m, uint8_t *out, int device);
/* pks[i] = sks[i] * gen (k keys, 128 B each) */
int pv_bls_pubkeys(const uint8_t *gen, const uint8_t *sks, uint64_t k, uint8_t *pks, int device);
/* HIP-event durations of the last verify call on `device`: message hashing and the check kernel */
int pv_bls_kernel_ms(int device, float *hash_ms, float *verify_ms);
const char *pv_bls_last_error(void);
void pv_bls_shutdown(void);

#ifdef __cplusplus
}
#endif

#endif /* PLENUM_VERIFY_H */
