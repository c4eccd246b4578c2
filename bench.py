"""Bench: Ed25519 verifies/s on MI355X (BASELINE.json metric, config C2).

    python bench.py [--gpus N --steps K --warmup W]          (N > 1: starts the N ranks itself)
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A "step" is one pass of the hot path (hash kernel + curve kernel: libsodium-
exact Ed25519 verification) over one rank's batch of 1,000,000 synthetic
signed requests (distinct keys, 256 B payloads, ~5 % tampered) that is already
resident in HBM, plus — when N > 1 — the RCCL all-gather of every rank's
packed verdict bitmap.  Weak scaling: each rank owns a disjoint index range.

`--gpus N` means N GPUs whichever way the script is started: under
torch.distributed.run (WORLD_SIZE set) it must equal WORLD_SIZE; started
directly with N > 1 it launches the N rank processes itself (fresh children,
created before this process makes any GPU call, one per GPU, RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_ADDR=127.0.0.1 / a free MASTER_PORT) and exits with their
status.  N larger than the visible GPU count is refused (exit 2) unless the
ranks share GPU 0 (PV_BENCH_SHARE_GPU=1, the gloo rehearsal).

Rank 0 prints ONE JSON line.  `value` = all ranks' verifies / max-over-ranks
time.  `roofline` prices the dominant (curve) kernel against the measured
v_mad_u64_u32 issue rate; `cpu_baseline` times libsodium 1.0.18 (the native
call under Plenum's Verifier.verify) on the host cores, on rank 0 after the
timed region and the final barrier (every N).
"""
import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, 'indy-plenum_amd'))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from plenum_gpu import _native as nat  # noqa: E402
from plenum_gpu import synth  # noqa: E402
from plenum_gpu.device import SyntheticBatch, tally_device, tally_device_async  # noqa: E402
from plenum_gpu.quorums import Quorums  # noqa: E402

METRIC = 'Ed25519 verifies/sec at 1/2/4/8 MI355X vs libsodium on host cores'
# BASELINE.json configs as bench workloads (per rank; weak scaling).  c2 is the
# headline (configs[1]); c3/c4 are the pool-tally and sharded mixed-payload cases.
CONFIGS = {
    'c2': dict(mode=synth.FIXED, n=1_000_000, cfg=2, mlen=256, mlen_max=256, key_mod=0,
               workload='C2: 1M Ed25519 request signatures per GPU, distinct keys, 256 B payloads, ~5% tampered '
                        '(BASELINE.json configs[1])'),
    'c3': dict(mode=synth.COMMIT, n=2_500_000, cfg=3, mlen=0, mlen_max=0, key_mod=0, n_nodes=25,
               workload='C3: 25-node pool (f=8), 100k 3PC batches of per-node COMMIT signatures per GPU, '
                        'verify + n-f quorum tally (BASELINE.json configs[2])'),
    'c1': dict(mode=None, n=10_000, cfg=1, mlen=0, mlen_max=0, key_mod=0,
               workload='C1: Plenum request authentication, CoreAuthNr.authenticate over 10k signed write requests '
                        '(256-char payload, DidSigner abbreviated verkeys), batched through ReqAuthenticator-style '
                        'authenticate_batch (BASELINE.json configs[0])'),
    'c4': dict(mode=synth.RANGE, n=8_000_000, cfg=4, mlen=128, mlen_max=4096, key_mod=1 << 20,
               workload='C4: 64M signatures over 8 GPUs = 8M per GPU, payloads uniform 128 B-4 KB, key pool 2^20, '
                        '~5% tampered, RCCL all-gather of verdict bitmaps (BASELINE.json configs[3])'),
}

# Algorithmic work of the curve kernel per verify, counted by the host
# instrumentation build of the same code (tests/test_hostcheck.py pins these):
# field multiplies x 100 + squarings x 55 v_mad_u64_u32 (radix 2^25.5 schoolbook).
# Generic batches (curve_mode PV_CURVE_HALF, the default): half-size scalars, 128
# doublings; decompression of -A and -R (each multiplies by sqrt(-1) for about
# half of all points: the mean is a whole number of multiplies), two 9-entry
# tables, 33 windows, identity test instead of an inversion.  Deferred records
# (~0.2 %) take the full-length verdict (W_*_FULL: 253 doublings + inversion).
# s' B uses signed radix-2^16 digits (8 pairs of affine adds from the tables of
# B and 2^128 B; radix 256 needed 16 pairs: 1299 multiplies per verify).
W_MUL_PER_VERIFY = 1187.0
W_SQ_PER_VERIFY = 1022.0
W_MAD_PER_VERIFY = int(W_MUL_PER_VERIFY * 100 + W_SQ_PER_VERIFY * 55)
W_MUL_FULL, W_SQ_FULL = 1587.5, 1517.0
W_MAD_FULL = int(W_MUL_FULL * 100 + W_SQ_FULL * 55)
# curve_mode PV_CURVE_GROUPED: full-length scalars, CURVE_K = 8 signatures per lane
# sharing one inversion (7 of every 8 254-squaring inversions become 3 multiplies;
# the keyed kernels below share theirs the same way)
W_MUL_GROUPED, W_SQ_GROUPED = 1580.5, 1294.75
W_MAD_GROUPED = int(W_MUL_GROUPED * 100 + W_SQ_GROUPED * 55)
# keyed batches (prepared keys, 8-way comb of -A over the 32-bit words of h):
# 28 doublings instead of 253, no decompression; decompression and the comb
# tables (7 x 29 doublings, 64 affine multiples, one shared inversion) run once
# per distinct key in k_keys
# (base-point digits in radix 2^16 from the eight chunk tables k * 2^(32 q) * B:
# 16 affine adds instead of 32, 762 -> 650 multiplies per verify)
W_MUL_KEYED, W_SQ_KEYED = 649.0, 143.75
W_MUL_KEYPREP, W_SQ_KEYPREP = 1547.5, 1321.0
W_MAD_KEYED = int(W_MUL_KEYED * 100 + W_SQ_KEYED * 55)
# wide key format (radix-256 comb, --key-format wide; C3's node keys by default):
# 24 doublings and 32 key adds per verify; 8 tables x 128 multiples per key,
# built by 128 lanes that each redo the decode and A_q's doublings (latency over
# work: 7.3x the one-lane-per-table work per key, 1.2 -> ~0.7 ms for 25 keys)
# (host op counts, tests/test_hostcheck.py::test_keyed_wide_raw_vectors_and_op_counts)
W_MUL_KEYED_WIDE, W_SQ_KEYED_WIDE = 413.0, 127.75
W_MUL_KEYPREP_WIDE, W_SQ_KEYPREP_WIDE = 69940.0, 126080.0
W_MAD_KEYED_WIDE = int(W_MUL_KEYED_WIDE * 100 + W_SQ_KEYED_WIDE * 55)
# v_mad_u64_u32 issue ceiling of one MI355X measured by tools/ubench/mad_peak.hip
# (profiles/r01_mad_peak.json, best over 1..8 waves/SIMD): lane-ops/s, whole chip.
P_MAD_PER_S = 3.3896e13


# BLS COMMIT check (row f4, --config c3bls): Fp multiplies / squarings of ONE
# check as k_bls_verify runs it (sigma decoding, the two-pairing Miller product
# over precomputed lines, the final exponentiation), counted by the host build
# of csrc/pv_bn254.h (tests/test_bls_oracle.py::test_check_op_counts_pin_bench);
# a 254-bit Montgomery multiply in 10 x 28-bit limbs is 100 + 80 v_mad_i64_i32
# (p's limbs 1 and 3 are zero), a squaring 55 + 80.
BLS_W_MUL, BLS_W_SQR = 11895, 510
BLS_MAD_MUL, BLS_MAD_SQR = 180, 135
BLS_W_MAD = BLS_W_MUL * BLS_MAD_MUL + BLS_W_SQR * BLS_MAD_SQR


def _mad_peak():
    """Best v_mad_u64_u32 lane-ops/s over 1..8 waves/SIMD (tools/ubench/mad_peak.hip,
    profiles/r01_mad_peak.json): the chip's integer multiply-add issue ceiling."""
    path = os.path.join(REPO, 'profiles', 'r01_mad_peak.json')
    try:
        with open(path) as fh:
            return max(float(r['lane_ops_per_s']) for r in json.load(fh)['results']
                       if r['insn'] == 'v_mad_u64_u32')
    except (OSError, KeyError, ValueError):
        return P_MAD_PER_S


TUNED = {}   # pv_tuning fields set from PV_* variables (main)
CURVE_PMC = os.path.join(REPO, 'profiles', 'r05_curve_pmc.json')   # tools/gpu_final_r05.sh on the round-5 build
BLS_PMC = os.path.join(REPO, 'profiles', 'r06_bls_pmc.json')   # tools/gpu_bls_fx6.sh, round-6 build
# the keyed configs' curve launches (tools/gpu_pmc_r05.sh on the round-5 build)
KEYED_PMC = {'c3': os.path.join(REPO, 'profiles', 'r05_c3_pmc.json'),
             'c4': os.path.join(REPO, 'profiles', 'r05_c4_pmc.json')}


def _pmc(path, key):
    try:
        with open(path) as fh:
            return json.load(fh).get(key)
    except (OSError, ValueError):
        return None


def _key_prep_roofline(batch, config, peak, reps=3):
    """k_keys (the narrow-format key preparation of a keyed step) priced like the
    curve: W_MAD_KEYPREP per distinct key / its HIP-event duration on the launch
    stream (pv_keys_prepare_device runs on torch's current stream), after the
    timed region; HBM bytes per launch from the committed PMC profile (C4)."""
    k = int(batch.keys[0].shape[0])
    batch.prepare_keys()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        batch.prepare_keys()
    b.record()
    b.synchronize()
    ms = a.elapsed_time(b) / reps
    if batch.wide:
        # k_keys_wide (C3's node keys): 128 lanes per key redo the decode and the
        # chain to A_q (latency over work), so its MAD fraction is not a kernel
        # efficiency; W = the host-counted work of the 128 slices of one key
        wk = W_MUL_KEYPREP_WIDE * 100 + W_SQ_KEYPREP_WIDE * 55
        return {'kernel': 'k_keys_wide', 'keys': k, 'ms': round(ms, 4),
                'achieved': round(wk * k / (ms * 1e-3) / 1e12, 3), 'peak': round(peak / 1e12, 3),
                'frac': round(wk * k / (ms * 1e-3) / peak, 4), 'traffic': None,
                'note': 'W = {} v_mad lane-ops per key over its 128 table slices (host op count) / HIP-event '
                        'duration, {} launches after the timed region'.format(int(wk), reps)}
    work = (W_MUL_KEYPREP * 100 + W_SQ_KEYPREP * 55) * k
    traffic = _pmc(KEYED_PMC[config], 'key_prep_hbm_bytes_per_launch') if config == 'c4' else None
    return {'kernel': 'k_keys', 'keys': k, 'ms': round(ms, 4), 'achieved': round(work / (ms * 1e-3) / 1e12, 3),
            'peak': round(peak / 1e12, 3), 'frac': round(work / (ms * 1e-3) / peak, 4),
            'traffic': round(traffic * k / (1 << 20)) if traffic else None,
            'note': 'W_MAD_KEYPREP = {} v_mad lane-ops per key (host op count) / HIP-event duration, {} '
                    'launches after the timed region; traffic: PMC FETCH+WRITE of the C4 launch '
                    '(2^20 keys) scaled per key'.format(int(W_MUL_KEYPREP * 100 + W_SQ_KEYPREP * 55), reps)}


def _traffic_per_launch(config='c2', n=None):
    """HBM bytes per curve launch of the config's full-size line from the committed
    rocprofv3 PMC summary (C2: r05_curve_pmc.json; C3 / C4: the keyed curve launch
    of r05_c3 / r05_c4_pmc.json, scaled per signature to the line's n), or None."""
    if config == 'c2':
        return _pmc(CURVE_PMC, 'hbm_bytes_per_launch') if n == CONFIGS['c2']['n'] else None
    per = _pmc(KEYED_PMC[config], 'hbm_bytes_per_unit') if config in KEYED_PMC else None
    return per * n if per and n else None


# SURVEY.md 8(d)'s second work term, W_valu, ALGORITHMIC:
# the non-MAD operations the curve stage's algorithm needs per half-size verify,
# counted per primitive on the host build of the kernel code (tools/hostcheck op
# counters; pinned by tests/test_hostcheck.py::test_op_counts_pin_valu_constants)
# times each primitive's instruction cost in the radix-2^25.5 field code, split
# by issue class:
#   fe_mul   9 x 19 g_j (v_mul_u32_u24) + 10 column carries (v_lshrrev_b64) + the
#            x19 wrap -> 20 half-rate; 5 x 2 f_odd + 10 masks + 2 adds -> 17 full-rate
#   fe_sq    5 x 19 f / 38 f + 10 carries + wrap -> 16 half; 8 x 2 f + 10 masks + 2 -> 20 full
#            (the 13-operand squaring of pv_field.h sq_avail; was 2f_0..9 + 4f_odd)
#   fe_add   10 full; fe_sub / fe_neg 20 full (+2p, -g); fe_carry 30 full (shift, mask, add);
#            fe_carry_even 15 full
# Only work the timed kernel (k_curve_half) does is charged: the SHA-512 of
# R||A||M runs in k_hash, before it.
W_ADD_PER_VERIFY, W_SUB_PER_VERIFY, W_CARRY_PER_VERIFY = 595, 778, 36
W_CARRY_EVEN_PER_VERIFY = 128   # the doublings' T: carries out of the even limbs only (fe_carry_even)
W_SQ2X_PER_VERIFY = 128         # the doublings' 2Z^2 as one squaring (fe_sq2x: 3 more prepared operands)
HALF_COST = {'mul': 20, 'sq': 16}
FULL_COST = {'mul': 17, 'sq': 20, 'add': 10, 'sub': 20, 'carry': 30, 'carry_even': 15}
W_HALF_PER_VERIFY = HALF_COST['mul'] * W_MUL_PER_VERIFY + HALF_COST['sq'] * W_SQ_PER_VERIFY
W_FULL_PER_VERIFY = (FULL_COST['mul'] * W_MUL_PER_VERIFY + FULL_COST['sq'] * W_SQ_PER_VERIFY
                     + FULL_COST['add'] * W_ADD_PER_VERIFY + FULL_COST['sub'] * W_SUB_PER_VERIFY
                     + FULL_COST['carry'] * W_CARRY_PER_VERIFY + FULL_COST['carry_even'] * W_CARRY_EVEN_PER_VERIFY
                     + 3 * W_SQ2X_PER_VERIFY)


# k_hash: one SHA-512 compression of R||A||M per 128-byte block, as pv_sha512.h
# writes it in its minimal gfx950 form.  Per block, by
# instruction: 80 rounds x (Sigma0, Sigma1: 3 64-bit rotates = 6 v_alignbit_b32
# each; Sigma xors, Ch, Maj: 2 v_bitop3_b32 each; 7 64-bit adds incl. K + W as
# v_lshl_add_u64) + 64 schedule words x (sigma0, sigma1: 2 rotates + a shift =
# 5 v_alignbit_b32 + 1 v_lshrrev_b32 each, 2 v_bitop3_b32 each; 3 64-bit adds)
# + the 8 state adds + the big-endian decode of 16 words (2 v_perm_b32 each).
SHA_W_PER_BLOCK = {'v_alignbit_b32': 80 * 12 + 64 * 10, 'v_bitop3_b32': 80 * 8 + 64 * 4,
                   'v_lshl_add_u64': 80 * 7 + 64 * 3 + 8, 'v_lshrrev_b32': 64 * 2, 'v_perm_b32': 32}
SHA_INSN_PER_BLOCK = sum(SHA_W_PER_BLOCK.values())   # 3416
C4_PMC_HASH_BLOCKS = 141038165   # SHA-512 blocks of the C4 launch the PMC passes measured (synth is deterministic)
INT_RATES = [os.path.join(REPO, 'profiles', 'r06_int_rates.json'), os.path.join(REPO, 'profiles', 'r01_int_rates.json')]
# k_sha256 (row f3): one SHA-256 compression per 64-byte block, pv_sha256.h's
# native 32-bit form: 64 rounds x (Sigma0, Sigma1: 3 v_alignbit_b32 each; their
# xors, Ch, Maj: 1 v_bitop3_b32 each; K + W, the three-way t1 sum as v_add3_u32 +
# v_add_u32, t2, e, a) + 48 schedule words x (sigma0, sigma1: 2 alignbit + 1
# v_lshrrev_b32 + 1 bitop3 each; the four-way sum as v_add3_u32 + v_add_u32) + 8
# state adds + the big-endian decode of 16 words (v_perm_b32)
SHA256_W_PER_BLOCK = {'v_alignbit_b32': 64 * 6 + 48 * 4, 'v_bitop3_b32': 64 * 4 + 48 * 2, 'v_lshrrev_b32': 48 * 2,
                      'v_add3_u32': 64 + 48, 'v_add_u32': 64 * 5 + 48 + 8, 'v_perm_b32': 16}
SHA256_INSN_PER_BLOCK = sum(SHA256_W_PER_BLOCK.values())   # 1528


def _insn_rates(peak):
    """Measured lane-ops/s of each instruction (tools/ubench/int_rates.hip, the
    newest committed run), scaled so that its v_mad_u64_u32 equals the best MAD
    ceiling `peak` (the run's first kernels can start below the sustained clock;
    scaling up only raises the ceilings the fractions are priced against)."""
    for path in INT_RATES:
        try:
            with open(path) as fh:
                res = json.load(fh)['results']
        except (OSError, KeyError, ValueError):
            continue
        r = {}
        for x in res:
            r[x['insn']] = max(r.get(x['insn'], 0.0), float(x['lane_ops_per_s']))
        scale = peak / r['v_mad_u64_u32']
        return {k: v * scale for k, v in r.items()}, os.path.relpath(path, REPO)
    return None, None


def hash_compressions(off):
    """SHA-512 blocks of SHA-512(R || A || M) over a batch: ceil((64 + len M + 17) / 128)
    per signature, from the device msg_off."""
    ln = off[1:] - off[:-1]
    return int(((ln + 81 + 127) // 128).sum().item())


def _hash_roofline(blocks, ms, peak):
    """k_hash priced like the curve: SHA_INSN_PER_BLOCK lane-instructions per
    SHA-512 block x the blocks of one launch / its HIP-event duration (pre-checks
    + k_hash on the launch stream, pv_kernel_timing_sha), against the issue
    ceiling of that instruction mix at the measured per-instruction rates."""
    rates, src = _insn_rates(peak)
    if not rates or ms <= 0:
        return None
    miss = [k for k in SHA_W_PER_BLOCK if k not in rates]
    for k in miss:   # an older rates file: price the missing ones at the half-rate alignbit's rate
        rates[k] = rates['v_alignbit_b32']
    t_block = sum(w / rates[k] for k, w in SHA_W_PER_BLOCK.items())   # s per block, whole chip
    # the C4 k_hash launch's PMC passes (tools/gpu_pmc_r05.sh; k_hash unchanged since):
    # HBM bytes and executed VALU instructions per SHA-512 block
    pmc = None
    try:
        with open(KEYED_PMC['c4']) as fh:
            kh = json.load(fh)['kernels']['pv::k_hash']
        pblocks = C4_PMC_HASH_BLOCKS
        pmc = {'hbm_bytes_per_block': round(kh['hbm_bytes_per_launch'] / pblocks, 1),
               'executed_valu_insn_per_block': round(kh['SQ_INSTS_VALU'] * 64 / pblocks, 1),
               'l2_hit_rate': round(kh['l2_hit_rate'], 3),
               'source': os.path.relpath(KEYED_PMC['c4'], REPO) + ' (k_hash of the 8M-signature C4 launch, '
                                                                  '{} blocks)'.format(pblocks)}
    except (OSError, KeyError, ValueError, TypeError):
        pass
    ceiling = 1.0 / t_block
    rate = blocks / (ms * 1e-3)
    return {'kernel': 'k_hash (+ k_precheck)', 'blocks': blocks, 'ms': round(ms, 4),
            'achieved': round(rate * SHA_INSN_PER_BLOCK / 1e12, 3),
            'peak': round(ceiling * SHA_INSN_PER_BLOCK / 1e12, 3), 'unit': 'T lane-instructions/s',
            'frac': round(rate / ceiling, 4), 'blocks_per_s': round(rate, 1),
            'ceiling_blocks_per_s': round(ceiling, 1), 'insn_per_block': dict(SHA_W_PER_BLOCK),
            'traffic': round(pmc['hbm_bytes_per_block'] * blocks) if pmc else None, 'pmc': pmc,
            'rates_source': src + (' (no rate for {}: priced at v_alignbit_b32)'.format(miss) if miss else ''),
            'note': 'W = {} lane-instructions per SHA-512 block (pv_sha512.h, counted per instruction class) x '
                    'ceil((len M + 81) / 128) blocks per signature from msg_off; time = HIP events from the '
                    'launch start to the end of k_hash (pre-checks included, k_lattice excluded)'.format(
                        SHA_INSN_PER_BLOCK)}


def _sha256_roofline(blocks, ms, peak, step_blocks=None, step_ms=None):
    """k_sha256 priced per SHA-256 block like k_hash: SHA256_INSN_PER_BLOCK
    lane-instructions x the blocks of one launch / its duration, against that
    instruction mix at the measured per-instruction rates."""
    rates, src = _insn_rates(peak)
    if not rates or ms <= 0:
        return None
    t_block = sum(w / rates[k] for k, w in SHA256_W_PER_BLOCK.items())
    ceiling = 1.0 / t_block
    rate = blocks / (ms * 1e-3)
    out = {'bound': 'valu', 'kernel': 'k_sha256 (leaf digests, prefix 0x00)', 'blocks': blocks, 'ms': round(ms, 4),
           'achieved': round(rate * SHA256_INSN_PER_BLOCK / 1e12, 3),
           'peak': round(ceiling * SHA256_INSN_PER_BLOCK / 1e12, 3), 'unit': 'T lane-instructions/s',
           'frac': round(rate / ceiling, 4), 'traffic': None, 'insn_per_block': dict(SHA256_W_PER_BLOCK),
           'rates_source': src,
           'note': 'W = {} lane-instructions per SHA-256 block (pv_sha256.h, per instruction class) x ceil((1 + 256 + '
                   '9) / 64) = 5 blocks per leaf; time = HIP events around pv_sha256_batch_device on the launch '
                   'stream, after the timed region'.format(SHA256_INSN_PER_BLOCK)}
    if step_blocks and step_ms:
        out['per_step'] = {'blocks': step_blocks, 'ms': round(step_ms, 4),
                           'frac': round(step_blocks / (step_ms * 1e-3) / ceiling, 4),
                           'note': 'every block of the step (5 per leaf + 2 per internal node) / the step time: '
                                   'the 20 level launches charged too'}
    return out


def _class_rates(peak):
    """Issue rates of the half-rate class (64-bit shifts / adds, v_alignbit,
    v_mul_u32_u24, v_add_co) and of full-rate 32-bit VALU, as ratios to
    v_mad_u64_u32 measured in ONE micro-benchmark run (profiles/r01_int_rates.json)
    scaled to the best MAD ceiling `peak`."""
    path = os.path.join(REPO, 'profiles', 'r01_int_rates.json')
    with open(path) as fh:
        r = {x['insn']: float(x['lane_ops_per_s']) for x in json.load(fh)['results']}
    mad = r['v_mad_u64_u32']
    half = sum(r[k] for k in ('v_alignbit_b32', 'v_lshrrev_b64', 'v_lshl_add_u64', 'v_mul_u32_u24', 'v_add_co_u32')) / 5
    full = (r['v_add_u32'] + r['v_xor_b32']) / 2
    return peak * half / mad, peak * full / mad


def _combined_issue(kernel_rate, peak):
    """SURVEY.md 8(d)'s integer-ALU roofline for the C2 curve kernel,
    1 / (W_mad/P_mad + W_half/P_half + W_full/P_full), every W from the algorithm
    (constants above, pinned by host op counts) and every P measured (the MAD
    ceiling; the other two classes at their measured ratios to it).  Beside it,
    `issue_efficiency` prices the instructions the kernel actually EXECUTES
    (rocprofv3 SQ_INSTS_VALU, profiles/r05_curve_pmc.json) the same way."""
    try:
        p_half, p_full = _class_rates(peak)
    except (OSError, KeyError, ValueError):
        return None
    t = W_MAD_PER_VERIFY / peak + W_HALF_PER_VERIFY / p_half + W_FULL_PER_VERIFY / p_full
    rate = 1.0 / t
    out = {'model': 'SURVEY.md 8(d): 1 / (W_mad/P_mad + W_half/P_half + W_full/P_full), algorithmic W',
           'w_mad_per_verify': W_MAD_PER_VERIFY, 'w_half_per_verify': int(W_HALF_PER_VERIFY),
           'w_full_per_verify': int(W_FULL_PER_VERIFY), 'p_mad': round(peak / 1e12, 3),
           'p_half': round(p_half / 1e12, 3), 'p_full': round(p_full / 1e12, 3), 'unit': 'T lane-ops/s',
           'roofline_verifies_per_s': round(rate, 1), 'frac': round(kernel_rate / rate, 4),
           'source': 'W from tools/hostcheck op counters x per-primitive costs (bench.py); '
                     'P ratios from profiles/r01_int_rates.json'}
    try:
        with open(CURVE_PMC) as fh:
            d = json.load(fh)
        insts = float(d['kernels'][d['curve_kernel']]['SQ_INSTS_VALU'])
        n, deferred = int(d['c2_signatures']), int(d['c2_deferred'])
        mad_lane_ops = W_MAD_PER_VERIFY * (n - deferred) + W_MAD_FULL * deferred
        other = (insts * 64 - mad_lane_ops) / n
        # executed non-MAD instructions priced at the half-rate class (the
        # bulk of them: 64-bit shifts, v_mul_u32_u24, add-with-carry)
        rate_exec = 1.0 / (W_MAD_PER_VERIFY / peak + other / p_half)
        out['issue_efficiency'] = {'executed_non_mad_per_verify': round(other), 'rate_at_executed_work': round(rate_exec, 1),
                                   'frac': round(kernel_rate / rate_exec, 4),
                                   'source': 'rocprofv3 SQ_INSTS_VALU of the C2 curve launch (profiles/r05_curve_pmc.json)'}
    except (OSError, KeyError, ValueError):
        pass
    return out


def cpu_baseline(batch, workload, seconds=1.5, sample=8192):
    """libsodium crypto_sign_verify_detached on the host cores over the first
    `sample` signatures of this rank's workload (copied to host)."""
    so = os.path.join(REPO, 'oracle', 'liboracle.so')
    if not os.path.exists(so):
        return None
    lib = ctypes.CDLL(so)
    lib.cpu_baseline_rate.restype = ctypes.c_double
    lib.cpu_baseline_rate.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_double,
                                      ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_uint64)]
    pk = batch.pk[:sample].cpu().numpy().copy()
    sig = batch.sig[:sample].cpu().numpy().copy()
    off = batch.off[:sample + 1].cpu().numpy().astype(np.uint64)
    blob = batch.blob[:int(off[-1]) + 16].cpu().numpy().copy()
    threads = len(os.sched_getaffinity(0))
    threads = min(threads, int(os.environ.get('OMP_NUM_THREADS', threads)))
    kind = ctypes.c_int()
    acc = ctypes.c_uint64()
    p = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
    sodium = b'/opt/conda/lib/libsodium.so.23'
    rate = lib.cpu_baseline_rate(sodium, p(pk), p(sig), p(blob), p(off), sample, threads, seconds,
                                 ctypes.byref(kind), ctypes.byref(acc))
    rate1 = lib.cpu_baseline_rate(sodium, p(pk), p(sig), p(blob), p(off), sample, 1, min(seconds, 1.0),
                                  ctypes.byref(kind), ctypes.byref(acc))
    cpu = ''
    try:
        with open('/proc/cpuinfo') as fh:
            for line in fh:
                if line.startswith('model name'):
                    cpu = line.split(':', 1)[1].strip()
                    break
    except OSError:
        pass
    name = 'libsodium 1.0.18 crypto_sign_verify_detached' if kind.value == 0 else \
        'C restatement oracle/ed25519_oracle.c (libsodium not loadable)'
    return {'value': round(rate, 1), 'unit': 'verifies/s', 'cores': threads,
            'kind': 'reference' if kind.value == 0 else 'port',
            'sample': '{} ({} threads, {:.1f} s wall; 1 thread: {:.1f} verifies/s) over the first {} signatures '
                      'of the {} workload, host {}'.format(name, threads, seconds, rate1, sample, workload, cpu)}


class _SodiumVerifyKey:
    """libsodium 1.0.18 crypto_sign_open on the host: the native call under the
    reference's VerifyKey.verify (stp_core/crypto/nacl_wrappers.py:86-108).
    cpu_baseline only: the product has no CPU verify path."""
    lib = None

    def __init__(self, raw):
        if _SodiumVerifyKey.lib is None:
            _SodiumVerifyKey.lib = ctypes.CDLL('/opt/conda/lib/libsodium.so.23')
            _SodiumVerifyKey.lib.sodium_init()
        self.raw = bytes(raw)

    def verify(self, sm):
        m = ctypes.create_string_buffer(len(sm))
        mlen = ctypes.c_ulonglong()
        return _SodiumVerifyKey.lib.crypto_sign_open(m, ctypes.byref(mlen), sm, ctypes.c_ulonglong(len(sm)),
                                                     self.raw) == 0


def _sodium_did_verifier():
    from plenum_gpu.base58 import b58decode
    from plenum_gpu.verifier import DidVerifier

    class SodiumDidVerifier(DidVerifier):
        """DidVerifier (plenum/common/verifier.py:25-54) verifying on the host with libsodium."""
        @DidVerifier.verkey.setter
        def verkey(self, value):
            self._verkey = value
            raw = b58decode(value)
            if len(raw) != 32:
                raise ValueError('The key must be exactly 32 bytes long')
            self._sk = _SodiumVerifyKey(raw)
            self._vr = None

        @property
        def raw_verkey(self):
            return None   # never served from the GPU prefetch cache

        def verify(self, sig, msg):
            return self._sk.verify(bytes(sig) + bytes(msg))
    return SodiumDidVerifier


def end_to_end(batch, dedup, reps=5):
    """Host-buffer rate of pv_verify_batch on this rank's workload: pk/sig/M in
    pageable host memory -> H2D (chunked, overlapped with the kernels) -> one
    fused verify launch per chunk + a deferred pass -> D2H verdicts.  SURVEY.md 8(d)'s second number; never `value`."""
    pk, sig = batch.pk.cpu().numpy(), batch.sig.cpu().numpy()
    off = batch.off.cpu().numpy().astype(np.uint64)
    blob = batch.blob.cpu().numpy()[:int(off[-1])]
    want = ~batch.tamper.cpu().numpy().astype(bool)
    mism, rate = 0, {}
    try:
        for staging in ('pageable', 'pinned'):   # A/B of the host staging; `value` = the default (pinned)
            nat.set_host_staging(staging)
            got = nat.verify_batch_arrays(pk, sig, blob, off, device_mask=1 << batch.device.index, dedup_keys=dedup)
            mism += int((got != want).sum())
            # second untimed call: the first calls after a staging switch (re)allocate and
            # first-touch the page-locked slots and the second workspace
            nat.verify_batch_arrays(pk, sig, blob, off, device_mask=1 << batch.device.index, dedup_keys=dedup)
            calls = []
            for _ in range(reps):
                t0 = time.perf_counter()
                nat.verify_batch_arrays(pk, sig, blob, off, device_mask=1 << batch.device.index, dedup_keys=dedup)
                calls.append(time.perf_counter() - t0)
            rate[staging] = sum(calls) / reps
            rate[staging + '_calls'] = [round(c * 1e3, 3) for c in calls]
    finally:
        nat.set_host_staging('pinned')
    # caller buffers already page-locked (torch pin_memory()): the library DMAs
    # pk / sig / blob straight from them, only the offsets are staged
    locked = [torch.from_numpy(np.ascontiguousarray(a)).pin_memory() for a in (pk, sig, blob, off)]
    lpk, lsig, lblob, loff = (t.numpy() for t in locked)
    got = nat.verify_batch_arrays(lpk, lsig, lblob, loff, device_mask=1 << batch.device.index, dedup_keys=dedup)
    mism += int((got != want).sum())
    nat.verify_batch_arrays(lpk, lsig, lblob, loff, device_mask=1 << batch.device.index, dedup_keys=dedup)
    calls = []
    for _ in range(reps):
        t0 = time.perf_counter()
        nat.verify_batch_arrays(lpk, lsig, lblob, loff, device_mask=1 << batch.device.index, dedup_keys=dedup)
        calls.append(time.perf_counter() - t0)
    rate['locked'] = sum(calls) / reps
    dt = rate['pinned']
    return {'value': round(batch.n / dt, 1), 'unit': 'verifies/s', 'ms': round(dt * 1e3, 3),
            'verdict_mismatches': mism,
            'calls_ms': rate['pinned_calls'],
            'pageable_staging': {'value': round(batch.n / rate['pageable'], 1),
                                 'ms': round(rate['pageable'] * 1e3, 3)},
            'page_locked_inputs': {'value': round(batch.n / rate['locked'], 1), 'ms': round(rate['locked'] * 1e3, 3),
                                   'note': 'the same call with the caller\'s buffers already page-locked (torch '
                                           'pin_memory()): pk / sig / blob DMA\'d directly, no gather copy'},
            'path': 'pv_verify_batch from pageable host numpy buffers ({:.0f} MB in, {} B out): chunks gathered by '
                    'host threads into two page-locked slots (leading chunks of 32k and 64k signatures), DMA on a '
                    'copy stream overlapped with one fused pre-check + hash + lattice + curve launch per chunk '
                    '(k_chunk_half; chunks alternate over two compute streams), one lane-quad pass over the '
                    'deferred records, D2H verdicts through a page-locked buffer; 2 untimed calls, then mean '
                    'of {} calls'.format(
                        (pk.nbytes + sig.nbytes + blob.nbytes + off.nbytes) / 1e6, batch.n, reps)}


def small_batch_latency(batch, sizes=(1, 100, 1000), reps=20):
    """Host-buffer call time of Plenum's per-pass batch sizes (stp_core/config.py:32-33:
    <= 100 client / 1,000 node messages) on this rank's first signatures: the
    one-launch latency kernel, with the keys uncached (top level)
    and in the persistent device key cache ('cached': the keyed latency kernel,
    DESIGN.md 4f).  Median and min of `reps` calls."""
    pk, sig = batch.pk.cpu().numpy(), batch.sig.cpu().numpy()
    off = batch.off.cpu().numpy().astype(np.uint64)
    blob = batch.blob.cpu().numpy()
    want = ~batch.tamper.cpu().numpy().astype(bool)
    mask = 1 << batch.device.index

    def measure():
        res, bad = {}, 0
        for n in sizes:
            args = (pk[:n], sig[:n], blob[:int(off[n])], off[:n + 1])
            got = nat.verify_batch_arrays(*args, device_mask=mask)
            bad += int((got != want[:n]).sum())
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                nat.verify_batch_arrays(*args, device_mask=mask)
                ts.append(time.perf_counter() - t0)
            ts.sort()
            res[str(n)] = {'ms_median': round(ts[reps // 2] * 1e3, 3), 'ms_min': round(ts[0] * 1e3, 3)}
        return res, bad

    nat.keycache_clear()
    out, mism = measure()
    nat.keycache_add(pk[:max(sizes)])
    try:
        out['cached'], m2 = measure()
    finally:
        nat.keycache_clear()
    out['verdict_mismatches'] = mism + m2
    return out


def main_c1(args):
    """C1: the Plenum request-authentication path end to end (host preprocessing
    + one GPU verify per batch) vs the same per-request path on libsodium."""
    from plenum_gpu.client_authn import CoreAuthNr
    cfg = CONFIGS['c1']
    n = args.n or cfg['n']
    torch.cuda.set_device(0)
    reqs, ids = synth.c1_requests(n)
    authnr = CoreAuthNr(['buy'], [], [])
    for idr, vk in ids:
        authnr.addIdr(idr, vk)
    want = [[idr] for idr, _ in ids]
    for _ in range(args.warmup):
        authnr.authenticate_batch(reqs, pause_gc=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = authnr.authenticate_batch(reqs, pause_gc=True)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    mism = sum(1 for a, b in zip(out, want) if a != b)
    value = n * args.steps / elapsed
    res = {
        'metric': METRIC, 'value': round(value, 1), 'unit': 'verifies/s', 'n_gpus': 1, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': round(elapsed / args.steps * 1e3, 3), 'higher_is_better': True,
        'scaling': 'weak', 'vs_baseline': None, 'dtype': 'u32',
        'data': 'synthetic signed requests (plenum_gpu/synth.py c1_requests), one signature per request',
        'config': {'workload': cfg['workload'], 'name': 'c1', 'requests': n, 'host_threads': 1},
        'verdict_mismatches': mism,
        'roofline': None,
        'note': 'host-bound: base58/serialization/key resolution per request on 1 thread (native _host module); '
                'the GPU verify of the batch is a few percent of the step',
        'cpu_baseline': None,
    }
    if not args.no_cpu_baseline:
        sv = _sodium_did_verifier()
        base = CoreAuthNr(['buy'], [], [])
        base._verifier = lambda verifier, verkey, idr: verifier(verkey, identifier=idr)  # fresh key per call, as the reference
        for idr, vk in ids:
            base.addIdr(idr, vk)
        done, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < 3.0:
            r = reqs[done % n]
            assert base.authenticate(r, verifier=sv) == [r['identifier']]
            done += 1
        rate = done / (time.perf_counter() - t0)
        res['cpu_baseline'] = {
            'value': round(rate, 1), 'unit': 'verifies/s', 'cores': 1, 'kind': 'port',
            'sample': '{} requests (3 s) through the same CoreAuthNr.authenticate path one request at a time, '
                      'verification by libsodium 1.0.18 crypto_sign_open on 1 host thread (the node verifies on its '
                      'single Looper thread)'.format(done)}
    if TUNED:
        res['tuning'] = dict(TUNED)
    print(json.dumps(res), flush=True)
    return 0 if mism == 0 else 3


def main_bls(args):
    """Row f4: the BLS COMMIT check of a 25-node pool (C3's shape): every node's
    COMMIT of every 3PC batch carries a BLS signature over that batch's
    MultiSignatureValue (plenum/bls/bls_bft_replica_plenum.py:194-213); a step
    verifies all of them (pv_bls_verify_batch_device: hash each message once,
    group by key, one two-pairing check per COMMIT) and tallies the n - f COMMIT
    quorum per batch over the COMMITs that pass (pv_tally_votes_device).
    Synthetic keys/messages; signatures made on the GPU; ~5 % corrupted."""
    import hashlib
    from plenum_gpu import base58
    from plenum_gpu.bls import GENERATOR, MultiSignatureValue
    from plenum_gpu.device import _p, _stream
    nn = 25
    nb = (args.n or 2_500_000) // nn
    n = nb * nn
    q = Quorums(nn).commit.value
    torch.cuda.set_device(0)
    dev = torch.device('cuda', 0)
    nat.ensure_init(1)
    lib = nat.load()
    r_order = 0x2523648240000001ba344d8000000007ff9f800000000010a10000000000000d
    sks = np.frombuffer(b''.join((int.from_bytes(hashlib.sha256(b'plenum-gpu/bls-node' + bytes([i])).digest(), 'big')
                                  % r_order).to_bytes(32, 'big') for i in range(nn)), np.uint8).reshape(nn, 32)
    gen = base58.b58decode(GENERATOR)
    pks = nat.bls_pubkeys(gen, sks)
    assert not nat.bls_set_keys(gen, pks).any()

    def root(tag, b):
        return base58.b58encode(hashlib.sha256(tag + b.to_bytes(8, 'little')).digest()).decode()
    msgs = [MultiSignatureValue(1, root(b'state', b), root(b'pool', b // 100), root(b'txn', b), 1700000000 + b)
            .as_single_value() for b in range(nb)]
    blob_h, off_h = nat.pack_messages(msgs)
    blob = torch.zeros(blob_h.size + 64, dtype=torch.uint8, device=dev)
    blob[:blob_h.size] = torch.from_numpy(blob_h.copy()).to(dev)
    off = torch.from_numpy(off_h.astype(np.int64)).to(dev)
    midx = torch.arange(nb, dtype=torch.int32, device=dev).repeat_interleave(nn)
    kidx = torch.arange(nn, dtype=torch.int32, device=dev).repeat(nb)
    sig = torch.empty((n, 128), dtype=torch.uint8, device=dev)
    sk_d = torch.from_numpy(sks.copy()).to(dev)
    nat._bls_check('pv_bls_sign_batch_device', lib.pv_bls_sign_batch_device(
        _p(sk_d), _p(blob), _p(off), nb, _p(midx), _p(kidx), n, _p(sig), 0, _stream(dev)))
    # ~5 % corrupted: half a flipped bit of x (decodes to O), half another batch's signature
    g = torch.Generator(device=dev)
    g.manual_seed(41)
    bad = torch.rand(n, device=dev, generator=g) < 0.05
    bidx = torch.nonzero(bad).flatten()
    half = bidx[: bidx.numel() // 2]
    sig[half, 7] ^= 0x10
    other = bidx[bidx.numel() // 2:]
    sig[other] = sig[(other + nn) % n]
    expect = ~bad
    sender = kidx.clone()
    batch_off = torch.arange(nb + 1, dtype=torch.int64, device=dev) * nn
    verdict = torch.empty(n, dtype=torch.uint8, device=dev)
    votes = torch.empty(nb, dtype=torch.int32, device=dev)
    reached = torch.empty(nb, dtype=torch.uint8, device=dev)

    def step():
        nat._bls_check('pv_bls_verify_batch_device', lib.pv_bls_verify_batch_device(
            _p(sig), _p(blob), _p(off), nb, _p(midx), _p(kidx), n, _p(verdict), 0, _stream(dev)))
        tally_device(verdict, sender, batch_off, nn, q, votes, reached)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    hash_ms = verify_ms = 0.0
    for _ in range(args.steps):
        step()
        h, v = nat.bls_kernel_ms(0)
        hash_ms += h
        verify_ms += v
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    got = verdict.bool()
    mism = int((got != expect).sum().item())
    want_votes = expect.view(nb, nn).sum(1)
    q_mism = int(((want_votes >= q) != reached.bool()).sum().item()) + int((want_votes != votes).sum().item())
    value = n * args.steps / elapsed
    verify_ms /= args.steps
    hash_ms /= args.steps
    peak = _mad_peak()
    achieved = BLS_W_MAD * n / (verify_ms * 1e-3)
    out = {
        'metric': 'BLS COMMIT checks/sec (verify_sig over AMCL BN254, row f4) on 1 MI355X', 'value': round(value, 1),
        'unit': 'checks/s', 'n_gpus': 1, 'steps': args.steps, 'warmup': args.warmup,
        'ms_per_step': round(elapsed / args.steps * 1e3, 3), 'higher_is_better': True, 'scaling': 'weak',
        'vs_baseline': None, 'dtype': 'i32 limbs (GF(p) 254-bit, v_mad_i64_i32)',
        'data': 'synthetic: 25 node keys, one MultiSignatureValue per 3PC batch, signatures made on the GPU, '
                '~5% corrupted; parity UNPINNED (ursa absent), verdicts checked against the synthetic spec',
        'config': {'workload': 'C3-BLS: 25-node pool (f=8), {} 3PC batches, every COMMIT BLS-verified + n-f tally'
                   .format(nb), 'name': 'c3bls', 'checks': n, 'batches': nb},
        'verdict_mismatches': mism, 'quorum_mismatches': q_mism, 'quorums_reached': int(reached.sum().item()),
        'kernel_ms': {'hash': round(hash_ms, 3), 'verify': round(verify_ms, 3)},
        'roofline': {'bound': 'valu', 'kernel': 'k_bls_verify_pair (+ k_bls_sigprep)', 'achieved': round(achieved / 1e12, 3),
                     'peak': round(peak / 1e12, 3), 'unit': 'T v_mad lane-ops/s', 'frac': round(achieved / peak, 4),
                     'work_per_check': BLS_W_MAD,
                     'traffic': (round(_pmc(BLS_PMC, 'hbm_bytes_per_unit') * n, 1)
                                 if _pmc(BLS_PMC, 'hbm_bytes_per_unit') else None),
                     'traffic_source': 'HBM bytes per check from rocprofv3 FETCH_SIZE / WRITE_SIZE passes '
                                       '(profiles/r06_bls_pmc.json) x the checks of this launch',
                     'note': 'W = {} Fp mul x 180 + {} sqr x 135 v_mad_i64_i32 per check (host op counts of '
                             'the one-lane schedule; the lane pair repeats the inversion of the final '
                             'exponentiation on both lanes, not counted); time = the sigma-prep + pair kernels'
                             .format(BLS_W_MUL, BLS_W_SQR)},
    }
    # the per-COMMIT regime: host calls of 1 check, one 3PC batch (25 COMMITs,
    # one message) and 10 batches (pv_bls_verify_batch, host buffers)
    sig_h = sig[:250].cpu().numpy()
    mi_h = midx[:250].cpu().numpy().astype(np.uint32)
    ki_h = kidx[:250].cpu().numpy().astype(np.uint32)
    lat, lat_bad = {}, 0
    for m in (1, 25, 250):
        vb = nat.bls_verify_arrays(sig_h[:m], blob_h, off_h[:int(mi_h[m - 1]) + 2], mi_h[:m], ki_h[:m])
        lat_bad += int((vb != expect[:m].cpu().numpy()).sum())
        ts = []
        for _ in range(5):
            t1 = time.perf_counter()
            nat.bls_verify_arrays(sig_h[:m], blob_h, off_h[:int(mi_h[m - 1]) + 2], mi_h[:m], ki_h[:m])
            ts.append(time.perf_counter() - t1)
        ts.sort()
        lat[str(m)] = {'ms_median': round(ts[2] * 1e3, 3), 'ms_min': round(ts[0] * 1e3, 3)}
    lat['verdict_mismatches'] = lat_bad
    out['small_batch_latency'] = lat
    if not args.no_cpu_baseline:
        orc = ctypes.CDLL(os.path.join(REPO, 'oracle', 'libbls_oracle.so'))
        sample = 2000
        threads = min(16, os.cpu_count() or 1)
        sig_h = np.ascontiguousarray(sig[:sample].cpu().numpy())
        mi = np.ascontiguousarray(midx[:sample].cpu().numpy().astype(np.uint32))
        ki = np.ascontiguousarray(kidx[:sample].cpu().numpy().astype(np.uint32))
        blob16 = np.concatenate([blob_h, np.zeros(16, np.uint8)])
        res = np.zeros(sample, np.uint8)
        pp = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
        t0 = time.perf_counter()
        orc.bls_oracle_verify_batch(pp(sig_h), None, pp(blob16), pp(off_h), pp(mi), pp(ki), pp(np.ascontiguousarray(pks)),
                                    gen, ctypes.c_uint64(sample), pp(res), threads)
        dt = time.perf_counter() - t0
        out['cpu_baseline'] = {'value': round(sample / dt, 1), 'unit': 'checks/s', 'cores': threads, 'kind': 'port',
                               'sample': '{} checks of this workload, oracle/bn254_oracle.c (2 pairings per check, '
                                         'as ursa) on {} host threads'.format(sample, threads),
                               'agrees_with_gpu': bool((res.astype(bool) == got[:sample].cpu().numpy()).all())}
    if TUNED:
        out['tuning'] = dict(TUNED)
    print(json.dumps(out), flush=True)


def main_f3(args):
    """Row f3: ledger Merkle tree hash (leaf SHA-256 + RFC 6962 levels) of 1M x 256 B
    leaves resident in HBM, vs the same tree hash with hashlib on one host thread."""
    import hashlib
    from plenum_gpu.device import _p, _stream
    n = args.n or (1 << 20)
    ln = 256
    torch.cuda.set_device(0)
    dev = torch.device('cuda', 0)
    nat.ensure_init(1)
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    blob = torch.zeros(n * ln + 16, dtype=torch.uint8, device=dev)
    blob[:n * ln] = torch.randint(0, 256, (n * ln,), dtype=torch.uint8, device=dev, generator=g)
    off = torch.arange(n + 1, dtype=torch.int64, device=dev) * ln
    leaves = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    root = torch.zeros(32, dtype=torch.uint8, device=dev)
    lib = nat.load()

    def step():
        nat._check('pv_merkle_root_device', lib.pv_merkle_root_device(_p(blob), _p(off), n, _p(leaves), _p(root), 0,
                                                                      _stream(dev)))
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # the leaf kernel alone, for its roofline: pv_sha256_batch_device over the same
    # leaves (k_sha256, prefix 0x00), HIP events on the launch stream
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    nat._check('pv_sha256_batch_device', lib.pv_sha256_batch_device(_p(blob), _p(off), n, 0, _p(leaves), 0,
                                                                    _stream(dev)))
    ev0.record()
    for _ in range(5):
        nat._check('pv_sha256_batch_device', lib.pv_sha256_batch_device(_p(blob), _p(off), n, 0, _p(leaves), 0,
                                                                        _stream(dev)))
    ev1.record()
    ev1.synchronize()
    leaf_ms = ev0.elapsed_time(ev1) / 5
    leaf_blocks = n * ((1 + ln + 9 + 63) // 64)
    step_blocks = leaf_blocks + (n - 1) * ((1 + 64 + 9 + 63) // 64)
    # check: root of the same leaves with hashlib (level-wise RFC 6962)
    host = blob[:n * ln].cpu().numpy()
    lvl = [hashlib.sha256(b'\x00' + host[i * ln:(i + 1) * ln].tobytes()).digest() for i in range(n)]
    leaf_hashes = list(lvl)
    t1 = time.perf_counter()
    while len(lvl) > 1:
        nxt = [hashlib.sha256(b'\x01' + lvl[i] + lvl[i + 1]).digest() for i in range(0, len(lvl) - 1, 2)]
        if len(lvl) % 2:
            nxt.append(lvl[-1])
        lvl = nxt
    mism = int(bytes(root.cpu().numpy()) != lvl[0])
    # CPU baseline: the same tree hash on one host thread over a bounded sample
    sample = min(n, 1 << 17)
    t0 = time.perf_counter()
    lv = [hashlib.sha256(b'\x00' + host[i * ln:(i + 1) * ln].tobytes()).digest() for i in range(sample)]
    while len(lv) > 1:
        nx = [hashlib.sha256(b'\x01' + lv[i] + lv[i + 1]).digest() for i in range(0, len(lv) - 1, 2)]
        if len(lv) % 2:
            nx.append(lv[-1])
        lv = nx
    cpu_rate = sample / (time.perf_counter() - t0)
    del t1
    # CompactMerkleTree.extend's bulk step from host leaves (GpuTreeHasher._hash_full,
    # ledger/compact_merkle_tree.py:183): n - 1 leaves = one full subtree per set bit
    from plenum_gpu.merkle import GpuTreeHasher
    th = GpuTreeHasher()
    host_leaves = [host[i * ln:(i + 1) * ln].tobytes() for i in range(n - 1)]
    th._hash_full(host_leaves, 0, n - 1)
    t0 = time.perf_counter()
    ext_root, ext_hashes = th._hash_full(host_leaves, 0, n - 1)
    ext_s = time.perf_counter() - t0
    lv = leaf_hashes[:n - 1]
    while len(lv) > 1:
        nx = [hashlib.sha256(b'\x01' + lv[i] + lv[i + 1]).digest() for i in range(0, len(lv) - 1, 2)]
        if len(lv) % 2:
            nx.append(lv[-1])
        lv = nx
    mism += int(ext_root != lv[0]) + int(len(ext_hashes) != bin(n - 1).count('1'))
    # CompactMerkleTree.append x 10k (ledger/compact_merkle_tree.py:155-160): per
    # leaf _hash_full(leaves, 0, 1) + one hash_children per carry, then the root
    # fold — the call pattern of the reference tree driven by GpuTreeHasher
    # (single hashes stay on hashlib: no GPU call per node)
    n_app = min(10_000, n - 1)

    def appends(hasher):
        size, hashes = 0, []
        for i in range(n_app):
            h, _ = hasher._hash_full(host_leaves, i, i + 1)
            s = size
            while s & 1:            # carries: merge equal-size subtrees
                h = hasher.hash_children(hashes.pop(), h)
                s >>= 1
            hashes.append(h)
            size += 1
        return hasher._hash_fold(tuple(hashes))
    t0 = time.perf_counter()
    app_root = appends(th)
    app_s = time.perf_counter() - t0
    lv = leaf_hashes[:n_app]
    while len(lv) > 1:
        nx = [hashlib.sha256(b'\x01' + lv[i] + lv[i + 1]).digest() for i in range(0, len(lv) - 1, 2)]
        if len(lv) % 2:
            nx.append(lv[-1])
        lv = nx
    mism += int(app_root != lv[0])
    # small batches: sha256_batch / merkle_root around the host/GPU dispatch size
    from plenum_gpu import merkle as mk_mod
    small = []
    for k in (64, 256, 1024, 4096, 16384):
        msgs = host_leaves[:k]
        row = {'items': k}
        for tag, thr in (('host', 1 << 62), ('gpu', 0)):
            mk_mod.GPU_MIN_ITEMS = thr
            mk_mod.sha256_batch(msgs, prefix=0)
            t0 = time.perf_counter()
            for _ in range(5):
                mk_mod.sha256_batch(msgs, prefix=0)
            row[tag + '_us'] = round((time.perf_counter() - t0) / 5 * 1e6, 1)
        small.append(row)
    mk_mod.GPU_MIN_ITEMS = 512
    value = n * args.steps / elapsed
    res = {
        'metric': 'Merkle tree hash leaves/sec (ledger TreeHasher.hash_full_tree, SHA-256)', 'value': round(value, 1),
        'unit': 'leaves/s', 'n_gpus': 1, 'steps': args.steps, 'warmup': args.warmup,
        'ms_per_step': round(elapsed / args.steps * 1e3, 3), 'higher_is_better': True, 'scaling': 'weak',
        'vs_baseline': None, 'dtype': 'u32', 'data': 'synthetic random leaves resident in HBM',
        'config': {'workload': 'SURVEY.md 8(f) f3: Merkle tree hash of 1M x 256 B ledger leaves (leaf digests + '
                               'RFC 6962 levels), one GPU', 'name': 'f3', 'leaves': n, 'leaf_bytes': ln},
        'verdict_mismatches': mism,
        'input_gbps': round(n * ln * args.steps / elapsed / 1e9, 2),
        'compact_extend': {'value': round((n - 1) / ext_s, 1), 'unit': 'leaves/s', 'ms': round(ext_s * 1e3, 3),
                           'path': 'GpuTreeHasher._hash_full over {} host leaves (list of bytes packed once; {} full subtrees, '
                                   'one pv_merkle_root call each incl. H2D), root checked against '
                                   'hashlib'.format(n - 1, bin(n - 1).count('1'))},
        'compact_append': {'value': round(n_app / app_s, 1), 'unit': 'appends/s', 'appends': n_app,
                           'ms': round(app_s * 1e3, 3),
                           'path': 'CompactMerkleTree.append call pattern (_hash_full of 1 leaf + hash_children per '
                                   'carry + _hash_fold) on GpuTreeHasher; root checked against hashlib'},
        'sha256_batch_small': {'rows': small, 'dispatch_items': 512,
                               'path': 'sha256_batch(host list of 256 B leaves, prefix 0x00): hashlib vs one GPU '
                                       'call incl. pack + H2D + D2H, mean of 5'},
        'roofline': _sha256_roofline(leaf_blocks, leaf_ms, _mad_peak(), step_blocks, elapsed / args.steps * 1e3),
        'cpu_baseline': {'value': round(cpu_rate, 1), 'unit': 'leaves/s', 'cores': 1, 'kind': 'port',
                         'sample': 'hashlib SHA-256 tree hash (the reference TreeHasher algorithm, level-wise) over '
                                   'the first {} leaves on 1 host thread'.format(sample)},
    }
    if TUNED:
        res['tuning'] = dict(TUNED)
    print(json.dumps(res), flush=True)
    return 0 if mism == 0 else 3


# the other configs' lines, measured by the default (driver) run itself as short
# child runs after the C2 line's timed region: (config, steps, warmup)
OTHER_CONFIGS = (('c3', 10, 2), ('c4', 5, 1), ('c3bls', 3, 1), ('c1', 5, 1), ('f3', 5, 1))


def other_configs():
    """Short runs of C3, C4, C3-BLS, C1 and f3 (each a fresh child process of
    this script with --no-cpu-baseline, started after the C2 measurement), so the
    driver's own run records them; the headline `value` stays C2's.  -> {config:
    the child's line, trimmed to its measurement} or {config: {'error': ...}}."""
    import subprocess
    res = {}
    keep = ('metric', 'value', 'unit', 'steps', 'warmup', 'ms_per_step', 'verdict_mismatches', 'batches_per_s',
            'quorum_reached', 'kernel_ms', 'small_batch_latency')
    for name, steps, warm in OTHER_CONFIGS:
        t0 = time.perf_counter()
        try:
            p = subprocess.run([sys.executable, os.path.abspath(__file__), '--config', name, '--steps', str(steps),
                                '--warmup', str(warm), '--no-cpu-baseline', '--no-e2e'],
                               capture_output=True, text=True, timeout=300, cwd=REPO)
            line = json.loads(p.stdout.strip().splitlines()[-1]) if p.returncode in (0, 3) and p.stdout.strip() else None
        except (subprocess.TimeoutExpired, ValueError, IndexError) as e:
            res[name] = {'error': repr(e)[:200]}
            continue
        if line is None:
            res[name] = {'error': 'rc {}: {}'.format(p.returncode, p.stderr[-300:])}
            continue
        r = {k: line[k] for k in keep if k in line}
        r['workload'] = (line.get('config') or {}).get('workload')
        rf = line.get('roofline') or {}
        if rf:
            r['roofline'] = {k: rf.get(k) for k in ('kernel', 'achieved', 'peak', 'unit', 'frac', 'traffic', 'key_prep',
                                                    'hash', 'stages')
                             if k not in ('key_prep', 'hash', 'stages') or rf.get(k)}
            if r['roofline'].get('hash'):
                r['roofline']['hash'] = {k: r['roofline']['hash'][k] for k in ('ms', 'blocks', 'achieved', 'peak',
                                                                                'frac')}
        r['child_wall_s'] = round(time.perf_counter() - t0, 2)
        res[name] = r
    return res


def _free_port():
    import socket
    with socket.socket() as so:
        so.bind(('127.0.0.1', 0))
        return so.getsockname()[1]


def _visible_gpus():
    """GPUs this process may use, counted without initialising HIP
    (torch.cuda.device_count() does not create a context on this image)."""
    try:
        return torch.cuda.device_count()
    except Exception:   # noqa: BLE001 - no runtime: no GPUs
        return 0


def rank_plan(gpus, environ=None, visible=None):
    """How `bench.py --gpus N` runs, decided before any GPU call:
    -> ('error', message) | ('launch', N) (start N rank children) |
       ('run', world) (this process is a rank, or the only one).
    `gpus` None = the launcher's WORLD_SIZE (or 1)."""
    environ = os.environ if environ is None else environ
    share = environ.get('PV_BENCH_SHARE_GPU') == '1'
    ws = environ.get('WORLD_SIZE')
    if ws is not None:
        try:
            world = int(ws)
        except ValueError:
            return 'error', 'WORLD_SIZE={!r} is not an integer'.format(ws)
        if gpus is not None and gpus != world:
            return 'error', ('--gpus {} but WORLD_SIZE={} (the launcher started {} ranks): run it with '
                             '--gpus {}'.format(gpus, world, world, world))
        n = world
    else:
        n = 1 if gpus is None else gpus
    if n < 1:
        return 'error', '--gpus must be >= 1 (got {})'.format(n)
    if n > 1 and not share:
        vis = _visible_gpus() if visible is None else visible
        if n > vis:
            return 'error', ('--gpus {} but only {} GPU(s) are visible (PV_BENCH_SHARE_GPU=1 runs every rank on '
                             'GPU 0 for a rehearsal)'.format(n, vis))
    if ws is None and n > 1:
        return 'launch', n
    return 'run', n


def launch_ranks(n, argv):
    """Start ranks 0..n-1 as fresh child processes of this script (same argv,
    --gpus n), each with the torch.distributed env of one rank on GPU `rank`.
    stdout / stderr are inherited: rank 0 alone prints the JSON line.  When a
    rank fails, the others get SIGTERM (exact PIDs) after a grace period, so a
    peer stuck in a collective cannot outlive the job.  -> exit status."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK='0', MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port),
                   HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get('HSA_ENABLE_IPC_MODE_LEGACY', '0'),
                   PV_BENCH_LAUNCHER='self')
        procs.append(subprocess.Popen([sys.executable, '-u', os.path.abspath(__file__)] + argv, env=env, cwd=REPO))
    rcs = [None] * n
    failed_at = None
    while any(rc is None for rc in rcs):
        for r, p in enumerate(procs):
            if rcs[r] is None:
                rcs[r] = p.poll()
                if rcs[r] not in (None, 0, 3) and failed_at is None:
                    failed_at = time.monotonic()
                    print('bench.py: rank {} exited with {}'.format(r, rcs[r]), file=sys.stderr, flush=True)
        if failed_at is not None and time.monotonic() - failed_at > 30:
            for r, p in enumerate(procs):
                if rcs[r] is None:
                    p.terminate()
            for r, p in enumerate(procs):
                if rcs[r] is None:
                    try:
                        rcs[r] = p.wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        p.kill()
                        rcs[r] = p.wait()
        time.sleep(0.05)
    bad = [rc for rc in rcs if rc not in (0, 3)]
    if bad:
        return bad[0] if bad[0] > 0 else 1
    return 3 if 3 in rcs else 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=None,
                    help='GPUs (ranks); default: WORLD_SIZE under a launcher, else 1.  N > 1 without a launcher '
                         'starts the N ranks itself')
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--config', choices=sorted(CONFIGS) + ['f3', 'c3bls'], default='c2',
                    help='workload (default c2, the headline; f3 = ledger Merkle hashing)')
    ap.add_argument('--n', '--count', dest='n', type=int, default=None,
                    help='signatures per GPU (default: the config\'s); spell it --count under torch.distributed.run')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-e2e', action='store_true', help='skip the host-buffer (PCIe-inclusive) measurement')
    ap.add_argument('--key-mod', type=int, default=None,
                    help='experiment: override the config key pool size (keys = i mod N; the line records it)')
    ap.add_argument('--key-format', choices=('auto', 'narrow', 'wide'), default='auto',
                    help='prepared-key format: auto = wide (radix-256 comb) for node keys (c3), narrow for key pools')
    ap.add_argument('--no-key-cache', action='store_true',
                    help='c3/c4: re-decompress every key per signature instead of preparing each distinct key once')
    ap.add_argument('--keys-serial', action='store_true',
                    help='c3/c4 pipelined: prepare the keys before the hash stage on the step\'s stream (default: on '
                         'the slot\'s side stream, beside the hash stage; pv_verify_keys_device_async)')
    ap.add_argument('--collective', action='store_true',
                    help='create the process group and run the verdict / quorum all-gathers even at one rank '
                         '(RCCL exercised on a one-GPU box; the gathered bytes are checked like at N > 1)')
    ap.add_argument('--no-other-configs', action='store_true',
                    help='c2 at N = 1: skip the short runs of the other configs (C3, C4, C3-BLS, C1, f3) whose '
                         'lines the default run reports under "other_configs"')
    ap.add_argument('--sequential', action='store_true',
                    help='one stream, each step after the previous one (default: consecutive steps alternate over '
                         'two streams and two workspaces, so step k + 1 starts while step k\'s curve grid drains)')
    args = ap.parse_args()
    # --gpus N means N ranks: decided before this process touches the GPU (a
    # self-launch starts fresh children; no exec from a process with a context)
    action, nranks = rank_plan(args.gpus)
    if action == 'error':
        print('bench.py: ' + nranks, file=sys.stderr, flush=True)
        return 2
    if action == 'launch':
        argv = sys.argv[1:]
        if args.gpus is None:
            argv += ['--gpus', str(nranks)]
        return launch_ranks(nranks, argv)
    if nranks > 1 and args.config in ('c1', 'c3bls', 'f3'):
        print('bench.py: --config {} is a one-GPU line (no sharded path); run it with --gpus 1'.format(args.config),
              file=sys.stderr, flush=True)
        return 2
    # PV_* schedule knobs (A/B runs of tools/*.sh): an explicit opt-in here --
    # the library never reads the environment; a non-default setting is
    # reported in the line
    TUNED.update(nat.tuning_from_env())
    if args.config == 'c1':
        return main_c1(args)
    if args.config == 'c3bls':
        return main_bls(args)
    if args.config == 'f3':
        return main_f3(args)

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    # production: one rank per GPU over RCCL ("nccl").  Rehearsal of the N > 1
    # path on a one-GPU box: PV_BENCH_BACKEND=gloo PV_BENCH_SHARE_GPU=1 puts every
    # rank on GPU 0 and runs the same collectives through host copies.
    backend = os.environ.get('PV_BENCH_BACKEND', 'nccl')
    if os.environ.get('PV_BENCH_SHARE_GPU') == '1':
        local = 0
    # the collectives run when there is more than one rank, or at one rank when
    # asked (--collective: RCCL initialised and used on a one-GPU lease)
    coll = world > 1 or args.collective
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    if coll:
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=dev)
        else:
            dist.init_process_group(backend)

    def coll_dev(t):
        return t if backend == 'nccl' else t.cpu()

    def all_gather(out, inp):
        if backend == 'nccl':
            dist.all_gather_into_tensor(out, inp)
        else:
            o = out.cpu()
            dist.all_gather_into_tensor(o, inp.cpu())
            out.copy_(o)

    cfg = dict(CONFIGS[args.config])
    if args.key_mod is not None:
        cfg['key_mod'] = args.key_mod
    n = args.n or cfg['n']
    n_nodes = cfg.get('n_nodes', 25)
    if cfg['mode'] == synth.COMMIT:
        n -= n % n_nodes
    batch = SyntheticBatch(local, n, cfg['mlen'], cfg=cfg['cfg'], first=rank * n, key_mod=cfg['key_mod'],
                           mode=cfg['mode'], mlen_max=cfg['mlen_max'], n_nodes=n_nodes)
    # keys repeat in c3 (node keys: the wide comb) and c4 (key pool: the narrow one)
    wide = args.key_format == 'wide' or (args.key_format == 'auto' and cfg['mode'] == synth.COMMIT)
    key_cache = batch.use_key_cache(not args.no_key_cache, wide=wide)
    batch.make_slots()
    torch.cuda.synchronize()
    pipelined = not args.sequential
    # pipelined steps: step k runs on stream k % 2 with verify workspace and
    # outputs k % 2 (pv_*_async), so step k + 1's hash and curve grids start on
    # CUs that step k's curve grid has finished with; a slot is reused two
    # steps later on the same stream (ordered)
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)] if pipelined else None
    slots = 2 if pipelined else 1
    gathered = [torch.zeros(world * batch.bitmap.numel(), dtype=torch.int64, device=dev)
                for _ in range(slots)] if coll else None
    tally = None
    if cfg['mode'] == synth.COMMIT:
        nb = n // n_nodes
        q = Quorums(n_nodes).commit.value
        tally = dict(nb=nb, q=q, boff=torch.arange(nb + 1, dtype=torch.int64, device=dev) * n_nodes,
                     votes=[torch.empty(nb, dtype=torch.int32, device=dev) for _ in range(slots)],
                     reached=[torch.empty(nb, dtype=torch.uint8, device=dev) for _ in range(slots)],
                     gathered=[torch.empty(world * nb, dtype=torch.uint8, device=dev) for _ in range(slots)],
                     bad=torch.zeros(1, dtype=torch.int32, device=dev))

    def finish(slot, verdict, bitmap):
        if tally is not None:
            # enqueue-only tally: the sender range flag is read once after the
            # timed region, so no step waits on the host (steps stay pipelined)
            tally_device_async(verdict, batch.sender, tally['boff'], n_nodes, tally['q'], tally['votes'][slot],
                               tally['reached'][slot], tally['bad'], streams[slot] if pipelined else None)
        if coll:
            all_gather(gathered[slot], bitmap)
            if tally is not None:   # C3: batch-sharded tallies, gather the quorum bits
                all_gather(tally['gathered'][slot], tally['reached'][slot])

    counter = [0]

    def step():
        if not pipelined:
            batch.verify()
            finish(0, batch.verdict, batch.bitmap)
            return
        slot = counter[0] & 1
        counter[0] += 1
        with torch.cuda.stream(streams[slot]):
            verdict, bitmap = batch.verify_async(slot, streams[slot], keys_beside=not args.keys_serial)
            finish(slot, verdict, bitmap)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    calib = 0
    if pipelined:
        # the kernels' own durations: a few steps one after the other with HIP
        # events on the launch stream, right before the timed region (pipelined
        # launches overlap, so their intervals hold the other stream's work)
        calib = 5
        nat.kernel_timing(local, True)
        tc0 = time.perf_counter()
        for _ in range(calib):
            batch.verify()
        torch.cuda.synchronize()
        calib_wall = (time.perf_counter() - tc0) / calib
        calib_sums = nat.kernel_timing(local, False)
        calib_sha = nat.kernel_timing_sha(local)
    if coll:
        dist.barrier()
    torch.cuda.synchronize()
    # HIP events around each verify launch of the timed steps (sequential
    # schedule); pipelined launches overlap, so their kernels are timed on
    # the sequential calibration steps before the timed region instead
    nat.kernel_timing(local, not pipelined)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if coll:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if coll:
        t = coll_dev(torch.tensor([elapsed], dtype=torch.float64, device=dev))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # correctness of the measured passes (every output slot): verdict == not
    # tampered, bitmap == verdict, quorum bits == the spec's
    tamper = batch.tamper.cpu().numpy().astype(bool)
    mism = 0
    used = min(slots, args.steps + args.warmup)
    if tally is not None:
        mism += int(tally['bad'].item() != 0)   # a sender index out of range in any step
    for slot in range(used):
        v_t, b_t, _ = batch.slot_out[slot]
        verdict = v_t.cpu().numpy().astype(bool)
        mism += int((verdict == tamper).sum())
        bits = np.unpackbits(b_t.cpu().numpy().view(np.uint8), bitorder='little')[:n].astype(bool)
        mism += int((bits != verdict).sum())
        if tally is not None:
            want_votes, want_reached = synth.c3_expected(rank * tally['nb'], tally['nb'], n_nodes, tally['q'])
            mism += int((tally['votes'][slot].cpu().numpy() != want_votes.astype(np.int32)).sum())
            mism += int((tally['reached'][slot].cpu().numpy().astype(bool) != want_reached).sum())
            if coll:
                _, all_reached = synth.c3_expected(0, world * tally['nb'], n_nodes, tally['q'])
                mism += int((tally['gathered'][slot].cpu().numpy().astype(bool) != all_reached).sum())
        if coll:
            # own slice of the gathered bitmaps == own verdicts, and every rank holds
            # the same gathered bytes (checksums equal under MIN and MAX)
            g = gathered[slot].cpu().numpy()
            allbits = np.unpackbits(g.view(np.uint8), bitorder='little')
            per = batch.bitmap.numel() * 64
            mine = allbits[rank * per: rank * per + n].astype(bool)
            mism += int((mine != verdict).sum())
            import hashlib
            ck = int.from_bytes(hashlib.sha256(g.tobytes()).digest()[:7], 'little')
            cks = [coll_dev(torch.tensor([ck], dtype=torch.int64, device=dev)) for _ in range(2)]
            dist.all_reduce(cks[0], op=dist.ReduceOp.MIN)
            dist.all_reduce(cks[1], op=dist.ReduceOp.MAX)
            mism += int(cks[0].item() != cks[1].item())
    ranks = None
    if coll:
        m = coll_dev(torch.tensor([mism], dtype=torch.int64, device=dev))
        dist.all_reduce(m)
        mism = int(m.item())
        # which GPU every rank ran on (HIP ordinal + PCI bus id), gathered
        props = torch.cuda.get_device_properties(dev)
        mine = torch.tensor([rank, dev.index, int(getattr(props, 'pci_bus_id', -1) or -1)], dtype=torch.int64,
                            device=dev)
        allr = torch.zeros(world * 3, dtype=torch.int64, device=dev)
        all_gather(allr, mine)
        ranks = {'world_size': dist.get_world_size(), 'backend': dist.get_backend(),
                 'launcher': os.environ.get('PV_BENCH_LAUNCHER', 'external (torch.distributed.run)'),
                 'devices': [{'rank': int(a), 'device': int(b), 'pci_bus_id': int(c)}
                             for a, b, c in allr.view(world, 3).cpu().tolist()]}
        if ranks['world_size'] != world:
            mism += 1

    # kernel-level timing for the roofline: HIP events on the launch stream,
    # recorded during the timed steps above (averaged over those launches)
    h_sum, c_sum, launches = nat.kernel_timing(local, False)
    sha_sum = nat.kernel_timing_sha(local)
    seq_ms_step = elapsed / args.steps * 1e3
    if pipelined:
        h_sum, c_sum, launches = calib_sums
        sha_sum = calib_sha
        seq_ms_step = calib_wall * 1e3
    ms_sha = sha_sum / max(1, launches)
    ms_hash, ms_curve = h_sum / max(1, launches), c_sum / max(1, launches)
    kernel_ms_on = ('{} sequential calibration steps right before the timed region (pipelined launches overlap)'
                    .format(calib) if pipelined else 'the timed steps')
    curve_mode, deferred = nat.curve_stats(local)
    if key_cache and batch.wide:
        kernel, work = 'k_curve<keyed, wide>', W_MAD_KEYED_WIDE * n
        wpv = {'fe_mul': W_MUL_KEYED_WIDE, 'fe_sq': W_SQ_KEYED_WIDE, 'mad': W_MAD_KEYED_WIDE,
               'per_distinct_key': {'fe_mul': W_MUL_KEYPREP_WIDE, 'fe_sq': W_SQ_KEYPREP_WIDE}}
    elif key_cache:
        kernel, work = 'k_curve<keyed>', W_MAD_KEYED * n
        wpv = {'fe_mul': W_MUL_KEYED, 'fe_sq': W_SQ_KEYED, 'mad': W_MAD_KEYED,
               'per_distinct_key': {'fe_mul': W_MUL_KEYPREP, 'fe_sq': W_SQ_KEYPREP}}
    elif curve_mode == 'grouped':
        kernel, work = 'k_curve', W_MAD_GROUPED * n
        wpv = {'fe_mul': W_MUL_GROUPED, 'fe_sq': W_SQ_GROUPED, 'mad': W_MAD_GROUPED}
    else:
        kernel, work = 'k_curve_half', W_MAD_PER_VERIFY * (n - deferred) + W_MAD_FULL * deferred
        wpv = {'fe_mul': W_MUL_PER_VERIFY, 'fe_sq': W_SQ_PER_VERIFY, 'mad': W_MAD_PER_VERIFY,
               'deferred_full_length': {'count': deferred, 'fe_mul': W_MUL_FULL, 'fe_sq': W_SQ_FULL,
                                        'mad': W_MAD_FULL}}
    ms_step = elapsed / args.steps * 1e3
    # HBM bytes of the dominant launch, from the committed PMC profile of the same
    # line shape (the curve kernel the profile measured)
    traffic = None
    if args.config == 'c2' and not key_cache and curve_mode == 'half':
        traffic = _traffic_per_launch('c2', n)
    elif args.config == 'c3' and key_cache and batch.wide:
        traffic = _traffic_per_launch('c3', n)
    elif args.config == 'c4' and key_cache and not batch.wide:
        traffic = _traffic_per_launch('c4', n)
    # the dominant kernel is priced on its own HIP-event duration: in the timed
    # steps when they run one after the other; when they are pipelined the
    # launches overlap (a launch's interval includes the other stream's tail),
    # so on the sequential calibration steps right before the timed region.
    # per_step: the same work over the pipelined per-step time, every kernel of
    # the step charged to the curve (a lower bound on its rate).
    achieved = work / (ms_curve * 1e-3)
    achieved_step = work / (ms_step * 1e-3)
    peak = _mad_peak()
    key_prep = None
    if key_cache:
        key_prep = _key_prep_roofline(batch, args.config, peak)
    hash_rf = _hash_roofline(hash_compressions(batch.off), ms_sha, peak)
    # the stages of one sequential step: their HIP-event
    # durations against the wall time of the sequential steps they were timed on
    stage_sum = (key_prep['ms'] if key_prep else 0.0) + ms_hash + ms_curve
    stages = {'key_prep_ms': key_prep['ms'] if key_prep else None, 'sha_ms': round(ms_sha, 4),
              'lattice_ms': round(ms_hash - ms_sha, 4) if not key_cache else None,
              'hash_interval_ms': round(ms_hash, 4), 'curve_ms': round(ms_curve, 4),
              'sum_ms': round(stage_sum, 4), 'sequential_ms_per_step': round(seq_ms_step, 4),
              'sum_over_sequential': round(stage_sum / seq_ms_step, 4) if seq_ms_step else None,
              'note': 'HIP-event durations of the priced stages (k_keys after the timed region; hash interval = '
                      'memset + pre-checks + k_hash (+ k_lattice on generic batches); curve) vs the wall time per '
                      'step of the {}'.format('5 sequential calibration steps' if pipelined else 'sequential timed steps')}

    total = world * n * args.steps
    value = total / elapsed
    out = {
        'metric': METRIC, 'value': round(value, 1), 'unit': 'verifies/s', 'n_gpus': world,
        'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(elapsed / args.steps * 1e3, 3),
        'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': 'u32',
        'data': 'synthetic (device-generated, deterministic: plenum_gpu/synth.py)',
        'config': {'workload': cfg['workload'], 'name': args.config,
                   'signatures_per_gpu': n, 'msg_bytes': [cfg['mlen'], cfg['mlen_max']] if cfg['mlen'] != cfg['mlen_max']
                   else cfg['mlen'], 'mean_msg_bytes': round(batch.blob_bytes / max(1, n), 1),
                   'key_pool': cfg['key_mod'] or ('node keys' if cfg['mode'] == synth.COMMIT else 'distinct'),
                   'key_cache': 'prepared once per step per distinct key (inside the timed step), {} format'.format(
                       'wide (radix-256 comb)' if batch.wide else 'narrow (radix-16 comb)') if key_cache else 'off', 'tampered': int(tamper.sum()),
                   'parallelism': 'dp{} (disjoint index shards) + {} all-gather of verdict bitmaps'.format(
                       world, 'RCCL' if backend == 'nccl' else backend + ' (rehearsal, ranks share GPU 0)')
                   if coll else 'single GPU'},
        'verdict_mismatches': mism,
        'kernel_ms': {'hash': round(ms_hash, 4), 'curve': round(ms_curve, 4), 'timed_on': kernel_ms_on},
        'roofline': {'bound': 'valu', 'kernel': kernel,
                     'achieved': round(achieved / 1e12, 3), 'peak': round(peak / 1e12, 3),
                     'unit': 'Tmad/s (v_mad_u64_u32 lane-ops)', 'frac': round(achieved / peak, 4),
                     'timing': 'curve MAD work per launch / HIP-event duration of the curve launch ({})'.format(
                         kernel_ms_on),
                     'per_step': {'ms': round(ms_step, 4), 'achieved': round(achieved_step / 1e12, 3),
                                  'frac': round(achieved_step / peak, 4),
                                  'note': 'curve MAD work per step / per-step time of the timed region (every kernel '
                                          'of the step charged to the curve)'},
                     'traffic': traffic,
                     'key_prep': key_prep,
                     'hash': hash_rf,
                     'stages': stages,
                     'work_per_verify': wpv,
                     'combined_issue': _combined_issue(n / (ms_curve * 1e-3), peak)
                     if (args.config, n) == ('c2', CONFIGS['c2']['n']) and curve_mode == 'half' else None},
        'curve_mode': curve_mode if not key_cache else 'keyed',
        'schedule': 'pipelined: consecutive steps alternate over 2 streams + 2 verify workspaces/output sets '
                    '(step k + 1 starts while step k drains; all K steps complete inside the timed region)'
                    if pipelined else 'sequential: one stream',
        'cpu_baseline': None,
    }
    if key_cache and pipelined:
        out['key_schedule'] = ('serial: key preparation before the hash stage on the step\'s stream'
                               if args.keys_serial else
                               'pv_verify_keys_device_async: key preparation on the slot\'s side stream while the '
                               'hash stage runs when the key grid is under one wave per SIMD (C3\'s node keys), '
                               'else before it on the step\'s stream (C4\'s key pool)')
    if tally is not None:
        out['config']['batches_per_gpu'] = tally['nb']
        out['config']['quorum'] = tally['q']
        out['batches_per_s'] = round(world * tally['nb'] * args.steps / elapsed, 1)
        out['quorum_reached'] = int(tally['reached'][0].sum().item())
    if ranks is not None:
        out['ranks'] = ranks
    if coll:
        # every rank has finished its timed region and checks: rank 0 prices the
        # host baseline while the others wait at the closing barrier
        dist.barrier()
    if rank == 0 and not args.no_cpu_baseline:
        out['cpu_baseline'] = cpu_baseline(batch, args.config.upper())
    if world == 1 and args.config == 'c2' and not args.no_e2e:
        out['end_to_end'] = end_to_end(batch, key_cache)
        mism += out['end_to_end']['verdict_mismatches']
        out['small_batch_latency'] = small_batch_latency(batch)
        mism += out['small_batch_latency']['verdict_mismatches']
    if world == 1 and args.config == 'c2' and not args.n and not args.no_other_configs and not args.collective:
        out['other_configs'] = other_configs()
        mism += sum(int(r.get('verdict_mismatches') or 0) for r in out['other_configs'].values())
    if rank == 0:
        if TUNED:
            out['tuning'] = dict(TUNED)
        print(json.dumps(out), flush=True)
    if coll:
        dist.barrier()
        dist.destroy_process_group()
    return 0 if mism == 0 else 3


if __name__ == '__main__':
    sys.exit(main())
