"""Parity of the HIP verify path (through the C-ABI) with the libsodium-1.0.18
golden fixtures and the oracle; size-independent properties at full size."""
import os

import numpy as np
import pytest

import _oracle as orc
from conftest import split_sm

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def nat():
    from plenum_gpu import _native
    _native.ensure_init()
    return _native


def test_raw_vectors_bit_exact(nat, raw_vectors):
    r = raw_vectors
    got = nat.verify_batch_arrays(r['pk'], r['sig'], r['blob'], r['off'])
    assert (got == r['verdict'].astype(bool)).all()


def test_adversarial_bit_exact(nat, adversarial):
    from plenum_gpu.nacl_wrappers import verify_signed_batch
    rows = split_sm(adversarial)
    got = verify_signed_batch([(pk, sm) for _, pk, sm, _ in rows])
    wrong = [rows[k][0] for k in range(len(rows)) if got[k] != rows[k][3]]
    assert not wrong, wrong


def test_tally_fixture_verdicts(nat, tally_fx):
    t = tally_fx
    got = nat.verify_batch_arrays(t['pk'], t['sig'], t['blob'], t['off'])
    assert (got == t['verdict'].astype(bool)).all()


def test_empty_and_single(nat, raw_vectors):
    r = raw_vectors
    assert nat.verify_batch_arrays(np.zeros((0, 32), np.uint8), np.zeros((0, 64), np.uint8),
                                   np.zeros(0, np.uint8), np.zeros(1, np.uint64)).size == 0
    for i in (0, 1, 2):
        o = r['off']
        got = nat.verify_batch_arrays(r['pk'][i:i + 1], r['sig'][i:i + 1], r['blob'][int(o[i]):int(o[i + 1])],
                                      np.array([0, o[i + 1] - o[i]], np.uint64))
        assert got[0] == bool(r['verdict'][i])


@pytest.mark.parametrize('path', ['default', 'chunks'])
def test_random_ragged_vs_oracle(nat, path):
    """Ragged messages (0 B - 5 KB) with ~10 % corrupted, against the oracle:
    through the latency kernel (default size routing) and through the fused
    chunk path (latency path off: per-lane SHA-512 of ragged lengths inside
    k_chunk_half, deferred records in the list pass)."""
    if path == 'chunks':
        nat.set_lat_max(0)
    try:
        _random_ragged_vs_oracle(nat)
    finally:
        nat.set_lat_max(nat.LAT_MAX_DEFAULT)


def _random_ragged_vs_oracle(nat):
    rng = np.random.default_rng(2026)
    n = 6000
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    msgs = [rng.integers(0, 256, int(rng.choice([0, 1, 47, 48, 175, 176, int(rng.integers(0, 5000))])),
                         dtype=np.uint8).tobytes() for _ in range(n)]
    blob, off = nat.pack_messages(msgs)
    pk, sig = nat.sign_batch_arrays(seeds, blob, off)
    # corrupt ~10 %: random bit anywhere in R, S or M
    for i in rng.choice(n, n // 10, replace=False):
        which = rng.integers(0, 3)
        if which == 0 or len(msgs[i]) == 0:
            sig[i, rng.integers(0, 64)] ^= 1 << int(rng.integers(0, 8))
        else:
            m = bytearray(msgs[i])
            m[rng.integers(0, len(m))] ^= 1 << int(rng.integers(0, 8))
            msgs[i] = bytes(m)
    blob, off = nat.pack_messages(msgs)
    got = nat.verify_batch_arrays(pk, sig, blob, off)
    want = orc.verify_batch(pk, sig, blob, off)
    assert (got == want).all()
    assert 0.05 < (~got).mean() < 0.15


def test_batch_larger_than_persistent_grid(nat):
    """More signatures than resident curve lanes: grid-stride loop and bitmap words."""
    from plenum_gpu import synth
    n = 300_000
    rng = np.random.default_rng(3)
    seeds = np.repeat(rng.integers(0, 256, (1000, 32), dtype=np.uint8), n // 1000, axis=0)
    blob = rng.integers(0, 256, n * 64, dtype=np.uint8)
    off = np.arange(n + 1, dtype=np.uint64) * 64
    pk, sig = nat.sign_batch_arrays(seeds, blob, off)
    bad = rng.choice(n, 5000, replace=False)
    sig[bad, 40] ^= 4
    got = nat.verify_batch_arrays(pk, sig, blob, off)
    want = np.ones(n, bool)
    want[bad] = False
    assert (got == want).all()


def test_invalid_arguments_raise(nat):
    with pytest.raises(ValueError):
        nat.verify_batch_arrays(np.zeros((2, 32), np.uint8), np.zeros((1, 64), np.uint8), np.zeros(0, np.uint8),
                                np.zeros(3, np.uint64))
    with pytest.raises(nat.PlenumGpuError):
        nat.verify_batch_arrays(np.zeros((2, 32), np.uint8), np.zeros((2, 64), np.uint8), np.zeros(10, np.uint8),
                                np.array([0, 8, 4], np.uint64))


def test_multi_device_mask_shards(nat, raw_vectors):
    """device_mask = every initialised device (one box: 1 GPU) gives the same verdicts."""
    r = raw_vectors
    got = nat.verify_batch_arrays(r['pk'], r['sig'], r['blob'], r['off'], device_mask=0)
    assert (got == r['verdict'].astype(bool)).all()


def test_sign_matches_oracle_and_fixture(nat, raw_vectors):
    import hashlib
    import struct
    r = raw_vectors
    idx = [i for i in range(len(r['verdict'])) if not r['tampered'][i]][:1500]
    seeds = np.stack([np.frombuffer(hashlib.sha512(b'plenum-gpu/rawkey' + struct.pack('<Q', i % 2500)).digest()[:32],
                                    np.uint8) for i in idx])
    msgs = [r['blob'][int(r['off'][i]):int(r['off'][i + 1])].tobytes() for i in idx]
    blob, off = nat.pack_messages(msgs)
    pk, sig = nat.sign_batch_arrays(seeds, blob, off)
    assert (pk == r['pk'][idx]).all() and (sig == r['sig'][idx]).all()


def _adv_soa(adversarial, reps=1):
    rows = [(pk, sm, v) for _, pk, sm, v in split_sm(adversarial) if len(sm) >= 64] * reps
    pk = np.frombuffer(b''.join(r[0] for r in rows), np.uint8).reshape(-1, 32)
    sig = np.frombuffer(b''.join(r[1][:64] for r in rows), np.uint8).reshape(-1, 64)
    blob, off = orc_pack([r[1][64:] for r in rows])
    return pk, sig, blob, off, np.array([r[2] for r in rows])


def orc_pack(msgs):
    off = np.zeros(len(msgs) + 1, np.uint64)
    off[1:] = np.cumsum([len(m) for m in msgs])
    return np.frombuffer(b''.join(msgs), np.uint8), off


@pytest.mark.parametrize('dedup', [False, True])
def test_adversarial_prepared_keys(nat, adversarial, dedup):
    """Every adversarial row three times: with PV_FLAG_DEDUP_KEYS each
    distinct key (small order, non-canonical, off-curve, mixed order ...) is
    prepared once on the device; verdicts equal the fixture either way."""
    pk, sig, blob, off, want = _adv_soa(adversarial, reps=3)
    got = nat.verify_batch_arrays(pk, sig, blob, off, dedup_keys=dedup)
    assert (got == want).all()


def test_keyed_device_path_c3_and_c4(nat):
    """Device key cache (pv_keys_prepare_device + pv_verify_keyed_device) on
    COMMIT votes (25 node keys) and on a 4096-key pool with ragged payloads:
    identical verdicts to the unkeyed path, == not tampered."""
    from plenum_gpu import synth
    from plenum_gpu.device import SyntheticBatch
    for b in (SyntheticBatch(0, 25 * 4000, 0, cfg=3, first=25 * 77, mode=synth.COMMIT, n_nodes=25),
              SyntheticBatch(0, 60000, 128, cfg=4, first=12345, key_mod=4096, mode=synth.RANGE, mlen_max=4096)):
        v0 = b.verify().cpu().numpy().copy()
        assert b.use_key_cache()
        v1 = b.verify().cpu().numpy()
        assert (v0 == v1).all()
        assert (v1.astype(bool) == ~b.tamper.cpu().numpy().astype(bool)).all()
        bits = np.unpackbits(b.bitmap.cpu().numpy().view(np.uint8), bitorder='little')[:b.n]
        assert (bits == v1).all()
        th, tc = b.time_kernels(1)
        assert th > 0 and tc > 0


@pytest.mark.parametrize('shape', ['c2', 'c4_keyed'])
def test_host_pipeline_multi_chunk(nat, shape):
    """pv_verify_batch runs a shard as a pipeline of chunks (H2D of chunk c+1 on
    the copy stream overlaps the kernels of chunk c, chunks alternate over two
    compute streams and workspaces; >= 32768 signatures per chunk): a 200k
    batch spans 1-6 chunks.  Verdicts == not tampered; the keyed case
    (4096-key pool, ragged 128 B - 4 KB payloads) indexes the chunk's key
    indices and shard-relative message offsets, with the key table built on
    stream 0 and consumed on both."""
    from plenum_gpu import synth
    from plenum_gpu.device import SyntheticBatch
    if shape == 'c2':
        b = SyntheticBatch(0, 200000, 256, cfg=2, first=4242)
    else:
        b = SyntheticBatch(0, 200000, 128, cfg=4, first=999, key_mod=4096, mode=synth.RANGE, mlen_max=4096)
    pk, sig = b.pk.cpu().numpy(), b.sig.cpu().numpy()
    off = b.off.cpu().numpy().astype(np.uint64)
    blob = b.blob.cpu().numpy()[:int(off[-1])]
    want = ~b.tamper.cpu().numpy().astype(bool)
    # pinned staging ring with threaded and single-thread gathers (4 chunks:
    # a 32768 ramp chunk + 4 x ~41808 signatures; 16 chunks: 6 x ~33333, so
    # chunks 2.. wait for their slot's previous DMA and reuse a workspace; the
    # tail case below: 4 x ~32769), one chunk, and the runtime's pageable
    # staging
    try:
        for staging, threads, chunks in (('pinned', 8, 4), ('pinned', 1, 1), ('pageable', 0, 4), ('pinned', 8, 16)):
            nat.set_host_staging(staging, threads, chunks)
            for dedup in (False, True):
                got = nat.verify_batch_arrays(pk, sig, blob, off, dedup_keys=dedup)
                assert (got == want).all(), (shape, staging, threads, dedup, int((got != want).sum()))
            # two full chunks and a 3-signature tail chunk
            got = nat.verify_batch_arrays(pk[:131075], sig[:131075], blob[:int(off[131075])], off[:131076])
            assert (got == want[:131075]).all(), (shape, staging, threads)
    finally:
        nat.set_host_staging('pinned', 8, 8)


def test_host_fused_chunks_and_deferred_pass(nat, raw_vectors, adversarial):
    """Host-buffer chunks run one fused launch each (k_chunk_half: hash +
    lattice + half-size curve per task) and the deferred records one
    lane-quad pass over a device-side index list: same verdicts as the
    per-chunk hash / lattice / curve schedule on a 200k C2 batch (~400
    deferred, several chunks); with curve_mode PV_CURVE_FULL every record is listed,
    so the list pass loops over 200k entries with its fixed grid; the
    fixtures (mixed-order, non-canonical, small-order cases) through the
    chunk path (latency path off) match libsodium in both modes."""
    from plenum_gpu.device import SyntheticBatch
    from plenum_gpu.nacl_wrappers import verify_signed_batch
    from conftest import split_sm
    b = SyntheticBatch(0, 200000, 256, cfg=2, first=5151)
    off = b.off.cpu().numpy().astype(np.uint64)
    pk, sig, blob = b.pk.cpu().numpy(), b.sig.cpu().numpy(), b.blob.cpu().numpy()[:int(off[-1])]
    want = ~b.tamper.cpu().numpy().astype(bool)
    rows = split_sm(adversarial)
    r = raw_vectors
    try:
        nat.set_host_staging('pinned', 8, 8)
        for fused in (True, False):
            nat.set_host_fused(fused)
            got = nat.verify_batch_arrays(pk, sig, blob, off, dedup_keys=False)
            assert (got == want).all(), (fused, int((got != want).sum()))
        nat.set_host_fused(True)
        nat.set_lat_max(0)
        for mode in ('half', 'full'):
            nat.set_curve_mode(mode)
            got = nat.verify_batch_arrays(pk, sig, blob, off, dedup_keys=False)
            assert (got == want).all(), (mode, int((got != want).sum()))
            got = nat.verify_batch_arrays(r['pk'], r['sig'], r['blob'], r['off'])
            assert (got == r['verdict'].astype(bool)).all(), mode
            got = verify_signed_batch([(p, sm) for _, p, sm, _ in rows])
            wrong = [rows[k][0] for k in range(len(rows)) if got[k] != rows[k][3]]
            assert not wrong, (mode, wrong)
    finally:
        nat.set_host_fused(True)
        nat.set_curve_mode('half')
        nat.set_lat_max(nat.LAT_MAX_DEFAULT)


def test_host_page_locked_inputs_direct(nat):
    """Caller buffers that are already page-locked (torch pin_memory()) are DMA'd
    directly (no gather copy): verdicts of a multi-chunk shard == not tampered,
    and a decreasing offset is still refused before any kernel reads it."""
    import torch
    from plenum_gpu.device import SyntheticBatch
    b = SyntheticBatch(0, 131075, 256, cfg=2, first=4242)
    off = b.off.cpu().numpy().astype(np.uint64)
    t = [b.pk.cpu().pin_memory(), b.sig.cpu().pin_memory(), b.blob.cpu()[:int(off[-1])].pin_memory(),
         torch.from_numpy(off.view(np.int64)).pin_memory()]
    pk, sig, blob, loff = t[0].numpy(), t[1].numpy(), t[2].numpy(), t[3].numpy().view(np.uint64)
    want = ~b.tamper.cpu().numpy().astype(bool)
    nat.set_host_staging('pinned', 8, 8)
    got = nat.verify_batch_arrays(pk, sig, blob, loff, dedup_keys=False)
    assert (got == want).all(), int((got != want).sum())
    bad = loff.copy()
    bad[90001] = bad[90000] - 1
    with pytest.raises(nat.PlenumGpuError, match='monotone'):
        nat.verify_batch_arrays(pk, sig, blob, bad, dedup_keys=False)


def test_host_offsets_checked_before_launch(nat):
    """msg_off is validated chunk by chunk while it is gathered: a decreasing
    offset in the middle of a multi-chunk shard is PV_EINVAL (no kernel reads
    it), and the next call on the same device is unaffected."""
    from plenum_gpu.device import SyntheticBatch
    b = SyntheticBatch(0, 100000, 64, cfg=2, first=777)
    pk, sig = b.pk.cpu().numpy(), b.sig.cpu().numpy()
    off = b.off.cpu().numpy().astype(np.uint64)
    blob = b.blob.cpu().numpy()[:int(off[-1])]
    want = ~b.tamper.cpu().numpy().astype(bool)
    bad = off.copy()
    bad[70001] = bad[70000] - 1
    for staging in ('pinned', 'pageable'):
        nat.set_host_staging(staging, 8, 8)
        with pytest.raises(nat.PlenumGpuError, match='monotone'):
            nat.verify_batch_arrays(pk, sig, blob, bad, dedup_keys=False)
        assert (nat.verify_batch_arrays(pk, sig, blob, off, dedup_keys=False) == want).all()
    nat.set_host_staging('pinned', 8, 8)
    # a Looper-pass-sized call (one gather, one DMA, one launch: run_small)
    small = off[:501].copy()
    small[300] = small[299] - 1
    with pytest.raises(nat.PlenumGpuError, match='monotone'):
        nat.verify_batch_arrays(pk[:500], sig[:500], blob[:int(off[500])], small)
    assert (nat.verify_batch_arrays(pk[:500], sig[:500], blob[:int(off[500])], off[:501]) == want[:500]).all()


def test_host_staging_slot_cap(nat):
    """A shard whose smallest chunk (65536 signatures) exceeds one 512 MiB
    pinned slot runs with pageable staging: 70k x 8 KiB messages (573 MB) in
    one chunk.  Verdicts == not tampered."""
    from plenum_gpu.device import SyntheticBatch
    b = SyntheticBatch(0, 70000, 8192, cfg=2, first=555)
    pk, sig = b.pk.cpu().numpy(), b.sig.cpu().numpy()
    off = b.off.cpu().numpy().astype(np.uint64)
    blob = b.blob.cpu().numpy()[:int(off[-1])]
    want = ~b.tamper.cpu().numpy().astype(bool)
    got = nat.verify_batch_arrays(pk, sig, blob, off, dedup_keys=False)
    assert (got == want).all(), int((got != want).sum())


@pytest.mark.parametrize('key_mod', [4096, 0])
def test_host_dedup_sampled(nat, key_mod):
    """Shards of >= 262144 signatures decide PV_FLAG_DEDUP_KEYS from a key
    sample first (pooled keys: prepared-key path; distinct keys: full pass
    skipped).  Verdicts == not tampered either way, pinned staging."""
    from plenum_gpu import synth
    from plenum_gpu.device import SyntheticBatch
    if key_mod:
        b = SyntheticBatch(0, 300000, 128, cfg=4, first=777, key_mod=key_mod, mode=synth.RANGE, mlen_max=512)
    else:
        b = SyntheticBatch(0, 300000, 200, cfg=2, first=31337)
    pk, sig = b.pk.cpu().numpy(), b.sig.cpu().numpy()
    off = b.off.cpu().numpy().astype(np.uint64)
    blob = b.blob.cpu().numpy()[:int(off[-1])]
    want = ~b.tamper.cpu().numpy().astype(bool)
    for dedup in (True, False):
        got = nat.verify_batch_arrays(pk, sig, blob, off, dedup_keys=dedup)
        assert (got == want).all(), (key_mod, dedup, int((got != want).sum()))
