"""Keyed latency kernel (k_verify_quad_keyed) and the persistent device key
cache of host-buffer calls (pv_keycache_add): verdicts must equal the
libsodium-1.0.18 fixtures whatever mix of cached / uncached keys a call holds,
and the device keyed path of small batches must equal the synthetic spec and
the keyed throughput kernel (tuning.lat_keyed_max = 0)."""
import numpy as np
import pytest

from conftest import split_sm

pytestmark = pytest.mark.gpu


@pytest.fixture
def nat():
    from plenum_gpu import _native as nat
    nat.ensure_init()
    nat.keycache_clear()
    yield nat
    nat.keycache_clear()
    nat.set_lat_keyed_max(nat.LAT_KEYED_MAX_DEFAULT)


def _slice(r, start, n):
    o = r['off'][start:start + n + 1]
    return r['pk'][start:start + n], r['sig'][start:start + n], r['blob'][int(o[0]):int(o[-1])], o - o[0]


def test_cached_keys_raw_vectors(nat, raw_vectors):
    """Every raw-vector key cached: ragged Looper-pass sizes through the keyed
    latency kernel, then half the keys cached (each call mixes the keyed and
    the generic list kernel), then none; always the fixture's verdicts."""
    r = raw_vectors
    want = r['verdict'].astype(bool)
    sizes = ((0, 1), (5, 7), (11, 8), (100, 9), (200, 100), (1000, 1000), (17, 2048), (0, 3000))
    nat.keycache_add(r['pk'])
    assert nat.keycache_size() == len(np.unique(r['pk'], axis=0))
    for start, n in sizes:
        got = nat.verify_batch_arrays(*_slice(r, start, n))
        assert (got == want[start:start + n]).all(), ('all cached', start, n)
    nat.keycache_clear()
    nat.keycache_add(r['pk'][::2])
    for start, n in sizes:
        got = nat.verify_batch_arrays(*_slice(r, start, n))
        assert (got == want[start:start + n]).all(), ('half cached', start, n)
    nat.keycache_clear()
    assert nat.keycache_size() == 0
    got = nat.verify_batch_arrays(*_slice(r, 0, 3000))
    assert (got == want).all()


def test_cached_keys_adversarial(nat, adversarial):
    """The adversarial fixture with every key cached: keys libsodium refuses
    (small order, non-canonical, not on the curve, the blocklist) are cached as
    refused, mixed-order keys keep their cofactorless verdicts, R edge cases
    (non-canonical y, small order, off curve) take the decode of -R."""
    from plenum_gpu.nacl_wrappers import verify_signed_batch
    rows = split_sm(adversarial)
    nat.keycache_add([pk for _, pk, _, _ in rows])
    got = verify_signed_batch([(pk, sm) for _, pk, sm, _ in rows])
    wrong = [rows[k][0] for k in range(len(rows)) if got[k] != rows[k][3]]
    assert not wrong, wrong
    # one signature at a time (the per-request Node.verifySignature shape)
    for k in range(0, len(rows), 7):
        _, pk, sm, v = rows[k]
        assert bool(verify_signed_batch([(pk, sm)])[0]) == v, rows[k][0]


def test_keycache_dedup_and_add_idr(nat, raw_vectors):
    """Adding cached keys again changes nothing; SimpleAuthNr.addIdr queues the
    registered DID's key and the next verify call adds it."""
    from plenum_gpu import base58
    from plenum_gpu.client_authn import SimpleAuthNr
    r = raw_vectors
    nat.keycache_add(r['pk'][:10])
    nat.keycache_add(np.concatenate([r['pk'][:10], r['pk'][:10]]))
    assert nat.keycache_size() == len(np.unique(r['pk'][:10], axis=0))
    a = SimpleAuthNr()
    a.addIdr('did1', base58.b58encode(bytes(r['pk'][20])).decode())
    a.addIdr('did2', 'not base58 0OIl')   # resolves to nothing: left to the request path
    got = nat.verify_batch_arrays(*_slice(r, 20, 1))
    assert got[0] == bool(r['verdict'][20])
    assert nat.keycache_size() == len(np.unique(r['pk'][:10], axis=0)) + 1


@pytest.mark.parametrize('n', [1, 8, 100, 1000, 8192])
def test_keyed_device_latency_kernel(nat, n):
    """Device keyed batches up to tuning.lat_keyed_max take k_verify_quad_keyed:
    verdicts and bitmap equal the synthetic spec (~5 % tampered) and the keyed
    throughput kernel (latency path disabled)."""
    from plenum_gpu.device import SyntheticBatch
    b = SyntheticBatch(0, n, 256, cfg=6, first=4242, key_mod=max(1, n // 8))
    assert b.use_key_cache(True)
    want = ~b.tamper.cpu().numpy().astype(bool)
    res = []
    for lat in (nat.LAT_KEYED_MAX_DEFAULT, 0):
        nat.set_lat_keyed_max(lat)
        b.bitmap.fill_(-1)
        v = b.verify().cpu().numpy().astype(bool)
        bits = np.unpackbits(b.bitmap.cpu().numpy().view(np.uint8), bitorder='little')[:n].astype(bool)
        assert (v == want).all(), lat
        assert (bits == v).all(), lat
        res.append(v)
    assert (res[0] == res[1]).all()


def test_wide_keys_c3_shape_and_adversarial(nat, adversarial):
    """Wide (radix-256) prepared keys on the GPU: a C3-shaped batch (25 node
    keys, 250k COMMIT votes) equals the synthetic spec and the narrow format,
    and the adversarial fixture (every refused, small-order, non-canonical and
    mixed-order key) gives libsodium's verdicts through
    pv_keys_prepare_wide_device + pv_verify_keyed_wide_device."""
    import torch
    from plenum_gpu import synth
    from plenum_gpu.device import SyntheticBatch, _p, _stream
    b = SyntheticBatch(0, 250_000, 0, cfg=3, mode=synth.COMMIT, first=0)
    want = ~b.tamper.cpu().numpy().astype(bool)
    res = []
    for wide in (True, False):
        assert b.use_key_cache(True, wide=wide)
        b.bitmap.fill_(-1)
        v = b.verify().cpu().numpy().astype(bool)
        bits = np.unpackbits(b.bitmap.cpu().numpy().view(np.uint8), bitorder='little')[:b.n].astype(bool)
        assert (v == want).all(), wide
        assert (bits == v).all(), wide
        res.append(v)
    assert (res[0] == res[1]).all()
    # adversarial fixture, one signature per row, keys deduplicated
    rows = [r for r in split_sm(adversarial) if len(r[2]) >= 64]
    pk = np.stack([np.frombuffer(r[1], np.uint8) for r in rows])
    upk, kidx = np.unique(pk, axis=0, return_inverse=True)
    msgs = [r[2][64:] for r in rows]
    off = np.zeros(len(rows) + 1, np.int64)
    off[1:] = np.cumsum([len(m) for m in msgs])
    dev = torch.device('cuda', 0)
    t_upk = torch.from_numpy(np.ascontiguousarray(upk)).to(dev)
    t_kidx = torch.from_numpy(np.ascontiguousarray(kidx.reshape(-1).astype(np.int32))).to(dev)
    t_sig = torch.from_numpy(np.stack([np.frombuffer(r[2][:64], np.uint8) for r in rows])).to(dev)
    t_blob = torch.zeros(int(off[-1]) + 64, dtype=torch.uint8, device=dev)
    if off[-1]:
        t_blob[:int(off[-1])] = torch.from_numpy(np.frombuffer(b''.join(msgs), np.uint8).copy()).to(dev)
    t_off = torch.from_numpy(off).to(dev)
    ktab = torch.empty(len(upk) * nat.PV_KEY_WORDS_WIDE, dtype=torch.int32, device=dev)
    verdict = torch.empty(len(rows), dtype=torch.uint8, device=dev)
    lib = nat.load()
    nat._check('pv_keys_prepare_wide_device',
               lib.pv_keys_prepare_wide_device(_p(t_upk), len(upk), _p(ktab), 0, _stream(dev)))
    nat._check('pv_verify_keyed_wide_device',
               lib.pv_verify_keyed_wide_device(_p(ktab), _p(t_kidx), _p(t_upk), _p(t_sig), _p(t_blob), _p(t_off),
                                               len(rows), _p(verdict), None, 0, _stream(dev)))
    got = verdict.cpu().numpy().astype(bool)
    wrong = [rows[k][0] for k in range(len(rows)) if got[k] != rows[k][3]]
    assert not wrong, wrong


def test_completion_word_over_many_calls(nat, raw_vectors):
    """Zero-copy calls complete by a word the host polls: all-cached calls get it
    from the keyed kernel's last block (a device block counter it re-arms), mixed
    and uncached calls from k_signal.  Interleave the three kinds over 120 calls of
    ragged sizes (1..1,000 signatures, 1..125 blocks) so that every sequence
    number, counter re-arm and hand-over between the two completion paths is
    exercised; each call must return its own fixture verdicts."""
    r = raw_vectors
    want = r['verdict'].astype(bool)
    nat.keycache_add(r['pk'][:1500])
    rng = np.random.default_rng(7)
    for c in range(120):
        n = int(rng.choice([1, 2, 7, 8, 9, 63, 64, 65, 250, 1000]))
        kind = c % 3
        if kind == 0:     # every key cached: the kernel writes the word
            start = int(rng.integers(0, 1500 - n + 1))
        elif kind == 1:   # straddles the cached range: keyed + list kernels, then k_signal
            start = max(0, 1500 - n // 2 - 1)
        else:             # no key cached: the generic latency kernel, then k_signal
            start = int(rng.integers(1500, len(want) - n + 1))
        got = nat.verify_batch_arrays(*_slice(r, start, n))
        assert (got == want[start:start + n]).all(), (c, kind, start, n)


def test_completion_word_synchronize_fallback(nat, raw_vectors):
    """With no spin budget (pv_test_set_spin_ns(0)) every zero-copy call gives up
    on its completion word and reaches the hipStreamSynchronize fallback; the
    verdicts must still be the fixture's, for the kernel-written word (all keys
    cached) and the k_signal word (mixed / uncached), and a later call with the
    default budget must not see a stale word from the fallback calls."""
    r = raw_vectors
    want = r['verdict'].astype(bool)
    nat.keycache_add(r['pk'][:1500])
    try:
        nat.test_set_spin_ns(0)
        for start, n in ((0, 1), (3, 64), (1490, 20), (2000, 9), (1700, 1000)):
            got = nat.verify_batch_arrays(*_slice(r, start, n))
            assert (got == want[start:start + n]).all(), ('fallback', start, n)
    finally:
        nat.test_set_spin_ns(20_000_000)
    for start, n in ((5, 8), (2100, 7)):
        got = nat.verify_batch_arrays(*_slice(r, start, n))
        assert (got == want[start:start + n]).all(), ('after', start, n)
    with pytest.raises(Exception):
        nat.test_set_spin_ns(-1)
