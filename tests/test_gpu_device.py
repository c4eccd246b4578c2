"""Device-resident path (torch tensors through the *_device C-ABI entry
points): synthetic generator vs its host spec, and C2-size properties."""
import numpy as np
import pytest

import _oracle as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def torch_dev():
    import torch
    assert torch.cuda.is_available()
    return torch


def test_synth_matches_host_spec(torch_dev):
    from plenum_gpu import synth
    from plenum_gpu.device import SyntheticBatch
    n, mlen, first = 3000, 256, 123456
    b = SyntheticBatch(0, n, mlen, cfg=2, first=first)
    seeds, msgs, tamper = synth.host_batch(2, first, n, mlen)
    assert (b.seeds.cpu().numpy() == seeds).all()
    assert (b.tamper.cpu().numpy().astype(bool) == tamper).all()
    pk = b.pk.cpu().numpy()
    sig = b.sig.cpu().numpy()
    blob = b.blob.cpu().numpy()[:n * mlen]
    off = np.arange(n + 1, dtype=np.uint64) * mlen
    pk2, sig2 = orc.sign_batch(seeds, np.frombuffer(b''.join(msgs), np.uint8), off)
    assert (pk == pk2).all()
    for j in range(n):
        m2, s2 = (msgs[j], sig2[j].tobytes())
        if tamper[j]:
            m2, s2 = synth.apply_tamper(first + j, m2, s2)
        assert blob[j * mlen:(j + 1) * mlen].tobytes() == m2
        assert sig[j].tobytes() == s2
    v = b.verify().cpu().numpy().astype(bool)
    assert (v == ~tamper).all()
    want = orc.verify_batch(pk, sig, blob, off)
    assert (v == want).all()


def test_c2_full_size_properties(torch_dev):
    """BASELINE configs[1] size: 1M signatures, every tampered one rejected,
    every other accepted, bitmap == verdicts, idempotent across passes."""
    from plenum_gpu.device import SyntheticBatch
    n = 1_000_000
    b = SyntheticBatch(0, n, 256, cfg=2, first=0)
    v1 = b.verify().cpu().numpy().copy()
    tamper = b.tamper.cpu().numpy().astype(bool)
    assert (v1.astype(bool) == ~tamper).all()
    assert 0.045 < tamper.mean() < 0.055
    bits = np.unpackbits(b.bitmap.cpu().numpy().view(np.uint8), bitorder='little')[:n].astype(bool)
    assert (bits == v1.astype(bool)).all()
    v2 = b.verify().cpu().numpy()
    assert (v1 == v2).all()
    # spot-check against the oracle
    idx = np.random.default_rng(0).choice(n, 300, replace=False)
    pk = b.pk.cpu().numpy()[idx]
    sig = b.sig.cpu().numpy()[idx]
    blob_all = b.blob.cpu().numpy()
    msgs = b''.join(blob_all[i * 256:(i + 1) * 256].tobytes() for i in idx)
    want = orc.verify_batch(pk, sig, np.frombuffer(msgs, np.uint8), np.arange(301, dtype=np.uint64) * 256)
    assert (want == v1[idx].astype(bool)).all()


def test_curve_modes_identical(torch_dev, raw_vectors, adversarial):
    """The half-size path (default; throughput kernel and both latency-mode
    kernels: lane quads and lane pairs), every record through its full-length
    form (curve_mode PV_CURVE_FULL: the throughput kernel's full-length tasks and the
    quad kernel's deferred form) and the grouped kernel give identical verdicts
    and bitmaps on a 200k C2-shaped batch and on every fixture; the half path's
    deferred records really ran."""
    from plenum_gpu import _native as nat
    from plenum_gpu.device import SyntheticBatch
    from plenum_gpu.nacl_wrappers import verify_signed_batch
    from conftest import split_sm
    n = 200_000
    b = SyntheticBatch(0, n, 256, cfg=2, first=777)
    tamper = b.tamper.cpu().numpy().astype(bool)
    rows = split_sm(adversarial)
    r = raw_vectors
    try:
        for mode in ('half', 'half_quad', 'half_pair', 'full', 'full_quad', 'grouped'):
            # half/full: one lane per signature everywhere; *_quad / *_pair: the
            # latency kernels for the 200k batch and every fixture
            lat = mode.split('_')[1] if '_' in mode else None
            nat.set_lat_max(1 << 20 if lat else 0)
            nat.set_lat_kernel(lat or 'quad')
            mode = mode.split('_')[0]
            nat.set_curve_mode(mode)
            b.bitmap.fill_(-1)     # the half path must clear it itself
            v = b.verify().cpu().numpy().astype(bool)
            got_mode, deferred = nat.curve_stats(0)
            assert got_mode == mode
            if mode == 'half':
                assert 0 < deferred < n // 100      # ~0.2 % of random h
            elif mode == 'full':
                assert deferred == int((~tamper).sum()) or deferred >= n * 0.9
            assert (v == ~tamper).all(), (mode, lat)
            bits = np.unpackbits(b.bitmap.cpu().numpy().view(np.uint8), bitorder='little')[:n].astype(bool)
            assert (bits == v).all(), (mode, lat)
            got = nat.verify_batch_arrays(r['pk'], r['sig'], r['blob'], r['off'])
            assert (got == r['verdict'].astype(bool)).all(), (mode, lat)
            got = verify_signed_batch([(pk, sm) for _, pk, sm, _ in rows])
            wrong = [rows[k][0] for k in range(len(rows)) if got[k] != rows[k][3]]
            assert not wrong, (mode, lat, wrong)
    finally:
        nat.set_curve_mode('half')
        nat.set_lat_max(nat.LAT_MAX_DEFAULT)
        nat.set_lat_kernel('quad')


def test_latency_kernel_small_batches(torch_dev, raw_vectors):
    """Looper-pass sizes through the default latency kernel (lane quads):
    ragged batch sizes around the 8-signatures-per-block grid, each checked
    against the libsodium verdicts of the raw-vector fixture."""
    from plenum_gpu import _native as nat
    r = raw_vectors
    off = r['off']
    for start, n in ((0, 1), (5, 7), (11, 8), (100, 9), (200, 100), (1000, 1000), (17, 2048)):
        o = off[start:start + n + 1]
        blob = r['blob'][int(o[0]):int(o[-1])]
        got = nat.verify_batch_arrays(r['pk'][start:start + n], r['sig'][start:start + n], blob, o - o[0])
        assert (got == r['verdict'][start:start + n].astype(bool)).all(), (start, n)


def test_kernel_timer(torch_dev):
    from plenum_gpu.device import SyntheticBatch
    b = SyntheticBatch(0, 65536, 256, cfg=2)
    th, tc = b.time_kernels(2)
    assert th > 0 and tc > 0 and tc > th
    # live timing of ordinary verify calls (bench.py's timed region)
    from plenum_gpu import _native as nat
    nat.kernel_timing(0, True)
    for _ in range(3):
        b.verify()
    h, c, k = nat.kernel_timing(0, False)
    assert k == 3 and h > 0 and c > h
    assert nat.kernel_timing(0, False)[2] == 3      # stopped: no more launches recorded
    b.verify()
    assert nat.kernel_timing(0, False)[2] == 3


def _check_against_spec(b, mode, cfg, first, n, lo, hi, key_mod=0, n_nodes=25):
    from plenum_gpu import synth
    seeds, msgs, tamper, senders = synth.host_batch_ex(mode, cfg, first, n, lo, hi, key_mod, n_nodes)
    assert (b.seeds.cpu().numpy() == seeds).all()
    assert (b.tamper.cpu().numpy().astype(bool) == tamper).all()
    if mode == synth.COMMIT:
        assert (b.sender.cpu().numpy().astype(np.uint32) == senders).all()
    off = b.off.cpu().numpy().astype(np.uint64)
    lens = np.array([len(m) for m in msgs], np.uint64)
    assert (np.diff(off) == lens).all() and off[0] == 0
    blob = b.blob.cpu().numpy()[:int(off[-1])]
    pk2, sig2 = orc.sign_batch(seeds, np.frombuffer(b''.join(msgs), np.uint8), off)
    pk = b.pk.cpu().numpy()
    sig = b.sig.cpu().numpy()
    assert (pk == pk2).all()
    for j in range(n):
        m2, s2 = msgs[j], sig2[j].tobytes()
        if tamper[j]:
            m2, s2 = synth.apply_tamper(first + j, m2, s2)
        assert blob[int(off[j]):int(off[j + 1])].tobytes() == m2
        assert sig[j].tobytes() == s2
    v = b.verify().cpu().numpy().astype(bool)
    assert (v == ~tamper).all()
    assert (v == orc.verify_batch(pk, sig, blob, off)).all()


def test_synth_range_matches_host_spec(torch_dev):
    """C4 layout: ragged 128..4096-byte messages, key pool 2^20."""
    from plenum_gpu import synth
    from plenum_gpu.device import SyntheticBatch
    n, first = 700, (1 << 20) - 300
    b = SyntheticBatch(0, n, 128, cfg=4, first=first, key_mod=1 << 20, mode=synth.RANGE, mlen_max=4096)
    _check_against_spec(b, synth.RANGE, 4, first, n, 128, 4096, key_mod=1 << 20)
    # the key pool wraps: signature i and i + 2^20 share a key
    seeds = b.seeds.cpu().numpy()
    assert (seeds[300] == np.frombuffer(synth.seed(4, 0), np.uint8)).all()


def test_synth_commit_matches_host_spec(torch_dev):
    """C3 layout: 25-node COMMIT votes of 3PC batches 9990..10029 (ppSeqNo digits change)."""
    from plenum_gpu import synth
    from plenum_gpu.device import SyntheticBatch
    n_nodes = 25
    first = 9990 * n_nodes
    b = SyntheticBatch(0, 40 * n_nodes, 0, cfg=3, first=first, mode=synth.COMMIT, n_nodes=n_nodes)
    _check_against_spec(b, synth.COMMIT, 3, first, 40 * n_nodes, 0, 0, n_nodes=n_nodes)


def test_c3_full_size_quorums(torch_dev):
    """BASELINE configs[2]: 25-node pool (f = 8), 100k 3PC batches of COMMIT
    votes: verify 2.5M signatures + n - f tally on one GPU; every quorum bit and
    vote count equals the spec's voter-set count (synth.c3_expected)."""
    import torch
    from plenum_gpu import synth
    from plenum_gpu.device import SyntheticBatch, tally_device
    from plenum_gpu.quorums import Quorums
    n_nodes, nb = 25, 100_000
    q = Quorums(n_nodes)
    assert (q.f, q.commit.value, q.prepare.value) == (8, 17, 16)
    b = SyntheticBatch(0, nb * n_nodes, 0, cfg=3, mode=synth.COMMIT, n_nodes=n_nodes)
    v = b.verify()
    assert (v.cpu().numpy().astype(bool) == ~b.tamper.cpu().numpy().astype(bool)).all()
    dev = b.pk.device
    boff = torch.arange(nb + 1, dtype=torch.int64, device=dev) * n_nodes
    votes = torch.empty(nb, dtype=torch.int32, device=dev)
    reached = torch.empty(nb, dtype=torch.uint8, device=dev)
    tally_device(v, b.sender, boff, n_nodes, q.commit.value, votes, reached)
    want_votes, want_reached = synth.c3_expected(0, nb, n_nodes, q.commit.value)
    assert (votes.cpu().numpy() == want_votes.astype(np.int32)).all()
    assert (reached.cpu().numpy().astype(bool) == want_reached).all()
    assert 0.2 < want_reached.mean() < 0.9


def test_c4_shape_properties(torch_dev):
    """BASELINE configs[3] per-GPU shape at reduced count: ragged 128..4096-byte
    messages, key pool 2^20, ~5 % tampered; verdict == not tampered."""
    from plenum_gpu import synth
    from plenum_gpu.device import SyntheticBatch
    n = 300_000
    b = SyntheticBatch(0, n, 128, cfg=4, first=5 * n, key_mod=1 << 20, mode=synth.RANGE, mlen_max=4096)
    v = b.verify().cpu().numpy().astype(bool)
    tamper = b.tamper.cpu().numpy().astype(bool)
    assert (v == ~tamper).all()
    assert 0.045 < tamper.mean() < 0.055


def test_c4_full_shard(torch_dev):
    """BASELINE configs[3] as configured, per GPU: the full 8M-signature shard of
    the 64M / 8-GPU batch (payloads uniform 128 B..4 KB, key pool 2^20, ~5 %
    tampered), through the unkeyed path and the prepared-key path.  Size-
    independent properties on all 8M (verdict == not tampered, bitmap ==
    verdicts, both paths identical) and a 2048-signature oracle spot check
    spread over the shard."""
    import torch
    from plenum_gpu import synth
    from plenum_gpu.device import SyntheticBatch
    n = 8_000_000
    b = SyntheticBatch(0, n, 128, cfg=4, first=3 * n, key_mod=1 << 20, mode=synth.RANGE, mlen_max=4096)
    tamper = b.tamper.cpu().numpy().astype(bool)
    assert 0.049 < tamper.mean() < 0.051
    verdicts = []
    for keyed in (False, True):
        assert b.use_key_cache(keyed) == keyed
        b.bitmap.zero_()
        v = b.verify().cpu().numpy().astype(bool)
        bits = np.unpackbits(b.bitmap.cpu().numpy().view(np.uint8), bitorder='little')[:n].astype(bool)
        assert (bits == v).all()
        assert (v == ~tamper).all()
        verdicts.append(v)
    assert (verdicts[0] == verdicts[1]).all()
    rng = np.random.default_rng(44)
    idx = np.sort(rng.choice(n, 2048, replace=False))
    it = torch.from_numpy(idx).to(b.pk.device)
    pk = b.pk[it].cpu().numpy()
    sig = b.sig[it].cpu().numpy()
    off = b.off.cpu().numpy()
    msgs = [b.blob[int(off[i]):int(off[i + 1])].cpu().numpy() for i in idx]
    loff = np.zeros(len(idx) + 1, np.uint64)
    loff[1:] = np.cumsum([len(m) for m in msgs])
    want = orc.verify_batch(pk, sig, np.concatenate(msgs), loff)
    assert (verdicts[0][idx] == want).all()
    assert not want.all() and want.any()


@pytest.mark.parametrize('keyed,beside', [(False, True), (True, True), (True, False), ('wide', True)])
def test_pipelined_async_slots(torch_dev, keyed, beside):
    """bench.py's pipelined schedule: passes alternate over two streams with
    verify workspaces / output sets 0 and 1 (pv_*_device_async), several in
    flight at once; every slot's verdicts and bitmap equal the synchronous
    pass, and the generic path matches the oracle on a sample.  Keyed passes
    either prepare the keys on the slot's side stream beside the hash stage
    (pv_verify_keys_device_async, `beside`) or before it on the same stream;
    either way every slot's key table equals the synchronous preparation's."""
    torch = torch_dev
    from plenum_gpu import synth
    from plenum_gpu.device import SyntheticBatch
    n = 200_000
    if keyed == 'wide':   # C3's shape: 25 node keys in the radix-256 format
        b = SyntheticBatch(0, 25 * 8000, 0, cfg=3, first=25 * 31, mode=synth.COMMIT, n_nodes=25)
        b.use_key_cache(True, wide=True)
        n = b.n
    else:
        b = SyntheticBatch(0, n, 128, cfg=4, mode=1, mlen_max=1024, key_mod=4096 if keyed else 0)
        b.use_key_cache(keyed)
    b.make_slots()
    if keyed:   # padding words of the tables are never written: the same fill in both slots
        for slot in range(2):
            b.slot_out[slot][2].fill_(-1)
    want = b.verify().cpu().numpy().copy()
    want_bits = b.bitmap.cpu().numpy().copy()
    want_tab = b.ktab.cpu().numpy().copy() if keyed else None
    tamper = b.tamper.cpu().numpy().astype(bool)
    assert (want.astype(bool) == ~tamper).all()
    for slot in range(2):
        b.slot_out[slot][0].fill_(7)
        b.slot_out[slot][1].zero_()
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(b.device), torch.cuda.Stream(b.device)]
    for k in range(6):
        with torch.cuda.stream(streams[k & 1]):
            b.verify_async(k & 1, streams[k & 1], keys_beside=beside)
    torch.cuda.synchronize()
    for slot in range(2):
        v, bm, kt = b.slot_out[slot]
        assert (v.cpu().numpy() == want).all()
        assert (bm.cpu().numpy() == want_bits).all()
        if keyed:
            assert (kt.cpu().numpy() == want_tab).all()
    if not keyed:
        idx = np.random.default_rng(1).choice(n, 200, replace=False)
        off = b.off.cpu().numpy().astype(np.uint64)
        blob = b.blob.cpu().numpy()
        pk, sig = b.pk.cpu().numpy()[idx], b.sig.cpu().numpy()[idx]
        msgs = [blob[int(off[i]):int(off[i + 1])].tobytes() for i in idx]
        soff = np.zeros(len(idx) + 1, np.uint64)
        soff[1:] = np.cumsum([len(m) for m in msgs])
        got = orc.verify_batch(pk, sig, np.frombuffer(b''.join(msgs), np.uint8), soff)
        assert (got == want[idx].astype(bool)).all()


def test_async_slot_rejected(torch_dev):
    """Workspace slots other than 0 and 1 are refused through the C-ABI."""
    import ctypes
    from plenum_gpu import _native as nat
    from plenum_gpu.device import SyntheticBatch, _p
    b = SyntheticBatch(0, 64, 32, cfg=2)
    s = ctypes.c_void_p(torch_dev.cuda.current_stream(b.device).cuda_stream)
    rc = nat.load().pv_verify_batch_device_async(_p(b.pk), _p(b.sig), _p(b.blob), _p(b.off), b.n, _p(b.verdict),
                                                 _p(b.bitmap), 0, s, 2)
    assert rc != 0
    # the one-call key preparation + keyed verify: bad slot, bad format, signatures without keys
    import torch
    kt = torch.empty(nat.PV_KEY_WORDS, dtype=torch.int32, device=b.device)
    ki = torch.zeros(b.n, dtype=torch.int32, device=b.device)
    lib = nat.load()
    for k, wide, slot in ((1, 0, 2), (1, 2, 0), (0, 0, 0)):
        rc = lib.pv_verify_keys_device_async(_p(b.pk), k, _p(kt), _p(ki), _p(b.sig), _p(b.blob), _p(b.off), b.n,
                                             _p(b.verdict), _p(b.bitmap), wide, 0, s, slot)
        assert rc != 0, (k, wide, slot)
