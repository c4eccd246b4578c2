"""BLS COMMIT check on the GPU (row f4) against the fixture and the C oracle.

PARITY UNPINNED: the checker is oracle/bn254_oracle.c (a
restatement of python-ursa 0.1.1 / AMCL BN254, which are absent); the fixture's
verdicts come from the naive pure-Python pairing, its generator and message
bytes from the reference."""
import ctypes
import hashlib
import json
import os

import numpy as np
import pytest

import _bn254_py as bn
from conftest import REPO, golden

pytestmark = pytest.mark.gpu
ORACLE = os.path.join(REPO, 'oracle', 'libbls_oracle.so')


@pytest.fixture(scope='module')
def fx():
    with open(golden('bls.json')) as fh:
        return json.load(fh)


@pytest.fixture(scope='module')
def nat():
    from plenum_gpu import _native
    _native.ensure_init()
    return _native


@pytest.fixture(scope='module')
def orc():
    return ctypes.CDLL(ORACLE)


def _pack(msgs):
    from plenum_gpu import _native
    return _native.pack_messages(list(msgs))


def test_fixture_cases_raw(fx, nat):
    gb = bytes.fromhex(fx['generator_hex'])
    extra = sorted({c['pk'] for c in fx['cases'] if 'pk' in c})
    pks = [bytes.fromhex(k['pk']) for k in fx['keys']] + [bytes.fromhex(p) for p in extra]
    st = nat.bls_set_keys(gb, np.frombuffer(b''.join(pks), np.uint8))
    assert list(st[:len(fx['keys'])]) == [0] * len(fx['keys']) and all(s == 1 for s in st[len(fx['keys']):])
    msgs = sorted({c['msg'] for c in fx['cases']})
    blob, off = _pack(bytes.fromhex(m) for m in msgs)
    sig = np.zeros((len(fx['cases']), 128), np.uint8)
    sl = np.zeros(len(fx['cases']), np.uint64)
    kidx, midx = [], []
    for j, c in enumerate(fx['cases']):
        b = bytes.fromhex(c['sig'])
        sl[j] = len(b)
        sig[j, :min(128, len(b))] = np.frombuffer(b[:128], np.uint8)
        kidx.append(c['key'] if 'key' in c else len(fx['keys']) + extra.index(c['pk']))
        midx.append(msgs.index(c['msg']))
    got = nat.bls_verify_arrays(sig, blob, off, np.array(midx, np.uint32), np.array(kidx, np.uint32), sig_len=sl)
    want = [c['verdict'] for c in fx['cases']]
    bad = [fx['cases'][j]['label'] for j in range(len(want)) if got[j] != want[j]]
    assert not bad, bad


def test_fixture_cases_mirror(fx, nat):
    from plenum_gpu.bls import (BlsCryptoVerifierGpu, BlsGroupParamsLoaderIndyCrypto, IndyCryptoBlsUtils, VerKey)
    v = BlsCryptoVerifierGpu(BlsGroupParamsLoaderIndyCrypto().load_group_params())
    items = []
    for c in fx['cases']:
        pk = VerKey(bytes.fromhex(fx['keys'][c['key']]['pk'] if 'key' in c else c['pk']))
        items.append((IndyCryptoBlsUtils.bls_to_str(VerKey(bytes.fromhex(c['sig']))), bytes.fromhex(c['msg']), pk))
    got = v.verify_sig_batch(items)
    assert list(got) == [c['verdict'] for c in fx['cases']]
    # the per-call entry point and the None rules of verify_sig (:73-82)
    assert v.verify_sig(*items[0]) is True
    assert v.verify_sig(items[0][0], items[0][1], None) is False
    assert v.verify_sig('0OIl', items[0][1], items[0][2]) is False


def test_key_status_outside_g2(fx, nat):
    gb = bytes.fromhex(fx['generator_hex'])
    q = bn.twist_point_outside_g2()
    st = nat.bls_set_keys(gb, np.frombuffer(bn.g2_to_bytes(q) + bytes.fromhex(fx['keys'][0]['pk']), np.uint8))
    assert list(st) == [2, 0]
    with pytest.raises(nat.PlenumGpuError):
        bad = bytearray(gb)
        bad[3] ^= 1
        nat.bls_set_keys(bytes(bad), np.zeros((0, 128), np.uint8))
    # a failed pv_bls_set_keys leaves NO key set: verify -> PV_ENOTINIT
    with pytest.raises(nat.PlenumGpuError) as e:
        nat.bls_verify_arrays(np.zeros((1, 128), np.uint8), *_pack([b'm']), np.zeros(1, np.uint32),
                              np.zeros(1, np.uint32))
    assert e.value.code == -77


def test_device_entry_out_of_range_indices(fx, nat):
    """pv_bls_verify_batch_device does not check indices on the host: a check with
    key_idx >= the key count or msg_idx >= n_msgs gets verdict 0 and touches
    nothing out of range; the in-range checks of the same call are unaffected."""
    import torch
    from plenum_gpu.device import _p, _stream
    gb = bytes.fromhex(fx['generator_hex'])
    nk = len(fx['keys'])
    st = nat.bls_set_keys(gb, np.frombuffer(b''.join(bytes.fromhex(k['pk']) for k in fx['keys']), np.uint8))
    assert not st.any()
    good = [c for c in fx['cases'] if c.get('verdict') and 'key' in c and len(c['sig']) == 256][:2]
    assert len(good) == 2
    msgs = [bytes.fromhex(c['msg']) for c in good]
    blob_h, off_h = _pack(msgs)
    dev = torch.device('cuda', 0)
    sig = torch.from_numpy(np.stack([np.frombuffer(bytes.fromhex(c['sig']), np.uint8) for c in good] * 3)).to(dev)
    blob = torch.zeros(blob_h.size + 64, dtype=torch.uint8, device=dev)
    blob[:blob_h.size] = torch.from_numpy(blob_h.copy()).to(dev)
    off = torch.from_numpy(off_h.astype(np.int64)).to(dev)
    kid = [good[0]['key'], good[1]['key'], nk + 5, 0xffffffff, good[0]['key'], good[1]['key']]
    mid = [0, 1, 0, 1, 7, 0xffffffff]
    kidx = torch.tensor(np.array(kid, np.uint32).view(np.int32), device=dev)
    midx = torch.tensor(np.array(mid, np.uint32).view(np.int32), device=dev)
    verdict = torch.full((6,), 9, dtype=torch.uint8, device=dev)
    lib = nat.load()
    nat._bls_check('pv_bls_verify_batch_device', lib.pv_bls_verify_batch_device(
        _p(sig), _p(blob), _p(off), 2, _p(midx), _p(kidx), 6, _p(verdict), 0, _stream(dev)))
    assert verdict.cpu().tolist() == [1, 1, 0, 0, 0, 0]


def test_10k_checks_vs_oracle(fx, nat, orc):
    """25 node keys, 400 COMMIT messages (the reference's MultiSignatureValue
    layout), 10,000 checks signed on the GPU, ~10 % corrupted four ways; every
    verdict against the C oracle (16 host threads)."""
    from plenum_gpu.bls import MultiSignatureValue
    gb = bytes.fromhex(fx['generator_hex'])
    rng = np.random.default_rng(9)
    nk, nm, n = 25, 400, 10_000
    sks = np.frombuffer(b''.join((int.from_bytes(hashlib.sha256(b'k' + bytes([i])).digest(), 'big') % bn.R)
                                 .to_bytes(32, 'big') for i in range(nk)), np.uint8).reshape(nk, 32)
    pks = nat.bls_pubkeys(gb, sks)
    # the GPU key generator against the oracle's
    want_pk = ctypes.create_string_buffer(128)
    orc.bls_oracle_pubkey(sks[3].tobytes(), gb, want_pk)
    assert pks[3].tobytes() == want_pk.raw
    msgs = [MultiSignatureValue(1, 'S' * 44, 'P' * 44, 'T%043d' % b, 1700000000 + b).as_single_value()
            for b in range(nm)]
    blob, off = _pack(msgs)
    midx = rng.integers(0, nm, n).astype(np.uint32)
    kidx = rng.integers(0, nk, n).astype(np.uint32)
    sig = nat.bls_sign_arrays(sks, blob, off, midx, kidx)
    s1 = ctypes.create_string_buffer(128)
    orc.bls_oracle_sign(sks[kidx[0]].tobytes(), msgs[midx[0]], len(msgs[midx[0]]), s1)
    assert sig[0].tobytes() == s1.raw
    bad = rng.choice(n, n // 10, replace=False)
    for q, j in enumerate(bad):
        kind = q % 4
        if kind == 0:
            midx[j] = (midx[j] + 1) % nm            # another message
        elif kind == 1:
            kidx[j] = (kidx[j] + 1) % nk            # another key
        elif kind == 2:
            sig[j, 1 + rng.integers(0, 64)] ^= np.uint8(1 << rng.integers(0, 8))   # bit flip (mostly off-curve)
        else:
            sig[j, 0] = 3                            # compressed form, one of the two parities
    st = nat.bls_set_keys(gb, pks)
    assert not st.any()
    got = nat.bls_verify_arrays(sig, blob, off, midx, kidx)
    want = np.zeros(n, np.uint8)
    keys = np.ascontiguousarray(pks)
    blob16 = np.concatenate([blob, np.zeros(16, np.uint8)])
    p = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
    orc.bls_oracle_verify_batch(p(sig), None, p(blob16), p(off), p(midx), p(kidx), p(keys), gb, ctypes.c_uint64(n),
                                p(want), 16)
    assert (got == want.astype(bool)).all(), np.nonzero(got != want.astype(bool))[0][:10]
    assert 0.85 * n < got.sum() < 0.95 * n
    h_ms, v_ms = nat.bls_kernel_ms()
    assert v_ms > 0
    # 10k checks take the lane-quad kernel by default (pv_tuning.bls_quad_max =
    # 32768, bls_oct_max = 4096); the lane-pair kernel (both 0) and the lane-octet
    # kernel (bls_oct_max above n) give the same verdicts
    for kw in ({'bls_quad_max': 0, 'bls_oct_max': 0}, {'bls_oct_max': 1 << 20}):
        prev = nat.set_tuning(**kw)
        try:
            other = nat.bls_verify_arrays(sig, blob, off, midx, kidx)
        finally:
            nat.set_tuning(**prev)
        assert (other == got).all(), (kw, np.nonzero(other != got)[0][:10])


def test_commit_batch_and_quorum(fx, nat):
    """validate_commit's rule over 25-node COMMITs of 30 batches, then the n - f
    quorum on the tally kernel, against the Python voter-set count."""
    from plenum_gpu.bls import (CM_BLS_SIG_WRONG, BlsCryptoVerifierGpu, BlsGroupParamsLoaderIndyCrypto,
                                IndyCryptoBlsUtils, MultiSignatureValue, VerKey, commit_quorums)
    from plenum_gpu.quorums import Quorums
    gb = bytes.fromhex(fx['generator_hex'])
    nn, nb = 25, 30
    q = Quorums(nn)
    sks = np.frombuffer(b''.join((int.from_bytes(hashlib.sha256(b'n' + bytes([i])).digest(), 'big') % bn.R)
                                 .to_bytes(32, 'big') for i in range(nn)), np.uint8).reshape(nn, 32)
    pks = nat.bls_pubkeys(gb, sks)
    vals = [MultiSignatureValue(1, 'S%043d' % b, 'P' * 44, 'T%043d' % b, 1700000000 + b) for b in range(nb)]
    msgs = [v.as_single_value() for v in vals]
    blob, off = _pack(msgs)
    midx = np.repeat(np.arange(nb, dtype=np.uint32), nn)
    kidx = np.tile(np.arange(nn, dtype=np.uint32), nb)
    sig = nat.bls_sign_arrays(sks, blob, off, midx, kidx)
    rng = np.random.default_rng(5)
    n_bad = [int(rng.integers(0, 13)) for _ in range(nb)]     # 0..12 wrong COMMITs per batch
    commits, senders, expect_ok = [], [], []
    for b in range(nb):
        wrong = set(rng.choice(nn, n_bad[b], replace=False).tolist())
        for i in range(nn):
            s = sig[b * nn + i].tobytes()
            if i in wrong:
                s = sig[b * nn + (i + 1) % nn].tobytes()         # another node's signature
            commits.append((VerKey(pks[i].tobytes()), {'1': IndyCryptoBlsUtils.bls_to_str(VerKey(s))}, {1: vals[b]}))
            senders.append(i)
            expect_ok.append(i not in wrong)
    v = BlsCryptoVerifierGpu(BlsGroupParamsLoaderIndyCrypto().load_group_params())
    res = v.validate_commit_batch(commits)
    assert [r is None for r in res] == expect_ok
    assert all(r in (None, CM_BLS_SIG_WRONG) for r in res)
    # a ledger the audit transaction does not cover
    assert v.validate_commit_batch([(commits[0][0], {'7': commits[0][1]['1']}, {1: vals[0]})]) == [CM_BLS_SIG_WRONG]
    votes, reached = commit_quorums([r is None for r in res], np.array(senders, np.uint32),
                                    np.arange(nb + 1, dtype=np.uint64) * nn, nn, q.commit.value)
    assert list(votes) == [nn - k for k in n_bad]
    assert list(reached) == [nn - k >= q.commit.value for k in n_bad]
    assert 0 < sum(reached) < nb


def test_verify_after_shutdown_reinit(fx, nat):
    """shutdown() releases the device key set (pv_bls_shutdown); the content
    index of the key set must go with it, so a verifier built after re-init with
    the same generator rebuilds the set instead of trusting stale indices
    (ADVICE r5).  Also: a set released behind the index (pv_bls_shutdown called
    directly) is detected through pv_bls_keyset_info and rebuilt."""
    from plenum_gpu.bls import (BlsCryptoVerifierGpu, BlsGroupParamsLoaderIndyCrypto, IndyCryptoBlsUtils, VerKey)
    c = next(c for c in fx['cases'] if c['verdict'] and 'key' in c)
    item = (IndyCryptoBlsUtils.bls_to_str(VerKey(bytes.fromhex(c['sig']))), bytes.fromhex(c['msg']),
            VerKey(bytes.fromhex(fx['keys'][c['key']]['pk'])))
    params = BlsGroupParamsLoaderIndyCrypto().load_group_params()
    assert BlsCryptoVerifierGpu(params).verify_sig(*item) is True
    nat.shutdown()
    nat.ensure_init()
    assert BlsCryptoVerifierGpu(params).verify_sig(*item) is True
    nat.load().pv_bls_shutdown()
    assert BlsCryptoVerifierGpu(params).verify_sig(*item) is True
