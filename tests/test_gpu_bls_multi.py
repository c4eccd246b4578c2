"""The rest of the BLS verifier drop-in on the GPU (row f4): verify_multi_sig,
create_multi_sig, verify_key_proof_of_possession
(crypto/bls/indy_crypto/bls_crypto_indy_crypto.py:84-109) and the COMMIT batch
seam (plenum_gpu/commit_ingress.py), against the C oracle.

PARITY UNPINNED: the checker is oracle/bn254_oracle.c, a
restatement of python-ursa 0.1.1 / AMCL BN254 (absent here); the oracle itself
is cross-checked with the naive pure-Python pairing in tests/test_bls_oracle.py."""
import ctypes
import hashlib
import json
import os

import numpy as np
import pytest

import _bn254_py as bn
from _commit_cases import Commit, FakeBlsReplica, PrePrepare, audit_txn
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


@pytest.fixture(scope='module')
def pool(fx, nat):
    """25 node keys and their signatures over 40 ledger values"""
    from plenum_gpu.bls import MultiSignatureValue
    gb = bytes.fromhex(fx['generator_hex'])
    nn, nm = 25, 40
    sks = np.frombuffer(b''.join((int.from_bytes(hashlib.sha256(b'm' + bytes([i])).digest(), 'big') % bn.R)
                                 .to_bytes(32, 'big') for i in range(nn)), np.uint8).reshape(nn, 32)
    pks = nat.bls_pubkeys(gb, sks)
    vals = [MultiSignatureValue(1 + b % 3, 'S%043d' % b, 'P' * 44, 'T%043d' % b, 1700000000 + b) for b in range(nm)]
    msgs = [v.as_single_value() for v in vals]
    blob, off = nat.pack_messages(msgs)
    midx = np.repeat(np.arange(nm, dtype=np.uint32), nn)
    kidx = np.tile(np.arange(nn, dtype=np.uint32), nm)
    sig = nat.bls_sign_arrays(sks, blob, off, midx, kidx).reshape(nm, nn, 128)
    return dict(gb=gb, sks=sks, pks=pks, vals=vals, msgs=msgs, sig=sig, nn=nn, nm=nm)


def _verifier():
    from plenum_gpu.bls import BlsCryptoVerifierGpu, BlsGroupParamsLoaderIndyCrypto
    return BlsCryptoVerifierGpu(BlsGroupParamsLoaderIndyCrypto().load_group_params())


def _s(b):
    from plenum_gpu.bls import IndyCryptoBlsUtils, Signature
    return IndyCryptoBlsUtils.bls_to_str(Signature(bytes(b)))


def test_create_multi_sig_vs_oracle(pool, orc):
    """MultiSignature.new over 17..25 participants per 3PC batch, every set in one launch"""
    v = _verifier()
    rng = np.random.default_rng(3)
    sets, parts = [], []
    for b in range(pool['nm']):
        p = sorted(rng.choice(pool['nn'], int(rng.integers(17, 26)), replace=False).tolist())
        parts.append(p)
        sets.append([_s(pool['sig'][b, i]) for i in p])
    got = v.create_multi_sig_batch(sets)
    from plenum_gpu.bls import IndyCryptoBlsUtils, MultiSignature
    for b, p in enumerate(parts):
        want = ctypes.create_string_buffer(128)
        raw = b''.join(pool['sig'][b, i].tobytes() for i in p)
        orc.bls_oracle_aggregate_sigs(raw, ctypes.c_uint64(len(p)), want)
        assert IndyCryptoBlsUtils.bls_from_str(got[b], MultiSignature).as_bytes() == want.raw, b
    assert v.create_multi_sig(sets[0]) == got[0]
    # sigma + (-sigma) = O, AMCL's (0, 1); an empty set is O too
    s0 = bn.g1_from_bytes(pool['sig'][0, 0].tobytes())
    o = v.create_multi_sig([_s(pool['sig'][0, 0]), _s(bn.g1_to_bytes(bn.g1_neg(s0)))])
    inf = b'\x04' + bytes(63) + b'\x01' + bytes(63)
    assert IndyCryptoBlsUtils.bls_from_str(o, MultiSignature).as_bytes() == inf
    assert IndyCryptoBlsUtils.bls_from_str(v.create_multi_sig([]), MultiSignature).as_bytes() == inf
    # a doubled signature (the same signer twice): the doubling case of the sum
    d = v.create_multi_sig([_s(pool['sig'][0, 0])] * 2)
    assert IndyCryptoBlsUtils.bls_from_str(d, MultiSignature).as_bytes() == bn.g1_to_bytes(bn.g1_add(s0, s0))
    # an undecodable signature: ursa's MultiSignature.new fails on the None
    with pytest.raises(AttributeError):
        v.create_multi_sig([_s(pool['sig'][0, 0]), '0OIl'])


def test_verify_multi_sig_vs_oracle(pool, orc, nat):
    """PRE-PREPARE multi-signature checks: correct participant sets, a missing
    or an extra key, a wrong signer inside the aggregate, another message, an
    off-twist key, an empty key list — every verdict against the oracle."""
    from plenum_gpu.bls import IndyCryptoBlsUtils, MultiSignature, VerKey
    v = _verifier()
    rng = np.random.default_rng(11)
    nn, nm = pool['nn'], pool['nm']
    keys = [VerKey(pool['pks'][i].tobytes()) for i in range(nn)]
    items, expect_true = [], []
    for b in range(nm):
        p = sorted(rng.choice(nn, int(rng.integers(17, 26)), replace=False).tolist())
        sigs = [_s(pool['sig'][b, i]) for i in p]
        kind = b % 8
        msg = pool['msgs'][b]
        ks = [keys[i] for i in p]
        ok = True
        if kind == 1:
            ks, ok = ks[:-1], False                               # a participant's key missing
        elif kind == 2:
            others = [i for i in range(nn) if i not in p]
            if others:
                ks, ok = ks + [keys[others[0]]], False            # a key that did not sign
        elif kind == 3:
            sigs[0], ok = _s(pool['sig'][(b + 1) % nm, p[0]]), False   # one signer signed another value
        elif kind == 4:
            msg, ok = pool['msgs'][(b + 1) % nm], False           # another message
        elif kind == 5:
            ks = ks + [VerKey(bytes(128))]                        # an off-twist key adds O
        elif kind == 6:
            ks = ks + ks[:1]                                      # a key twice (doubling in the sum)
            sigs = sigs + sigs[:1]
        ms = v.create_multi_sig(sigs)
        items.append((ms, msg, ks))
        expect_true.append(ok)
    got = v.verify_multi_sig_batch(items)
    want = []
    for ms, msg, ks in items:
        raw = IndyCryptoBlsUtils.bls_from_str(ms, MultiSignature).as_bytes()
        want.append(orc.bls_oracle_verify_multi(raw, ctypes.c_uint64(128), msg, ctypes.c_uint64(len(msg)),
                                                b''.join(k.as_bytes() for k in ks), ctypes.c_uint64(len(ks)),
                                                pool['gb']))
    assert list(got) == [bool(w) for w in want]
    assert list(got) == expect_true
    # the per-call entry point and the None rules (:84-97)
    assert v.verify_multi_sig(*items[0]) is True
    assert v.verify_multi_sig(items[0][0], items[0][1], list(items[0][2]) + [None]) is False
    assert v.verify_multi_sig('0OIl', items[0][1], items[0][2]) is False
    # an empty key list sums to O: only sigma = O verifies
    o = v.create_multi_sig([])
    assert v.verify_multi_sig(o, b'x', []) is True
    assert v.verify_multi_sig(items[0][0], items[0][1], []) is False
    # the single-key set of pv_bls_set_keys survives a multi-signature call
    assert v.verify_sig(_s(pool['sig'][0, 3]), pool['msgs'][0], keys[3]) is True
    v.verify_multi_sig(*items[0])
    assert v.verify_sig(_s(pool['sig'][0, 3]), pool['msgs'][0], keys[3]) is True


def test_verify_key_proof_of_possession(pool, nat, orc):
    """Bls.verify_pop: e(pop, g) == e(H(pk bytes), pk); pop = sk * H(pk bytes)"""
    from plenum_gpu.bls import ProofOfPossession, VerKey
    v = _verifier()
    nn = pool['nn']
    blob, off = nat.pack_messages([pool['pks'][i].tobytes() for i in range(nn)])
    idx = np.arange(nn, dtype=np.uint32)
    pops = nat.bls_sign_arrays(pool['sks'], blob, off, idx, idx)
    for i in (0, 7, 24):
        pk = pool['pks'][i].tobytes()
        want = orc.bls_oracle_verify(pops[i].tobytes(), ctypes.c_uint64(128), pk, ctypes.c_uint64(128), pk,
                                     pool['gb'])
        assert want == 1
        assert v.verify_key_proof_of_possession(ProofOfPossession(pops[i].tobytes()), VerKey(pk)) is True
    assert v.verify_key_proof_of_possession(ProofOfPossession(pops[1].tobytes()),
                                            VerKey(pool['pks'][2].tobytes())) is False
    assert v.verify_key_proof_of_possession(None, VerKey(pool['pks'][2].tobytes())) is False
    assert v.verify_key_proof_of_possession(ProofOfPossession(pops[1].tobytes()), None) is False
    # node_handler.py:207-213 decodes both from base58 first: a short proof is None -> False
    from plenum_gpu.bls import IndyCryptoBlsUtils
    assert IndyCryptoBlsUtils.bls_from_str(_s(pops[0][:64]), ProofOfPossession) is None


def test_commit_ingress_30_batches_one_gpu_pass(pool, nat):
    """30 3PC batches x 25 COMMITs (two ledgers each, ~1 in 6 wrong) through the
    COMMIT seam: ONE pv_bls_verify_batch call, then the reference's unchanged
    per-COMMIT validate_commit consumes the verdicts without a GPU call."""
    from plenum_gpu.bls import MultiSignatureValue, VerKey
    from plenum_gpu.commit_ingress import CommitIngress, replica_commit_items
    v = _verifier()
    nn, nb = pool['nn'], 30
    keys = {'Node%d' % i: VerKey(pool['pks'][i].tobytes()) for i in range(nn)}
    # per batch b, ledger 1 covers value 2b, ledger 2 value 2b + 1 (pool vals: ledger id 1 + k % 3)
    pps, audit, sig_of = {}, {}, {}
    sks = pool['sks']
    msgs, rows = [], []
    for b in range(nb):
        pps[b + 1] = PrePrepare(0, 0, b + 1, 1700000000 + b, 1, 'S', 'T', 'P' * 44)
        audit[b + 1] = audit_txn({1: 'SA%041d' % b, 2: 'SB%041d' % b}, {1: 'TA%041d' % b, 2: 'TB%041d' % b})
        for lid, sr, tr in ((1, 'SA%041d' % b, 'TA%041d' % b), (2, 'SB%041d' % b, 'TB%041d' % b)):
            msgs.append(MultiSignatureValue(lid, sr, 'P' * 44, tr, 1700000000 + b).as_single_value())
    blob, off = nat.pack_messages(msgs)
    midx = np.repeat(np.arange(2 * nb, dtype=np.uint32), nn)
    kidx = np.tile(np.arange(nn, dtype=np.uint32), 2 * nb)
    sig = nat.bls_sign_arrays(sks, blob, off, midx, kidx).reshape(2 * nb, nn, 128)
    rng = np.random.default_rng(7)
    commits, bad = [], []
    for b in range(nb):
        for i in range(nn):
            s1, s2 = sig[2 * b, i], sig[2 * b + 1, i]
            wrong = rng.random() < 1 / 6
            if wrong:
                s2 = sig[2 * b + 1, (i + 1) % nn]
            commits.append((Commit(0, 0, b + 1, {'1': _s(s1), '2': _s(s2)}), 'Node%d:0' % i))
            bad.append(wrong)
    rep = FakeBlsReplica(v, keys, audit, MultiSignatureValue)
    ing = CommitIngress(v, replica_commit_items(rep, lambda view, seq: pps.get(seq)))
    before = v.gpu_calls
    results = []
    ing.service(commits, lambda c, s: results.append(rep.validate_commit(c, s, pps[c.ppSeqNo])))
    assert v.gpu_calls - before == 1
    assert ing.last_pass['checks'] == 2 * nn * nb
    assert results == [2 if w else None for w in bad]
    assert 0 < sum(bad) < len(bad)
    # without the seam every COMMIT's check is its own GPU call
    before = v.gpu_calls
    for c, s in commits[:3]:
        rep.validate_commit(c, s, pps[c.ppSeqNo])
    assert v.gpu_calls - before == 6


def test_key_set_grows_one_key_at_a_time(pool, nat):
    """VERDICT r4 item 7 / ADVICE r4: the device key set is keyed by content and
    grows incrementally.  25 node keys met one at a time through verify_sig (the
    COMMIT path) cost one k_bls_lines point each (pv_bls_add_keys), a second
    verifier of the same generator re-prepares nothing, and proofs of possession
    of 25 further keys (node_handler.py:207-213) run against per-call key sets:
    the persistent set does not grow."""
    from plenum_gpu.bls import ProofOfPossession, VerKey
    nat.bls_set_keys(pool['gb'], np.zeros((0, 128), np.uint8))
    n0, p0 = nat.bls_keyset_info()
    assert n0 == 0
    v, v2 = _verifier(), _verifier()
    for i in range(pool['nn']):
        key = VerKey(pool['pks'][i].tobytes())
        assert v.verify_sig(_s(pool['sig'][i % pool['nm'], i]), pool['msgs'][i % pool['nm']], key) is True
        assert nat.bls_keyset_info() == (i + 1, p0 + i + 1)
        # the same key again, from either verifier: no preparation
        assert v2.verify_sig(_s(pool['sig'][i % pool['nm'], i]), pool['msgs'][i % pool['nm']], key) is True
        assert v.verify_sig(_s(pool['sig'][i % pool['nm'], i]), pool['msgs'][(i + 1) % pool['nm']], key) is False
        assert nat.bls_keyset_info() == (i + 1, p0 + i + 1)
    # 25 new keys' proofs of possession: per-call sets, the device set unchanged
    sks = np.frombuffer(b''.join((int.from_bytes(hashlib.sha256(b'pop' + bytes([i])).digest(), 'big') % bn.R)
                                 .to_bytes(32, 'big') for i in range(25)), np.uint8).reshape(25, 32)
    pks = nat.bls_pubkeys(pool['gb'], sks)
    blob, off = nat.pack_messages([pks[i].tobytes() for i in range(25)])
    idx = np.arange(25, dtype=np.uint32)
    pops = nat.bls_sign_arrays(sks, blob, off, idx, idx)
    for i in range(25):
        assert v.verify_key_proof_of_possession(ProofOfPossession(pops[i].tobytes()), VerKey(pks[i].tobytes())) is True
        assert v.verify_key_proof_of_possession(ProofOfPossession(pops[(i + 1) % 25].tobytes()),
                                                VerKey(pks[i].tobytes())) is False
    assert nat.bls_keyset_info() == (pool['nn'], p0 + pool['nn'])
    items = [(ProofOfPossession(pops[i].tobytes()), VerKey(pks[(i * 7) % 25].tobytes())) for i in range(25)]
    assert list(v.verify_key_proofs_batch(items)) == [(i * 7) % 25 == i for i in range(25)]
    # a set for another generator replaces this one (content, not owner, decides)
    gq = bytes(nat.bls_pubkeys(pool['gb'], sks[:1])[0])
    nat.bls_key_indices(gq, [pool['pks'][0].tobytes()])
    assert nat.bls_keyset_info()[0] == 1
    key0 = VerKey(pool['pks'][0].tobytes())
    assert v.verify_sig(_s(pool['sig'][0, 0]), pool['msgs'][0], key0) is True
    assert nat.bls_keyset_info()[0] == 1

