"""Host-side mirror of the reference interfaces: data formats (base58,
signing serializer), key resolution, quorum sizes and the full
CoreAuthNr / ReqAuthenticator control flow against the golden fixture.

On CPU the GPU verdict source is replaced by the oracle (a test double for
this control-flow test only; the same fixture runs through the real HIP path
in tests/test_gpu_plenum.py)."""
import os

import numpy as np
import pytest

import _oracle as orc
import _plenum_cases as pc
from plenum_gpu import base58
from plenum_gpu.exceptions import InvalidKey
from plenum_gpu.quorums import Quorums, getMaxFailures
from plenum_gpu.serialization import serialize_msg_for_signing
from plenum_gpu.verifier import DidVerifier


def test_base58_roundtrip_and_edges():
    for raw in [b'', b'\0', b'\0\0\x01', os.urandom(32), os.urandom(16), b'\xff' * 64]:
        enc = base58.b58encode(raw)
        assert base58.b58decode(enc) == raw
        assert base58.b58decode(enc.decode() + '  \n') == raw
    assert base58.b58encode(b'\0\0ab') .startswith(b'11')
    for bad in ['0abc', 'Oops', 'Il', 'ab+c']:
        with pytest.raises(ValueError):
            base58.b58decode(bad)


def test_base58_matches_shim_semantics():
    import importlib.util
    spec = importlib.util.spec_from_file_location('shim_b58', os.path.join(os.path.dirname(__file__), '..', 'oracle',
                                                                            'shims', 'base58.py'))
    shim = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(shim)
    rng = np.random.default_rng(1)
    for _ in range(200):
        raw = bytes(rng.integers(0, 3, int(rng.integers(0, 40)), dtype=np.uint8))
        assert base58.b58encode(raw) == shim.b58encode(raw)
        assert base58.b58decode(shim.b58encode(raw)) == shim.b58decode(shim.b58encode(raw))


def test_serializer_kats(kat):
    for case in kat['serializer']:
        assert serialize_msg_for_signing(case['in']).decode() == case['out']
    for case in kat['serializer_ignore']:
        assert serialize_msg_for_signing(case['in'], topLevelKeysToIgnore=case['ignore']).decode() == case['out']


def test_serializer_rejects_unacceptable_types():
    with pytest.raises(Exception, match='invalid type found'):
        serialize_msg_for_signing({'a': (1, 2)})


def test_didverifier_kats(kat):
    """plenum/test/common/test_verifier.py:6-28"""
    k = kat['did_abbrev']
    assert DidVerifier(k['verkey'], identifier=k['identifier']).verkey == k['expected']
    for vk in (None, ''):
        with pytest.raises(ValueError) as ei:
            DidVerifier(vk, identifier=k['identifier'])
        assert str(ei.value) == "'verkey' should be a non-empty string"
    odd = kat['did_odd']
    with pytest.raises(InvalidKey) as ei:
        DidVerifier(odd['verkey'])
    assert type(ei.value).__name__ == odd['exc'] and str(ei.value) == odd['str']


def test_quorums_kat(kat):
    for q in kat['quorums']:
        Q = Quorums(q['n'])
        assert (Q.f, Q.commit.value, Q.prepare.value, Q.propagate.value, Q.weak.value, Q.strong.value) == \
            (q['f'], q['commit'], q['prepare'], q['propagate'], q['weak'], q['strong'])
        assert getMaxFailures(q['n']) == q['f']
    assert Quorums(25).commit.value == 17 and Quorums(25).prepare.value == 16


@pytest.fixture
def oracle_backend(monkeypatch):
    """Test double: GPU verdict source -> oracle (CPU control-flow test only)."""
    from plenum_gpu import nacl_wrappers

    def fake(items):
        out = np.zeros(len(items), dtype=bool)
        for k, (pk, sm) in enumerate(items):
            out[k] = orc.sign_open(bytes(sm), bytes(pk))
        return out
    monkeypatch.setattr(nacl_wrappers, 'verify_signed_batch', fake)
    return fake


def test_plenum_requests_per_request(plenum_requests, oracle_backend):
    bad = pc.check_per_request(plenum_requests)
    assert not bad, bad[:5]


def test_plenum_requests_batched(plenum_requests, oracle_backend):
    bad = pc.check_batched(plenum_requests)
    assert not bad, bad[:5]


def test_fixture_covers_every_outcome(plenum_requests):
    kinds = {c['core'].get('exc', 'ok') for c in plenum_requests['cases']}
    assert {'ok', 'InsufficientCorrectSignatures', 'InvalidSignatureFormat', 'CouldNotAuthenticate',
            'InvalidKey', 'InsufficientSignatures', 'MissingSignature'} <= kinds


def test_batched_replay_respects_overrides(plenum_requests, oracle_backend):
    """authenticate_batch's replay reuses the prefetch's per-request values only
    for the stock entry points: a subclass overriding authenticate keeps its
    own per-request path (every request goes through the override), with the
    same outcomes as the stock class on the golden fixture."""
    import copy
    from plenum_gpu.client_authn import CoreAuthNr
    fx = plenum_requests

    class Counting(CoreAuthNr):
        calls = 0

        def authenticate(self, req_data, *a, **kw):
            Counting.calls += 1
            return super().authenticate(req_data, *a, **kw)

    stock = CoreAuthNr(fx['write_types'], fx['query_types'], fx['action_types'], state=pc.DictState(fx['state_nyms']))
    sub = Counting(fx['write_types'], fx['query_types'], fx['action_types'], state=pc.DictState(fx['state_nyms']))
    for idr, vk in fx['registry'].items():
        stock.addIdr(idr, vk)
        sub.addIdr(idr, vk)
    assert stock._replay_reuses_prefetch() and not sub._replay_reuses_prefetch()
    reqs = [copy.deepcopy(c['req']) for c in fx['cases'] if c.get('threshold') is None]
    a = [pc.outcome_core(x) for x in stock.authenticate_batch(copy.deepcopy(reqs))]
    b = [pc.outcome_core(x) for x in sub.authenticate_batch(copy.deepcopy(reqs))]
    assert a == b and Counting.calls == len(reqs)
