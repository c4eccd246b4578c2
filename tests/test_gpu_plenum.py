"""The golden Plenum request fixture (reference CoreAuthNr / ReqAuthenticator
over libsodium) through the plenum_gpu mirror on the REAL HIP path."""
import pytest

import _plenum_cases as pc

pytestmark = pytest.mark.gpu


def test_per_request(plenum_requests):
    bad = pc.check_per_request(plenum_requests)
    assert not bad, bad[:5]


def test_batched(plenum_requests):
    bad = pc.check_batched(plenum_requests)
    assert not bad, bad[:5]


def test_propagate_vector_kat(kat):
    from plenum_gpu.nacl_wrappers import verify_signed_batch
    items = [(bytes.fromhex(c['pk']), bytes.fromhex(c['sig']) + bytes.fromhex(c['M'])) for c in kat['propagate_vector']]
    assert list(verify_signed_batch(items)) == [c['verdict'] for c in kat['propagate_vector']]


def test_didverifier_verify_batch(kat):
    import os
    from plenum_gpu import base58
    from plenum_gpu.nacl_wrappers import SigningKey
    from plenum_gpu.verifier import DidVerifier
    sk = SigningKey(os.urandom(32))
    vk = base58.b58encode(bytes(sk.verify_key)).decode()
    v = DidVerifier(vk)
    msgs = [os.urandom(40) for _ in range(20)]
    sigs = [sk.sign(m).signature for m in msgs]
    pairs = [(s, m) for s, m in zip(sigs, msgs)]
    pairs[3] = (sigs[4], msgs[3])
    pairs[7] = (sigs[7][:63], msgs[7])
    got = v.verify_batch(pairs)
    assert list(got) == [k not in (3, 7) for k in range(20)]
    assert [v.verify(s, m) for s, m in pairs] == list(got)
