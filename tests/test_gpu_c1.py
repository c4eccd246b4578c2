"""C1 at its full 10k-request size (BASELINE configs[0]) against the REFERENCE:
CoreAuthNr.authenticate_batch over synth.c1_requests(10000) with the mutations
below gives, per request, what the reference CoreAuthNr(['buy'], [], []).authenticate
gave in this container (tests/golden/c1_10k.json, oracle/gen_golden.py gen_c1):
the same identifier lists for the accepted requests and the same exception class
and text for every rejected one (plenum/server/client_authn.py:230-266 via the a3
loop :84-118).  The requests regenerated here (GPU signer) are checked to be the
fixture's input byte for byte (digest of the request dicts)."""
import hashlib
import json

import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


def _digest(obj):
    return hashlib.sha256(json.dumps(obj, sort_keys=True, separators=(',', ':')).encode()).hexdigest()


def _mutate(reqs):
    """oracle/gen_golden.py c1_mutate, same order"""
    n = len(reqs)
    for k in range(0, n, 41):       # ~2.4 %: payload changed after signing
        reqs[k]['reqId'] += 1
    for k in range(7, n, 173):      # a non-base58 character in the signature
        reqs[k]['signature'] = '0' + reqs[k]['signature'][1:]
    for k in range(11, n, 211):     # a truncated signature (decoded length != 64)
        reqs[k]['signature'] = reqs[k]['signature'][:-3]
    return reqs


def _check(batch, fx):
    fails, ok = {}, []
    for k, x in enumerate(batch):
        if isinstance(x, Exception):
            fails[str(k)] = [type(x).__name__, str(x)]
        else:
            ok.append([k, list(x)])
    assert set(fails) == set(fx['failures']), sorted(set(fails) ^ set(fx['failures']))[:5]
    bad = [k for k in fails if fails[k] != fx['failures'][k]]
    assert not bad, [(k, fails[k], fx['failures'][k]) for k in bad[:3]]
    assert len(ok) == fx['ok_count'] and _digest(ok) == fx['ok_digest']


def test_c1_10k_matches_reference_outcomes():
    from plenum_gpu import _native as nat
    from plenum_gpu import synth
    from plenum_gpu.client_authn import CoreAuthNr
    with open(golden('c1_10k.json')) as fh:
        fx = json.load(fh)
    n = fx['n']
    reqs, ids = synth.c1_requests(n)
    assert _digest([list(i) for i in ids]) == fx['identities_digest']
    _mutate(reqs)
    assert _digest(reqs) == fx['requests_digest']
    authnr = CoreAuthNr(['buy'], [], [])
    for k, (idr, vk) in enumerate(ids):
        if k % 997 != 5:            # never registered (no state either): the reference's lookup raises
            authnr.addIdr(idr, vk)
    # addIdr put the DIDs' keys in the device key cache: the keyed latency kernel
    _check(authnr.authenticate_batch(reqs), fx)
    assert nat.keycache_size() > 0.9 * n
    # without the cache: the generic kernels
    nat.keycache_clear()
    _check(authnr.authenticate_batch(reqs), fx)
    kinds = {v[0] for v in fx['failures'].values()}
    assert {'InsufficientCorrectSignatures', 'InvalidSignatureFormat'} <= kinds, kinds
    assert fx['ok_count'] > 0.9 * n
