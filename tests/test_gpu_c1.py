"""C1 at its full 10k-request size (BASELINE configs[0]):
CoreAuthNr.authenticate_batch over synth.c1_requests(10000) gives, per request,
exactly what the per-request CoreAuthNr.authenticate replay gives -- identifier
lists for valid requests, the same exception class and text for the tampered
ones (plenum/server/client_authn.py:230-266 via the a3 loop :84-118)."""
import pytest

pytestmark = pytest.mark.gpu


def _outcome(x):
    if isinstance(x, Exception):
        return (type(x).__name__, str(x))
    return ('ok', list(x))


def test_c1_10k_batch_equals_per_request():
    from plenum_gpu import synth
    from plenum_gpu.client_authn import CoreAuthNr
    n = 10_000
    reqs, ids = synth.c1_requests(n)
    authnr = CoreAuthNr(['buy'], [], [])
    unknown = set()
    for k, (idr, vk) in enumerate(ids):
        if k % 997 != 5:            # a few identifiers stay unknown (no state: the lookup raises)
            authnr.addIdr(idr, vk)
        else:
            unknown.add(k)
    for k in range(0, n, 41):       # ~2.4 %: payload changed after signing
        reqs[k]['reqId'] += 1
    for k in range(7, n, 173):      # a non-base58 character in the signature
        reqs[k]['signature'] = '0' + reqs[k]['signature'][1:]
    for k in range(11, n, 211):     # a truncated signature (decoded length != 64)
        reqs[k]['signature'] = reqs[k]['signature'][:-3]
    batch = authnr.authenticate_batch(reqs)
    single = []
    for r in reqs:
        try:
            single.append(authnr.authenticate(r))
        except Exception as ex:  # noqa: BLE001 -- the outcome is what is compared
            single.append(ex)
    got = [_outcome(x) for x in batch]
    want = [_outcome(x) for x in single]
    bad = [k for k in range(n) if got[k] != want[k]]
    assert not bad, [(k, got[k], want[k]) for k in bad[:5]]
    # addIdr put the DIDs' keys in the device key cache, so both runs above took
    # the keyed latency kernel; without the cache the generic kernels agree too
    from plenum_gpu import _native as nat
    assert nat.keycache_size() > 0.9 * n
    nat.keycache_clear()
    uncached = [_outcome(x) for x in authnr.authenticate_batch(reqs)]
    bad = [k for k in range(n) if uncached[k] != want[k]]
    assert not bad, [(k, uncached[k], want[k]) for k in bad[:5]]
    kinds = {w[0] for w in want}
    assert {'ok', 'InsufficientCorrectSignatures', 'InvalidSignatureFormat'} <= kinds, kinds
    assert all(want[k][0] != 'ok' for k in unknown)
    assert sum(w[0] == 'ok' for w in want) > 0.9 * n
