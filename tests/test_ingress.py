"""Batched ingestion (plenum_gpu/ingress.py) on CPU: request
keys equal the reference's Request.key (golden fixture from the reference code),
and a service pass collects exactly the requests verifySignature would
authenticate, once each."""
import _ingress_cases as ic


def test_request_key_matches_reference():
    from plenum_gpu.ingress import request_key
    fx = ic.load()
    for c in fx['cases']:
        assert request_key(c['req']) == c['key'], c['kind']


def test_requests_in_messages():
    from plenum_gpu.ingress import BatchIngress, is_client_request
    fx = ic.load()
    ing = BatchIngress(ra := ic.make_ra(fx))
    assert ra is ing.authenticator
    for c in fx['cases']:
        assert is_client_request(c['req'])
        assert ing.requests_in(c['req'], from_node=False) == [c['req']]
        assert ing.requests_in(c['req'], from_node=True) == []   # node stack: only PROPAGATE carries requests
    for p in fx['propagates']:
        assert ing.requests_in(p, from_node=True) == [p['request']]
        assert ing.requests_in(p, from_node=False) == []
    for b in fx['batches']:
        got = ing.requests_in(b, from_node=True)
        assert len(got) == len(b['messages'])
    bad = {'op': 'BATCH', 'messages': ['{not json', '{"op": "PROPAGATE", "request": {"reqId": 1}}'],
           'signature': None}
    assert ing.requests_in(bad, from_node=True) == [{'reqId': 1}]
    assert ing.requests_in({'op': 'LEDGER_STATUS'}, from_node=False) == []


def test_collect_dedups_by_request_key():
    from plenum_gpu.ingress import BatchIngress
    fx = ic.load()
    ing = BatchIngress(ic.make_ra(fx))
    client, node = ic.service_pass(fx)
    reqs, keys = ing.collect(client + [(m, f) for m, f in node if m.get('op') == 'PROPAGATE'], from_node=False)
    assert len(reqs) == len(fx['cases'])       # PROPAGATEs are not client-stack requests
    reqs, keys = ing.collect(node, from_node=True)
    distinct = {c['key'] for c in fx['cases'][::3]}
    assert set(keys) == distinct and len(keys) == len(distinct)
    assert ing.last_pass['requests'] == len(fx['propagates']) + sum(len(b['messages']) for b in fx['batches'])


def test_prefetch_never_caches_unauthenticated(monkeypatch):
    """Host logic of the pre-pass: prefetch only fills verdict
    caches; `_verified_reqs` is written by the per-message authenticate alone,
    and a pass's unconsumed verdicts are dropped at its end.  The verifier is
    stubbed (all accepted) — this checks cache bookkeeping, not verdicts."""
    import numpy as np
    from plenum_gpu import nacl_wrappers
    from plenum_gpu.ingress import BatchIngress, request_key
    fx = ic.load()
    ra = ic.make_ra(fx)
    ing = BatchIngress(ra)
    calls = []

    def stub(items):
        calls.append(len(items))
        return np.ones(len(items), bool)
    monkeypatch.setattr(nacl_wrappers, 'verify_signed_batch', stub)
    client, _ = ic.service_pass(fx)
    # every handler drops its message before verifySignature
    ing.service(client, lambda w: None)
    assert len(calls) == 1 and calls[0] > 0
    assert ra._verified_reqs == {}
    assert all(not a._verdicts()._d for a in ra._authenticators)
    # a handler that authenticates one request caches exactly that one
    first = fx['cases'][0]['req']

    def one(w):
        if w[0] is client[0][0]:
            ra.authenticate(w[0], key=request_key(w[0]))
    ing.service(client, one)
    assert list(ra._verified_reqs) == [request_key(first)]
    assert len(calls) == 2          # served from the pass's prefetched verdicts
