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
