"""Batched ingestion on the GPU: one verify pass per service pass, then the
unchanged per-message authenticate(req, key) sees exactly the reference
ReqAuthenticator outcomes of the golden fixture (generated from the reference)."""
import pytest

import _ingress_cases as ic

pytestmark = pytest.mark.gpu


def test_service_pass_outcomes_and_one_gpu_pass(monkeypatch):
    from plenum_gpu import nacl_wrappers
    from plenum_gpu.ingress import BatchIngress, request_key
    fx = ic.load()
    ra = ic.make_ra(fx)
    ing = BatchIngress(ra)
    calls = []
    real = nacl_wrappers.verify_signed_batch

    def counting(items):
        calls.append(len(items))
        return real(items)
    monkeypatch.setattr(nacl_wrappers, 'verify_signed_batch', counting)
    client, node = ic.service_pass(fx)

    seen = []

    def handler(wrapped):   # the node's per-message path: verifySignature -> authenticate(req, key)
        msg, _ = wrapped
        for req in ing.requests_in(msg, from_node=False):
            try:
                seen.append((request_key(req), ic.outcome(ra.authenticate(req, key=request_key(req)))))
            except Exception as ex:  # noqa: BLE001
                seen.append((request_key(req), ic.outcome(ex)))
    assert ing.service(client, handler) == len(client)
    # one GPU pass for the whole client pass (tampered/unknown ones re-run per message)
    assert calls[0] == sum(len(c['req'].get('signatures') or {'x': 1}) for c in fx['cases']
                           if c['kind'] != 'unknown')
    want = {c['key']: c['reqauth'] for c in fx['cases']}
    assert len(seen) == len(fx['cases'])
    for key, got in seen:
        assert got == want[key]
    # the per-message authenticate calls (not the pre-pass) cached the accepted ones
    accepted = [c for c in fx['cases'] if 'result' in c['reqauth']]
    assert all(c['key'] in ra._verified_reqs for c in accepted)
    assert len(ra._verified_reqs) == len({c['key'] for c in accepted})
    # node pass: every PROPAGATEd request is already verified -> no new GPU work
    n_calls = len(calls)
    ing.prefetch(node, from_node=True)
    ing.end_pass()
    assert ing.last_pass['distinct'] == len({c['key'] for c in fx['cases'][::3]})
    assert sum(calls[n_calls:]) <= sum(1 for c in fx['cases'][::3] if 'result' not in c['reqauth']) * 2


def test_fresh_node_pass_verifies_propagates_once(monkeypatch):
    from plenum_gpu import nacl_wrappers
    from plenum_gpu.ingress import BatchIngress
    fx = ic.load()
    ra = ic.make_ra(fx)
    ing = BatchIngress(ra)
    calls = []
    real = nacl_wrappers.verify_signed_batch

    def counting(items):
        calls.append(len(items))
        return real(items)
    monkeypatch.setattr(nacl_wrappers, 'verify_signed_batch', counting)
    _, node = ic.service_pass(fx)
    reqs, keys = ing.prefetch(node, from_node=True)
    assert not ra._verified_reqs          # the pre-pass authenticates nothing
    assert len(calls) == 1
    by_key = {c['key']: c['reqauth'] for c in fx['cases']}
    for req, key in zip(reqs, keys):
        try:
            got = ic.outcome(ra.authenticate(req, key=key))
        except Exception as ex:  # noqa: BLE001
            got = ic.outcome(ex)
        assert got == by_key[key]
    # accepted requests were served from the prefetched verdicts: only the
    # rejected ones (whose verdict the replay consumed too) cost nothing more
    assert len(calls) == 1
    ing.end_pass()


def test_dropped_request_leaves_no_cache_entry():
    """A validly signed request the node drops before verifySignature (blacklist,
    static validation: node.py:1625-1657) is never cached."""
    from plenum_gpu.ingress import BatchIngress
    fx = ic.load()
    ra = ic.make_ra(fx)
    ing = BatchIngress(ra)
    client, _ = ic.service_pass(fx)
    assert ing.service(client, lambda w: None) == len(client)
    assert ra._verified_reqs == {}
    assert all(not a._verdicts()._d for a in ra._authenticators)
