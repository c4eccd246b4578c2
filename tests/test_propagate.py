"""Row f4 host logic: the Requests-store layout `propagate_groups` builds from a
PROPAGATE stream reproduces the reference store (plenum/server/propagator.py:
20-46, 111-134) on the reference-generated fixture, with the fixture's own
signature verdicts (ReqAuthenticator in the reference).  The GPU tally over
these groups is tests/test_gpu_tally.py::test_propagate_fixture_gpu."""
import numpy as np

import _propagate_cases as pc


def test_fixture_shape():
    fx = pc.load()
    kinds = {c['kind'] for c in fx['cases']}
    assert kinds == {'valid', 'tampered', 'resigned'}
    assert not all(c['valid'] for c in fx['cases'])
    assert any(isinstance(s, dict) for st in fx['streams'] for s, _ in st['events'])
    assert any(o['reached'] for st in fx['streams'] for o in st['outcome'].values())
    assert any(not o['reached'] for st in fx['streams'] for o in st['outcome'].values())


def test_groups_match_reference_store():
    from plenum_gpu.models import propagate_groups
    fx = pc.load()
    valid = [c['valid'] for c in fx['cases']]
    for st in fx['streams']:
        keys, senders, verdict = pc.stream_arrays(fx, st, valid)
        order, off, sidx, counts, names, last = propagate_groups(keys, senders, verdict)
        assert order == st['order']
        q = st['quorum']
        for j, key in enumerate(order):
            want = st['outcome'][key]
            a, b = int(off[j]), int(off[j + 1])
            assert b - a == want['votes']                       # Requests.votes: every sender
            assert int(counts[a:b].sum()) == want['str_votes']  # the digest group's count
            assert (want['str_votes'] >= q) == want['reached']
            if want['reached']:
                run = np.cumsum(counts[a:b])
                k = a + int(np.searchsorted(run, q))
                assert names[int(sidx[k])] == want['finalised_by']
                ev = int(last[k])
                assert st['events'][ev][0] == want['finalised_by'] and fx['cases'][st['events'][ev][1]]['key'] == key
