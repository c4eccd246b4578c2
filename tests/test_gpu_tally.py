"""Quorum tally kernel vs the reference voter-set semantics."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_tally_fixture(tally_fx):
    from plenum_gpu.models import tally_batches
    t = tally_fx
    votes, reached = tally_batches(t['verdict'], t['sender'], t['batch_off'], int(t['n_nodes']),
                                   int(t['commit_quorum']))
    assert (votes == t['vote_count']).all()
    assert (reached == t['commit_reached'].astype(bool)).all()
    _, reached_p = tally_batches(t['verdict'], t['sender'], t['batch_off'], int(t['n_nodes']),
                                 int(t['prepare_quorum']))
    assert (reached_p == t['prepare_reached'].astype(bool)).all()


@pytest.mark.parametrize('n_nodes', [4, 25, 64, 65, 200, 1024])
def test_tally_random_vs_sets(n_nodes):
    from plenum_gpu.models import Commits, tally_batches
    from plenum_gpu.quorums import Quorums
    rng = np.random.default_rng(n_nodes)
    nb = 700
    sizes = rng.integers(0, 2 * n_nodes + 3, nb)
    off = np.zeros(nb + 1, np.uint64)
    off[1:] = np.cumsum(sizes)
    m = int(off[-1])
    sender = rng.integers(0, n_nodes, m).astype(np.uint32)
    verdict = rng.random(m) < 0.8
    q = Quorums(n_nodes).commit.value
    votes, reached = tally_batches(verdict, sender, off, n_nodes, q)

    class C:
        def __init__(self, b):
            self.viewNo, self.ppSeqNo = 0, b
    commits = Commits()
    for b in range(nb):
        c = C(b)
        for k in range(int(off[b]), int(off[b + 1])):
            if verdict[k]:
                commits.addVote(c, 'Node%d' % sender[k])
        assert votes[b] == commits._votes_count(c)
        assert reached[b] == commits.hasQuorum(c, q)


def test_propagate_f_plus_1_quorums():
    """Row f4: PROPAGATE f+1 quorums per request through the GPU tally equal the
    reference ReqState.req_with_acceptable_quorum voter-set semantics."""
    from plenum_gpu.models import propagate_quorums
    from plenum_gpu.quorums import Quorums
    rng = np.random.default_rng(4)
    n_nodes = 25
    q = Quorums(n_nodes).propagate
    keys, senders, verdict = [], [], []
    for r in range(2000):
        for _ in range(int(rng.integers(0, 14))):
            keys.append('req%d' % r)
            senders.append('Node%d' % int(rng.integers(1, n_nodes + 1)))   # duplicates happen
            verdict.append(bool(rng.random() < 0.9))
    got = propagate_quorums(keys, senders, verdict, n_nodes)
    want = {}
    for k, s, v in zip(keys, senders, verdict):
        want.setdefault(k, set())
        if v:
            want[k].add(s)
    assert set(got) == set(want)
    for k, voters in want.items():
        assert got[k] == (len(voters), q.is_reached(len(voters))), k
