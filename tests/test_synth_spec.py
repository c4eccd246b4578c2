"""Host restatement of the synthetic workloads (plenum_gpu/synth.py): the C3
COMMIT layout against the reference's voter-set semantics (our restated
plenum/server/models.py Commits), and the C4 length law.  CPU only."""
import numpy as np

from plenum_gpu import synth
from plenum_gpu.models import Commits
from plenum_gpu.quorums import Quorums


def test_commit_layout_votes_match_commits_voter_sets():
    n_nodes = 25
    q = Quorums(n_nodes).commit.value
    votes, reached = synth.c3_expected(0, 3000, n_nodes, q)

    class C:
        def __init__(self, b):
            self.viewNo, self.ppSeqNo = 0, b + 1
    commits = Commits()
    seen_dup = seen_fail = seen_ok = 0
    for b in range(3000):
        senders, bad = synth.c3_slots(b, n_nodes)
        c = C(b)
        for s in range(n_nodes):
            if not bad[s]:
                commits.addVote(c, 'Node%d' % (senders[s] + 1))
        assert votes[b] == commits._votes_count(c)
        assert reached[b] == commits.hasQuorum(c, q)
        seen_dup += int(len(set(senders.tolist())) < n_nodes)
        seen_fail += int(not reached[b])
        seen_ok += int(reached[b])
    # both quorum outcomes and the duplicate-sender case occur
    assert seen_dup > 5 and seen_fail > 100 and seen_ok > 100


def test_commit_messages_are_the_signing_serialization():
    from plenum_gpu.serialization import serialize_msg_for_signing
    for b in (0, 8, 9, 98, 99, 99999):
        m = serialize_msg_for_signing({'instId': 0, 'viewNo': 0, 'ppSeqNo': b + 1, 'op': 'COMMIT'})
        assert m == synth.commit_message(b + 1)
        assert len(m) == synth.msg_len(synth.COMMIT, 3, b * 25 + 7, 0, 0, 25)


def test_range_lengths_uniform_in_bounds():
    lens = np.array([synth.msg_len(synth.RANGE, 4, i, 128, 4096) for i in range(20000)])
    assert lens.min() >= 128 and lens.max() <= 4096
    assert abs(lens.mean() - 2112) < 40
