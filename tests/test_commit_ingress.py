"""COMMIT batch seam (plenum_gpu/commit_ingress.py), CPU only: which triples the
pre-pass collects for the reference's validate_commit walk, and that the
unchanged per-COMMIT path is then served from the prefetched verdicts (one
verifier pass per Looper pass).  The verifier here is a recording stand-in; the
GPU test (tests/test_gpu_bls_multi.py) runs the same seam on the kernels."""
from _commit_cases import STASH_VIEW_3PC, Commit, FakeBlsReplica, MiniStasher, PrePrepare, audit_txn

from plenum_gpu.bls import MultiSignatureValue
from plenum_gpu.commit_ingress import CommitIngress, replica_commit_items


class RecordingVerifier:
    """verify_sig answers 'good' signatures True; counts per-call and batched work"""

    def __init__(self):
        self.single, self.batches, self._pre = 0, [], {}

    def verify_sig(self, sig, msg, pk):
        if pk is not None:
            hit = self._pre.get((sig, bytes(msg), pk))
            if hit is not None:
                return hit
        self.single += 1
        return sig.startswith('good')

    def prefetch(self, items):
        todo = [(s, bytes(m), pk) for s, m, pk in items if pk is not None]
        self.batches.append(todo)
        for k in todo:
            self._pre[k] = k[0].startswith('good')
        return len(todo)

    def drop_prefetched(self):
        self._pre.clear()


def _pool(nn=4, nb=3):
    v = RecordingVerifier()
    keys = {'N%d' % i: 'pk%d' % i for i in range(nn)}
    audit = {b: audit_txn({1: 'S%d' % b, 2: 'X%d' % b}, {1: 'T%d' % b, 2: 'Y%d' % b}) for b in range(1, nb + 1)}
    rep = FakeBlsReplica(v, keys, audit, MultiSignatureValue)
    pps = {b: PrePrepare(0, 0, b, 1700000000 + b, 1, 'S', 'T', 'P' * 44) for b in range(1, nb + 1)}
    return v, rep, pps


def test_collect_follows_validate_commit_walk():
    v, rep, pps = _pool()
    items = replica_commit_items(rep, lambda view, seq: pps.get(seq))
    c = Commit(0, 0, 1, {'1': 'good-a', '2': 'good-b'})
    got = items(c, 'N1:0')
    assert [(s, pk) for s, _m, pk in got] == [('good-a', 'pk1'), ('good-b', 'pk1')]
    assert got[0][1] == MultiSignatureValue(1, 'S1', 'P' * 44, 'T1', 1700000001).as_single_value()
    assert items(Commit(0, 0, 1, None), 'N1:0') == []                 # no BLS_SIGS
    assert items(Commit(0, 0, 9, {'1': 'x'}), 'N1:0') == []           # no pre-prepare / audit txn
    assert [s for s, _m, _k in items(Commit(0, 0, 1, {'1': 'a', '5': 'b', '2': 'c'}), 'N0:0')] == ['a']
    assert items(Commit(0, 0, 1, {'1': 'a'}), 'N9:0') == []           # sender without a key


def test_pass_serves_per_commit_checks_from_one_prefetch():
    nn, nb = 4, 3
    v, rep, pps = _pool(nn, nb)
    ing = CommitIngress(v, replica_commit_items(rep, lambda view, seq: pps.get(seq)))
    commits = []
    for b in range(1, nb + 1):
        for i in range(nn):
            sig = ('bad' if (b + i) % 3 == 0 else 'good') + '-%d-%d' % (b, i)
            commits.append((Commit(0, 0, b, {'1': sig, '2': 'good-x%d' % i}), 'N%d:0' % i))
    results = []
    n = ing.service(commits, lambda c, s: results.append(rep.validate_commit(c, s, pps[c.ppSeqNo])))
    assert n == len(commits) and v.single == 0 and len(v.batches) == 1
    assert ing.last_pass == {'commits': nn * nb, 'checks': 2 * nn * nb, 'verified': 2 * nn * nb}
    assert results == [2 if c.blsSigs['1'].startswith('bad') else None for c, _s in commits]
    # after the pass the verdicts are gone: the same COMMIT goes to the verifier again
    rep.validate_commit(commits[0][0], commits[0][1], pps[1])
    assert v.single == 2


def test_pass_routes_commits_through_the_stasher():
    """in the reference process_commit is reached only through the
    ordering service's StashingRouter, which stashes a COMMIT whose handler
    returns (STASH_VIEW_3PC, reason).  With `stasher` the seam takes that route:
    the future-view COMMITs are stashed, not dropped, and replayed later -- then
    checked by their own verify_sig calls (the pass's verdicts are gone)."""
    nn, nb = 4, 3
    v, rep, pps = _pool(nn, nb)
    ing = CommitIngress(v, replica_commit_items(rep, lambda view, seq: pps.get(seq)))
    view = {'no': 0}
    results = []

    def process_commit(commit, sender):     # ordering_service.py:436-455, _validate -> STASH_VIEW_3PC
        if commit.viewNo > view['no']:
            return STASH_VIEW_3PC, 'future view'
        results.append((commit.ppSeqNo, sender, rep.validate_commit(commit, sender, pps[commit.ppSeqNo])))
        return None

    commits = [(Commit(0, b % 2, b, {'1': ('bad' if i == 1 else 'good') + '-%d-%d' % (b, i)}), 'N%d:0' % i)
               for b in range(1, nb + 1) for i in range(nn)]
    stasher = MiniStasher()
    assert ing.service(commits, process_commit, stasher=stasher) == len(commits)
    future = [c for c, _s in commits if c.viewNo == 1]
    assert len(stasher.stashed[STASH_VIEW_3PC]) == len(future) > 0
    assert ing.last_results == [c.viewNo == 0 for c, _s in commits]   # stasher._process: True = processed
    assert len(results) == len(commits) - len(future) and v.single == 0
    view['no'] = 1
    stasher.process_all_stashed()
    assert len(results) == len(commits) and v.single == len(future)
    assert sorted(results) == sorted((c.ppSeqNo, s, 2 if c.blsSigs['1'].startswith('bad') else None)
                                     for c, s in commits)

