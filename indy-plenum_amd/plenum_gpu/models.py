"""3PC vote tracking (plenum/server/models.py:16-114) and the batch quorum tally.

TrackedMsgs / Prepares / Commits keep the reference's voter-SET semantics: a
duplicate sender counts once, and a quorum of q is reached iff the set has at
least q members (`_has_enough_votes`, :41-45).  `tally_batches` evaluates that
predicate for many 3PC batches at once on the GPU (k_tally: one wavefront per
batch ORs the valid senders' bits into the voter set and pop-counts it).

Quorum values come from Quorums(n): COMMIT n-f, PREPARE n-f-1
(plenum/server/quorums.py:23-24).
"""
from collections import namedtuple

import numpy as np

from . import _native

ThreePhaseVotes = namedtuple('ThreePhaseVotes', ['voters', 'msg'])


class TrackedMsgs(dict):
    def _get_key(self, msg):
        raise NotImplementedError

    def _new_vote_msg(self, msg):
        return ThreePhaseVotes(voters=set(), msg=msg)

    def _add_msg(self, msg, voter: str):
        key = self._get_key(msg)
        if key not in self:
            self[key] = self._new_vote_msg(msg)
        self[key].voters.add(voter)

    def _has_msg(self, msg) -> bool:
        return self._get_key(msg) in self

    def _has_vote(self, msg, voter: str) -> bool:
        entry = self.get(self._get_key(msg))
        return entry is not None and voter in entry.voters

    def _votes_count(self, msg) -> int:
        entry = self.get(self._get_key(msg))
        return 0 if entry is None else len(entry.voters)

    def _has_enough_votes(self, msg, count) -> bool:
        return self._votes_count(msg) >= count


class Prepares(TrackedMsgs):
    """(viewNo, ppSeqNo) -> voters"""

    def _get_key(self, prepare):
        return prepare.viewNo, prepare.ppSeqNo

    def addVote(self, prepare, voter: str) -> None:
        self._add_msg(prepare, voter)

    def hasPrepare(self, prepare) -> bool:
        return self._has_msg(prepare)

    def hasPrepareFrom(self, prepare, voter: str) -> bool:
        return self._has_vote(prepare, voter)

    def hasQuorum(self, prepare, quorum: int) -> bool:
        return self._has_enough_votes(prepare, quorum)


class Commits(TrackedMsgs):
    """(viewNo, ppSeqNo) -> voters"""

    def _get_key(self, commit):
        return commit.viewNo, commit.ppSeqNo

    def addVote(self, commit, voter: str) -> None:
        self._add_msg(commit, voter)

    def hasCommit(self, commit) -> bool:
        return self._has_msg(commit)

    def hasCommitFrom(self, commit, voter: str) -> bool:
        return self._has_vote(commit, voter)

    def hasQuorum(self, commit, quorum: int) -> bool:
        return self._has_enough_votes(commit, quorum)


def tally_batches(verdict, sender, batch_off, n_nodes, quorum):
    """GPU quorum tally.

    verdict   (m,) bool/u8   the vote of message k counts (signature valid)
    sender    (m,) int       node index of message k's sender (< n_nodes)
    batch_off (b+1,) int     messages of batch j are batch_off[j]:batch_off[j+1]
    -> votes (b,) u32 distinct valid senders, reached (b,) bool votes >= quorum
    """
    return _native.tally_arrays(np.asarray(verdict, np.uint8), np.asarray(sender, np.uint32),
                                np.asarray(batch_off, np.uint64), int(n_nodes), int(quorum))


def propagate_quorums(req_keys, senders, verdict, n_nodes, node_index=None):
    """PROPAGATE f+1 quorum per request (row f4): ReqState.req_with_acceptable_quorum
    (plenum/server/propagator.py:36-44) over many requests at once with the same
    GPU tally as COMMITs — one vote per distinct sender whose PROPAGATE carried a
    valid request signature, reached iff votes >= Quorums(n).propagate (f + 1).

    req_keys (m,) request key of each PROPAGATE, senders (m,) node names (or
    indices), verdict (m,) bool.  Returns {key: (votes, reached)} in first-seen order.
    """
    from .quorums import Quorums
    order, groups = [], {}
    for k, key in enumerate(req_keys):
        if key not in groups:
            groups[key] = []
            order.append(key)
        groups[key].append(k)
    names = dict(node_index or {})
    idx = []
    for s in senders:
        if isinstance(s, (int, np.integer)):
            idx.append(int(s))
        else:
            if s not in names:
                names[s] = len(names)
            idx.append(names[s])
    flat, off = [], [0]
    for key in order:
        flat.extend(groups[key])
        off.append(len(flat))
    flat = np.asarray(flat, np.int64)
    sender = np.asarray(idx, np.uint32)[flat] if len(flat) else np.zeros(0, np.uint32)
    ver = np.asarray(verdict, bool)[flat] if len(flat) else np.zeros(0, bool)
    votes, reached = tally_batches(ver, sender, np.asarray(off, np.uint64), max(n_nodes, len(names)),
                                   Quorums(n_nodes).propagate.value)
    return {key: (int(votes[j]), bool(reached[j])) for j, key in enumerate(order)}
