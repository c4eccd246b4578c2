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


PropagateQuorum = namedtuple('PropagateQuorum', ['votes', 'reached', 'finalised_by', 'event'])


def propagate_groups(req_keys, senders, verdict):
    """Host half of `propagate_quorums`: the layout of the reference Requests
    store (plenum/server/propagator.py:20-46, 111-134) after a stream of
    PROPAGATEs, as tally input.

    A PROPAGATE enters the store only when its request's signature verified
    (Node.validateNodeMsg -> verifySignature, node.py:2624-2655): `verdict`
    False drops it.  `Requests.add_propagate` keys the store by request key and
    keeps ONE entry per sender (`propagates[sender] = req`: a re-sent PROPAGATE
    replaces the copy, never adds a vote, and keeps the sender's first position).
    `req_with_acceptable_quorum` counts only `str` senders (the reference's
    workaround for byte-named senders); every other sender is stored but never
    counted.  All copies under one key share one digest (key == digest,
    request.py:82-84), so the count is the number of distinct str senders.

    Returns (order, batch_off, sender_idx, counts, names, first): `order` the
    keys in the order their first accepted PROPAGATE arrived; batch j =
    [batch_off[j], batch_off[j+1]) of the flat (sender_idx, counts) arrays, one
    entry per (key, sender) in first-arrival order (counts 0 for non-str
    senders); names[i] the str sender of index i; first[k] the last accepted
    event index of flat entry k (the copy the store holds).
    """
    names, index = [], {}
    groups = {}            # key -> {sender: flat position} (dict: insertion order)
    latest = {}            # (key, sender) -> last accepted event index
    for ev, (key, snd, ok) in enumerate(zip(req_keys, senders, verdict)):
        if not ok:
            continue
        g = groups.setdefault(key, {})
        g.setdefault(snd, None)
        latest[(key, snd)] = ev
    order = list(groups)
    off = [0]
    sender_idx, counts, last = [], [], []
    for key in order:
        for snd in groups[key]:
            counted = isinstance(snd, str)
            if counted and snd not in index:
                index[snd] = len(names)
                names.append(snd)
            sender_idx.append(index[snd] if counted else 0)
            counts.append(1 if counted else 0)
            last.append(latest[(key, snd)])
        off.append(len(sender_idx))
    return (order, np.asarray(off, np.uint64), np.asarray(sender_idx, np.uint32), np.asarray(counts, np.uint8),
            names, np.asarray(last, np.int64))


def propagate_quorums(req_keys, senders, verdict, n_nodes):
    """PROPAGATE f+1 quorum per request (row f4) for a whole stream of
    PROPAGATEs at once: `Requests.add_propagate` for every PROPAGATE whose
    request signature verified, then `req_with_acceptable_quorum(
    Quorums(n_nodes).propagate)` per request (plenum/server/propagator.py:38-46,
    111-134), with the voter sets counted by the GPU tally (k_tally).

    req_keys (m,) request key of each PROPAGATE in arrival order, senders (m,)
    sender names (non-str names are stored but never counted, as in the
    reference), verdict (m,) bool signature verdicts.  Returns
    {key: PropagateQuorum(votes, reached, finalised_by, event)} in the store's
    order: votes = distinct str senders, reached = votes >= f + 1,
    finalised_by = the str sender whose copy req_with_acceptable_quorum returns
    (the (f+1)-th distinct str sender in arrival order; None if not reached),
    event = index of that copy's PROPAGATE in the stream.
    """
    from .quorums import Quorums
    if not (len(req_keys) == len(senders) == len(verdict)):
        raise ValueError('req_keys, senders and verdict must have one entry per PROPAGATE')
    order, off, sender_idx, counts, names, last = propagate_groups(req_keys, senders, verdict)
    q = Quorums(n_nodes).propagate.value
    if not order:
        return {}
    if len(names) > 1024:
        raise ValueError('at most 1024 distinct senders per stream (got {})'.format(len(names)))
    votes, reached = tally_batches(counts, sender_idx, off, max(1, len(names)), q)
    out = {}
    for j, key in enumerate(order):
        by, ev = None, None
        if reached[j]:
            seen = 0
            for k in range(int(off[j]), int(off[j + 1])):
                seen += int(counts[k])
                if seen == q:
                    by, ev = names[int(sender_idx[k])], int(last[k])
                    break
        out[key] = PropagateQuorum(int(votes[j]), bool(reached[j]), by, ev)
    return out
