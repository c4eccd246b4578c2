"""Quorum sizes (plenum/server/quorums.py:4-39, plenum/common/util.py:220-232)."""
from math import floor


def getMaxFailures(nodeCount: int) -> int:
    """f = floor((n - 1) / 3) for n >= 4, else 0."""
    return int(floor((nodeCount - 1) / 3)) if nodeCount >= 4 else 0


class Quorum:
    def __init__(self, value: int):
        self.value = value

    def is_reached(self, msg_count: int) -> bool:
        return msg_count >= self.value

    def __repr__(self):
        return '{}({!r})'.format(self.__class__.__name__, self.value)


class Quorums:
    def __init__(self, n):
        f = getMaxFailures(n)
        self.n = n
        self.f = f
        strong, weak = n - f, f + 1
        self.weak = Quorum(weak)
        self.strong = Quorum(strong)
        self.propagate = Quorum(weak)
        self.prepare = Quorum(strong - 1)
        self.commit = Quorum(strong)
        self.reply = Quorum(weak)
        self.view_change = Quorum(strong)
        self.election = Quorum(strong)
        self.view_change_ack = Quorum(strong - 1)
        self.view_change_done = Quorum(strong)
        self.same_consistency_proof = Quorum(weak)
        self.consistency_proof = Quorum(weak)
        self.ledger_status = Quorum(strong - 1)
        self.ledger_status_last_3PC = Quorum(weak)
        self.checkpoint = Quorum(strong - 1)
        self.timestamp = Quorum(weak)
        self.bls_signatures = Quorum(strong)
        self.observer_data = Quorum(weak)
        self.backup_instance_faulty = Quorum(weak)

    def __str__(self):
        return '{}'.format(self.__dict__)
