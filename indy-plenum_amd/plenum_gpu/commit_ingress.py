"""COMMIT batch seam: the BLS checks of one Looper pass's COMMITs in one GPU pass
(VERDICT r3 "what's missing" 2).

The reference validates each COMMIT as it arrives:
  OrderingService.process_commit -> _validate_commit
    (plenum/server/consensus/ordering_service.py:434-488)
  -> BlsBftReplicaPlenum.validate_commit (plenum/bls/bls_bft_replica_plenum.py:55-75)
  -> _validate_signature (:194-213) -> bls_crypto_verifier.verify_sig(sig, msg, pk)
so a pass over n COMMITs makes n separate pairing checks — on the GPU one lone
check is one lane's ~2.2 M-MAD chain (~10 ms), the wrong shape for the device.

`CommitIngress` sits in front of the unchanged handlers, as `BatchIngress`
(plenum_gpu/ingress.py) does for client requests: it collects, for every COMMIT
of the pass, the (signature, message, key) triples `validate_commit` would check,
runs ONE `BlsCryptoVerifierGpu.prefetch` (one pv_bls_verify_batch call), and the
node's unchanged per-COMMIT path — `_validate_commit` -> `validate_commit` ->
`verify_sig` — answers from those verdicts.  The pre-pass decides nothing: which
COMMITs are checked, in what order, and what is reported stay the reference's;
verdicts no handler consumed are dropped at the end of the pass.
"""
from functools import partial
from typing import Callable, Iterable, List, Optional, Tuple

# plenum/common/constants.py:121-122,173,176; plenum/common/types.py:67
TXN_PAYLOAD = 'txn'
TXN_PAYLOAD_DATA = 'data'
AUDIT_TXN_STATE_ROOT = 'stateRoot'
AUDIT_TXN_LEDGER_ROOT = 'ledgerRoot'
BLS_SIGS = 'blsSigs'


def replica_commit_items(bls_replica, get_preprepare: Callable) -> Callable:
    """The triples `BlsBftReplicaPlenum.validate_commit(commit, sender, pre_prepare)`
    checks, computed with the replica's own helpers (bls_bft_replica_plenum.py:55-75,
    186-213) but without verifying: -> items(commit, sender) -> [(sig str,
    message bytes, pk)].  `get_preprepare(viewNo, ppSeqNo)` is the ordering
    service's (ordering_service.py:472).  The walk stops where validate_commit
    would return early (no BLS_SIGS, no audit txn, a ledger the audit txn does
    not cover, a sender without a key)."""
    cls = type(bls_replica)

    def items(commit, sender) -> List[tuple]:
        sigs = getattr(commit, BLS_SIGS, None)
        if sigs is None:
            return []
        pre_prepare = get_preprepare(commit.viewNo, commit.ppSeqNo)
        if pre_prepare is None:
            return []
        audit_txn = bls_replica._get_correct_audit_transaction(pre_prepare)
        if not audit_txn:
            return []
        payload = audit_txn[TXN_PAYLOAD][TXN_PAYLOAD_DATA]
        out = []
        for lid, sig in sigs.items():
            lid = int(lid)
            if lid not in payload[AUDIT_TXN_STATE_ROOT] or lid not in payload[AUDIT_TXN_LEDGER_ROOT]:
                break
            fake_pp = cls._create_fake_pre_prepare_for_multi_sig(lid, payload[AUDIT_TXN_STATE_ROOT][lid],
                                                                 payload[AUDIT_TXN_LEDGER_ROOT][lid], pre_prepare)
            pool_root_hash = bls_replica._get_pool_root_hash(fake_pp, serialize=False)
            pk = bls_replica._bls_bft.bls_key_register.get_key_by_name(bls_replica.get_node_name(sender),
                                                                       pool_root_hash)
            if not pk:
                break
            value = bls_replica._create_multi_sig_value_for_pre_prepare(fake_pp, bls_replica._get_pool_root_hash(fake_pp))
            out.append((sig, value.as_single_value(), pk))
        return out

    return items


class CommitIngress:
    """Pre-verify the BLS signatures of one pass's COMMITs in one GPU pass.

    verifier: the node's BlsCryptoVerifierGpu (the one its BlsBftReplica calls).
    commit_items: (commit, sender) -> [(sig str, message bytes, pk)], the triples
    validate_commit would check (replica_commit_items builds it from a replica).
    """

    def __init__(self, verifier, commit_items: Callable):
        self.verifier = verifier
        self.commit_items = commit_items
        self.last_pass = {'commits': 0, 'checks': 0, 'verified': 0}
        self.last_results = []

    def collect(self, wrapped: Iterable[Tuple[object, str]]) -> List[tuple]:
        items = []
        for commit, sender in wrapped:
            try:
                items.extend(self.commit_items(commit, sender))
            except Exception:  # noqa: BLE001 - malformed: the per-COMMIT path reports it
                continue
        return items

    def prefetch(self, wrapped: Iterable[Tuple[object, str]]) -> int:
        """One GPU pass over the pass's COMMIT signatures; returns the number of
        distinct checks run.  Call end_pass() after the handlers ran."""
        wrapped = list(wrapped)
        items = self.collect(wrapped)
        verified = self.verifier.prefetch(items) if items else 0
        self.last_pass = {'commits': len(wrapped), 'checks': len(items), 'verified': verified}
        return verified

    def end_pass(self):
        """Drop the verdicts no handler consumed."""
        self.verifier.drop_prefetched()

    def service(self, wrapped: Iterable[Tuple[object, str]], handler: Callable, limit: Optional[int] = None,
                stasher=None) -> int:
        """The pass: pre-verify, then hand each (commit, sender) to the node's
        unchanged handler (OrderingService.process_commit) in arrival order.

        In the reference a COMMIT reaches process_commit only through the
        ordering service's StashingRouter (ordering_service.py:198 subscribes
        `partial(stasher._process, process_commit)`), which reads the handler's
        `(code, reason)` return to stash the COMMIT for later (STASH_VIEW_3PC,
        STASH_CATCH_UP, STASH_WAITING_FIRST_BATCH_IN_VIEW, ...) or discard it
        (stashing_router.py:167-185).  Pass that router as `stasher` and each
        COMMIT takes the same route: `stasher._process(handler, commit, sender)`.
        A COMMIT stashed here is replayed by the router later, after end_pass(),
        and its check then runs as its own verify_sig call.  Without `stasher`
        the handler is called directly (a handler that already routes, e.g. the
        network bus's `process_incoming`).  `last_results` keeps what each call
        returned, in order.  Returns the number of COMMITs handed on."""
        wrapped = list(wrapped)
        if limit is not None:
            wrapped = wrapped[:limit]
        dispatch = handler if stasher is None else partial(stasher._process, handler)
        self.prefetch(wrapped)
        self.last_results = []
        try:
            for commit, sender in wrapped:
                self.last_results.append(dispatch(commit, sender))
        finally:
            self.end_pass()
        return len(wrapped)
