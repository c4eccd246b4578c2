"""A minimal BlsBftReplicaPlenum stand-in for the COMMIT batch seam tests.

It carries exactly the members `plenum_gpu.commit_ingress.replica_commit_items`
reads, each restating the reference method it stands for, and `validate_commit`
restates the reference's per-COMMIT check (plenum/bls/bls_bft_replica_plenum.py:
55-75 + _validate_signature :194-213) calling `verify_sig` once per ledger — the
unchanged node path the seam must serve from its prefetched verdicts."""
from collections import namedtuple
from types import SimpleNamespace

PrePrepare = namedtuple('PrePrepare', 'instId viewNo ppSeqNo ppTime ledgerId stateRootHash txnRootHash '
                                      'poolStateRootHash')
Commit = namedtuple('Commit', 'instId viewNo ppSeqNo blsSigs')
CM_BLS_SIG_WRONG = 2


def replica_name_to_node_name(name):
    """plenum/server/consensus/utils.py:8-11"""
    return None if name is None else name.rsplit(':', maxsplit=1)[0]


class FakeBlsReplica:
    def __init__(self, verifier, keys_by_node, audit_by_pp_seq_no, msv_cls):
        self.verifier = verifier
        self.audit = audit_by_pp_seq_no
        self.msv_cls = msv_cls
        self._bls_bft = SimpleNamespace(
            bls_key_register=SimpleNamespace(get_key_by_name=lambda name, root=None: keys_by_node.get(name)),
            bls_crypto_verifier=verifier)

    @staticmethod
    def _create_fake_pre_prepare_for_multi_sig(lid, state_root_hash, txn_root_hash, pre_prepare):   # :332-353
        return pre_prepare._replace(ledgerId=lid, stateRootHash=state_root_hash, txnRootHash=txn_root_hash)

    def _get_correct_audit_transaction(self, pp):                                                  # :318-329
        return self.audit.get(pp.ppSeqNo)

    def _get_pool_root_hash(self, pre_prepare, serialize=True):                                    # :289-296
        return pre_prepare.poolStateRootHash if serialize else pre_prepare.poolStateRootHash.encode()

    @staticmethod
    def get_node_name(replica_name):                                                               # :355-357
        return replica_name_to_node_name(replica_name)

    def _create_multi_sig_value_for_pre_prepare(self, pre_prepare, pool_state_root_hash):          # :186-192
        return self.msv_cls(ledger_id=pre_prepare.ledgerId, state_root_hash=pre_prepare.stateRootHash,
                            pool_state_root_hash=pool_state_root_hash, txn_root_hash=pre_prepare.txnRootHash,
                            timestamp=pre_prepare.ppTime)

    def _validate_signature(self, sender, bls_sig, pre_prepare):                                   # :194-213
        pool_root_hash = self._get_pool_root_hash(pre_prepare, serialize=False)
        pk = self._bls_bft.bls_key_register.get_key_by_name(self.get_node_name(sender), pool_root_hash)
        if not pk:
            return False
        message = self._create_multi_sig_value_for_pre_prepare(pre_prepare, self._get_pool_root_hash(pre_prepare))
        return self._bls_bft.bls_crypto_verifier.verify_sig(bls_sig, message.as_single_value(), pk)

    def validate_commit(self, commit, sender, pre_prepare):                                        # :55-75
        if commit.blsSigs is None:
            return None
        audit_txn = self._get_correct_audit_transaction(pre_prepare)
        if not audit_txn:
            return None
        payload = audit_txn['txn']['data']
        for lid, sig in commit.blsSigs.items():
            lid = int(lid)
            if lid not in payload['stateRoot'] or lid not in payload['ledgerRoot']:
                return CM_BLS_SIG_WRONG
            if not self._validate_signature(sender, sig, self._create_fake_pre_prepare_for_multi_sig(
                    lid, payload['stateRoot'][lid], payload['ledgerRoot'][lid], pre_prepare)):
                return CM_BLS_SIG_WRONG
        return None


def audit_txn(state_roots, ledger_roots):
    return {'txn': {'data': {'stateRoot': state_roots, 'ledgerRoot': ledger_roots}}}


# plenum/common/stashing_router.py:11-13, plenum/server/replica_validator_enums.py:6
DISCARD, PROCESS, STASH = -1, 0, 1
STASH_VIEW_3PC = 2


class MiniStasher:
    """The part of the reference StashingRouter a COMMIT passes through:
    _process (stashing_router.py:167-185: None / PROCESS = processed, DISCARD =
    dropped, any other code = stashed under that code) and process_all_stashed
    (:117-136, replaying through the subscribed handler)."""

    def __init__(self):
        self.stashed, self.discarded, self.handler = {}, [], None

    def _process(self, handler, message, *args):
        self.handler = handler
        result = handler(message, *args)
        code, reason = result if result else (None, None)
        if not code:
            return True
        if code == DISCARD:
            self.discarded.append((message, args, reason))
            return True
        self.stashed.setdefault(code, []).append((message, *args))
        return False

    def process_all_stashed(self, code=None):
        for c in sorted(self.stashed) if code is None else [code]:
            data, self.stashed[c] = self.stashed.get(c, []), []
            for msg_tuple in data:
                self._process(self.handler, *msg_tuple)

