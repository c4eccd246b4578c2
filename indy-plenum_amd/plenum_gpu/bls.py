"""BLS COMMIT check on the GPU -- drop-in mirror of the
reference's BLS verifier surface, batched.

Reference path (every COMMIT of every 3PC batch):
  BlsBftReplicaPlenum.validate_commit (plenum/bls/bls_bft_replica_plenum.py:55-75)
    -> _validate_signature (:194-213): pk = bls_key_register.get_key_by_name(sender),
       message = MultiSignatureValue(...).as_single_value()
    -> BlsCryptoVerifierIndyCrypto.verify_sig (crypto/bls/indy_crypto/bls_crypto_indy_crypto.py:73-82)
    -> python-ursa Bls.verify(signature, message, pk, generator).
Here: `BlsCryptoVerifierGpu.verify_sig` keeps that signature and semantics (None
signature or key -> False) and `verify_sig_batch` runs many checks in ONE GPU
pass (pv_bls_verify_batch: every message hashed once, checks grouped by key, the
generator's and keys' lines precomputed once per key set);
`validate_commit_batch` is `validate_commit`'s rule for a batch of COMMITs, and
`commit_quorums` feeds the verdicts to the n - f tally kernel (pv_tally_votes,
ordering_service.py:457-488 rule 3 + models.py voter sets).

PARITY UNPINNED: ursa / Milagro AMCL are not importable here and
the reference holds no BLS vector.  The generator constant and the message bytes
(MultiSignatureValue.as_single_value, msgpack of the sorted dict) are the
reference's own and are pinned by tests/golden/bls.json; the verdicts are pinned
only against the restatements the tests hold.  No CPU fallback:
the checks run on the HIP kernels or raise.
"""
from collections import OrderedDict, namedtuple
from typing import Dict, Optional, Sequence

import numpy as np

from . import _native
from . import base58

GroupParams = namedtuple('GroupParams', 'group_name, g')   # crypto/bls/bls_crypto.py:5-6

# BlsGroupParamsLoaderIndyCrypto.load_group_params (bls_crypto_indy_crypto.py:15-20)
GENERATOR = ('3LHpUjiyFC2q2hD7MnwwNmVXiuaFbQx2XkAFJWzswCjgN1utjsCeLzHsKk1nJvFEaS4fcrUmVAkdhtPCYbrVyATZcmzwJReTcJq'
             'wqBCPTmTQ9uWPwz6rEncKb2pYYYFcdHa8N17HzVyTqKfgPi4X9pMetfT3A5xCHq54R2pDNYWVLDX')

CM_BLS_SIG_WRONG = 2          # crypto/bls/bls_bft_replica.py:9
PPR_BLS_MULTISIG_WRONG = 1    # :8
REPR_SIZE = 128               # python-ursa's representation size of a G1 / G2 element
MULTI_MAX = 65535             # checks per pv_bls_verify_multi_batch call


class BlsGroupParamsLoaderIndyCrypto:
    def load_group_params(self) -> GroupParams:
        return GroupParams('generator', GENERATOR)


class IndyCryptoError(Exception):
    """what ursa raises for a representation it cannot parse"""


class BlsEntity:
    """Byte holder with ursa's BlsEntity surface (as_bytes / from_bytes).
    The curve arithmetic never runs on the host: decoding happens in the kernels."""
    __slots__ = ('_b',)

    def __init__(self, b: bytes):
        self._b = bytes(b)

    def as_bytes(self) -> bytes:
        return self._b

    @classmethod
    def from_bytes(cls, b):
        return cls(b)

    def __eq__(self, other):
        return type(self) is type(other) and self._b == other._b

    def __hash__(self):
        return hash((type(self).__name__, self._b))


class VerKey(BlsEntity):
    @classmethod
    def from_bytes(cls, b):
        if len(b) != REPR_SIZE:
            raise IndyCryptoError('Invalid len of bytes representation for PointG2')
        return cls(b)


class Generator(VerKey):
    pass


class Signature(BlsEntity):
    """Any length is carried: a representation that is not 128 bytes fails to
    decode inside the check (pv_bls_verify_batch sig_len), i.e. verify_sig
    returns False -- ursa's from_bytes error surfaces the same way (bls_from_str
    -> None -> False)."""


class MultiSignature(Signature):
    pass


class ProofOfPossession(BlsEntity):
    """A G1 point (ursa ProofOfPossession.from_bytes: 128 bytes or IndyCryptoError)."""

    @classmethod
    def from_bytes(cls, b):
        if len(b) != REPR_SIZE:
            raise IndyCryptoError('Invalid len of bytes representation for PointG1')
        return cls(b)


class IndyCryptoBlsUtils:
    """crypto/bls/indy_crypto/bls_crypto_indy_crypto.py:23-66"""
    SEED_LEN = 32

    @staticmethod
    def bls_to_str(v: BlsEntity) -> str:
        return base58.b58encode(v.as_bytes()).decode('utf-8')

    @staticmethod
    def bls_from_str(v: str, cls) -> Optional[BlsEntity]:
        try:
            bts = base58.b58decode(v)
        except ValueError:
            return None
        try:
            return cls.from_bytes(bts)
        except IndyCryptoError:
            return None

    @staticmethod
    def bls_pk_from_str(v: str) -> Optional[VerKey]:
        return IndyCryptoBlsUtils.bls_from_str(v, VerKey)


class PlenumTypeError(TypeError):
    """common/exceptions.py:16-33 (message format kept)"""

    def __init__(self, v_name, v_value, v_exp_t):
        super().__init__("variable '{}', type {}, expected: {}".format(v_name, type(v_value), v_exp_t))


class MultiSignatureValue:
    """crypto/bls/bls_multi_signature.py:7-81: the value a COMMIT's BLS signature
    covers; as_single_value() = msgpack of the field dict sorted by key
    (multi_signature_value_serializer = MsgPackSerializer,
    common/serializers/serialization.py:21, msgpack_serializer.py:21-31)."""

    def __init__(self, ledger_id: int, state_root_hash: str, pool_state_root_hash: str, txn_root_hash: str,
                 timestamp: int):
        for name, val, t in (('ledger_id', ledger_id, int), ('state_root_hash', state_root_hash, str),
                             ('pool_state_root_hash', pool_state_root_hash, str),
                             ('txn_root_hash', txn_root_hash, str), ('timestamp', timestamp, int)):
            if not isinstance(val, t):
                raise PlenumTypeError(name, val, t)
        self.ledger_id = ledger_id
        self.state_root_hash = state_root_hash
        self.pool_state_root_hash = pool_state_root_hash
        self.txn_root_hash = txn_root_hash
        self.timestamp = timestamp

    def as_dict(self):
        return OrderedDict(sorted(self.__dict__.items()))

    def as_single_value(self) -> bytes:
        import msgpack
        return msgpack.packb(self.as_dict(), use_bin_type=True)

    def as_list(self):
        return [self.ledger_id, self.state_root_hash, self.pool_state_root_hash, self.txn_root_hash, self.timestamp]

    def __eq__(self, other):
        return isinstance(other, MultiSignatureValue) and self.as_dict() == other.as_dict()

    def __str__(self):
        return str(self.as_dict())


class BlsCryptoVerifierGpu:
    """BlsCryptoVerifierIndyCrypto (bls_crypto_indy_crypto.py:68-109): the four
    methods of the reference verifier with the same signatures and None rules,
    plus batch entry points.  Keys are prepared on the device the first time
    they are seen and kept there, keyed by their bytes (pv_bls_add_keys appends
    only the new ones; verifiers of one generator share the set).  A proof of
    possession is checked against a per-call key set instead
    (pv_bls_verify_multi_batch), so keys of rejected NODE txns never join it.

    Prefetch seam (CommitIngress, plenum_gpu/commit_ingress.py): `prefetch`
    verifies many (signature, message, key) triples in one GPU pass and keeps
    the verdicts; `verify_sig` answers from them, so the reference's unchanged
    per-COMMIT `_validate_signature` -> `verify_sig` makes no GPU call for a
    prefetched COMMIT.  `drop_prefetched` ends the pass."""

    def __init__(self, params: GroupParams, device: int = 0):
        self._generator = IndyCryptoBlsUtils.bls_from_str(params.g, Generator)
        if self._generator is None:
            raise ValueError('bad BLS group generator')
        self._device = device
        self._status = []        # status of every key in the device set (after the last _key_indices)
        self._prefetched = {}    # (signature str, message bytes, pk bytes) -> verdict
        self.gpu_calls = 0       # native verify calls made (tests of the prefetch seam)

    # -- key set
    def _key_indices(self, pks):
        idx, self._status = _native.bls_key_indices(self._generator.as_bytes(), pks, device=self._device)
        return idx

    def key_status(self, pk: VerKey) -> int:
        """PV_BLS_KEY_OK / _INFINITY / _NOT_IN_G2 of a key (prepares it)"""
        return int(self._status[self._key_indices([pk.as_bytes()])[0]])

    # -- single-key checks
    def _verify_raw(self, rows) -> np.ndarray:
        """rows: [(signature bytes, message bytes, pk bytes)] -> bool array (one GPU pass)"""
        n = len(rows)
        if not n:
            return np.zeros(0, bool)
        sigs, sig_len, msgs, midx = [], [], {}, []
        for b, message, _pk in rows:
            sig_len.append(len(b))
            sigs.append(b[:REPR_SIZE].ljust(REPR_SIZE, b'\0'))
            midx.append(msgs.setdefault(bytes(message), len(msgs)))
        kidx = np.array(self._key_indices([r[2] for r in rows]), np.uint32)
        blob, off = _native.pack_messages(list(msgs))
        self.gpu_calls += 1
        return _native.bls_verify_arrays(np.frombuffer(b''.join(sigs), np.uint8), blob, off,
                                         np.array(midx, np.uint32), kidx, sig_len=np.array(sig_len, np.uint64),
                                         device=self._device)

    def verify_sig_batch(self, items) -> np.ndarray:
        """items: [(signature: str, message: bytes, bls_pk: VerKey | None)] ->
        bool array, entry i == verify_sig(*items[i])."""
        out = np.zeros(len(items), bool)
        rows, where = [], []
        for i, (signature, message, bls_pk) in enumerate(items):
            s = IndyCryptoBlsUtils.bls_from_str(signature, Signature)
            if s is None or bls_pk is None:
                continue
            rows.append((s.as_bytes(), message, bls_pk.as_bytes()))
            where.append(i)
        if rows:
            out[np.array(where)] = self._verify_raw(rows)
        return out

    def verify_sig(self, signature: str, message: bytes, bls_pk: Optional[VerKey]) -> bool:
        """bls_crypto_indy_crypto.py:73-82"""
        if self._prefetched and bls_pk is not None:
            hit = self._prefetched.get((signature, bytes(message), bls_pk.as_bytes()))
            if hit is not None:
                return hit
        return bool(self.verify_sig_batch([(signature, message, bls_pk)])[0])

    # -- the prefetch seam (COMMITs of one Looper pass)
    def prefetch(self, items) -> int:
        """Verify [(signature str, message bytes, bls_pk VerKey | None)] in one GPU
        pass and keep the verdicts for verify_sig; returns the number verified."""
        todo = {}
        for signature, message, bls_pk in items:
            if bls_pk is None or not isinstance(signature, str):
                continue
            k = (signature, bytes(message), bls_pk.as_bytes())
            if k not in self._prefetched:
                todo.setdefault(k, (signature, k[1], bls_pk))
        if todo:
            got = self.verify_sig_batch(list(todo.values()))
            for k, v in zip(todo, got):
                self._prefetched[k] = bool(v)
        return len(todo)

    def drop_prefetched(self):
        self._prefetched.clear()

    # -- multi-signatures (PRE-PREPARE path, ordering)
    def verify_multi_sig_batch(self, items) -> np.ndarray:
        """items: [(signature: str, message: bytes, pks: Sequence[VerKey | None])] ->
        bool array, entry i == verify_multi_sig(*items[i]); ONE GPU pass (the
        keys of every check summed on the device, lines of each sum, the checks)."""
        out = np.zeros(len(items), bool)
        if len(items) > MULTI_MAX:           # pv_bls_verify_multi_batch takes at most 65535 checks
            for s0 in range(0, len(items), MULTI_MAX):
                out[s0:s0 + MULTI_MAX] = self.verify_multi_sig_batch(items[s0:s0 + MULTI_MAX])
            return out
        sigs, sig_len, msgs, midx, keys, pk_off, where = [], [], {}, [], [], [0], []
        for i, (signature, message, pks) in enumerate(items):
            if None in pks:                  # :86-88
                continue
            ms = IndyCryptoBlsUtils.bls_from_str(signature, MultiSignature)
            if ms is None:                   # :90-93
                continue
            b = ms.as_bytes()
            sig_len.append(len(b))
            sigs.append(b[:REPR_SIZE].ljust(REPR_SIZE, b'\0'))
            midx.append(msgs.setdefault(bytes(message), len(msgs)))
            for pk in pks:
                kb = pk.as_bytes()
                keys.append(kb[:REPR_SIZE].ljust(REPR_SIZE, b'\0'))
            pk_off.append(len(keys))
            where.append(i)
        if where:
            blob, off = _native.pack_messages(list(msgs))
            self.gpu_calls += 1
            got = _native.bls_verify_multi_arrays(
                self._generator.as_bytes(), np.frombuffer(b''.join(sigs), np.uint8), blob, off,
                np.array(midx, np.uint32), np.frombuffer(b''.join(keys), np.uint8), np.array(pk_off, np.uint64),
                sig_len=np.array(sig_len, np.uint64), device=self._device)
            out[np.array(where)] = got
        return out

    def verify_multi_sig(self, signature: str, message: bytes, pks: Sequence[Optional[VerKey]]) -> bool:
        """bls_crypto_indy_crypto.py:84-97: e(sigma, g) == e(H(m), sum of pks)"""
        return bool(self.verify_multi_sig_batch([(signature, message, pks)])[0])

    def create_multi_sig_batch(self, sets) -> list:
        """sets: [Sequence[signature str]] -> [multi-signature str], entry j ==
        create_multi_sig(sets[j]); one GPU launch sums every set."""
        raw, set_off = [], [0]
        for signatures in sets:
            for s in signatures:
                sig = IndyCryptoBlsUtils.bls_from_str(s, Signature)
                if sig is None or len(sig.as_bytes()) != REPR_SIZE:
                    # ursa: bls_from_str -> None, then MultiSignature.new reads None.c_instance
                    raise AttributeError("'NoneType' object has no attribute 'c_instance'")
                raw.append(sig.as_bytes())
            set_off.append(len(raw))
        if not sets:
            return []
        sigs = np.frombuffer(b''.join(raw), np.uint8) if raw else np.zeros(0, np.uint8)
        out = _native.bls_aggregate_sigs(sigs, np.array(set_off, np.uint64), device=self._device)
        return [IndyCryptoBlsUtils.bls_to_str(MultiSignature(row.tobytes())) for row in out]

    def create_multi_sig(self, signatures: Sequence[str]) -> str:
        """bls_crypto_indy_crypto.py:99-102: MultiSignature.new = the sum of the G1 points"""
        return self.create_multi_sig_batch([signatures])[0]

    def verify_key_proof_of_possession(self, key_proof: Optional[ProofOfPossession],
                                       bls_pk: Optional[VerKey]) -> bool:
        """bls_crypto_indy_crypto.py:104-109 -> ursa Bls.verify_pop:
        e(pop, g) == e(H(pk bytes), pk), H = PointG1::from_hash(SHA-256(ver_key.as_bytes()))
        with as_bytes() the key's 128-byte representation as given (ursa keeps it).
        PARITY UNPINNED like every BLS verdict here."""
        if key_proof is None or bls_pk is None:
            return False
        return bool(self.verify_key_proofs_batch([(key_proof, bls_pk)])[0])

    def verify_key_proofs_batch(self, items) -> np.ndarray:
        """items: [(key_proof ProofOfPossession | None, bls_pk VerKey | None)] ->
        bool array, entry i == verify_key_proof_of_possession(*items[i]).  The
        keys are checked against a per-call key set (each a one-key "sum",
        pv_bls_verify_multi_batch): a NODE txn's key joins the verifier's device
        set only when it signs COMMITs, never because its proof was checked."""
        out = np.zeros(len(items), bool)
        rows, where = [], []
        for i, (key_proof, bls_pk) in enumerate(items):
            if key_proof is None or bls_pk is None:
                continue
            rows.append((key_proof.as_bytes(), bls_pk.as_bytes()))
            where.append(i)
        for s0 in range(0, len(rows), MULTI_MAX):
            part = rows[s0:s0 + MULTI_MAX]
            msgs, midx = {}, []
            for _pop, pk in part:
                midx.append(msgs.setdefault(pk, len(msgs)))
            blob, off = _native.pack_messages(list(msgs))
            self.gpu_calls += 1
            got = _native.bls_verify_multi_arrays(
                self._generator.as_bytes(), np.frombuffer(b''.join(p[:REPR_SIZE].ljust(REPR_SIZE, b'\0') for p, _ in part),
                                                          np.uint8),
                blob, off, np.array(midx, np.uint32),
                np.frombuffer(b''.join(pk[:REPR_SIZE].ljust(REPR_SIZE, b'\0') for _, pk in part), np.uint8),
                np.arange(len(part) + 1, dtype=np.uint64), sig_len=np.array([len(p) for p, _ in part], np.uint64),
                device=self._device)
            out[np.array(where[s0:s0 + MULTI_MAX])] = got
        return out

    # -- COMMITs
    def validate_commit_batch(self, commits) -> list:
        """validate_commit's BLS rule for many COMMITs (bls_bft_replica_plenum.py:55-75).

        commits: [(bls_pk VerKey | None, bls_sigs {ledger_id: sig str} | None,
                   values {ledger_id: MultiSignatureValue})] where `values` holds
        the MultiSignatureValue _validate_signature builds for each ledger the
        audit transaction covers.  -> per COMMIT: None (no BLS_SIGS, or every
        signature verifies) or CM_BLS_SIG_WRONG."""
        items, owner = [], []
        res = [None] * len(commits)
        for c, (pk, sigs, values) in enumerate(commits):
            if sigs is None:
                continue
            for lid, sig in sigs.items():
                v = values.get(int(lid))
                if v is None:                      # ledger not in the audit txn
                    res[c] = CM_BLS_SIG_WRONG
                    continue
                items.append((sig, v.as_single_value(), pk))
                owner.append(c)
        if items:
            ok = self.verify_sig_batch(items)
            for c, good in zip(owner, ok):
                if not good:
                    res[c] = CM_BLS_SIG_WRONG
        return res


def commit_quorums(verdicts, senders, batch_off, n_nodes, quorum):
    """n - f COMMIT quorum per 3PC batch from per-COMMIT verdicts (True = the
    COMMIT counts) and sender indices, on the tally kernel (voter SET semantics,
    plenum/server/models.py:16-114): -> (votes, reached)."""
    return _native.tally_arrays(np.asarray(verdicts, np.uint8), senders, batch_off, n_nodes, quorum)


__all__ = ['GroupParams', 'GENERATOR', 'BlsGroupParamsLoaderIndyCrypto', 'IndyCryptoError', 'BlsEntity', 'VerKey',
           'Generator', 'Signature', 'MultiSignature', 'ProofOfPossession', 'IndyCryptoBlsUtils', 'MultiSignatureValue',
           'BlsCryptoVerifierGpu', 'CM_BLS_SIG_WRONG', 'PPR_BLS_MULTISIG_WRONG', 'commit_quorums']
