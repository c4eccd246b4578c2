"""Batched ingestion of one node service pass.

The reference authenticates one message at a time: `ZStack.processReceived`
(stp_zmq/zstack.py:606-646) hands each deserialized message to the node's
handler, `Node.validateClientMsg` / `validateNodeMsg` call `verifySignature`
(plenum/server/node.py:1618-1655, 1478-1505, 2624-2655), and node `Batch`es
are unpacked and handled message by message (`unpackNodeMsg`, node.py:1507-1527).
A PROPAGATE carries the client request it relays (node.py:2635-2637), so the
same request is usually authenticated once as a client message and again for
every PROPAGATE of it.

`BatchIngress` sits in front of those unchanged handlers: for the messages a
service pass received it collects every request that `verifySignature` would
authenticate (client requests, PROPAGATE.request, both also inside BATCHes),
keys them by `Request.key` (plenum/common/request.py:82-120), drops duplicates,
and runs ONE `ReqAuthenticator.prefetch` — one GPU pass.  The pre-pass only
computes signature VERDICTS: it authenticates nothing and never writes the
verified-request cache (`_verified_reqs`).  The node's unchanged per-message
path — blacklist check, static validation, then `verifySignature` ->
`authenticate(req, key)` (node.py:1625-1657) — consumes those verdicts instead
of calling the verifier, and so fills `_verified_reqs` exactly when and as the
reference does; a request a handler drops before authenticating leaves no trace.
Verdicts the pass did not consume are dropped at its end.  Message order,
handlers and outcomes are unchanged; only where the signature work happens moves.
"""
import json
from hashlib import sha256
from typing import Callable, Iterable, List, Optional, Tuple

from .constants import IDENTIFIER, OPERATION, SIGNATURE, SIGNATURES
from .serialization import serialize_msg_for_signing

OP_FIELD_NAME = 'op'
PROPAGATE = 'PROPAGATE'
BATCH = 'BATCH'
REQ_ID = 'reqId'
PROTOCOL_VERSION = 'protocolVersion'
TAA_ACCEPTANCE = 'taaAcceptance'
ENDORSER = 'endorser'
MSGS = 'messages'


def idr_from_req_data(data: dict):
    """plenum/common/util.py idr_from_req_data: the identifier, or the sorted
    signer set joined by ',' (Request.gen_idr_from_sigs)."""
    if data.get(IDENTIFIER):
        return data[IDENTIFIER]
    sigs = data.get(SIGNATURES)
    return ','.join(sorted(sigs.keys())) if sigs else None


def signing_state(req: dict, plugin_fields: Iterable[str] = ()) -> dict:
    """Request(**req).signingState() (plenum/common/request.py:95-120)."""
    state = {IDENTIFIER: idr_from_req_data(req), REQ_ID: req.get(REQ_ID), OPERATION: req.get(OPERATION)}
    for k in (PROTOCOL_VERSION, TAA_ACCEPTANCE, ENDORSER):
        if req.get(k) is not None:
            state[k] = req[k]
    if req.get(SIGNATURES) is not None:
        state[SIGNATURES] = req[SIGNATURES]
    if req.get(SIGNATURE) is not None:
        state[SIGNATURE] = req[SIGNATURE]
    for nm in plugin_fields:
        val = req.get(nm)
        if val:
            state[nm] = val
    return state


def request_key(req: dict, plugin_fields: Iterable[str] = ()) -> str:
    """Request(**req).key = sha256(serialize_msg_for_signing(signingState())).hexdigest()
    (plenum/common/request.py:82-90); plenum_gpu.merkle.request_digests batches it on the GPU."""
    return sha256(serialize_msg_for_signing(signing_state(req, plugin_fields))).hexdigest()


def is_client_request(msg) -> bool:
    """validateClientMsg's request test (node.py:1629-1632)."""
    return isinstance(msg, dict) and bool(msg.get(OPERATION) and msg.get(REQ_ID) and idr_from_req_data(msg))


class BatchIngress:
    """Pre-authenticate the requests of one service pass in one GPU pass.

    req_authenticator: a ReqAuthenticator (plenum_gpu.req_authenticator) — the
    node's `clientAuthNr`.  deserialize: the stack's `deserializeMsg` for BATCH
    members (JSON, stp_zmq/zstack.py:881-885).
    """

    def __init__(self, req_authenticator, plugin_fields: Iterable[str] = (),
                 deserialize: Callable = None):
        self.authenticator = req_authenticator
        self.plugin_fields = tuple(plugin_fields)
        self.deserialize = deserialize or _deserialize
        self.last_pass = {'messages': 0, 'requests': 0, 'distinct': 0, 'verified': 0}

    # ------------------------------------------------------------ collection
    def requests_in(self, msg, from_node: bool) -> List[dict]:
        """Requests `verifySignature` would authenticate for this message:
        a client request itself; PROPAGATE.request from a node; BATCH members
        (deserialized as unpackNodeMsg / unpackClientMsg do; undecodable
        members are skipped there too)."""
        if not isinstance(msg, dict):
            return []
        op = msg.get(OP_FIELD_NAME)
        if op == BATCH:
            out = []
            members = msg.get(MSGS)
            if not isinstance(members, list):
                return out
            for m in members:
                try:
                    m = self.deserialize(m)
                except Exception:  # noqa: BLE001 - unpackNodeMsg logs and skips
                    continue
                out.extend(self.requests_in(m, from_node))
            return out
        if from_node:
            if op == PROPAGATE and isinstance(msg.get('request'), dict):
                return [msg['request']]
            return []
        return [msg] if is_client_request(msg) else []

    def collect(self, wrapped: Iterable[Tuple[dict, str]], from_node: bool) -> Tuple[List[dict], List[str]]:
        """Distinct (by Request.key) requests of a pass, in arrival order."""
        reqs, keys, seen = [], [], set()
        n = 0
        for msg, _frm in wrapped:
            for req in self.requests_in(msg, from_node):
                n += 1
                try:
                    key = request_key(req, self.plugin_fields)
                except Exception:  # noqa: BLE001 - malformed: the per-message path reports it
                    continue
                if key in seen:
                    continue
                seen.add(key)
                reqs.append(req)
                keys.append(key)
        self.last_pass['requests'] = n
        return reqs, keys

    # ------------------------------------------------------------ the pass
    def prefetch(self, wrapped: Iterable[Tuple[dict, str]], from_node: bool = False):
        """One GPU verification pass over the signatures of the pass's distinct
        requests; the verdicts wait in the authenticators for the per-message
        `authenticate` calls (nothing is authenticated here).  Returns the
        distinct (requests, keys); call `end_pass()` after the handlers ran."""
        wrapped = list(wrapped)
        reqs, keys = self.collect(wrapped, from_node)
        self.last_pass.update(messages=len(wrapped), distinct=len(reqs))
        self.last_pass['verified'] = self.authenticator.prefetch(reqs, keys) if reqs else 0
        return reqs, keys

    def end_pass(self):
        """Drop the verdicts of the pass no handler consumed."""
        self.authenticator.drop_prefetched()

    def service(self, wrapped: Iterable[Tuple[dict, str]], handler: Callable, from_node: bool = False,
                limit: Optional[int] = None) -> int:
        """ZStack.processReceived's dispatch loop with the batch pre-pass: up to
        `limit` messages are pre-authenticated together, then handed one by one
        to `handler((msg, frm))` — the node's unchanged handleOneClientMsg /
        handleOneNodeMsg."""
        wrapped = list(wrapped)
        if limit is not None:
            wrapped = wrapped[:limit]
        self.prefetch(wrapped, from_node)
        try:
            for w in wrapped:
                handler(w)
        finally:
            self.end_pass()
        return len(wrapped)


def _deserialize(m):
    if isinstance(m, bytes):
        m = m.decode()
    return json.loads(m) if isinstance(m, str) else m
