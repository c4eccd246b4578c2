"""Authenticator registry + verified-request cache
(plenum/server/req_authenticator.py:11-72) with batch entry points.

`verify_batch(reqs, keys)` lets every registered authenticator that supports
it prefetch GPU verdicts for the requests it would handle, then runs the
unchanged per-request `authenticate(req, key)` on each: it IS a batch of
`authenticate` calls, so accepted requests land in `_verified_reqs` exactly as
they would after per-request calls (:34-35, :53-57), and rejected requests
surface the same exception the per-request path raises.

`prefetch(reqs, keys)` only fills the authenticators' (pk, sig||msg) verdict
caches and authenticates nothing: `_verified_reqs` keeps being written solely
by the node's own `authenticate(req, key)` calls, i.e. after its blacklist and
static-validation checks (node.py:1625-1657).  `drop_prefetched()` forgets the
verdicts no handler consumed.  This is the form a service pass uses
(plenum_gpu.ingress.BatchIngress).
"""
from copy import deepcopy
from typing import Optional

from .client_authn import ClientAuthNr
from .constants import OPERATION, SIGNATURE, TXN_TYPE
from .exceptions import NoAuthenticatorFound


class ReqAuthenticator:
    def __init__(self):
        self._authenticators = []
        self._verified_reqs = {}

    def register_authenticator(self, authenticator: ClientAuthNr):
        self._authenticators.append(authenticator)

    def authenticate(self, req_data, key=None):
        typ = req_data.get(OPERATION, {}).get(TXN_TYPE)
        if key and self._check_and_verify_existing_req(req_data, key):
            return self._verified_reqs[key]['identifiers']
        identifiers = set()
        for authnr in self._authenticators:
            if authnr.is_query(typ):
                return set()
            if authnr.is_write(typ) or authnr.is_action(typ):
                identifiers.update(authnr.authenticate(deepcopy(req_data)) or set())
        if not identifiers:
            raise NoAuthenticatorFound
        if key:
            self._verified_reqs[key] = {'signature': req_data.get(SIGNATURE), 'identifiers': identifiers}
        return identifiers

    def _check_and_verify_existing_req(self, req_data: dict, key: str):
        entry = self._verified_reqs.get(key)
        return entry is not None and req_data.get(SIGNATURE) == entry['signature']

    def prefetch(self, reqs, keys=None):
        """One GPU verification pass per authenticator over the signatures of
        `reqs` it would check; verdicts are kept for the per-request path and
        nothing is authenticated or cached in `_verified_reqs`.  Returns the
        number of signatures verified."""
        keys = list(keys) if keys is not None else [None] * len(reqs)
        if len(keys) != len(reqs):
            raise ValueError('keys must match reqs')
        n = 0
        for authnr in self._authenticators:
            prefetch = getattr(authnr, 'verify_batch', None)
            if prefetch is None:
                continue
            mine = []
            for req, key in zip(reqs, keys):
                if key and self._check_and_verify_existing_req(req, key):
                    continue
                typ = req.get(OPERATION, {}).get(TXN_TYPE) if isinstance(req, dict) else None
                if authnr.is_write(typ) or authnr.is_action(typ):
                    mine.append(req)
            if mine:
                n += prefetch(mine) or 0
        return n

    def drop_prefetched(self):
        """Forget prefetched verdicts no `authenticate` consumed."""
        for authnr in self._authenticators:
            drop = getattr(authnr, 'drop_prefetched', None)
            if drop is not None:
                drop()

    def verify_batch(self, reqs, keys=None):
        """Authenticate a batch: one GPU verification pass per authenticator,
        then the per-request path.  Returns [identifiers set | exception]."""
        keys = list(keys) if keys is not None else [None] * len(reqs)
        self.prefetch(reqs, keys)
        out = []
        for req, key in zip(reqs, keys):
            try:
                out.append(self.authenticate(req, key=key))
            except Exception as ex:
                out.append(ex)
        self.drop_prefetched()
        return out

    @property
    def core_authenticator(self):
        if not self._authenticators:
            raise RuntimeError('No authenticator registered yet')
        return self._authenticators[0]

    def get_authnr_by_type(self, authnr_type) -> Optional[ClientAuthNr]:
        for authnr in self._authenticators:
            if isinstance(authnr, authnr_type):
                return authnr
        return None

    def clean_from_verified(self, key):
        self._verified_reqs.pop(key, None)
