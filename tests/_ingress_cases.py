"""Shared checks for the batched-ingestion fixture (tests/golden/ingress.json)."""
import copy
import json
import os

from conftest import GOLDEN


def load():
    with open(os.path.join(GOLDEN, 'ingress.json')) as fh:
        return json.load(fh)


def make_ra(fx):
    from plenum_gpu.client_authn import CoreAuthNr
    from plenum_gpu.req_authenticator import ReqAuthenticator
    authnr = CoreAuthNr(fx['write_types'], [], [])
    for idr, vk in fx['registry'].items():
        authnr.addIdr(idr, vk)
    ra = ReqAuthenticator()
    ra.register_authenticator(authnr)
    return ra


def outcome(x):
    if isinstance(x, BaseException):
        return {'exc': type(x).__name__, 'str': str(x)}
    return {'result': sorted(x)}


def service_pass(fx):
    """A client pass (every request) and a node pass (PROPAGATEs + BATCHes)."""
    client = [(copy.deepcopy(c['req']), 'cli%d' % k) for k, c in enumerate(fx['cases'])]
    node = [(copy.deepcopy(p), 'Node%d' % (k % 4 + 2)) for k, p in enumerate(fx['propagates'])]
    node += [(copy.deepcopy(b), 'Node3') for b in fx['batches']]
    return client, node
