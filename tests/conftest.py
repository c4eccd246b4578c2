import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, 'indy-plenum_amd')
GOLDEN = os.path.join(REPO, 'tests', 'golden')
if PKG not in sys.path:
    sys.path.insert(0, PKG)
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs the HIP kernels through the C-ABI)')
    config.addinivalue_line('markers', 'slow: long CPU test')


def golden(name):
    return os.path.join(GOLDEN, name)


@pytest.fixture(scope='session')
def raw_vectors():
    return dict(np.load(golden('raw_vectors.npz')))


@pytest.fixture(scope='session')
def adversarial():
    return dict(np.load(golden('adversarial.npz')))


@pytest.fixture(scope='session')
def tally_fx():
    return dict(np.load(golden('tally.npz')))


@pytest.fixture(scope='session')
def kat():
    import json
    with open(golden('kat.json')) as fh:
        return json.load(fh)


@pytest.fixture(scope='session')
def plenum_requests():
    import json
    with open(golden('plenum_requests.json')) as fh:
        return json.load(fh)


def split_sm(adv):
    """adversarial fixture -> list of (label, pk bytes, sm bytes, verdict)"""
    out = []
    off = adv['sm_off']
    for k in range(len(adv['label'])):
        sm = adv['sm_blob'][int(off[k]):int(off[k + 1])].tobytes()
        out.append((str(adv['label'][k]), adv['pk'][k].tobytes(), sm, bool(adv['verdict'][k])))
    return out
