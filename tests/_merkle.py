"""Merkle checker helpers (tests only): the RFC 6962 tree hash restated with
hashlib, level-wise (an odd last node moves up), and the reference fixture."""
import hashlib
import json
import os

from conftest import GOLDEN


def leaf(d):
    return hashlib.sha256(b'\x00' + d).digest()


def node(l, r):
    return hashlib.sha256(b'\x01' + l + r).digest()


def mth_levelwise(leaves):
    if not leaves:
        return hashlib.sha256(b'').digest()
    lvl = [leaf(d) for d in leaves]
    while len(lvl) > 1:
        nxt = [node(lvl[i], lvl[i + 1]) for i in range(0, len(lvl) - 1, 2)]
        if len(lvl) % 2:
            nxt.append(lvl[-1])
        lvl = nxt
    return lvl[0]


def fixture():
    with open(os.path.join(GOLDEN, 'merkle.json')) as fh:
        d = json.load(fh)
    d['leaves'] = [bytes.fromhex(x) for x in d['leaves']]
    return d
