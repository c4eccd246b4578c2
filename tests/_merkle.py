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


def compact_fixture():
    """Reference CompactMerkleTree states after each append/extend
    (oracle/gen_compact_merkle.py)."""
    with open(os.path.join(GOLDEN, 'merkle_compact.json')) as fh:
        return json.load(fh)['steps']


def fixture():
    with open(os.path.join(GOLDEN, 'merkle.json')) as fh:
        d = json.load(fh)
    d['leaves'] = [bytes.fromhex(x) for x in d['leaves']]
    return d


def hash_full(leaves, l_idx, r_idx):
    """ledger/tree_hasher.py:30-62 TreeHasher._hash_full restated with hashlib."""
    width = r_idx - l_idx
    if width == 0:
        return hashlib.sha256(b'').digest(), ()
    if width == 1:
        h = leaf(leaves[l_idx])
        return h, (h,)
    split = 2 ** ((width - 1).bit_length() - 1)
    l_root, l_hashes = hash_full(leaves, l_idx, l_idx + split)
    r_root, r_hashes = hash_full(leaves, l_idx + split, r_idx)
    root = node(l_root, r_root)
    return root, ((root,) if split * 2 == width else l_hashes + r_hashes)


class CompactTree:
    """ledger/compact_merkle_tree.py:13-193 CompactMerkleTree's (tree_size, hashes)
    state under append/extend, restated over a pluggable hasher (no hash store):
    _push_subtree :99-141, __push_subtree_hash :143-158, extend :167-193."""

    def __init__(self, hasher):
        self.h, self.size, self.hashes = hasher, 0, ()

    def _min_h(self):
        return (self.size & -self.size).bit_length()

    def _push_hash(self, sub_h, sub_hash):
        size, min_h = 1 << (sub_h - 1), self._min_h()
        if sub_h < min_h or min_h == 0:
            self.size, self.hashes = self.size + size, self.hashes + (sub_hash,)
            return
        prev = self.hashes[-1]
        self.size, self.hashes = self.size - size, self.hashes[:-1]
        self._push_hash(sub_h + 1, self.h.hash_children(prev, sub_hash))

    def _push_subtree(self, leaves):
        root, _ = self.h._hash_full(leaves, 0, len(leaves))
        self._push_hash((len(leaves) & -len(leaves)).bit_length(), root)

    def extend(self, new_leaves):
        size, idx = len(new_leaves), 0
        while True:
            max_h = self._min_h()
            max_size = 1 << (max_h - 1) if max_h > 0 else 0
            if max_h > 0 and size - idx >= max_size:
                self._push_subtree(new_leaves[idx:idx + max_size])
                idx += max_size
            else:
                break
        if idx < size:
            root, hashes = self.h._hash_full(new_leaves, idx, size)
            self.size, self.hashes = self.size + size - idx, self.hashes + tuple(hashes)

    def root(self):
        return self.h._hash_fold(self.hashes) if self.hashes else self.h.hash_empty()


class HashlibHasher:
    """TreeHasher restated with hashlib (checker side of CompactTree)."""

    def hash_empty(self):
        return hashlib.sha256(b'').digest()

    def hash_children(self, l, r):
        return node(l, r)

    def _hash_full(self, leaves, l_idx, r_idx):
        return hash_full(leaves, l_idx, r_idx)

    def _hash_fold(self, hashes):
        rev = iter(hashes[::-1])
        acc = next(rev)
        for cur in rev:
            acc = node(cur, acc)
        return acc
