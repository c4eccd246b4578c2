"""Batch SHA-256 and Merkle tree hashing on the GPU.

* `sha256_batch(msgs, prefix=None)` -> list of 32-byte digests, one GPU pass
  (pv_sha256_batch).  `request_digests(reqs)` gives every request's
  `Request.key` (plenum/common/request.py:82-90) with the native serializer and
  one GPU pass.
* `GpuTreeHasher` mirrors ledger/tree_hasher.py `TreeHasher` (hash_empty,
  hash_leaf, hash_children, hash_full_tree, _hash_full, _hash_fold) with
  `hash_full_tree`, `hash_leaves` and `_hash_full` (CompactMerkleTree.extend's
  bulk step) computed on the GPU (pv_merkle_root): leaf = SHA-256(0x00 || data),
  node = SHA-256(0x01 || left || right), RFC 6962 shape.

Size dispatch (not a fallback): one GPU call costs tens to hundreds of
microseconds of launch + PCIe round trip, one SHA-256 of a leaf or an inner
node costs ~0.5 µs in hashlib.  So single hashes (`hash_leaf`,
`hash_children`, `_hash_fold`, `hash_empty` — what `CompactMerkleTree.append`
and its carry chain call per leaf, ledger/compact_merkle_tree.py:138-160) and
batches / subtrees below `GPU_MIN_ITEMS` items are hashed on the host with
hashlib, exactly as the reference TreeHasher does (ledger/tree_hasher.py:4,
21-28); larger batches and subtrees go to the GPU, which is required for them
(no CPU fallback there: a missing library or GPU raises).
"""
import ctypes
import hashlib

import numpy as np

from . import _native as nat

# batches / (sub)trees with fewer items than this are hashed on the host
# (profiles/r02_f3_small.jsonl: hashlib and one GPU call break even near
# 256 leaves of 256 B; the GPU is 2x faster at 1024); tests set it to 0 to
# push every size through the GPU kernels
GPU_MIN_ITEMS = 512


def _leaf(d):
    return hashlib.sha256(b'\x00' + bytes(d)).digest()


def _node(left, right):
    return hashlib.sha256(b'\x01' + bytes(left) + bytes(right)).digest()


def _host_mth(leaves):
    """RFC 6962 Merkle Tree Hash, level-wise (an odd last node moves up: the
    same shape as ledger/tree_hasher.py:45-62's split at the largest power of
    two below n)."""
    if not leaves:
        return hashlib.sha256(b'').digest(), []
    lh = [_leaf(d) for d in leaves]
    lvl = lh
    while len(lvl) > 1:
        nxt = [_node(lvl[i], lvl[i + 1]) for i in range(0, len(lvl) - 1, 2)]
        if len(lvl) & 1:
            nxt.append(lvl[-1])
        lvl = nxt
    return lvl[0], lh


def _pack(msgs):
    msgs = [bytes(m) for m in msgs]
    blob, off = nat.pack_messages(msgs)
    return np.ascontiguousarray(blob, np.uint8), np.ascontiguousarray(off, np.uint64)


def sha256_batch(msgs, prefix=None):
    """[bytes] -> [32-byte digest of (prefix || m)]; prefix None or a byte value."""
    n = len(msgs)
    if n == 0:
        return []
    if n < GPU_MIN_ITEMS:
        pre = b'' if prefix is None else bytes([int(prefix)])
        return [hashlib.sha256(pre + bytes(m)).digest() for m in msgs]
    nat.ensure_init()
    blob, off = _pack(msgs)
    out = np.zeros((n, 32), np.uint8)
    p = -1 if prefix is None else int(prefix)
    nat._check('pv_sha256_batch', nat.load().pv_sha256_batch(nat._ptr(blob), nat._ptr(off), n, p, nat._ptr(out)))
    return [out[i].tobytes() for i in range(n)]


def request_digests(reqs, plugin_fields=()):
    """Request(**r).key (sha256 hex of the signing state) for every request, one GPU pass."""
    from .ingress import signing_state
    from .serialization import serialize_msg_for_signing
    return [d.hex() for d in sha256_batch([serialize_msg_for_signing(signing_state(r, plugin_fields)) for r in reqs])]


def merkle_root(leaves, with_leaf_hashes=False):
    """RFC 6962 Merkle Tree Hash of `leaves` (bytes each) on the GPU."""
    n = len(leaves)
    if n < GPU_MIN_ITEMS:
        root, lh = _host_mth(leaves)
        return (root, lh) if with_leaf_hashes else root
    nat.ensure_init()
    blob, off = _pack(leaves)
    root = np.zeros(32, np.uint8)
    lh = np.zeros((max(n, 1), 32), np.uint8) if with_leaf_hashes else None
    nat._check('pv_merkle_root', nat.load().pv_merkle_root(nat._ptr(blob), nat._ptr(off), n, nat._ptr(root),
                                                           nat._ptr(lh) if lh is not None else ctypes.c_void_p(0)))
    if with_leaf_hashes:
        return root.tobytes(), [lh[i].tobytes() for i in range(n)]
    return root.tobytes()


class GpuTreeHasher:
    """ledger/tree_hasher.py TreeHasher with the bulk operations on the GPU."""

    def __repr__(self):
        return 'GpuTreeHasher()'

    def hash_empty(self):
        return hashlib.sha256(b'').digest()

    def hash_leaf(self, data):
        return _leaf(data)

    def hash_leaves(self, leaves):
        return sha256_batch(leaves, prefix=0x00)

    def hash_children(self, left, right):
        return _node(left, right)

    def hash_full_tree(self, leaves):
        return merkle_root(leaves)

    def _hash_full(self, leaves, l_idx, r_idx):
        """ledger/tree_hasher.py:30-62 TreeHasher._hash_full: (root, hashes) of
        leaves[l_idx:r_idx], hashes = roots of the full (2^k) subtrees that form
        the range, largest first ((root,) when the width is a power of two).
        CompactMerkleTree._push_subtree / extend (ledger/compact_merkle_tree.py:125,
        183) call it with whole batches of new leaves: each full subtree's
        root is one GPU Merkle Tree Hash over its leaves, and the range root is
        their right fold (the split at the largest power of two below the width
        is exactly the subtree decomposition, so the fold equals the MTH)."""
        if l_idx < 0 or r_idx < l_idx or r_idx > len(leaves):
            raise IndexError("{},{} not a valid range over [0,{}]".format(l_idx, r_idx, len(leaves)))
        width = r_idx - l_idx
        if width == 0:
            return self.hash_empty(), ()
        hashes, a = [], 0
        big = width >= GPU_MIN_ITEMS
        if big:
            nat.ensure_init()
            blob, off = _pack(leaves[l_idx:r_idx])   # packed once; each subtree is an offset window
            lib = nat.load()
        for bit in range(width.bit_length() - 1, -1, -1):
            if width >> bit & 1:
                if (1 << bit) < GPU_MIN_ITEMS:
                    hashes.append(_host_mth(leaves[l_idx + a:l_idx + a + (1 << bit)])[0])
                else:
                    root = np.zeros(32, np.uint8)
                    nat._check('pv_merkle_root', lib.pv_merkle_root(nat._ptr(blob), nat._ptr(off[a:]), 1 << bit,
                                                                    nat._ptr(root), ctypes.c_void_p(0)))
                    hashes.append(root.tobytes())
                a += 1 << bit
        hashes = tuple(hashes)
        if len(hashes) == 1:
            return hashes[0], hashes
        return self._hash_fold(hashes), hashes

    def _hash_fold(self, hashes):
        """ledger/tree_hasher.py:64-69: right fold of hash_children over `hashes`."""
        rev = iter(hashes[::-1])
        accum = next(rev)
        for cur in rev:
            accum = self.hash_children(cur, accum)
        return accum
