"""Row f3 on CPU: the kernels' SHA-256 block loader and Merkle node (host
instrumentation build of pv_sha256.h) against hashlib, and the level-wise tree
shape the GPU uses against the reference TreeHasher / CompactMerkleTree roots."""
import ctypes
import hashlib
import os

import numpy as np

import _merkle as mk
import _oracle as orc
from test_hostcheck import _load


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


def test_sha256_block_loader_vs_hashlib():
    hc = _load()
    rng = np.random.default_rng(5)
    lens = list(range(0, 140)) + [183, 184, 191, 192, 255, 256, 1000, 4097]
    msgs = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in lens]
    blob = orc.padded(np.frombuffer(b''.join(msgs), np.uint8))
    off = np.zeros(len(msgs) + 1, np.uint64)
    off[1:] = np.cumsum([len(m) for m in msgs])
    for prefix in (-1, 0, 1, 0xab):
        out = np.zeros((len(msgs), 32), np.uint8)
        hc.hc_sha256(_p(blob), _p(off), ctypes.c_uint64(len(msgs)), ctypes.c_int(prefix), _p(out))
        pre = b'' if prefix < 0 else bytes([prefix])
        for i, m in enumerate(msgs):
            assert out[i].tobytes() == hashlib.sha256(pre + m).digest(), (prefix, len(m))


def test_sha256_node_vs_hashlib():
    hc = _load()
    for _ in range(50):
        lr = np.frombuffer(os.urandom(64), np.uint8).copy()
        out = np.zeros(32, np.uint8)
        hc.hc_sha256_node(_p(lr), _p(out))
        assert out.tobytes() == hashlib.sha256(b'\x01' + lr.tobytes()).digest()


def test_levelwise_shape_matches_reference_roots():
    fx = mk.fixture()
    for t in fx['trees']:
        assert mk.mth_levelwise(fx['leaves'][:t['size']]).hex() == t['root'], t['size']
    for i, h in enumerate(fx['leaf_hashes']):
        assert mk.leaf(fx['leaves'][i]).hex() == h


def test_compact_tree_restatement_vs_reference_states():
    """tests/_merkle.py CompactTree + hash_full (the checker the GPU test uses)
    reproduce the reference CompactMerkleTree's (tree_size, hashes, root) after
    every append/extend of oracle/gen_compact_merkle.py, and hash_full's roots
    match the reference TreeHasher roots of tests/golden/merkle.json."""
    import _merkle as mk
    fx = mk.fixture()
    leaves = fx['leaves']
    for t in fx['trees']:
        assert mk.hash_full(leaves, 0, t['size'])[0].hex() == t['root'], t['size']
    tree, pos = mk.CompactTree(mk.HashlibHasher()), 0
    for st in mk.compact_fixture():
        tree.extend(leaves[pos:pos + st['extend']])
        pos += st['extend']
        assert tree.size == st['tree_size'] == pos
        assert [h.hex() for h in tree.hashes] == st['hashes']
        assert tree.root().hex() == st['root'] == mk.mth_levelwise(leaves[:pos]).hex()


def test_small_work_never_touches_the_library(monkeypatch):
    """single hashes and small batches (CompactMerkleTree.append's
    hash_leaf + carry chain of hash_children, ledger/compact_merkle_tree.py:138-160)
    run on hashlib as the reference TreeHasher does — no GPU call per node — and
    match the reference fixtures."""
    from plenum_gpu import _native, merkle
    from plenum_gpu.merkle import GpuTreeHasher, merkle_root, sha256_batch

    def boom(*a, **k):
        raise AssertionError('GPU library used for a small batch')
    monkeypatch.setattr(_native, 'load', boom)
    monkeypatch.setattr(_native, 'ensure_init', boom)
    fx = mk.fixture()
    th = GpuTreeHasher()
    for t in fx['trees']:
        if t['size'] < merkle.GPU_MIN_ITEMS:
            assert th.hash_full_tree(fx['leaves'][:t['size']]).hex() == t['root']
    root, lh = merkle_root(fx['leaves'][:70], with_leaf_hashes=True)
    assert [h.hex() for h in lh] == fx['leaf_hashes']
    assert sha256_batch([b'abc'], prefix=None) == [hashlib.sha256(b'abc').digest()]
    tree = mk.CompactTree(th)
    pos = 0
    leaves = fx['leaves']
    for st in mk.compact_fixture():
        k = st['extend']
        if pos + k >= merkle.GPU_MIN_ITEMS:
            break
        tree.extend(leaves[pos:pos + k])
        pos += k
        assert tree.size == st['tree_size'] and [h.hex() for h in tree.hashes] == st['hashes']
        assert tree.root().hex() == st['root']
    for i in range(pos, pos + 50):        # append = extend by one leaf
        tree.extend([leaves[i % len(leaves)]])
    assert tree.size == pos + 50
