"""Row f3 on the GPU: batch SHA-256 and the RFC 6962 Merkle tree hash through
the C-ABI, against hashlib and the reference TreeHasher roots (tests/golden/merkle.json)."""
import hashlib
import os

import numpy as np
import pytest

import _merkle as mk

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=['all_gpu', 'dispatch'])
def gpu_min(request, monkeypatch):
    """'all_gpu': every batch / subtree through the GPU kernels (GPU_MIN_ITEMS = 0);
    'dispatch': the production size dispatch (small ones on hashlib)."""
    from plenum_gpu import merkle
    if request.param == 'all_gpu':
        monkeypatch.setattr(merkle, 'GPU_MIN_ITEMS', 0)
    return request.param


def test_sha256_batch_vs_hashlib():
    from plenum_gpu.merkle import sha256_batch
    rng = np.random.default_rng(9)
    msgs = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes()
            for n in list(range(0, 200)) + list(rng.integers(0, 5000, 300))]
    for prefix in (None, 0, 1):
        got = sha256_batch(msgs, prefix)
        pre = b'' if prefix is None else bytes([prefix])
        assert got == [hashlib.sha256(pre + m).digest() for m in msgs]


def test_merkle_roots_match_reference():
    from plenum_gpu.merkle import GpuTreeHasher, merkle_root
    fx = mk.fixture()
    th = GpuTreeHasher()
    for t in fx['trees']:
        assert th.hash_full_tree(fx['leaves'][:t['size']]).hex() == t['root'], t['size']
    root, lh = merkle_root(fx['leaves'][:70], with_leaf_hashes=True)
    assert [h.hex() for h in lh] == fx['leaf_hashes']
    assert th.hash_empty() == hashlib.sha256(b'').digest()
    assert th.hash_leaf(fx['leaves'][3]).hex() == fx['leaf_hashes'][3]
    for k, i in enumerate(range(0, 20, 2)):
        l, r = fx['leaves'][i][:32].ljust(32, b'x'), fx['leaves'][i + 1][:32].ljust(32, b'y')
        assert th.hash_children(l, r).hex() == fx['children'][k]


def test_hash_full_and_compact_tree_extend():
    """GpuTreeHasher._hash_full / _hash_fold (ledger/tree_hasher.py:30-69) ==
    the hashlib restatement for ragged ranges (subtree hashes and root), range
    roots == the reference fixture's roots, and a CompactMerkleTree-style
    sequence of append/extend calls (ledger/compact_merkle_tree.py:99-193)
    driven by the GPU hasher keeps the reference CompactMerkleTree's
    (tree_size, hashes, root) after every call (tests/golden/merkle_compact.json)."""
    from plenum_gpu.merkle import GpuTreeHasher
    fx = mk.fixture()
    leaves, th = fx['leaves'], GpuTreeHasher()
    roots = {t['size']: t['root'] for t in fx['trees']}
    for l, r in [(0, 0), (0, 1), (3, 4), (0, 2), (1, 4), (0, 5), (7, 20), (0, 64), (5, 1030), (0, 1030), (512, 1023)]:
        got = th._hash_full(leaves, l, r)
        assert got == mk.hash_full(leaves, l, r), (l, r)
        if l == 0 and r in roots:
            assert got[0].hex() == roots[r]
    with pytest.raises(IndexError):
        th._hash_full(leaves, 3, 2)
    with pytest.raises(IndexError):
        th._hash_full(leaves, 0, len(leaves) + 1)
    gpu, ref = mk.CompactTree(th), mk.CompactTree(mk.HashlibHasher())
    pos = 0
    for st in mk.compact_fixture():   # reference CompactMerkleTree states
        k = st['extend']
        gpu.extend(leaves[pos:pos + k])
        ref.extend(leaves[pos:pos + k])
        pos += k
        assert (gpu.size, gpu.hashes) == (ref.size, ref.hashes), pos
        assert gpu.size == st['tree_size'] and [h.hex() for h in gpu.hashes] == st['hashes'], pos
        assert gpu.root().hex() == st['root'] == ref.root().hex()
        if pos in roots:
            assert gpu.root().hex() == roots[pos]


def test_request_digests_match_request_key():
    import _ingress_cases as ic
    from plenum_gpu.merkle import request_digests
    fx = ic.load()
    assert request_digests([c['req'] for c in fx['cases']]) == [c['key'] for c in fx['cases']]


def test_full_size_root_and_device_path():
    """1M leaves x 256 B (the f3 bench shape): device path root == hashlib level-wise root."""
    import torch
    from plenum_gpu import _native as nat
    from plenum_gpu.device import _p, _stream
    n, ln = 1 << 20, 256
    rng = np.random.default_rng(1)
    data = rng.integers(0, 256, n * ln, dtype=np.uint8)
    leaves = [data[i * ln:(i + 1) * ln].tobytes() for i in range(n)]
    want = mk.mth_levelwise(leaves)
    dev = torch.device('cuda', 0)
    nat.ensure_init(1)
    blob = torch.zeros(n * ln + 16, dtype=torch.uint8, device=dev)
    blob[:n * ln] = torch.from_numpy(data).to(dev)
    off = (torch.arange(n + 1, dtype=torch.int64, device=dev) * ln)
    root = torch.zeros(32, dtype=torch.uint8, device=dev)
    nat._check('pv_merkle_root_device', nat.load().pv_merkle_root_device(_p(blob), _p(off), n, _p(None), _p(root), 0,
                                                                         _stream(dev)))
    assert bytes(root.cpu().numpy()) == want
    # odd sizes through the device path too, either side of the one-workgroup
    # tail (k_merkle_tail takes over at <= 256 nodes)
    for m in (1, 2, 3, 255, 256, 257, 1023, 1025, 2047, 2049, 4097, 6001):
        nat._check('pv_merkle_root_device', nat.load().pv_merkle_root_device(_p(blob), _p(off), m, _p(None), _p(root),
                                                                             0, _stream(dev)))
        assert bytes(root.cpu().numpy()) == mk.mth_levelwise(leaves[:m]), m
