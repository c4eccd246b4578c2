"""Row f3 on the GPU: batch SHA-256 and the RFC 6962 Merkle tree hash through
the C-ABI, against hashlib and the reference TreeHasher roots (tests/golden/merkle.json)."""
import hashlib
import os

import numpy as np
import pytest

import _merkle as mk

pytestmark = pytest.mark.gpu


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
    # odd sizes through the device path too
    for m in (1, 2, 3, 1023, 1025):
        nat._check('pv_merkle_root_device', nat.load().pv_merkle_root_device(_p(blob), _p(off), m, _p(None), _p(root),
                                                                             0, _stream(dev)))
        assert bytes(root.cpu().numpy()) == mk.mth_levelwise(leaves[:m]), m
