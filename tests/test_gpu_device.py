"""Device-resident path (torch tensors through the *_device C-ABI entry
points): synthetic generator vs its host spec, and C2-size properties."""
import numpy as np
import pytest

import _oracle as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def torch_dev():
    import torch
    assert torch.cuda.is_available()
    return torch


def test_synth_matches_host_spec(torch_dev):
    from plenum_gpu import synth
    from plenum_gpu.device import SyntheticBatch
    n, mlen, first = 3000, 256, 123456
    b = SyntheticBatch(0, n, mlen, cfg=2, first=first)
    seeds, msgs, tamper = synth.host_batch(2, first, n, mlen)
    assert (b.seeds.cpu().numpy() == seeds).all()
    assert (b.tamper.cpu().numpy().astype(bool) == tamper).all()
    pk = b.pk.cpu().numpy()
    sig = b.sig.cpu().numpy()
    blob = b.blob.cpu().numpy()[:n * mlen]
    off = np.arange(n + 1, dtype=np.uint64) * mlen
    pk2, sig2 = orc.sign_batch(seeds, np.frombuffer(b''.join(msgs), np.uint8), off)
    assert (pk == pk2).all()
    for j in range(n):
        m2, s2 = (msgs[j], sig2[j].tobytes())
        if tamper[j]:
            m2, s2 = synth.apply_tamper(first + j, m2, s2)
        assert blob[j * mlen:(j + 1) * mlen].tobytes() == m2
        assert sig[j].tobytes() == s2
    v = b.verify().cpu().numpy().astype(bool)
    assert (v == ~tamper).all()
    want = orc.verify_batch(pk, sig, blob, off)
    assert (v == want).all()


def test_c2_full_size_properties(torch_dev):
    """BASELINE configs[1] size: 1M signatures, every tampered one rejected,
    every other accepted, bitmap == verdicts, idempotent across passes."""
    from plenum_gpu.device import SyntheticBatch
    n = 1_000_000
    b = SyntheticBatch(0, n, 256, cfg=2, first=0)
    v1 = b.verify().cpu().numpy().copy()
    tamper = b.tamper.cpu().numpy().astype(bool)
    assert (v1.astype(bool) == ~tamper).all()
    assert 0.045 < tamper.mean() < 0.055
    bits = np.unpackbits(b.bitmap.cpu().numpy().view(np.uint8), bitorder='little')[:n].astype(bool)
    assert (bits == v1.astype(bool)).all()
    v2 = b.verify().cpu().numpy()
    assert (v1 == v2).all()
    # spot-check against the oracle
    idx = np.random.default_rng(0).choice(n, 300, replace=False)
    pk = b.pk.cpu().numpy()[idx]
    sig = b.sig.cpu().numpy()[idx]
    blob_all = b.blob.cpu().numpy()
    msgs = b''.join(blob_all[i * 256:(i + 1) * 256].tobytes() for i in idx)
    want = orc.verify_batch(pk, sig, np.frombuffer(msgs, np.uint8), np.arange(301, dtype=np.uint64) * 256)
    assert (want == v1[idx].astype(bool)).all()


def test_kernel_timer(torch_dev):
    from plenum_gpu.device import SyntheticBatch
    b = SyntheticBatch(0, 65536, 256, cfg=2)
    th, tc = b.time_kernels(2)
    assert th > 0 and tc > 0 and tc > th
