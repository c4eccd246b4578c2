"""Device-resident entry points for torch users (bench, multi-GPU ranks).

PyTorch is plumbing here: it owns HBM allocations and the stream; every
computation is a HIP kernel in libplenum_verify.so reached through the
C-ABI's *_device functions.  Tensors must live on the device the call names.
"""
import ctypes

import torch

from . import _native as nat


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class SyntheticBatch:
    """A signed synthetic batch resident in HBM (SoA: pk, sig, blob+off).

    mode: synth.FIXED (C2, len = mlen), synth.RANGE (C4, len uniform in
    [mlen, mlen_max]), synth.COMMIT (C3: n signatures = n / n_nodes 3PC
    batches of COMMIT votes; `sender` holds each vote's node index)."""

    def __init__(self, device, n, mlen, cfg=2, first=0, key_mod=0, mode=0, mlen_max=None, n_nodes=25):
        self.device = torch.device('cuda', device) if isinstance(device, int) else device
        nat.ensure_init(1 << self.device.index)
        dev = self.device
        self.n, self.mlen, self.cfg, self.first, self.mode = n, mlen, cfg, first, mode
        self.n_nodes = n_nodes
        mlen_max = mlen if mlen_max is None else mlen_max
        u8 = dict(dtype=torch.uint8, device=dev)
        lib = nat.load()
        self.off = torch.empty(n + 1, dtype=torch.int64, device=dev)
        nat._check('pv_synth_layout_device',
                   lib.pv_synth_layout_device(cfg, mode, first, n, mlen, mlen_max, n_nodes, _p(self.off), dev.index,
                                              _stream(dev)))
        self.blob_bytes = int(self.off[n].item())
        self.blob = torch.empty(self.blob_bytes + 16, **u8)
        self.seeds = torch.empty((n, 32), **u8)
        self.pk = torch.empty((n, 32), **u8)
        self.sig = torch.empty((n, 64), **u8)
        self.tamper = torch.empty(n, **u8)
        self.sender = torch.empty(n, dtype=torch.int32, device=dev)
        self.verdict = torch.empty(n, **u8)
        self.bitmap = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
        nat._check('pv_synth_fill_device',
                   lib.pv_synth_fill_device(cfg, mode, first, n, key_mod, n_nodes, _p(self.off), _p(self.blob),
                                            _p(self.seeds), _p(self.pk), _p(self.sig), _p(self.tamper),
                                            _p(self.sender), dev.index, _stream(dev)))

    def verify(self):
        """One pass of the hot path over the batch (hash + curve kernels)."""
        lib = nat.load()
        nat._check('pv_verify_batch_device',
                   lib.pv_verify_batch_device(_p(self.pk), _p(self.sig), _p(self.blob), _p(self.off), self.n,
                                              _p(self.verdict), _p(self.bitmap), self.device.index,
                                              _stream(self.device)))
        return self.verdict

    def time_kernels(self, iters):
        """Average (hash_ms, curve_ms) per launch from HIP events on the launch stream."""
        lib = nat.load()
        a, b = ctypes.c_float(), ctypes.c_float()
        nat._check('pv_time_verify_device',
                   lib.pv_time_verify_device(_p(self.pk), _p(self.sig), _p(self.blob), _p(self.off), self.n,
                                             _p(self.verdict), _p(self.bitmap), self.device.index,
                                             _stream(self.device), iters, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value


def verify_device(pk, sig, blob, off, verdict, bitmap=None):
    """Verify device-resident SoA tensors; blob needs >= 16 bytes of tail padding."""
    dev = pk.device
    nat.ensure_init(1 << dev.index)
    n = pk.shape[0]
    nat._check('pv_verify_batch_device',
               nat.load().pv_verify_batch_device(_p(pk), _p(sig), _p(blob), _p(off), n, _p(verdict), _p(bitmap),
                                                 dev.index, _stream(dev)))
    return verdict


def tally_device(verdict, sender, batch_off, n_nodes, quorum, votes, reached):
    dev = verdict.device
    nat.ensure_init(1 << dev.index)
    nb = batch_off.shape[0] - 1
    nat._check('pv_tally_device',
               nat.load().pv_tally_device(_p(verdict), _p(sender), _p(batch_off), nb, n_nodes, quorum, _p(votes),
                                          _p(reached), dev.index, _stream(dev)))
    return votes, reached
