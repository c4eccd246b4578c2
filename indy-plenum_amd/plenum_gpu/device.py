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
        self.n_nodes, self.key_mod = n_nodes, key_mod
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
        self.keys = None   # (unique pk (k,32), key index (n,)) once use_key_cache() ran
        self.ktab = None
        self.wide = False  # wide (radix-256) key format: node keys

    def key_index(self):
        """(unique keys, key index) of this batch from the synth spec: COMMIT
        votes use the sender node's key, a key pool key (first + j) mod key_mod."""
        dev = self.device
        if self.mode == 2:
            k = self.n_nodes
            kidx = self.sender.to(torch.int64)
        elif self.key_mod:
            k = min(self.key_mod, self.n)
            kidx = (torch.arange(self.n, dtype=torch.int64, device=dev) + self.first) % self.key_mod
        else:
            return None
        # one signature per key holds its bytes: the first occurrence
        first = torch.full((k if self.mode == 2 else self.key_mod,), -1, dtype=torch.int64, device=dev)
        pos = torch.arange(self.n, dtype=torch.int64, device=dev)
        first.scatter_reduce_(0, kidx, pos, reduce='amin', include_self=False)
        if (first < 0).any():
            # key pool larger than the batch: index only the keys present
            present = torch.nonzero(first >= 0).flatten()
            remap = torch.full_like(first, -1)
            remap[present] = torch.arange(present.numel(), device=dev)
            kidx = remap[kidx]
            first = first[present]
        return self.pk[first].contiguous(), kidx.to(torch.int32).contiguous()

    def use_key_cache(self, on=True, wide=False):
        """Verify through prepared keys (pv_keys_prepare_device + keyed kernels);
        wide: the radix-256 key format (pv_keys_prepare_wide_device), for keys
        that sign many messages per preparation (node keys)."""
        if not on:
            self.keys = self.ktab = None
            self.wide = False
            return False
        ki = self.key_index()
        if ki is None:
            return False
        self.keys = ki
        self.wide = bool(wide)
        words = nat.PV_KEY_WORDS_WIDE if self.wide else nat.PV_KEY_WORDS
        self.ktab = torch.empty(ki[0].shape[0] * words, dtype=torch.int32, device=self.device)
        return True

    def prepare_keys(self):
        upk, _ = self.keys
        fn = 'pv_keys_prepare_wide_device' if self.wide else 'pv_keys_prepare_device'
        nat._check(fn, getattr(nat.load(), fn)(_p(upk), upk.shape[0], _p(self.ktab), self.device.index,
                                               _stream(self.device)))

    def verify(self):
        """One pass of the hot path over the batch (hash + curve kernels; with
        the key cache: key preparation + keyed hash + keyed curve)."""
        lib = nat.load()
        if self.keys is not None:
            self.prepare_keys()
            upk, kidx = self.keys
            fn = 'pv_verify_keyed_wide_device' if self.wide else 'pv_verify_keyed_device'
            nat._check(fn, getattr(lib, fn)(_p(self.ktab), _p(kidx), _p(upk), _p(self.sig), _p(self.blob),
                                            _p(self.off), self.n, _p(self.verdict), _p(self.bitmap),
                                            self.device.index, _stream(self.device)))
            return self.verdict
        nat._check('pv_verify_batch_device',
                   lib.pv_verify_batch_device(_p(self.pk), _p(self.sig), _p(self.blob), _p(self.off), self.n,
                                              _p(self.verdict), _p(self.bitmap), self.device.index,
                                              _stream(self.device)))
        return self.verdict

    def make_slots(self):
        """Output buffers for two batches in flight (pipelined steps): slot 0 is
        (verdict, bitmap, ktab), slot 1 a second set.  Call after use_key_cache."""
        self.slot_out = [(self.verdict, self.bitmap, self.ktab),
                         (torch.empty_like(self.verdict), torch.zeros_like(self.bitmap),
                          None if self.ktab is None else torch.empty_like(self.ktab))]

    def verify_async(self, slot, stream, keys_beside=True):
        """Enqueue one pass of the hot path on `stream` with workspace/output
        `slot` (pv_*_async): returns (verdict, bitmap) of the slot without
        waiting.  Two passes in flight must use different slots.  With the key
        cache, keys_beside prepares the keys on the slot's side stream while the
        hash stage runs (pv_verify_keys_device_async); False runs the two
        stages one after the other on `stream`."""
        lib = nat.load()
        verdict, bitmap, ktab = self.slot_out[slot]
        s = ctypes.c_void_p(stream.cuda_stream)
        dev = self.device.index
        if self.keys is not None and keys_beside:
            upk, kidx = self.keys
            nat._check('pv_verify_keys_device_async',
                       lib.pv_verify_keys_device_async(_p(upk), upk.shape[0], _p(ktab), _p(kidx), _p(self.sig),
                                                       _p(self.blob), _p(self.off), self.n, _p(verdict), _p(bitmap),
                                                       int(self.wide), dev, s, slot))
        elif self.keys is not None:
            upk, kidx = self.keys
            w = '_wide' if self.wide else ''
            fp, fv = 'pv_keys_prepare{}_device_async'.format(w), 'pv_verify_keyed{}_device_async'.format(w)
            nat._check(fp, getattr(lib, fp)(_p(upk), upk.shape[0], _p(ktab), dev, s, slot))
            nat._check(fv, getattr(lib, fv)(_p(ktab), _p(kidx), _p(upk), _p(self.sig), _p(self.blob), _p(self.off),
                                            self.n, _p(verdict), _p(bitmap), dev, s, slot))
        else:
            nat._check('pv_verify_batch_device_async',
                       lib.pv_verify_batch_device_async(_p(self.pk), _p(self.sig), _p(self.blob), _p(self.off),
                                                        self.n, _p(verdict), _p(bitmap), dev, s, slot))
        return verdict, bitmap

    def time_kernels(self, iters):
        """Average (hash_ms, curve_ms) per launch from HIP events on the launch stream."""
        lib = nat.load()
        a, b = ctypes.c_float(), ctypes.c_float()
        if self.keys is not None:
            if self.wide:
                raise NotImplementedError('kernel timing of the wide key format: use _native.kernel_timing')
            upk, kidx = self.keys
            nat._check('pv_time_verify_keyed_device',
                       lib.pv_time_verify_keyed_device(_p(self.ktab), _p(kidx), _p(upk), _p(self.sig), _p(self.blob),
                                                       _p(self.off), self.n, _p(self.verdict), _p(self.bitmap),
                                                       self.device.index, _stream(self.device), iters,
                                                       ctypes.byref(a), ctypes.byref(b)))
            return a.value, b.value
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


def tally_device_async(verdict, sender, batch_off, n_nodes, quorum, votes, reached, bad, stream=None):
    """Enqueue the quorum tally on `stream` (default: the current stream) without
    waiting; `bad` (int32 device tensor, zeroed by the caller) becomes nonzero if
    a sender index is out of range (pv_tally_votes_device_async)."""
    dev = verdict.device
    nat.ensure_init(1 << dev.index)
    nb = batch_off.shape[0] - 1
    s = ctypes.c_void_p(stream.cuda_stream) if stream is not None else _stream(dev)
    nat._check('pv_tally_votes_device_async',
               nat.load().pv_tally_votes_device_async(_p(verdict), _p(sender), _p(batch_off), nb, n_nodes, quorum,
                                                      _p(votes), _p(reached), _p(bad), dev.index, s))
    return votes, reached


def tally_device(verdict, sender, batch_off, n_nodes, quorum, votes, reached):
    dev = verdict.device
    nat.ensure_init(1 << dev.index)
    nb = batch_off.shape[0] - 1
    nat._check('pv_tally_votes_device',
               nat.load().pv_tally_votes_device(_p(verdict), _p(sender), _p(batch_off), nb, n_nodes, quorum,
                                                _p(votes), _p(reached), dev.index, _stream(dev)))
    return votes, reached
