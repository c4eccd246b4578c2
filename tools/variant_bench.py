"""Interleaved A/B timing of library variants in ONE process (guide §5.4 rule 24).

    python tools/variant_bench.py lib_a.so lib_b.so ... [--n N --rounds R]

Each variant is loaded with its own ctypes handle, pv_init'ed, and times the
verify kernels (HIP events on the launch stream) over the same device-resident
synthetic C2 batch; verdicts must agree across variants.
"""
import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'indy-plenum_amd'))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from plenum_gpu import _native as nat  # noqa: E402
from plenum_gpu.device import SyntheticBatch, _p  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('libs', nargs='+')
    ap.add_argument('--n', type=int, default=1_000_000)
    ap.add_argument('--rounds', type=int, default=5)
    ap.add_argument('--mode', type=int, default=0, help='synth layout: 0 FIXED (C2), 1 RANGE (C4), 2 COMMIT (C3)')
    ap.add_argument('--mlen', type=int, default=256)
    ap.add_argument('--mlen-max', type=int, default=None)
    ap.add_argument('--key-mod', type=int, default=0)
    ap.add_argument('--cfg', type=int, default=2)
    ap.add_argument('--keyed', action='store_true', help='prepared-key path (key pool --key-mod or COMMIT node keys)')
    ap.add_argument('--no-check', action='store_true', help='timing experiments whose verdicts are knowingly wrong')
    a = ap.parse_args()
    b = SyntheticBatch(0, a.n, a.mlen, cfg=a.cfg, mode=a.mode, mlen_max=a.mlen_max, key_mod=a.key_mod)
    torch.cuda.synchronize()
    tamper = b.tamper.cpu().numpy().astype(bool)
    libs = []
    for path in a.libs:
        lib = ctypes.CDLL(os.path.abspath(path))
        for name, res, args in nat.SIGNATURES:
            if not hasattr(lib, name):
                continue
            getattr(lib, name).restype = res
            getattr(lib, name).argtypes = args
        assert lib.pv_init(1) == 0, lib.pv_last_error()
        libs.append((os.path.basename(path), lib))
    res = {n: [] for n, _ in libs}
    keys = b.key_index() if a.keyed else None
    kms = {}
    if a.keyed:
        assert keys is not None, 'keyed timing needs --key-mod or --mode 2'
        ktab = torch.empty(keys[0].shape[0] * nat.PV_KEY_WORDS, dtype=torch.int32, device=b.device)
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for r in range(a.rounds):
        for name, lib in libs:
            h, c = ctypes.c_float(), ctypes.c_float()
            b.verdict.zero_()
            if keys is not None:
                upk, kidx = keys
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                assert lib.pv_keys_prepare_device(_p(upk), upk.shape[0], _p(ktab), 0, stream) == 0, lib.pv_last_error()
                e1.record()
                e1.synchronize()
                kms.setdefault(name, []).append(e0.elapsed_time(e1))
                rc = lib.pv_time_verify_keyed_device(_p(ktab), _p(kidx), _p(upk), _p(b.sig), _p(b.blob), _p(b.off),
                                                     a.n, _p(b.verdict), _p(b.bitmap), 0, stream, 2,
                                                     ctypes.byref(h), ctypes.byref(c))
            else:
                rc = lib.pv_time_verify_device(_p(b.pk), _p(b.sig), _p(b.blob), _p(b.off), a.n, _p(b.verdict),
                                               _p(b.bitmap), 0, stream, 2, ctypes.byref(h), ctypes.byref(c))
            assert rc == 0, lib.pv_last_error()
            v = b.verdict.cpu().numpy().astype(bool)
            assert a.no_check or (v == ~tamper).all(), name
            res[name].append((h.value, c.value))
    out = {}
    for name, vals in res.items():
        cs = sorted(v[1] for v in vals)
        hs = sorted(v[0] for v in vals)
        out[name] = {'curve_ms_median': cs[len(cs) // 2], 'curve_ms_min': cs[0], 'hash_ms_median': hs[len(hs) // 2],
                     'verifies_per_s_kernel': a.n / ((cs[len(cs) // 2] + hs[len(hs) // 2]) * 1e-3)}
        if name in kms:
            ks = sorted(kms[name])
            out[name]['keys_ms_median'] = ks[len(ks) // 2]
            out[name]['distinct_keys'] = int(keys[0].shape[0])
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
