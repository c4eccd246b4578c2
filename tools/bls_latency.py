"""BLS host-call latency by batch size (pv_bls_verify_batch from host arrays):
25 node keys, one COMMIT message per 25 checks, signatures made on the GPU.
One JSON line per size: median / min ms of 5 calls after 2 untimed ones.

    python tools/bls_latency.py [sizes...]
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'indy-plenum_amd'))
from plenum_gpu import _native as nat  # noqa: E402
from plenum_gpu.bls import MultiSignatureValue  # noqa: E402

R = 0x2523648240000001ba344d8000000007ff9f800000000010a10000000000000d
GEN = bytes.fromhex(json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'tests', 'golden',
                                                'bls.json')))['generator_hex'])


def main(sizes):
    nat.tuning_from_env()   # applies the PV_* knobs that are set (explicit opt-in)
    nk = 25
    sks = np.frombuffer(b''.join((int.from_bytes(hashlib.sha256(b'k' + bytes([i])).digest(), 'big') % R)
                                 .to_bytes(32, 'big') for i in range(nk)), np.uint8).reshape(nk, 32)
    pks = nat.bls_pubkeys(GEN, sks)
    nat.bls_set_keys(GEN, pks)
    n = max(sizes)
    nm = (n + nk - 1) // nk
    msgs = [MultiSignatureValue(1, 'S' * 44, 'P' * 44, 'T%043d' % b, 1700000000 + b).as_single_value()
            for b in range(nm)]
    blob = np.frombuffer(b''.join(msgs), np.uint8)
    off = np.zeros(nm + 1, np.uint64)
    off[1:] = np.cumsum([len(m) for m in msgs])
    midx = (np.arange(n) // nk).astype(np.uint32)
    kidx = (np.arange(n) % nk).astype(np.uint32)
    sig = nat.bls_sign_arrays(sks, blob, off, midx, kidx)
    for m in sizes:
        nmm = int(midx[m - 1]) + 1
        args = (sig[:m], blob, off[:nmm + 1], midx[:m], kidx[:m])
        for _ in range(2):
            v = nat.bls_verify_arrays(*args)
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            v = nat.bls_verify_arrays(*args)
            ts.append(time.perf_counter() - t0)
        ts.sort()
        print(json.dumps({'checks': m, 'ms_median': round(ts[2] * 1e3, 3), 'ms_min': round(ts[0] * 1e3, 3),
                          'checks_per_s': round(m / ts[2]), 'all_valid': bool(v.all())}), flush=True)


if __name__ == '__main__':
    main([int(x) for x in sys.argv[1:]] or [1, 25, 250, 2048, 8192, 16384, 32768, 65536])
