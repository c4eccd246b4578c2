"""A/B of pv_verify_batch's host-buffer pipeline on the C2 batch (1M x 256 B):
staging mode, gather threads and chunk count (PV_HOST_CHUNKS is read at
pv_init, so each chunk count runs in its own process).  Prints one JSON line
per setting.  Run on the GPU box:  python tools/ab_staging.py [chunks]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'indy-plenum_amd'))


def main():
    from plenum_gpu import _native as nat
    from plenum_gpu.device import SyntheticBatch
    nat.tuning_from_env()   # the A/B knobs: explicit opt-in (pv_init reads no env)
    nat.ensure_init()
    b = SyntheticBatch(0, 1000000, 256, cfg=2)
    pk, sig = b.pk.cpu().numpy(), b.sig.cpu().numpy()
    off = b.off.cpu().numpy().astype(np.uint64)
    blob = b.blob.cpu().numpy()[:int(off[-1])]
    want = ~b.tamper.cpu().numpy().astype(bool)
    for staging, threads, dedup in (('pageable', 0, False), ('pinned', 1, False), ('pinned', 4, False),
                                    ('pinned', 8, False), ('pinned', 16, False), ('pinned', 8, True)):
        nat.set_host_staging(staging, threads)
        got = nat.verify_batch_arrays(pk, sig, blob, off, dedup_keys=dedup)
        mism = int((got != want).sum())
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            nat.verify_batch_arrays(pk, sig, blob, off, dedup_keys=dedup)
            ts.append(time.perf_counter() - t0)
        print(json.dumps({'chunks': os.environ.get('PV_HOST_CHUNKS', '4'), 'staging': staging, 'threads': threads, 'dedup': dedup,
                          'ms_min': round(min(ts) * 1e3, 3), 'ms_mean': round(sum(ts) / len(ts) * 1e3, 3),
                          'verifies_per_s': round(1e6 / min(ts)), 'mismatches': mism}), flush=True)
    # pooled keys (C4 shape: 2^16-key pool, 128 B - 4 KB) with and without dedup
    from plenum_gpu import synth
    b = SyntheticBatch(0, 1000000, 128, cfg=4, key_mod=1 << 16, mode=synth.RANGE, mlen_max=4096)
    pk, sig = b.pk.cpu().numpy(), b.sig.cpu().numpy()
    off = b.off.cpu().numpy().astype(np.uint64)
    blob = b.blob.cpu().numpy()[:int(off[-1])]
    want = ~b.tamper.cpu().numpy().astype(bool)
    nat.set_host_staging('pinned', 8)
    for dedup in (False, True):
        got = nat.verify_batch_arrays(pk, sig, blob, off, dedup_keys=dedup)
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            nat.verify_batch_arrays(pk, sig, blob, off, dedup_keys=dedup)
            ts.append(time.perf_counter() - t0)
        print(json.dumps({'pooled_keys': 1 << 16, 'dedup': dedup, 'ms_min': round(min(ts) * 1e3, 3),
                          'verifies_per_s': round(1e6 / min(ts)), 'mismatches': int((got != want).sum())}),
              flush=True)
    t0 = time.perf_counter()
    nat.verify_batch_arrays(pk[:1], sig[:1], blob[:int(off[1])], off[:2])
    print(json.dumps({'one_signature_ms': round((time.perf_counter() - t0) * 1e3, 3)}))


if __name__ == '__main__':
    main()
