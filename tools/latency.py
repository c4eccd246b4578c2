"""Host-buffer latency of pv_verify_batch vs batch size (256 B messages,
distinct keys, pinned staging): the Looper-pass regime of SURVEY.md 8(b).
Prints one JSON line per size.  Run on the GPU box:  python tools/latency.py"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'indy-plenum_amd'))


SIZES = [int(x) for x in os.environ.get('PV_LAT_SIZES', '1,16,100,256,1000,1024,2048,4096,8192,16384,32768,65536').split(',')]


def main():
    from plenum_gpu import _native as nat
    from plenum_gpu.device import SyntheticBatch
    nat.tuning_from_env()   # the A/B knobs: explicit opt-in (pv_init reads no env)
    nat.ensure_init()
    b = SyntheticBatch(0, max(SIZES), 256, cfg=2, first=99)
    pk, sig = b.pk.cpu().numpy(), b.sig.cpu().numpy()
    off = b.off.cpu().numpy().astype(np.uint64)
    blob = b.blob.cpu().numpy()[:int(off[-1])]
    want = ~b.tamper.cpu().numpy().astype(bool)
    lat = os.environ.get('PV_LAT_MAX')
    cached = os.environ.get('PV_LAT_CACHED') == '1'   # keys in the device key cache (keyed latency kernel)
    nat.keycache_clear()
    if cached:
        nat.keycache_add(pk)
    for n in SIZES:
        args = (pk[:n], sig[:n], blob[:int(off[n])], off[:n + 1])
        got = nat.verify_batch_arrays(*args, dedup_keys=False)
        ts = []
        for _ in range(10):
            t0 = time.perf_counter()
            nat.verify_batch_arrays(*args, dedup_keys=False)
            ts.append(time.perf_counter() - t0)
        print(json.dumps({'n': n, 'lat_max': lat or 'default', 'cached': cached, 'ms_min': round(min(ts) * 1e3, 3), 'ms_median': round(sorted(ts)[5] * 1e3, 3),
                          'verifies_per_s': round(n / min(ts)), 'mismatches': int((got != want[:n]).sum())}),
              flush=True)


if __name__ == '__main__':
    main()
