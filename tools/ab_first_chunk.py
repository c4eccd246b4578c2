"""Host-buffer C2 call (1M x 256 B, pinned staging) for one PV_HOST_CHUNKS /
PV_HOST_FIRST_PCT setting (both read at pv_init: one process per setting).
Prints one JSON line.  Run on the GPU box (tools/gpu_first_chunk.sh)."""
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
    got = nat.verify_batch_arrays(pk, sig, blob, off, dedup_keys=False)
    nat.verify_batch_arrays(pk, sig, blob, off, dedup_keys=False)
    ts = []
    for _ in range(8):
        t0 = time.perf_counter()
        nat.verify_batch_arrays(pk, sig, blob, off, dedup_keys=False)
        ts.append(time.perf_counter() - t0)
    ts.sort()
    print(json.dumps({'chunks': os.environ.get('PV_HOST_CHUNKS', '8'), 'first_pct': os.environ.get('PV_HOST_FIRST_PCT', '50'),
                      'staging': os.environ.get('PV_HOST_STAGING', 'pinned'),
                      'ms_min': round(ts[0] * 1e3, 3), 'ms_median': round(ts[4] * 1e3, 3),
                      'mismatches': int((got != want).sum())}), flush=True)


if __name__ == '__main__':
    main()
