"""Host-buffer calls of pv_verify_batch on the C2 batch (1M x 256 B): verdict
mismatches against the synthetic tamper mask and call times (ms), pageable and
page-locked inputs, one JSON line (A/B of library builds via PLENUM_GPU_LIB):
  python3 tools/e2e_calls.py [calls]"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'indy-plenum_amd'))


def main():
    from plenum_gpu import _native as nat
    from plenum_gpu.device import SyntheticBatch
    nat.tuning_from_env()
    nat.ensure_init()
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    b = SyntheticBatch(0, 1000000, 256, cfg=2)
    pk, sig = b.pk.cpu().numpy(), b.sig.cpu().numpy()
    off = b.off.cpu().numpy().astype(np.uint64)
    blob = b.blob.cpu().numpy()[:int(off[-1])]
    want = ~b.tamper.cpu().numpy().astype(bool)
    out = {'lib': os.path.basename(os.environ.get('PLENUM_GPU_LIB', 'default'))}
    locked = [torch.from_numpy(np.ascontiguousarray(a)).pin_memory().numpy() for a in (pk, sig, blob, off)]
    for name, args in (('pageable', (pk, sig, blob, off)), ('locked', locked)):
        mism = 0
        for _ in range(2):
            mism += int((nat.verify_batch_arrays(*args, dedup_keys=False) != want).sum())
        calls = []
        for _ in range(reps):
            t0 = time.perf_counter()
            got = nat.verify_batch_arrays(*args, dedup_keys=False)
            calls.append(round((time.perf_counter() - t0) * 1e3, 3))
            mism += int((got != want).sum())
        out[name] = {'mean_ms': round(sum(calls) / reps, 3), 'median_ms': sorted(calls)[reps // 2], 'calls_ms': calls,
                     'mismatches': mism}
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
