"""Three host-buffer calls of pv_verify_batch on the C2 batch (1M x 256 B),
for a rocprofv3 kernel + memory-copy timeline of the pinned pipeline:
  rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d DIR -- python3 tools/e2e_trace.py"""
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
    for _ in range(4):
        t0 = time.perf_counter()
        nat.verify_batch_arrays(pk, sig, blob, off, dedup_keys=False)
        print('call ms', round((time.perf_counter() - t0) * 1e3, 3), 'at', time.perf_counter_ns(), flush=True)


if __name__ == '__main__':
    main()
