"""Host-buffer C2 call (1M x 256 B) from page-locked caller buffers (torch
pin_memory()): one JSON line for the current PV_HOST_ROUNDS setting (read at
pv_init).  Run on the GPU box: tools/gpu_locked.sh"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'indy-plenum_amd'))


def main():
    import torch
    from plenum_gpu import _native as nat
    from plenum_gpu.device import SyntheticBatch
    nat.tuning_from_env()   # the A/B knobs: explicit opt-in (pv_init reads no env)
    nat.ensure_init()
    b = SyntheticBatch(0, 1000000, 256, cfg=2)
    off = b.off.cpu().numpy().astype(np.uint64)
    t = [b.pk.cpu().pin_memory(), b.sig.cpu().pin_memory(), b.blob.cpu()[:int(off[-1])].pin_memory(),
         torch.from_numpy(off.view(np.int64)).pin_memory()]
    pk, sig, blob, loff = t[0].numpy(), t[1].numpy(), t[2].numpy(), t[3].numpy().view(np.uint64)
    want = ~b.tamper.cpu().numpy().astype(bool)
    got = nat.verify_batch_arrays(pk, sig, blob, loff, dedup_keys=False)
    nat.verify_batch_arrays(pk, sig, blob, loff, dedup_keys=False)
    ts = []
    for _ in range(8):
        t0 = time.perf_counter()
        nat.verify_batch_arrays(pk, sig, blob, loff, dedup_keys=False)
        ts.append(time.perf_counter() - t0)
    ts.sort()
    print(json.dumps({'inputs': 'page-locked', 'host_rounds': os.environ.get('PV_HOST_ROUNDS', '1'),
                      'ms_min': round(ts[0] * 1e3, 3), 'ms_median': round(ts[4] * 1e3, 3),
                      'mismatches': int((got != want).sum())}), flush=True)


if __name__ == '__main__':
    main()
