"""A/B of the host-buffer chunk schedule on the C2 batch (1M x 256 B, pageable
inputs), interleaved, ms per call: pv_set_host_fused MODES (default "1 2").
Round 3 measured a build whose mode 1 ran the last chunk on the device
schedule beside the earlier chunks' deferred pass against mode 2 (all fused +
one deferred pass): equal (profiles/r03_ab_last_chunk_device_schedule_notadopted.jsonl,
code reverted); the current library has modes 1 (fused) and 0 (unfused).
python tools/ab_host_fused.py [reps] [modes...]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'indy-plenum_amd'))


def main(reps=8, modes=(1, 0)):
    from plenum_gpu import _native as nat
    from plenum_gpu.device import SyntheticBatch
    nat.tuning_from_env()   # the A/B knobs: explicit opt-in (pv_init reads no env)
    nat.ensure_init()
    b = SyntheticBatch(0, 1 << 20, 256, cfg=2, first=1)
    off = b.off.cpu().numpy().astype(np.uint64)
    pk, sig, blob = b.pk.cpu().numpy(), b.sig.cpu().numpy(), b.blob.cpu().numpy()[:int(off[-1])]
    want = ~b.tamper.cpu().numpy().astype(bool)
    ts = {m: [] for m in modes}
    bad = 0
    for r in range(reps + 1):
        for mode in modes:
            nat.set_host_fused(mode)
            t0 = time.perf_counter()
            got = nat.verify_batch_arrays(pk, sig, blob, off, dedup_keys=False)
            dt = time.perf_counter() - t0
            bad += int((got != want).sum())
            if r:
                ts[mode].append(dt * 1e3)
    nat.set_host_fused(1)
    for mode in modes:
        v = sorted(ts[mode])
        print(json.dumps({'host_fused': mode, 'ms_median': round(v[len(v) // 2], 3), 'ms_min': round(v[0], 3),
                          'verifies_per_s_median': round(len(want) / (v[len(v) // 2] / 1e3)), 'mismatches': bad}))


if __name__ == '__main__':
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 8, tuple(int(x) for x in sys.argv[2:]) or (1, 0))
