"""Debug helper: one host-buffer verify through pv_verify_batch, full error text."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'indy-plenum_amd'))
import numpy as np  # noqa: E402
from plenum_gpu import _native as nat  # noqa: E402

nat.tuning_from_env()   # the A/B knobs: explicit opt-in (pv_init reads no env)
nat.ensure_init()
rng = np.random.default_rng(0)
for n in (1, 2, 5, 64, 1000):
    for dedup in (False, True):
        pk = rng.integers(0, 256, (n, 32), dtype=np.uint8)
        sig = rng.integers(0, 256, (n, 64), dtype=np.uint8)
        blob = rng.integers(0, 256, 40 * n, dtype=np.uint8)
        off = np.arange(n + 1, dtype=np.uint64) * 40
        try:
            v = nat.verify_batch_arrays(pk, sig, blob, off, dedup_keys=dedup)
            print(n, dedup, 'ok', int(v.sum()), flush=True)
        except Exception as ex:  # noqa: BLE001
            print(n, dedup, 'ERR', ex, flush=True)
            sys.exit(1)
