"""The multi-device branch of pv_verify_batch: a fresh child
process calls the test-only pv_test_init_dup(2) (two engine devices on GPU 0), so the
per-device worker threads, shard offset rebasing and per-shard error
aggregation run on a one-GPU box (tests/_multidev_worker.py)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def test_two_engine_devices_shard_and_fail_per_shard():
    p = subprocess.run([sys.executable, '-u', os.path.join(HERE, '_multidev_worker.py')],
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out['devices'] == 2, out
    assert {'keycache_1', 'keycache_1000', 'keycache_3000'} <= set(out), out
    for k, v in out.items():
        if k.startswith(('golden_', 'c4_', 'keycache_')) or k == 'after_errors':
            assert v is True, (k, out)
    assert out['shard_error'] and 'device 1' in out['shard_error'] and 'not monotone' in out['shard_error'], out
    assert out['boundary_error'] and 'shard 1' in out['boundary_error'], out
