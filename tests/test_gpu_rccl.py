"""RCCL on the hardware at hand: the only collective of
SURVEY.md §8(e) -- the all-gather of verdict bitmaps (and C3's quorum bits) --
runs through a ONE-rank "nccl" process group on the lease's GPU, both from
plenum_gpu.dist (tests/_rccl_worker.py) and from bench.py's own loop with the
collective forced at world == 1 (--collective).  Each runs as a fresh child
process so RCCL is initialised before any other GPU call of that process."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env():
    return dict(os.environ, RANK='0', WORLD_SIZE='1', LOCAL_RANK='0', MASTER_ADDR='127.0.0.1',
                MASTER_PORT=str(_free_port()), HSA_ENABLE_IPC_MODE_LEGACY='0')


def test_one_rank_rccl_gathers_equal_local_verdicts():
    p = subprocess.run([sys.executable, '-u', os.path.join(HERE, '_rccl_worker.py')], env=_env(),
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out['backend'] == 'nccl' and out['world'] == 1, out
    for k in ('golden_ok', 'verdicts_ok', 'bitmap_gather_equals_local', 'bitmap_equals_packed',
              'quorum_gather_equals_local', 'quorums_ok'):
        assert out[k], (k, out)


def test_bench_loop_with_rccl_collective_at_one_rank():
    """bench.py's N > 1 data path (bitmap + quorum all-gathers on every step's
    stream, max-over-ranks timing, gathered-bytes checks) with RCCL at world 1"""
    p = subprocess.run([sys.executable, '-u', os.path.join(REPO, 'bench.py'), '--config', 'c3', '--n', '250000',
                        '--steps', '3', '--warmup', '1', '--collective', '--no-cpu-baseline', '--no-e2e'],
                       env=_env(), capture_output=True, text=True, timeout=300, cwd=REPO)
    assert p.returncode == 0, p.stderr[-3000:] + p.stdout[-2000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line['verdict_mismatches'] == 0, line
    assert 'RCCL' in line['config']['parallelism'], line['config']
