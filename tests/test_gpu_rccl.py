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


def test_bench_self_launches_two_ranks_gloo_shared_gpu():
    """`bench.py --gpus 2` with no launcher starts its two rank processes itself
    (VERDICT r5 item 1); here they share GPU 0 over gloo.  The line must report
    n_gpus 2 and world size 2 from the process group, both ranks' devices, no
    mismatch (which includes the gathered quorum bits == synth.c3_expected over
    both ranks' batches) and keep cpu_baseline + roofline at N > 1."""
    env = {k: v for k, v in os.environ.items()
           if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT')}
    env.update(PV_BENCH_BACKEND='gloo', PV_BENCH_SHARE_GPU='1', HSA_ENABLE_IPC_MODE_LEGACY='0')
    p = subprocess.run([sys.executable, '-u', os.path.join(REPO, 'bench.py'), '--gpus', '2', '--config', 'c3',
                        '--steps', '2', '--warmup', '1', '--no-e2e'],
                       env=env, capture_output=True, text=True, timeout=420, cwd=REPO)
    assert p.returncode == 0, p.stderr[-3000:] + p.stdout[-2000:]
    lines = [ln for ln in p.stdout.strip().splitlines() if ln.startswith('{')]
    assert len(lines) == 1, p.stdout[-2000:]
    line = json.loads(lines[0])
    assert line['n_gpus'] == 2 and line['verdict_mismatches'] == 0, line
    r = line['ranks']
    assert r['world_size'] == 2 and r['backend'] == 'gloo' and r['launcher'] == 'self', r
    assert sorted(d['rank'] for d in r['devices']) == [0, 1] and all(d['device'] == 0 for d in r['devices'])
    assert line['cpu_baseline'] and line['cpu_baseline']['value'] > 0, line.get('cpu_baseline')
    assert line['roofline'] and line['roofline']['frac'] > 0
    assert line['batches_per_s'] > 0 and line['config']['batches_per_gpu'] == 100_000
