"""bench.py --gpus N means N GPUs: the rank plan is decided
before any GPU call -- refuse a --gpus / WORLD_SIZE mismatch and more ranks
than visible GPUs, launch N rank children when no launcher started the ranks,
run as one rank under torch.distributed.run.  CPU only: nothing here reaches a
GPU (the refusals exit before the first one)."""
import os
import subprocess
import sys

import pytest

from conftest import REPO

sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_plan_refuses_gpus_world_size_mismatch():
    act, msg = bench.rank_plan(3, {'WORLD_SIZE': '2'}, visible=8)
    assert act == 'error' and '--gpus 3' in msg and 'WORLD_SIZE=2' in msg


def test_plan_refuses_more_ranks_than_gpus_unless_shared():
    act, msg = bench.rank_plan(8, {}, visible=1)
    assert act == 'error' and 'visible' in msg
    assert bench.rank_plan(8, {'WORLD_SIZE': '8'}, visible=4)[0] == 'error'
    assert bench.rank_plan(2, {'PV_BENCH_SHARE_GPU': '1'}, visible=1) == ('launch', 2)
    assert bench.rank_plan(0, {}, visible=8)[0] == 'error'
    assert bench.rank_plan(None, {'WORLD_SIZE': 'x'}, visible=8)[0] == 'error'


def test_plan_launch_run_and_launcher_world():
    assert bench.rank_plan(None, {}, visible=0) == ('run', 1)
    assert bench.rank_plan(1, {}, visible=0) == ('run', 1)
    assert bench.rank_plan(8, {}, visible=8) == ('launch', 8)
    # under torch.distributed.run every rank runs; --gpus may be omitted
    assert bench.rank_plan(8, {'WORLD_SIZE': '8', 'RANK': '3'}, visible=8) == ('run', 8)
    assert bench.rank_plan(None, {'WORLD_SIZE': '4'}, visible=8) == ('run', 4)


@pytest.mark.parametrize('argv,env,needle', [
    (['--gpus', '3'], {'WORLD_SIZE': '2', 'RANK': '0'}, 'WORLD_SIZE=2'),
    (['--gpus', '64'], {}, 'visible'),
    (['--gpus', '2', '--config', 'c1'], {'PV_BENCH_SHARE_GPU': '1'}, None),
])
def test_bench_exits_nonzero_before_any_gpu_call(argv, env, needle):
    e = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK')}
    e.update(env)
    if needle is None:
        # a one-GPU line under a launcher of 2 ranks: refused by each rank
        e.update(WORLD_SIZE='2', RANK='0')
        needle = 'one-GPU line'
    p = subprocess.run([sys.executable, os.path.join(REPO, 'bench.py')] + argv, env=e, cwd=REPO,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 2, (p.returncode, p.stderr[-2000:])
    assert needle in p.stderr and not p.stdout.strip()
