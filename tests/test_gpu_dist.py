"""N > 1 with the GPU in the loop: two ranks, launched as
fresh child processes, each run the real HIP verify on GPU 0 (shared) and
all-gather packed verdict bitmaps over gloo (tests/_gpu_dist_worker.py).  The
RCCL form of the same gather is bench.py's production path; its CPU form is
tests/test_dist.py."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_ranks_hip_verify_allgather():
    world, port = 2, _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK='0', MASTER_ADDR='127.0.0.1',
                   MASTER_PORT=str(port), PV_DIST_N='100000')
        procs.append(subprocess.Popen([sys.executable, '-u', os.path.join(HERE, '_gpu_dist_worker.py')], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    res = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        assert p.returncode == 0, e[-3000:]
        res.append(json.loads(o.strip().splitlines()[-1]))
    assert sorted(x['rank'] for x in res) == list(range(world))
    for x in res:
        assert x['golden_ok'] and x['golden_n'] == 3000, x
        for tag in ('unkeyed', 'keyed'):
            assert x[tag + '_all_ok'] and x[tag + '_own_ok'], x
            assert 0.045 * world * 100000 < x[tag + '_tampered'] < 0.055 * world * 100000, x
