"""N > 1 path on CPU: world_size-2 gloo ranks shard the batch, verify their
shard (the oracle stands in for the GPU here), and all-gather the packed
verdict bitmaps; the gathered verdicts must equal the golden ones."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from plenum_gpu.dist import pack_bits, shard_range, unpack_gathered, words_per_rank

HERE = os.path.dirname(os.path.abspath(__file__))


def test_shards_cover_and_bitmaps_roundtrip():
    rng = np.random.default_rng(0)
    for n in (0, 1, 63, 64, 65, 1000, 4097):
        for world in (1, 2, 3, 4, 8):
            ranges = [shard_range(n, r, world) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == n
            assert all(ranges[r][1] == ranges[r + 1][0] for r in range(world - 1))
            v = rng.integers(0, 2, n).astype(bool)
            w = words_per_rank(n, world)
            gathered = np.concatenate([pack_bits(v[s:e], w) for s, e in ranges]) if n else np.zeros(0, np.int64)
            if n:
                assert (unpack_gathered(gathered, n, world) == v).all()


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    try:
        sys.path.insert(0, HERE)
        import conftest  # noqa: F401  (sets sys.path)
        import torch.distributed as dist
        import _oracle as orc
        from plenum_gpu.dist import verify_sharded
        os.environ['MASTER_ADDR'] = '127.0.0.1'
        os.environ['MASTER_PORT'] = str(port)
        dist.init_process_group('gloo', rank=rank, world_size=world)
        r = dict(np.load(os.path.join(HERE, 'golden', 'raw_vectors.npz')))
        n = 777
        off = r['off'][:n + 1]
        got = verify_sharded(r['pk'][:n], r['sig'][:n], r['blob'][:int(off[-1])], off, rank, world,
                             orc.verify_batch)
        ok = bool((got == r['verdict'][:n].astype(bool)).all())
        dist.destroy_process_group()
        q.put((rank, ok))
    except Exception as ex:  # pragma: no cover - reported to the parent
        q.put((rank, repr(ex)))


@pytest.mark.parametrize('world', [2])
def test_gloo_sharded_verify_allgather(world):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert sorted(res) == [(r, True) for r in range(world)], res


def _tally_worker(rank, world, port, q):
    try:
        sys.path.insert(0, HERE)
        import conftest  # noqa: F401
        import torch
        import torch.distributed as dist
        from plenum_gpu import synth
        from plenum_gpu.dist import gather_quorums
        os.environ['MASTER_ADDR'] = '127.0.0.1'
        os.environ['MASTER_PORT'] = str(port)
        dist.init_process_group('gloo', rank=rank, world_size=world)
        n_nodes, nb = 25, 300
        # rank r owns 3PC batches [r*nb, (r+1)*nb): verdicts from the C3 spec, tally rank-local
        # (the GPU tally kernel is covered by tests/test_gpu_tally.py; here the
        # rank-local voter sets are counted in Python, the collective is real)
        first = rank * nb
        reached = np.zeros(nb, bool)
        for j, b in enumerate(range(first, first + nb)):
            snd, bad = synth.c3_slots(b, n_nodes)
            reached[j] = len(set(snd[~bad].tolist())) >= 17
        got = gather_quorums(torch.from_numpy(reached.astype(np.uint8))).numpy().astype(bool)
        _, want = synth.c3_expected(0, world * nb, n_nodes, 17)
        dist.destroy_process_group()
        q.put((rank, bool((got == want).all())))
    except Exception as ex:  # pragma: no cover
        q.put((rank, repr(ex)))


def test_gloo_c3_quorum_bits_allgather():
    """C3 over 2 ranks: batches shard by batch, each rank tallies its own, the
    per-batch quorum bits are all-gathered and equal the spec's voter-set count."""
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tally_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert sorted(res) == [(r, True) for r in range(world)], res
