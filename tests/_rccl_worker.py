"""Child process of tests/test_gpu_rccl.py: a ONE-rank "nccl" (RCCL) process
group initialised on the lease's GPU before any other GPU call, then the
collectives of SURVEY.md §8(e) on device tensors -- plenum_gpu.dist's
gather_verdicts (packed verdict bitmaps of a real HIP verify) and
gather_quorums (per-3PC-batch quorum bits from the tally kernel).  At one rank
the gathered bitmap must equal the local verdicts.  Prints one JSON line."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import conftest  # noqa: E402,F401  (sys.path)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    dev = torch.device('cuda', 0)
    # first GPU call of the process: RCCL's communicator on device 0
    dist.init_process_group('nccl', rank=0, world_size=1, device_id=dev)
    out = {'backend': dist.get_backend(), 'world': dist.get_world_size()}
    from plenum_gpu import _native as nat
    from plenum_gpu import synth
    from plenum_gpu.device import SyntheticBatch
    from plenum_gpu.dist import gather_quorums, gather_verdicts, pack_bits, verify_sharded, words_per_rank
    # (1) the golden raw vectors (libsodium verdicts) through verify_sharded on a device bitmap
    r = dict(np.load(os.path.join(HERE, 'golden', 'raw_vectors.npz')))
    got = verify_sharded(r['pk'], r['sig'], r['blob'], r['off'], 0, 1,
                         lambda pk, sig, blob, off: nat.verify_batch_arrays(pk, sig, blob, off), device=dev)
    out['golden_ok'] = bool((got == r['verdict'].astype(bool)).all())
    # (2) a device-resident C3-shape batch: verify, bitmap all-gather, tally, quorum all-gather
    nn, nb = 25, 4000
    b = SyntheticBatch(0, nn * nb, 0, cfg=3, first=0, mode=synth.COMMIT, n_nodes=nn)   # bench.py's C3 spec
    b.use_key_cache(True, wide=True)
    b.verify()
    torch.cuda.synchronize()
    verdict = b.verdict.cpu().numpy().astype(bool)
    n = verdict.size
    words = words_per_rank(n, 1)
    bm = b.bitmap[:words].contiguous()
    gathered = gather_verdicts(bm, n, 1)
    out['bitmap_gather_equals_local'] = bool((gathered == verdict).all())
    out['verdicts_ok'] = bool((verdict == ~b.tamper.cpu().numpy().astype(bool)).all())
    host_bm = torch.from_numpy(pack_bits(verdict, words).copy()).to(dev)
    out['bitmap_equals_packed'] = bool(torch.equal(bm, host_bm))
    from plenum_gpu.quorums import Quorums
    q = Quorums(nn).commit.value
    votes, reached = nat.tally_arrays(verdict.astype(np.uint8), b.sender.cpu().numpy(),
                                      np.arange(nb + 1, dtype=np.int64) * nn, nn, q)
    rt = torch.from_numpy(np.ascontiguousarray(reached).astype(np.uint8)).to(dev)
    g = gather_quorums(rt)
    out['quorum_gather_equals_local'] = bool(torch.equal(g.cpu(), rt.cpu()))
    want_votes, want_reached = synth.c3_expected(0, nb, nn, q)
    out['quorums_ok'] = bool((np.asarray(reached).astype(bool) == want_reached).all())
    out['n'] = int(n)
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
