"""One rank of the 2-rank GPU rehearsal (tests/test_gpu_dist.py): every rank
runs the REAL HIP verify on GPU 0 (shared), and the ranks all-gather packed
verdict bitmaps over gloo — the N > 1 data path of bench.py / plenum_gpu.dist
with the GPU in it.  Started as a fresh child process per rank (never an exec
of a GPU process).  Prints one JSON line with this rank's checks."""
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
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    n_c4 = int(os.environ.get('PV_DIST_N', '100000'))
    from plenum_gpu import _native as nat
    from plenum_gpu import synth
    from plenum_gpu.device import SyntheticBatch
    from plenum_gpu.dist import unpack_gathered, verify_sharded, words_per_rank
    dist.init_process_group('gloo', rank=rank, world_size=world)
    out = {'rank': rank}
    # (1) host-buffer HIP verify of the golden raw vectors (libsodium verdicts), sharded
    r = dict(np.load(os.path.join(HERE, 'golden', 'raw_vectors.npz')))
    got = verify_sharded(r['pk'], r['sig'], r['blob'], r['off'], rank, world,
                         lambda pk, sig, blob, off: nat.verify_batch_arrays(pk, sig, blob, off, device_mask=1))
    out['golden_ok'] = bool((got == r['verdict'].astype(bool)).all())
    out['golden_n'] = int(len(got))
    # (2) device-resident C4-shape shard per rank (ragged 128..4096 B, key pool 2^20),
    # unkeyed and keyed passes, bitmaps all-gathered
    b = SyntheticBatch(0, n_c4, 128, cfg=4, first=rank * n_c4, key_mod=1 << 20, mode=synth.RANGE, mlen_max=4096)
    n_all = world * n_c4
    words = words_per_rank(n_all, world)
    for keyed in (False, True):
        b.use_key_cache(keyed)
        b.bitmap.zero_()
        b.verify()
        torch.cuda.synchronize()
        mine = b.bitmap.cpu()
        g = torch.zeros(world * words, dtype=torch.int64)
        dist.all_gather_into_tensor(g, torch.nn.functional.pad(mine, (0, words - mine.numel())))
        t = torch.from_numpy(np.packbits(b.tamper.cpu().numpy().astype(np.uint8), bitorder='little'))
        tg = torch.zeros(world * t.numel(), dtype=torch.uint8)
        dist.all_gather_into_tensor(tg, t)
        tamper_all = np.unpackbits(tg.numpy(), bitorder='little').reshape(world, -1)[:, :n_c4].reshape(-1).astype(bool)
        v_all = unpack_gathered(g.numpy(), n_all, world)
        verdict = b.verdict.cpu().numpy().astype(bool)
        tag = 'keyed' if keyed else 'unkeyed'
        out[tag + '_all_ok'] = bool((v_all == ~tamper_all).all())
        out[tag + '_own_ok'] = bool((v_all[rank * n_c4:(rank + 1) * n_c4] == verdict).all())
        out[tag + '_tampered'] = int((~v_all).sum())
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
