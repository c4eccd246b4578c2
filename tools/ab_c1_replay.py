"""Interleaved A/B of authenticate_batch's replay on the C1 workload (10k
signed requests, one GPU verify per batch): the replay reusing the prefetch's
per-request values vs the plain per-request replay (both with the cyclic GC
paused for the call, as authenticate_batch does).  Run on the GPU box.
First measurement (before the pause): reuse median 123 ms, plain 61 ms, reuse
with GC off 49 ms (profiles/r02_ab_c1_replay.json)."""
import gc
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'indy-plenum_amd'))


def main():
    import torch
    from plenum_gpu import synth
    from plenum_gpu.client_authn import CoreAuthMixin, CoreAuthNr
    torch.cuda.set_device(0)
    reqs, ids = synth.c1_requests(10000)
    a = CoreAuthNr(['buy'], [], [])
    for idr, vk in ids:
        a.addIdr(idr, vk)
    want = [[idr] for idr, _ in ids]
    stock = CoreAuthMixin._replay_reuses_prefetch
    res = {'reuse': [], 'plain': []}
    for r in range(6):
        for mode in res:
            CoreAuthMixin._replay_reuses_prefetch = stock if mode != 'plain' else (lambda self: False)
            t0 = time.perf_counter()
            out = a.authenticate_batch(reqs, pause_gc=True)
            res[mode].append(time.perf_counter() - t0)
            assert out == want and gc.isenabled()
    CoreAuthMixin._replay_reuses_prefetch = stock
    print(json.dumps({k: {'ms_min': round(min(v) * 1e3, 2), 'ms_median': round(sorted(v)[3] * 1e3, 2)}
                      for k, v in res.items()}))


if __name__ == '__main__':
    main()
