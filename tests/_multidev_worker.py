"""Child process of tests/test_gpu_multidev.py: pv_test_init_dup(2) (test-only
init entry point) opens two engine devices on HIP device 0, so pv_verify_batch with a two-device mask runs
its multi-device branch (one worker thread per device, each run_shard on its
own streams, workspaces and page-locked rings; errors aggregated per shard --
csrc/pv_api.cpp pv_verify_batch).  Prints one JSON line."""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), 'indy-plenum_amd'))
sys.path.insert(0, HERE)


def main():
    from plenum_gpu import _native as nat
    nat.test_init_dup(2)
    out = {'devices': nat.load().pv_device_count()}
    r = dict(np.load(os.path.join(HERE, 'golden', 'raw_vectors.npz')))
    want = r['verdict'].astype(bool)
    for mask in (0, 0b11, 0b10):
        for dedup in (True, False):
            got = nat.verify_batch_arrays(r['pk'], r['sig'], r['blob'], r['off'], device_mask=mask, dedup_keys=dedup)
            out['golden_mask{}_dedup{}'.format(mask, int(dedup))] = bool((got == want).all())
    # the persistent key cache on both engine devices: every golden key cached,
    # shards of Looper-pass size (mask 0b11 splits 1,000 signatures 500 / 500)
    nat.keycache_add(r['pk'])
    for n_small in (1, 1000, 3000):
        o = r['off'][:n_small + 1]
        got = nat.verify_batch_arrays(r['pk'][:n_small], r['sig'][:n_small], r['blob'][:int(o[-1])], o,
                                      device_mask=0b11)
        out['keycache_{}'.format(n_small)] = bool((got == want[:n_small]).all())
    nat.keycache_clear()
    # a C4-shaped batch: 300k signatures, 128 B - 4 KB messages, a pool of 4096
    # keys (the dedup flag takes the keyed path), 5 % tampered
    rng = np.random.default_rng(44)
    n = 300_000
    lens = rng.integers(128, 4097, n).astype(np.uint64)
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum(lens)
    blob = rng.integers(0, 256, int(off[-1]), dtype=np.uint8)
    pool = rng.integers(0, 256, (4096, 32), dtype=np.uint8)
    seeds = pool[rng.integers(0, 4096, n)]
    pk, sig = nat.sign_batch_arrays(seeds, blob, off)
    bad = rng.choice(n, n // 20, replace=False)
    sig[bad[: len(bad) // 2], 33] ^= 1
    blob[off[bad[len(bad) // 2:]].astype(np.int64)] ^= 0x80
    expect = np.ones(n, bool)
    expect[bad] = False
    for dedup in (True, False):
        got = nat.verify_batch_arrays(pk, sig, blob, off, device_mask=0b11, dedup_keys=dedup)
        out['c4_dedup{}'.format(int(dedup))] = bool((got == expect).all())
    # an error inside shard 1 only (offsets decrease in the middle of the
    # second half): the call fails, and the message names device 1
    off2 = off.copy()
    j = 3 * n // 4
    off2[j] = off2[j + 1] + 1
    try:
        nat.verify_batch_arrays(pk, sig, blob, off2, device_mask=0b11)
        out['shard_error'] = None
    except nat.PlenumGpuError as ex:
        out['shard_error'] = str(ex)
    # a shard boundary that decreases: rejected before any shard runs
    off3 = off.copy()
    off3[n // 2] = off3[n] + 1000
    try:
        nat.verify_batch_arrays(pk, sig, blob, off3, device_mask=0b11)
        out['boundary_error'] = None
    except nat.PlenumGpuError as ex:
        out['boundary_error'] = str(ex)
    # the engine still works after both errors
    got = nat.verify_batch_arrays(pk[:5000], sig[:5000], blob, off[:5001], device_mask=0b11)
    out['after_errors'] = bool((got == expect[:5000]).all())
    print(json.dumps(out))


if __name__ == '__main__':
    main()
