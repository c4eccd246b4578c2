"""Quick GPU parity smoke: fixtures through the C-ABI (development aid)."""
import os, sys, time, ctypes
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'indy-plenum_amd'))
from plenum_gpu import _native as nat

t0 = time.time()
nat.ensure_init()
print('init', time.time() - t0, flush=True)
g = os.path.join(REPO, 'tests', 'golden')
r = np.load(os.path.join(g, 'raw_vectors.npz'))
t0 = time.time()
v = nat.verify_batch_arrays(r['pk'], r['sig'], r['blob'], r['off'])
print('raw: n=%d mismatches=%d time=%.3f' % (len(v), int((v != r['verdict'].astype(bool)).sum()), time.time() - t0), flush=True)
a = np.load(os.path.join(g, 'adversarial.npz'))
sm_off = a['sm_off']; blob = a['sm_blob']
pks, sigs, msgs, expect, labels = [], [], [], [], []
for k in range(len(a['label'])):
    sm = blob[int(sm_off[k]):int(sm_off[k + 1])].tobytes()
    if len(sm) < 64:
        continue
    pks.append(a['pk'][k]); sigs.append(np.frombuffer(sm[:64], np.uint8)); msgs.append(sm[64:])
    expect.append(bool(a['verdict'][k])); labels.append(str(a['label'][k]))
b, o = nat.pack_messages(msgs)
v = nat.verify_batch_arrays(np.array(pks), np.array(sigs), b, o)
bad = [labels[k] for k in range(len(v)) if v[k] != expect[k]]
print('adversarial: n=%d mismatches=%d %s' % (len(v), len(bad), bad[:20]), flush=True)
t = np.load(os.path.join(g, 'tally.npz'))
v = nat.verify_batch_arrays(t['pk'], t['sig'], t['blob'], t['off'])
print('tally verify mismatches', int((v != t['verdict'].astype(bool)).sum()), flush=True)
votes, reached = nat.tally_arrays(t['verdict'], t['sender'], t['batch_off'], int(t['n_nodes']), int(t['commit_quorum']))
print('tally votes mismatches', int((votes != t['vote_count']).sum()), 'reached mismatches', int((reached != t['commit_reached'].astype(bool)).sum()), flush=True)
# sign parity vs oracle
orc = ctypes.CDLL(os.path.join(REPO, 'oracle', 'liboracle.so'))
n = 300
rng = np.random.default_rng(5)
seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
msgs = [rng.integers(0, 256, int(rng.integers(0, 600)), dtype=np.uint8).tobytes() for _ in range(n)]
b, o = nat.pack_messages(msgs)
pk, sig = nat.sign_batch_arrays(seeds, b, o)
pk2 = np.zeros((n, 32), np.uint8); sig2 = np.zeros((n, 64), np.uint8)
orc.oracle_sign_batch(ctypes.c_void_p(seeds.ctypes.data), ctypes.c_void_p(b.ctypes.data), ctypes.c_void_p(o.ctypes.data), ctypes.c_uint64(n), ctypes.c_void_p(pk2.ctypes.data), ctypes.c_void_p(sig2.ctypes.data))
print('sign pk mismatches', int((pk != pk2).any(axis=1).sum()), 'sig mismatches', int((sig != sig2).any(axis=1).sum()), flush=True)
# throughput probe on 256 B messages
n = 1 << 17
seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
blob = rng.integers(0, 256, n * 256, dtype=np.uint8)
off = np.arange(n + 1, dtype=np.uint64) * 256
t0 = time.time(); pk, sig = nat.sign_batch_arrays(seeds, blob, off); print('sign %d: %.3f s' % (n, time.time() - t0), flush=True)
for rep in range(3):
    t0 = time.time(); v = nat.verify_batch_arrays(pk, sig, blob, off); dt = time.time() - t0
    print('verify %d: %.3f s -> %.3e/s (host-buffer path) all_valid=%s' % (n, dt, n / dt, bool(v.all())), flush=True)
