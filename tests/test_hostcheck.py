"""Host instrumentation build of the kernel algorithms (tools/hostcheck):
the exact per-lane schedule the HIP kernels run, compiled with g++, checked
against the golden fixtures with every field-multiply input bound-asserted,
plus op counts (the roofline's algorithmic work) and an ASan/UBSan run."""
import ctypes
import os
import random
import subprocess

import numpy as np
import pytest

import _oracle as orc
from conftest import REPO, split_sm

HC_DIR = os.path.join(REPO, 'tools', 'hostcheck')
P = 2 ** 255 - 19
L = 2 ** 252 + 27742317777372353535851937790883648493


def _load(name='libhostcheck.so'):
    subprocess.run(['make', '-s', '-C', HC_DIR, name], check=True)
    return ctypes.CDLL(os.path.join(HC_DIR, name))


@pytest.fixture(scope='module')
def hc():
    return _load()


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


def hc_verify(hc, pk, sig, blob, off):
    n = len(pk)
    v = np.zeros(n, np.uint8)
    pk = np.ascontiguousarray(pk, np.uint8)
    sig = np.ascontiguousarray(sig, np.uint8)
    b = orc.padded(blob)
    off = np.ascontiguousarray(off, np.uint64)
    hc.hc_verify_batch(_p(pk), _p(sig), _p(b), _p(off), ctypes.c_uint64(n), _p(v))
    return v.astype(bool)


def counts(hc):
    c = np.zeros(6, np.uint64)
    bad = hc.hc_get_counts(_p(c))
    return c, bad


def test_raw_vectors_bit_exact_and_bounded(hc, raw_vectors):
    r = raw_vectors
    sel = np.arange(0, len(r['verdict']), 5)
    pk, sig = r['pk'][sel], r['sig'][sel]
    msgs = [r['blob'][int(r['off'][i]):int(r['off'][i + 1])].tobytes() for i in sel]
    off = np.zeros(len(sel) + 1, np.uint64)
    off[1:] = np.cumsum([len(m) for m in msgs])
    hc.hc_reset_counts()
    got = hc_verify(hc, pk, sig, np.frombuffer(b''.join(msgs), np.uint8), off)
    _, bad = counts(hc)
    assert bad == 0, 'a field-multiply input exceeded the LOOSE bound'
    assert (got == r['verdict'][sel].astype(bool)).all()


def test_adversarial_bit_exact(hc, adversarial):
    rows = [row for row in split_sm(adversarial) if len(row[2]) >= 64]
    pk = np.stack([np.frombuffer(r[1], np.uint8) for r in rows])
    sig = np.stack([np.frombuffer(r[2][:64], np.uint8) for r in rows])
    msgs = [r[2][64:] for r in rows]
    off = np.zeros(len(rows) + 1, np.uint64)
    off[1:] = np.cumsum([len(m) for m in msgs])
    hc.hc_reset_counts()
    got = hc_verify(hc, pk, sig, np.frombuffer(b''.join(msgs), np.uint8), off)
    _, bad = counts(hc)
    assert bad == 0
    wrong = [rows[k][0] for k in range(len(rows)) if got[k] != rows[k][3]]
    assert not wrong, wrong


def test_sign_matches_oracle(hc):
    rng = np.random.default_rng(11)
    n = 40
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    msgs = [rng.integers(0, 256, int(rng.integers(0, 300)), dtype=np.uint8).tobytes() for _ in range(n)]
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum([len(m) for m in msgs])
    blob = orc.padded(np.frombuffer(b''.join(msgs), np.uint8))
    pk = np.zeros((n, 32), np.uint8)
    sig = np.zeros((n, 64), np.uint8)
    hc.hc_sign_batch(_p(seeds), _p(blob), _p(off), ctypes.c_uint64(n), _p(pk), _p(sig))
    pk2, sig2 = orc.sign_batch(seeds, blob[:-16], off)
    assert (pk == pk2).all() and (sig == sig2).all()


def _fe_bytes(x):
    return x.to_bytes(32, 'little')


def _fe_cases():
    rnd = random.Random(5)
    vals = [0, 1, 2, 19, P - 1, P, P + 1, 2 ** 255 - 1, 2 ** 254, 2 ** 26 - 1, 2 ** 26]
    vals += [rnd.randrange(2 ** 255) for _ in range(200)]
    return vals


def test_field_mul_sq_inv_vs_bigint(hc):
    out = ctypes.create_string_buffer(32)
    vals = _fe_cases()
    for a in vals:
        b = vals[(vals.index(a) * 7 + 3) % len(vals)]
        hc.hc_fe_mul(_fe_bytes(a), _fe_bytes(b), out)
        assert int.from_bytes(out.raw, 'little') == (a * b) % P
        hc.hc_fe_sq(_fe_bytes(a), out)
        assert int.from_bytes(out.raw, 'little') == (a * a) % P
        hc.hc_fe_invert(_fe_bytes(a), out)
        assert int.from_bytes(out.raw, 'little') == pow(a % P, P - 2, P)


def test_scalar_reduce_and_muladd_vs_bigint(hc):
    rnd = random.Random(9)
    out = ctypes.create_string_buffer(32)
    cases = [0, 1, L - 1, L, L + 1, 2 * L, 2 ** 512 - 1, 2 ** 256, (2 ** 252) * L] + \
            [rnd.randrange(2 ** 512) for _ in range(300)]
    for x in cases:
        hc.hc_sc_reduce64(x.to_bytes(64, 'little'), out)
        assert int.from_bytes(out.raw, 'little') == x % L
    for _ in range(300):
        a, b, c = (rnd.randrange(2 ** 256) for _ in range(3))
        hc.hc_sc_muladd(a.to_bytes(32, 'little'), b.to_bytes(32, 'little'), c.to_bytes(32, 'little'), out)
        assert int.from_bytes(out.raw, 'little') == (a * b + c) % L


def test_op_counts_pin_bench_constants(hc):
    """The curve kernel's algorithmic work per verify (bench.py W_*), counted on
    the exact kernel schedule: groups of CURVE_K = 4 signatures share the final
    inversion."""
    import bench
    n = 16
    seeds = np.frombuffer(os.urandom(32 * n), np.uint8).reshape(n, 32)
    blob = np.frombuffer(os.urandom(256 * n), np.uint8)
    off = np.arange(n + 1, dtype=np.uint64) * 256
    pk, sig = orc.sign_batch(seeds, blob, off)
    hc.hc_btable((ctypes.c_uint32 * (4 * 129 * 32))())  # base-point table outside the counted region
    hc.hc_reset_counts()
    assert hc_verify(hc, pk, sig, blob, off).all()
    c, bad = counts(hc)
    assert bad == 0
    assert int(c[1]) == int(bench.W_SQ_PER_VERIFY * n)
    # decompression multiplies by sqrt(-1) for about half of all keys
    assert (bench.W_MUL_PER_VERIFY - 0.5) * n <= int(c[0]) <= (bench.W_MUL_PER_VERIFY + 0.5) * n
    assert int(c[4]) == 3 * n  # SHA-512 blocks for |R||A||M| = 320 B


def test_asan_ubsan_run(adversarial):
    """Host code under AddressSanitizer/UBSan (no GPU sanitizers on this pool)."""
    so = os.path.join(HC_DIR, 'libhostcheck_asan.so')
    subprocess.run(['make', '-s', '-C', HC_DIR, 'libhostcheck_asan.so'], check=True)
    import sys
    code = r'''
import ctypes, numpy as np, sys
sys.path.insert(0, {tests!r})
from conftest import split_sm
hc = ctypes.CDLL({so!r})
a = dict(np.load({fx!r}))
rows = [r for r in split_sm(a) if 64 <= len(r[2]) <= 5000]
pk = np.stack([np.frombuffer(r[1], np.uint8) for r in rows])
sig = np.stack([np.frombuffer(r[2][:64], np.uint8) for r in rows])
msgs = [r[2][64:] for r in rows]
off = np.zeros(len(rows) + 1, np.uint64); off[1:] = np.cumsum([len(m) for m in msgs])
blob = np.concatenate([np.frombuffer(b''.join(msgs), np.uint8), np.zeros(16, np.uint8)])
v = np.zeros(len(rows), np.uint8)
P = lambda x: ctypes.c_void_p(x.ctypes.data)
hc.hc_verify_batch(P(pk), P(sig), P(blob), P(off), ctypes.c_uint64(len(rows)), P(v))
assert all(bool(v[k]) == rows[k][3] for k in range(len(rows)))
print('ok', len(rows))
'''.format(tests=os.path.dirname(__file__), so=so, fx=os.path.join(os.path.dirname(__file__), 'golden', 'adversarial.npz'))
    asan = subprocess.run(['gcc', '-print-file-name=libasan.so'], capture_output=True, text=True).stdout.strip()
    env = dict(os.environ, LD_PRELOAD=asan, ASAN_OPTIONS='detect_leaks=0', UBSAN_OPTIONS='halt_on_error=1')
    r = subprocess.run([sys.executable, '-c', code], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert 'runtime error' not in r.stderr, r.stderr


def _adv_arrays(adversarial):
    """adversarial fixture as SoA arrays with the reference's sig||msg framing (len(sm) >= 64 only)."""
    rows = [(pk, sm, v) for _, pk, sm, v in split_sm(adversarial) if len(sm) >= 64]
    pk = np.frombuffer(b''.join(r[0] for r in rows), np.uint8).reshape(-1, 32)
    sig = np.frombuffer(b''.join(r[1][:64] for r in rows), np.uint8).reshape(-1, 64)
    msgs = [r[1][64:] for r in rows]
    off = np.zeros(len(rows) + 1, np.uint64)
    off[1:] = np.cumsum([len(m) for m in msgs])
    return pk, sig, np.frombuffer(b''.join(msgs), np.uint8), off, np.array([r[2] for r in rows])


def test_keyed_path_adversarial_bit_exact(hc, adversarial):
    """Prepared-key path (key_prepare + keyed curve): every adversarial key
    (small order, non-canonical, off-curve, mixed order) and signature gives
    the fixture's verdict."""
    pk, sig, blob, off, want = _adv_arrays(adversarial)
    upk, kidx = np.unique(pk, axis=0, return_inverse=True)
    kidx = np.ascontiguousarray(kidx.reshape(-1), np.uint32)
    upk = np.ascontiguousarray(upk, np.uint8)
    n = len(pk)
    v = np.zeros(n, np.uint8)
    b = orc.padded(blob)
    hc.hc_reset_counts()
    sig = np.ascontiguousarray(sig)
    off = np.ascontiguousarray(off)
    hc.hc_verify_keyed(_p(upk), ctypes.c_uint64(len(upk)), _p(kidx), _p(sig), _p(b), _p(off), ctypes.c_uint64(n), _p(v))
    _, bad = counts(hc)
    assert bad == 0
    assert (v.astype(bool) == want).all()


def test_op_counts_pin_keyed_constants(hc):
    """Work split of the prepared-key (comb) path (bench.py W_*_KEYED / W_*_KEYPREP):
    16 signatures under ONE prepared key vs 16 keys prepared."""
    import bench
    n = 16
    seeds = np.frombuffer(os.urandom(32 * n), np.uint8).reshape(n, 32)
    blob = np.frombuffer(os.urandom(256 * n), np.uint8)
    off = np.arange(n + 1, dtype=np.uint64) * 256
    pk, sig = orc.sign_batch(seeds, blob, off)
    hc.hc_btable((ctypes.c_uint32 * (4 * 129 * 32))())
    v = np.zeros(n, np.uint8)

    def run(upk, kidx, s, b):
        bp = orc.padded(b)   # keep the buffer alive across the call
        hc.hc_reset_counts()
        hc.hc_verify_keyed(_p(upk), ctypes.c_uint64(len(upk)), _p(kidx), _p(s), _p(bp), _p(off),
                           ctypes.c_uint64(n), _p(v))
        assert v.all()
        c, bad = counts(hc)
        assert bad == 0
        return c
    c_many = run(np.ascontiguousarray(pk), np.arange(n, dtype=np.uint32), np.ascontiguousarray(sig), blob)
    one = np.ascontiguousarray(pk[:1])
    c_one = run(one, np.zeros(n, np.uint32), np.ascontiguousarray(np.repeat(sig[:1], n, 0)), np.tile(blob[:256], n))
    prep_sq = (int(c_many[1]) - int(c_one[1])) / (n - 1)
    assert prep_sq == bench.W_SQ_KEYPREP
    assert (int(c_one[1]) - prep_sq) / n == bench.W_SQ_KEYED
    # the decompression multiplies by sqrt(-1) for about half of all keys
    prep_mul = (int(c_many[0]) - int(c_one[0])) / (n - 1)
    assert abs(prep_mul - bench.W_MUL_KEYPREP) <= 1.0
    assert abs((int(c_one[0]) - prep_mul) / n - bench.W_MUL_KEYED) <= 0.2
