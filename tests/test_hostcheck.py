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
    c = np.zeros(8, np.uint64)
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


def _signed_batch(n, seed):
    rng = np.random.default_rng(seed)
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    blob = rng.integers(0, 256, 256 * n, dtype=np.uint8)
    off = np.arange(n + 1, dtype=np.uint64) * 256
    pk, sig = orc.sign_batch(seeds, blob, off)
    return pk, sig, blob, off


def _run_mode(hc, pk, sig, blob, off, force_full):
    n = len(pk)
    v = np.zeros(n, np.uint8)
    nd = ctypes.c_uint64()
    b = orc.padded(blob)
    hc.hc_btable((ctypes.c_uint32 * (8 * 129 * 32))())  # base-point tables outside the counted region
    hc.hc_reset_counts()
    hc.hc_verify_batch_mode(_p(np.ascontiguousarray(pk)), _p(np.ascontiguousarray(sig)), _p(b),
                            _p(np.ascontiguousarray(off)), ctypes.c_uint64(n), _p(v), int(force_full), ctypes.byref(nd))
    c, bad = counts(hc)
    assert bad == 0, 'a field-multiply input exceeded the LOOSE bound'
    return v.astype(bool), c, nd.value


def test_op_counts_pin_bench_constants(hc):
    """The curve stage's algorithmic work per verify (bench.py W_*), counted on
    the exact kernel schedule: the half-size path (no deferred record in this
    seeded batch) and the full-length verdict every deferred record takes."""
    import bench
    n = 32
    pk, sig, blob, off = _signed_batch(n, 3)
    ok, c, nd = _run_mode(hc, pk, sig, blob, off, False)
    assert ok.all() and nd == 0
    assert int(c[1]) == int(bench.W_SQ_PER_VERIFY * n)
    # the decompressions of -A and -R each multiply by sqrt(-1) for about half of all points
    assert abs(int(c[0]) / n - bench.W_MUL_PER_VERIFY) <= 0.5
    assert int(c[4]) == 3 * n  # SHA-512 blocks for |R||A||M| = 320 B
    assert int(c[5]) == 2 * n  # h mod L, d S mod L
    ok, c, nd = _run_mode(hc, pk, sig, blob, off, True)
    assert ok.all() and nd == n
    assert int(c[1]) == int(bench.W_SQ_FULL * n)
    assert abs(int(c[0]) / n - bench.W_MUL_FULL) <= 0.5


def test_op_counts_pin_valu_constants(hc):
    """The algorithmic non-MAD work of the roofline's combined figure
    (bench.W_ADD / W_SUB / W_CARRY_PER_VERIFY), counted on the exact kernel
    schedule of a half-size verify with a 256-byte message.  The 3 SHA-512 blocks
    of R||A||M are counted too but not charged: they run in k_hash, not in the
    timed curve kernel."""
    import bench
    n = 32
    pk, sig, blob, off = _signed_batch(n, 3)
    ok, c, nd = _run_mode(hc, pk, sig, blob, off, False)
    assert ok.all() and nd == 0
    # the conditional sqrt(-1) multiply of the decompressions adds one fe_add
    assert abs(int(c[2]) / n - bench.W_ADD_PER_VERIFY) <= 1.0
    assert int(c[6]) == bench.W_SUB_PER_VERIFY * n
    assert abs(int(c[3]) / n - bench.W_CARRY_PER_VERIFY) <= 1.0
    assert int(c[7]) == bench.W_CARRY_EVEN_PER_VERIFY * n
    assert int(c[4]) == 3 * n
    assert bench.W_HALF_PER_VERIFY == 20 * bench.W_MUL_PER_VERIFY + 16 * bench.W_SQ_PER_VERIFY
    assert bench.W_HALF_PER_VERIFY > 0 and bench.W_FULL_PER_VERIFY > 0


def test_op_counts_pin_grouped_constants(hc):
    """curve_mode PV_CURVE_GROUPED: groups of CURVE_K = 8 signatures share the final inversion."""
    import bench
    n = 16
    pk, sig, blob, off = _signed_batch(n, 4)
    hc.hc_btable((ctypes.c_uint32 * (8 * 129 * 32))())
    hc.hc_reset_counts()
    v = np.zeros(n, np.uint8)
    b = orc.padded(blob)
    hc.hc_verify_batch_grouped(_p(pk), _p(sig), _p(b), _p(off), ctypes.c_uint64(n), _p(v))
    c, bad = counts(hc)
    assert bad == 0 and v.all()
    assert int(c[1]) == int(bench.W_SQ_GROUPED * n)
    assert abs(int(c[0]) / n - bench.W_MUL_GROUPED) <= 0.5


def test_half_and_full_paths_agree_on_fixtures(hc, raw_vectors, adversarial):
    """Every fixture verdict through the half-size path AND with every record
    forced through the full-length verdict (the two code paths of k_curve_half)."""
    r = raw_vectors
    sel = np.arange(0, len(r['verdict']), 3)
    msgs = [r['blob'][int(r['off'][i]):int(r['off'][i + 1])].tobytes() for i in sel]
    off = np.zeros(len(sel) + 1, np.uint64)
    off[1:] = np.cumsum([len(m) for m in msgs])
    blob = np.frombuffer(b''.join(msgs), np.uint8)
    want = r['verdict'][sel].astype(bool)
    for force in (False, True):
        got, _, nd = _run_mode(hc, r['pk'][sel], r['sig'][sel], blob, off, force)
        assert (got == want).all()
    pk, sig, blob, off, want = _adv_arrays(adversarial)
    for force in (False, True):
        got, _, nd = _run_mode(hc, pk, sig, blob, off, force)
        assert (got == want).all()



def _run_quad(hc, pk, sig, blob, off, force_full):
    n = len(pk)
    v = np.zeros(n, np.uint8)
    nd = ctypes.c_uint64()
    b = orc.padded(blob)
    hc.hc_btable((ctypes.c_uint32 * (8 * 129 * 32))())
    hc.hc_reset_counts()
    hc.hc_verify_batch_quad(_p(np.ascontiguousarray(pk)), _p(np.ascontiguousarray(sig)), _p(b),
                            _p(np.ascontiguousarray(off)), ctypes.c_uint64(n), _p(v), int(force_full), ctypes.byref(nd))
    _, bad = counts(hc)
    assert bad == 0, 'a field-multiply input exceeded the LOOSE bound'
    return v.astype(bool), nd.value


def test_lane_quad_schedule_on_fixtures(hc, raw_vectors, adversarial):
    """The latency kernel's lane-quad schedule (k_verify_quad, pv_quad.h) with the
    four lanes of a quad emulated in lockstep: every raw-vector and adversarial
    verdict, half-size records and every record in its deferred (full-length)
    form, every field-multiply input bound-checked."""
    r = raw_vectors
    sel = np.arange(0, len(r['verdict']), 7)
    msgs = [r['blob'][int(r['off'][i]):int(r['off'][i + 1])].tobytes() for i in sel]
    off = np.zeros(len(sel) + 1, np.uint64)
    off[1:] = np.cumsum([len(m) for m in msgs])
    blob = np.frombuffer(b''.join(msgs), np.uint8)
    want = r['verdict'][sel].astype(bool)
    for force in (False, True):
        got, nd = _run_quad(hc, r['pk'][sel], r['sig'][sel], blob, off, force)
        assert (got == want).all()
        if force:
            assert nd >= int(want.sum())
    pk, sig, blob, off, want = _adv_arrays(adversarial)
    for force in (False, True):
        got, _ = _run_quad(hc, pk, sig, blob, off, force)
        wrong = np.nonzero(got != want)[0]
        assert len(wrong) == 0, wrong


L8 = 8 * L
PAT33 = int('8' * 33, 16)


def _half(hc, h):
    c = ctypes.create_string_buffer(20)
    d = ctypes.create_string_buffer(20)
    neg = ctypes.c_uint32()
    st = hc.hc_half_scalars(h.to_bytes(32, 'little'), c, d, ctypes.byref(neg))
    return st, int.from_bytes(c.raw, 'little'), int.from_bytes(d.raw, 'little'), neg.value


def test_half_scalars_lattice_properties(hc):
    """c == d h (mod 8L), d odd and positive, |c| + 0x88..8 and d + 0x88..8 < 2^132
    (33 signed radix-16 digits) for every HS_HALF result; edge values of h; and
    the deferral rate of random h stays at the simulated ~0.2 %."""
    rnd = random.Random(17)
    cases = [0, 1, 2, 3, 8, L - 1, L - 2, 2 ** 128 - 1, 2 ** 128, 2 ** 128 + 1, 2 ** 252, L // 2, L // 3,
             (2 ** 252) // 7, 2 ** 200 + 3] + [rnd.randrange(L) for _ in range(4000)]
    deferred = 0
    for h in cases:
        st, c, d, neg = _half(hc, h)
        assert st in (1, 2)
        if st == 2:
            deferred += 1
            continue
        cs = -c if neg else c
        assert d % 2 == 1 and d > 0, h
        assert (cs - d * h) % L8 == 0, h
        assert c + PAT33 < 2 ** 132 and d + PAT33 < 2 ** 132, h
    assert _half(hc, 0)[0] == 1 and _half(hc, 5)[0] == 1   # tiny h: c = h, d = 1
    assert deferred / len(cases) < 0.01


def test_sc_mul_small_vs_bigint(hc):
    rnd = random.Random(23)
    out = ctypes.create_string_buffer(32)
    for _ in range(300):
        d = rnd.randrange(2 ** 132)
        s = rnd.randrange(L)
        hc.hc_sc_mul_small(d.to_bytes(20, 'little'), s.to_bytes(32, 'little'), out)
        assert int.from_bytes(out.raw, 'little') == (d * s) % L


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


def _run_keyed_wide(hc, pk, sig, blob, off):
    upk, kidx = np.unique(pk, axis=0, return_inverse=True)
    kidx = np.ascontiguousarray(kidx.reshape(-1), np.uint32)
    upk = np.ascontiguousarray(upk, np.uint8)
    n = len(pk)
    v = np.zeros(n, np.uint8)
    b = orc.padded(blob)
    hc.hc_reset_counts()
    hc.hc_verify_keyed_wide(_p(upk), ctypes.c_uint64(len(upk)), _p(kidx), _p(np.ascontiguousarray(sig)), _p(b),
                            _p(np.ascontiguousarray(off)), ctypes.c_uint64(n), _p(v))
    c, bad = counts(hc)
    assert bad == 0
    return v, c, len(upk)


def test_keyed_wide_adversarial_bit_exact(hc, adversarial):
    """Wide (radix-256) prepared keys: every adversarial key and signature gives
    the fixture's verdict through key_prepare_wide_slice + the wide comb, every
    multiply bound-checked."""
    pk, sig, blob, off, want = _adv_arrays(adversarial)
    v, _, _ = _run_keyed_wide(hc, pk, sig, blob, off)
    assert (v.astype(bool) == want).all()


def test_keyed_wide_raw_vectors_and_op_counts(hc, raw_vectors):
    """Raw vectors through the wide keyed path, and its work per verify / per
    prepared key pinned for the bench (bench.W_*_KEYED_WIDE, W_*_KEYPREP_WIDE)."""
    import bench
    r = raw_vectors
    pk, sig = r['pk'][:300], r['sig'][:300]
    off = r['off'][:301] - r['off'][0]
    blob = r['blob'][int(r['off'][0]):int(r['off'][300])]
    v, _, _ = _run_keyed_wide(hc, pk, sig, blob, off)
    assert (v == r['verdict'][:300]).all()
    # one signature verified 16 and 32 times under one prepared key: the
    # difference is the per-verify work, the rest the preparation (whose decode
    # of A, redone by all 128 lanes, takes a data-dependent extra multiply)
    seeds = np.frombuffer(os.urandom(32), np.uint8).reshape(1, 32)
    blob = np.frombuffer(os.urandom(256), np.uint8)
    spk, ssig = orc.sign_batch(seeds, blob, np.array([0, 256], np.uint64))
    hc.hc_btable((ctypes.c_uint32 * (8 * 129 * 32))())
    c = {}
    for n in (16, 32):
        off = np.arange(n + 1, dtype=np.uint64) * 256
        vb, c[n], k = _run_keyed_wide(hc, np.repeat(spk, n, 0), np.repeat(ssig, n, 0), np.tile(blob, n), off)
        assert vb.all() and k == 1
    per_mul, per_sq = [(int(c[32][i]) - int(c[16][i])) / 16 for i in (0, 1)]
    assert per_sq == bench.W_SQ_KEYED_WIDE
    assert abs(per_mul - bench.W_MUL_KEYED_WIDE) <= 0.6, per_mul
    prep_mul, prep_sq = [int(c[16][i]) - 16 * p for i, p in ((0, per_mul), (1, per_sq))]
    assert prep_sq == bench.W_SQ_KEYPREP_WIDE
    assert abs(prep_mul - bench.W_MUL_KEYPREP_WIDE) <= 128, prep_mul


def _run_keyed_quad(hc, pk, sig, blob, off, small=False):
    """small: the 4-signature-block form (8 comb sides per signature)"""
    upk, kidx = np.unique(pk, axis=0, return_inverse=True)
    kidx = np.ascontiguousarray(kidx.reshape(-1), np.uint32)
    upk = np.ascontiguousarray(upk, np.uint8)
    n = len(pk)
    v = np.zeros(n, np.uint8)
    b = orc.padded(blob)
    hc.hc_reset_counts()
    fn = hc.hc_verify_keyed_quad_small if small else hc.hc_verify_keyed_quad
    fn(_p(upk), ctypes.c_uint64(len(upk)), _p(kidx), _p(np.ascontiguousarray(sig)), _p(b),
       _p(np.ascontiguousarray(off)), ctypes.c_uint64(n), _p(v))
    _, bad = counts(hc)
    assert bad == 0
    return v


@pytest.mark.parametrize('small', [False, True], ids=['4sides', '8sides'])
def test_keyed_quad_schedule_adversarial_bit_exact(hc, adversarial, small):
    """Keyed latency kernel's schedule (k_verify_quad_keyed, pv_quad.h
    q_comb_side: each side's comb share on an emulated lane quad, -R added on
    side 1, the sides' exchange tree, identity test; the hash wave's split
    SHA-512), in both block forms (8 signatures x 4 sides; 4 x 8 for small
    calls): every adversarial case gives the fixture's verdict, every multiply
    bound-checked."""
    pk, sig, blob, off, want = _adv_arrays(adversarial)
    v = _run_keyed_quad(hc, pk, sig, blob, off, small)
    assert (v.astype(bool) == want).all()


@pytest.mark.parametrize('small', [False, True], ids=['4sides', '8sides'])
def test_keyed_quad_schedule_raw_vectors(hc, raw_vectors, small):
    r = raw_vectors
    sel = slice(0, 600)
    pk, sig = r['pk'][sel], r['sig'][sel]
    off = r['off'][:601] - r['off'][0]
    blob = r['blob'][int(r['off'][0]):int(r['off'][600])]
    v = _run_keyed_quad(hc, pk, sig, blob, off, small)
    assert (v == r['verdict'][sel]).all()


def test_op_counts_pin_keyed_constants(hc):
    """Work split of the prepared-key (comb) path (bench.py W_*_KEYED / W_*_KEYPREP):
    16 signatures under ONE prepared key vs 16 keys prepared."""
    import bench
    n = 16
    seeds = np.frombuffer(os.urandom(32 * n), np.uint8).reshape(n, 32)
    blob = np.frombuffer(os.urandom(256 * n), np.uint8)
    off = np.arange(n + 1, dtype=np.uint64) * 256
    pk, sig = orc.sign_batch(seeds, blob, off)
    hc.hc_btable((ctypes.c_uint32 * (8 * 129 * 32))())
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
    assert abs((int(c_one[0]) - prep_mul) / n - bench.W_MUL_KEYED) <= 0.2, (int(c_one[0]) - prep_mul) / n
