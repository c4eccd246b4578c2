"""The generated BN254 asm columns (csrc/pv_bn254_asm.h, tools/gen_bn_madchains.py)
against the C++ column sums of pv_bn254.h bn::mul / bn::sqr, on the CPU.

The asm itself only runs on the GPU (tests/test_gpu_bls.py checks the kernel
against the C oracle); here the generator's column lists -- which products and
which reduction terms each asm chain sums -- are replayed in Python and must
give the same limbs as a restatement of the C++ loops, for random lazy operands
at the bounds pv_bn254.h states (|limb| < 2^29).  The committed header must also
be exactly what the generator prints."""
import importlib.util
import os
import random
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GEN = os.path.join(REPO, 'tools', 'gen_bn_madchains.py')
HDR = os.path.join(REPO, 'indy-plenum_amd', 'csrc', 'pv_bn254_asm.h')


def _gen():
    spec = importlib.util.spec_from_file_location('gen_bn_madchains', GEN)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


G = _gen()
NL, PL = G.NL, G.PL
M28 = (1 << 28) - 1
NP = (-pow(G.P, -1, 1 << 28)) % (1 << 28)


def _s64(x):
    x &= (1 << 64) - 1
    return x - (1 << 64) if x >> 63 else x


def _s32(x):
    x &= (1 << 32) - 1
    return x - (1 << 32) if x >> 31 else x


def ref_mul(a, b, sqr=False):
    """pv_bn254.h bn::mul / bn::sqr (C++ loops), int64 column sums."""
    d = [2 * x for x in a]
    m = [0] * NL
    r = [0] * NL
    carry = 0
    for k in range(2 * NL - 1):
        acc = carry
        lo = 0 if k < NL else k - NL + 1
        if sqr:
            i = lo
            while 2 * i < k:
                acc += a[i] * d[k - i]
                i += 1
            if k % 2 == 0:
                acc += a[k // 2] * a[k // 2]
        else:
            for i in range(lo, min(k, NL - 1) + 1):
                acc += a[i] * b[k - i]
        if k < NL:
            for i in range(k):
                if PL[k - i]:
                    acc += m[i] * PL[k - i]
            m[k] = ((acc & 0xffffffff) * NP) & M28
            acc += m[k] * PL[0]
        else:
            for i in range(k - NL + 1, NL):
                if PL[k - i]:
                    acc += m[i] * PL[k - i]
            r[k - NL] = _s32(acc & M28)
        assert -(1 << 63) <= acc < (1 << 63)
        carry = _s64(acc) >> 28
    r[NL - 1] = _s32(carry)
    return r


def gen_mul(a, b, sqr=False):
    """The same product through the generator's per-column term lists."""
    d = [2 * x for x in a]
    m = [0] * NL
    r = [0] * NL
    acc = 0
    for k in range(2 * NL - 1):
        prods, reds = G.column(k, sqr)
        for kind, i, j in prods:
            acc += a[i] * (a[j] if kind == 'aa' else (d[j] if kind == 'ad' else b[j]))
        for i, j in reds:
            acc += m[i] * PL[j]
        acc = _s64(acc)
        if k < NL:
            m[k] = ((acc & 0xffffffff) * NP) & M28
            acc = _s64(acc + m[k] * PL[0])
        else:
            r[k - NL] = _s32(acc & M28)
        acc >>= 28
    r[NL - 1] = _s32(acc)
    return r


def test_generated_header_is_current():
    out = subprocess.run([sys.executable, GEN], check=True, capture_output=True, text=True).stdout
    with open(HDR) as fh:
        assert fh.read() == out


def test_column_terms_cover_the_cxx_sums():
    """Every (product, reduction) term of the C++ loops appears exactly once."""
    n_prod = sum(len(G.column(k, False)[0]) for k in range(2 * NL - 1))
    n_red = sum(len(G.column(k, False)[1]) for k in range(2 * NL - 1))
    n_sq = sum(len(G.column(k, True)[0]) for k in range(2 * NL - 1))
    nz = sum(1 for j in range(1, NL) if PL[j])
    assert n_prod == NL * NL and n_sq == NL * (NL + 1) // 2
    assert n_red == NL * nz          # the P[0] term of each m_k is added in C++


def test_asm_columns_equal_cxx_mul_and_sqr():
    rnd = random.Random(1234)
    lim = 1 << 29
    for t in range(400):
        if t < 8:   # extremes
            v = (lim - 1) if t & 1 else -(lim - 1)
            a = [v] * NL
            b = [-v if t & 2 else v] * NL
        else:
            a = [rnd.randrange(-lim + 1, lim) for _ in range(NL)]
            b = [rnd.randrange(-lim + 1, lim) for _ in range(NL)]
        assert gen_mul(a, b) == ref_mul(a, b), t
        assert gen_mul(a, None, sqr=True) == ref_mul(a, None, sqr=True), t
