"""Pure-Python BN254 (Milagro AMCL's curve, the one python-ursa 0.1.1's BLS uses)
-- TEST INFRASTRUCTURE ONLY, small cases (a pairing takes ~1 s here).

Two independent pairing computations are kept side by side:

* `pairing_naive(P, Q)`: the optimal-ate Miller loop on the UNTWISTED point
  psi(Q) in E(Fp12), affine lines in general Fp12 arithmetic, Frobenius as a
  generic p-th power, final exponentiation as ONE pow by (p^12 - 1)/r.
* `pairing_fast(P, lines(Q))`: the schedule the HIP kernel runs
  (csrc/pv_bn254.h): precomputed lines of the twisted point normalised to
  1 + beta*w (beta = B'*x_P/y_P + C'/y_P * v), sparse multiplications, the
  easy part f^((p^6-1)(p^2+1)) and the hard part as Scott et al.'s chain in
  f^u, f^u^2, f^u^3.

tests/test_bls_oracle.py checks that both agree, that the C oracle
(oracle/bn254_oracle.c) agrees with them, and the reference's one BLS constant
(the G2 generator, crypto/bls/indy_crypto/bls_crypto_indy_crypto.py:19).

Parameters (AMCL BN254, SEXTIC_TWIST = D_TYPE, SIGN_OF_X = NEGATIVEX):
u = -0x4080000000000001, p = 36u^4+36u^3+24u^2+6u+1, r = 36u^4+36u^3+18u^2+6u+1,
E: y^2 = x^3 + 2 over Fp, E': y^2 = x^3 + 2/xi over Fp2 = Fp[i]/(i^2+1),
xi = 1 + i, Fp6 = Fp2[v]/(v^3 - xi), Fp12 = Fp6[w]/(w^2 - v).
"""
import hashlib

U = -0x4080000000000001
P = 36 * U ** 4 + 36 * U ** 3 + 24 * U ** 2 + 6 * U + 1
R = 36 * U ** 4 + 36 * U ** 3 + 18 * U ** 2 + 6 * U + 1
B = 2
ATE = abs(6 * U + 2)            # 0x18300000000000004; 6u + 2 < 0


def inv(a):
    return pow(a, P - 2, P)


# ------------------------------------------------------------------ Fp2
class F2:
    __slots__ = ('a', 'b')

    def __init__(self, a, b=0):
        self.a, self.b = a % P, b % P

    def __add__(s, o): return F2(s.a + o.a, s.b + o.b)
    def __sub__(s, o): return F2(s.a - o.a, s.b - o.b)
    def __neg__(s): return F2(-s.a, -s.b)
    def __mul__(s, o):
        if isinstance(o, int):
            return F2(s.a * o, s.b * o)
        return F2(s.a * o.a - s.b * o.b, s.a * o.b + s.b * o.a)
    def __eq__(s, o): return s.a == o.a and s.b == o.b
    def conj(s): return F2(s.a, -s.b)
    def inv(s):
        t = inv(s.a * s.a + s.b * s.b)
        return F2(s.a * t, -s.b * t)
    def is_zero(s): return s.a == 0 and s.b == 0
    def mul_xi(s): return F2(s.a - s.b, s.a + s.b)       # (a + bi)(1 + i)
    def __repr__(s): return 'F2({:#x}, {:#x})'.format(s.a, s.b)


F2_0, F2_1 = F2(0), F2(1)
XI = F2(1, 1)
BT = F2(B) * XI.inv()           # twist constant 2/xi = 1 - i


def f2pow(x, e):
    r, b = F2_1, x
    while e:
        if e & 1:
            r = r * b
        b = b * b
        e >>= 1
    return r


# ------------------------------------------------------------------ Fp6 / Fp12
class F6:
    __slots__ = ('c',)

    def __init__(self, c0, c1=F2_0, c2=F2_0):
        self.c = (c0, c1, c2)

    def __add__(s, o): return F6(*(x + y for x, y in zip(s.c, o.c)))
    def __sub__(s, o): return F6(*(x - y for x, y in zip(s.c, o.c)))
    def __neg__(s): return F6(*(-x for x in s.c))
    def __mul__(s, o):
        a0, a1, a2 = s.c
        b0, b1, b2 = o.c
        return F6(a0 * b0 + (a1 * b2 + a2 * b1).mul_xi(),
                  a0 * b1 + a1 * b0 + (a2 * b2).mul_xi(),
                  a0 * b2 + a1 * b1 + a2 * b0)
    def mul_v(s): return F6(s.c[2].mul_xi(), s.c[0], s.c[1])
    def __eq__(s, o): return s.c == o.c
    def is_zero(s): return all(x.is_zero() for x in s.c)
    def inv(s):
        a0, a1, a2 = s.c
        t0 = a0 * a0 - (a1 * a2).mul_xi()
        t1 = (a2 * a2).mul_xi() - a0 * a1
        t2 = a1 * a1 - a0 * a2
        d = (a0 * t0 + (a2 * t1).mul_xi() + (a1 * t2).mul_xi()).inv()
        return F6(t0 * d, t1 * d, t2 * d)


F6_0, F6_1 = F6(F2_0), F6(F2_1)


class F12:
    __slots__ = ('a', 'b')

    def __init__(self, a, b=F6_0):
        self.a, self.b = a, b

    def __add__(s, o): return F12(s.a + o.a, s.b + o.b)
    def __sub__(s, o): return F12(s.a - o.a, s.b - o.b)
    def __neg__(s): return F12(-s.a, -s.b)
    def __mul__(s, o):
        return F12(s.a * o.a + (s.b * o.b).mul_v(), s.a * o.b + s.b * o.a)
    def __eq__(s, o): return s.a == o.a and s.b == o.b
    def conj(s): return F12(s.a, -s.b)
    def is_zero(s): return s.a.is_zero() and s.b.is_zero()
    def inv(s):
        d = (s.a * s.a - (s.b * s.b).mul_v()).inv()
        return F12(s.a * d, -(s.b * d))


F12_1 = F12(F6_1)


def f12pow(x, e):
    r, b = F12_1, x
    while e:
        if e & 1:
            r = r * b
        b = b * b
        e >>= 1
    return r


def f12_from_fp(x):
    return F12(F6(F2(x)))


W = F12(F6_0, F6_1)              # w
W2 = W * W                       # = v
W3 = W2 * W


# ------------------------------------------------------------------ curves
def g1_on_curve(pt):
    if pt is None:
        return True
    x, y = pt
    return (y * y - x * x * x - B) % P == 0


def g1_add(p1, p2):
    if p1 is None:
        return p2
    if p2 is None:
        return p1
    (x1, y1), (x2, y2) = p1, p2
    if x1 == x2:
        if (y1 + y2) % P == 0:
            return None
        lam = 3 * x1 * x1 * inv(2 * y1) % P
    else:
        lam = (y2 - y1) * inv(x2 - x1) % P
    x3 = (lam * lam - x1 - x2) % P
    return x3, (lam * (x1 - x3) - y1) % P


def g1_mul(pt, k):
    acc = None
    for bit in bin(k)[2:] if k > 0 else '':
        acc = g1_add(acc, acc)
        if bit == '1':
            acc = g1_add(acc, pt)
    return acc


def g1_neg(pt):
    return None if pt is None else (pt[0], (-pt[1]) % P)


def g2_on_curve(q):
    if q is None:
        return True
    x, y = q
    return y * y == x * x * x + BT


def g2_add(q1, q2):
    if q1 is None:
        return q2
    if q2 is None:
        return q1
    (x1, y1), (x2, y2) = q1, q2
    if x1 == x2:
        if (y1 + y2).is_zero():
            return None
        lam = x1 * x1 * 3 * (y1 * 2).inv()
    else:
        lam = (y2 - y1) * (x2 - x1).inv()
    x3 = lam * lam - x1 - x2
    return x3, lam * (x1 - x3) - y1


def g2_mul(q, k):
    acc = None
    for bit in bin(k)[2:] if k > 0 else '':
        acc = g2_add(acc, acc)
        if bit == '1':
            acc = g2_add(acc, q)
    return acc


def g2_neg(q):
    return None if q is None else (q[0], -q[1])


# ------------------------------------------------------------------ encodings (AMCL)
def g2_from_bytes(b):
    """ECP2::frombytes: x.a | x.b | y.a | y.b, 32-byte big-endian each, reduced
    mod p (FP::new_big); a point off the twist -> infinity (None)."""
    assert len(b) == 128
    c = [int.from_bytes(b[32 * k:32 * k + 32], 'big') for k in range(4)]
    q = (F2(c[0], c[1]), F2(c[2], c[3]))
    return q if g2_on_curve(q) else None


def g2_to_bytes(q):
    x, y = q
    return b''.join(v.to_bytes(32, 'big') for v in (x.a, x.b, y.a, y.b))


def sqrt_fp(a):
    """AMCL FP::sqrt for p = 3 mod 4: a^((p+1)/4) (no sign normalisation)."""
    return pow(a, (P + 1) // 4, P)


def is_qr(a):
    return pow(a % P, (P - 1) // 2, P) == 1


def g1_from_bytes(b):
    """ECP::frombytes (the signature point): 0x04 | x | y (uncompressed) or
    0x02/0x03 | x (compressed, y parity = prefix & 1); x or y >= p, an unknown
    prefix, or a point off the curve -> infinity (None).  Length must be 128
    (python-ursa's representation size; bytes past the encoding are ignored)."""
    if len(b) != 128:
        raise ValueError('signature representation must be 128 bytes')
    x = int.from_bytes(b[1:33], 'big')
    if x >= P:
        return None
    if b[0] == 4:
        y = int.from_bytes(b[33:65], 'big')
        if y >= P:
            return None
        return (x, y) if g1_on_curve((x, y)) else None
    if b[0] in (2, 3):
        rhs = (x * x * x + B) % P
        if not is_qr(rhs):
            return None
        y = sqrt_fp(rhs)
        if (y & 1) != (b[0] & 1):
            y = (P - y) % P
        return x, y
    return None


def g1_to_bytes(pt):
    x, y = pt
    return b'\x04' + x.to_bytes(32, 'big') + y.to_bytes(32, 'big') + bytes(63)


def hash_to_g1(msg):
    """ursa Bls::_hash: PointG1::from_hash(SHA-256(msg)): x = digest (big-endian)
    taken mod p, ECP::new_big: y = (x^3+2)^((p+1)/4) when x^3+2 is a square,
    else (or for rhs = 0) increment the integer and retry."""
    x0 = int.from_bytes(hashlib.sha256(msg).digest(), 'big')
    while True:
        x = x0 % P
        rhs = (x * x * x + B) % P
        if is_qr(rhs):
            return x, sqrt_fp(rhs)
        x0 += 1


# ------------------------------------------------------------------ naive pairing
def untwist(q):
    x, y = q
    return f12_from_f2(x) * W2, f12_from_f2(y) * W3


def f12_from_f2(x):
    return F12(F6(x))


def _line_naive(t, q2, p):
    """line through t, q2 (points of E(Fp12), affine) evaluated at p (Fp12 coords)"""
    (x1, y1), (x2, y2) = t, q2
    if x1 == x2 and y1 == y2:
        lam = (x1 * x1 * f12_from_fp(3)) * (y1 * f12_from_fp(2)).inv()
    else:
        lam = (y2 - y1) * (x2 - x1).inv()
    xp, yp = p
    val = yp - y1 - lam * (xp - x1)
    x3 = lam * lam - x1 - x2
    return val, (x3, lam * (x1 - x3) - y1)


def miller_naive(pt, q):
    if pt is None or q is None:
        return F12_1
    Q = untwist(q)
    Pp = (f12_from_fp(pt[0]), f12_from_fp(pt[1]))
    f, T = F12_1, Q
    for i in range(ATE.bit_length() - 2, -1, -1):
        l, T = _line_naive(T, T, Pp)
        f = f * f * l
        if (ATE >> i) & 1:
            l, T = _line_naive(T, Q, Pp)
            f = f * l
    # 6u + 2 < 0: f_{-s} = 1 / (f_s * v_{sQ}); the vertical line and the
    # inverse-vs-conjugate difference vanish in the final exponentiation
    f = f.inv()
    T = (T[0], -T[1])
    Q1 = (f12pow(Q[0], P), f12pow(Q[1], P))
    Q2 = (f12pow(Q1[0], P), f12pow(Q1[1], P))
    l, T = _line_naive(T, Q1, Pp)
    f = f * l
    l, T = _line_naive(T, (Q2[0], -Q2[1]), Pp)
    return f * l


def pairing_naive(pt, q):
    return f12pow(miller_naive(pt, q), (P ** 12 - 1) // R)


# ------------------------------------------------------------------ fast pairing (kernel schedule)
FROB_X1 = f2pow(XI, (P - 1) // 3)        # twist Frobenius: x^p * xi^((p-1)/3)
FROB_Y1 = f2pow(XI, (P - 1) // 2)
FROB_X2 = f2pow(XI, (P * P - 1) // 3)    # p^2: in Fp
FROB_Y2 = f2pow(XI, (P * P - 1) // 2)


def g2_frob(q):
    x, y = q
    return x.conj() * FROB_X1, y.conj() * FROB_Y1


def g2_frob2(q):
    x, y = q
    return x * FROB_X2, y * FROB_Y2


def _line_tw(t, q2):
    """affine line on the twist through t, q2 -> ((B', C'), t + q2): the untwisted
    line at P is y_P + B' x_P w + C' v w (B' = -lambda', C' = lambda' x' - y')."""
    (x1, y1), (x2, y2) = t, q2
    if x1 == x2 and y1 == y2:
        lam = x1 * x1 * 3 * (y1 * 2).inv()
    else:
        lam = (y2 - y1) * (x2 - x1).inv()
    x3 = lam * lam - x1 - x2
    return (-lam, lam * x1 - y1), (x3, lam * (x1 - x3) - y1)


def lines(q):
    """the 70 normalised lines (B', C') of the optimal-ate loop for a fixed q,
    in consumption order: per bit i = 63..0 the doubling line then (bits 63,
    57, 56, 2) the addition line; then the lines with pi(q) and -pi^2(q)."""
    out, T = [], q
    for i in range(ATE.bit_length() - 2, -1, -1):
        l, T = _line_tw(T, T)
        out.append(l)
        if (ATE >> i) & 1:
            l, T = _line_tw(T, q)
            out.append(l)
    T = g2_neg(T)
    l, T = _line_tw(T, g2_frob(q))
    out.append(l)
    l, T = _line_tw(T, g2_neg(g2_frob2(q)))
    out.append(l)
    return out


def _mul_line(f, xq, yq, ln):
    """f * (1 + beta w), beta = B' xq + (C' yq) v"""
    b0, b1 = ln[0] * xq, ln[1] * yq
    beta = F6(b0, b1)
    return F12(f.a + (f.b * beta).mul_v(), f.b + f.a * beta)


def miller_fast(terms):
    """terms: [(P or None, lines)] -> the product of the normalised Miller values"""
    prep = []
    for pt, ln in terms:
        if pt is None:
            continue
        yi = inv(pt[1])
        prep.append((pt[0] * yi % P, yi, ln))
    f, k = F12_1, 0
    for i in range(ATE.bit_length() - 2, -1, -1):
        f = f * f
        for xq, yq, ln in prep:
            f = _mul_line(f, xq, yq, ln[k])
        k += 1
        if (ATE >> i) & 1:
            for xq, yq, ln in prep:
                f = _mul_line(f, xq, yq, ln[k])
            k += 1
    f = f.conj()
    for j in range(2):
        for xq, yq, ln in prep:
            f = _mul_line(f, xq, yq, ln[k])
        k += 1
    return f


def frob12(f, n=1):
    return f12pow(f, P ** n)         # generic (test infrastructure)


def final_exp_fast(f):
    f = f.conj() * f.inv()                       # ^(p^6 - 1)
    f = frob12(f, 2) * f                         # ^(p^2 + 1)
    def pu(x):                                   # x^u in the cyclotomic subgroup (u < 0)
        return f12pow(x, -U).conj()
    fu = pu(f)
    fu2 = pu(fu)
    fu3 = pu(fu2)
    y0 = frob12(f) * frob12(f, 2) * frob12(f, 3)
    y1 = f.conj()
    y2 = frob12(fu2, 2)
    y3 = frob12(fu).conj()
    y4 = (fu * frob12(fu2)).conj()
    y5 = fu2.conj()
    y6 = (fu3 * frob12(fu3)).conj()
    t0 = y6 * y6 * y4 * y5
    t1 = y3 * y5 * t0
    t0 = t0 * y2
    t1 = t1 * t1 * t0
    t1 = t1 * t1
    t0 = t1 * y1
    t1 = t1 * y0
    t0 = t0 * t0 * t1
    return t0


def verify_sig(sig128, msg, pk128, gen128):
    """Bls.verify(signature, message, ver_key, gen): e(sigma, g) == e(H(m), pk)
    (reference call site crypto/bls/indy_crypto/bls_crypto_indy_crypto.py:73-82)."""
    try:
        s = g1_from_bytes(sig128)
    except ValueError:
        return False
    g = g2_from_bytes(gen128)
    pk = g2_from_bytes(pk128)
    h = hash_to_g1(msg)
    return pairing_naive(s, g) == pairing_naive(h, pk)


def f2_sqrt(a):
    """a square root of a in Fp2 (None if a is not a square), p = 3 mod 4
    (test data generation: points on the twist outside G2)"""
    if a.is_zero():
        return F2_0
    # a^((p^2 - 1)/2) == 1 <=> square; for p = 3 mod 4 use the norm method
    n = (a.a * a.a + a.b * a.b) % P
    if not is_qr(n):
        return None
    s = sqrt_fp(n)
    for sn in (s, (-s) % P):
        t = (a.a + sn) * inv(2) % P
        if is_qr(t):
            x = sqrt_fp(t)
            y = a.b * inv(2 * x) % P if x else 0
            r = F2(x, y)
            if r * r == a:
                return r
    return None


def twist_point_outside_g2(seed=1):
    """a point on E' (y^2 = x^3 + 2/xi) whose order is not r"""
    x0 = seed
    while True:
        x = F2(x0, 1)
        y = f2_sqrt(x * x * x + BT)
        if y is not None:
            q = (x, y)
            if g2_mul(q, R) is not None:
                return q
        x0 += 1
