import random, sys, statistics
L = 2**252 + 27742317777372353535851937790883648493
N = 8 * L
PAT = int('8' * 33, 16)


def fits(v):
    return v + PAT < 2**132


def half(h):
    ra, ta = N, 0   # magnitudes; sign(t_i) = (-1)^(i+1)
    rb, tb = h, 1
    i = 1
    steps = 0
    while rb >= 2**128:
        q = ra // rb
        if q >= 2**32 - 1:
            return None, None, steps, 'hugeq'
        ra, rb = rb, ra - q * rb
        ta, tb = tb, ta + q * tb
        i += 1
        steps += 1
    neg_i = (i % 2 == 0)
    if tb % 2 == 1:
        return (-rb if neg_i else rb), tb, steps, 'i'
    if fits(ra) and fits(ta):
        return (ra if neg_i else -ra), ta, steps, 'im1'
    if rb > 0:
        q = ra // rb
        if q < 2**32 - 1:
            r2, t2 = ra - q * rb, ta + q * tb
            if fits(r2) and fits(t2):
                return (r2 if neg_i else -r2), t2, steps, 'ip1'
    return None, None, steps, 'fail'


def check(h, c, d):
    assert d % 2 == 1 and d > 0
    assert (c - d * h) % N == 0, (h, c, d)
    assert fits(abs(c)) and fits(d)


random.seed(1)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
hist = {}
steps_all = []
for k in range(n):
    h = random.randrange(L)
    c, d, s, w = half(h)
    steps_all.append(s)
    hist[w] = hist.get(w, 0) + 1
    if c is not None:
        check(h, c, d)
print({k: v / n for k, v in hist.items()})
random.shuffle(steps_all)
wm = [max(steps_all[j:j + 64]) for j in range(0, n - 64, 64)]
steps_all.sort()
print('steps mean', sum(steps_all) / n, 'p50', steps_all[n // 2], 'p99', steps_all[int(n * .99)], 'max',
      steps_all[-1], 'wave max mean', statistics.mean(wm))
for h in [0, 1, 2, 5, L - 1, 2**128 - 1, 2**128, 2**200 + 3, 2**252]:
    c, d, s, w = half(h)
    print(h.bit_length(), w, s)
    if c is not None:
        check(h, c, d)
