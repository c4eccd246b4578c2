"""Smallest set of prepared operand multiples for a radix-2^25.5 squaring
(pv_field.h sq_avail): product (i, j), i <= j, of f^2 has the coefficient
c = (1 if i == j else 2) * (2 if i, j both odd) * (19 if i + j >= 10) and is
formed as (m_i f_i)(m_j f_j) with m_i m_j = c.  Each prepared m f_i (m != 1)
costs one VALU op per squaring; exhaustive branch-and-bound over the choices.

    python tools/sq_prep_search.py      -> 13 [(0, 2), ..., (9, 38)]"""
M = [1, 2, 4, 19, 38]


def main():
    need = []
    for i in range(10):
        for j in range(i, 10):
            c = (1 if i == j else 2) * (2 if (i % 2 and j % 2) else 1) * (19 if i + j >= 10 else 1)
            opts = [frozenset(x for x in ((i, a), (j, b)) if x[1] != 1) for a in M for b in M if a * b == c]
            if not any(len(o) == 0 for o in opts):
                need.append(opts)
    need.sort(key=len)
    best = [99, None]

    def solve(k, chosen):
        if len(chosen) >= best[0]:
            return
        for q in range(k, len(need)):
            if not any(o <= chosen for o in need[q]):
                for o in need[q]:
                    solve(q + 1, chosen | o)
                return
        best[0], best[1] = len(chosen), sorted(chosen)

    solve(0, frozenset())
    print(best[0], best[1])


if __name__ == '__main__':
    main()
