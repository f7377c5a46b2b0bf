import sympy as sp
from fractions import Fraction as Fr

def winograd_mats(points, m, r):
    n = m + r - 1
    pts = [sp.Rational(p) for p in points]
    assert len(pts) == n - 1
    AT = sp.zeros(m, n)
    for i in range(m):
        for j in range(n - 1):
            AT[i, j] = pts[j] ** i
        AT[i, n - 1] = 1 if i == m - 1 else 0
    G = sp.zeros(n, r)
    for j in range(n - 1):
        den = 1
        for l in range(n - 1):
            if l != j:
                den *= (pts[j] - pts[l])
        for k in range(r):
            G[j, k] = pts[j] ** k / den
    G[n - 1, r - 1] = 1
    BT = sp.Matrix(n, n, lambda a, b: sp.Symbol('b_%d_%d' % (a, b)))
    eqs = []
    for i in range(m):
        for k in range(r):
            for l in range(n):
                eqs.append(sum(AT[i, j] * G[j, k] * BT[j, l] for j in range(n)) - (1 if l == i + k else 0))
    sol = sp.solve(eqs, list(BT))
    BT = BT.subs(sol)
    assert all(x.is_number for x in BT), 'underdetermined'
    return AT, G, BT

if __name__ == '__main__':
    for pts in ([0, 1, -1], [0, 1, -1, 2, -2], [0, 1, -1, sp.Rational(1, 2), -sp.Rational(1, 2)]):
        m = len(pts) + 1 - 2
        AT, G, BT = winograd_mats(pts, m, 3)
        print('points', pts)
        sp.pprint(AT); sp.pprint(G); sp.pprint(BT)
