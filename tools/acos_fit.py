"""Coefficients of hs_math.h's hs_acos (the limb IK's fp64 acos): asin(z) = z + z t P(t), t = z^2, with P of
degree d interpolating f(t) = (asin(sqrt t) - sqrt t) / (t sqrt t) at Chebyshev nodes of [0, 0.25] in 40-digit
arithmetic (mpmath), and the resulting acos's error against glibc's (math.acos) in ulps on 10^5 points of
[-1, 1] plus points clustered at +-1. Tuning aid; the product uses the degree-11 row.
    python tools/acos_fit.py"""
import numpy as np, math, mpmath as mp
mp.mp.dps = 40
a = mp.mpf("0.25")
# f(t) = (asin(sqrt t) - sqrt t) / (t sqrt t), degree-d minimax-ish fit by Chebyshev interpolation in high precision
def f(t):
    if t == 0: return mp.mpf(1) / 6
    z = mp.sqrt(t)
    return (mp.asin(z) - z) / (t * z)
for deg in (11, 12, 13, 14):
    n = deg + 1
    nodes = [a / 2 * (1 + mp.cos(mp.pi * (k + mp.mpf(0.5)) / n)) for k in range(n)]
    # solve Vandermonde in high precision (monomials in t)
    A = mp.matrix([[nd ** j for j in range(n)] for nd in nodes])
    b = mp.matrix([f(nd) for nd in nodes])
    c = mp.lu_solve(A, b)
    coef = [float(c[j]) for j in range(n)]
    # worst error of f approximation
    ts = [a * k / 2000 for k in range(2001)]
    e = max(abs(sum(mp.mpf(coef[j]) * tt ** j for j in range(n)) - f(tt)) / f(tt) for tt in ts)
    xs = np.concatenate([np.linspace(-1, 1, 100001), 1 - np.logspace(-16, 0, 1000), -1 + np.logspace(-16, 0, 1000)])
    def asin_p(zv):
        tt = zv * zv
        p = coef[-1]
        for cc in coef[-2::-1]:
            p = p * tt + cc
        return zv + zv * tt * p
    def acos_c(x):
        ax = abs(x)
        if ax <= 0.5:
            return math.pi / 2 - asin_p(x)
        s = math.sqrt((1 - ax) / 2)
        r = 2 * asin_p(s)
        return r if x > 0 else math.pi - r
    err = max(abs(acos_c(x) - math.acos(x)) / math.ulp(math.acos(x)) for x in xs if math.acos(x) > 0)
    print(deg, "f rel err", float(e), "max ulp err vs glibc", err)
    print("  ", repr(coef))
