"""Derive the 2^f polynomial used by pac_exp2 (csrc/pac_common.h): a
Chebyshev (near-minimax) fit of 2^f on [-1/2, 1/2] in 60-digit arithmetic,
coefficients rounded to double, then the evaluated error (fma Horner in
float64) measured against mpmath on a dense grid.  Usage: python tools/fit_exp2.py [deg]"""
import sys

import mpmath as mp
import numpy as np

mp.mp.dps = 60


def fit(deg):
    poly, err = mp.chebyfit(lambda x: mp.power(2, x), [-0.5, 0.5], deg + 1, error=True)
    return [float(c) for c in poly], float(err)        # highest degree first


def horner(c, f):
    p = np.full_like(f, c[0])
    for a in c[1:]:
        p = np.fma(p, f, a) if hasattr(np, "fma") else p * f + a
    return p


def measure(c, n=200001):
    xs = np.linspace(-0.5, 0.5, n)
    worst = 0.0
    for x in xs[::97]:
        p = c[0]
        for a in c[1:]:
            p = float(mp.mpf(p) * mp.mpf(x) + mp.mpf(a))   # fma: one rounding
        ref = mp.power(2, mp.mpf(x))
        worst = max(worst, abs(float((mp.mpf(p) - ref) / ref)))
    return worst


if __name__ == "__main__":
    deg = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    c, e = fit(deg)
    print("degree", deg, "fit error", e, "evaluated rel error", measure(c))
    for a in c:
        print("    %r," % a)
