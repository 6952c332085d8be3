#!/usr/bin/env python3
"""Compare the MFMA f64 probe output with candidate CPU formulas (fma chain k ascending etc.)."""
import sys
import numpy as np
from fractions import Fraction

reps = 4096
raw = np.fromfile(sys.argv[1], dtype=np.float64)
A = raw[:reps * 64].reshape(reps, 16, 4)
B = raw[reps * 64:reps * 128].reshape(reps, 4, 16)
C = raw[reps * 128:reps * 384].reshape(reps, 16, 16)
D = raw[reps * 384:].reshape(reps, 16, 16)
import math


def fma(a, b, c):
    return float(Fraction(a) * Fraction(b) + Fraction(c))


cands = {
    "chain_k_asc_c_first": lambda a, b, c: fma(a[3], b[3], fma(a[2], b[2], fma(a[1], b[1], fma(a[0], b[0], c)))),
    "chain_k_desc_c_first": lambda a, b, c: fma(a[0], b[0], fma(a[1], b[1], fma(a[2], b[2], fma(a[3], b[3], c)))),
    "exact_dot_plus_c_one_round": lambda a, b, c: float(sum(Fraction(a[k]) * Fraction(b[k]) for k in range(4)) + Fraction(c)),
}
hits = {k: 0 for k in cands}
n = 0
for r in range(0, reps, 8):
    for i in range(16):
        for j in range(16):
            a = A[r, i, :]; b = B[r, :, j]; c = C[r, i, j]
            n += 1
            for name, f in cands.items():
                if f(a, b, c) == D[r, i, j]:
                    hits[name] += 1
print("elements", n)
for k, v in hits.items():
    print("%-30s %d / %d" % (k, v, n))
