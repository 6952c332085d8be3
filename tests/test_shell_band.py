"""The nested walker's squared-radius constraint test for the Gaussian shell (WalkTarget::
setup_constraint / constraint, mcg_nested_kernel.h) restated with the same double arithmetic:
every S it classifies as passing or failing must give the same answer as the exact comparison
lik(y) >= thr on the evaluated likelihood (nested.ml:54-59; portable sqrt of the RNG/math spec).
Probed densely around the band edges, for thresholds far from and very close to the peak."""
import math

import numpy as np

EPS = 2.220446049250313e-16


def bands(c0, c1, c2, thr):
    inf = math.inf
    g = c2 - thr
    if not (g >= 0.0) or not (c1 > 0.0) or not (c0 >= 0.0):
        return (inf, -inf, -inf if g >= 0 else inf, inf if g >= 0 else -inf)
    delta = math.sqrt(2.0 * g) / c1
    df = 64.0 * EPS * (abs(c2) + abs(thr) + 1.0)
    dr = max(df / (c1 * c1 * max(delta, 1e-300)), math.sqrt(2.0 * df) / c1)
    band = 1e-9 * (c0 + delta) + 4.0 * dr
    r_lo, r_hi = c0 - delta, c0 + delta
    a_lo, a_hi = max(r_lo + band, 0.0), r_hi - band
    in_lo, in_hi = (a_lo * a_lo, a_hi * a_hi) if a_hi >= a_lo else (inf, -inf)
    out_lo = (r_lo - band) ** 2 if r_lo - band > 0.0 else -inf
    out_hi = (r_hi + band) * (r_hi + band)
    return in_lo, in_hi, out_lo, out_hi


def exact(L, S, c0, c1, c2, thr):
    r = L.or_sqrt(S)
    qq = (r - c0) * c1
    return (c2 - 0.5 * qq * qq) >= thr


def test_shell_band_agrees_with_exact_comparison(oracle):
    L = oracle.lib()
    rng = np.random.default_rng(7)
    checked = 0
    for _ in range(300):
        c0 = float(rng.uniform(0.5, 4.0))                  # shell radius
        c1 = 1.0 / float(rng.uniform(0.01, 0.3))           # 1 / width
        c2 = float(rng.uniform(-40.0, 10.0))               # log-normaliser (peak ll)
        g = float(10.0 ** rng.uniform(-15, 1.5))           # peak - threshold: wide to tiny
        thr = c2 - g
        in_lo, in_hi, out_lo, out_hi = bands(c0, c1, c2, thr)
        edges = [e for e in (in_lo, in_hi, out_lo, out_hi) if math.isfinite(e) and e > 0]
        probes = [e * (1.0 + t) for e in edges for t in np.linspace(-1e-8, 1e-8, 41)]
        probes += [e + k * math.ulp(e) for e in edges for k in range(-4, 5)]
        probes += list(rng.uniform(0.0, (c0 + 2.0 / c1) ** 2 * 1.5, 50))
        for S in probes:
            if S < 0:
                continue
            ins = in_lo <= S <= in_hi
            outs = S < out_lo or S > out_hi
            assert not (ins and outs)
            if ins or outs:
                assert exact(L, S, c0, c1, c2, thr) == ins, (c0, c1, c2, thr, S)
                checked += 1
    assert checked > 10000


def test_shell_band_threshold_above_peak_fails_everything():
    in_lo, in_hi, out_lo, out_hi = bands(2.0, 10.0, 1.0, 1.5)
    assert in_lo > in_hi and out_lo == math.inf
