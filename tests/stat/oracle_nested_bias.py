"""Finite-walk bias of Nested.nested_evidence (nested.ml:122-146) on the C2 target (D-dim diagonal
Gaussian in [-10,10]^D), measured on the oracle -- at k = 1 that is the reference algorithm
itself.  Many seeds of one (D, nlive, k, nmcmc) setting, 8 worker processes.

Not collected by pytest (statistical, minutes of CPU).  Usage: D nlive k nmcmc nseed"""
import math
import os
import sys
from multiprocessing import Pool

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "oracle"), ROOT]
import oracle as O  # noqa: E402
from bench import analytic_log_z, c2_target  # noqa: E402

D, NLIVE, K, NMCMC, NSEED = (int(a) for a in sys.argv[1:6])
MU, SG, _ = c2_target(D)


def run(seed):
    m = O.Model(D, 1, np.concatenate([MU, SG]), 1,
                np.concatenate([-10 * np.ones(D), 10 * np.ones(D), [-D * math.log(20.0)]]))
    r = O.nested(m, seed, nlive=NLIVE, nmcmc=NMCMC, k=K, mode_hop=0.1)
    H = float(np.sum(np.exp(r["log_wts"]) * r["ll"]) - r["log_ev"])
    return r["log_ev"] - analytic_log_z(MU, SG), math.sqrt(H / NLIVE)


if __name__ == "__main__":
    with Pool(8) as p:
        res = p.map(run, range(1, NSEED + 1))
    d = np.array([a for a, _ in res])
    s = float(np.mean([b for _, b in res]))
    print("D %d nlive %d k %d nmcmc %d: mean delta %+.4f +- %.4f  sd %.4f sigma %.4f  bias/sigma %+.2f"
          % (D, NLIVE, K, NMCMC, d.mean(), d.std(ddof=1) / math.sqrt(len(d)), d.std(ddof=1), s, d.mean() / s))
