"""Bias of the nested-sampling log Z on the C2 target (D=32 diagonal Gaussian in [-10,10]^32):
many seeds per (nlive, k, nmcmc, mode_hopping_frac) setting; prints mean delta, its standard
error, the seed-to-seed sd and sqrt(H/nlive).  Usage: nested_bias.py NSEED nlive:k:nmcmc:hop ..."""
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "mcmc-ocaml_amd"), ROOT]
from bench import analytic_log_z, c2_target  # noqa: E402
from mcmc_amd import Context, nested, targets as T  # noqa: E402

D = 32
mu, sg, _ = c2_target(D)
lik, pri = T.diag_gauss(mu, sg), T.box(-10 * np.ones(D), 10 * np.ones(D))
truth = analytic_log_z(mu, sg)
nseed = int(sys.argv[1])
for spec in sys.argv[2:]:
    nlive, k, nmcmc, hop = spec.split(":")
    nlive, k, nmcmc, hop = int(nlive), int(k), int(nmcmc), float(hop)
    d, s = [], []
    t = time.perf_counter()
    for seed in range(1, nseed + 1):
        ctx = Context(seed=1000 + seed)
        out = nested.nested_evidence(lik, pri, nlive=nlive, nmcmc=nmcmc, k=k, mode_hopping_frac=hop, ctx=ctx)
        w = np.exp(out[3])
        H = float(np.sum(w * out.ll) - out[0])
        d.append(out[0] - truth)
        s.append(math.sqrt(H / nlive))
        ctx.close()
    d = np.array(d)
    print("nlive %6d k %5d nmcmc %5d hop %.2f: mean delta %+.4f +- %.4f sd %.4f sigma %.4f "
          "(bias %+.2f sigma) wall %.1fs" % (nlive, k, nmcmc, hop, d.mean(), d.std(ddof=1) / math.sqrt(len(d)),
                                          d.std(ddof=1), np.mean(s), d.mean() / np.mean(s),
                                          time.perf_counter() - t), flush=True)
