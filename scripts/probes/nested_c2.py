"""Nested-sampling log Z of the C2 target (D=32 diagonal Gaussian in [-10,10]^32) for a few
(nlive, k, nmcmc) settings: accuracy vs the analytic value and wall time."""
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
for nlive, k, nmcmc in [(32768, 2048, 200), (32768, 2048, 400), (32768, 1024, 400)]:
    for seed in (1, 2, 3, 4, 5, 6):
        ctx = Context(seed=seed)
        t = time.perf_counter()
        out = nested.nested_evidence(lik, pri, nlive=nlive, nmcmc=nmcmc, k=k, mode_hopping_frac=0.1, ctx=ctx)
        dt = time.perf_counter() - t
        w = np.exp(out[3])
        H = float(np.sum(w * out.ll) - out[0])
        sig = math.sqrt(H / nlive)
        print("nlive %6d k %5d nmcmc %4d seed %d: logZ %.4f truth %.4f delta %+.4f sigma %.4f (%.2f sigma) "
              "ndead %d wall %.2fs" % (nlive, k, nmcmc, seed, out[0], truth, out[0] - truth, sig,
                                         abs(out[0] - truth) / sig, out.n_dead, dt), flush=True)
        ctx.close()
