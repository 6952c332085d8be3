"""Where the C3 nested_evidence wall goes (points=False, the bench's value): mcg_nested (device
generations + host fold) against fetch (mcg_nested_get: ll, lp, weights), after a warm-up run;
MCG_NESTED_PROFILE=1 adds mcg_nested's own host-side split."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "mcmc-ocaml_amd")]
from mcmc_amd import Context, nested, targets as T  # noqa: E402

D = 16
lik, pri = T.gauss_shell(np.zeros(D), 2.0, 0.1), T.box(-6 * np.ones(D), 6 * np.ones(D))
with Context(seed=1) as ctx:
    for rep in range(4):
        t0 = time.perf_counter()
        r = nested.run_nested(lik, pri, 0.01, 100, 131072, 0.1, 4096, None, ctx)
        t1 = time.perf_counter()
        out = nested.fetch(ctx, r, D, False, 4096)
        t2 = time.perf_counter()
        print("rep %d: run_nested %.2f ms, fetch %.2f ms, n_gen %d, n_total %d" % (
            rep, 1e3 * (t1 - t0), 1e3 * (t2 - t1), r.n_gen, r.n_total), flush=True)
        out = None
