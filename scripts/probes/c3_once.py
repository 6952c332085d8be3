"""One C3 nested run (D = 16 shell, nlive 131,072, k 4,096, nmcmc 100) after a warm-up run, for
kernel-trace profiles of the walker (MCG_NEST_LANES selects the lane split)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "mcmc-ocaml_amd")]
from mcmc_amd import Context, nested, targets as T  # noqa: E402

D = 16
lik, pri = T.gauss_shell(np.zeros(D), 2.0, 0.1), T.box(-6 * np.ones(D), 6 * np.ones(D))
for rep in range(3):
    with Context(seed=1) as ctx:
        t = time.perf_counter()
        out = nested.nested_evidence(lik, pri, nlive=131072, nmcmc=100, k=4096, mode_hopping_frac=0.1, ctx=ctx)
        print("lanes %s rep %d: log Z %.5f n_gen %d wall %.4f s" % (os.environ.get("MCG_NEST_LANES", "default"), rep,
              out[0], out.n_gen, time.perf_counter() - t), flush=True)
