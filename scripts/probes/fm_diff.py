"""Where a fused walk + merge nested run first departs from the oracle (and the two-launch path):
the batched parity cases of tests/test_gpu_nested.py, per path, the first differing dead point."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (os.path.join(ROOT, "mcmc-ocaml_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)
import warnings
warnings.simplefilter("ignore")
import oracle as O  # noqa: E402
from mcmc_amd import Context, nested, targets as T  # noqa: E402

D = 3
lik = T.gauss_shell(np.zeros(D), 1.0, 0.2)
pri = T.box(-2 * np.ones(D), 2 * np.ones(D))
m = O.Model(lik.ndim, lik.kind, lik.params, pri.kind, pri.params, 1, [1.0])
for k, fixed in [(4, False), (16, True), (100, False), (16, False), (4, True)]:
    o = O.nested(m, 5, quirk=not fixed, nlive=300, nmcmc=15, mode_hop=0.1, k=k)
    for fm in ("1", "0"):
        os.environ["MCG_NESTED_FM"] = fm
        ctx = Context(seed=5, flags=1 if fixed else 0)
        g = nested.nested_evidence(lik, pri, ctx=ctx, nlive=300, nmcmc=15, mode_hopping_frac=0.1, k=k)
        ctx.close()
        n = min(len(g.ll), len(o["ll"]))
        bad = np.nonzero(g.ll[:n] != o["ll"][:n])[0]
        first = int(bad[0]) if len(bad) else -1
        print("k %d fixed %d fm %s: n_dead gpu %d oracle %d, first ll diff %d (gen %d), log_ev %.6f vs %.6f"
              % (k, fixed, fm, g.n_dead, o["n_dead"], first, first // k if first >= 0 else -1, g[0], o["log_ev"]),
              flush=True)
        if first >= 0:
            print("   gpu", g.ll[first:first + 3], "oracle", o["ll"][first:first + 3], flush=True)
