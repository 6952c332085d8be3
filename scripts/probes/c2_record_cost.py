"""C2 launch time with and without the per-step records (Welford + harmonic mean)."""
import math, sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "mcmc-ocaml_amd"))
import numpy as np
from mcmc_amd import Context, targets as T

D, N, S = 32, 65536, 1000
rng = np.random.default_rng(42)
mu, sg = rng.uniform(-1, 1, D), rng.uniform(0.5, 2, D)
for acc in (True, False, True, False):
    ctx = Context(seed=1)
    ctx.set_model(T.diag_gauss(mu, sg), T.box(-10 * np.ones(D), 10 * np.ones(D)), T.gauss(2.38 / math.sqrt(D)))
    ctx.init(rng.normal(mu[:, None], sg[:, None], size=(D, N)))
    ctx.run(nbin=S, nskip=1, n_rec=1, record_x=False, record_llp=False, accumulate=acc)
    ctx.sync()
    ctx.set_timing(True)
    for _ in range(10):
        ctx.run(nbin=0 if acc else S, nskip=1, n_rec=S if acc else 0, record_x=False, record_llp=False,
                accumulate=acc, append=acc)
    ctx.sync()
    t = ctx.kernel_timing("mh")
    print("accumulate" if acc else "no records", "%.4f ms" % (t["total_ms"] / max(1, t["launches"])), t["launches"])
    ctx.close()
