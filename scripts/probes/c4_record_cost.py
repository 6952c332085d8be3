"""C4 launch time with and without the per-step records (Welford + harmonic mean): an upper
bound on what a faster record path could recover.  Prints avg launch ms for each."""
import math, time, sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "mcmc-ocaml_amd"))
import numpy as np
from mcmc_amd import Context, targets as T

D, N, M, S = 8, 32768, 32768, 1000
rng = np.random.default_rng(4)
pts = rng.normal(size=(M, D))
lo, hi = -10 * np.ones(D), 10 * np.ones(D)
for acc in (True, False, True, False):
    ctx = Context(seed=1)
    ctx.set_model(T.diag_gauss(np.zeros(D), np.ones(D)), T.box(lo, hi), T.KdInterp(pts, lo, hi))
    ctx.init(rng.normal(size=(D, N)))
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
