"""Where the bench's timed region goes beyond its kernels: K runs of S sweeps (synced), then the
end-of-run reduction (tile kernel, copy, host combine), timed separately, with and without the
per-launch HIP events.  Measured (round 2, session 4): runs + sync = the kernels' own time, the
tile kernel + copy ~0.12 ms, the host combine ~0.02 ms; the first ~20 launches of a process run
~7 % slower than later ones (2.71-2.75 -> 2.51-2.53 ms per launch), which running the nested
leg first did not remove."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "mcmc-ocaml_amd"), ROOT]
from bench import c2_target  # noqa: E402
from mcmc_amd import Context, targets as T  # noqa: E402
from mcmc_amd.parallel import reduce_stats  # noqa: E402

D, N, S, K = 32, 65536, 1000, 10
mu, sg, s = c2_target(D)
ctx = Context(seed=1)
ctx.set_model(T.diag_gauss(mu, sg), T.box(-10 * np.ones(D), 10 * np.ones(D)), T.gauss(s))
ctx.init(np.random.default_rng(1000).normal(mu[:, None], sg[:, None], size=(D, N)))
ctx.run(nbin=S, nskip=1, n_rec=1, record_x=False, record_llp=False, record_accept=False, accumulate=True)
ctx.sync()
for timing in (False, True, False, True):
    ctx.set_timing(timing)
    t0 = time.perf_counter()
    for _ in range(K):
        ctx.run(nbin=0, nskip=1, n_rec=S, record_x=False, record_llp=False, record_accept=False,
                accumulate=True, append=True)
    t1 = time.perf_counter()
    ctx.sync()
    t2 = time.perf_counter()
    tiles = ctx.tile_stats()
    t3 = time.perf_counter()
    reduce_stats(D, tiles)
    t4 = time.perf_counter()
    kt = ctx.kernel_timing("mh") if timing else None
    print("timing %d: enqueue %.3f ms, runs+sync %.3f ms, tile_stats %.3f ms, combine %.3f ms%s" % (
        timing, (t1 - t0) * 1e3, (t2 - t0) * 1e3, (t3 - t2) * 1e3, (t4 - t3) * 1e3,
        "" if kt is None else ", kernel events %.3f ms/launch" % (kt["total_ms"] / max(kt["launches"], 1))), flush=True)
