import os, sys, time
import numpy as np
sys.path[:0] = [os.path.join(os.getcwd(), "mcmc-ocaml_amd")]
from mcmc_amd import Context, nested, targets as T
D = 16
lik, pri = T.gauss_shell(np.zeros(D), 2.0, 0.1), T.box(-6 * np.ones(D), 6 * np.ones(D))
with Context(seed=1) as ctx:
    for rep in range(3):
        t = time.perf_counter()
        out = nested.nested_evidence(lik, pri, nlive=131072, nmcmc=100, k=4096, mode_hopping_frac=0.1, ctx=ctx, points=False)
        print("rep %d wall %.4f s" % (rep, time.perf_counter() - t), flush=True)
