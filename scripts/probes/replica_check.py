#!/usr/bin/env python3
"""Nested replicas of the bench's D=32 target in one process: each replica's log Z, then their
merge (mcg_nested_merge), against the analytic value."""
import os, sys, math
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "mcmc-ocaml_amd"))
import numpy as np
import bench
from mcmc_amd import Context, nested as _nested, targets as T
from mcmc_amd.parallel import replica_seed

D, nl, k, nm = 32, 32768, 2048, 200
mu, sg, s = bench.c2_target(D)
lik, pri = T.diag_gauss(mu, sg), T.box(-10 * np.ones(D), 10 * np.ones(D))
truth = bench.analytic_log_z(mu, sg)
runs = []
for r in range(int(sys.argv[1]) if len(sys.argv) > 1 else 2):
    with Context(seed=replica_seed(7, r)) as c:
        o = _nested.nested_evidence(lik, pri, nlive=nl, nmcmc=nm, k=k, mode_hopping_frac=0.1, ctx=c)
    print("replica %d: log Z %.5f (delta %+.4f) n_dead %d n_gen %d ll[0] %.3f ll[-1] %.3f sorted %s" % (
        r, o[0], o[0] - truth, o.n_dead, o.n_gen, o.ll[0], o.ll[-1], bool(np.all(np.diff(o.ll) >= 0))), flush=True)
    runs.append((o, nl, k))
m = _nested.merge_runs(runs)
print("merged: log Z %.5f (delta %+.4f)" % (m[0], m[0] - truth))
