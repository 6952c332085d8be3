#!/usr/bin/env python3
"""Two processes running the bench's D=32 nested replica concurrently on one GPU: each run must
equal the same run made alone (deterministic kernels), and its ll must be nondecreasing."""
import os, sys, math, subprocess
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "..", "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mcmc-ocaml_amd"))


def run(r, nl=32768, k=2048, nm=200):
    import numpy as np
    import bench
    from mcmc_amd import Context, nested as _nested, targets as T
    from mcmc_amd.parallel import replica_seed
    D = 32
    mu, sg, s = bench.c2_target(D)
    lik, pri = T.diag_gauss(mu, sg), T.box(-10 * np.ones(D), 10 * np.ones(D))
    mh = None
    if os.environ.get("WITH_MH"):
        # the bench's MH context, alive (and timed) while the nested run goes
        mh = Context(seed=1, chain_offset=r * 65536)
        mh.set_model(lik, pri, T.gauss(s))
        mh.init(np.random.default_rng(1000 + r).normal(mu[:, None], sg[:, None], size=(D, 65536)))
        mh.run(nbin=100, nskip=1, n_rec=1, record_x=False, record_llp=False, record_accept=False, accumulate=True)
        mh.set_timing(True)
        for _ in range(5):
            mh.run(nbin=0, nskip=1, n_rec=100, record_x=False, record_llp=False, record_accept=False,
                   accumulate=True, append=True)
        mh.tile_stats()
        mh.sync()
    with Context(seed=replica_seed(7, r)) as c:
        o = _nested.nested_evidence(lik, pri, nlive=nl, nmcmc=nm, k=k, mode_hopping_frac=0.1, ctx=c)
    d = np.diff(o.ll)
    bad = np.nonzero(d < 0)[0]
    print("proc %d seed-rank %d: log Z %.6f n_dead %d n_gen %d sorted %s first-bad %s" % (
        os.getpid(), r, o[0], o.n_dead, o.n_gen, bad.size == 0, bad[:5].tolist()), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        run(int(sys.argv[1]))
        sys.exit(0)
    print("alone:", flush=True)
    for r in (0, 1):
        subprocess.run([sys.executable, __file__, str(r)], check=True)
    print("concurrent:", flush=True)
    ps = [subprocess.Popen([sys.executable, __file__, str(r)]) for r in (0, 1)]
    rc = [p.wait() for p in ps]
    sys.exit(max(rc))
