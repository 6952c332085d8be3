"""Round 6: the one-lane kD kernel at D 64 whose final state store came out wrong in round 5
(LABLOG.md round 5, test_gpu_fuzz).  Runs mh_kernel<64, 1, LIK, KD> from a library that
compiles it (MCG_LIBRARY=lib/libmcg_kd64.so, gen_instances + ("GMIX"|"DIAG", "KD", 64, 1)) and
compares records, bitmap, final state and ll with the oracle; prints every mismatching dim."""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "mcmc-ocaml_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import oracle as O  # noqa: E402
from mcmc_amd import Context, targets as T  # noqa: E402

D = 64
for lik_name in ("gmix", "diag"):
    for nbin, n_rec in ((0, 1), (3, 1), (0, 5), (2, 4)):
        rng = np.random.default_rng(11)
        if lik_name == "gmix":
            lik = T.gauss_mix(rng.uniform(-2, 2, (2, D)), rng.uniform(0.3, 1.5, (2, D)))
        else:
            lik = T.diag_gauss(rng.uniform(-1, 1, D), rng.uniform(0.5, 1.5, D))
        pri = T.box(-4 * np.ones(D), 4 * np.ones(D))
        lo, hi = -3 * np.ones(D), 3 * np.ones(D)
        pts = np.clip(rng.normal(0.0, 1.0, size=(200, D)), -2.9, 2.9)
        kdp = T.KdInterp(pts, lo, hi)
        okd = O.KdTree(pts, lo, hi)
        N = 256
        x0 = rng.uniform(-1.5, 1.5, size=(D, N))
        seed = 77
        ctx = Context(seed=seed, lanes_per_chain=1)
        ctx.set_model(lik, pri, kdp)
        ctx.init(x0)
        ctx.run(nbin=nbin, nskip=1, n_rec=n_rec, record_x=True, record_llp=True, record_accept=True, accumulate=True)
        rx, rll, rlp, bits = ctx.records(x=True, llp=True, accept=True)
        x, ll, lp = ctx.state()
        ctx.close()
        m = O.Model(D, lik.kind, lik.params, pri.kind, pri.params, 3, [0.0], okd)
        ll0 = np.array([m.loglik(x0[:, i]) for i in range(N)])
        lp0 = np.array([m.logprior(x0[:, i]) for i in range(N)])
        o = O.mh_run(m, seed, x0, ll0, lp0, nbin=nbin, nskip=1, n_rec=n_rec, nthreads=8)
        res = []
        for name, a, b in (("bits", bits, o["bits"]), ("rec_x", rx, o["rec_x"]), ("rec_ll", rll, o["rec_ll"]),
                           ("x", x, o["x"]), ("ll", ll, o["ll"]), ("lp", lp, o["lp"])):
            a, b = np.asarray(a), np.asarray(b)
            bad = np.argwhere(a != b) if a.shape == b.shape else None
            res.append("%s %s" % (name, "shape" if bad is None else len(bad)))
        print(lik_name, "nbin", nbin, "n_rec", n_rec, " | ".join(res), flush=True)
        xb = np.argwhere(np.asarray(x) != o["x"])
        if len(xb):
            dims = sorted(set(xb[:, 0].tolist()))
            d, c = xb[0]
            print("   final x wrong in dims", dims[:16], "chains", len(set(xb[:, 1].tolist())),
                  "| gpu", x[d, c], "oracle", o["x"][d, c], "last record gpu", np.asarray(rx)[-1][d, c],
                  "x0", x0[d, c], flush=True)
