#!/usr/bin/env python3
"""Regenerates the golden fixtures of tests/test_golden.py from the CPU oracle (oracle/oracle.c).

The reference (OCaml) cannot be built or run here, so these fixtures pin the
restatement itself: any change of the RNG/math spec must regenerate them, and
the GPU path must reproduce them bit for bit.

  python tests/golden/make_golden.py
"""
import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle as O  # noqa: E402

LIK_DIAG, LIK_SHELL = 1, 3
PRIOR_BOX, PRIOR_OPEN = 1, 2
PROP_GAUSS, PROP_KD = 1, 3


def c2_mini():
    """C2-mini: 128 chains x D=32, box prior, isotropic proposal, 256 steps, seed 1."""
    D, N = 32, 128
    rng = np.random.default_rng(42)
    mu = rng.uniform(-1, 1, D)
    sg = rng.uniform(0.5, 2, D)
    s = 2.38 / math.sqrt(D) * float(np.median(sg))
    lik = np.concatenate([mu, sg])
    pri = np.concatenate([-10 * np.ones(D), 10 * np.ones(D), [-D * math.log(20.0)]])
    m = O.Model(D, LIK_DIAG, lik, PRIOR_BOX, pri, PROP_GAUSS, [s])
    x0 = np.random.default_rng(1).normal(mu[:, None], sg[:, None], size=(D, N))
    ll0 = np.array([m.loglik(x0[:, i]) for i in range(N)])
    lp0 = np.array([m.logprior(x0[:, i]) for i in range(N)])
    r = O.mh_run(m, 1, x0, ll0, lp0, nbin=0, nskip=1, n_rec=257, record_x=False, record_llp=True,
                 record_accept=True, accumulate=True)
    tiles = O.tile_stats(D, N, 257, r)
    mean, sd, lz = O.combine_tiles(D, tiles)
    np.savez_compressed(os.path.join(HERE, "c2_mini.npz"), lik=lik, pri=pri, s=s, x0=x0, bits=r["bits"],
                        x=r["x"], ll=r["ll"], lp=r["lp"], nacc=r["nacc"], mean=mean, sd=sd, log_z_hm=lz)


def c3_mini():
    """C3-mini: nested sampling of the test/nested_test.ml Gaussian, nlive 64, nmcmc 20, k = 1."""
    lik = np.array([0.5, 0.5, 0.1, 0.1])
    pri = np.array([0.0, 0.0, 1.0, 1.0, 0.0])
    m = O.Model(2, LIK_DIAG, lik, PRIOR_OPEN, pri, PROP_GAUSS, [1.0])
    r = O.nested(m, 3, nlive=64, nmcmc=20, k=1, mode_hop=0.1)
    rk = O.nested(m, 3, nlive=64, nmcmc=20, k=4, mode_hop=0.1)
    np.savez_compressed(os.path.join(HERE, "c3_mini.npz"), lik=lik, pri=pri, ll=r["ll"], log_ev=r["log_ev"],
                        log_dev=r["log_dev"], n_dead=r["n_dead"], ll_k4=rk["ll"], log_ev_k4=rk["log_ev"],
                        log_dev_k4=rk["log_dev"])


def c4_mini():
    """C4-mini: kD tree over 256 points, D = 3, plus 64 MH steps of the interpolated proposal."""
    D = 3
    rng = np.random.default_rng(11)
    pts = rng.normal(size=(256, D))
    lo, hi = -5 * np.ones(D), 5 * np.ones(D)
    t = O.KdTree(pts, lo, hi)
    e = t.export()
    q = rng.uniform(-5, 5, size=(64, D))
    dens = np.array([t.jump_prob(p) for p in q])
    lik = np.concatenate([np.zeros(D), np.ones(D)])
    pri = np.concatenate([lo, hi, [-D * math.log(10.0)]])
    m = O.Model(D, LIK_DIAG, lik, PRIOR_BOX, pri, PROP_KD, [0.0], t)
    x0 = rng.normal(size=(D, 96))
    ll0 = np.array([m.loglik(x0[:, i]) for i in range(96)])
    lp0 = np.array([m.logprior(x0[:, i]) for i in range(96)])
    r = O.mh_run(m, 8, x0, ll0, lp0, nbin=4, nskip=1, n_rec=64, record_x=False, record_llp=False)
    np.savez_compressed(os.path.join(HERE, "c4_mini.npz"), pts=pts, lo=lo, hi=hi, q=q, dens=dens, x0=x0,
                        bits=r["bits"], x=r["x"], **{"tree_" + k: v for k, v in e.items()})


def reductions():
    """Harmonic mean / moments of a fixed ll vector (evidence.ml:101-107, stats.ml:58-87)."""
    rng = np.random.default_rng(5)
    ll = rng.normal(-3.0, 1.0, size=1000)
    xs = rng.normal(size=(1000, 4))
    hm = O.lib().or_harmonic_mean_naive(O.dptr(ll), len(ll))
    mu = np.zeros(4); sd = np.zeros(4)
    O.lib().or_multi_mean(O.dptr(xs), 1000, 4, O.dptr(mu))
    O.lib().or_multi_std(O.dptr(xs), 1000, 4, O.dptr(sd))
    le, ld, w = O.evidence_weights(np.sort(ll), 50, 1)
    np.savez_compressed(os.path.join(HERE, "reductions.npz"), ll=ll, xs=xs, hm=hm, mean=mu, sd=sd,
                        log_ev=le, log_dev=ld, log_wts=w)


def next_mini():
    """SURVEY §8(f) components: a combine_jump_proposals MH run (mcmc.ml:165-185), a
    reversible-jump run (mcmc.ml:89-153), the kD evidence integrals (evidence.ml:145-221) of its
    model-A samples, and the merge of two nested runs."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import evidence_ref as R
    # mixture: Gaussian + shift-uniform (density) + symmetric shift-uniform (ljp 0), D = 3
    D, N = 3, 96
    mix = np.array([3.0, 0.5, 1, 1, 0.6, 0.8, 1.0,
                    1.0, 2, 1, -0.4, -0.4, -0.4, 0.2, 0.2, 0.2,
                    0.7, 2, 0, -1.0, -1.0, -1.0, 1.0, 1.0, 1.0])
    lik = np.array([0.3, -0.5, 1.0, 0.5, 1.0, 2.0])
    pri = np.array([-8, -8, -8, 8, 8, 8, -3 * math.log(16.0)])
    m = O.Model(D, LIK_DIAG, lik, PRIOR_BOX, pri, 5, mix)
    x0 = np.random.default_rng(12).normal(size=(D, N))
    ll0 = np.array([m.loglik(x0[:, i]) for i in range(N)])
    lp0 = np.array([m.logprior(x0[:, i]) for i in range(N)])
    r = O.mh_run(m, 14, x0, ll0, lp0, nbin=3, nskip=2, n_rec=40, record_x=True, record_llp=True)
    # reversible jump: 1-D model A (Gaussian), 2-D model B (shell), independence transitions
    a = dict(ndim=1, lik=(LIK_DIAG, [0.3, 0.6]), prior=(0, []), jump=(1, [0.5]), into=(3, [0.3, 0.6]), p=0.4)
    b = dict(ndim=2, lik=(LIK_SHELL, [0.0, 0.0, 1.0, 0.2]), prior=(PRIOR_BOX, [-3, -3, 3, 3, 0.0]),
             jump=(1, [0.3]), into=(3, [0.0, 0.0, 1.0, 1.0]), p=0.6)
    NR = 80
    xa = np.full((1, NR), 0.3)
    xb = np.tile(np.array([[1.0], [0.0]]), (1, NR))
    rj = O.rj_run(a, b, 21, xa, xb, nbin=5, nskip=2, n_rec=50)
    # evidence integrals over the model-A records of the RJ run (1-D samples with repeats)
    inA = rj["rec_tag"].T.reshape(-1) == 0
    pts = rj["rec_x"][:, 0, :].T.reshape(-1)[inA][:, None]
    ll = rj["rec_ll"].T.reshape(-1)[inA]
    lp = rj["rec_lp"].T.reshape(-1)[inA]
    direct = R.evidence_direct(pts, ll, lp, n=16)
    lebesgue = R.evidence_lebesgue(pts, ll, lp, n=16, eps=0.5)
    # run merge of two nested runs of the nested_test.ml Gaussian
    mn = O.Model(2, LIK_DIAG, [0.5, 0.5, 0.1, 0.1], PRIOR_OPEN, [0, 0, 1, 1, 0.0], PROP_GAUSS, [1.0])
    runs = [O.nested(mn, sd, nlive=40, nmcmc=20, k=2) for sd in (31, 32)]
    order, mle, mld, mw = O.nested_merge([(q["ll"], 40, 2) for q in runs])
    np.savez_compressed(os.path.join(HERE, "next_mini.npz"), mix=mix, mix_lik=lik, mix_pri=pri, mix_x0=x0,
                        mix_bits=r["bits"], mix_rec_x=r["rec_x"], mix_x=r["x"],
                        rj_tag=rj["rec_tag"], rj_rec_x=rj["rec_x"], rj_rec_ll=rj["rec_ll"], rj_nb=rj["nb"],
                        ev_pts=pts, ev_ll=ll, ev_lp=lp, ev_direct=direct, ev_lebesgue=lebesgue,
                        merge_ll0=runs[0]["ll"], merge_ll1=runs[1]["ll"], merge_order=order,
                        merge_log_ev=mle, merge_log_dev=mld, merge_wts=mw)


if __name__ == "__main__":
    O.build()
    c2_mini()
    c3_mini()
    c4_mini()
    reductions()
    next_mini()
    print("golden fixtures written to", HERE)
