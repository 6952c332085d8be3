"""The DIAG_GAUSS prior kind (MCG_PRIOR_DIAG_GAUSS, include/mcg.h) on the oracle: its log density
is Stats.log_multi_gaussian (stats.ml:98-108) in canonical form, and with it the nested
walkers' MH test `log u < log_prior y - log_prior x` (nested.ml:54-59) is a real test.  The
analytic evidence of a Gaussian likelihood under a Gaussian prior pins the whole loop:
Z = prod_d N(mu_L,d; mu_P,d, sqrt(sigma_L,d^2 + sigma_P,d^2))."""
import math

import numpy as np
import pytest

LIK_DIAG, PRIOR_GAUSS = 1, 3


def _gauss_lz(muL, sL, muP, sP):
    v = sL ** 2 + sP ** 2
    return float(np.sum(-0.5 * np.log(2 * math.pi * v) - 0.5 * (muL - muP) ** 2 / v))


def _model(O, muL, sL, muP, sP, s=0.5):
    D = len(muL)
    return O.Model(D, LIK_DIAG, np.concatenate([muL, sL]), PRIOR_GAUSS, np.concatenate([muP, sP]),
                   1, [s])


def test_gauss_prior_is_log_multi_gaussian(oracle):
    """Canonical form within 1e-13 of the literal reference sum; the literal mode is that sum."""
    O = oracle
    rng = np.random.default_rng(3)
    for D in (1, 3, 8, 13, 32):
        muP, sP = rng.normal(size=D), rng.uniform(0.3, 3.0, D)
        m = _model(O, np.zeros(D), np.ones(D), muP, sP)
        for _ in range(20):
            x = rng.normal(muP, 2 * sP)
            lit = sum(-0.91893853320467274178 - math.log(s) - 0.5 * ((xi - mu) / s) ** 2
                      for xi, mu, s in zip(x, muP, sP))
            assert abs(m.logprior(x) - lit) <= 1e-13 * max(abs(lit), 1.0)
            O.lib().or_set_literal(1)
            try:
                assert m.logprior(x) == pytest.approx(lit, rel=1e-15, abs=1e-15)
            finally:
                O.lib().or_set_literal(0)


def test_gauss_prior_equals_diag_likelihood_bits(oracle):
    """The prior shares the DIAG_GAUSS likelihood's canonical constants and sum: bit-equal."""
    O = oracle
    rng = np.random.default_rng(4)
    D = 20
    mu, sg = rng.normal(size=D), rng.uniform(0.5, 2.0, D)
    a = O.Model(D, LIK_DIAG, np.concatenate([mu, sg]), 0, [], 1, [1.0])
    b = _model(O, np.zeros(D), np.ones(D), mu, sg)
    for _ in range(50):
        x = rng.normal(size=D) * 3
        assert a.loglik(x) == b.logprior(x)


def test_nested_gauss_prior_analytic_evidence(oracle):
    """Nested sampling draws the live points from the Gaussian prior and runs the walkers'
    prior-weighted MH test; log Z lands on the analytic value.  Six seeds: each within 4 sigma,
    their mean within 3 sigma / sqrt(6) (sigma = sqrt(H / nlive))."""
    O = oracle
    D = 3
    muL, sL = np.array([0.4, -0.3, 0.2]), np.array([0.3, 0.5, 0.4])
    muP, sP = np.array([0.0, 0.1, -0.2]), np.array([1.0, 1.5, 0.8])
    lz = _gauss_lz(muL, sL, muP, sP)
    m = _model(O, muL, sL, muP, sP)
    nlive, deltas, sig = 400, [], []
    for seed in range(11, 17):
        o = O.nested(m, seed, nlive=nlive, nmcmc=40, k=1, mode_hop=0.1)
        w = np.exp(o["log_wts"])
        H = float(np.sum(w * o["ll"]) - o["log_ev"])
        s = math.sqrt(H / nlive)
        assert abs(o["log_ev"] - lz) < 4 * s
        deltas.append(o["log_ev"] - lz)
        sig.append(s)
        # the posterior of a Gaussian x Gaussian: precision-weighted mean
        post_mu = (muL / sL ** 2 + muP / sP ** 2) / (1 / sL ** 2 + 1 / sP ** 2)
        mean = (w[:, None] * o["pts"]).sum(axis=0)
        assert np.all(np.abs(mean - post_mu) < 0.1)
        # every dead and live point carries its own prior log density
        for i in range(0, len(o["lp"]), 97):
            assert o["lp"][i] == m.logprior(o["pts"][i])
    assert abs(np.mean(deltas)) < 3 * np.mean(sig) / math.sqrt(len(deltas))


def test_nested_gauss_prior_walker_test_is_live(oracle):
    """With a box prior every passing proposal is accepted; with the Gaussian prior some passing
    proposals are rejected by log u >= lp(y) - lp(x).  Observable: the same likelihood, seed and
    walk under a prior of sigma 10 (nearly flat over the likelihood) and of sigma 0.5 give
    different dead-point sequences from the first generation on."""
    O = oracle
    D = 2
    muL, sL = np.array([0.2, -0.1]), np.array([0.2, 0.3])
    a = O.nested(_model(O, muL, sL, np.zeros(D), 10 * np.ones(D)), 5, nlive=50, nmcmc=10, k=1,
                 max_iter=20)
    b = O.nested(_model(O, muL, sL, np.zeros(D), 0.5 * np.ones(D)), 5, nlive=50, nmcmc=10, k=1,
                 max_iter=20)
    assert not np.array_equal(a["ll"][:20], b["ll"][:20])


def test_mh_gauss_prior_posterior_moments(oracle):
    """Mcmc.mcmc_array under a Gaussian prior samples the product posterior."""
    O = oracle
    D = 4
    muL, sL = np.array([1.0, -1.0, 0.5, 0.0]), np.array([0.5, 0.8, 1.0, 0.3])
    muP, sP = np.zeros(D), np.array([1.0, 0.5, 2.0, 0.3])
    m = _model(O, muL, sL, muP, sP, s=0.6)
    N = 512
    prec = 1 / sL ** 2 + 1 / sP ** 2
    post_mu, post_sd = (muL / sL ** 2 + muP / sP ** 2) / prec, 1 / np.sqrt(prec)
    x0 = np.random.default_rng(1).normal(post_mu[:, None], post_sd[:, None], size=(D, N))
    ll = np.array([m.loglik(x0[:, i]) for i in range(N)])
    lp = np.array([m.logprior(x0[:, i]) for i in range(N)])
    r = O.mh_run(m, 3, x0, ll, lp, nbin=100, nskip=1, n_rec=400, record_x=True, record_llp=True,
                 nthreads=8)
    xs = r["rec_x"].transpose(1, 0, 2).reshape(D, -1)
    assert np.all(np.abs(xs.mean(axis=1) - post_mu) < 0.05 * post_sd + 0.01)
    assert np.all(np.abs(xs.std(axis=1) / post_sd - 1) < 0.05)
    np.testing.assert_array_equal(r["rec_lp"][-1], [m.logprior(r["rec_x"][-1][:, i]) for i in range(N)])
