"""The Gaussian-mixture likelihood kind (MCG_LIK_GAUSS_MIX) on the oracle: the multimodal target
of test/nested_test.ml:41-64, log ((exp g1) +. (exp g2) +. (exp g3) +. (exp g4)) with
g_i = Stats.log_multi_gaussian mu_i sigma_i x (nested_test.ml:52-57, stats.ml:103-108).

The kernels (and the oracle by default) compute each g_i in the DIAG canonical form and fold the
components with a one-pass max-shifted log-sum-exp (csrc/mcg_mh_kernel.h eval_lik); the oracle's
literal mode restates the reference's arithmetic.  Both are checked here, and the reference's
own four-Gaussian test runs on the oracle."""
import ctypes as C
import math

import numpy as np
import pytest

LIK_DIAG, LIK_GMIX, PRIOR_OPEN, PROP_GAUSS = 1, 6, 2, 1

MUS = np.array([[0.25, 0.25], [0.25, 0.75], [0.75, 0.25], [0.75, 0.75]])   # nested_test.ml:42-45
SIGMA = np.array([0.05, 0.05])                                              # nested_test.ml:46


def mix_params(mus, sigmas):
    mus = np.atleast_2d(mus)
    sigmas = np.broadcast_to(np.atleast_2d(sigmas), mus.shape)
    return np.concatenate([[len(mus)], np.concatenate([mus, sigmas], axis=1).ravel()])


def four_gaussians(O):
    # open unit square prior (nested_test.ml:47-51), lp = 0 inside
    return O.Model(2, LIK_GMIX, mix_params(MUS, SIGMA), PRIOR_OPEN, [0, 0, 1, 1, 0.0], PROP_GAUSS, [1.0])


@pytest.fixture
def literal(oracle):
    L = oracle.lib()
    yield L
    L.or_set_literal(0)


def reference_formula(x, mus, sigmas):
    """nested_test.ml:52-57 over stats.ml:98-108, operation for operation."""
    tot = None
    for mu, sg in zip(mus, sigmas):
        r = 0.0
        for i in range(len(mu)):
            dx = (x[i] - mu[i]) / sg[i]
            r = r + ((-0.91893853320467274178 - math.log(sg[i])) - 0.5 * dx * dx)
        e = math.exp(r + 0.0)
        tot = e if tot is None else tot + e
    return math.log(tot)


def test_one_component_mixture_is_the_diag_gaussian(oracle):
    """A one-component mixture is DIAG_GAUSS bit for bit: M + log 1 = M exactly."""
    rng = np.random.default_rng(3)
    for D in (1, 2, 5, 13, 32):
        mu, sg = rng.uniform(-1, 1, D), rng.uniform(0.3, 2, D)
        a = oracle.Model(D, LIK_DIAG, np.concatenate([mu, sg]))
        b = oracle.Model(D, LIK_GMIX, mix_params(mu, sg))
        for _ in range(20):
            x = rng.normal(mu, 2 * sg)
            assert a.loglik(x) == b.loglik(x)


def test_mixture_literal_mode_is_the_reference_formula(oracle, literal):
    """The literal mode is nested_test.ml:52-57 bit for bit; the canonical form is within 1e-13
    (relative to max(|ll|, 1)) of it, on points near every mode and far from all of them (the
    latter is where the reference's exp underflows to 0 for every component below g = -745: the
    canonical form's max shift keeps those finite)."""
    m = four_gaussians(oracle)
    rng = np.random.default_rng(5)
    xs = np.concatenate([MUS[rng.integers(0, 4, 300)] + rng.normal(0, 0.08, (300, 2)),
                         rng.uniform(0, 1, (200, 2))])
    canon = np.array([m.loglik(x) for x in xs])
    literal.or_set_literal(1)
    lit = np.array([m.loglik(x) for x in xs])
    literal.or_set_literal(0)
    ref = np.array([reference_formula(x, MUS, [SIGMA] * 4) for x in xs])
    np.testing.assert_array_equal(lit, ref)
    assert np.all(np.isfinite(canon))
    assert np.max(np.abs(canon - lit) / np.maximum(np.abs(lit), 1.0)) <= 1e-13
    # far out: the reference gives log 0 = -inf, the canonical form the finite log-sum
    far = np.array([3.0, -2.0])
    g = np.array([np.sum(-0.5 * ((far - mu) / SIGMA) ** 2 - np.log(SIGMA)) - math.log(2 * math.pi) for mu in MUS])
    assert g.max() < -745.2                            # exp(g_i) = 0 in the reference
    want = g.max() + math.log(np.sum(np.exp(g - g.max())))
    assert abs(m.loglik(far) - want) <= 1e-13 * abs(want)


def test_mixture_mh_accept_decisions_under_literal_arithmetic(oracle, literal):
    """Every proposal of 256 chains x 256 steps judged with both arithmetics: no decision flips."""
    m = four_gaussians(oracle)
    rng = np.random.default_rng(11)
    N, steps = 256, 256
    x0 = np.ascontiguousarray(MUS[rng.integers(0, 4, N)].T + rng.normal(0, 0.05, (2, N)))
    m = oracle.Model(2, LIK_GMIX, mix_params(MUS, SIGMA), PRIOR_OPEN, [0, 0, 1, 1, 0.0], PROP_GAUSS, [0.04])
    ll0 = np.array([m.loglik(x0[:, i]) for i in range(N)])
    lp0 = np.array([m.logprior(x0[:, i]) for i in range(N)])
    flips = np.zeros(N, np.int64)
    mrel, mmar = C.c_double(), C.c_double()
    rc = literal.or_mh_literal_shadow(C.byref(m.s), 1, N, 0, steps, oracle.dptr(x0), oracle.dptr(ll0),
                                      oracle.dptr(lp0), flips.ctypes.data_as(C.POINTER(C.c_int64)),
                                      C.byref(mrel), C.byref(mmar))
    assert rc == 0
    assert flips.sum() == 0
    assert mrel.value <= 1e-13


@pytest.mark.parametrize("nlive,k", [(64, 1), (1000, 16)])
def test_four_gaussians_nested_under_literal_arithmetic(oracle, literal, nlive, k):
    """The four-Gaussian nested run retires the same points in the same order in both
    arithmetics and agrees on log Z to 1e-12."""
    m = four_gaussians(oracle)
    a = oracle.nested(m, 7, nlive=nlive, nmcmc=20, k=k)
    literal.or_set_literal(1)
    b = oracle.nested(m, 7, nlive=nlive, nmcmc=20, k=k)
    literal.or_set_literal(0)
    assert a["n_dead"] == b["n_dead"] and a["n_gen"] == b["n_gen"]
    np.testing.assert_array_equal(a["pts"], b["pts"])
    assert np.max(np.abs(a["ll"] - b["ll"]) / np.maximum(np.abs(a["ll"]), 1.0)) <= 1e-13
    assert abs(a["log_ev"] - b["log_ev"]) <= 1e-12 * max(abs(a["log_ev"]), 1.0)


def test_nested_four_gaussians_reference_test(oracle):
    """test/nested_test.ml:41-64 on the oracle at the reference's defaults (nlive 1000, nmcmc
    1000, mode_hopping_frac 0.1, epsrel 0.01, k = 1): Z = 4 within 2 err and err < 0.5.  The DE
    mode hop (d = 1 on the difference of two live points, mcmc.ml:209-210) carries walkers
    between the four separated modes.

    The reference's `within 2 err` is a ~1.5-sigma check on one unseeded run, so it is made on
    an ensemble of 8 consecutive seeds (41-48, no selection): every run within 4 err with
    err < 0.5, at least 6 of 8 within 2 err, the mean of (Z - 4)/err within 3 standard errors
    (sd 1.4, as the single-Gaussian ensembles) of 0, and each run's posterior mass about equal
    over the four modes.  (16 seeds: mean 0.02, sd 1.27, 14 of 16 within 2 err.)"""
    zs = []
    for seed in range(41, 49):
        r = oracle.nested(four_gaussians(oracle), seed, nlive=1000, nmcmc=1000, mode_hop=0.1, k=1)
        ev = math.exp(r["log_ev"])
        err = math.exp(oracle.lib().or_log_total_error_estimate(r["log_ev"], r["log_dev"], 1000))
        assert err < 0.5
        assert abs(ev - 4.0) < 4 * err, (seed, ev, err)
        zs.append((ev - 4.0) / err)
        w = np.exp(r["log_wts"])
        assert abs(w.sum() - 1.0) < 1e-8
        q = (r["pts"][:, 0] > 0.5).astype(int) * 2 + (r["pts"][:, 1] > 0.5).astype(int)
        mass = np.array([w[q == j].sum() for j in range(4)])
        assert np.all(np.abs(mass - 0.25) < 0.08), (seed, mass)
    zs = np.array(zs)
    assert np.sum(np.abs(zs) < 2) >= 6, zs
    assert abs(zs.mean()) < 3 * 1.4 / math.sqrt(len(zs)), zs
