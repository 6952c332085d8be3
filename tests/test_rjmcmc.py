"""Reversible-jump MCMC (Mcmc.make_rjmcmc_sampler / rjmcmc_array, mcmc.ml:89-153): the
reference's own statistical tests (test/mcmc_test.ml:114-182) restated on the oracle (CPU)."""
import numpy as np

LIK_FLAT, LIK_DIAG, LIK_SHELL = 0, 1, 3
PRIOR_FLAT, PRIOR_BOX, PRIOR_GAUSS = 0, 1, 3
RJ_GAUSS, RJ_WRAP, RJ_INDEP, RJ_KD = 1, 2, 3, 4


def gaussians_models(mu1, s1, mu2, s2, p1, p2):
    """test_rjmcmc_gaussians: each model's posterior is a normalised N(mu_i, s_i) (the reference
    splits it as 0.5/0.5 and 0.3/0.7 between likelihood and prior; only the sum enters), the
    internal and transition jumps are independence draws from that Gaussian."""
    def m(mu, s, p):
        g = (RJ_INDEP, [mu, s])
        return dict(ndim=1, lik=(LIK_DIAG, [mu, s]), prior=(PRIOR_FLAT, []), jump=g, into=g, p=p)
    return m(mu1, s1, p1), m(mu2, s2, p2)


def test_rjmcmc_gaussians_reference_test(oracle):
    """mcmc_test.ml:114-150: model fractions p1, p2 within 10 %, evidence ratio p1/p2 +- 0.1."""
    rng = np.random.default_rng(11)
    mu1, s1, mu2, s2 = rng.random(), 0.2 + rng.random(), rng.random(), 0.2 + rng.random()
    a, b = gaussians_models(mu1, s1, mu2, s2, 0.1, 0.9)
    N = 1000
    r = oracle.rj_run(a, b, 3, np.full((1, N), mu1), np.full((1, N), mu2), nbin=50, nskip=10, n_rec=1000)
    nb = int(r["rec_tag"].sum())
    na = r["rec_tag"].size - nb
    pp1, pp2 = na / (na + nb), nb / (na + nb)
    assert abs(pp1 - 0.1) < 0.1 * 0.1 and abs(pp2 - 0.9) < 0.1 * 0.9
    assert abs(na / nb - 0.1 / 0.9) < 0.1
    assert int(r["nb"].sum()) == nb


def top_hat_models(O, npts=4000, seed=1):
    """test_rjmcmc_top_hats_interp: flat likelihoods on [0,1]^2 and [0.25,0.75]^2 (as box priors
    with lp_in 0, which gives the same posterior), wrapping-uniform internal jumps, kD
    interpolated transitions built from samples of each model."""
    rng = np.random.default_rng(seed)
    lo, hi = np.zeros(2), np.ones(2)
    p1 = rng.random((npts, 2))
    p2 = 0.25 + 0.5 * rng.random((npts, 2))
    k1, k2 = O.KdTree(p1, lo, hi), O.KdTree(p2, lo, hi)
    wrap = (RJ_WRAP, [0, 0, 1, 1, 0.5, 0.5])
    a = dict(ndim=2, lik=(LIK_FLAT, []), prior=(PRIOR_BOX, [0, 0, 1, 1, 0.0]), jump=wrap,
             into=(RJ_KD, []), kd=k1, p=0.5)
    b = dict(ndim=2, lik=(LIK_FLAT, []), prior=(PRIOR_BOX, [0.25, 0.25, 0.75, 0.75, 0.0]), jump=wrap,
             into=(RJ_KD, []), kd=k2, p=0.5)
    return a, b, (p1, p2)


def test_rjmcmc_top_hats_interp_reference_test(oracle):
    """mcmc_test.ml:152-182: evidence ratio Z1/Z2 = 4 +- 0.1 with kD transition jumps."""
    a, b, _ = top_hat_models(oracle)
    N = 1000
    r = oracle.rj_run(a, b, 5, np.full((2, N), 0.5), np.full((2, N), 0.5), nbin=50, nskip=10, n_rec=1000)
    nb = int(r["rec_tag"].sum())
    na = r["rec_tag"].size - nb
    assert abs(na / nb - 4.0) < 0.1


def test_rjmcmc_records_follow_schedule_and_padding(oracle):
    """Different dimensions: samples of the smaller model have zero padding; lp carries log p."""
    mu = np.array([0.2, -0.1])
    a = dict(ndim=2, lik=(LIK_DIAG, [0.2, -0.1, 1.0, 0.5]), prior=(PRIOR_FLAT, []),
             jump=(RJ_GAUSS, [0.8]), into=(RJ_INDEP, [0.2, -0.1, 1.0, 0.5]), p=0.3)
    b = dict(ndim=3, lik=(LIK_SHELL, [0, 0, 0, 1.0, 0.2]), prior=(PRIOR_BOX, [-3, -3, -3, 3, 3, 3, 0.0]),
             jump=(RJ_GAUSS, [0.3]), into=(RJ_INDEP, [0, 0, 0, 1, 1, 1]), p=0.7)
    N = 300
    r = oracle.rj_run(a, b, 9, np.tile(mu[:, None], (1, N)), np.zeros((3, N)) + 0.5, nbin=3, nskip=2, n_rec=50)
    inA = r["rec_tag"] == 0
    assert inA.any() and (~inA).any()
    assert np.all(r["rec_x"][:, 2, :][inA] == 0.0)
    np.testing.assert_allclose(r["rec_lp"][inA], np.log(0.3))
    np.testing.assert_allclose(r["rec_lp"][~inA], np.log(0.7))


def gauss_prior_models():
    """Two models with Gaussian priors lpa / lpb (Stats.log_multi_gaussian, mcmc.ml:116-118): a
    Gaussian likelihood N(mu, s) under a N(0, tau) prior per dim, so Z = prod_d N(mu_d; 0,
    sqrt(s_d^2 + tau_d^2)); internal and transition jumps are independence draws from the exact
    posterior N(m, v) (precision 1/s^2 + 1/tau^2)."""
    def m(mu, s, tau, p):
        mu, s, tau = (np.asarray(v, float) for v in (mu, s, tau))
        prec = 1 / s ** 2 + 1 / tau ** 2
        post = (RJ_INDEP, list(mu / s ** 2 / prec) + list(1 / np.sqrt(prec)))
        z = np.prod(np.exp(-mu ** 2 / (2 * (s ** 2 + tau ** 2))) / np.sqrt(2 * np.pi * (s ** 2 + tau ** 2)))
        return dict(ndim=len(mu), lik=(LIK_DIAG, list(mu) + list(s)), prior=(PRIOR_GAUSS, [0.0] * len(mu) + list(tau)),
                    jump=post, into=post, p=p), z
    (a, za), (b, zb) = m([0.3], [0.5], [1.0], 0.4), m([0.2, -0.4], [0.6, 0.8], [1.5, 1.5], 0.6)
    return a, b, (0.4 * za) / (0.6 * zb)


def test_rjmcmc_gaussian_priors_evidence_ratio(oracle):
    """Gaussian model priors in the reversible-jump sampler: the model count ratio estimates
    pa Z_A / (pb Z_B) (analytic, ~4.1), within 3 %; a chain in model A has lp = log pa + the
    prior's log density."""
    a, b, ratio = gauss_prior_models()
    N = 1000
    r = oracle.rj_run(a, b, 17, np.full((2, N), 0.1), np.full((2, N), 0.1), nbin=50, nskip=5, n_rec=600)
    nb = int(r["rec_tag"].sum())
    na = r["rec_tag"].size - nb
    assert abs(na / nb / ratio - 1.0) < 0.03, (na / nb, ratio)
    inA = r["rec_tag"] == 0
    x = r["rec_x"][:, 0, :][inA]
    lp_expect = np.log(0.4) - 0.5 * np.log(2 * np.pi) - 0.5 * x ** 2
    np.testing.assert_allclose(r["rec_lp"][inA], lp_expect, rtol=1e-12, atol=1e-12)
