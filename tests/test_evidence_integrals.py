"""Evidence.evidence_direct / evidence_lebesgue (evidence.ml:145-221) through libmcg's host
implementation (mcg_evidence.cpp): exact agreement with the list-based restatement in
oracle/evidence_ref.py, and the reference's own statistical tests (test/evidence_test.ml) on
MCMC output of the oracle sampler.  Host-only."""
import math

import numpy as np
import pytest

LIK_DIAG, PRIOR_FLAT, PRIOR_BOX, PROP_MIXTURE = 1, 0, 1, 5


def mcmc_samples(O, mu, sigma, prior, n, seed, step):
    """one chain of Mcmc.mcmc_array with x + random_between (-step) step per dim (symmetric)."""
    D = len(mu)
    prior_kind, prior_params = prior
    mix = [1.0, 1.0, 2.0, 0.0] + list(-np.asarray(step)) + list(step)
    m = O.Model(D, LIK_DIAG, np.concatenate([mu, sigma]), prior_kind, prior_params, PROP_MIXTURE, mix)
    x0 = np.asarray(mu, float)[:, None]
    r = O.mh_run(m, seed, x0, [m.loglik(x0[:, 0])], [m.logprior(x0[:, 0])], nbin=0, nskip=1, n_rec=n,
                 record_accept=False, accumulate=False)
    from mcmc_amd.mcmc import Samples
    return Samples(r["rec_x"], r["rec_ll"], r["rec_lp"])


@pytest.fixture(scope="module")
def E(gpu_lib):
    from mcmc_amd import evidence
    return evidence


@pytest.fixture(scope="module")
def R():
    import evidence_ref
    return evidence_ref


@pytest.mark.parametrize("nbox", [1, 8, 64])
def test_direct_matches_restatement(oracle, E, R, nbox):
    from mcmc_amd.mcmc import remove_repeat_samples
    s = mcmc_samples(oracle, [0.4, 0.6], [1.2, 1.5], (PRIOR_FLAT, []), 3000, 3, [0.6, 0.75])
    pts, ll, lp = remove_repeat_samples(s)
    # keep a few exact duplicates (non-consecutive repeats) to exercise the dedup
    pts, ll, lp = np.concatenate([pts, pts[:50]]), np.concatenate([ll, ll[:50]]), np.concatenate([lp, lp[:50]])
    assert E.evidence_direct((pts, ll, lp), n=nbox) == R.evidence_direct(pts, ll, lp, n=nbox)


@pytest.mark.parametrize("nbox,eps", [(64, 0.2), (16, 1.0), (4, 1e9)])
def test_lebesgue_matches_restatement(oracle, E, R, nbox, eps):
    s = mcmc_samples(oracle, [0.5, 0.45], [0.08, 0.06], (PRIOR_BOX, [0, 0, 1, 1, 0.0]), 3000, 5, [0.04, 0.03])
    pts, ll, lp = s.value[:, :, 0], s.log_likelihood[:, 0], s.log_prior[:, 0]
    assert E.evidence_lebesgue((pts, ll, lp), n=nbox, eps=eps) == R.evidence_lebesgue(pts, ll, lp, n=nbox, eps=eps)


def test_evidence_direct_2d_reference_test(oracle, E):
    """test/evidence_test.ml:54-62: evidence of a normalised 2-D Gaussian posterior from 10,000
    MCMC samples with repeats removed: 1 +- 0.5."""
    from mcmc_amd.mcmc import remove_repeat_samples
    rng = np.random.default_rng(21)
    mu, sigma = rng.random(2), rng.random(2) + 1.0
    s = mcmc_samples(oracle, mu, sigma, (PRIOR_FLAT, []), 10000, 7, sigma / 2)
    ev = E.evidence_direct(remove_repeat_samples(s), n=64)
    assert abs(ev - 1.0) < 0.5


def test_evidence_lebesgue_2d_reference_test(oracle, E):
    """test/evidence_test.ml:78-86: Gaussian of width <= 0.1 in the unit square, eps 0.2."""
    rng = np.random.default_rng(22)
    mu, sigma = 0.3 + 0.4 * rng.random(2), 0.05 + 0.05 * rng.random(2)
    s = mcmc_samples(oracle, mu, sigma, (PRIOR_BOX, [0, 0, 1, 1, 0.0]), 10000, 9, sigma / 2)
    ev = E.evidence_lebesgue(s, n=64, eps=0.2)
    assert abs(ev - 1.0) < 0.5


def test_harmonic_mean_of_samples_matches_linear_formula(oracle, E, R):
    s = mcmc_samples(oracle, [0.2], [0.7], (PRIOR_FLAT, []), 2000, 11, [0.7])
    got = E.evidence_harmonic_mean(s)
    assert abs(got - R.evidence_harmonic_mean(s.log_likelihood[:, 0])) < 1e-12 * got


def test_argument_errors(E):
    from mcmc_amd._lib import InvalidArgument
    with pytest.raises(InvalidArgument):
        E.evidence_direct((np.zeros((0, 2)), np.zeros(0), np.zeros(0)))


def test_harmonic_mean_naive_mode(oracle, E, R):
    """naive=True: the reference's linear-space loop (evidence.ml:101-107), including its
    overflow (exp(-ll) = inf -> Z = 0) and underflow (all 1/exp(ll) = 0 -> Z = inf)."""
    s = mcmc_samples(oracle, [0.2], [0.7], (PRIOR_FLAT, []), 2000, 11, [0.7])
    ll = np.ascontiguousarray(s.log_likelihood[:, 0])
    got = E.evidence_harmonic_mean(s, naive=True)
    want = oracle.lib().or_harmonic_mean_naive(oracle.dptr(ll), len(ll))
    assert abs(got - want) < 1e-13 * want
    pts = np.zeros((2, 1))
    assert E.evidence_harmonic_mean((pts, np.array([-800.0, 0.0]), np.zeros(2)), naive=True) == 0.0
    assert E.evidence_harmonic_mean((pts, np.array([800.0, 800.0]), np.zeros(2)), naive=True) == np.inf
    lz = E.log_evidence_harmonic_mean((pts, np.array([-800.0, 0.0]), np.zeros(2)))   # log-space form
    assert abs(lz - (np.log(2.0) - 800.0)) < 1e-12 * 800
