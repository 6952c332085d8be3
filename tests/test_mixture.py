"""Mcmc.combine_jump_proposals (mcmc.ml:165-185) as the MIXTURE proposal kind: the reference's own
statistical tests restated on the oracle (CPU), and the C-ABI's argument checking."""
import math

import numpy as np
import pytest

LIK_DIAG, PRIOR_FLAT, PROP_MIXTURE = 1, 0, 5
MIX_GAUSS, MIX_SHIFT, MIX_WRAP, MIX_KD = 1, 2, 3, 4


def mixture_params(comps):
    """comps: (p, kind, ljp_mode, params) -> include/mcg.h MIXTURE parameter vector."""
    out = [float(len(comps))]
    for p, kind, mode, params in comps:
        out += [p, kind, mode] + list(params)
    return np.array(out)


def run_chains(O, comps, mu, sigma, nchains, nrec, nskip, seed=5, kd=None):
    D = len(mu)
    m = O.Model(D, LIK_DIAG, np.concatenate([mu, sigma]), PRIOR_FLAT, [], PROP_MIXTURE,
                mixture_params(comps), kd)
    x0 = np.tile(np.asarray(mu, float)[:, None], (1, nchains))
    ll0 = np.array([m.loglik(x0[:, i]) for i in range(nchains)])
    lp0 = np.zeros(nchains)
    return O.mh_run(m, seed, x0, ll0, lp0, nbin=100, nskip=nskip, n_rec=nrec, record_x=True,
                    record_llp=False, record_accept=False, accumulate=False, nthreads=8)


def test_combine_jump_proposal_reference_test(oracle):
    """test/mcmc_test.ml:184-207: left jump x - U (weight 1) and right jump x + U (weight 2) with
    their one-sided log_jump_probs on a N(0, 1) target: mean 0 +- 0.05, sigma 1 +- 1%."""
    comps = [(1.0, MIX_SHIFT, 1, [-1.0, 0.0]), (2.0, MIX_SHIFT, 1, [0.0, 1.0])]
    r = run_chains(oracle, comps, [0.0], [1.0], 1000, 1000, 5)
    xs = r["rec_x"][:, 0, :].ravel()
    assert abs(xs.mean()) < 0.05
    assert abs(xs.std() - 1.0) < 1e-2


def test_left_biased_proposal_reference_test(oracle):
    """test/mcmc_test.ml:63-85: x - U sigma with prob 0.75, x + U sigma with 0.25; the log_jump_prob
    is log 0.75 / log 0.25 by side (the mixture's density differs by the constant -log sigma on
    both sides, which cancels).  Mean and sigma within 20 sigma/sqrt(n)."""
    rng = np.random.default_rng(3)
    mu, sigma = rng.random(), rng.random() + 1.0
    comps = [(0.75, MIX_SHIFT, 1, [-sigma, 0.0]), (0.25, MIX_SHIFT, 1, [0.0, sigma])]
    r = run_chains(oracle, comps, [mu], [sigma], 200, 500, 1)
    xs = r["rec_x"][:, 0, :].ravel()
    err = 20.0 * sigma / math.sqrt(len(xs))
    assert abs(xs.mean() - mu) < err
    assert abs(xs.std() - sigma) < err


def test_mixed_kinds_sample_the_target(oracle):
    """Gaussian + symmetric-uniform (ljp 0) + wrapping-uniform components on a 3-D Gaussian."""
    mu, sg = np.array([0.3, -0.5, 1.0]), np.array([0.5, 1.0, 2.0])
    comps = [(0.5, MIX_GAUSS, 1, [0.6, 1.0, 1.5]),
             (0.3, MIX_SHIFT, 0, [-1.0, -1.0, -1.0, 1.0, 1.0, 1.0]),
             (0.2, MIX_WRAP, 0, [-20, -20, -20, 20, 20, 20, 1.0, 2.0, 3.0])]
    r = run_chains(oracle, comps, mu, sg, 400, 500, 2)
    xs = r["rec_x"].transpose(1, 0, 2).reshape(3, -1)
    np.testing.assert_allclose(xs.mean(axis=1), mu, atol=0.05 * sg.max())
    np.testing.assert_allclose(xs.std(axis=1), sg, rtol=0.03)


def test_kd_component_samples_the_target(oracle):
    """Interpolate_pdf kD jump mixed with a local Gaussian jump (Farr-Mandel usage)."""
    D = 2
    rng = np.random.default_rng(8)
    pts = rng.normal(size=(512, D))
    kd = oracle.KdTree(pts, -10 * np.ones(D), 10 * np.ones(D))
    comps = [(0.7, MIX_KD, 1, []), (0.3, MIX_GAUSS, 1, [0.5, 0.5])]
    r = run_chains(oracle, comps, np.zeros(D), np.ones(D), 400, 500, 2, kd=kd)
    xs = r["rec_x"].transpose(1, 0, 2).reshape(D, -1)
    np.testing.assert_allclose(xs.mean(axis=1), 0.0, atol=0.05)
    np.testing.assert_allclose(xs.std(axis=1), 1.0, rtol=0.04)


def test_private_log_sum_is_log_one_plus_exp(oracle):
    """Two equal components with ljp 0: log_jp = log_sum_logs(log .5, log .5) = 0 up to rounding,
    identical forward and backward, so the proposal is exactly symmetric (ratio term 0)."""
    comps = [(1.0, MIX_SHIFT, 0, [-0.5, 0.5]), (1.0, MIX_GAUSS, 0, [0.3])]
    r = run_chains(oracle, comps, [0.0], [1.0], 64, 200, 1)
    assert np.isfinite(r["rec_x"]).all()


def test_mixture_argument_errors(gpu_lib):
    """C-ABI validation happens on the host: no device needed to reject bad descriptors."""
    import ctypes as C
    L = gpu_lib
    assert hasattr(L.lib(), "mcg_set_proposal")
    from mcmc_amd import targets as T
    with pytest.raises(ValueError):
        T.combine_jump_proposals([(1.0, T.Proposal(L.PROP_DE, [0.0]))], 2)


def _walk_falls_through(w, u):
    """the pick of mcmc.ml:168-173 in IEEE double: True when u passes every weight"""
    for p in w:
        if u < p:
            return False
        u = u - p
    return True


def _normalised(p):
    tot = 0.0
    for x in p:
        tot = tot + x
    return [x / tot for x in p]


# weights whose rounded normalised walk lets the largest draw through (found by search)
FALL_THROUGH_WEIGHTS = [float.fromhex(h) for h in ("0x1.7fad7432340e0p+8", "0x1.0569a03eef9cap-10",
                                                    "0x1.ea6aec618a7e9p+9")]


def test_mixture_pick_fall_through_is_decided_by_the_largest_draw():
    """The reference raises Failure when u passes every normalised weight (mcmc.ml:173).  The
    walk is monotone in u, so that happens for some draw iff it happens for the largest u53 draw,
    1 - 2^-53 -- the check mcg_set_proposal makes (pack_mixture).  Random weight vectors: no
    smaller draw falls through when the largest does not; the crafted vector falls through for the
    largest draw only near the top of (0, 1)."""
    rng = np.random.default_rng(3)
    umax = 1.0 - 2.0 ** -53
    for _ in range(3000):
        w = _normalised(list(rng.random(rng.integers(2, 9)) * rng.choice([1.0, 1e-3, 1e3], 1)))
        if not _walk_falls_through(w, umax):
            us = np.concatenate([rng.random(64), umax - rng.integers(1, 64, 16) * 2.0 ** -53])
            assert not any(_walk_falls_through(w, float(u)) for u in us)
    w = _normalised(FALL_THROUGH_WEIGHTS)
    assert _walk_falls_through(w, umax)
    assert not _walk_falls_through(w, 0.5)


@pytest.mark.gpu
def test_mixture_refuses_fall_through_weights():
    """mcg_set_proposal refuses weights the reference's pick can fall through, with MCG_EFAIL
    (Failure) and the reference's message; the same components with ordinary weights run."""
    from mcmc_amd import Context, targets as T
    from mcmc_amd._lib import Failure
    lik = T.diag_gauss([0.0], [1.0])
    pri = T.flat_prior()
    comps = lambda ws: [(w, T.gauss([0.5])) for w in ws]
    with Context(seed=1) as ctx:
        with pytest.raises(Failure, match="no jump proposal to select"):
            ctx.set_model(lik, pri, T.combine_jump_proposals(comps(FALL_THROUGH_WEIGHTS), 1))
        ctx.set_model(lik, pri, T.combine_jump_proposals(comps([1.0, 2.0, 3.0]), 1))
        ctx.init(np.zeros((1, 64)))
        ctx.run(nbin=10, nskip=1, n_rec=1)
