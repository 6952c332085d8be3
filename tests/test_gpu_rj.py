"""GPU parity of the reversible-jump kernel (mcg_rj_kernel.h) against the oracle's restatement
of Mcmc.make_rjmcmc_sampler / rjmcmc_array (mcmc.ml:89-153): bit-exact records, model tags,
final states and counters; the reference's statistical tests on the GPU path."""
import numpy as np
import pytest

from test_rjmcmc import (LIK_DIAG, LIK_FLAT, LIK_SHELL, PRIOR_BOX, PRIOR_FLAT, PRIOR_GAUSS, gauss_prior_models,
                         gaussians_models, top_hat_models)

pytestmark = pytest.mark.gpu


def to_desc(T, m, kd_pts=None):
    """oracle model dict -> targets.RjModel."""
    def lik():
        kind, p = m["lik"]
        if kind == LIK_FLAT:
            return T.flat(m["ndim"])
        if kind == LIK_DIAG:
            return T.diag_gauss(p[:m["ndim"]], p[m["ndim"]:])
        return T.gauss_shell(p[:m["ndim"]], p[m["ndim"]], p[m["ndim"] + 1])

    def prior():
        kind, p = m["prior"]
        if kind == PRIOR_FLAT:
            return T.flat_prior()
        D = m["ndim"]
        if kind == PRIOR_GAUSS:
            return T.gauss_prior(p[:D], p[D:2 * D])
        return T.box(p[:D], p[D:2 * D], p[2 * D])

    kd = T.rj_kd(kd_pts, np.zeros(m["ndim"]), np.ones(m["ndim"])) if kd_pts is not None else None

    def jump(spec):
        kind, p = spec
        if kind == 1:
            return T.rj_gauss(p)
        if kind == 2:
            return T.rj_wrap(p[:m["ndim"]], p[m["ndim"]:2 * m["ndim"]], p[2 * m["ndim"]:])
        if kind == 3:
            return T.rj_indep_gauss(p[:m["ndim"]], p[m["ndim"]:])
        return kd

    return T.RjModel(lik(), prior(), jump(m["jump"]), jump(m["into"]), m["p"])


def run_both(oracle, a, b, xa, xb, seed, nbin, nskip, n_rec, kd_pts=(None, None), tags=None):
    from mcmc_amd import Context, mcmc, targets as T
    ctx = Context(seed=seed)
    N = xa.shape[1]
    s = mcmc.rjmcmc_array(n_rec, to_desc(T, a, kd_pts[0]), to_desc(T, b, kd_pts[1]), (xa, xb),
                          nchains=N, nbin=nbin, nskip=nskip, ctx=ctx, models=tags)
    x, ll, lp = ctx.state()
    acc, _ = ctx.counters()
    ctx.close()
    o = oracle.rj_run(a, b, seed, xa, xb, nbin=nbin, nskip=nskip, n_rec=n_rec, tags=tags)
    return s, (x, ll, lp, acc), o


def assert_rj_same(s, st, o):
    np.testing.assert_array_equal(s.model, o["rec_tag"])
    np.testing.assert_array_equal(s.value, o["rec_x"])
    np.testing.assert_array_equal(s.log_likelihood, o["rec_ll"])
    np.testing.assert_array_equal(s.log_prior, o["rec_lp"])
    x, ll, lp, acc = st
    np.testing.assert_array_equal(x, o["x"])
    np.testing.assert_array_equal(ll, o["ll"])
    assert acc == int(o["nacc"].sum())
    assert s.counts[1] == int(o["nb"].sum())


def test_rj_gaussians_bit_exact(oracle):
    a, b = gaussians_models(0.3, 0.6, 0.8, 0.4, 0.1, 0.9)
    N = 200
    s, st, o = run_both(oracle, a, b, np.full((1, N), 0.3), np.full((1, N), 0.8), 3, 5, 2, 40)
    assert_rj_same(s, st, o)


def test_rj_top_hats_kd_bit_exact(oracle):
    a, b, pts = top_hat_models(oracle, npts=500)
    N = 150
    s, st, o = run_both(oracle, a, b, np.full((2, N), 0.5), np.full((2, N), 0.5), 5, 4, 3, 30, kd_pts=pts)
    assert_rj_same(s, st, o)


def test_rj_mixed_dimensions_bit_exact(oracle):
    a = dict(ndim=2, lik=(LIK_DIAG, [0.2, -0.1, 1.0, 0.5]), prior=(PRIOR_FLAT, []),
             jump=(1, [0.8]), into=(3, [0.2, -0.1, 1.0, 0.5]), p=0.3)
    b = dict(ndim=3, lik=(LIK_SHELL, [0, 0, 0, 1.0, 0.2]), prior=(PRIOR_BOX, [-3, -3, -3, 3, 3, 3, 0.0]),
             jump=(1, [0.3]), into=(3, [0, 0, 0, 1, 1, 1]), p=0.7)
    N = 130
    rng = np.random.default_rng(2)
    tags = rng.integers(0, 2, N).astype(np.uint8)
    s, st, o = run_both(oracle, a, b, rng.normal(size=(2, N)), 0.5 + 0.1 * rng.normal(size=(3, N)),
                        9, 3, 2, 50, tags=tags)
    assert_rj_same(s, st, o)


def test_rj_top_hats_evidence_ratio_on_gpu(oracle):
    """mcmc_test.ml:152-182 on the GPU path: Z1/Z2 = 4 +- 0.1."""
    from mcmc_amd import Context, mcmc, targets as T
    a, b, pts = top_hat_models(oracle)
    N = 4096
    ctx = Context(seed=17)
    s = mcmc.rjmcmc_array(500, to_desc(T, a, pts[0]), to_desc(T, b, pts[1]),
                          (np.full((2, N), 0.5), np.full((2, N), 0.5)), nchains=N, nbin=50, nskip=10,
                          ctx=ctx, record_x=False)
    ctx.close()
    assert abs(mcmc.rjmcmc_evidence_ratio(s) - 4.0) < 0.1


def test_rj_gaussian_priors_bit_exact(oracle):
    """DIAG_GAUSS priors per model (lpa / lpb, mcmc.ml:116-118), models of different dimension
    (the smaller one's prior padded with zero constants): records, tags, state and counters equal
    the oracle's bit for bit, and the model count ratio is the analytic pa Z_A / (pb Z_B)."""
    a, b, ratio = gauss_prior_models()
    N = 512
    s, st, o = run_both(oracle, a, b, np.full((1, N), 0.1), np.full((2, N), 0.1), 21, 20, 3, 200)
    assert_rj_same(s, st, o)
    np.testing.assert_array_equal(st[2], o["lp"])
    na, nb = s.counts
    assert abs(na / nb / ratio - 1.0) < 0.08, (na / nb, ratio)
