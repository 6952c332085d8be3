"""The BASELINE.json configs at their full sizes on the GPU (the headline numbers' own workloads),
checked through size-independent properties: analytic evidence, posterior moments, sortedness,
and -- where the oracle finishes in seconds -- a bit-exact slice of the full-size run (Philox
streams are per global chain, so chains [0, 1024) of a 32,768-chain run are the oracle's
1,024-chain run)."""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def T():
    from mcmc_amd import targets
    return targets


def shell_log_z(D, r, w, half):
    """Analytic log Z of one Gaussian shell inside [-half, half]^D (radial quadrature)."""
    rr = np.linspace(max(r - 12 * w, 0.0), r + 12 * w, 200001)
    lsurf = math.log(2.0) + (D / 2) * math.log(math.pi) - math.lgamma(D / 2)
    f = np.exp(-(rr - r) ** 2 / (2 * w * w) + (D - 1) * np.log(np.maximum(rr, 1e-300)) - (D - 1) * math.log(r))
    return (lsurf + (D - 1) * math.log(r) + math.log(np.trapezoid(f, rr))
            - math.log(math.sqrt(2 * math.pi) * w) - D * math.log(2 * half))


def test_c3_full_size_shell_evidence(T):
    """C3 exactly as BASELINE configs[2] / SURVEY 8(d): D = 16 Gaussian shell (r 2, w 0.1) in
    U[-6, 6]^16, nlive 131,072, k 4,096, nmcmc 100, mode_hop 0.1, epsrel 0.01.  The stop test
    fires, the points come out in ascending ll, the weights sum to 1, and log Z is within
    3 sigma_H of the analytic -27.7814 (sigma_H = sqrt(H / nlive))."""
    from mcmc_amd import Context, nested
    D, nlive = 16, 131072
    truth = shell_log_z(D, 2.0, 0.1, 6.0)
    assert abs(truth - (-27.7814)) < 1e-3
    with Context(seed=1) as ctx:
        out = nested.nested_evidence(T.gauss_shell(np.zeros(D), 2.0, 0.1), T.box(-6 * np.ones(D), 6 * np.ones(D)),
                                     epsrel=0.01, nmcmc=100, nlive=nlive, mode_hopping_frac=0.1, k=4096,
                                     ctx=ctx, points=False)
    assert out.converged
    assert np.all(np.diff(out.ll) >= 0)
    w = np.exp(out[3])
    assert abs(w.sum() - 1.0) < 1e-8
    H = float(np.sum(w * out.ll) - out[0])
    sigma = math.sqrt(H / nlive)
    assert abs(out[0] - truth) <= 3 * sigma, (out[0], truth, sigma)
    assert out.n_dead % 4096 == 0 and out.n_dead > 10 * nlive


def test_c4_full_size_moments_and_oracle_slice(oracle, T):
    """C4 as BASELINE configs[3]: D = 8 N(0, 1) target, kD interp proposal from M = 32,768 exact
    draws, 32,768 chains.  The moments of 100 recorded sweeps match the target, and the accept
    bitmap of chains [0, 1024) equals the oracle's run of those 1,024 chains bit for bit."""
    from mcmc_amd import Context
    D, N, M, steps = 8, 32768, 32768, 100
    rng = np.random.default_rng(4)
    pts = rng.normal(size=(M, D))
    lo, hi = -10 * np.ones(D), 10 * np.ones(D)
    lik, pri = T.diag_gauss(np.zeros(D), np.ones(D)), T.box(lo, hi)
    x0 = rng.normal(size=(D, N))
    with Context(seed=3) as ctx:
        ctx.set_model(lik, pri, T.KdInterp(pts, lo, hi))
        ctx.init(x0)
        ctx.run(nbin=0, nskip=1, n_rec=steps + 1, record_x=False, record_llp=False, record_accept=True,
                accumulate=True)
        _, _, _, bits = ctx.records(x=False, llp=False, accept=True)
        mean, sd, _ = ctx.stats()
        acc, rej = ctx.counters()
    assert 0.0 < acc / (acc + rej) < 0.05           # the kD proposal at M = 32,768: ~0.1 %
    np.testing.assert_allclose(mean, 0.0, atol=0.02)
    np.testing.assert_allclose(sd, 1.0, atol=0.02)
    okd = oracle.KdTree(pts, lo, hi)
    m = oracle.Model(D, lik.kind, lik.params, pri.kind, pri.params, 3, [0.0], okd)
    xs = np.ascontiguousarray(x0[:, :1024])
    ll0 = np.array([m.loglik(xs[:, i]) for i in range(1024)])
    lp0 = np.array([m.logprior(xs[:, i]) for i in range(1024)])
    o = oracle.mh_run(m, 3, xs, ll0, lp0, nbin=0, nskip=1, n_rec=steps + 1, record_x=False, record_llp=False,
                      accumulate=False, nthreads=8)
    np.testing.assert_array_equal(bits[:, :1024 // 64], o["bits"])


def test_c5_full_size_per_gpu_moments(T):
    """C5 as one GPU's share of BASELINE configs[4]: D = 64 full-covariance Gaussian,
    131,072 chains on the matrix-core kernel; 200 recorded sweeps give the target's mean and
    marginal sds (per dim, within the Monte Carlo error of correlated chains)."""
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))
    import bench_c5 as b
    from mcmc_amd import Context
    mu, cov, s = b.c5_target()
    N = 131072
    with Context(seed=1) as ctx:
        ctx.set_model(T.fullcov_gauss(mu, cov), T.flat_prior(), T.gauss(s))
        ctx.init(b.start_points(mu, cov, 0, N))
        ctx.run(nbin=50, nskip=1, n_rec=200, record_x=False, record_llp=False, accumulate=True)
        mean, sd, lz = ctx.stats()
        acc, rej = ctx.counters()
    sdt = np.sqrt(np.diag(cov))
    assert 0.3 < acc / (acc + rej) < 0.8              # scale from the smallest eigenvalue: ~0.58
    assert np.max(np.abs(mean - mu) / sdt) < 0.02
    assert np.max(np.abs(sd / sdt - 1)) < 0.02
    assert np.isfinite(lz)
