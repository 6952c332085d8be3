"""GPU parity of the DIAG_GAUSS prior kind (include/mcg.h) against the oracle, bit for bit: the MH
kernel's generic step (a separable likelihood under a Gaussian prior runs mh_kernel's
kUniGaussPrior instance, not the fused box step), the kD register path, the DE and mixture
proposals, padded widths, and the nested walkers whose MH test log u < lp(y) - lp(x)
(nested.ml:54-59) is live under this prior, at k = 1 and k > 1 and on every walker lane split."""
import math

import numpy as np
import pytest

from test_gpu_mh import assert_same, run_gpu, run_oracle
from test_gpu_nested import assert_nested_same, gpu_nested, oracle_nested

pytestmark = [pytest.mark.gpu, pytest.mark.filterwarnings("ignore:nested_evidence. max_dead")]


@pytest.fixture(scope="module")
def T():
    from mcmc_amd import targets
    return targets


def _prior(T, D, seed=0, scale=1.5):
    rng = np.random.default_rng(100 + seed)
    return T.gauss_prior(rng.uniform(-0.5, 0.5, D), rng.uniform(0.5, 1.0, D) * scale)


@pytest.mark.parametrize("D,lanes", [(32, 1), (32, 2), (32, 4), (32, 8), (5, 1), (13, 1), (16, 4)])
def test_mh_diag_lik_gauss_prior_bit_exact(oracle, T, D, lanes):
    rng = np.random.default_rng(D)
    mu, sg = rng.uniform(-1, 1, D), rng.uniform(0.5, 2, D)
    lik, pri = T.diag_gauss(mu, sg), _prior(T, D)
    x0 = rng.normal(mu[:, None], sg[:, None], size=(D, 300))
    s = 2.38 / math.sqrt(D)
    g = run_gpu(lik, pri, T.gauss(s), x0, 7, nbin=3, nskip=2, n_rec=40, lanes=lanes)
    o = run_oracle(oracle, lik, pri, T.gauss(s), x0, 7, 3, 2, 40)
    assert_same(g, o)
    np.testing.assert_array_equal(g["lp"], o["lp"])
    assert np.all(np.isfinite(g["rec_lp"]))


@pytest.mark.parametrize("D", [4, 16])
def test_mh_flat_and_shell_lik_gauss_prior_bit_exact(oracle, T, D):
    rng = np.random.default_rng(D + 1)
    x0 = rng.normal(size=(D, 130))
    for lik in (T.flat(D), T.gauss_shell(np.zeros(D), 1.5, 0.3)):
        pri = _prior(T, D, 1)
        g = run_gpu(lik, pri, T.gauss(0.4), x0, 9, nbin=0, nskip=1, n_rec=50)
        o = run_oracle(oracle, lik, pri, T.gauss(0.4), x0, 9, 0, 1, 50)
        assert_same(g, o)


def test_mh_fullcov_gauss_prior_runs_one_lane_kernel_bit_exact(oracle, T):
    """Full covariance at D 16 takes the one-lane kernel under a Gaussian prior (the matrix-core
    step tests a box only)."""
    from mcmc_amd import Context
    D = 16
    rng = np.random.default_rng(2)
    A = rng.normal(size=(D, D))
    cov = A @ A.T / D + np.eye(D)
    mu = rng.normal(size=D)
    lik, pri = T.fullcov_gauss(mu, cov), _prior(T, D, 2)
    x0 = rng.normal(mu[:, None], 1.0, size=(D, 96))
    g = run_gpu(lik, pri, T.gauss(0.3), x0, 4, nbin=2, nskip=1, n_rec=30)
    o = run_oracle(oracle, lik, pri, T.gauss(0.3), x0, 4, 2, 1, 30)
    assert_same(g, o)
    with Context(seed=4) as c:
        c.set_model(lik, pri, T.gauss(0.3))
        c.init(x0)
        c.run(nbin=1, nskip=1, n_rec=1)
        assert c.lanes() == 1


def test_mh_de_and_mixture_gauss_prior_bit_exact(oracle, T):
    D = 6
    rng = np.random.default_rng(5)
    mu, sg = rng.normal(size=D), rng.uniform(0.5, 1.5, D)
    lik, pri = T.diag_gauss(mu, sg), _prior(T, D, 3)
    x0 = rng.normal(mu[:, None], sg[:, None], size=(D, 100))
    samples = rng.normal(mu, sg, size=(64, D))
    de = T.differential_evolution_proposal(samples, 0.2)
    from mcmc_amd import Context
    ctx = Context(seed=3)
    ctx.set_model(lik, pri, de)
    ctx.init(x0)
    ctx.run(nbin=0, nskip=1, n_rec=40, record_x=True, record_llp=True, record_accept=True)
    rx, rll, rlp, bits = ctx.records(x=True, llp=True, accept=True)
    ctx.close()
    m = oracle.Model(D, lik.kind, lik.params, pri.kind, pri.params, 4,
                     np.concatenate([[0.2, len(samples)], samples.ravel()]))
    ll0 = np.array([m.loglik(x0[:, i]) for i in range(100)])
    lp0 = np.array([m.logprior(x0[:, i]) for i in range(100)])
    o = oracle.mh_run(m, 3, x0, ll0, lp0, nbin=0, nskip=1, n_rec=40, nthreads=8)
    np.testing.assert_array_equal(rx, o["rec_x"])
    np.testing.assert_array_equal(rlp, o["rec_lp"])
    np.testing.assert_array_equal(bits, o["bits"])
    mix = T.combine_jump_proposals([(0.7, T.gauss(0.3)), (0.3, T.shift_uniform(-0.2 * np.ones(D), 0.2 * np.ones(D)))], D)
    g = run_gpu(lik, pri, mix, x0, 8, nbin=1, nskip=1, n_rec=30)
    o = run_oracle(oracle, lik, pri, mix, x0, 8, 1, 1, 30)
    assert_same(g, o)


def test_mh_kd_gauss_prior_bit_exact(oracle, T):
    """The kD proposal on 4 lanes (two dims per lane, the C4 register path) under a Gaussian prior."""
    D = 8
    rng = np.random.default_rng(6)
    mu, sg = np.zeros(D), np.ones(D)
    pts = rng.normal(size=(2000, D))
    lo, hi = -5 * np.ones(D), 5 * np.ones(D)
    kd = T.KdInterp(pts, lo, hi)
    lik, pri = T.diag_gauss(mu, sg), _prior(T, D, 4)
    x0 = rng.normal(size=(D, 256))
    g = run_gpu(lik, pri, kd, x0, 2, nbin=2, nskip=1, n_rec=30, lanes=4)
    okd = oracle.KdTree(pts, lo, hi)
    o = run_oracle(oracle, lik, pri, kd, x0, 2, 2, 1, 30, kd=okd)
    assert_same(g, o)


@pytest.mark.parametrize("D,lik_name,k", [(3, "diag", 1), (3, "diag", 16), (16, "diag", 1), (16, "shell", 8),
                                          (32, "diag", 16), (9, "diag", 4)])
def test_nested_gauss_prior_bit_exact(oracle, T, D, lik_name, k):
    """Walkers on 1 (D 3, padded D 9), 4 (D 16) and 8 (D 32) lanes; prior draws of the live set
    by normals; the walkers' MH test under the Gaussian prior."""
    rng = np.random.default_rng(D + k)
    if lik_name == "diag":
        lik = T.diag_gauss(rng.uniform(-0.3, 0.3, D), rng.uniform(0.2, 0.5, D))
    else:
        lik = T.gauss_shell(np.zeros(D), 1.0, 0.2)
    pri = _prior(T, D, 5, scale=1.0)
    g = gpu_nested(lik, pri, 13, nlive=200, nmcmc=25, mode_hopping_frac=0.1, k=k, max_dead=40 * k)
    o = oracle_nested(oracle, lik, pri, 13, nlive=200, nmcmc=25, mode_hop=0.1, k=k, max_iter=40 * k)
    assert_nested_same(g, o)


@pytest.mark.parametrize("lik_name", ["diag", "shell"])
def test_nested_gauss_prior_large_k_eight_lanes_bit_exact(oracle, T, lik_name):
    """k 8,192 at D 16: the walkers' default 8-lane split (two dims per lane) beyond 4,096
    walkers, two walker waves per draw-table workgroup, under the Gaussian prior."""
    D, k = 16, 8192
    rng = np.random.default_rng(29)
    lik = (T.diag_gauss(rng.uniform(-0.3, 0.3, D), rng.uniform(0.2, 0.5, D)) if lik_name == "diag"
           else T.gauss_shell(np.zeros(D), 1.0, 0.2))
    pri = _prior(T, D, 5, scale=1.0)
    g = gpu_nested(lik, pri, 31, nlive=16384, nmcmc=6, mode_hopping_frac=0.1, k=k, max_dead=3 * k)
    o = oracle_nested(oracle, lik, pri, 31, nlive=16384, nmcmc=6, mode_hop=0.1, k=k, max_iter=3 * k)
    assert_nested_same(g, o)


def test_nested_gauss_prior_converged_bit_exact_and_analytic(oracle, T):
    """A converged run (the stop test fires) equal to the oracle, and log Z within 4 sigma of the
    analytic Gaussian x Gaussian evidence."""
    D = 4
    muL, sL = np.array([0.3, -0.2, 0.1, 0.4]), np.array([0.2, 0.3, 0.25, 0.4])
    muP, sP = np.array([0.0, 0.1, -0.1, 0.2]), np.array([1.0, 0.7, 1.2, 0.9])
    lik, pri = T.diag_gauss(muL, sL), T.gauss_prior(muP, sP)
    g = gpu_nested(lik, pri, 17, nlive=500, nmcmc=40, mode_hopping_frac=0.1, k=4)
    o = oracle_nested(oracle, lik, pri, 17, nlive=500, nmcmc=40, mode_hop=0.1, k=4)
    assert_nested_same(g, o)
    v = sL ** 2 + sP ** 2
    lz = float(np.sum(-0.5 * np.log(2 * math.pi * v) - 0.5 * (muL - muP) ** 2 / v))
    w = np.exp(g[3])
    H = float(np.sum(w * g.ll) - g[0])
    assert abs(g[0] - lz) < 4 * math.sqrt(H / 500)
