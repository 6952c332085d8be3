"""GPU tests of the Gaussian-mixture likelihood (MCG_LIK_GAUSS_MIX): the multimodal target of
test/nested_test.ml:41-64 -- four Gaussians (sigma 0.05) on the open unit square, ll = log of the
sum of the four component densities (nested_test.ml:52-57) -- bit-exact against the oracle in MH
and in nested sampling (k = 1 and k > 1), and the reference's own check (Z = 4 within 2 err,
err < 0.5) on an ensemble of GPU runs at the reference's defaults."""
import math

import numpy as np
import pytest

from test_gpu_mh import assert_same, run_gpu, run_oracle
from test_gpu_nested import assert_nested_same, gpu_nested, oracle_nested

pytestmark = [pytest.mark.gpu, pytest.mark.filterwarnings("ignore:nested_evidence. max_dead")]

MUS = np.array([[0.25, 0.25], [0.25, 0.75], [0.75, 0.25], [0.75, 0.75]])   # nested_test.ml:42-45
SIGMA = np.array([0.05, 0.05])                                              # nested_test.ml:46


@pytest.fixture(scope="module")
def T():
    from mcmc_amd import targets
    return targets


def four_gaussians(T):
    return T.gauss_mix(MUS, SIGMA), T.box([0, 0], [1, 1], 0.0, open_=True)


@pytest.mark.parametrize("case", ["four", "random5", "one"])
def test_gauss_mix_mh_bit_exact(oracle, T, case):
    """MH over the mixture (Gaussian random walk): records, bitmap, state, counters and tiles
    equal the oracle's bit for bit -- the four-Gaussian target, a random 3-component mixture at
    D = 5, and a one-component mixture (which is DIAG_GAUSS bit for bit)."""
    rng = np.random.default_rng(12)
    if case == "four":
        lik, pri = four_gaussians(T)
        D, s = 2, 0.04
        x0 = MUS[rng.integers(0, 4, 300)].T + rng.normal(0, 0.05, (2, 300))
    elif case == "random5":
        D, s = 5, 0.3
        lik = T.gauss_mix(rng.uniform(-2, 2, (3, D)), rng.uniform(0.3, 1.0, (3, D)))
        pri = T.box(-5 * np.ones(D), 5 * np.ones(D))
        x0 = rng.normal(0, 1.5, (D, 300))
    else:
        D, s = 7, 0.5
        mu, sg = rng.uniform(-1, 1, D), rng.uniform(0.5, 1.5, D)
        lik = T.gauss_mix(mu[None], sg[None])
        pri = T.box(-6 * np.ones(D), 6 * np.ones(D))
        x0 = rng.normal(mu[:, None], sg[:, None], (D, 300))
    x0 = np.ascontiguousarray(np.clip(x0, 0.01, 0.99) if case == "four" else x0)
    g = run_gpu(lik, pri, T.gauss(s), x0, 17, nbin=10, nskip=2, n_rec=60)
    o = run_oracle(oracle, lik, pri, T.gauss(s), x0, 17, 10, 2, 60)
    assert_same(g, o)
    assert 0 < g["nacc"] < g["nacc"] + g["nrej"]
    if case == "one":
        d = run_gpu(T.diag_gauss(lik.params[1:1 + D], lik.params[1 + D:]), pri, T.gauss(s), x0, 17,
                    nbin=10, nskip=2, n_rec=60)
        for key in ("ll0", "bits", "rec_x", "rec_ll", "x", "ll", "tiles"):
            np.testing.assert_array_equal(g[key], d[key])
        assert g["nacc"] == d["nacc"]


def test_gauss_mix_de_proposal_bit_exact(oracle, T):
    """The mixture with Mcmc.differential_evolution_proposal over samples of all four modes and
    mode hopping 0.2 (d = 1 jumps carry chains between modes): GPU == oracle bit for bit."""
    rng = np.random.default_rng(8)
    lik, pri = four_gaussians(T)
    samples = MUS[rng.integers(0, 4, 400)] + rng.normal(0, 0.05, (400, 2))
    de = T.differential_evolution_proposal(samples, 0.2)
    x0 = np.ascontiguousarray(np.clip(MUS[rng.integers(0, 4, 256)].T + rng.normal(0, 0.05, (2, 256)), 0.01, 0.99))
    g = run_gpu(lik, pri, de, x0, 23, nbin=5, nskip=1, n_rec=80)
    o = run_oracle(oracle, lik, pri, T.Proposal(4, np.concatenate([[0.2, 400], samples.ravel()])), x0, 23, 5, 1, 80)
    assert_same(g, o)


@pytest.mark.parametrize("nlive,k,nmcmc", [(300, 1, 20), (1000, 16, 50)])
def test_four_gaussians_nested_bit_exact(oracle, T, nlive, k, nmcmc):
    """nested_test.ml:41-64's target through the GPU nested sampler, run to its own stop test:
    every dead point, the stop generation, log Z, log dZ and the weights equal the oracle's (k = 1
    is the reference algorithm; k = 16 the batched retirement)."""
    lik, pri = four_gaussians(T)
    g = gpu_nested(lik, pri, 29, nlive=nlive, nmcmc=nmcmc, mode_hopping_frac=0.1, k=k)
    o = oracle_nested(oracle, lik, pri, 29, nlive=nlive, nmcmc=nmcmc, mode_hop=0.1, k=k)
    assert g.converged
    assert_nested_same(g, o)


def test_nested_four_gaussians_reference_test(T):
    """test/nested_test.ml:41-64 on the GPU at the reference's defaults (nlive 1000, nmcmc 1000,
    mode_hopping_frac 0.1, epsrel 0.01, k = 1): Z = 4 within 2 err, err < 0.5.  Ensemble of 8
    consecutive seeds (61-68, no selection): every run within 4 err with err < 0.5, at least 6
    of 8 within 2 err, the mean of (Z - 4)/err within 3 standard errors (sd 1.4) of 0, and each
    run's posterior mass about equal over the four modes (the mode hops work)."""
    from mcmc_amd import nested
    lik, pri = four_gaussians(T)
    zs = []
    for seed in range(61, 69):
        out = gpu_nested(lik, pri, seed, nlive=1000, nmcmc=1000, mode_hopping_frac=0.1, k=1)
        log_ev, log_dev, pts, w = out
        ev = math.exp(log_ev)
        err = math.exp(nested.log_total_error_estimate(log_ev, log_dev, 1000))
        assert out.converged and err < 0.5
        assert abs(ev - 4.0) < 4 * err, (seed, ev, err)
        zs.append((ev - 4.0) / err)
        ww = np.exp(w)
        assert abs(ww.sum() - 1.0) < 1e-8
        q = (pts[:, 0] > 0.5).astype(int) * 2 + (pts[:, 1] > 0.5).astype(int)
        mass = np.array([ww[q == j].sum() for j in range(4)])
        assert np.all(np.abs(mass - 0.25) < 0.08), (seed, mass)
    zs = np.array(zs)
    print("four Gaussians, 8 GPU runs: (Z - 4)/err =", np.round(zs, 2))
    assert np.sum(np.abs(zs) < 2) >= 6, zs
    assert abs(zs.mean()) < 3 * 1.4 / math.sqrt(len(zs)), zs
