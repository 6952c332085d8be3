"""Any ndim (include/mcg.h "Any ndim"): an ndim without compiled kernels runs on the next compiled
width with zero-padded dims -- zero likelihood terms, zero proposal steps, unbounded box, prior
draws at 0 -- and the padding never crosses the C-ABI.  The reference is generic over the
parameter vector's length (mcmc.mli:58-72, nested.mli:50-61); these tests run widths 9, 10, 20
and 33 (padded to 12, 12, 24 and 48; full covariance to 16 and 32) bit-exact against the oracle,
which runs at the real ndim: the padded dims add +0 to the canonical sums and take no Philox
draws the real dims use (dims 4c..4c+3 draw from call c), so the real dims compute exactly as at
their own width."""
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


def diag_model(T, D, seed=3):
    rng = np.random.default_rng(seed + D)
    mu, sg = rng.uniform(-1, 1, D), rng.uniform(0.5, 2, D)
    return T.diag_gauss(mu, sg), mu, sg


@pytest.mark.parametrize("D", [9, 10, 20, 33])
@pytest.mark.parametrize("lanes", [0, 1])
def test_diag_mh_padded_widths_bit_exact(oracle, T, D, lanes):
    """DIAG_GAUSS with an isotropic step and a box prior (the C2 model) at widths with no
    compiled kernel, on the auto lane split and on one lane per chain: records, bitmap, state,
    counters and tiles equal the oracle's at the real width."""
    lik, mu, sg = diag_model(T, D)
    pri = T.box(-10 * np.ones(D), 10 * np.ones(D))
    prop = T.gauss(2.38 / math.sqrt(D) * float(np.median(sg)))
    x0 = np.random.default_rng(D).normal(mu[:, None], sg[:, None], size=(D, 160))
    g = run_gpu(lik, pri, prop, x0, 5, nbin=7, nskip=3, n_rec=40, lanes=lanes)
    o = run_oracle(oracle, lik, pri, prop, x0, 5, 7, 3, 40)
    assert_same(g, o)


@pytest.mark.parametrize("D", [10, 20])
def test_other_kinds_padded_bit_exact(oracle, T, D):
    """Shell, Gaussian mixture and per-dim proposal scales with an asymmetric box at padded
    widths: GPU == oracle bit for bit."""
    rng = np.random.default_rng(40 + D)
    x0 = rng.normal(size=(D, 96))
    shell = T.gauss_shell(np.zeros(D), 2.0, 0.3)
    xs = 2.0 * x0 / np.linalg.norm(x0, axis=0)
    for lik, prop, x in ((shell, T.gauss(0.05), xs),
                         (T.gauss_mix(rng.uniform(-1, 1, (3, D)), rng.uniform(0.5, 1.5, (3, D))), T.gauss(0.2), x0),
                         (diag_model(T, D)[0], T.gauss(np.linspace(0.1, 0.4, D)), x0)):
        pri = T.box(-4.0 - np.arange(D) / D, 4.5 * np.ones(D))
        g = run_gpu(lik, pri, prop, x, 7, nbin=3, nskip=1, n_rec=50)
        o = run_oracle(oracle, lik, pri, prop, x, 7, 3, 1, 50)
        assert_same(g, o)


@pytest.mark.parametrize("D", [10, 20])
def test_fullcov_padded_matrix_core_bit_exact(oracle, T, D):
    """Full covariance at D = 10 and 20 runs on the matrix-core kernel at width 16 / 32 with a
    zero-padded precision factor: GPU == oracle bit for bit."""
    from mcmc_amd import Context
    rng = np.random.default_rng(D)
    Q, _ = np.linalg.qr(rng.normal(size=(D, D)))
    cov = (Q * np.exp(rng.uniform(-1, 1, D))) @ Q.T
    mu = rng.uniform(-1, 1, D)
    lik = T.fullcov_gauss(mu, 0.5 * (cov + cov.T))
    pri = T.box(-8 * np.ones(D), 8 * np.ones(D))
    prop = T.gauss(0.3)
    x0 = rng.normal(mu[:, None], 1.0, size=(D, 256))
    g = run_gpu(lik, pri, prop, x0, 11, nbin=4, nskip=2, n_rec=30)
    o = run_oracle(oracle, lik, pri, prop, x0, 11, 4, 2, 30)
    assert_same(g, o)
    ctx = Context(seed=11)
    ctx.set_model(lik, pri, prop)
    ctx.init(x0)
    ctx.run(nbin=1, n_rec=0, record_x=False, record_llp=False)
    assert ctx.lanes() == 4                                  # the matrix-core kernel ran
    ctx.close()


def test_de_proposal_padded_bit_exact(oracle, T):
    """differential_evolution_proposal at D = 13 (samples padded with zero columns; the DE
    scale 2.38/sqrt(2 ndim) from the real ndim): GPU == oracle bit for bit."""
    D = 13
    lik, mu, sg = diag_model(T, D)
    rng = np.random.default_rng(2)
    samples = rng.normal(mu, sg, size=(300, D))
    pri = T.box(-10 * np.ones(D), 10 * np.ones(D))
    x0 = rng.normal(mu[:, None], sg[:, None], size=(D, 128))
    g = run_gpu(lik, pri, T.differential_evolution_proposal(samples, 0.25), x0, 3, nbin=2, nskip=1, n_rec=40)
    o = run_oracle(oracle, lik, pri, T.Proposal(4, np.concatenate([[0.25, 300], samples.ravel()])), x0, 3, 2, 1, 40)
    assert_same(g, o)


@pytest.mark.parametrize("D,k", [(9, 1), (10, 8), (20, 24), (33, 40)])
def test_nested_padded_widths_bit_exact(oracle, T, D, k):
    """The nested sampler at padded widths (shell for D = 9 / 33, DIAG for 10 / 20), run to its
    stop test: the dead points (rows stripped of the padding), stop generation, log Z and
    weights equal the oracle's at the real width; the observer sees the stripped rows."""
    from mcmc_amd import Context, nested
    if D in (9, 33):
        lik = T.gauss_shell(np.zeros(D), 1.0, 0.2)
    else:
        lik = diag_model(T, D)[0]
    pri = T.box(-2 * np.ones(D), 2 * np.ones(D))
    g = gpu_nested(lik, pri, 19, nlive=200, nmcmc=12, mode_hopping_frac=0.1, k=k)
    o = oracle_nested(oracle, lik, pri, 19, nlive=200, nmcmc=12, mode_hop=0.1, k=k)
    assert g.converged
    assert_nested_same(g, o)
    seen = []
    ctx = Context(seed=19)
    out = nested.nested_evidence(lik, pri, nlive=200, nmcmc=12, k=k, ctx=ctx, observer=lambda s: seen.append(s[0]))
    ctx.close()
    np.testing.assert_array_equal(np.array(seen), out[2][:out.n_dead])


def test_unpaddable_combinations_fail_loudly(T):
    """A kD proposal whose padded width has no kD kernel (round 6: kD pads to 12 / 16 on every
    kind, 24 / 32 on the lane-split ones), or ndim past the widest kernel, is refused with a
    message (MCG_EINVAL), not run wrong."""
    from mcmc_amd import Context
    from mcmc_amd._lib import InvalidArgument
    ctx = Context(seed=1)
    for D, lik in ((40, T.diag_gauss(np.zeros(40), np.ones(40))),
                   (20, T.gauss_mix(np.zeros((2, 20)), np.ones((2, 20))))):
        pts = np.random.default_rng(0).normal(size=(64, D))
        with pytest.raises(InvalidArgument, match="kD"):
            ctx.set_model(lik, T.flat_prior(), T.KdInterp(pts, -5 * np.ones(D), 5 * np.ones(D)))
    D = 65
    ctx.set_model(T.diag_gauss(np.zeros(D), np.ones(D)), T.flat_prior(), T.gauss(0.1))
    with pytest.raises(InvalidArgument, match="no compiled"):
        ctx.init(np.zeros((D, 8)))
        ctx.run(nbin=1, n_rec=0)
    ctx.close()


@pytest.mark.parametrize("D,lik_kind", [(9, "diag"), (13, "shell"), (20, "diag"), (30, "shell"), (10, "mix"),
                                        (11, "fullcov")])
@pytest.mark.parametrize("lanes", [0, 1])
def test_kd_proposal_padded_widths_bit_exact(oracle, T, D, lik_kind, lanes):
    """Round 6: the kD interpolated proposal (interpolate_pdf.ml:101-142) at an ndim without a kD
    kernel of its own runs zero-padded (widths 12, 16, 24, 32): the tree is the caller's D-dim
    tree, the device leaf boxes get [0, 0] in the pad dims, so the draws of the real dims (dims
    2c, 2c + 1 from call c), log q and every decision equal the oracle's at the real ndim.  (lanes
    1 at widths 24 / 32 has no kernel: the split is kept.)"""
    from mcmc_amd import Context
    rng = np.random.default_rng(70 + D)
    if lik_kind == "diag":
        lik = diag_model(T, D)[0]
    elif lik_kind == "shell":
        lik = T.gauss_shell(rng.uniform(-0.3, 0.3, D), 1.5, 0.4)
    elif lik_kind == "mix":
        lik = T.gauss_mix(rng.uniform(-1, 1, (2, D)), rng.uniform(0.5, 1.5, (2, D)))
    else:
        A = rng.normal(size=(D, D))
        lik = T.fullcov_gauss(rng.uniform(-1, 1, D), A @ A.T / D + np.eye(D))
    lo, hi = -3 * np.ones(D), 3 * np.ones(D)
    pts = np.clip(rng.normal(0.0, 1.0, size=(400, D)), -2.9, 2.9)
    kdp = T.KdInterp(pts, lo, hi)
    okd = oracle.KdTree(pts, lo, hi)
    pri = T.box(-4 * np.ones(D), 4 * np.ones(D))
    x0 = rng.uniform(-1.5, 1.5, size=(D, 200))
    g = run_gpu(lik, pri, kdp, x0, 19, nbin=4, nskip=2, n_rec=9, lanes=lanes if D <= 16 else 0)
    m = oracle.Model(D, lik.kind, lik.params, pri.kind, pri.params, 3, [0.0], okd)
    ll0 = np.array([m.loglik(x0[:, i]) for i in range(x0.shape[1])])
    lp0 = np.array([m.logprior(x0[:, i]) for i in range(x0.shape[1])])
    o = oracle.mh_run(m, 19, x0, ll0, lp0, nbin=4, nskip=2, n_rec=9, nthreads=8)
    o["ll0"], o["lp0"] = ll0, lp0
    o["tiles"] = oracle.tile_stats(D, x0.shape[1], 9, o)
    assert_same(g, o)
    if D > 16:
        with Context(seed=19) as ctx:
            ctx.set_model(lik, pri, kdp)
            ctx.init(x0)
            ctx.run(nbin=1, nskip=1, n_rec=1)
            assert ctx.lanes() >= D // 16
