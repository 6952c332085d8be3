"""GPU parity tests of the batched MH kernel against the CPU oracle (bit-exact), through the
C-ABI (mcmc_amd -> libmcg.so).  Every comparison is exact: accept bitmap, records, final
state, counters and tile statistics must be bit-identical to oracle/oracle.c on the same seed."""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LIK_FLAT, LIK_DIAG, LIK_FULLCOV, LIK_SHELL, LIK_GDATA, LIK_CDATA = range(6)


@pytest.fixture(scope="module")
def T():
    from mcmc_amd import targets
    return targets


def run_gpu(lik, prior, prop, x0, seed, nbin, nskip, n_rec, lanes=0, chain_offset=0, spl=0,
            accumulate=True):
    from mcmc_amd import Context
    ctx = Context(seed=seed, lanes_per_chain=lanes, chain_offset=chain_offset, steps_per_launch=spl)
    ctx.set_model(lik, prior, prop)
    ctx.init(x0)
    x_init, ll_init, lp_init = ctx.state()
    ctx.run(nbin=nbin, nskip=nskip, n_rec=n_rec, record_x=True, record_llp=True,
            record_accept=True, accumulate=accumulate)
    rx, rll, rlp, bits = ctx.records(x=True, llp=True, accept=True)
    x, ll, lp = ctx.state()
    acc, rej = ctx.counters()
    tiles = ctx.tile_stats() if accumulate else None
    out = dict(rec_x=rx, rec_ll=rll, rec_lp=rlp, bits=bits, x=x, ll=ll, lp=lp, nacc=acc,
               nrej=rej, tiles=tiles, ll0=ll_init, lp0=lp_init, lanes=None)
    ctx.close()
    return out


def run_oracle(O, lik, prior, prop, x0, seed, nbin, nskip, n_rec, chain_offset=0, kd=None):
    D = lik.ndim
    m = O.Model(D, lik.kind, lik.params, prior.kind, prior.params,
                prop.kind if kd is None else 3, prop.params if kd is None else [0.0], kd)
    N = x0.shape[1]
    ll0 = np.array([m.loglik(x0[:, i]) for i in range(N)])
    lp0 = np.array([m.logprior(x0[:, i]) for i in range(N)])
    r = O.mh_run(m, seed, x0, ll0, lp0, nbin=nbin, nskip=nskip, n_rec=n_rec, chain_offset=chain_offset,
                 nthreads=8)
    r["ll0"], r["lp0"] = ll0, lp0
    r["tiles"] = O.tile_stats(D, N, n_rec, r)
    return r


def assert_same(g, o):
    np.testing.assert_array_equal(g["ll0"], o["ll0"])
    np.testing.assert_array_equal(g["lp0"], o["lp0"])
    np.testing.assert_array_equal(g["bits"], o["bits"])
    np.testing.assert_array_equal(g["rec_x"], o["rec_x"])
    np.testing.assert_array_equal(g["rec_ll"], o["rec_ll"])
    np.testing.assert_array_equal(g["rec_lp"], o["rec_lp"])
    np.testing.assert_array_equal(g["x"], o["x"])
    np.testing.assert_array_equal(g["ll"], o["ll"])
    np.testing.assert_array_equal(g["lp"], o["lp"])
    assert g["nacc"] == int(o["nacc"].sum())
    # every step of every chain is counted once, accepted or rejected (mcmc.ml:27-35)
    assert g["nrej"] == o["x"].shape[1] * o["nsteps"] - int(o["nacc"].sum())
    if g["tiles"] is not None:
        np.testing.assert_array_equal(g["tiles"], o["tiles"])


def c2_model(T, D=32, seed=42):
    rng = np.random.default_rng(seed)
    mu = rng.uniform(-1, 1, D)
    sg = rng.uniform(0.5, 2, D)
    s = 2.38 / math.sqrt(D) * float(np.median(sg))
    return T.diag_gauss(mu, sg), T.box(-10 * np.ones(D), 10 * np.ones(D)), T.gauss(s), mu, sg


@pytest.mark.parametrize("lanes", [1, 2, 4, 8])
def test_c2_mini_bit_exact(oracle, T, lanes):
    """C2-mini: D=32 diagonal Gaussian, box prior, isotropic proposal, 192 chains, 300 steps."""
    lik, pri, prop, mu, sg = c2_model(T)
    N = 192
    x0 = np.random.default_rng(1).normal(mu[:, None], sg[:, None], size=(32, N))
    g = run_gpu(lik, pri, prop, x0, 1, nbin=20, nskip=1, n_rec=280, lanes=lanes)
    o = run_oracle(oracle, lik, pri, prop, x0, 1, 20, 1, 280)
    assert_same(g, o)


@pytest.mark.parametrize("lanes", [1, 4])
@pytest.mark.parametrize("case", ["per_dim", "flat", "open_box", "asym_box"])
def test_fused_step_constant_forms_bit_exact(oracle, T, lanes, case):
    """The fused step's constant forms: per-dim proposal scales / per-dim box bounds (loaded
    every step); one scale + one box [lo, hi] for all dims (kernel arguments, register-resident
    likelihood constants); and the symmetric box [-h, h] tested as |y| <= h -- with FLAT,
    OPEN_BOX and asymmetric priors, and chains started near the faces so the box rejects."""
    lik, pri, prop, mu, sg = c2_model(T)
    D, N = 32, 128
    if case == "per_dim":
        prop = T.gauss(0.3 * sg)
        pri = T.box(-3.0 - np.arange(D) / D, 3.0 + np.arange(D) / D)
    elif case == "flat":
        pri = T.flat_prior()
    elif case == "open_box":
        pri = T.box(-2.5 * np.ones(D), 2.5 * np.ones(D), open_=True)
    else:
        pri = T.box(-2.5 * np.ones(D), 2.45 * np.ones(D))
    x0 = np.clip(np.random.default_rng(6).normal(mu[:, None], sg[:, None], size=(D, N)), -2.4, 2.4)
    g = run_gpu(lik, pri, prop, x0, 9, nbin=5, nskip=1, n_rec=120, lanes=lanes)
    o = run_oracle(oracle, lik, pri, prop, x0, 9, 5, 1, 120)
    assert_same(g, o)


def test_multi_launch_and_thinning_equivalence(oracle, T):
    """Slicing the run into launches of 7 steps, with nbin/nskip thinning, changes nothing."""
    lik, pri, prop, mu, sg = c2_model(T, D=16)
    x0 = np.random.default_rng(2).normal(mu[:, None], sg[:, None], size=(16, 100))
    g = run_gpu(lik, pri, prop, x0, 3, nbin=13, nskip=5, n_rec=40, spl=7)
    o = run_oracle(oracle, lik, pri, prop, x0, 3, 13, 5, 40)
    assert_same(g, o)


@pytest.mark.parametrize("lanes", [1, 4])
def test_gauss_shell_bit_exact(oracle, T, lanes):
    D = 16
    lik = T.gauss_shell(np.zeros(D), 2.0, 0.1)
    pri = T.box(-6 * np.ones(D), 6 * np.ones(D))
    x0 = np.random.default_rng(4).normal(size=(D, 80))
    x0 = 2.0 * x0 / np.linalg.norm(x0, axis=0)
    g = run_gpu(lik, pri, T.gauss(0.03), x0, 5, nbin=0, nskip=2, n_rec=60, lanes=lanes)
    o = run_oracle(oracle, lik, pri, T.gauss(0.03), x0, 5, 0, 2, 60)
    assert_same(g, o)


@pytest.mark.parametrize("D", [1, 3, 5, 8])
def test_fullcov_bit_exact(oracle, T, D):
    rng = np.random.default_rng(D)
    A = rng.normal(size=(D, D))
    cov = A @ A.T + D * np.eye(D)
    mu = rng.normal(size=D)
    lik = T.fullcov_gauss(mu, cov)
    x0 = rng.normal(mu[:, None], 1.0, size=(D, 70))
    g = run_gpu(lik, T.flat_prior(), T.gauss(0.5), x0, 6, nbin=5, nskip=1, n_rec=50)
    o = run_oracle(oracle, lik, T.flat_prior(), T.gauss(0.5), x0, 6, 5, 1, 50)
    assert_same(g, o)


@pytest.mark.parametrize("D", [16, 32, 48, 64])
def test_fullcov_matrix_core_bit_exact(oracle, T, D):
    """C5 path: the MFMA full-covariance kernel (4 lanes per chain, mcg_fullcov_kernel.h) and the
    one-lane VALU kernel both reproduce the oracle bit for bit (100 chains: a partial wave)."""
    rng = np.random.default_rng(100 + D)
    Q, _ = np.linalg.qr(rng.normal(size=(D, D)))
    lam = np.exp(rng.uniform(math.log(0.1), math.log(10.0), D))
    cov = (Q * lam) @ Q.T
    cov = 0.5 * (cov + cov.T)
    mu = rng.uniform(-1, 1, D)
    lik = T.fullcov_gauss(mu, cov)
    pri = T.box(-30 * np.ones(D), 30 * np.ones(D))
    prop = T.gauss(2.38 / math.sqrt(D) * math.sqrt(lam.min()))
    x0 = mu[:, None] + np.linalg.cholesky(cov) @ rng.normal(size=(D, 100))
    o = run_oracle(oracle, lik, pri, prop, x0, 9, 3, 2, 40)
    for lanes in (4, 1):
        g = run_gpu(lik, pri, prop, x0, 9, nbin=3, nskip=2, n_rec=40, lanes=lanes)
        assert_same(g, o)


@pytest.mark.parametrize("cauchy", [False, True])
def test_gaussian_cauchy_c1_bit_exact(oracle, T, cauchy):
    """C1: bin/gaussian_cauchy.ml data likelihoods, wrapping-uniform proposal
    (dx = sigma / (sqrt nsamp * ndim), :118-129), box prior (:133-147)."""
    rng = np.random.default_rng(9)
    nd, nsamp = 1, 10
    mus = rng.uniform(-1, 1, nd); sigmas = rng.uniform(0.1, 0.2, nd)
    data = rng.normal(mus, sigmas, size=(nsamp, nd))
    lik = T.cauchy_data(data) if cauchy else T.gauss_data(data)
    lo = np.concatenate([[-1.0] * nd, [0.1] * nd]); hi = np.concatenate([[1.0] * nd, [0.2] * nd])
    lp_in = -nd * (math.log(2.0) + math.log(0.1))
    pri = T.box(lo, hi, lp_in)
    dx = np.concatenate([sigmas, sigmas]) / (math.sqrt(nsamp) * nd)
    prop = T.uniform_wrapping(lo, hi, dx)
    x0 = np.tile(np.concatenate([mus, sigmas])[:, None], (1, 64))
    g = run_gpu(lik, pri, prop, x0, 7, nbin=0, nskip=1, n_rec=500)
    o = run_oracle(oracle, lik, pri, prop, x0, 7, 0, 1, 500)
    assert_same(g, o)


def test_kd_interp_proposal_bit_exact(oracle, T):
    """C4-mini: Interpolate_pdf kD-tree independence proposal, D=3, 256 training points."""
    rng = np.random.default_rng(10)
    D = 3
    mu = np.zeros(D); sg = np.ones(D)
    pts = rng.normal(size=(256, D))
    lo, hi = -5 * np.ones(D), 5 * np.ones(D)
    kdp = T.KdInterp(pts, lo, hi)
    okd = oracle.KdTree(pts, lo, hi)
    lik = T.diag_gauss(mu, sg)
    pri = T.box(lo, hi)
    x0 = rng.normal(size=(D, 96))
    g = run_gpu(lik, pri, kdp, x0, 8, nbin=4, nskip=1, n_rec=64)
    o = run_oracle(oracle, lik, pri, T.gauss(1.0), x0, 8, 4, 1, 64, kd=okd)
    assert_same(g, o)


@pytest.mark.parametrize("D,lanes,uniform_box,nch", [(8, 1, True, 160), (8, 2, True, 160),
                                                      (8, 2, False, 100), (16, 2, False, 160),
                                                      (16, 4, True, 100), (8, 4, True, 160),
                                                      (8, 4, False, 100), (16, 8, True, 100),
                                                      (4, 2, False, 160)])
def test_kd_interp_lane_splits_bit_exact(oracle, T, D, lanes, uniform_box, nch):
    """The kD draw split over 1, 2, 4 or 8 lanes per chain (each lane its dims' box bounds and
    uniforms, the likelihood / prior constants staged in LDS) -- four-dim lane blocks, or two dims
    per lane (D = 2 lanes: the pair-chained canonical accumulator) -- with the box prior as kernel
    arguments or as per-dim bounds: the oracle's chains bit for bit."""
    rng = np.random.default_rng(11 + D)
    mu = np.linspace(-0.2, 0.2, D); sg = np.linspace(0.8, 1.2, D)
    pts = rng.normal(size=(512, D))
    lo = -5 * np.ones(D) if uniform_box else np.linspace(-5.5, -4.5, D)
    hi = 5 * np.ones(D) if uniform_box else np.linspace(4.5, 5.5, D)
    kdp = T.KdInterp(pts, lo, hi)
    okd = oracle.KdTree(pts, lo, hi)
    lik, pri = T.diag_gauss(mu, sg), T.box(lo, hi)
    x0 = rng.normal(size=(D, nch))       # 100 chains: a partial last wave
    g = run_gpu(lik, pri, kdp, x0, 9, nbin=3, nskip=2, n_rec=40, lanes=lanes)
    o = run_oracle(oracle, lik, pri, T.gauss(1.0), x0, 9, 3, 2, 40, kd=okd)
    assert_same(g, o)
    from mcmc_amd import Context
    ctx = Context(seed=9, lanes_per_chain=lanes)
    ctx.set_model(lik, pri, kdp)
    ctx.init(x0)
    ctx.run(nbin=1, n_rec=0, record_x=False, record_llp=False)
    assert ctx.lanes() == lanes
    ctx.close()


def test_kd_tree_export_matches_oracle(oracle, T):
    import ctypes as C
    import mcmc_amd._lib as L
    from mcmc_amd import Context
    rng = np.random.default_rng(11)
    pts = rng.normal(size=(300, 4))
    pts[:40] = pts[0]                      # duplicates -> multi-point leaf (kd_tree.ml:159-160)
    lo, hi = -6 * np.ones(4), 6 * np.ones(4)
    ctx = Context(seed=0)
    ctx.set_model(T.diag_gauss(np.zeros(4), np.ones(4)), T.box(lo, hi), T.KdInterp(pts, lo, hi))
    nn, nl = C.c_int64(), C.c_int64()
    L.check(L.lib().mcg_kd_info(ctx.ptr, C.byref(nn), C.byref(nl)))
    g = dict(dim=np.zeros(nn.value, np.int32), split=np.zeros(nn.value), right=np.zeros(nn.value, np.int32),
             leaf=np.zeros(nn.value, np.int32), count=np.zeros(nl.value, np.int32),
             box=np.zeros((nl.value, 2, 4)), logq=np.zeros(nl.value))
    L.check(L.lib().mcg_kd_export(ctx.ptr, L.i32ptr(g["dim"]), L.dptr(g["split"]), L.i32ptr(g["right"]),
                                  L.i32ptr(g["leaf"]), L.i32ptr(g["count"]), L.dptr(g["box"]),
                                  L.dptr(g["logq"])))
    e = oracle.KdTree(pts, lo, hi).export()
    for k in ("dim", "split", "right", "leaf", "count", "box"):
        np.testing.assert_array_equal(g[k], e[k], err_msg=k)


def test_sharded_chains_equal_single_context(oracle, T):
    """GPU-count invariance: two contexts holding chains [0,256) and [256,512) (chain_offset)
    reproduce one context holding all 512, and their tiles combine to identical statistics."""
    from mcmc_amd.context import combine_tiles
    lik, pri, prop, mu, sg = c2_model(T)
    x0 = np.random.default_rng(12).normal(mu[:, None], sg[:, None], size=(32, 512))
    full = run_gpu(lik, pri, prop, x0, 13, nbin=10, nskip=1, n_rec=100)
    a = run_gpu(lik, pri, prop, x0[:, :256], 13, nbin=10, nskip=1, n_rec=100, chain_offset=0)
    b = run_gpu(lik, pri, prop, x0[:, 256:], 13, nbin=10, nskip=1, n_rec=100, chain_offset=256)
    np.testing.assert_array_equal(full["x"], np.concatenate([a["x"], b["x"]], axis=1))
    np.testing.assert_array_equal(full["tiles"], np.concatenate([a["tiles"], b["tiles"]]))
    m1 = combine_tiles(32, full["tiles"])
    m2 = combine_tiles(32, np.concatenate([a["tiles"], b["tiles"]]))
    for u, v in zip(m1, m2):
        np.testing.assert_array_equal(u, v)


def test_append_runs_equal_one_run(oracle, T):
    """mcg_run(append) continues records/statistics: nbin run + 3 appended chunks == one run."""
    from mcmc_amd import Context
    lik, pri, prop, mu, sg = c2_model(T, D=8)
    x0 = np.random.default_rng(14).normal(mu[:, None], sg[:, None], size=(8, 300))
    ctx = Context(seed=15)
    ctx.set_model(lik, pri, prop)
    ctx.init(x0)
    ctx.run(nbin=10, nskip=1, n_rec=1, record_x=False, record_llp=False, accumulate=True)
    for _ in range(3):
        ctx.run(nbin=0, nskip=2, n_rec=5, record_x=False, record_llp=False, accumulate=True,
                append=True)
    tiles = ctx.tile_stats()
    x, _, _ = ctx.state()
    o = run_oracle(oracle, lik, pri, prop, x0, 15, 10, 2, 16)
    np.testing.assert_array_equal(x, o["x"])
    np.testing.assert_array_equal(tiles, o["tiles"])


# ---------------------------------------------------------------- statistics at full size
def test_c2_full_size_properties(T):
    """C2 at its full size (65,536 chains, D=32): posterior moments from the on-device
    accumulators match the target (size-independent properties), acceptance is sane."""
    from mcmc_amd import Context
    lik, pri, prop, mu, sg = c2_model(T)
    N = 65536
    x0 = np.random.default_rng(16).normal(mu[:, None], sg[:, None], size=(32, N))
    ctx = Context(seed=1)
    ctx.set_model(lik, pri, prop)
    ctx.init(x0)
    ctx.run(nbin=100, nskip=1, n_rec=200, record_x=False, record_llp=False, record_accept=True,
            accumulate=True)
    mean, sd, log_z = ctx.stats()
    acc, rej = ctx.counters()
    frac = acc / (acc + rej)
    assert 0.15 < frac < 0.45
    np.testing.assert_allclose(mean, mu, atol=0.02)
    np.testing.assert_allclose(sd, sg, rtol=0.02)
    assert np.isfinite(log_z)


@pytest.mark.parametrize("D", [1, 3, 16])
def test_mixture_bit_exact(oracle, T, D):
    """Mcmc.combine_jump_proposals (mcmc.ml:165-185): Gaussian, shift-uniform (density and
    constant-zero log_jump_prob) and wrapping-uniform components; GPU == oracle bit for bit."""
    rng = np.random.default_rng(40 + D)
    mu, sg = rng.uniform(-1, 1, D), rng.uniform(0.5, 2, D)
    lik, pri = T.diag_gauss(mu, sg), T.box(-8 * np.ones(D), 8 * np.ones(D))
    mix = T.combine_jump_proposals([
        (0.4, T.gauss(0.7 * sg)),
        (1.0, T.shift_uniform(-0.5 * sg, 0.2 * sg)),
        (0.6, T.shift_uniform(-sg, sg), 0),
        (0.5, T.uniform_wrapping(-8 * np.ones(D), 8 * np.ones(D), sg))], D)
    x0 = mu[:, None] + sg[:, None] * rng.normal(size=(D, 200))
    o = run_oracle(oracle, lik, pri, mix, x0, 13, 4, 2, 30)
    g = run_gpu(lik, pri, mix, x0, 13, nbin=4, nskip=2, n_rec=30)
    assert_same(g, o)


@pytest.mark.parametrize("D", [2, 5])
def test_mixture_with_kd_component_bit_exact(oracle, T, D):
    """kD interpolated jump (Interpolate_pdf) mixed with a local Gaussian jump."""
    rng = np.random.default_rng(60 + D)
    pts = rng.normal(size=(300, D))
    lo, hi = -6 * np.ones(D), 6 * np.ones(D)
    lik, pri = T.diag_gauss(np.zeros(D), np.ones(D)), T.box(lo, hi)
    kdp = T.KdInterp(pts, lo, hi)
    mix = T.combine_jump_proposals([(0.7, kdp), (0.3, T.gauss(0.4))], D)
    x0 = rng.normal(size=(D, 150))
    kd = oracle.KdTree(pts, lo, hi)
    m = oracle.Model(D, lik.kind, lik.params, pri.kind, pri.params, mix.kind, mix.params, kd)
    ll0 = np.array([m.loglik(x0[:, i]) for i in range(x0.shape[1])])
    lp0 = np.array([m.logprior(x0[:, i]) for i in range(x0.shape[1])])
    o = oracle.mh_run(m, 21, x0, ll0, lp0, nbin=3, nskip=1, n_rec=40, nthreads=8)
    o["ll0"], o["lp0"] = ll0, lp0
    o["tiles"] = oracle.tile_stats(D, x0.shape[1], 40, o)
    g = run_gpu(lik, pri, mix, x0, 21, nbin=3, nskip=1, n_rec=40)
    assert_same(g, o)


def test_wrap_uniform_far_steps_bit_exact(oracle, T):
    """Mcmc.uniform_wrapping (mcmc.ml:187-196) with dx = 200 box widths (~100 reflections per
    proposal, beyond the old 64-reflection cap) and with dx = 1e5 widths (past the exact-loop
    bound: the closed-form fold): GPU == oracle bit for bit and every recorded point in the box."""
    D = 4
    lo, hi = -np.ones(D), np.ones(D)
    lik = T.diag_gauss(np.zeros(D), 0.5 * np.ones(D))
    pri = T.box(lo, hi, -D * math.log(2.0))
    x0 = np.random.default_rng(21).uniform(-1, 1, size=(D, 320))
    for widths in (200.0, 1e5):
        prop = T.uniform_wrapping(lo, hi, widths * (hi - lo))
        g = run_gpu(lik, pri, prop, x0, 23, nbin=2, nskip=1, n_rec=60)
        o = run_oracle(oracle, lik, pri, prop, x0, 23, 2, 1, 60)
        assert_same(g, o)
        assert np.all(g["rec_x"] >= -1.0) and np.all(g["rec_x"] <= 1.0)
        assert 0 < g["nacc"] < g["nacc"] + g["nrej"]


@pytest.mark.parametrize("mode_hop", [0.0, 0.3])
@pytest.mark.parametrize("lik_name", ["diag", "fullcov"])
def test_differential_evolution_proposal_bit_exact(oracle, T, mode_hop, lik_name):
    """Mcmc.differential_evolution_proposal (mcmc.ml:198-218) as the MH jump over a 500-sample
    array: GPU == oracle bit for bit (records, bitmap, state, counters, tiles); mode hopping 0
    (the scale draw never consulted) and 0.3."""
    rng = np.random.default_rng(31)
    D = 4
    mu, sg = rng.uniform(-1, 1, D), rng.uniform(0.5, 1.5, D)
    if lik_name == "diag":
        lik = T.diag_gauss(mu, sg)
    else:
        lik = T.fullcov_gauss(mu, np.diag(sg ** 2) + 0.1)
    pri = T.box(-10 * np.ones(D), 10 * np.ones(D), -D * math.log(20.0))
    samples = rng.normal(mu, sg, size=(500, D))
    de = T.differential_evolution_proposal(samples, mode_hop)
    x0 = rng.normal(mu[:, None], sg[:, None], size=(D, 200))
    g = run_gpu(lik, pri, de, x0, 41, nbin=3, nskip=2, n_rec=50)
    de_params = np.concatenate([[mode_hop, 500], samples.ravel()])
    o = run_oracle(oracle, lik, pri, T.Proposal(4, de_params), x0, 41, 3, 2, 50)
    assert_same(g, o)
    assert 0 < g["nacc"] < g["nacc"] + g["nrej"]


def test_differential_evolution_proposal_reference_width(T):
    """test/mcmc_test.ml:213-224 on the GPU: 1e6 samples ~ N(10, 1), mode_hopping_frac 1.0,
    proposals from [0] have mean 0 and sd sqrt 2 within 5e-3 (flat target: every proposal of
    one MH step of 1e6 chains is accepted, so the state is 1e6 independent proposals)."""
    from mcmc_amd import Context
    n = 1_000_000
    samples = np.random.default_rng(1).normal(10.0, 1.0, size=(n, 1))
    ctx = Context(seed=3)
    ctx.set_model(T.flat(1), T.flat_prior(), T.differential_evolution_proposal(samples, 1.0))
    ctx.init(np.zeros((1, n)), np.zeros(n), np.zeros(n))
    ctx.run(nbin=1, n_rec=0, record_x=False, record_llp=False)
    z = ctx.state()[0][0]
    assert ctx.counters() == (n, 0)
    assert abs(z.mean()) < 5e-3
    assert abs(z.std(ddof=1) - math.sqrt(2.0)) < 5e-3
    ctx.close()


def _c5_target(T, D=64, seed=5):
    rng = np.random.default_rng(seed)
    Q, _ = np.linalg.qr(rng.normal(size=(D, D)))
    lam = np.exp(rng.uniform(math.log(0.1), math.log(10.0), D))
    cov = (Q * lam) @ Q.T
    cov = 0.5 * (cov + cov.T)
    mu = rng.uniform(-1, 1, D)
    s = 2.38 / math.sqrt(D) * math.sqrt(lam.min())
    return T.fullcov_gauss(mu, cov), mu, cov, s


def _assert_shards_equal_full(full, parts):
    cat = lambda k, ax: np.concatenate([p[k] for p in parts], axis=ax)
    np.testing.assert_array_equal(full["x"], cat("x", 1))
    np.testing.assert_array_equal(full["ll"], cat("ll", 0))
    np.testing.assert_array_equal(full["lp"], cat("lp", 0))
    np.testing.assert_array_equal(full["rec_x"], cat("rec_x", 2))
    np.testing.assert_array_equal(full["rec_ll"], cat("rec_ll", 1))
    # accept bitmap rows: chain c of shard r is chain r*N + c of the full run (N % 64 == 0)
    np.testing.assert_array_equal(full["bits"], cat("bits", 1))
    np.testing.assert_array_equal(full["tiles"], cat("tiles", 0))
    assert full["nacc"] == sum(p["nacc"] for p in parts)


def test_sharded_fullcov_matrix_core_equals_single_context(T):
    """C5's sharding (BASELINE configs[4]) on the matrix-core kernel
    (mh_fullcov_kernel<64>, 4 lanes per chain): two contexts at chain_offset 0 and 256 reproduce
    one 512-chain context bit for bit -- state, records, accept bitmap, tiles -- and the tiles
    combine to identical moments / harmonic-mean evidence."""
    from mcmc_amd.context import combine_tiles
    lik, mu, cov, s = _c5_target(T)
    pri, prop = T.flat_prior(), T.gauss(s)
    x0 = mu[:, None] + np.linalg.cholesky(cov) @ np.random.default_rng(6).normal(size=(64, 512))
    full = run_gpu(lik, pri, prop, x0, 19, nbin=7, nskip=1, n_rec=40)
    a = run_gpu(lik, pri, prop, x0[:, :256], 19, nbin=7, nskip=1, n_rec=40, chain_offset=0)
    b = run_gpu(lik, pri, prop, x0[:, 256:], 19, nbin=7, nskip=1, n_rec=40, chain_offset=256)
    _assert_shards_equal_full(full, [a, b])
    for u, v in zip(combine_tiles(64, full["tiles"]), combine_tiles(64, np.concatenate([a["tiles"], b["tiles"]]))):
        np.testing.assert_array_equal(u, v)


def test_sharded_kd_interp_equals_single_context(T):
    """C4's kD independence proposal (lanes split per chain) sharded over two contexts at
    chain_offset 0 and 256 equals one 512-chain context bit for bit (shards are whole 256-chain
    tiles, as the multi-GPU runs use)."""
    rng = np.random.default_rng(22)
    D = 8
    pts = rng.normal(size=(4096, D))
    lo, hi = -10 * np.ones(D), 10 * np.ones(D)
    lik, pri, kdp = T.diag_gauss(np.zeros(D), np.ones(D)), T.box(lo, hi), T.KdInterp(pts, lo, hi)
    x0 = rng.normal(size=(D, 512))
    full = run_gpu(lik, pri, kdp, x0, 29, nbin=5, nskip=1, n_rec=30)
    a = run_gpu(lik, pri, kdp, x0[:, :256], 29, nbin=5, nskip=1, n_rec=30, chain_offset=0)
    b = run_gpu(lik, pri, kdp, x0[:, 256:], 29, nbin=5, nskip=1, n_rec=30, chain_offset=256)
    _assert_shards_equal_full(full, [a, b])


@pytest.mark.parametrize("lanes,lik_kind,prior_kind,nbin,nskip,spl", [
    (4, "diag", "box", 3, 1, 0),          # the C4 shape: groups of 4 steps and a 3-step tail
    (4, "shell", "open", 5, 3, 7),        # launches of 7 steps: every group offset, tails in each
    (2, "diag", "flat", 6, 2, 0),         # four dims a lane (P = 2: two group steps per stagger)
    (2, "flat", "box", 1, 1, 5),
    (4, "diag", "gauss", 2, 5, 9),
])
def test_kd_grouped_step_bit_exact(oracle, T, lanes, lik_kind, prior_kind, nbin, nskip, spl):
    """Round 6: the kD proposal on P > 1 lanes evaluates four steps' proposals together, then
    accepts them in order (mh_kernel kd_group).  Step counts that leave tails, launches split at
    every offset (steps_per_launch), records every 1 / 2 / 3 / 5 steps, each likelihood and prior
    kind of the register path: records, bitmap, state, counters and tiles equal the oracle's."""
    D = 8
    rng = np.random.default_rng(90 + lanes + nbin)
    pts = rng.normal(size=(1500, D))
    lo, hi = -4.0 * np.ones(D), 4.0 * np.ones(D)
    kd, okd = T.KdInterp(pts, lo, hi), oracle.KdTree(pts, lo, hi)
    if lik_kind == "diag":
        lik = T.diag_gauss(rng.uniform(-0.5, 0.5, D), rng.uniform(0.7, 1.5, D))
    elif lik_kind == "shell":
        lik = T.gauss_shell(np.zeros(D), 1.5, 0.5)
    else:
        lik = T.flat(D)
    if prior_kind == "box":
        pri = T.box(-3.5 * np.ones(D), 3.5 * np.ones(D))
    elif prior_kind == "open":
        pri = T.box(-3.0 * np.ones(D), 3.2 * np.ones(D), open_=True)
    elif prior_kind == "gauss":
        pri = T.gauss_prior(np.zeros(D), 2.0 * np.ones(D))
    else:
        pri = T.flat_prior()
    x0 = rng.uniform(-1.0, 1.0, size=(D, 320))
    g = run_gpu(lik, pri, kd, x0, 5, nbin=nbin, nskip=nskip, n_rec=23, lanes=lanes, spl=spl)
    o = run_oracle(oracle, lik, pri, kd, x0, 5, nbin, nskip, 23, kd=okd)
    assert_same(g, o)


@pytest.mark.parametrize("lanes,prior_kind,nbin,spl,appends", [
    (4, "box", 0, 0, 2),       # the C4 shape: record 0 is the start state, so records run one off
    (4, "gauss", 3, 7, 1),     # burn-in, then groups at every offset in launches of 7 steps
    (2, "box", 2, 0, 3),       # four dims a lane
])
def test_kd_grouped_records_bit_exact(oracle, T, lanes, prior_kind, nbin, spl, appends):
    """Round 6: when every step of a kD group records only into the moments and harmonic-mean
    partials (no recorded rows -- the C4 bench's shape), the group runs its accepts first, then
    its records.  Moments / harmonic-mean tiles, accept bitmap, state and counters equal the
    oracle's over appended runs (record indices offset against the groups)."""
    from mcmc_amd import Context
    D, N = 8, 320
    rng = np.random.default_rng(7 + lanes + nbin)
    pts = rng.normal(size=(1200, D))
    lo, hi = -4.0 * np.ones(D), 4.0 * np.ones(D)
    kd, okd = T.KdInterp(pts, lo, hi), oracle.KdTree(pts, lo, hi)
    lik = T.diag_gauss(rng.uniform(-0.5, 0.5, D), rng.uniform(0.7, 1.5, D))
    pri = T.box(-3.5 * np.ones(D), 3.5 * np.ones(D)) if prior_kind == "box" else \
        T.gauss_prior(np.zeros(D), 2.0 * np.ones(D))
    x0 = rng.uniform(-1.0, 1.0, size=(D, N))
    n_rec = 21
    ctx = Context(seed=9, lanes_per_chain=lanes, steps_per_launch=spl)
    ctx.set_model(lik, pri, kd)
    ctx.init(x0)
    ctx.run(nbin=nbin, nskip=1, n_rec=n_rec, record_x=False, record_llp=False, record_accept=True,
            accumulate=True)
    bits = [ctx.records(x=False, llp=False, accept=True)[3]]
    for _ in range(appends - 1):
        ctx.run(nbin=0, nskip=1, n_rec=n_rec, record_x=False, record_llp=False, record_accept=True,
                accumulate=True, append=True)
        bits.append(ctx.records(x=False, llp=False, accept=True)[3])
    x, ll, lp = ctx.state()
    acc, rej = ctx.counters()
    tiles = ctx.tile_stats()
    ctx.close()
    # the oracle: one run of the same total steps (appended runs continue the record count)
    m = oracle.Model(D, lik.kind, lik.params, pri.kind, pri.params, 3, [0.0], okd)
    ll0 = np.array([m.loglik(x0[:, i]) for i in range(N)])
    lp0 = np.array([m.logprior(x0[:, i]) for i in range(N)])
    total = n_rec * appends
    o = oracle.mh_run(m, 9, x0, ll0, lp0, nbin=nbin, nskip=1, n_rec=total, record_x=False, record_llp=False,
                      nthreads=8)
    np.testing.assert_array_equal(x, o["x"])
    np.testing.assert_array_equal(ll, o["ll"])
    np.testing.assert_array_equal(lp, o["lp"])
    assert acc == int(o["nacc"].sum())
    np.testing.assert_array_equal(np.concatenate(bits, axis=0), o["bits"])
    np.testing.assert_array_equal(tiles, oracle.tile_stats(D, N, total, o))
