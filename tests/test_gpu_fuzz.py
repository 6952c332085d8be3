"""Randomised GPU parity sweep (round 5): MH on seeded random combinations of dimension (compiled
widths and zero-padded ones), likelihood kind, prior kind, proposal, lanes per chain, chain count
(full and partial waves / tiles) and record schedule, each compared bit for bit with the oracle
(accept bitmap, records, final state, counters, tile statistics) -- the combinations the targeted
tests do not enumerate.  Nested sampling gets the same treatment over dimension, likelihood,
prior, k and walk length."""
import math

import numpy as np
import pytest

from test_gpu_mh import assert_same, run_gpu, run_oracle

pytestmark = [pytest.mark.gpu, pytest.mark.filterwarnings("ignore:nested_evidence. max_dead")]

DIMS = [1, 2, 3, 4, 5, 7, 8, 9, 12, 13, 16, 17, 24, 31, 32, 33, 40, 48, 64]


@pytest.fixture(scope="module")
def T():
    from mcmc_amd import targets
    return targets


def _likelihood(T, rng, kind, D):
    if kind == "diag":
        return T.diag_gauss(rng.uniform(-1, 1, D), rng.uniform(0.3, 2.0, D))
    if kind == "shell":
        return T.gauss_shell(rng.uniform(-0.5, 0.5, D), rng.uniform(0.5, 2.0), rng.uniform(0.1, 0.5))
    if kind == "fullcov":
        A = rng.normal(size=(D, D))
        cov = A @ A.T / D + np.diag(rng.uniform(0.2, 1.0, D))
        return T.fullcov_gauss(rng.uniform(-1, 1, D), cov)
    m = int(rng.integers(1, 4))
    return T.gauss_mix(rng.uniform(-2, 2, (m, D)), rng.uniform(0.3, 1.5, (m, D)))


def _prior(T, rng, kind, D):
    if kind == "flat":
        return T.flat_prior()
    if kind == "box":
        return T.box(-4 * np.ones(D), 4 * np.ones(D))
    if kind == "asym_box":
        return T.box(-rng.uniform(2, 5, D), rng.uniform(2, 5, D))
    if kind == "open_box":
        return T.box(-3 * np.ones(D), 3 * np.ones(D), open_=True)
    return T.gauss_prior(rng.uniform(-0.5, 0.5, D), rng.uniform(1.0, 3.0, D))


def _mh_case(i):
    rng = np.random.default_rng(1000 + i)
    D = int(rng.choice(DIMS))
    lik = str(rng.choice(["diag", "shell", "fullcov", "mix"]))
    pri = str(rng.choice(["flat", "box", "asym_box", "open_box", "gauss"]))
    prop = str(rng.choice(["gauss", "gauss", "wrap", "mix", "kd", "mixkd"]))
    if prop in ("kd", "mixkd"):
        D = int(rng.choice([1, 2, 3, 4, 5, 6, 7, 8, 16]))      # kD: compiled widths, unpadded
    lanes = int(rng.choice([0, 0, 1, 2, 4, 8]))
    N = int(rng.choice([1, 63, 64, 200, 256, 257, 700]))
    nbin, nskip, n_rec = int(rng.integers(0, 12)), int(rng.integers(1, 4)), int(rng.integers(1, 9))
    return dict(i=i, D=D, lik=lik, pri=pri, prop=prop, lanes=lanes, N=N, nbin=nbin, nskip=nskip, n_rec=n_rec)


MH_CASES = [_mh_case(i) for i in range(64)]


@pytest.mark.parametrize("case", MH_CASES, ids=lambda c: "%(i)d-D%(D)d-%(lik)s-%(pri)s-%(prop)s-p%(lanes)d-n%(N)d" % c)
def test_mh_random_combinations_bit_exact(oracle, T, case):
    rng = np.random.default_rng(5000 + case["i"])
    D = case["D"]
    lik = _likelihood(T, rng, case["lik"], D)
    pri = _prior(T, rng, case["pri"], D)
    step = 2.38 / math.sqrt(D) * rng.uniform(0.3, 1.2)
    wrap = T.uniform_wrapping(-3 * np.ones(D), 3 * np.ones(D), rng.uniform(0.2, 1.0, D))
    okd = None
    if case["prop"] in ("kd", "mixkd"):
        # Interpolate_pdf over a training sample inside [-3, 3]^D (the proposal's support)
        lo, hi = -3 * np.ones(D), 3 * np.ones(D)
        pts = np.clip(rng.normal(0.0, 1.0, size=(int(rng.integers(20, 300)), D)), -2.9, 2.9)
        kdp = T.KdInterp(pts, lo, hi)
        okd = oracle.KdTree(pts, lo, hi)
    if case["prop"] == "wrap":
        prop = wrap
    elif case["prop"] == "mix":
        prop = T.combine_jump_proposals([(0.5, T.gauss(step)), (0.3, T.shift_uniform(-0.3 * np.ones(D), 0.2 * np.ones(D))),
                                         (0.2, wrap)], D)
    elif case["prop"] == "kd":
        prop = kdp
    elif case["prop"] == "mixkd":
        prop = T.combine_jump_proposals([(0.6, kdp), (0.4, T.gauss(step))], D)
    else:
        prop = T.gauss(step)
    # starts inside every prior's support (the wrapping proposal's range is [-3, 3])
    x0 = rng.uniform(-1.5, 1.5, size=(D, case["N"]))
    seed = int(rng.integers(1, 2**31))
    g = run_gpu(lik, pri, prop, x0, seed, case["nbin"], case["nskip"], case["n_rec"], lanes=case["lanes"])
    if case["prop"] in ("kd", "mixkd"):
        m = oracle.Model(D, lik.kind, lik.params, pri.kind, pri.params, prop.kind if case["prop"] == "mixkd" else 3,
                         prop.params if case["prop"] == "mixkd" else [0.0], okd)
        N = x0.shape[1]
        ll0 = np.array([m.loglik(x0[:, i]) for i in range(N)])
        lp0 = np.array([m.logprior(x0[:, i]) for i in range(N)])
        o = oracle.mh_run(m, seed, x0, ll0, lp0, nbin=case["nbin"], nskip=case["nskip"], n_rec=case["n_rec"], nthreads=8)
        o["ll0"], o["lp0"] = ll0, lp0
        o["tiles"] = oracle.tile_stats(D, N, case["n_rec"], o)
    else:
        o = run_oracle(oracle, lik, pri, prop, x0, seed, case["nbin"], case["nskip"], case["n_rec"])
    assert_same(g, o)


@pytest.mark.parametrize("D", [24, 48, 64])
@pytest.mark.parametrize("lik_kind", ["diag", "shell", "fullcov", "mix"])
@pytest.mark.parametrize("prop_kind", ["wrap", "mix"])
def test_wide_one_lane_proposals_bit_exact(oracle, T, D, lik_kind, prop_kind):
    """The wrapping-uniform and mixture proposals at the widest one-lane widths (their kernels
    spill ~1.5 KB a lane): every likelihood kind, bit for bit."""
    rng = np.random.default_rng(D * 7 + len(lik_kind) + len(prop_kind))
    lik = _likelihood(T, rng, lik_kind, D)
    pri = _prior(T, rng, "asym_box", D)
    wrap = T.uniform_wrapping(-3 * np.ones(D), 3 * np.ones(D), rng.uniform(0.05, 0.3, D))
    if prop_kind == "wrap":
        prop = wrap
    else:
        prop = T.combine_jump_proposals([(0.5, T.gauss(0.1)), (0.3, T.shift_uniform(-0.05 * np.ones(D), 0.04 * np.ones(D))),
                                         (0.2, wrap)], D)
    x0 = rng.uniform(-1.0, 1.0, size=(D, 300))
    g = run_gpu(lik, pri, prop, x0, 77, 5, 1, 12)
    o = run_oracle(oracle, lik, pri, prop, x0, 77, 5, 1, 12)
    assert_same(g, o)


@pytest.mark.parametrize("D,lanes_auto", [(16, 1), (32, 2), (48, 4), (64, 4)])
@pytest.mark.parametrize("lik_kind", ["diag", "mix"])
@pytest.mark.parametrize("prop_kind", ["wrap", "de"])
def test_wide_proposals_split_over_lanes_bit_exact(oracle, T, D, lanes_auto, lik_kind, prop_kind):
    """Round 6: the wrapping-uniform and DE proposals on a separable or mixture likelihood split a
    wide chain over lanes (at most 16 dims a lane: the one-lane D 48 / 64 kernels spilled 0.2-1.7
    KB a lane).  The runtime picks the split; one lane forced and the split both equal the oracle
    bit for bit."""
    from mcmc_amd import Context
    rng = np.random.default_rng(D * 13 + len(lik_kind) + len(prop_kind))
    lik = _likelihood(T, rng, lik_kind, D)
    pri = _prior(T, rng, "asym_box", D)
    if prop_kind == "wrap":
        prop = T.uniform_wrapping(-3 * np.ones(D), 3 * np.ones(D), rng.uniform(0.05, 0.3, D))
        oprop = prop
    else:
        samples = rng.normal(0.0, 0.8, size=(200, D))
        prop = T.differential_evolution_proposal(samples, 0.2)
        oprop = T.Proposal(4, np.concatenate([[0.2, 200], samples.ravel()]))
    x0 = rng.uniform(-1.0, 1.0, size=(D, 300))
    o = run_oracle(oracle, lik, pri, oprop, x0, 31, 3, 2, 7)
    for lanes in (0, 1):
        g = run_gpu(lik, pri, prop, x0, 31, 3, 2, 7, lanes=lanes)
        assert_same(g, o)
    with Context(seed=31) as ctx:
        ctx.set_model(lik, pri, prop)
        ctx.init(x0)
        ctx.run(nbin=1, nskip=1, n_rec=1)
        assert ctx.lanes() == lanes_auto


def _nested_case(i):
    rng = np.random.default_rng(2000 + i)
    D = int(rng.choice([1, 2, 3, 4, 6, 8, 9, 12, 16, 20, 32]))
    lik = str(rng.choice(["diag", "shell", "fullcov", "mix"]))
    pri = str(rng.choice(["box", "asym_box", "open_box", "gauss"]))
    nlive = int(rng.choice([50, 120, 300, 513]))
    k = int(rng.choice([1, 1, 3, 16, 40]))
    k = min(k, nlive - 1)
    nmcmc = int(rng.choice([5, 13, 30]))
    return dict(i=i, D=D, lik=lik, pri=pri, nlive=nlive, k=k, nmcmc=nmcmc)


NESTED_CASES = [_nested_case(i) for i in range(24)]


@pytest.mark.parametrize("case", NESTED_CASES, ids=lambda c: "%(i)d-D%(D)d-%(lik)s-%(pri)s-n%(nlive)d-k%(k)d-m%(nmcmc)d" % c)
def test_nested_random_combinations_bit_exact(oracle, T, case):
    from test_gpu_nested import assert_nested_same, gpu_nested, oracle_nested
    rng = np.random.default_rng(6000 + case["i"])
    D = case["D"]
    lik = _likelihood(T, rng, case["lik"], D)
    pri = _prior(T, rng, case["pri"], D)
    seed = int(rng.integers(1, 2**31))
    k, nl = case["k"], case["nlive"]
    maxd = k * 25
    g = gpu_nested(lik, pri, seed, nlive=nl, nmcmc=case["nmcmc"], mode_hopping_frac=0.1, k=k, max_dead=maxd)
    o = oracle_nested(oracle, lik, pri, seed, nlive=nl, nmcmc=case["nmcmc"], mode_hop=0.1, k=k, max_iter=maxd)
    assert_nested_same(g, o)


@pytest.mark.parametrize("D", [3, 9, 24, 40, 64])
@pytest.mark.parametrize("lik_kind", ["diag", "shell", "fullcov", "mix"])
def test_differential_evolution_every_kind_and_width_bit_exact(oracle, T, D, lik_kind):
    """Mcmc.differential_evolution_proposal (mcmc.ml:198-218) at compiled and zero-padded widths for
    every likelihood kind, mode hopping 0.2: GPU == oracle bit for bit."""
    rng = np.random.default_rng(D * 11 + len(lik_kind))
    lik = _likelihood(T, rng, lik_kind, D)
    pri = _prior(T, rng, "box", D)
    samples = rng.normal(0.0, 0.8, size=(300, D))
    de = T.differential_evolution_proposal(samples, 0.2)
    x0 = rng.uniform(-1.0, 1.0, size=(D, 257))
    g = run_gpu(lik, pri, de, x0, 91, 4, 2, 6)
    o = run_oracle(oracle, lik, pri, T.Proposal(4, np.concatenate([[0.2, 300], samples.ravel()])), x0, 91, 4, 2, 6)
    assert_same(g, o)
