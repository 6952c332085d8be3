"""GPU tests of a context's state across calls: the Philox step counter and the accept / reject
tallies run on across mcg_init (as the reference's global Random state and its global counters,
mcmc.ml:27-35, do), host uploads are ordered after in-flight kernels, and a nested run's result
reports whether the stop test fired.  Every draw is checked bit for bit against the oracle at
the step index it must have used."""
import math
import warnings

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def T():
    from mcmc_amd import targets
    return targets


def c2_model(T, D=8, seed=42):
    rng = np.random.default_rng(seed)
    mu, sg = rng.uniform(-1, 1, D), rng.uniform(0.5, 2, D)
    s = 2.38 / math.sqrt(D) * float(np.median(sg))
    return T.diag_gauss(mu, sg), T.box(-10 * np.ones(D), 10 * np.ones(D)), T.gauss(s), mu, sg


def oracle_model(O, lik, pri, prop):
    return O.Model(lik.ndim, lik.kind, lik.params, pri.kind, pri.params, prop.kind, prop.params)


def oracle_start(m, x0):
    N = x0.shape[1]
    return (np.array([m.loglik(x0[:, i]) for i in range(N)]),
            np.array([m.logprior(x0[:, i]) for i in range(N)]))


def test_make_mcmc_sampler_successive_steps_draw_successive_indices(oracle, T):
    """Two step() calls of Mcmc.make_mcmc_sampler (mcmc.ml:37-56) from the returned state are the
    oracle's steps 0 and 1, not step 0 twice; the counters add up over both calls."""
    from mcmc_amd import Context, mcmc
    lik, pri, prop, mu, sg = c2_model(T)
    N = 256
    x0 = np.random.default_rng(3).normal(mu[:, None], sg[:, None], size=(8, N))
    m = oracle_model(oracle, lik, pri, prop)
    ll0, lp0 = oracle_start(m, x0)
    ctx = Context(seed=5)
    step = mcmc.make_mcmc_sampler(lik, pri, prop, ctx=ctx)
    s1 = step((x0, ll0, lp0))
    s2 = step(s1)
    o1 = oracle.mh_run(m, 5, x0, ll0, lp0, nbin=1, n_rec=0, record_x=False, record_llp=False,
                       record_accept=False, accumulate=False, step0=0)
    o2 = oracle.mh_run(m, 5, o1["x"], o1["ll"], o1["lp"], nbin=1, n_rec=0, record_x=False,
                       record_llp=False, record_accept=False, accumulate=False, step0=1)
    for s, o in ((s1, o1), (s2, o2)):
        np.testing.assert_array_equal(s[0], o["x"])
        np.testing.assert_array_equal(s[1], o["ll"])
        np.testing.assert_array_equal(s[2], o["lp"])
    # the same draw twice would move an accepted chain by the same vector again
    d1, d2 = s1[0] - x0, s2[0] - s1[0]
    both = np.all(d1 != 0, axis=0) & np.all(d2 != 0, axis=0)
    assert both.any()
    assert not np.any(np.all(d1[:, both] == d2[:, both], axis=0))
    acc, rej = ctx.counters()
    assert acc == int(o1["nacc"].sum() + o2["nacc"].sum()) and acc + rej == 2 * N
    assert ctx.rng_step() == 2
    ctx.close()


def test_run_then_reinit_without_sync_matches_oracle(oracle, T):
    """mcg_run returns without a sync; an immediate init() of new chains must wait for the
    in-flight MH kernel (no torn state), and the second run continues the Philox step counter."""
    from mcmc_amd import Context
    lik, pri, prop, mu, sg = c2_model(T)
    N = 4096
    rng = np.random.default_rng(7)
    xa = rng.normal(mu[:, None], sg[:, None], size=(8, N))
    xb = rng.normal(mu[:, None], sg[:, None], size=(8, N))
    m = oracle_model(oracle, lik, pri, prop)
    ctx = Context(seed=9)
    ctx.set_model(lik, pri, prop)
    ctx.init(xa)
    ctx.run(nbin=2000, n_rec=0, record_x=False, record_llp=False)   # long, left in flight
    ctx.init(xb)
    ctx.run(nbin=30, n_rec=0, record_x=False, record_llp=False)
    x, ll, lp = ctx.state()
    acc, rej = ctx.counters()
    lla, lpa = oracle_start(m, xa)
    oa = oracle.mh_run(m, 9, xa, lla, lpa, nbin=2000, n_rec=0, record_x=False, record_llp=False,
                       record_accept=False, accumulate=False, nthreads=8)
    llb, lpb = oracle_start(m, xb)
    ob = oracle.mh_run(m, 9, xb, llb, lpb, nbin=30, n_rec=0, record_x=False, record_llp=False,
                       record_accept=False, accumulate=False, step0=2000, nthreads=8)
    np.testing.assert_array_equal(x, ob["x"])
    np.testing.assert_array_equal(ll, ob["ll"])
    np.testing.assert_array_equal(lp, ob["lp"])
    # Mcmc's counters are global until reset_counters: both chain sets count
    assert acc == int(oa["nacc"].sum() + ob["nacc"].sum())
    assert acc + rej == 2030 * N
    ctx.reset_counters()
    assert ctx.counters() == (0, 0)
    ctx.close()


def test_set_model_after_run_waits_for_the_kernel(oracle, T):
    """A new likelihood uploaded right after an unsynchronised run must not reach that run."""
    from mcmc_amd import Context
    lik, pri, prop, mu, sg = c2_model(T)
    lik2 = T.diag_gauss(mu + 0.5, sg * 1.5)
    N = 4096
    x0 = np.random.default_rng(8).normal(mu[:, None], sg[:, None], size=(8, N))
    m = oracle_model(oracle, lik, pri, prop)
    ctx = Context(seed=4)
    ctx.set_model(lik, pri, prop)
    ctx.init(x0)
    ctx.run(nbin=2000, n_rec=0, record_x=False, record_llp=False)
    ctx.set_model(lik2, pri, prop)           # would race the kernel without the drain
    x, ll, _ = ctx.state()
    ll0, lp0 = oracle_start(m, x0)
    o = oracle.mh_run(m, 4, x0, ll0, lp0, nbin=2000, n_rec=0, record_x=False, record_llp=False,
                      record_accept=False, accumulate=False, nthreads=8)
    np.testing.assert_array_equal(x, o["x"])
    np.testing.assert_array_equal(ll, o["ll"])
    ctx.close()


def test_reseed_restarts_the_stream(oracle, T):
    """Context.reseed (Random.init): the step counter returns to 0, so a run after a reseed to
    the same seed repeats a fresh context's run exactly; without it a repeated run differs."""
    from mcmc_amd import Context
    lik, pri, prop, mu, sg = c2_model(T)
    x0 = np.random.default_rng(11).normal(mu[:, None], sg[:, None], size=(8, 512))
    ctx = Context(seed=21)
    ctx.set_model(lik, pri, prop)
    outs = []
    for reseed in (False, False, True):
        if reseed:
            ctx.reseed(21)
        ctx.init(x0)
        ctx.run(nbin=20, n_rec=0, record_x=False, record_llp=False)
        outs.append(ctx.state()[0])
    assert not np.array_equal(outs[0], outs[1])
    np.testing.assert_array_equal(outs[0], outs[2])
    ctx.close()


def test_nested_cap_reports_unconverged_and_failed_run_clears_result(T):
    """max_dead reached before the stop test: the result says converged = False (with a
    warning); a later run that fails leaves no stale result for mcg_nested_get."""
    from mcmc_amd import Context, nested
    from mcmc_amd._lib import McgError
    lik = T.diag_gauss([0.5, 0.5], [0.1, 0.1])
    pri = T.box([0, 0], [1, 1], 0.0, open_=True)
    ctx = Context(seed=2)
    with pytest.warns(nested.UnconvergedWarning):
        out = nested.nested_evidence(lik, pri, ctx=ctx, nlive=200, nmcmc=10, k=10, max_dead=100)
    assert not out.converged and out.n_dead == 100
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        full = nested.nested_evidence(lik, pri, ctx=ctx, nlive=200, nmcmc=10, k=10)
    assert full.converged and full.n_dead > 100
    with pytest.raises(McgError):          # max_dead below one generation: fails mid-setup
        nested.nested_evidence(lik, pri, ctx=ctx, nlive=200, nmcmc=10, k=10, max_dead=5)
    from mcmc_amd import _lib as L
    p = np.zeros((full.ll.size, 2)); a = np.zeros(full.ll.size)
    rc = L.lib().mcg_nested_get(ctx.ptr, L.dptr(p), L.dptr(a), L.dptr(a), L.dptr(a))
    assert rc == L.MCG_ESTATE
    ctx.close()


def test_nested_take_hands_over_the_arrays_once_per_run(T):
    """mcg_nested_take (what nested.fetch uses): the run's ll / lp / log weights handed over
    without a copy equal mcg_nested_get's copies of the same run (same seed); afterwards get
    refuses them (points still copy) and a second take fails until the next run; the handed-over
    arrays outlive the next run and the context."""
    import gc
    from mcmc_amd import Context, nested
    from mcmc_amd import _lib as L
    from mcmc_amd._lib import McgError
    lik = T.gauss_shell(np.zeros(4), 1.0, 0.2)
    pri = T.box(-2 * np.ones(4), 2 * np.ones(4))
    ctx = Context(seed=21)
    r = nested.run_nested(lik, pri, nlive=400, nmcmc=10, k=20, ctx=ctx)
    n = r.n_total
    p0 = np.zeros((n, 4)); a0, b0, w0 = np.zeros(n), np.zeros(n), np.zeros(n)
    L.check(L.lib().mcg_nested_get(ctx.ptr, L.dptr(p0), L.dptr(a0), L.dptr(b0), L.dptr(w0)), ctx.ptr)
    r = nested.run_nested(lik, pri, nlive=400, nmcmc=10, k=20, ctx=ctx)
    out = nested.fetch(ctx, r, 4, points=True, k=20)
    np.testing.assert_array_equal(out[2], p0)
    np.testing.assert_array_equal(out.ll, a0)
    np.testing.assert_array_equal(out.lp, b0)
    np.testing.assert_array_equal(out[3], w0)
    a = np.zeros(n)
    assert L.lib().mcg_nested_get(ctx.ptr, None, L.dptr(a), None, None) == L.MCG_ESTATE
    p = np.zeros((n, 4))
    L.check(L.lib().mcg_nested_get(ctx.ptr, L.dptr(p), None, None, None), ctx.ptr)
    np.testing.assert_array_equal(p, p0)
    with pytest.raises(McgError):
        nested.fetch(ctx, r, 4, points=False)
    ll_view = out.ll[5:50]                         # a view keeps the handed-over block alive
    nested.nested_evidence(lik, pri, nlive=300, nmcmc=10, k=20, ctx=ctx)
    ctx.close()
    del out
    gc.collect()
    np.testing.assert_array_equal(ll_view, a0[5:50])


def test_failed_set_rjmcmc_leaves_counters_unchanged(oracle, T):
    """mcg_set_rjmcmc folds the device tallies into the context totals before it validates the
    models; a model it then rejects (unsupported likelihood kind) must leave get_counters where
    it was: neither counting the accepts twice nor wrapping the rejects."""
    from mcmc_amd import Context, mcmc
    from mcmc_amd._lib import McgError
    lik, pri, prop, mu, sg = c2_model(T)
    x0 = np.random.default_rng(12).normal(mu[:, None], sg[:, None], size=(8, 1024))
    ctx = Context(seed=13)
    ctx.set_model(lik, pri, prop)
    ctx.init(x0)
    ctx.run(nbin=50, n_rec=0, record_x=False, record_llp=False)
    before = ctx.counters()
    assert before[0] > 0 and sum(before) == 50 * 1024
    data = T.cauchy_data(np.zeros((5, 1)))            # RJ rejects data likelihoods after the fold
    bad = T.RjModel(data, T.flat_prior(), T.rj_gauss(0.1), T.rj_indep_gauss([0, 1], [1, 1]), 0.5)
    good = T.RjModel(T.flat(2), T.flat_prior(), T.rj_gauss(0.1), T.rj_indep_gauss([0, 1], [1, 1]), 0.5)
    with pytest.raises(McgError):
        mcmc.rjmcmc_array(4, bad, good, (np.zeros(2), np.zeros(2)), nchains=8, ctx=ctx)
    assert ctx.counters() == before
    assert ctx.counters() == before                    # reading twice changes nothing either
    ctx.close()


def test_last_run_lanes_reports_the_lane_split(T):
    """mcg_last_run_lanes: the lanes per chain the last MH run used -- the runtime's auto choice
    (4 for a D = 32 Gaussian that does not fill the chip on fewer lanes), or the caller's."""
    from mcmc_amd import Context
    lik, pri, prop, mu, sg = c2_model(T, D=32)
    x0 = np.random.default_rng(5).normal(mu[:, None], sg[:, None], size=(32, 1024))
    for want, expect in ((0, 4), (1, 1), (2, 2)):
        with Context(seed=1, lanes_per_chain=want) as ctx:
            ctx.set_model(lik, pri, prop)
            ctx.init(x0)
            ctx.run(nbin=4, nskip=1, n_rec=1, record_x=False, record_llp=False,
                    record_accept=False, accumulate=False)
            assert ctx.lanes() == expect


def test_state_token_moves_with_every_state_change(T):
    """mcg_state_token (include/mcg.h): bumped by init, run, the setters, a nested run and reseed;
    unchanged by reads (state, counters, records).  The OCaml sampler keeps the chains resident
    only while it is unchanged since its own step."""
    import mcmc_amd._lib as L
    from mcmc_amd import Context, nested
    lik, pri, prop, mu, sg = c2_model(T)
    tok = lambda c: int(L.lib().mcg_state_token(c.ptr))
    with Context(seed=3) as ctx:
        ctx.set_model(lik, pri, prop)
        t0 = tok(ctx)
        ctx.init(np.random.default_rng(0).normal(mu[:, None], sg[:, None], size=(8, 64)))
        t1 = tok(ctx)
        ctx.run(nbin=2, nskip=1, n_rec=0, record_x=False, record_llp=False)
        t2 = tok(ctx)
        ctx.state(); ctx.counters(); ctx.sync()
        assert tok(ctx) == t2
        ctx.set_model(lik, pri, prop)
        t3 = tok(ctx)
        nested.nested_evidence(T.diag_gauss(mu, sg), pri, nlive=50, nmcmc=5, k=1, ctx=ctx, max_dead=20)
        t4 = tok(ctx)
        L.check(L.lib().mcg_reseed(ctx.ptr, 5), ctx.ptr)
        t5 = tok(ctx)
        assert t0 < t1 < t2 < t3 < t4 < t5


def test_likelihood_kind_change_keeps_prior_and_proposal(oracle, T):
    """at ndim 9 DIAG_GAUSS pads to width 12 and FULLCOV_GAUSS to 16.  Changing the
    kind before mcg_init keeps the caller's box prior and Gaussian proposal (re-laid out at the
    new width) instead of resetting them to FLAT / GAUSS(1): the run equals the oracle's with
    that prior and proposal.  After mcg_init the change is refused with an error naming the
    kernel widths."""
    import mcmc_amd._lib as L
    from mcmc_amd import Context
    D = 9
    rng = np.random.default_rng(9)
    mu, sg = rng.uniform(-0.5, 0.5, D), rng.uniform(0.5, 1.5, D)
    A = rng.normal(size=(D, D))
    cov = A @ A.T / D + np.eye(D)
    lo, hi = -1.5 * np.ones(D), 1.5 * np.ones(D)
    pri, prop = T.box(lo, hi), T.gauss(0.6)
    fc = T.fullcov_gauss(mu, cov)
    x0 = rng.uniform(-1, 1, size=(D, 80))
    with Context(seed=12) as ctx:
        ctx.set_model(T.diag_gauss(mu, sg), pri, prop)
        ctx.set_model(fc)                        # likelihood only: prior and proposal stay
        ctx.init(x0)
        ctx.run(nbin=0, nskip=1, n_rec=30, record_x=True, record_llp=True, record_accept=True)
        rx, rll, rlp, bits = ctx.records(x=True, llp=True, accept=True)
        m = oracle.Model(D, fc.kind, fc.params, pri.kind, pri.params, prop.kind, prop.params)
        ll0 = np.array([m.loglik(x0[:, i]) for i in range(80)])
        lp0 = np.array([m.logprior(x0[:, i]) for i in range(80)])
        o = oracle.mh_run(m, 12, x0, ll0, lp0, nbin=0, nskip=1, n_rec=30, nthreads=8)
        np.testing.assert_array_equal(rx, o["rec_x"])
        np.testing.assert_array_equal(rlp, o["rec_lp"])
        np.testing.assert_array_equal(bits, o["bits"])
        assert np.all(np.abs(rx) <= 1.5)
        with pytest.raises(L.McgError, match="kernel width 12"):
            ctx.set_model(T.diag_gauss(mu, sg))
