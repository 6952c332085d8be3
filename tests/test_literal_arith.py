"""How far the GPU's canonical arithmetic is from the reference's literal arithmetic.

The kernels (and the oracle by default) evaluate the log-target in a canonical form -- fma
residuals x/sigma - mu/sigma, an 8-accumulator sum, a host constant C = sum(-1/2 log 2pi -
log sigma) -- take the accept test's log u with a portable log, and fold the nested running
estimate with a portable log-sum.  The reference does Stats.log_multi_gaussian literally
(stats.ml:98-108), glibc log of the uniform (mcmc.ml:49) and Stats.log_sum_logs
(stats.ml:240-248).  The oracle's literal mode (or_set_literal) restates those, and these tests
drive both forms from the same Philox stream:

  - C2-mini (128 chains, D = 32, 256 steps): every proposal judged both ways along the canonical
    chain -- ll relative difference and flipped accept decisions -- and a whole run in each mode;
  - C3-mini (the nested_test.ml Gaussian, nlive 64 / 1000, k 1, 4, 16): dead-point sequence,
    stop generation and log Z in each mode.

Committed bounds: ll relative difference <= 1e-13 (observed <= 1e-15); zero
flipped accept decisions on these streams (the closest decision margin |log u - ratio| seen is
~3e-4, twelve orders of magnitude above the ll differences); identical stop generation and
log Z within 1e-12 relative."""
import ctypes as C
import math

import numpy as np
import pytest

LIK_DIAG, PRIOR_BOX, PRIOR_OPEN, PROP_GAUSS = 1, 1, 2, 1


@pytest.fixture
def literal(oracle):
    L = oracle.lib()
    yield L
    L.or_set_literal(0)


def _c2_mini(O, N=128, D=32, seed=42):
    rng = np.random.default_rng(seed)
    mu, sg = rng.uniform(-1, 1, D), rng.uniform(0.5, 2, D)
    s = 2.38 / math.sqrt(D) * float(np.median(sg))
    m = O.Model(D, LIK_DIAG, np.concatenate([mu, sg]), PRIOR_BOX,
                np.concatenate([-10 * np.ones(D), 10 * np.ones(D), [-D * math.log(20.0)]]), PROP_GAUSS, [s])
    x0 = np.ascontiguousarray(rng.normal(mu[:, None], sg[:, None], size=(D, N)))
    return m, x0, mu, sg


def test_literal_log_multi_gaussian_is_the_reference_formula(oracle, literal):
    """The literal mode's likelihood is stats.ml:98-108 term by term (checked against a Python
    restatement of the same operation order, bit for bit) and within 1e-13 of the canonical form."""
    m, x0, mu, sg = _c2_mini(oracle, N=64)
    canon = np.array([m.loglik(x0[:, i]) for i in range(64)])
    literal.or_set_literal(1)
    lit = np.array([m.loglik(x0[:, i]) for i in range(64)])
    literal.or_set_literal(0)
    for i in range(64):
        r = 0.0
        for d in range(len(mu)):
            dx = (x0[d, i] - mu[d]) / sg[d]
            r = r + ((-0.91893853320467274178 - math.log(sg[d])) - 0.5 * dx * dx)
        assert lit[i] == r + 0.0
    assert np.max(np.abs(lit - canon) / np.abs(canon)) <= 1e-13


def test_c2_mini_accept_decisions_under_literal_arithmetic(oracle, literal):
    m, x0, _, _ = _c2_mini(oracle)
    N, steps = x0.shape[1], 256
    ll0 = np.array([m.loglik(x0[:, i]) for i in range(N)])
    lp0 = np.array([m.logprior(x0[:, i]) for i in range(N)])
    flips = np.zeros(N, np.int64)
    mrel, mmar = C.c_double(), C.c_double()
    rc = literal.or_mh_literal_shadow(C.byref(m.s), 1, N, 0, steps, oracle.dptr(x0), oracle.dptr(ll0),
                                      oracle.dptr(lp0), flips.ctypes.data_as(C.POINTER(C.c_int64)),
                                      C.byref(mrel), C.byref(mmar))
    assert rc == 0
    print("C2-mini shadow: flipped decisions %d of %d, max ll rel diff %.3g, min margin %.3g"
          % (flips.sum(), N * steps, mrel.value, mmar.value))
    assert flips.sum() == 0
    assert mrel.value <= 1e-13
    assert mmar.value > 1e6 * mrel.value * np.abs(ll0).max()
    # whole runs in each mode from the same Philox stream: the same accept bitmap and records
    canon = oracle.mh_run(m, 1, x0, ll0, lp0, nbin=0, nskip=1, n_rec=steps + 1, nthreads=8)
    literal.or_set_literal(1)
    ll1 = np.array([m.loglik(x0[:, i]) for i in range(N)])
    lit = oracle.mh_run(m, 1, x0, ll1, lp0, nbin=0, nskip=1, n_rec=steps + 1, nthreads=8)
    literal.or_set_literal(0)
    np.testing.assert_array_equal(canon["bits"], lit["bits"])
    np.testing.assert_array_equal(canon["rec_x"], lit["rec_x"])
    assert np.max(np.abs(lit["rec_ll"] - canon["rec_ll"]) / np.abs(canon["rec_ll"])) <= 1e-13


@pytest.mark.parametrize("nlive,k", [(64, 1), (64, 4), (1000, 1), (1000, 16)])
def test_c3_mini_nested_under_literal_arithmetic(oracle, literal, nlive, k):
    """nested_test.ml's Gaussian: the canonical and literal runs retire the same points in the
    same order, stop at the same generation, and agree on log Z to 1e-12 relative."""
    m = oracle.Model(2, LIK_DIAG, [0.5, 0.5, 0.1, 0.1], PRIOR_OPEN, [0, 0, 1, 1, 0.0], PROP_GAUSS, [1.0])
    a = oracle.nested(m, 3, nlive=nlive, nmcmc=20, k=k)
    literal.or_set_literal(1)
    b = oracle.nested(m, 3, nlive=nlive, nmcmc=20, k=k)
    literal.or_set_literal(0)
    print("C3-mini nlive %d k %d: n_dead %d vs %d, log Z %.17g vs %.17g"
          % (nlive, k, a["n_dead"], b["n_dead"], a["log_ev"], b["log_ev"]))
    assert a["n_dead"] == b["n_dead"] and a["n_gen"] == b["n_gen"]
    np.testing.assert_array_equal(a["pts"], b["pts"])
    # relative to max(|ll|, 1): near the peak ll crosses 0 (the terms are O(1) and cancel)
    assert np.max(np.abs(a["ll"] - b["ll"]) / np.maximum(np.abs(a["ll"]), 1.0)) <= 1e-13
    assert abs(a["log_ev"] - b["log_ev"]) <= 1e-12 * max(abs(a["log_ev"]), 1.0)
