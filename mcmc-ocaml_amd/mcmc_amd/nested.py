"""Mirror of the reference's Nested module (nested.mli) over the HIP sampler."""
import atexit
import ctypes as C
import warnings
import weakref

import numpy as np

from . import _lib as L
from .context import Context


def nested_evidence(log_likelihood, log_prior, epsrel=0.01, nmcmc=1000, nlive=1000,
                    mode_hopping_frac=0.1, k=1, observer=None, ctx=None, seed=0, max_dead=0,
                    points=True):
    """Nested.nested_evidence (nested.ml:122-146).

    log_prior must be a box prior (draw_prior = uniform in the box).  Returns the
    nested_output tuple (nested.ml:20): (log_ev, log_dev, points (n, D), log_wts (n,)) where the
    points are dead points in retirement order followed by the final live points ascending in
    log-likelihood; `ll`, `lp` of every point are in the returned .ll / .lp attributes.
    points=False leaves the points on the device (no D2H copy of n x D doubles; points is None):
    log Z, log dZ, the weights and ll / lp are computed all the same."""
    ctx = ctx or Context(seed=seed)
    r = run_nested(log_likelihood, log_prior, epsrel, nmcmc, nlive, mode_hopping_frac, k, observer, ctx,
                   max_dead)
    return fetch(ctx, r, log_likelihood.ndim, points, k)


def _owned(ptr, n):
    """A numpy view of n doubles the library handed over (mcg_nested_take), released with
    mcg_free when the last array referring to it is collected."""
    if n == 0:
        L.lib().mcg_free(C.cast(ptr, C.c_void_p))
        return np.zeros(0)
    a = np.ctypeslib.as_array(ptr, shape=(n,))
    weakref.finalize(a, L.lib().mcg_free, C.cast(ptr, C.c_void_p).value)
    return a


def fetch(ctx, r, ndim, points=True, k=None):
    """nested_output of the context's last run (r: its McgNestedResult): the points copied by
    mcg_nested_get (points=True); ll, lp and the log weights handed over without a copy
    (mcg_nested_take), once per run."""
    n = r.n_total
    pts = None
    if points:
        pts = np.zeros((n, ndim))
        L.check(L.lib().mcg_nested_get(ctx.ptr, L.dptr(pts), None, None, None), ctx.ptr)
    pl, pp, pw = L._dp(), L._dp(), L._dp()
    L.check(L.lib().mcg_nested_take(ctx.ptr, C.byref(pl), C.byref(pp), C.byref(pw)), ctx.ptr)
    ll, lp, w = _owned(pl, n), _owned(pp, n), _owned(pw, n)
    return NestedOutput(r.log_ev, r.log_dev, pts, w, ll, lp, r.n_dead, r.n_gen, bool(r.converged), k)


def run_nested(log_likelihood, log_prior, epsrel=0.01, nmcmc=1000, nlive=1000, mode_hopping_frac=0.1,
               k=1, observer=None, ctx=None, max_dead=0):
    """The nested run alone (mcg_nested): its points stay on the device, for mcg_nested_get or a
    device-side exchange (Context.nested_rows_into).  Returns the McgNestedResult (log_ev,
    log_dev, n_dead, n_total, n_gen, converged); warns when max_dead ended the run."""
    ctx.set_model(log_likelihood, log_prior, None)
    o = L.McgNestedOpts(nlive, nmcmc, k, epsrel, mode_hopping_frac, max_dead)
    r = L.McgNestedResult()
    D = log_likelihood.ndim

    def _obs(user, pts, ll, lp, n):
        if observer is not None:
            p = np.ctypeslib.as_array(pts, shape=(n, D)).copy()
            a = np.ctypeslib.as_array(ll, shape=(n,)).copy()
            b = np.ctypeslib.as_array(lp, shape=(n,)).copy()
            for i in range(n):
                observer((p[i], a[i], b[i]))

    cb = L.OBSERVER(_obs) if observer is not None else L.OBSERVER()
    L.check(L.lib().mcg_nested(ctx.ptr, C.byref(o), C.byref(r), cb, None), ctx.ptr)
    if not r.converged:
        warnings.warn("nested_evidence: max_dead (%d dead points) reached before the stop test "
                      "(nested.ml:45-48) fired; log Z comes from an unconverged run" % r.n_dead,
                      UnconvergedWarning, stacklevel=3)
    return r


class UnconvergedWarning(RuntimeWarning):
    """A nested run stopped at its max_dead safety cap instead of the reference's stop test."""


class NestedOutput(tuple):
    """nested_output (nested.ml:20) plus ll / lp per point, counts and `converged` (False when
    the max_dead cap ended the run before remaining_integral_negligable fired) and `k`, the
    points retired per generation that the run actually used (None when unknown)."""
    def __new__(cls, log_ev, log_dev, pts, log_wts, ll, lp, n_dead, n_gen, converged=True, k=None):
        t = super().__new__(cls, (log_ev, log_dev, pts, log_wts))
        t.ll, t.lp, t.n_dead, t.n_gen, t.converged, t.k = ll, lp, n_dead, n_gen, converged, k
        return t


def merge_runs(runs):
    """Merge independent nested runs (replicas) into one run (include/mcg.h mcg_nested_merge).

    runs = [(output, nlive, k)] with output a nested_output-like tuple carrying .ll/.lp (or a
    (log_ev, log_dev, pts, log_wts, ll, lp) tuple).  Returns a NestedOutput over the union of the
    points in ascending ll; n_dead counts every point that is not among the final live points of
    the merged run's last run."""
    n_total = np.array([len(_ll(o)) for o, _, _ in runs], np.int64)
    nlive = np.array([nl for _, nl, _ in runs], np.int64)
    kk = np.array([k for _, _, k in runs], np.int64)
    ll = np.ascontiguousarray(np.concatenate([_ll(o) for o, _, _ in runs]), np.float64)
    lp = np.concatenate([_lp(o) for o, _, _ in runs])
    pts = None if any(o[2] is None for o, _, _ in runs) else np.concatenate([np.asarray(o[2]) for o, _, _ in runs])
    n = len(ll)
    order = np.zeros(n, np.int64)
    w = np.zeros(n)
    le, ld = C.c_double(), C.c_double()
    L.check(L.lib().mcg_nested_merge(len(runs), L.i64ptr(n_total), L.i64ptr(nlive), L.i64ptr(kk),
                                     L.dptr(ll), L.i64ptr(order), C.byref(le), C.byref(ld),
                                     L.dptr(w)))
    n_dead = int(n - nlive.sum())
    n_gen = int(sum(getattr(o, "n_gen", 0) for o, _, _ in runs))
    conv = all(getattr(o, "converged", True) for o, _, _ in runs)
    return NestedOutput(le.value, ld.value, None if pts is None else pts[order], w, ll[order], lp[order],
                        n_dead, n_gen, conv)


def evidence_weights(ll, nlive, k=1, chunk=0):
    """evidence_error_and_weights (nested.ml:81-120) on the host (include/mcg.h
    mcg_evidence_weights): ll in nested_output order (dead points in retirement order, then the
    nlive final live points ascending), k retirements per generation.  Returns (log Z, log dZ,
    log weights) -- the fold mcg_nested runs beside the GPU; `chunk` > 0 streams the dead points
    in chunks first, as the nested loop does."""
    ll = np.ascontiguousarray(ll, np.float64)
    w = np.zeros(len(ll))
    le, ld = C.c_double(), C.c_double()
    L.check(L.lib().mcg_evidence_weights(len(ll), int(nlive), int(k), L.dptr(ll), int(chunk), C.byref(le),
                                         C.byref(ld), L.dptr(w)))
    return le.value, ld.value, w


def _ll(o):
    return np.asarray(o.ll if hasattr(o, "ll") else o[4], np.float64)


def _lp(o):
    return np.asarray(o.lp if hasattr(o, "lp") else o[5], np.float64)


def log_total_error_estimate(log_ev, log_dev, nlive):
    """Nested.log_total_error_estimate (nested.ml:148-150)."""
    return L.lib().mcg_log_total_error_estimate(log_ev, log_dev, nlive)


_default_ctx = {}


def _close_default_contexts():
    for c in list(_default_ctx.values()):
        try:
            c.close()
        except Exception:
            pass
    _default_ctx.clear()


atexit.register(_close_default_contexts)


def _posterior_context(seed, device=0):
    """The context posterior draws use when the caller passes none: one per (seed, device) for
    the process, so repeated calls advance its draw counter and return new samples, as the
    reference's global Random state does (a fresh context per call would replay call 0).  Closed
    at interpreter exit, before the HIP runtime is torn down."""
    key = (int(seed), int(device))
    c = _default_ctx.get(key)
    if c is None:
        c = _default_ctx[key] = Context(seed=seed, device=device)
    return c


def posterior_indices(n, log_wts, ctx=None, seed=0, device=0):
    """The draws of Nested.posterior_samples (nested.ml:167-178) as indices into the points:
    cumulative weights and the reference's weight_binary_search_index (:152-165) on the device,
    one Philox draw per sample (include/mcg.h mcg_posterior_samples).  Repeated calls on one
    context -- the caller's, or without one the process-wide context of `seed` -- draw new
    samples (the reference's global Random state advances)."""
    ctx = ctx or _posterior_context(seed, device)
    w = np.ascontiguousarray(log_wts, dtype=np.float64)
    idx = np.zeros(int(n), np.int64)
    L.check(L.lib().mcg_posterior_samples(ctx.ptr, L.dptr(w), len(w), int(n), L.i64ptr(idx)), ctx.ptr)
    return idx


def posterior_samples(n, output, ctx=None, seed=0, device=0):
    """Nested.posterior_samples n output (nested.ml:167-178): n points resampled by weight from a
    nested_output (points (npts, D) and log weights); without a ctx, the process-wide context of
    (seed, device) draws them."""
    _, _, pts, log_wts = output[:4]
    if pts is None:
        raise ValueError("posterior_samples needs the points: run nested_evidence with points=True")
    assert len(pts) == len(log_wts)                 # nested.ml:169
    return np.asarray(pts)[posterior_indices(n, log_wts, ctx, seed, device)]
