"""Data descriptors replacing the reference's closures (mcmc.mli:58-60, nested.mli:50-61).

Each descriptor carries the kind constant and the parameter vector of include/mcg.h.
"""
import math

import numpy as np

from . import _lib as L


def _f64(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64).ravel())


class Likelihood:
    def __init__(self, kind, ndim, params):
        self.kind, self.ndim, self.params = kind, int(ndim), _f64(params)


class Prior:
    def __init__(self, kind, params):
        self.kind, self.params = kind, _f64(params)


class Proposal:
    def __init__(self, kind, params=(0.0,)):
        self.kind, self.params = kind, _f64(params)


# ---- likelihoods ----
def flat(ndim):
    return Likelihood(L.LIK_FLAT, ndim, [0.0])


def diag_gauss(mu, sigma):
    """Stats.log_multi_gaussian mu sigma (stats.ml:103-108)."""
    mu, sigma = _f64(mu), _f64(sigma)
    return Likelihood(L.LIK_DIAG_GAUSS, len(mu), np.concatenate([mu, sigma]))


def fullcov_gauss(mu, cov=None, prec_chol_upper=None):
    """Gaussian with full covariance; U = upper Cholesky factor of the precision (U^T U = cov^-1)."""
    mu = _f64(mu)
    if prec_chol_upper is None:
        prec = np.linalg.inv(np.asarray(cov, dtype=np.float64))
        prec = 0.5 * (prec + prec.T)
        prec_chol_upper = np.linalg.cholesky(prec).T
    U = np.asarray(prec_chol_upper, dtype=np.float64)
    return Likelihood(L.LIK_FULLCOV_GAUSS, len(mu), np.concatenate([mu, U.ravel()]))


def gauss_shell(center, radius, width):
    c = _f64(center)
    return Likelihood(L.LIK_GAUSS_SHELL, len(c), np.concatenate([c, [radius, width]]))


def gauss_mix(mus, sigmas):
    """log (sum_i exp (Stats.log_multi_gaussian mu_i sigma_i x)): the four-Gaussian target of
    test/nested_test.ml:41-64 (mus, sigmas: (m, D) arrays, or one sigma row for every component)."""
    mus = np.atleast_2d(np.asarray(mus, dtype=np.float64))
    sigmas = np.broadcast_to(np.atleast_2d(np.asarray(sigmas, dtype=np.float64)), mus.shape)
    m, D = mus.shape
    if not 1 <= m <= L.LIK_MIX_MAX:
        raise ValueError("gauss_mix: 1 <= components <= %d" % L.LIK_MIX_MAX)
    blocks = np.concatenate([mus, sigmas], axis=1).ravel()
    return Likelihood(L.LIK_GAUSS_MIX, D, np.concatenate([[m], blocks]))


def gauss_data(data):
    """bin/gaussian_cauchy.ml log_like_gaussian: state = (mu[nd], sigma[nd])."""
    data = np.asarray(data, dtype=np.float64)
    nd = data.shape[1]
    return Likelihood(L.LIK_GAUSS_DATA, 2 * nd, np.concatenate([[nd], data.ravel()]))


def cauchy_data(data):
    data = np.asarray(data, dtype=np.float64)
    nd = data.shape[1]
    return Likelihood(L.LIK_CAUCHY_DATA, 2 * nd, np.concatenate([[nd], data.ravel()]))


# ---- priors ----
def flat_prior():
    return Prior(L.PRIOR_FLAT, [])


def box(lo, hi, lp_in=None, open_=False):
    lo, hi = _f64(lo), _f64(hi)
    if lp_in is None:
        lp_in = -sum(math.log(h - l) for l, h in zip(lo, hi))
    return Prior(L.PRIOR_OPEN_BOX if open_ else L.PRIOR_BOX, np.concatenate([lo, hi, [lp_in]]))


def gauss_prior(mu, sigma):
    """log_prior = Stats.log_multi_gaussian mu sigma (stats.ml:98-108); nested sampling's
    draw_prior = Stats.draw_gaussian mu sigma per dim (stats.ml:113-124)."""
    mu, sigma = _f64(mu), _f64(sigma)
    if mu.shape != sigma.shape:
        raise ValueError("gauss_prior: mu and sigma must have the same length")
    return Prior(L.PRIOR_DIAG_GAUSS, np.concatenate([mu, sigma]))


# ---- proposals ----
def gauss(scale):
    """y = x + scale * N(0, 1) per dim (symmetric; log_jump_prob = 0)."""
    return Proposal(L.PROP_GAUSS, np.atleast_1d(_f64(scale)))


def uniform_wrapping(lo, hi, dx):
    """Mcmc.uniform_wrapping xmin xmax dx per dim (mcmc.ml:187-196)."""
    lo, hi, dx = _f64(lo), _f64(hi), _f64(dx)
    return Proposal(L.PROP_WRAP_UNIFORM, np.concatenate([lo, hi, dx]))


class KdInterp:
    """Interpolate_pdf.make pts low high (interpolate_pdf.ml:111-112) as an MH jump proposal."""

    def __init__(self, pts, low, high):
        self.pts = np.ascontiguousarray(np.asarray(pts, dtype=np.float64))
        self.low, self.high = _f64(low), _f64(high)
        self.kind = L.PROP_KD_INTERP


class DifferentialEvolution:
    """Mcmc.differential_evolution_proposal ?mode_hopping_frac to_float from_float samples
    (mcmc.ml:198-218) as an MH jump proposal: samples (M, D) (M >= 2), log_jump_prob = 0."""

    def __init__(self, samples, mode_hopping_frac=0.0):
        self.samples = np.ascontiguousarray(np.asarray(samples, dtype=np.float64))
        if self.samples.ndim == 1:
            self.samples = self.samples[:, None]
        self.mode_hopping_frac = float(mode_hopping_frac)
        self.kind = L.PROP_DE


def differential_evolution_proposal(samples, mode_hopping_frac=0.0):
    return DifferentialEvolution(samples, mode_hopping_frac)


def shift_uniform(a, b):
    """y = x + random_between a b per dim (the uniform jumps of test/mcmc_test.ml:50,71-74,186-188);
    only as a component of combine_jump_proposals."""
    a, b = _f64(a), _f64(b)
    p = Proposal(MIX_SHIFT_UNIFORM_KIND, np.concatenate([a, b]))
    return p


MIX_SHIFT_UNIFORM_KIND = -2     # Python-side tag; mapped to MCG_MIX_SHIFT_UNIFORM below


class Mixture(Proposal):
    """Mcmc.combine_jump_proposals [(p, jump, log_jump_prob)] (mcmc.ml:165-185).

    components: (p, proposal) or (p, proposal, ljp) with proposal from gauss / shift_uniform /
    uniform_wrapping / KdInterp and ljp = 1 for the component's log density (default for gauss,
    shift_uniform, KdInterp) or 0 for the constant-zero log_jump_prob callers pass for symmetric
    jumps (default, and the only choice, for uniform_wrapping)."""

    def __init__(self, components, ndim):
        parts = [float(len(components))]
        self.kd = None
        for comp in components:
            p, prop = comp[0], comp[1]
            if isinstance(prop, KdInterp):
                if self.kd is not None:
                    raise ValueError("combine_jump_proposals: one kD component at most")
                self.kd = prop
                kind, params, mode = L.MIX_KD_INTERP, [], 1
            elif prop.kind == L.PROP_GAUSS:
                s = prop.params
                params = np.full(ndim, s[0]) if len(s) == 1 else s
                kind, mode = L.MIX_GAUSS, 1
            elif prop.kind == MIX_SHIFT_UNIFORM_KIND:
                kind, params, mode = L.MIX_SHIFT_UNIFORM, prop.params, 1
            elif prop.kind == L.PROP_WRAP_UNIFORM:
                kind, params, mode = L.MIX_WRAP_UNIFORM, prop.params, 0
            else:
                raise ValueError("unsupported mixture component kind %r" % prop.kind)
            if len(comp) > 2:
                mode = int(comp[2])
            parts += [float(p), float(kind), float(mode)] + list(np.asarray(params, np.float64))
        super().__init__(L.PROP_MIXTURE, parts)


def combine_jump_proposals(components, ndim):
    return Mixture(components, ndim)


# ---- reversible-jump descriptors (Mcmc.make_rjmcmc_sampler, mcmc.ml:89-119) ----
class RjJump:
    """A jump of one RJ model: kind MCG_RJ_JUMP_* with its parameters (include/mcg.h)."""

    def __init__(self, kind, params=(), kd=None):
        self.kind, self.params, self.kd = kind, _f64(params if len(params) else [0.0]), kd
        self.n = len(params)


def rj_gauss(scale):
    """random-walk jump x + s z (log_jump_prob 0)."""
    return RjJump(L.RJ_JUMP_GAUSS, np.atleast_1d(_f64(scale)))


def rj_wrap(lo, hi, dx):
    """Mcmc.uniform_wrapping per dim (log_jump_prob 0)."""
    return RjJump(L.RJ_JUMP_WRAP, np.concatenate([_f64(lo), _f64(hi), _f64(dx)]))


def rj_indep_gauss(mu, sigma):
    """independence draw Stats.draw_gaussian mu sigma per dim; log_jump_prob _ y = log N(y)."""
    return RjJump(L.RJ_JUMP_INDEP_GAUSS, np.concatenate([_f64(mu), _f64(sigma)]))


def rj_kd(pts, low, high):
    """independence draw Interpolate_pdf.draw; log_jump_prob _ y = log (jump_prob y)."""
    return RjJump(L.RJ_JUMP_KD, [], KdInterp(pts, low, high))


class RjModel:
    """One model of a reversible-jump pair: likelihood, prior, internal jump, jump into it,
    model prior probability."""

    def __init__(self, log_likelihood, log_prior, jump, jump_into, model_prior):
        self.lik, self.prior, self.jump, self.into = log_likelihood, log_prior, jump, jump_into
        self.model_prior = float(model_prior)
        kds = [j.kd for j in (jump, jump_into) if j.kd is not None]
        if len(kds) == 2 and kds[0] is not kds[1]:
            raise ValueError("one kD tree per RJ model: pass the same rj_kd to jump and jump_into")
        self.kd = kds[0] if kds else None

    @property
    def ndim(self):
        return self.lik.ndim

    def c_struct(self):
        kd = self.kd
        return L.McgRjModel(self.ndim, self.lik.kind, L.dptr(self.lik.params), len(self.lik.params),
                            self.prior.kind, L.dptr(self.prior.params), len(self.prior.params),
                            self.jump.kind, L.dptr(self.jump.params), self.jump.n,
                            self.into.kind, L.dptr(self.into.params), self.into.n,
                            L.dptr(kd.pts) if kd else None, kd.pts.shape[0] if kd else 0,
                            L.dptr(kd.low) if kd else None, L.dptr(kd.high) if kd else None,
                            self.model_prior)
