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
