"""Mirror of Evidence.Make(MO) (evidence.ml:21-221).

evidence_harmonic_mean: on-device form -- the sampler folds every recorded sample into per-chain
log-space partials (max of -ll, sum exp(-ll - max)); tiles are reduced on the device and
combined on the host (also across GPUs after an all-gather of tile partials).  Given a sample
array instead of a context, the reference's formula n / sum 1/exp(ll) in log space.

evidence_direct / evidence_lebesgue: the kD-tree integrals over a sample array, computed by
libmcg on the host (mcg_evidence.cpp).  A sample array is a Samples (records of N chains,
flattened chain after chain) or (pts (n, D), ll (n,), lp (n,)).
"""
import numpy as np

from . import _lib as L


def _flat(samples):
    if hasattr(samples, "value"):
        x = np.asarray(samples.value)                       # (n, D, N)
        pts = x.transpose(2, 0, 1).reshape(-1, x.shape[1])   # chain-major
        ll = np.asarray(samples.log_likelihood).T.reshape(-1)
        lp = np.asarray(samples.log_prior).T.reshape(-1)
    else:
        pts, ll, lp = samples
        pts = np.asarray(pts, np.float64)
        if pts.ndim == 1:
            pts = pts[:, None]
    return (np.ascontiguousarray(pts, np.float64), np.ascontiguousarray(ll, np.float64),
            np.ascontiguousarray(lp, np.float64))


def evidence_harmonic_mean(ctx_or_samples, naive=False):
    """n / sum_i exp(-ll_i) (evidence.ml:101-107).  naive=True (sample arrays only) runs the
    reference's linear-space loop itself, 1/exp(ll) summed in order, so it also reproduces its
    overflow (ll < -709: the sum is inf and Z = 0) and underflow (ll > 709: 1/inf = 0)."""
    if naive:
        if hasattr(ctx_or_samples, "stats"):
            raise ValueError("naive harmonic mean needs the sample array, not a context")
        _, ll, _ = _flat(ctx_or_samples)
        with np.errstate(over="ignore", divide="ignore"):
            inv = (1.0 / np.exp(ll)).tolist()           # elementwise, as the reference's loop body
        linv = 0.0
        for v in inv:                                   # sequential left fold, in sample order
            linv += v
        return float(len(ll)) / linv if linv != 0.0 else float("inf")
    return float(np.exp(log_evidence_harmonic_mean(ctx_or_samples)))


def log_evidence_harmonic_mean(ctx_or_samples):
    if hasattr(ctx_or_samples, "stats"):
        _, _, log_z = ctx_or_samples.stats()
        return log_z
    _, ll, _ = _flat(ctx_or_samples)
    m = np.max(-ll)
    return float(np.log(len(ll)) - (m + np.log(np.sum(np.exp(-ll - m)))))


def evidence_direct(samples, n=64):
    """Evidence.evidence_direct ?n samples (evidence.ml:145-156)."""
    pts, ll, lp = _flat(samples)
    out = np.zeros(1)
    rc = L.lib().mcg_evidence_direct(pts.shape[1], len(ll), L.dptr(pts), L.dptr(ll), L.dptr(lp), n, L.dptr(out))
    L.check(rc, None)
    return float(out[0])


def evidence_lebesgue(samples, n=64, eps=0.1):
    """Evidence.evidence_lebesgue ?n ?eps samples (evidence.ml:194-221)."""
    pts, ll, lp = _flat(samples)
    out = np.zeros(1)
    rc = L.lib().mcg_evidence_lebesgue(pts.shape[1], len(ll), L.dptr(pts), L.dptr(ll), L.dptr(lp), n, eps,
                                       L.dptr(out))
    L.check(rc, None)
    return float(out[0])


def posterior_moments(ctx):
    """Stats.multi_mean / Stats.multi_std (stats.ml:58-87) of the recorded samples."""
    mean, sd, _ = ctx.stats()
    return mean, sd
