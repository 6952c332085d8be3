"""Mirror of the reference's Mcmc module (mcmc.mli) over the HIP sampler.

Differences forced by the GPU boundary:
  * closures -> descriptors (mcmc_amd.targets);
  * `start` is a batch of chains, shape (D, N) (a (D,) vector is one chain);
  * counters are per Context instead of global (mcmc.ml:27-28).
"""
from dataclasses import dataclass

import numpy as np

from .context import Context

_default_ctx = None


def default_context():
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(seed=0)
    return _default_ctx


@dataclass
class Samples:
    """Array of mcmc_sample records (mcmc.ml:17-25) for N chains, structure-of-arrays."""
    value: np.ndarray            # (n, D, N)
    log_likelihood: np.ndarray   # (n, N)
    log_prior: np.ndarray        # (n, N)
    accept_bits: np.ndarray = None   # (nsteps, ceil(N/64)) uint64


def reset_counters(ctx=None):                     # mcmc.mli:29
    (ctx or default_context()).reset_counters()


def get_counters(ctx=None):                       # mcmc.mli:30
    return (ctx or default_context()).counters()


def mcmc_array(n, log_likelihood, log_prior, jump_proposal, start, nbin=0, nskip=1, ctx=None,
               record_accept=False):
    """Mcmc.mcmc_array ?nbin ?nskip n ll lp jump ljp start (mcmc.ml:58-72).

    log_jump_prob is implied by the proposal descriptor (0 for the symmetric ones,
    log jump_prob for KdInterp)."""
    ctx = ctx or default_context()
    ctx.set_model(log_likelihood, log_prior, jump_proposal)
    ctx.init(start)
    ctx.run(nbin=nbin, nskip=nskip, n_rec=n, record_x=True, record_llp=True,
            record_accept=record_accept, accumulate=True)
    x, ll, lp, bits = ctx.records(x=True, llp=True, accept=record_accept)
    return Samples(x, ll, lp, bits)


def make_mcmc_sampler(log_likelihood, log_prior, jump_proposal, ctx=None):
    """Mcmc.make_mcmc_sampler (mcmc.ml:37-56): returns step(state) -> next state for a batch.

    state = (x (D, N), ll (N,), lp (N,)); each call is one MH step of every chain on the device.
    Successive calls draw at successive Philox steps (the context's step counter is never
    rewound, as the reference's global Random state is not), and the accept / reject tallies
    add up across calls until reset_counters (mcmc.ml:27-35)."""
    ctx = ctx or default_context()
    ctx.set_model(log_likelihood, log_prior, jump_proposal)

    def step(state):
        x, ll, lp = state
        ctx.init(x, ll, lp)
        ctx.run(nbin=1, nskip=1, n_rec=0, record_x=False, record_llp=False)
        return ctx.state()

    return step


@dataclass
class RjSamples:
    """('a, 'b) rjmcmc_sample array (mcmc.ml:87) for N chains, structure-of-arrays: value is
    padded to max(ndim_A, ndim_B) (dims beyond the sample's model are 0)."""
    model: np.ndarray            # (n, N) uint8: 0 = A, 1 = B
    value: np.ndarray            # (n, Dmax, N)
    log_likelihood: np.ndarray   # (n, N)
    log_prior: np.ndarray        # (n, N) includes log p_model (mcmc.ml:116-118)
    counts: tuple = (0, 0)       # rjmcmc_model_counts over every recorded sample


def rjmcmc_array(n, model_a, model_b, start, nchains=1, nbin=0, nskip=1, ctx=None, models=None,
                 record_x=True):
    """Mcmc.rjmcmc_array ?nbin ?nskip n lls lps jps ljps jintos ljpintos (pa, pb) (a, b)
    (mcmc.ml:121-139) for `nchains` chains.  model_a / model_b are targets.RjModel descriptors
    (likelihood, prior, internal jump, jump into the model, model prior); start = (a, b) start
    points (a (D_A,) / (D_A, N) array, likewise b).  Each chain starts in A or B by a fair coin
    (mcmc.ml:123) unless models (N,) gives the start models."""
    import ctypes as C
    from . import _lib as L
    ctx = ctx or default_context()
    sa, sb = model_a.c_struct(), model_b.c_struct()
    ctx._keep = [model_a, model_b]
    L.check(L.lib().mcg_set_rjmcmc(ctx.ptr, C.byref(sa), C.byref(sb)), ctx.ptr)
    a, b = start
    xa = np.ascontiguousarray(np.broadcast_to(np.reshape(a, (model_a.ndim, -1)), (model_a.ndim, nchains)), np.float64)
    xb = np.ascontiguousarray(np.broadcast_to(np.reshape(b, (model_b.ndim, -1)), (model_b.ndim, nchains)), np.float64)
    tags = None if models is None else np.ascontiguousarray(models, np.uint8)
    L.check(L.lib().mcg_rj_init(ctx.ptr, nchains, L.u8ptr(tags), L.dptr(xa), L.dptr(xb)), ctx.ptr)
    ctx.ndim = max(model_a.ndim, model_b.ndim)
    ctx.nchains = nchains
    ctx.run(nbin=nbin, nskip=nskip, n_rec=n, record_x=record_x, record_llp=True, accumulate=True)
    x, ll, lp, _ = ctx.records(x=record_x, llp=True)
    rec_model = np.zeros((n, nchains), np.uint8)
    L.check(L.lib().mcg_rj_get_models(ctx.ptr, None, L.u8ptr(rec_model)), ctx.ptr)
    return RjSamples(rec_model, x, ll, lp, rjmcmc_model_counts(ctx))


def rjmcmc_model_counts(ctx_or_samples):
    """Mcmc.rjmcmc_model_counts (mcmc.ml:141-149): (#A, #B) over the recorded samples."""
    if isinstance(ctx_or_samples, RjSamples):
        nb = int(ctx_or_samples.model.sum())
        return ctx_or_samples.model.size - nb, nb
    from . import _lib as L
    na = np.zeros(1, np.uint64); nb = np.zeros(1, np.uint64)
    L.check(L.lib().mcg_rj_model_counts(ctx_or_samples.ptr, L.u64ptr(na), L.u64ptr(nb)), ctx_or_samples.ptr)
    return int(na[0]), int(nb[0])


def rjmcmc_evidence_ratio(samples):
    """Mcmc.rjmcmc_evidence_ratio (mcmc.ml:151-153): #A / #B."""
    na, nb = samples.counts if isinstance(samples, RjSamples) else rjmcmc_model_counts(samples)
    return float(na) / float(nb)


def remove_repeat_samples(samples, chain=0):
    """Mcmc.remove_repeat_samples (=) (mcmc.ml:74-82) on one chain of a Samples: keeps record 0
    and every record whose value differs from the previous one.  Returns (pts (m, D), ll, lp)."""
    x = np.asarray(samples.value)[:, :, chain]
    keep = np.ones(len(x), bool)
    keep[1:] = np.any(x[1:] != x[:-1], axis=1)
    return (x[keep].copy(), np.asarray(samples.log_likelihood)[keep, chain].copy(),
            np.asarray(samples.log_prior)[keep, chain].copy())
