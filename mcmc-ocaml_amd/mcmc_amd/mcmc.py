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

    state = (x (D, N), ll (N,), lp (N,)); each call is one MH step of every chain on the device."""
    ctx = ctx or default_context()
    ctx.set_model(log_likelihood, log_prior, jump_proposal)

    def step(state):
        x, ll, lp = state
        ctx.init(x, ll, lp)
        ctx.run(nbin=1, nskip=1, n_rec=0, record_x=False, record_llp=False)
        return ctx.state()

    return step
