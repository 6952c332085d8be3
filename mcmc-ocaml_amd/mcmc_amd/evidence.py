"""Mirror of Evidence.Make(MO).evidence_harmonic_mean (evidence.ml:101-107).

On-device form: the sampler folds every recorded sample into per-chain log-space partials
(max of -ll, sum exp(-ll - max)); tiles are reduced on the device and combined on the host
(also across GPUs after an all-gather of tile partials).
"""
import numpy as np


def evidence_harmonic_mean(ctx):
    """n / sum_i exp(-ll_i) over the recorded samples of the context's last accumulate run."""
    _, _, log_z = ctx.stats()
    return float(np.exp(log_z))


def log_evidence_harmonic_mean(ctx):
    _, _, log_z = ctx.stats()
    return log_z


def posterior_moments(ctx):
    """Stats.multi_mean / Stats.multi_std (stats.ml:58-87) of the recorded samples."""
    mean, sd, _ = ctx.stats()
    return mean, sd
