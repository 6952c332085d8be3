"""mcmc_amd -- MI355X-native batched MCMC / nested sampling behind farr/mcmc-ocaml's API.

Host-side mirror of the reference's OCaml modules (Mcmc, Nested, Evidence) over the C-ABI
library libmcg.so (include/mcg.h).  The reference takes OCaml closures; a GPU kernel cannot
call them, so log_likelihood / log_prior / jump_proposal are passed as data descriptors
(mcmc_amd.targets).  Every call runs the HIP kernels; there is no CPU fallback.
"""
from . import targets  # noqa: F401
from .context import Context  # noqa: F401
from . import mcmc, nested, evidence  # noqa: F401
