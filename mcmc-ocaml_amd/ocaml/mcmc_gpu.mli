(* mcmc_gpu.mli -- OCaml binding of libmcg.so (include/mcg.h), the MI355X-native batched
   sampler behind farr/mcmc-ocaml's Mcmc / Nested / Evidence interfaces.

   Shipped as source: no OCaml toolchain exists in the build container (SURVEY.md §8c); the
   tested contract is the C-ABI (tests/test_abi.py, tests/test_gpu_*.py through ctypes).
   Requires the opam packages ctypes and ctypes-foreign (see INTEGRATION.md).

   Differences from the reference interface, forced by the GPU boundary:
   - closures become descriptors ([likelihood], [prior], [proposal]);
   - one call advances a whole batch of chains, coordinates are (D x N) Bigarrays;
   - counters live in a context ([ctx]) instead of globals (mcmc.ml:27-28). *)

type ctx

(** [create ?device ?seed ?chain_offset ()] -- the Philox key replaces Random.init. *)
val create : ?device:int -> ?seed:int64 -> ?chain_offset:int64 -> ?fixed_stop:bool -> unit -> ctx
val destroy : ctx -> unit

type mat = (float, Bigarray.float64_elt, Bigarray.c_layout) Bigarray.Array2.t
type vec = (float, Bigarray.float64_elt, Bigarray.c_layout) Bigarray.Array1.t

(** log_likelihood closures of mcmc.mli:58 as data *)
type likelihood =
  | Flat of int                                  (** ll = 0, ndim *)
  | Diag_gauss of float array * float array      (** Stats.log_multi_gaussian mu sigma *)
  | Fullcov_gauss of float array * float array array  (** mu, upper Cholesky factor of the precision *)
  | Gauss_shell of float array * float * float   (** centre, radius, width *)
  | Gauss_data of float array array              (** bin/gaussian_cauchy.ml log_like_gaussian *)
  | Cauchy_data of float array array             (** bin/gaussian_cauchy.ml log_like_cauchy *)

type prior =
  | Flat_prior
  | Box of float array * float array * float     (** lo, hi, log density inside (inclusive) *)
  | Open_box of float array * float array * float

type proposal =
  | Gauss of float array                         (** y = x + s N(0,1), symmetric *)
  | Uniform_wrapping of float array * float array * float array   (** Mcmc.uniform_wrapping *)
  | Interp of float array array * float array * float array        (** Interpolate_pdf.make *)

val set_model : ctx -> likelihood -> prior -> proposal option -> unit

(** Mcmc.reset_counters / get_counters (mcmc.mli:29-30) for this context. *)
val reset_counters : ctx -> unit
val get_counters : ctx -> int * int

(** Batched Mcmc.mcmc_array ?nbin ?nskip n (mcmc.mli:70-72): [start] is D x N; returns the
    records (n x D x N values, n x N log-likelihoods, n x N log-priors). *)
val mcmc_array :
  ?nbin:int -> ?nskip:int -> ctx -> int -> mat ->
  (float, Bigarray.float64_elt, Bigarray.c_layout) Bigarray.Genarray.t * mat * mat

(** On-device reductions of the last mcmc_array: Stats.multi_mean, Stats.multi_std and the
    log of Evidence.evidence_harmonic_mean (evidence.ml:101-107). *)
val stats : ctx -> float array * float array * float

(** Nested.nested_evidence (nested.mli:50-61) with the context's likelihood and box prior;
    [k] live points retired per generation (1 = the reference algorithm).  Returns the
    nested_output tuple: log Z, log dZ, points (n x D), log weights. *)
val nested_evidence :
  ?epsrel:float -> ?nmcmc:int -> ?nlive:int -> ?mode_hopping_frac:float -> ?k:int -> ctx ->
  float * float * float array array * float array

(** Nested.log_total_error_estimate (nested.mli:69). *)
val log_total_error_estimate : float -> float -> int -> float
