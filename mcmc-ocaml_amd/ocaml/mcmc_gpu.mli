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
  | Gauss_mix of float array array * float array array
      (** component means and sigmas: log of the sum of the components' log_multi_gaussian
          densities, the multimodal target of test/nested_test.ml:41-64 *)

type prior =
  | Flat_prior
  | Box of float array * float array * float     (** lo, hi, log density inside (inclusive) *)
  | Open_box of float array * float array * float
  | Gauss_prior of float array * float array
      (** mu, sigma: Stats.log_multi_gaussian mu sigma; nested sampling draws the live points
          with Stats.draw_gaussian per dim *)

(** components of Mcmc.combine_jump_proposals (mcmc.ml:165-185) *)
type mix_component =
  | Mix_gauss of float array                     (** x + s N(0,1) *)
  | Mix_shift_uniform of float array * float array   (** x + random_between a b (test/mcmc_test.ml) *)
  | Mix_wrap of float array * float array * float array   (** Mcmc.uniform_wrapping *)
  | Mix_interp                                   (** the mixture's kD tree (Interpolate_pdf.draw) *)

type proposal =
  | Gauss of float array                         (** y = x + s N(0,1), symmetric *)
  | Uniform_wrapping of float array * float array * float array   (** Mcmc.uniform_wrapping *)
  | Interp of float array array * float array * float array        (** Interpolate_pdf.make *)
  | Mixture of (float * mix_component * bool) list * (float array array * float array * float array) option
  (** combine_jump_proposals [(p, jump, density?)]: [density] = the component's log_jump_prob is
      its log density (else the constant 0 of a symmetric jump); the optional kD tree serves
      Mix_interp *)
  | De of float array array * float
  (** differential_evolution_proposal: the samples (M >= 2 rows of D), mode_hopping_frac *)

val set_model : ctx -> likelihood -> prior -> proposal option -> unit

(** Mcmc.differential_evolution_proposal ?mode_hopping_frac to_float from_float samples
    (mcmc.mli:215-218) over the samples' coordinates (log_jump_prob 0). *)
val differential_evolution_proposal : ?mode_hopping_frac:float -> float array array -> proposal

type state = mat * vec * vec
(** a batch of mcmc_sample records (mcmc.mli:33-42): values D x N, log-likelihoods, log-priors *)

(** Mcmc.make_mcmc_sampler (mcmc.mli:58-60) over a batch: sets the model on [ctx] and returns the
    step function; each call advances every chain of the state by one MH step (a rejected chain
    keeps its state, mcmc.ml:55) and continues the context's Philox stream.  Fed back the state
    it returned last, unmodified, with nothing else run on [ctx] in between (mcg_state_token), a
    step reuses the device-resident chains; any other argument -- a new state, or the returned
    Bigarrays mutated in place -- is uploaded first. *)
val make_mcmc_sampler : ctx -> likelihood -> prior -> proposal -> (state -> state)

(** [make_mcmc_sampler] whose step also returns how many chains accepted (from the context's
    accept total: one mcg_get_counters round trip per step while the sampler owns the context). *)
val make_mcmc_step : ctx -> likelihood -> prior -> proposal -> (state -> state * int)

(** Mcmc.reset_counters / get_counters (mcmc.mli:29-30) for this context. *)
val reset_counters : ctx -> unit

(** Random.init: new Philox key and the step counter back to 0.  Without it the counter runs
    on across [mcmc_array] calls on one context, as the reference's global Random state does. *)
val reseed : ctx -> int64 -> unit
val get_counters : ctx -> int * int

(** Batched Mcmc.mcmc_array ?nbin ?nskip n (mcmc.mli:70-72): [start] is D x N; returns the
    records (n x D x N values, n x N log-likelihoods, n x N log-priors). *)
val mcmc_array :
  ?nbin:int -> ?nskip:int -> ctx -> int -> mat ->
  (float, Bigarray.float64_elt, Bigarray.c_layout) Bigarray.Genarray.t * mat * mat

(** On-device reductions of the last mcmc_array: Stats.multi_mean, Stats.multi_std and the
    log of Evidence.evidence_harmonic_mean (evidence.ml:101-107). *)
val stats : ctx -> float array * float array * float

(** Nested.nested_evidence (nested.mli:50-61) with the context's likelihood and its box or Gauss_prior prior;
    [k] live points retired per generation (1 = the reference algorithm).  Returns the
    nested_output tuple: log Z, log dZ, points (n x D), log weights. *)
val nested_evidence :
  ?observer:(float array * float * float -> unit) ->
  ?epsrel:float -> ?nmcmc:int -> ?nlive:int -> ?mode_hopping_frac:float -> ?k:int -> ctx ->
  float * float * float array array * float array
(** [observer] (nested.mli:50) sees every retired point (value, log_likelihood, log_prior), in
    retirement order, after each generation of [k] retirements. *)

(** [nested_evidence] plus the log_likelihood and log_prior of every returned point (the
    like_prior halves of the reference's sample records). *)
val nested_run :
  ?observer:(float array * float * float -> unit) ->
  ?epsrel:float -> ?nmcmc:int -> ?nlive:int -> ?mode_hopping_frac:float -> ?k:int -> ctx ->
  (float * float * float array array * float array) * float array * float array

(** Nested.posterior_samples n output (nested.mli:77): n points drawn by weight on the device from
    the context's Philox stream (include/mcg.h mcg_posterior_samples). *)
val posterior_samples : ctx -> int -> float * float * float array array * float array -> float array array

(** Nested.log_total_error_estimate (nested.mli:69). *)
val log_total_error_estimate : float -> float -> int -> float

(** {2 Reversible jump (Mcmc.make_rjmcmc_sampler / rjmcmc_array, mcmc.ml:89-153)} *)
type rj_jump =
  | Rj_gauss of float array                      (** random walk, log_jump_prob 0 *)
  | Rj_wrap of float array * float array * float array
  | Rj_indep_gauss of float array * float array  (** independence draw N(mu, s) *)
  | Rj_interp                                    (** independence draw from the model's kD tree *)

type rj_model = {
  rj_lik : likelihood; rj_prior : prior; rj_jump : rj_jump; rj_into : rj_jump;
  rj_tree : (float array array * float array * float array) option; rj_model_prior : float }

(** [rjmcmc_array ctx n a b start_a start_b]: start_a is D_A x N, start_b D_B x N (the (a, b)
    pair per chain); each chain starts by a fair coin (mcmc.ml:123).  Returns the record model
    tags (n x N), values (n x Dmax x N, zero-padded), log-likelihoods and log-priors. *)
val rjmcmc_array :
  ?nbin:int -> ?nskip:int -> ctx -> int -> rj_model -> rj_model -> mat -> mat ->
  (int, Bigarray.int8_unsigned_elt, Bigarray.c_layout) Bigarray.Array2.t *
  (float, Bigarray.float64_elt, Bigarray.c_layout) Bigarray.Genarray.t * mat * mat

val rjmcmc_model_counts : ctx -> int * int
val rjmcmc_evidence_ratio : ctx -> float

(** {2 Evidence.evidence_direct / evidence_lebesgue (evidence.ml:145-221)} on samples
    (coordinates, log_likelihood, log_prior) *)
val evidence_direct : ?n:int -> (float array * float * float) array -> float
val evidence_lebesgue : ?n:int -> ?eps:float -> (float array * float * float) array -> float

(** {2 Nested replicas} merge runs [(ll in nested_output order, nlive, k)] into one run:
    (merged order, log Z, log dZ, log weights) *)
val nested_merge : (float array * int * int) list -> int array * float * float * float array

(** {2 Read_write (read_write.ml:19-101)} *)
val write_samples : string -> (float array * float * float) array -> unit
val read_samples : string -> (float array * float * float) array
val write_nested : string -> float * float * float array array * float array -> float array -> float array -> unit
val read_nested : string -> float * float * (float array * float * float) array * float array
