(* mcmc_gpu_compat.ml -- the reference's own record types over Mcmc_gpu, for dropping the GPU
   path in behind existing callers (INTEGRATION.md).  Compiled together with farr/mcmc-ocaml's
   Mcmc and Nested modules (mcmc.mli:33-42, nested.mli:21): every function returns
   [float array Mcmc.mcmc_sample] records, so a caller of Mcmc.mcmc_array / make_mcmc_sampler /
   Nested.nested_evidence / posterior_samples changes only its closures into descriptors.

   One chain here is one lane of the batched sampler: [mcmc_array] runs a batch of one chain
   (or, with [~chains], many chains whose records are concatenated chain after chain). *)

open Bigarray

let default_ctx = lazy (Mcmc_gpu.create ())

let sample v ll lp = { Mcmc.value = v; like_prior = { Mcmc.log_likelihood = ll; log_prior = lp } }

let column (x : Mcmc_gpu.mat) j = Array.init (Array2.dim1 x) (fun d -> x.{d, j})

(* Mcmc.reset_counters / get_counters (mcmc.mli:29-30) on the default context *)
let reset_counters () = Mcmc_gpu.reset_counters (Lazy.force default_ctx)
let get_counters () = Mcmc_gpu.get_counters (Lazy.force default_ctx)

(* Mcmc.make_mcmc_sampler (mcmc.mli:58-60) with descriptors for the four closures: a function of
   one sample returning the next; a rejected step returns the same physical record (mcmc.ml:55),
   decided by the step's accept count (Mcmc_gpu.get_counters before / after), not by comparing
   values.  Fed back its own last result (the usual loop) with its value array unmodified, the
   step reuses the device-resident chain (Mcmc_gpu.make_mcmc_sampler checks the context's state
   token and its own snapshot too) instead of uploading the record again. *)
let make_mcmc_sampler ?ctx lik pri prop =
  let ctx = match ctx with Some c -> c | None -> Lazy.force default_ctx in
  let step = Mcmc_gpu.make_mcmc_step ctx lik pri prop in
  let last = ref None in
  fun (s : float array Mcmc.mcmc_sample) ->
    let state = match !last with
      | Some (r, v0, st) when r == s && s.Mcmc.value = v0 -> st
      | _ ->
        let d = Array.length s.Mcmc.value in
        let x = Array2.create float64 c_layout d 1 in
        Array.iteri (fun i v -> x.{i, 0} <- v) s.Mcmc.value;
        (x, Array1.of_array float64 c_layout [| s.Mcmc.like_prior.Mcmc.log_likelihood |],
         Array1.of_array float64 c_layout [| s.Mcmc.like_prior.Mcmc.log_prior |]) in
    let ((x', ll', lp') as st', nacc) = step state in
    (* a rejected step returns the same record (mcmc.ml:53-56): decided by the step's accept
       count (one counter read per step, Mcmc_gpu.make_mcmc_step), not by comparing values *)
    let r = if nacc = 0 then s else sample (column x' 0) ll'.{0} lp'.{0} in
    last := Some (r, Array.copy r.Mcmc.value, st');
    r

(* Mcmc.mcmc_array ?nbin ?nskip n ... start (mcmc.mli:70-72): [chains] copies of [start] run
   side by side; their records come back chain after chain (n per chain) *)
let mcmc_array ?ctx ?(nbin = 0) ?(nskip = 1) ?(chains = 1) n lik pri prop (start : float array) :
    float array Mcmc.mcmc_sample array =
  let ctx = match ctx with Some c -> c | None -> Lazy.force default_ctx in
  Mcmc_gpu.set_model ctx lik pri (Some prop);
  let d = Array.length start in
  let x0 = Array2.create float64 c_layout d chains in
  for c = 0 to chains - 1 do Array.iteri (fun i v -> x0.{i, c} <- v) start done;
  let (xs, ll, lp) = Mcmc_gpu.mcmc_array ~nbin ~nskip ctx n x0 in
  Array.init (n * chains) (fun k ->
      let c = k / n and r = k mod n in
      sample (Array.init d (fun i -> Genarray.get xs [| r; i; c |])) ll.{r, c} lp.{r, c})

(* Nested.nested_evidence ?observer ?epsrel ?nmcmc ?nlive ?mode_hopping_frac (nested.mli:50-61)
   with the likelihood descriptor and a box prior (draw_prior = uniform in the box) or a
   Gauss_prior (draw_prior = Stats.draw_gaussian per dim, log_prior = Stats.log_multi_gaussian) *)
let nested_evidence ?ctx ?observer ?epsrel ?nmcmc ?nlive ?mode_hopping_frac ?k lik pri :
    float array Nested.nested_output =
  let ctx = match ctx with Some c -> c | None -> Lazy.force default_ctx in
  Mcmc_gpu.set_model ctx lik pri None;
  let observer = match observer with
    | None -> None
    | Some f -> Some (fun (v, ll, lp) -> f (sample v ll lp)) in
  let ((log_ev, log_dev, pts, wts), ll, lp) =
    Mcmc_gpu.nested_run ?observer ?epsrel ?nmcmc ?nlive ?mode_hopping_frac ?k ctx in
  (log_ev, log_dev, Array.mapi (fun i v -> sample v ll.(i) lp.(i)) pts, wts)

(* Nested.log_total_error_estimate (nested.mli:69) *)
let log_total_error_estimate = Mcmc_gpu.log_total_error_estimate

(* Nested.posterior_samples n output (nested.mli:77) *)
let posterior_samples ?ctx n ((log_ev, log_dev, samples, wts) : float array Nested.nested_output) :
    float array Mcmc.mcmc_sample array =
  let ctx = match ctx with Some c -> c | None -> Lazy.force default_ctx in
  let idx_src = Array.mapi (fun i _ -> [| float i |]) samples in
  let picked = Mcmc_gpu.posterior_samples ctx n (log_ev, log_dev, idx_src, wts) in
  Array.map (fun a -> samples.(int_of_float a.(0))) picked

(* Mcmc.differential_evolution_proposal ?mode_hopping_frac to_float from_float samples
   (mcmc.mli:215-218) over records *)
let differential_evolution_proposal ?mode_hopping_frac (samples : float array Mcmc.mcmc_sample array) =
  Mcmc_gpu.differential_evolution_proposal ?mode_hopping_frac (Array.map (fun s -> s.Mcmc.value) samples)
