(* mcmc_gpu.ml -- ctypes-foreign binding of libmcg.so (see mcmc_gpu.mli, INTEGRATION.md). *)
open Ctypes
open Foreign

let lib = Dl.dlopen ~filename:"libmcg.so" ~flags:[Dl.RTLD_NOW]
let fn name typ = foreign ~from:lib name typ

type ctx = unit ptr

(* mcg_opts (include/mcg.h) *)
type opts
let opts : opts structure typ = structure "mcg_opts"
let o_device = field opts "device" int32_t
let o_flags = field opts "flags" uint32_t
let o_seed = field opts "seed" uint64_t
let o_chain_offset = field opts "chain_offset" uint64_t
let o_lanes = field opts "lanes_per_chain" int32_t
let o_spl = field opts "steps_per_launch" int32_t
let () = seal opts

type run_opts
let run_opts : run_opts structure typ = structure "mcg_run_opts"
let r_nbin = field run_opts "nbin" int64_t
let r_nskip = field run_opts "nskip" int64_t
let r_nrec = field run_opts "n_rec" int64_t
let r_rx = field run_opts "record_x" int32_t
let r_rllp = field run_opts "record_llp" int32_t
let r_racc = field run_opts "record_accept" int32_t
let r_accum = field run_opts "accumulate" int32_t
let r_append = field run_opts "append" int32_t
let () = seal run_opts

type nested_opts
let nested_opts : nested_opts structure typ = structure "mcg_nested_opts"
let n_nlive = field nested_opts "nlive" int64_t
let n_nmcmc = field nested_opts "nmcmc" int64_t
let n_k = field nested_opts "k" int64_t
let n_epsrel = field nested_opts "epsrel" double
let n_mode_hop = field nested_opts "mode_hop" double
let n_max_dead = field nested_opts "max_dead" int64_t
let () = seal nested_opts

type nested_result
let nested_result : nested_result structure typ = structure "mcg_nested_result"
let nr_log_ev = field nested_result "log_ev" double
let nr_log_dev = field nested_result "log_dev" double
let nr_n_dead = field nested_result "n_dead" int64_t
let nr_n_total = field nested_result "n_total" int64_t
let nr_n_gen = field nested_result "n_gen" int64_t
let nr_converged = field nested_result "converged" int32_t
let () = seal nested_result

let c_ctx_create = fn "mcg_ctx_create" (ptr (ptr void) @-> ptr opts @-> returning int)
let c_ctx_destroy = fn "mcg_ctx_destroy" (ptr void @-> returning void)
let c_last_error = fn "mcg_last_error" (ptr void @-> returning string)
let c_set_likelihood = fn "mcg_set_likelihood" (ptr void @-> int32_t @-> int32_t @-> ptr double @-> size_t @-> returning int)
let c_set_prior = fn "mcg_set_prior" (ptr void @-> int32_t @-> ptr double @-> size_t @-> returning int)
let c_set_proposal = fn "mcg_set_proposal" (ptr void @-> int32_t @-> ptr double @-> size_t @-> returning int)
let c_set_kd = fn "mcg_set_kd_proposal" (ptr void @-> ptr double @-> int64_t @-> ptr double @-> ptr double @-> returning int)
let c_init = fn "mcg_init" (ptr void @-> int64_t @-> ptr double @-> ptr double @-> ptr double @-> returning int)
let c_run = fn "mcg_run" (ptr void @-> ptr run_opts @-> returning int)
let c_get_records = fn "mcg_get_records" (ptr void @-> ptr double @-> ptr double @-> ptr double @-> ptr uint64_t @-> returning int)
let c_get_counters = fn "mcg_get_counters" (ptr void @-> ptr uint64_t @-> ptr uint64_t @-> returning int)
let c_reset_counters = fn "mcg_reset_counters" (ptr void @-> returning int)
let c_reseed = fn "mcg_reseed" (ptr void @-> uint64_t @-> returning int)
let c_stats = fn "mcg_stats" (ptr void @-> ptr double @-> ptr double @-> ptr double @-> returning int)
let c_nested = fn "mcg_nested" (ptr void @-> ptr nested_opts @-> ptr nested_result @-> ptr void @-> ptr void @-> returning int)
let c_nested_get = fn "mcg_nested_get" (ptr void @-> ptr double @-> ptr double @-> ptr double @-> ptr double @-> returning int)
let c_log_total_error = fn "mcg_log_total_error_estimate" (double @-> double @-> int64_t @-> returning double)
let c_set_de = fn "mcg_set_de_proposal" (ptr void @-> ptr double @-> int64_t @-> double @-> returning int)
let c_get_state = fn "mcg_get_state" (ptr void @-> ptr double @-> ptr double @-> ptr double @-> returning int)
let c_state_token = fn "mcg_state_token" (ptr void @-> returning uint64_t)
let c_posterior = fn "mcg_posterior_samples" (ptr void @-> ptr double @-> int64_t @-> int64_t @-> ptr int64_t @-> returning int)
(* mcg_observer_fn: void (void* user, const double* pts, const double* ll, const double* lp, int64_t n) *)
let observer_t = ptr void @-> ptr double @-> ptr double @-> ptr double @-> int64_t @-> returning void
let c_nested_obs = fn "mcg_nested" (ptr void @-> ptr nested_opts @-> ptr nested_result @-> funptr observer_t @-> ptr void @-> returning int)

(* status codes -> the reference's exceptions (kd_tree.ml:70,97; nested.ml:71) *)
let check ctx rc =
  if rc <> 0 then begin
    let msg = c_last_error ctx in
    if rc = -1 then raise (Invalid_argument msg) else raise (Failure msg)
  end

type mat = (float, Bigarray.float64_elt, Bigarray.c_layout) Bigarray.Array2.t
type vec = (float, Bigarray.float64_elt, Bigarray.c_layout) Bigarray.Array1.t

type likelihood =
  | Flat of int
  | Diag_gauss of float array * float array
  | Fullcov_gauss of float array * float array array
  | Gauss_shell of float array * float * float
  | Gauss_data of float array array
  | Cauchy_data of float array array
  | Gauss_mix of float array array * float array array
      (* component means and sigmas: ll = log (sum_i exp (log_multi_gaussian mu_i sigma_i x)),
         test/nested_test.ml:52-57 *)

type prior =
  | Flat_prior
  | Box of float array * float array * float
  | Open_box of float array * float array * float
  | Gauss_prior of float array * float array
      (* mu, sigma: log_prior = Stats.log_multi_gaussian mu sigma, draw_prior =
         Stats.draw_gaussian per dim (stats.ml:98-124) *)

type mix_component =
  | Mix_gauss of float array
  | Mix_shift_uniform of float array * float array
  | Mix_wrap of float array * float array * float array
  | Mix_interp

type proposal =
  | Gauss of float array
  | Uniform_wrapping of float array * float array * float array
  | Interp of float array array * float array * float array
  | Mixture of (float * mix_component * bool) list * (float array array * float array * float array) option
  | De of float array array * float

let differential_evolution_proposal ?(mode_hopping_frac = 0.0) samples = De (samples, mode_hopping_frac)

let dims = Hashtbl.create 8

let create ?(device = 0) ?(seed = 0L) ?(chain_offset = 0L) ?(fixed_stop = false) () =
  let o = make opts in
  setf o o_device (Int32.of_int device);
  setf o o_flags (Unsigned.UInt32.of_int (if fixed_stop then 1 else 0));
  setf o o_seed (Unsigned.UInt64.of_int64 seed);
  setf o o_chain_offset (Unsigned.UInt64.of_int64 chain_offset);
  setf o o_lanes 0l;
  setf o o_spl 0l;
  let p = allocate (ptr void) null in
  let rc = c_ctx_create p (addr o) in
  if rc <> 0 then raise (Failure "mcg_ctx_create: no HIP device or libmcg.so unusable");
  !@p

let destroy ctx = c_ctx_destroy ctx

let carr a = CArray.start (CArray.of_list double (Array.to_list a))
let flatten m = Array.concat (Array.to_list m)

(* GAUSS_MIX parameters (include/mcg.h): m, then per component mu_i, sigma_i *)
let mix_params mus sigmas =
  let comps = Array.mapi (fun i mu -> Array.append mu sigmas.(i)) mus in
  Array.concat ([| float (Array.length mus) |] :: Array.to_list comps)

let set_model ctx lik pri prop =
  let kind, nd, params = match lik with
    | Flat d -> 0, d, [| 0.0 |]
    | Diag_gauss (mu, s) -> 1, Array.length mu, Array.append mu s
    | Fullcov_gauss (mu, u) -> 2, Array.length mu, Array.append mu (flatten u)
    | Gauss_shell (c, r, w) -> 3, Array.length c, Array.append c [| r; w |]
    | Gauss_data d -> 4, 2 * Array.length d.(0), Array.append [| float (Array.length d.(0)) |] (flatten d)
    | Cauchy_data d -> 5, 2 * Array.length d.(0), Array.append [| float (Array.length d.(0)) |] (flatten d)
    | Gauss_mix (mus, sigmas) -> 6, Array.length mus.(0), mix_params mus sigmas in
  check ctx (c_set_likelihood ctx (Int32.of_int kind) (Int32.of_int nd) (carr params)
               (Unsigned.Size_t.of_int (Array.length params)));
  Hashtbl.replace dims ctx nd;
  (match pri with
   | Flat_prior -> check ctx (c_set_prior ctx 0l (carr [| 0.0 |]) Unsigned.Size_t.zero)
   | Box (lo, hi, lp) | Open_box (lo, hi, lp) ->
     let k = match pri with Open_box _ -> 2l | _ -> 1l in
     let p = Array.concat [ lo; hi; [| lp |] ] in
     check ctx (c_set_prior ctx k (carr p) (Unsigned.Size_t.of_int (Array.length p)))
   | Gauss_prior (mu, sigma) ->
     let p = Array.append mu sigma in
     check ctx (c_set_prior ctx 3l (carr p) (Unsigned.Size_t.of_int (Array.length p))));
  match prop with
  | None -> ()
  | Some (Gauss s) -> check ctx (c_set_proposal ctx 1l (carr s) (Unsigned.Size_t.of_int (Array.length s)))
  | Some (Uniform_wrapping (lo, hi, dx)) ->
    let p = Array.concat [ lo; hi; dx ] in
    check ctx (c_set_proposal ctx 2l (carr p) (Unsigned.Size_t.of_int (Array.length p)))
  | Some (Interp (pts, lo, hi)) ->
    check ctx (c_set_kd ctx (carr (flatten pts)) (Int64.of_int (Array.length pts)) (carr lo) (carr hi))
  | Some (Mixture (comps, tree)) ->
    (* Mcmc.combine_jump_proposals (mcmc.ml:165-185): ncomp, then p, kind, ljp mode, params *)
    (match tree with
     | Some (pts, lo, hi) ->
       check ctx (c_set_kd ctx (carr (flatten pts)) (Int64.of_int (Array.length pts)) (carr lo) (carr hi))
     | None -> ());
    let comp (p, c, density) =
      let m = if density then 1.0 else 0.0 in
      match c with
      | Mix_gauss s -> Array.append [| p; 1.0; m |] s
      | Mix_shift_uniform (a, b) -> Array.concat [ [| p; 2.0; m |]; a; b ]
      | Mix_wrap (lo, hi, dx) -> Array.concat [ [| p; 3.0; 0.0 |]; lo; hi; dx ]
      | Mix_interp -> [| p; 4.0; 1.0 |] in
    let params = Array.concat ([| float (List.length comps) |] :: List.map comp comps) in
    check ctx (c_set_proposal ctx 5l (carr params) (Unsigned.Size_t.of_int (Array.length params)))
  | Some (De (samples, mh)) ->
    (* Mcmc.differential_evolution_proposal (mcmc.ml:198-218): samples kept in HBM *)
    check ctx (c_set_de ctx (carr (flatten samples)) (Int64.of_int (Array.length samples)) mh)

type state = mat * vec * vec

let get_counters ctx =
  let a = allocate uint64_t Unsigned.UInt64.zero and r = allocate uint64_t Unsigned.UInt64.zero in
  check ctx (c_get_counters ctx a r);
  (Unsigned.UInt64.to_int !@a, Unsigned.UInt64.to_int !@r)

(* Mcmc.make_mcmc_sampler (mcmc.ml:37-56) over a batch of chains: one MH step per call.  The
   chains stay on the device between calls: the step runs from the device copy (mcg_run +
   mcg_get_state, no mcg_init upload) only when all of these hold -- the argument is the state
   this sampler returned last (physically), its contents still equal the sampler's private
   snapshot of it (a caller may mutate the returned Bigarrays in place), and the context's state
   token (mcg_state_token) is the one seen right after that step (no other sampler, mcmc_array,
   nested run, model change or reset_counters used the context in between).  Otherwise the state
   is uploaded, and when the token moved the sampler first sets its own model again, so it never
   steps under another sampler's target.  [count]: also the number of accepted chains of the
   step, from the context's accept total -- read once per step (after it), the total before it
   being the one this sampler read after its own last step while the token is unchanged. *)
let make_core ~count ctx lik pri prop =
  set_model ctx lik pri (Some prop);
  let last = ref None in
  let tok_mine = ref (c_state_token ctx) in     (* the token right after this sampler's last use *)
  let acc_mine = ref None in                    (* the accept total read then *)
  let copy2 (a : mat) = let b = Bigarray.Array2.create Bigarray.float64 Bigarray.c_layout
                                (Bigarray.Array2.dim1 a) (Bigarray.Array2.dim2 a) in
    Bigarray.Array2.blit a b; b in
  let copy1 (a : vec) = let b = Bigarray.Array1.create Bigarray.float64 Bigarray.c_layout
                                (Bigarray.Array1.dim a) in
    Bigarray.Array1.blit a b; b in
  fun ((x : mat), (ll : vec), (lp : vec)) ->
    let d = Bigarray.Array2.dim1 x and nch = Bigarray.Array2.dim2 x in
    let ours = Unsigned.UInt64.equal !tok_mine (c_state_token ctx) in
    if not ours then set_model ctx lik pri (Some prop);
    let resident = ours && match !last with
      | Some ((x0, ll0, lp0), (sx, sll, slp), _) ->
        x == x0 && ll == ll0 && lp == lp0
        && x = sx && ll = sll && lp = slp
      | None -> false in
    if not resident then
      check ctx (c_init ctx (Int64.of_int nch) (bigarray_start array2 x) (bigarray_start array1 ll)
                   (bigarray_start array1 lp));
    let acc0 = if not count then 0 else match !acc_mine with
      | Some a when ours -> a
      | _ -> fst (get_counters ctx) in
    let o = make run_opts in
    setf o r_nbin 1L; setf o r_nskip 1L; setf o r_nrec 0L;
    setf o r_rx 0l; setf o r_rllp 0l; setf o r_racc 0l; setf o r_accum 0l; setf o r_append 0l;
    check ctx (c_run ctx (addr o));
    let open Bigarray in
    let x' = Array2.create float64 c_layout d nch in
    let ll' = Array1.create float64 c_layout nch and lp' = Array1.create float64 c_layout nch in
    check ctx (c_get_state ctx (bigarray_start array2 x') (bigarray_start array1 ll') (bigarray_start array1 lp'));
    let acc1 = if count then fst (get_counters ctx) else 0 in
    acc_mine := Some acc1;
    last := Some ((x', ll', lp'), (copy2 x', copy1 ll', copy1 lp'), c_state_token ctx);
    tok_mine := c_state_token ctx;
    ((x', ll', lp'), acc1 - acc0)

let make_mcmc_sampler ctx lik pri prop =
  let step = make_core ~count:false ctx lik pri prop in
  fun st -> fst (step st)

let make_mcmc_step ctx lik pri prop = make_core ~count:true ctx lik pri prop

let reset_counters ctx = check ctx (c_reset_counters ctx)

let reseed ctx seed = check ctx (c_reseed ctx (Unsigned.UInt64.of_int64 seed))

let bptr (b : (float, Bigarray.float64_elt, Bigarray.c_layout) Bigarray.Genarray.t) =
  bigarray_start genarray b

let mcmc_array ?(nbin = 0) ?(nskip = 1) ctx n (start : mat) =
  let d = Bigarray.Array2.dim1 start and nch = Bigarray.Array2.dim2 start in
  check ctx (c_init ctx (Int64.of_int nch) (bigarray_start array2 start)
               (from_voidp double null) (from_voidp double null));
  let o = make run_opts in
  setf o r_nbin (Int64.of_int nbin); setf o r_nskip (Int64.of_int nskip); setf o r_nrec (Int64.of_int n);
  setf o r_rx 1l; setf o r_rllp 1l; setf o r_racc 0l; setf o r_accum 1l; setf o r_append 0l;
  check ctx (c_run ctx (addr o));
  let open Bigarray in
  let xs = Genarray.create float64 c_layout [| n; d; nch |] in
  let ll = Array2.create float64 c_layout n nch and lp = Array2.create float64 c_layout n nch in
  check ctx (c_get_records ctx (bptr xs) (bigarray_start array2 ll) (bigarray_start array2 lp)
               (from_voidp uint64_t null));
  (xs, ll, lp)

let stats ctx =
  let d = Hashtbl.find dims ctx in
  let m = CArray.make double d and s = CArray.make double d and z = allocate double 0.0 in
  check ctx (c_stats ctx (CArray.start m) (CArray.start s) z);
  (Array.of_list (CArray.to_list m), Array.of_list (CArray.to_list s), !@z)

let nested_run ?observer ?(epsrel = 0.01) ?(nmcmc = 1000) ?(nlive = 1000) ?(mode_hopping_frac = 0.1)
    ?(k = 1) ctx =
  let d = Hashtbl.find dims ctx in
  let o = make nested_opts in
  setf o n_nlive (Int64.of_int nlive); setf o n_nmcmc (Int64.of_int nmcmc); setf o n_k (Int64.of_int k);
  setf o n_epsrel epsrel; setf o n_mode_hop mode_hopping_frac; setf o n_max_dead 0L;
  let r = make nested_result in
  (match observer with
   | None -> check ctx (c_nested ctx (addr o) (addr r) null null)
   | Some f ->
     (* the per-point ?observer of nested.ml:136, fed from libmcg's per-generation batches *)
     let cb _ pts ll lp n =
       for i = 0 to Int64.to_int n - 1 do
         f (Array.init d (fun j -> !@(pts +@ (i * d + j))), !@(ll +@ i), !@(lp +@ i))
       done in
     check ctx (c_nested_obs ctx (addr o) (addr r) cb null));
  if getf r nr_converged = 0l then
    prerr_endline "Mcmc_gpu.nested_evidence: max_dead cap reached before the stop test (unconverged)";
  let n = Int64.to_int (getf r nr_n_total) in
  let pts = CArray.make double (n * d) and ll = CArray.make double n
  and lp = CArray.make double n and w = CArray.make double n in
  check ctx (c_nested_get ctx (CArray.start pts) (CArray.start ll) (CArray.start lp) (CArray.start w));
  let pts = Array.init n (fun i -> Array.init d (fun j -> CArray.get pts (i * d + j))) in
  ((getf r nr_log_ev, getf r nr_log_dev, pts, Array.of_list (CArray.to_list w)),
   Array.of_list (CArray.to_list ll), Array.of_list (CArray.to_list lp))

let nested_evidence ?observer ?epsrel ?nmcmc ?nlive ?mode_hopping_frac ?k ctx =
  let (out, _, _) = nested_run ?observer ?epsrel ?nmcmc ?nlive ?mode_hopping_frac ?k ctx in
  out

let log_total_error_estimate log_ev log_dev nlive =
  c_log_total_error log_ev log_dev (Int64.of_int nlive)

(* Nested.posterior_samples (nested.ml:152-178): the draws on the device, the points picked here *)
let posterior_samples ctx n (_, _, (pts : float array array), (log_wts : float array)) =
  let npts = Array.length log_wts in
  assert (Array.length pts = npts);
  let idx = CArray.make int64_t (max n 1) in
  check ctx (c_posterior ctx (carr log_wts) (Int64.of_int npts) (Int64.of_int n) (CArray.start idx));
  Array.init n (fun i -> pts.(Int64.to_int (CArray.get idx i)))

(* ---- reversible jump (Mcmc.rjmcmc_array, mcmc.ml:121-139) ---- *)
type rj_jump =
  | Rj_gauss of float array
  | Rj_wrap of float array * float array * float array
  | Rj_indep_gauss of float array * float array
  | Rj_interp

type rj_model = {
  rj_lik : likelihood; rj_prior : prior; rj_jump : rj_jump; rj_into : rj_jump;
  rj_tree : (float array array * float array * float array) option; rj_model_prior : float }

type rj_model_s
let rj_model_s : rj_model_s structure typ = structure "mcg_rj_model"
let m_ndim = field rj_model_s "ndim" int32_t
let m_lik_kind = field rj_model_s "lik_kind" int32_t
let m_lik = field rj_model_s "lik_params" (ptr double)
let m_nlik = field rj_model_s "n_lik" size_t
let m_pri_kind = field rj_model_s "prior_kind" int32_t
let m_pri = field rj_model_s "prior_params" (ptr double)
let m_npri = field rj_model_s "n_prior" size_t
let m_jump_kind = field rj_model_s "jump_kind" int32_t
let m_jump = field rj_model_s "jump_params" (ptr double)
let m_njump = field rj_model_s "n_jump" size_t
let m_into_kind = field rj_model_s "into_kind" int32_t
let m_into = field rj_model_s "into_params" (ptr double)
let m_ninto = field rj_model_s "n_into" size_t
let m_kd_pts = field rj_model_s "kd_pts" (ptr double)
let m_kd_m = field rj_model_s "kd_M" int64_t
let m_kd_low = field rj_model_s "kd_low" (ptr double)
let m_kd_high = field rj_model_s "kd_high" (ptr double)
let m_p = field rj_model_s "model_prior" double
let () = seal rj_model_s

let c_set_rjmcmc = fn "mcg_set_rjmcmc" (ptr void @-> ptr rj_model_s @-> ptr rj_model_s @-> returning int)
let c_rj_init = fn "mcg_rj_init" (ptr void @-> int64_t @-> ptr uint8_t @-> ptr double @-> ptr double @-> returning int)
let c_rj_get_models = fn "mcg_rj_get_models" (ptr void @-> ptr uint8_t @-> ptr uint8_t @-> returning int)
let c_rj_counts = fn "mcg_rj_model_counts" (ptr void @-> ptr uint64_t @-> ptr uint64_t @-> returning int)

let lik_params = function
  | Flat d -> 0, d, [| 0.0 |]
  | Diag_gauss (mu, s) -> 1, Array.length mu, Array.append mu s
  | Fullcov_gauss (mu, u) -> 2, Array.length mu, Array.append mu (flatten u)
  | Gauss_shell (c, r, w) -> 3, Array.length c, Array.append c [| r; w |]
  | Gauss_data _ | Cauchy_data _ | Gauss_mix _ ->
    raise (Invalid_argument "rjmcmc: data and mixture likelihoods are not supported")

let rj_struct m =
  let s = make rj_model_s in
  let kind, nd, lp = lik_params m.rj_lik in
  let pk, pp = match m.rj_prior with
    | Flat_prior -> 0, [||]
    | Box (lo, hi, l) -> 1, Array.concat [ lo; hi; [| l |] ]
    | Open_box (lo, hi, l) -> 2, Array.concat [ lo; hi; [| l |] ]
    | Gauss_prior _ -> invalid_arg "Mcmc_gpu: reversible jump takes flat or box priors" in
  let jump = function
    | Rj_gauss sc -> 1, sc
    | Rj_wrap (lo, hi, dx) -> 2, Array.concat [ lo; hi; dx ]
    | Rj_indep_gauss (mu, sg) -> 3, Array.append mu sg
    | Rj_interp -> 4, [||] in
  let jk, jp = jump m.rj_jump and ik, ip = jump m.rj_into in
  let sz a = Unsigned.Size_t.of_int (Array.length a) in
  let arr a = if Array.length a = 0 then carr [| 0.0 |] else carr a in
  setf s m_ndim (Int32.of_int nd);
  setf s m_lik_kind (Int32.of_int kind); setf s m_lik (carr lp); setf s m_nlik (sz lp);
  setf s m_pri_kind (Int32.of_int pk); setf s m_pri (arr pp); setf s m_npri (sz pp);
  setf s m_jump_kind (Int32.of_int jk); setf s m_jump (arr jp); setf s m_njump (sz jp);
  setf s m_into_kind (Int32.of_int ik); setf s m_into (arr ip); setf s m_ninto (sz ip);
  (match m.rj_tree with
   | Some (pts, lo, hi) ->
     setf s m_kd_pts (carr (flatten pts)); setf s m_kd_m (Int64.of_int (Array.length pts));
     setf s m_kd_low (carr lo); setf s m_kd_high (carr hi)
   | None ->
     setf s m_kd_pts (from_voidp double null); setf s m_kd_m 0L;
     setf s m_kd_low (from_voidp double null); setf s m_kd_high (from_voidp double null));
  setf s m_p m.rj_model_prior;
  (s, nd)

let rjmcmc_array ?(nbin = 0) ?(nskip = 1) ctx n (ma : rj_model) (mb : rj_model) (a : mat) (b : mat) =
  let sa, da = rj_struct ma and sb, db = rj_struct mb in
  check ctx (c_set_rjmcmc ctx (addr sa) (addr sb));
  let nch = Bigarray.Array2.dim2 a in
  check ctx (c_rj_init ctx (Int64.of_int nch) (from_voidp uint8_t null) (bigarray_start array2 a)
               (bigarray_start array2 b));
  let dm = max da db in
  Hashtbl.replace dims ctx dm;
  let o = make run_opts in
  setf o r_nbin (Int64.of_int nbin); setf o r_nskip (Int64.of_int nskip); setf o r_nrec (Int64.of_int n);
  setf o r_rx 1l; setf o r_rllp 1l; setf o r_racc 0l; setf o r_accum 1l; setf o r_append 0l;
  check ctx (c_run ctx (addr o));
  let open Bigarray in
  let xs = Genarray.create float64 c_layout [| n; dm; nch |] in
  let ll = Array2.create float64 c_layout n nch and lp = Array2.create float64 c_layout n nch in
  let models = Array2.create int8_unsigned c_layout n nch in
  check ctx (c_get_records ctx (bptr xs) (bigarray_start array2 ll) (bigarray_start array2 lp)
               (from_voidp uint64_t null));
  check ctx (c_rj_get_models ctx (from_voidp uint8_t null) (bigarray_start array2 models));
  (models, xs, ll, lp)

(* Mcmc.rjmcmc_model_counts / rjmcmc_evidence_ratio (mcmc.ml:141-153) over the last run *)
let rjmcmc_model_counts ctx =
  let a = allocate uint64_t Unsigned.UInt64.zero and b = allocate uint64_t Unsigned.UInt64.zero in
  check ctx (c_rj_counts ctx a b);
  (Unsigned.UInt64.to_int !@a, Unsigned.UInt64.to_int !@b)

let rjmcmc_evidence_ratio ctx =
  let na, nb = rjmcmc_model_counts ctx in
  float na /. float nb

(* ---- Evidence.evidence_direct / evidence_lebesgue (evidence.ml:145-221) ---- *)
let c_ev_direct = fn "mcg_evidence_direct" (int32_t @-> int64_t @-> ptr double @-> ptr double @-> ptr double @-> int64_t @-> ptr double @-> returning int)
let c_ev_lebesgue = fn "mcg_evidence_lebesgue" (int32_t @-> int64_t @-> ptr double @-> ptr double @-> ptr double @-> int64_t @-> double @-> ptr double @-> returning int)

let sample_arrays (samples : (float array * float * float) array) =
  let n = Array.length samples in
  let d = let (v, _, _) = samples.(0) in Array.length v in
  let pts = carr (Array.concat (Array.to_list (Array.map (fun (v, _, _) -> v) samples))) in
  (n, d, pts, carr (Array.map (fun (_, l, _) -> l) samples), carr (Array.map (fun (_, _, p) -> p) samples))

let raise_rc rc = if rc = -1 then raise (Invalid_argument "evidence") else if rc <> 0 then raise (Failure "evidence")

let evidence_direct ?(n = 64) samples =
  let ns, d, pts, ll, lp = sample_arrays samples in
  let out = allocate double 0.0 in
  raise_rc (c_ev_direct (Int32.of_int d) (Int64.of_int ns) pts ll lp (Int64.of_int n) out);
  !@out

let evidence_lebesgue ?(n = 64) ?(eps = 0.1) samples =
  let ns, d, pts, ll, lp = sample_arrays samples in
  let out = allocate double 0.0 in
  raise_rc (c_ev_lebesgue (Int32.of_int d) (Int64.of_int ns) pts ll lp (Int64.of_int n) eps out);
  !@out

(* ---- nested replicas: merge runs (mcg_nested_merge) ---- *)
let c_nested_merge = fn "mcg_nested_merge" (int32_t @-> ptr int64_t @-> ptr int64_t @-> ptr int64_t @-> ptr double @-> ptr int64_t @-> ptr double @-> ptr double @-> ptr double @-> returning int)

(* runs: (log-likelihoods in nested_output order, nlive, k); returns (order, log Z, log dZ, log weights) *)
let nested_merge (runs : (float array * int * int) list) =
  let i64 l = CArray.start (CArray.of_list int64_t (List.map Int64.of_int l)) in
  let lls = Array.concat (List.map (fun (l, _, _) -> l) runs) in
  let n = Array.length lls in
  let order = CArray.make int64_t n and w = CArray.make double n in
  let le = allocate double 0.0 and ld = allocate double 0.0 in
  raise_rc (c_nested_merge (Int32.of_int (List.length runs))
              (i64 (List.map (fun (l, _, _) -> Array.length l) runs))
              (i64 (List.map (fun (_, nl, _) -> nl) runs)) (i64 (List.map (fun (_, _, k) -> k) runs))
              (carr lls) (CArray.start order) le ld (CArray.start w));
  (Array.of_list (List.map Int64.to_int (CArray.to_list order)), !@le, !@ld, Array.of_list (CArray.to_list w))

(* ---- Read_write text formats (read_write.ml:19-101) ---- *)
let c_write_rows = fn "mcg_write_rows" (string @-> int32_t @-> string_opt @-> int64_t @-> int32_t @-> ptr double @-> returning int)
let c_read_shape = fn "mcg_read_rows_shape" (string @-> int64_t @-> ptr int64_t @-> ptr int32_t @-> returning int)
let c_read_rows = fn "mcg_read_rows" (string @-> int64_t @-> int64_t @-> int32_t @-> ptr double @-> ptr double @-> int32_t @-> returning int)

let write_rows ?(append = false) ?header path (rows : float array array) =
  let nr = Array.length rows in
  let nc = if nr = 0 then 1 else Array.length rows.(0) in
  raise_rc (c_write_rows path (if append then 1l else 0l) header (Int64.of_int nr) (Int32.of_int nc)
              (carr (flatten rows)))

let read_rows ?(skip = 0) ?(nheader = 0) path =
  let nr = allocate int64_t 0L and nc = allocate int32_t 0l in
  raise_rc (c_read_shape path (Int64.of_int skip) nr nc);
  let nr = Int64.to_int !@nr and nc = Int32.to_int !@nc in
  let buf = CArray.make double (max 1 (nr * nc)) and hdr = CArray.make double (max 1 nheader) in
  raise_rc (c_read_rows path (Int64.of_int skip) (Int64.of_int nr) (Int32.of_int nc) (CArray.start buf)
              (if nheader > 0 then CArray.start hdr else from_voidp double null) (Int32.of_int nheader));
  (Array.init nr (fun i -> Array.init nc (fun j -> CArray.get buf (i * nc + j))),
   Array.init nheader (fun j -> CArray.get hdr j))

(* Read_write.write / read on (coords, log_likelihood, log_prior) samples *)
let write_samples path samples =
  write_rows path (Array.map (fun (v, l, p) -> Array.append v [| l; p |]) samples)

let read_samples path =
  let rows, _ = read_rows path in
  Array.map (fun r -> let d = Array.length r - 2 in (Array.sub r 0 d, r.(d), r.(d + 1))) rows

(* Read_write.write_nested / read_nested *)
let write_nested path (log_ev, log_dev, pts, wts) (ll : float array) (lp : float array) =
  let rows = Array.mapi (fun i v -> Array.append v [| ll.(i); lp.(i); wts.(i) |]) pts in
  write_rows ~header:(Printf.sprintf "%g %g\n" log_ev log_dev) path rows

let read_nested path =
  let rows, hdr = read_rows ~skip:1 ~nheader:2 path in
  let d = if Array.length rows = 0 then 0 else Array.length rows.(0) - 3 in
  (hdr.(0), hdr.(1), Array.map (fun r -> (Array.sub r 0 d, r.(d), r.(d + 1))) rows,
   Array.map (fun r -> r.(d + 2)) rows)
