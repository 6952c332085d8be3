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
let c_stats = fn "mcg_stats" (ptr void @-> ptr double @-> ptr double @-> ptr double @-> returning int)
let c_nested = fn "mcg_nested" (ptr void @-> ptr nested_opts @-> ptr nested_result @-> ptr void @-> ptr void @-> returning int)
let c_nested_get = fn "mcg_nested_get" (ptr void @-> ptr double @-> ptr double @-> ptr double @-> ptr double @-> returning int)
let c_log_total_error = fn "mcg_log_total_error_estimate" (double @-> double @-> int64_t @-> returning double)

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

type prior =
  | Flat_prior
  | Box of float array * float array * float
  | Open_box of float array * float array * float

type proposal =
  | Gauss of float array
  | Uniform_wrapping of float array * float array * float array
  | Interp of float array array * float array * float array

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

let set_model ctx lik pri prop =
  let kind, nd, params = match lik with
    | Flat d -> 0, d, [| 0.0 |]
    | Diag_gauss (mu, s) -> 1, Array.length mu, Array.append mu s
    | Fullcov_gauss (mu, u) -> 2, Array.length mu, Array.append mu (flatten u)
    | Gauss_shell (c, r, w) -> 3, Array.length c, Array.append c [| r; w |]
    | Gauss_data d -> 4, 2 * Array.length d.(0), Array.append [| float (Array.length d.(0)) |] (flatten d)
    | Cauchy_data d -> 5, 2 * Array.length d.(0), Array.append [| float (Array.length d.(0)) |] (flatten d) in
  check ctx (c_set_likelihood ctx (Int32.of_int kind) (Int32.of_int nd) (carr params)
               (Unsigned.Size_t.of_int (Array.length params)));
  Hashtbl.replace dims ctx nd;
  (match pri with
   | Flat_prior -> check ctx (c_set_prior ctx 0l (carr [| 0.0 |]) Unsigned.Size_t.zero)
   | Box (lo, hi, lp) | Open_box (lo, hi, lp) ->
     let k = match pri with Open_box _ -> 2l | _ -> 1l in
     let p = Array.concat [ lo; hi; [| lp |] ] in
     check ctx (c_set_prior ctx k (carr p) (Unsigned.Size_t.of_int (Array.length p))));
  match prop with
  | None -> ()
  | Some (Gauss s) -> check ctx (c_set_proposal ctx 1l (carr s) (Unsigned.Size_t.of_int (Array.length s)))
  | Some (Uniform_wrapping (lo, hi, dx)) ->
    let p = Array.concat [ lo; hi; dx ] in
    check ctx (c_set_proposal ctx 2l (carr p) (Unsigned.Size_t.of_int (Array.length p)))
  | Some (Interp (pts, lo, hi)) ->
    check ctx (c_set_kd ctx (carr (flatten pts)) (Int64.of_int (Array.length pts)) (carr lo) (carr hi))

let reset_counters ctx = check ctx (c_reset_counters ctx)

let get_counters ctx =
  let a = allocate uint64_t Unsigned.UInt64.zero and r = allocate uint64_t Unsigned.UInt64.zero in
  check ctx (c_get_counters ctx a r);
  (Unsigned.UInt64.to_int !@a, Unsigned.UInt64.to_int !@r)

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

let nested_evidence ?(epsrel = 0.01) ?(nmcmc = 1000) ?(nlive = 1000) ?(mode_hopping_frac = 0.1)
    ?(k = 1) ctx =
  let d = Hashtbl.find dims ctx in
  let o = make nested_opts in
  setf o n_nlive (Int64.of_int nlive); setf o n_nmcmc (Int64.of_int nmcmc); setf o n_k (Int64.of_int k);
  setf o n_epsrel epsrel; setf o n_mode_hop mode_hopping_frac; setf o n_max_dead 0L;
  let r = make nested_result in
  check ctx (c_nested ctx (addr o) (addr r) null null);
  let n = Int64.to_int (getf r nr_n_total) in
  let pts = CArray.make double (n * d) and ll = CArray.make double n
  and lp = CArray.make double n and w = CArray.make double n in
  check ctx (c_nested_get ctx (CArray.start pts) (CArray.start ll) (CArray.start lp) (CArray.start w));
  let pts = Array.init n (fun i -> Array.init d (fun j -> CArray.get pts (i * d + j))) in
  (getf r nr_log_ev, getf r nr_log_dev, pts, Array.of_list (CArray.to_list w))

let log_total_error_estimate log_ev log_dev nlive =
  c_log_total_error log_ev log_dev (Int64.of_int nlive)
