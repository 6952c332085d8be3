(* example_gaussian.ml -- test/mcmc_test.ml:40-59 on the GPU: 65,536 chains of a 1-D Gaussian. *)
let () =
  let ctx = Mcmc_gpu.create ~seed:1L () in
  let mu = 0.37 and sigma = 1.6 in
  Mcmc_gpu.set_model ctx (Mcmc_gpu.Diag_gauss ([| mu |], [| sigma |])) Mcmc_gpu.Flat_prior
    (Some (Mcmc_gpu.Gauss [| 2.4 *. sigma |]));
  let n = 65536 in
  let start = Bigarray.Array2.create Bigarray.float64 Bigarray.c_layout 1 n in
  Bigarray.Array2.fill start mu;
  let _ = Mcmc_gpu.mcmc_array ~nbin:100 ctx 1000 start in
  let (m, s, _) = Mcmc_gpu.stats ctx in
  let (na, nr) = Mcmc_gpu.get_counters ctx in
  Printf.printf "mean %g (%g) std %g (%g) accept %g\n" m.(0) mu s.(0) sigma
    (float na /. float (na + nr));
  Mcmc_gpu.destroy ctx
