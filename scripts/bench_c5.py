#!/usr/bin/env python3
"""C5 as BASELINE.json configs[4] names it: the D=64 full-covariance Gaussian, chains sharded
across GPUs (131,072 per GPU: 1,048,576 over 8), an RCCL all-gather of the tile partials for the
evidence / posterior-moment reductions.

  python scripts/bench_c5.py --gpus N [--steps K --warmup W --sweeps S]
  (or under python -m torch.distributed.run --nnodes=1 --nproc-per-node N ... --gpus N)

One process per GPU (RANK / LOCAL_RANK / WORLD_SIZE from the environment).  Rank r owns the
global chains [r*N, (r+1)*N) (chain_offset = r*N), so every chain's Philox stream and start point
depend on its global id only.  A bench step is one fused launch of S MH sweeps over every chain
of a rank.  The timed region is bracketed by a barrier + device sync on both sides and holds the
K steps plus the end-of-run reduction: tile kernel -> all-gather of the fixed 256-chain tile
partials -> every rank folds the tiles in global order (mcg_combine_tiles).  So the moments and
the harmonic-mean evidence are bit-identical for any number of ranks over the same global
chains (--total-chains fixes the global chain count: strong scaling; the default fixes the
per-GPU count: weak scaling).  Rank 0 prints one JSON line; `value` = every rank's MH steps /
the max over ranks of the timed region.

MCG_BENCH_BACKEND=gloo and MCG_BENCH_DEVICE=0 rehearse the flow with several ranks on one GPU.
"""
import argparse
import hashlib
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "mcmc-ocaml_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

HBM_PEAK_GBS = 8000.0
FP64_MATRIX_PEAK_TFS = 78.6      # MI355X FP64 matrix peak (MI355X_MICROARCH.md), dense
START_BLOCK = 8192               # start points drawn per block of global chain ids


def c5_target(D=64, seed=5):
    """Sigma = Q diag(lambda) Q^T, lambda log-uniform in [0.1, 10], Q from a seeded QR."""
    rng = np.random.default_rng(seed)
    Q, _ = np.linalg.qr(rng.normal(size=(D, D)))
    lam = np.exp(rng.uniform(math.log(0.1), math.log(10.0), D))
    cov = (Q * lam) @ Q.T
    cov = 0.5 * (cov + cov.T)
    mu = rng.uniform(-1, 1, D)
    s = 2.38 / math.sqrt(D) * math.sqrt(lam.min())
    return mu, cov, s


def start_points(mu, cov, g0, n):
    """Stationary starts of global chains [g0, g0 + n): block b of START_BLOCK chains comes from
    its own generator, so a chain's start does not depend on how the chains are sharded."""
    D = len(mu)
    Lc = np.linalg.cholesky(cov)
    x = np.empty((D, n))
    b0, b1 = g0 // START_BLOCK, (g0 + n - 1) // START_BLOCK
    for b in range(b0, b1 + 1):
        z = np.random.default_rng([5, b]).normal(size=(D, START_BLOCK))
        lo, hi = max(g0, b * START_BLOCK), min(g0 + n, (b + 1) * START_BLOCK)
        x[:, lo - g0:hi - g0] = mu[:, None] + Lc @ z[:, lo - b * START_BLOCK:hi - b * START_BLOCK]
    return x


def digest(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a, dtype=np.float64).tobytes())
    return h.hexdigest()[:16]


def cpu_baseline(mu, cov, s, seconds):
    """The oracle's full-covariance MH step (oracle/oracle.c, the restatement of mcmc.ml:37-56 with
    stats.ml's Gaussian in its precision-Cholesky form) on a bounded sample of the C5 target, on
    rank 0 only: bench.oracle_rate (cpu_threads() cores, median of 3).  Baseline only."""
    from bench import oracle_native, oracle_rate
    from mcmc_amd import targets as T
    O, build = oracle_native()
    D = len(mu)
    lik = T.fullcov_gauss(mu, cov)
    m = O.Model(D, lik.kind, lik.params, 0, (), 1, [s])
    Lc = np.linalg.cholesky(cov)
    rng = np.random.default_rng(7)
    return oracle_rate(O, m, lambda n: mu[:, None] + Lc @ rng.normal(size=(D, n)), seconds, build, "C5")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs (ranks); without WORLD_SIZE in the environment N > 1 launches N ranks")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--sweeps", type=int, default=500, help="MH sweeps per bench step (one launch)")
    ap.add_argument("--chains", type=int, default=131072, help="chains per GPU (weak scaling)")
    ap.add_argument("--total-chains", type=int, default=0,
                    help="global chain count split over the ranks (strong scaling; overrides --chains)")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--out", default=None, help="append the JSON line to this file")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=1.5,
                    help="wall seconds per repeat of the CPU baseline sample (rank 0)")
    args = ap.parse_args()

    sys.path.insert(0, ROOT)
    from bench import launch_ranks      # child torch.distributed.run before any GPU call
    rc = launch_ranks(args.gpus, os.path.abspath(__file__), sys.argv[1:])
    if rc is not None:
        sys.exit(rc)

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("MCG_BENCH_BACKEND", "nccl")
    if os.environ.get("MCG_BENCH_DEVICE"):
        local = int(os.environ["MCG_BENCH_DEVICE"])
    elif backend == "nccl" and world > torch.cuda.device_count():
        raise SystemExit("bench_c5: %d ranks over RCCL but only %d visible GPU(s)" % (world, torch.cuda.device_count()))
    dist = world > 1
    if dist:
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        tdist.init_process_group(backend)
    dev = torch.device("cuda", local)
    comm = dev if backend == "nccl" else None

    from mcmc_amd import Context, targets as T
    from mcmc_amd.parallel import reduce_stats

    D, S = 64, args.sweeps
    if args.total_chains:
        if args.total_chains % (world * 256):
            raise SystemExit("--total-chains must split into whole 256-chain tiles per rank")
        N = args.total_chains // world
        scaling = "strong"
    else:
        N = args.chains
        scaling = "weak"
    mu, cov, s = c5_target(D)
    ctx = Context(seed=args.seed, device=local, chain_offset=rank * N)
    ctx.set_model(T.fullcov_gauss(mu, cov), T.flat_prior(), T.gauss(s))
    ctx.init(start_points(mu, cov, rank * N, N))

    def barrier():
        ctx.sync()
        torch.cuda.synchronize(dev)
        if dist:
            tdist.barrier()
            torch.cuda.synchronize(dev)

    ctx.run(nbin=args.warmup * S, nskip=1, n_rec=1, record_x=False, record_llp=False,
            accumulate=True)
    ctx.set_timing(True)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.run(nbin=0, nskip=1, n_rec=S, record_x=False, record_llp=False, accumulate=True,
                append=True)
    mean, sd, log_z_hm = reduce_stats(D, ctx.tile_stats(), device=comm)
    barrier()
    elapsed = time.perf_counter() - t0
    elapsed_own = elapsed
    acc, rej = ctx.counters()
    timing = ctx.kernel_timing("mh")
    props = torch.cuda.get_device_properties(dev)
    me = {"rank": rank, "local_rank": local, "device": torch.cuda.current_device(),
          "pci_bus_id": getattr(props, "pci_bus_id", None), "uuid": str(getattr(props, "uuid", "")),
          "elapsed_s": elapsed_own, "avg_launch_ms": timing["total_ms"] / max(timing["launches"], 1),
          "launches": timing["launches"]}
    if dist:
        ranks = [None] * world
        tdist.all_gather_object(ranks, me)
    else:
        ranks = [me]
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=comm)
        tdist.all_reduce(tt, op=tdist.ReduceOp.MAX)
        elapsed = float(tt.item())
        cc = torch.tensor([acc, rej], dtype=torch.float64, device=comm)
        tdist.all_reduce(cc)
        acc, rej = (int(v) for v in cc.cpu().numpy())
    per_launch = timing["total_ms"] / max(timing["launches"], 1)
    # a bench step of S sweeps may run as several launches (the runtime caps a launch at
    # min(4096, 2^26 / N) sweeps): the framing uses the kernel time of all the timed launches
    kernel_ms_per_step = timing["total_ms"] / max(args.steps, 1)
    step_chain_steps = float(N) * S
    bytes_per_step = 8.0 * (D + 2)
    flops_per_step = 2.0 * D * (D + 1) / 2        # triangular quadratic form: D(D+1)/2 FMA
    ach_gbs = step_chain_steps * bytes_per_step / (kernel_ms_per_step * 1e-3) / 1e9
    ach_tfs = step_chain_steps * flops_per_step / (kernel_ms_per_step * 1e-3) / 1e12
    total_chains = N * world
    if rank == 0:
        from bench import rank_check
        rk = rank_check(ranks, world, backend, dist, tdist if dist else None)
        if dist and backend == "nccl" and not (rk["one_gpu_per_rank"] and rk["world_matches"]):
            raise SystemExit("bench_c5: %d ranks over RCCL drove %d distinct GPU(s): %s"
                             % (world, rk["distinct_gpus"], json.dumps(rk["per_rank"])))
        cpu = None if args.no_cpu_baseline else cpu_baseline(mu, cov, s, args.cpu_seconds)
        sdt = np.sqrt(np.diag(cov))
        line = {
            "metric": "C5 MH steps/s (whole job), D=64 full-covariance Gaussian",
            "value": float(total_chains) * S * args.steps / elapsed,
            "unit": "MH steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": scaling,
            "dtype": "f64",
            "data": "synthetic (Sigma = Q diag(lambda) Q^T, lambda log-U[0.1,10], seed 5; starts ~ target)",
            "config": {"workload": "C5 D=64 full-covariance Gaussian, %d chains over %d GPU(s) "
                                   "(%d per GPU), isotropic Gaussian proposal, %d MH sweeps per step, "
                                   "tile all-gather (%s) for moments + harmonic-mean evidence"
                                   % (total_chains, world, N, S, "RCCL" if backend == "nccl" else backend),
                       "ndim": D, "chains_total": total_chains, "chains_per_gpu": N,
                       "sweeps_per_step": S, "parallelism": "chains sharded, dp%d" % world,
                       "backend": backend},
            "roofline": {"bound": "hbm", "achieved": ach_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": ach_gbs / HBM_PEAK_GBS, "bytes_per_step": bytes_per_step,
                         "kernel": "mcg::mh_fullcov_kernel<64>", "avg_launch_ms": per_launch,
                         "launches": timing["launches"], "kernel_ms_per_step": kernel_ms_per_step,
                         "fp64_matrix": {"achieved": ach_tfs, "peak": FP64_MATRIX_PEAK_TFS,
                                         "unit": "TFLOP/s", "frac": ach_tfs / FP64_MATRIX_PEAK_TFS,
                                         "flops_per_step": flops_per_step}},
            "cpu_baseline": cpu,
            "ranks": rk,
            "accept_frac": acc / max(acc + rej, 1),
            "log_z_harmonic_mean": log_z_hm,
            "posterior_check": {"max_abs_mean_err_over_sd": float(np.max(np.abs(mean - mu) / sdt)),
                                "max_rel_sd_err": float(np.max(np.abs(sd / sdt - 1)))},
            "moments_digest": digest(mean, sd, [log_z_hm]),
        }
        s_line = json.dumps(line)
        print(s_line, flush=True)
        if args.out:
            with open(args.out, "a") as fh:
                fh.write(s_line + "\n")
    ctx.close()
    if dist:
        tdist.barrier()
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
