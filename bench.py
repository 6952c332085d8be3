#!/usr/bin/env python3
"""Headline benchmark: batched Metropolis-Hastings on the C2 workload of BASELINE.json.

  python bench.py [--gpus N --steps K --warmup W]   (N > 1: starts N ranks via a child
                                                   torch.distributed.run, or runs under one)

Workload (BASELINE.json configs[1]): D=32 diagonal-Gaussian log-target, isotropic Gaussian
proposal s = 2.38/sqrt(D) * median(sigma), flat box prior [-10, 10]^32, 65,536 independent chains
per GPU (weak scaling), starts drawn from the target.  One bench "step" = one fused kernel launch
of --sweeps MH sweeps over every chain (default 1,000: one launch at the runtime's own launch
length, which caps a launch at min(4096, 2^26/N) = 1,024 sweeps for 65,536 chains), so the default
--warmup 1 --steps 10 is the C2 job: nbin = 1,000 burn-in sweeps, then 10,000 recorded sweeps
whose samples are folded on the device into Welford moments and harmonic-mean partials.  (Each
launch also pays a fixed ~47 us: the chain state and accumulators round-trip through HBM; at 100
sweeps per launch that was 14 % of the launch, at 1,000 it is 1.7 %.  DESIGN.md §6.)  The timed region covers the K steps
plus the end-of-run reduction (tile kernel, RCCL all-gather of tile partials, host combine).
After it (outside `value`), the |delta log-evidence| half of the metric: Nested.nested_evidence on
the same target, one replica per GPU merged over the ranks (--nested-nlive per GPU).

Prints ONE JSON line (rank 0).  `value` = whole-job MH steps/s over all GPUs.
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(ROOT, "mcmc-ocaml_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

METRIC = "MH steps/s (whole node) + |Δlog-evidence|, D=32 Gaussian, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)


def c2_target(D, seed=42):
    rng = np.random.default_rng(seed)
    mu = rng.uniform(-1.0, 1.0, D)
    sg = rng.uniform(0.5, 2.0, D)
    s = 2.38 / math.sqrt(D) * float(np.median(sg))
    return mu, sg, s


def analytic_log_z(mu, sg, lo=-10.0, hi=10.0):
    """log Z = -D log(hi-lo) + sum_d log(Phi((hi-mu)/s) - Phi((lo-mu)/s))."""
    phi = lambda z: 0.5 * math.erfc(-z / math.sqrt(2.0))
    return sum(math.log(phi((hi - m) / s) - phi((lo - m) / s)) - math.log(hi - lo)
               for m, s in zip(mu, sg))


def cpu_baseline(args, mu, sg, s):
    """The oracle (C restatement of the reference's MH step) on a bounded sample of the same
    workload: every CPU this process may use (sched_getaffinity, capped at OMP_NUM_THREADS -- the
    GPU box grants 16 CPUs per GPU and exports OMP_NUM_THREADS=16, while its affinity mask shows
    the whole machine), built with -march=native on this host (oracle/Makefile `native`; the
    portable library otherwise), median of 3 timed repeats.  Baseline only."""
    D = args.ndim
    O, build = oracle_native()
    m = O.Model(D, 1, np.concatenate([mu, sg]), 1,
                np.concatenate([-10 * np.ones(D), 10 * np.ones(D), [-D * math.log(20.0)]]),
                1, [s])
    rng = np.random.default_rng(7)
    return oracle_rate(O, m, lambda n: rng.normal(mu[:, None], sg[:, None], size=(D, n)),
                       args.cpu_seconds, build, "C2")


def oracle_native():
    """The oracle library built with -march=native on this host (oracle/Makefile `native`), or the
    portable build if that fails.  Returns (oracle module, build description)."""
    import subprocess
    import oracle as O
    build = "-O3 -march=native (built on this host)"
    try:
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "native"], check=True,
                       capture_output=True, timeout=180)
        O.LIB_PATH = os.path.join(ROOT, "oracle", "_native", "liboracle.so")
    except (OSError, subprocess.SubprocessError) as e:
        build = "-O3 -march=x86-64-v3 (native build failed: %s)" % type(e).__name__
    return O, build


def oracle_rate(O, m, draw_x0, seconds, build, name):
    """MH steps/s of the oracle's batched sampler on model `m`: pthreads over chain blocks on
    cpu_threads() cores (64 x threads x 4 chains), a sample sized to ~`seconds` of wall time per
    repeat, median of 3; plus the single-core rate (256 chains, ~1 s)."""
    nproc = len(os.sched_getaffinity(0))
    threads = cpu_threads()
    D = m.ndim

    def run(nch, nsteps, nthreads):
        x0 = draw_x0(nch)
        ll = np.array([m.loglik(x0[:, i]) for i in range(nch)])
        lp = np.full(nch, m.logprior(x0[:, 0]))
        t = time.perf_counter()
        O.mh_run(m, 1, x0, ll, lp, nbin=nsteps, nskip=1, n_rec=1, record_x=False, record_llp=False,
                 record_accept=False, accumulate=False, nthreads=nthreads)
        return time.perf_counter() - t

    def median_rate(nch, nthreads, seconds):
        dt = run(nch, 20, nthreads)                       # size the sample
        nsteps = max(20, int(seconds * (nch * 20 / dt) / nch))
        rates = sorted(nch * nsteps / run(nch, nsteps, nthreads) for _ in range(3))
        return rates[1], nsteps, rates

    nch = 64 * threads * 4
    rate, nsteps, reps = median_rate(nch, threads, seconds)
    # one core: the single-threaded ocamlopt-equivalent proxy
    n1 = 256
    rate1, s1, reps1 = median_rate(n1, 1, 1.0)
    return dict(value=rate, unit="MH steps/s", cores=threads, kind="port", nproc=nproc,
                repeats=[float(r) for r in reps], statistic="median of 3",
                sample="%d chains x %d steps of the %s target per repeat (oracle/oracle.c, %s, %d threads "
                       "of %d in the affinity mask)" % (nch, nsteps, name, build, threads, nproc),
                single_core_value=rate1, single_core_repeats=[float(r) for r in reps1],
                single_core_sample="%d chains x %d steps, 1 thread, median of 3" % (n1, s1))


def pmc_traffic(D, N, S):
    """HBM bytes per launch of the dominant kernel from the committed PMC passes
    (profiles/pmc_traffic.json, written by scripts/pmc_traffic.py from scripts/gpu_profile.sh),
    when they were collected on this exact workload; else None."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as fh:
            t = json.load(fh)
    except (OSError, ValueError):
        return None
    if t.get("config") != {"ndim": D, "chains_per_gpu": N, "sweeps_per_step": S}:
        return None
    return t["traffic_bytes"]


def pmc_valu(D, N, S, avg_launch_ms):
    """VALU-issue framing of the dominant kernel (the bound that actually holds for the fused C2
    step: its HBM traffic is < 1 % of the algorithmic bytes) from the committed PMC pass
    (profiles/pmc_valu.json, scripts/pmc_valu.py): 4 SIMD cycles per wave64 VALU instruction over
    1,024 SIMDs, against the 2.4 GHz peak clock for this launch's live duration, and at the clock
    the chip held during the PMC pass (GRBM_GUI_ACTIVE)."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_valu.json")) as fh:
            v = json.load(fh)
    except (OSError, ValueError):
        return None
    if v.get("config") != {"ndim": D, "chains_per_gpu": N, "sweeps_per_step": S}:
        return None
    issue = 4.0 * v["valu_insts_per_launch"] / 1024.0        # SIMD cycles per SIMD
    return {"bound": "valu", "unit": "VALU issue cycles / SIMD cycles",
            "insts_per_launch": v["valu_insts_per_launch"],
            "insts_per_chain_step": v["valu_insts_per_chain_step"],
            "frac": issue / (2.4e9 * avg_launch_ms * 1e-3), "clock_ghz": 2.4,
            "frac_at_held_clock": v["valu_busy_frac_at_held_clock"],
            "source": "profiles/pmc_valu.json (rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE)"}


def launch_ranks(n, script, argv):
    """`--gpus N` without a launcher around us: start N ranks (one process per GPU) as a CHILD
    `python -m torch.distributed.run --nproc-per-node N ... script argv` and return its exit code.
    Called before anything imports torch or touches the GPU (a process that has initialised the
    GPU must not exec another program; here the parent never initialises it at all).  The ranks'
    stdout is inherited, so rank 0's one JSON line is the line this command prints.
    Returns None when no launch is needed (N = 1, or WORLD_SIZE already set by a launcher)."""
    import socket
    import subprocess
    world = os.environ.get("WORLD_SIZE")
    if world is not None:
        if int(world) != n:
            raise SystemExit("bench: --gpus %d but the launcher started WORLD_SIZE=%s ranks" % (n, world))
        return None
    if n <= 1:
        return None
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), script] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    # torch.distributed.run sets OMP_NUM_THREADS=1 in ranks when it is unset; rank 0's CPU
    # baseline keeps the thread count this process would have used at N = 1
    env.setdefault("MCG_CPU_THREADS", str(cpu_threads()))
    return subprocess.run(cmd, env=env).returncode


def cpu_threads():
    """CPUs this process may use: the affinity mask, capped at OMP_NUM_THREADS (the GPU box grants
    16 CPUs per GPU and exports OMP_NUM_THREADS=16, while its affinity mask shows the machine)."""
    nproc = len(os.sched_getaffinity(0))
    granted = int(os.environ.get("OMP_NUM_THREADS", nproc) or nproc)
    return int(os.environ.get("MCG_CPU_THREADS", min(nproc, granted)))


def launch_check(args):
    """--launch-check: the rank bring-up of the bench without the GPU work (CPU-testable).  Every
    rank joins the process group on `gloo`, rank 0 gathers (rank, local rank, world) and prints
    one JSON line with n_gpus = the world size."""
    import torch.distributed as tdist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        tdist.init_process_group("gloo")
        ranks = [None] * world
        tdist.all_gather_object(ranks, (rank, local, world))
    else:
        ranks = [(rank, local, world)]
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "gpus_arg": args.gpus,
                          "ranks": [list(r) for r in ranks], "cpu_threads": cpu_threads()}), flush=True)
    if world > 1:
        tdist.barrier()
        tdist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs (ranks); without WORLD_SIZE in the environment N > 1 launches N ranks")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--sweeps", type=int, default=1000, help="MH sweeps per bench step (one launch, <= 1024)")
    ap.add_argument("--chains", type=int, default=65536, help="chains per GPU")
    ap.add_argument("--ndim", type=int, default=32)
    ap.add_argument("--lanes", type=int, default=0, help="lanes per chain (0 = auto)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--nested-nlive", type=int, default=32768, help="live points per GPU (0 = skip)")
    ap.add_argument("--nested-k", type=int, default=2048)
    ap.add_argument("--nested-nmcmc", type=int, default=200)
    ap.add_argument("--nested-seeds", type=int, default=8,
                    help="extra single-GPU nested runs per rank (own seeds) for the bias estimate")
    ap.add_argument("--cpu-seconds", type=float, default=1.5,
                    help="wall seconds of the CPU baseline sample (x threads = CPU work)")
    ap.add_argument("--launch-check", action="store_true",
                    help="bring the ranks up (gloo) and print the rank map; no GPU work")
    args = ap.parse_args()

    rc = launch_ranks(args.gpus, os.path.abspath(__file__), sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
    if args.launch_check:
        return launch_check(args)

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # MCG_BENCH_BACKEND=gloo rehearses the multi-rank flow with CPU collectives (e.g. several ranks
    # sharing one GPU: MCG_BENCH_DEVICE=0); the driver's runs use RCCL ("nccl"), one GPU per rank.
    # With RCCL the process group is up at N = 1 too (a one-rank group on an in-process store), so
    # the timed region's all-gather of the tile partials runs over RCCL at every N.
    backend = os.environ.get("MCG_BENCH_BACKEND", "nccl")
    dist = world > 1 or backend == "nccl"
    if os.environ.get("MCG_BENCH_DEVICE"):
        local = int(os.environ["MCG_BENCH_DEVICE"])
    elif backend == "nccl" and world > torch.cuda.device_count():
        # one GPU per rank: fewer visible GPUs than ranks would put two ranks on one card (or
        # fail inside RCCL); refuse before any GPU work
        raise SystemExit("bench: %d ranks over RCCL but only %d visible GPU(s)" % (world, torch.cuda.device_count()))
    if dist:
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        if world > 1:
            tdist.init_process_group(backend)
        else:
            tdist.init_process_group(backend, store=tdist.HashStore(), rank=0, world_size=1)
    dev = torch.device("cuda", local)
    comm = dev if backend == "nccl" else None      # device of the collectives' tensors

    from mcmc_amd import Context, targets as T
    from mcmc_amd.parallel import reduce_stats, reduce_stats_device

    D, N, S = args.ndim, args.chains, args.sweeps
    mu, sg, s = c2_target(D)
    lik, pri, prop = T.diag_gauss(mu, sg), T.box(-10 * np.ones(D), 10 * np.ones(D)), T.gauss(s)
    ctx = Context(seed=1, device=local, chain_offset=rank * N, lanes_per_chain=args.lanes)
    ctx.set_model(lik, pri, prop)
    x0 = np.random.default_rng(1000 + rank).normal(mu[:, None], sg[:, None], size=(D, N))
    ctx.init(x0)

    def barrier():
        ctx.sync()
        torch.cuda.synchronize(dev)
        if dist:
            tdist.barrier()
            torch.cuda.synchronize(dev)

    # warmup = burn-in (nbin = W*S sweeps); record 0 = post-burn-in state (mcmc.ml:66)
    ctx.run(nbin=args.warmup * S, nskip=1, n_rec=1, record_x=False, record_llp=False,
            record_accept=False, accumulate=True)
    ctx.set_timing(True)
    if dist:      # the communicator is created by its first collective: not inside the timed region
        tdist.all_reduce(torch.zeros(1, dtype=torch.float64, device=comm))
    if comm is not None:
        # the first all_gather_into_tensor of a process sets RCCL's gather path up (~1 ms at N = 1):
        # one untimed pass of the same end-of-run reduction, on the burn-in state
        reduce_stats_device(ctx, comm)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.run(nbin=0, nskip=1, n_rec=S, record_x=False, record_llp=False, record_accept=False,
                accumulate=True, append=True)
    # end-of-run reduction: tile kernel into a device buffer -> RCCL all-gather of the tile
    # partials (device to device) -> host combine; gloo rehearsals gather host tiles
    if comm is not None:
        mean, sd, log_z_hm = reduce_stats_device(ctx, comm)
    else:
        mean, sd, log_z_hm = reduce_stats(D, ctx.tile_stats(), device=comm)
    barrier()
    elapsed = time.perf_counter() - t0
    elapsed_own = elapsed
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=comm)
        tdist.all_reduce(tt, op=tdist.ReduceOp.MAX)
        elapsed = float(tt.item())
    timing = ctx.kernel_timing("mh")
    acc, rej = ctx.counters()
    # per-rank record for the line's self-check (gathered to rank 0): which GPU this rank drove,
    # its own elapsed time and mean launch time
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
    # |delta log-evidence| leg (outside the timed region and `value`): Nested.nested_evidence on
    # the same target, one replica of --nested-nlive live points per GPU merged over the ranks
    nest = None
    if args.nested_nlive > 0:
        from mcmc_amd.parallel import nested_evidence_replicas
        barrier()
        tn = time.perf_counter()
        out = nested_evidence_replicas(lik, pri, nlive=args.nested_nlive * world, nmcmc=args.nested_nmcmc,
                                       k=args.nested_k, mode_hopping_frac=0.1, seed=7, device=local,
                                       comm_device=comm if dist else None, points=False)
        barrier()
        wall = time.perf_counter() - tn
        w = np.exp(out[3])
        H = float(np.sum(w * out.ll) - out[0])
        nest = dict(log_z=out[0], sigma=math.sqrt(max(H, 0.0) / (args.nested_nlive * world)), H=H,
                    nlive=args.nested_nlive * world, k=args.nested_k, nmcmc=args.nested_nmcmc,
                    n_dead=int(out.n_dead), wall_s=wall,
                    constrained_steps_per_s=float(out.n_gen) * args.nested_k * args.nested_nmcmc / wall)
        # bias estimate: independent single-GPU runs on every rank (seeds distinct over ranks),
        # their deltas gathered on rank 0 -- one run's delta is a single draw of sd ~ sigma
        if args.nested_seeds > 0:
            from mcmc_amd import Context, nested as _nested
            deltas, sig1 = [], []
            for i in range(args.nested_seeds):
                with Context(seed=100 + rank * args.nested_seeds + i, device=local) as c:
                    o = _nested.nested_evidence(lik, pri, nlive=args.nested_nlive, nmcmc=args.nested_nmcmc,
                                                k=args.nested_k, mode_hopping_frac=0.1, ctx=c, points=False)
                h = float(np.sum(np.exp(o[3]) * o.ll) - o[0])
                deltas.append(o[0] - analytic_log_z(mu, sg))
                sig1.append(math.sqrt(max(h, 0.0) / args.nested_nlive))
            if dist:
                allr = [None] * world
                tdist.all_gather_object(allr, (deltas, sig1))
                deltas = [x for r in allr for x in r[0]]
                sig1 = [x for r in allr for x in r[1]]
            d = np.array(deltas)
            nest["seed_sweep"] = dict(
                runs=len(d), nlive=args.nested_nlive, mean_delta=float(d.mean()),
                stderr=float(d.std(ddof=1) / math.sqrt(len(d))) if len(d) > 1 else None,
                sd_delta=float(d.std(ddof=1)) if len(d) > 1 else None, sigma=float(np.mean(sig1)),
                frac_within_1sigma=float(np.mean(np.abs(d) <= np.array(sig1))))

    steps_total = float(N) * world * S * args.steps
    value = steps_total / elapsed
    bytes_per_step = 8.0 * (D + 2)                     # chain-state read
    per_launch = timing["total_ms"] / max(timing["launches"], 1)
    launch_steps = float(N) * S                        # one launch = S sweeps of this rank
    achieved = launch_steps * bytes_per_step / (per_launch * 1e-3) / 1e9
    lz_true = analytic_log_z(mu, sg)
    if rank != 0:
        if dist:
            tdist.barrier()
            tdist.destroy_process_group()
        return
    # rank 0 only, at every N (the other ranks wait in the final barrier)
    rk = rank_check(ranks, world, backend, dist, tdist if dist else None)
    if backend == "nccl" and not (rk["one_gpu_per_rank"] and rk["world_matches"]):
        raise SystemExit("bench: %d ranks over RCCL drove %d distinct GPU(s) (world %d): %s"
                         % (world, rk["distinct_gpus"], rk["rccl_world"], json.dumps(rk["per_rank"])))
    cpu = None if args.no_cpu_baseline else cpu_baseline(args, mu, sg, s)
    line = {
        "metric": METRIC,
        "value": value,
        "unit": "MH steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (C2 target: mu~U[-1,1], sigma~U[0.5,2], seed 42; starts ~ target)",
        "config": {"workload": "C2 D=%d diagonal-Gaussian, %d chains/GPU, isotropic Gaussian "
                               "proposal, box prior [-10,10]^D, %d MH sweeps per step (one fused launch), "
                               "on-device Welford moments + harmonic-mean evidence, RCCL all-gather"
                               % (D, N, S),
                   "ndim": D, "chains_per_gpu": N, "sweeps_per_step": S,
                   "lanes_per_chain": ctx_lanes(ctx), "parallelism": "chains sharded, dp%d" % world},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": pmc_traffic(D, N, S),
                     "traffic_unit": "HBM bytes per launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE)",
                     "algorithmic_bytes_per_launch": launch_steps * bytes_per_step,
                     "kernel": "mcg::mh_kernel<32,P,DIAG_GAUSS,GAUSS>",
                     "bytes_per_step": bytes_per_step, "avg_launch_ms": per_launch,
                     "launches": timing["launches"],
                     "timing_source": "HIP events recorded on the context's stream around each of the "
                                      "K timed mh_kernel launches (mcg_kernel_timing), averaged",
                     "valu": pmc_valu(D, N, S, per_launch)},
        "cpu_baseline": cpu,
        "ranks": rk,
        "accept_frac": acc / max(acc + rej, 1),
        "log_evidence": log_evidence_line(nest, log_z_hm, lz_true),
        "posterior_check": {"max_abs_mean_err": float(np.max(np.abs(mean - mu))),
                            "max_rel_sd_err": float(np.max(np.abs(sd / sg - 1)))},
    }
    print(json.dumps(line), flush=True)
    if dist:
        tdist.barrier()
        tdist.destroy_process_group()


def rank_check(ranks, world, backend, dist, tdist):
    """The line's self-check of a multi-GPU run: the process group's own size and backend, each
    rank's GPU (ordinal, PCI bus, UUID), elapsed time and mean launch time, their spread, and
    whether every rank drove a GPU of its own (RCCL: one GPU per rank; a gloo rehearsal may share)."""
    el = [r["elapsed_s"] for r in ranks]
    lm = [r["avg_launch_ms"] for r in ranks]
    gpus = {(r["pci_bus_id"], r["uuid"], r["device"]) for r in ranks}
    return {"rccl_world": tdist.get_world_size() if dist else 1,
            "backend": tdist.get_backend() if dist else "none",
            "world_matches": (tdist.get_world_size() if dist else 1) == world == len(ranks),
            "distinct_gpus": len(gpus), "one_gpu_per_rank": len(gpus) == len(ranks),
            "per_rank": sorted(ranks, key=lambda r: r["rank"]),
            "elapsed_s_min": min(el), "elapsed_s_max": max(el),
            "avg_launch_ms_min": min(lm), "avg_launch_ms_max": max(lm),
            "launch_spread": max(lm) / min(lm) - 1.0 if min(lm) > 0 else None}


def log_evidence_line(nest, log_z_hm, lz_true):
    """|delta log Z| of the C2 target: nested sampling (the headline estimator) and the harmonic
    mean of the timed MH samples (evidence.ml:101-107; biased by ~D/2 nats at D = 32)."""
    line = {"analytic": lz_true, "harmonic_mean": log_z_hm, "harmonic_abs_delta": abs(log_z_hm - lz_true)}
    if nest is not None:
        d = abs(nest["log_z"] - lz_true)
        line.update({"estimator": "Nested.nested_evidence (nested.ml:122-146), replicas merged over GPUs",
                     "nested": nest["log_z"], "abs_delta": d, "sigma": nest["sigma"],
                     "within_1sigma": d <= nest["sigma"],
                     "nested_run": {k: nest[k] for k in ("nlive", "k", "nmcmc", "n_dead", "H", "wall_s",
                                                         "constrained_steps_per_s")}})
        if "seed_sweep" in nest:
            line["seed_sweep"] = nest["seed_sweep"]
    else:
        line.update({"estimator": "harmonic mean", "abs_delta": abs(log_z_hm - lz_true)})
    return line


def ctx_lanes(ctx):
    """Lanes per chain the timed launches used (the runtime's choice unless --lanes / env)."""
    return ctx.lanes()


if __name__ == "__main__":
    main()
