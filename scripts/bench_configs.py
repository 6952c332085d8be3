#!/usr/bin/env python3
"""Measurement lines for the non-headline BASELINE.json configs (C1, C3, C4, C5) on one MI355X.

bench.py measures the headline C2 workload (the driver's contract). This script runs each of the
other configs once at full size and prints one JSON line per config. Each line carries:
  - throughput of the config's unit (MH steps/s or constrained nested steps/s);
  - the SURVEY.md §8(d) algorithmic-bytes roofline framing from HIP-event kernel times;
  - the config's correctness property (analytic log Z, posterior moments, C1 oracle parity).

  python scripts/bench_configs.py [c1 c3 c4 c5] [--out gpurun_out/configs.jsonl]
"""
import argparse
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

from mcmc_amd import Context, nested, targets as T  # noqa: E402

HBM_PEAK_GBS = 8000.0
# uniformly random rows of a table that fits the 256 MiB Infinity Cache, gathered chip-wide
# (MI355X_MICROARCH.md, "Indexed rows: gather into LDS", 38 MB table: 8.6 TB/s)
IC_GATHER_PEAK_GBS = 8600.0


def roofline(kernel, steps_per_launch, bytes_per_step, timing):
    per_launch = timing["total_ms"] / max(timing["launches"], 1)
    if per_launch <= 0:            # no timed launch (e.g. under a profiler's kernel filter)
        return {"bound": "hbm", "kernel": kernel, "avg_launch_ms": None, "launches": timing["launches"]}
    ach = steps_per_launch * bytes_per_step / (per_launch * 1e-3) / 1e9
    return {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": ach / HBM_PEAK_GBS, "kernel": kernel, "bytes_per_step": bytes_per_step,
            "avg_launch_ms": per_launch, "launches": timing["launches"]}


def hbm_secondary(r):
    """The SURVEY §8(d) algorithmic-bytes framing kept beside a config's real bound, labelled: its
    bytes are those of an unfused step, not what the kernel moves (frac > 1 is possible)."""
    r = dict(r)
    r["role"] = ("secondary: SURVEY 8(d) algorithmic bytes of an unfused step against HBM peak; "
                 "not the bound of this kernel")
    return r


def ic_gather(kernel, steps_per_launch, bytes_per_step, timing, pmc=None):
    """Infinity-Cache random-row framing: the partner rows a constrained step gathers (2 random
    rows of the live set, which fits the Infinity Cache and no XCD's L2) per launch / the launch
    time, against the guide's chip-wide random-row gather rate."""
    per_launch = timing["total_ms"] / max(timing["launches"], 1)
    if per_launch <= 0:
        return {"bound": "infinity_cache", "kernel": kernel, "avg_launch_ms": None}
    ach = steps_per_launch * bytes_per_step / (per_launch * 1e-3) / 1e9
    r = {"bound": "infinity_cache", "achieved": ach, "peak": IC_GATHER_PEAK_GBS, "unit": "GB/s",
         "frac": ach / IC_GATHER_PEAK_GBS, "kernel": kernel, "bytes_per_step": bytes_per_step,
         "bytes_note": "two random D x 8-B partner rows per constrained step (DE pair, nested.ml:53)",
         "peak_source": "MI355X_MICROARCH.md: 38 MB table, uniformly random rows, 8.6 TB/s chip-wide",
         "avg_launch_ms": per_launch, "launches": timing["launches"]}
    if pmc:
        r["counters"] = pmc
    return r


def c3_pmc(k, nmcmc):
    """TCC hit / miss and fabric-read counters of the C3 walk kernel (profiles/pmc_c3_walk.json,
    scripts/pmc_c3.py) when they were collected at this k and nmcmc."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_c3_walk.json")) as fh:
            v = json.load(fh)
    except (OSError, ValueError):
        return None
    return v if v.get("config") == {"k": k, "nmcmc": nmcmc} else None


def valu_framing(name, D, N, S, avg_launch_ms):
    """VALU-issue framing from a committed PMC pass of this config (profiles/pmc_valu_<name>.json,
    scripts/pmc_valu.py): 4 SIMD cycles per wave64 VALU instruction over 1,024 SIMDs, against the
    2.4 GHz peak for this run's launch time, and at the clock held in the PMC pass."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_valu_%s.json" % name)) as fh:
            v = json.load(fh)
    except (OSError, ValueError):
        return None
    if v.get("config") != {"ndim": D, "chains_per_gpu": N, "sweeps_per_step": S} or not avg_launch_ms:
        return None
    issue = 4.0 * v["valu_insts_per_launch"] / 1024.0
    return {"bound": "valu", "insts_per_launch": v["valu_insts_per_launch"],
            "frac": issue / (2.4e9 * avg_launch_ms * 1e-3), "clock_ghz": 2.4,
            "frac_at_held_clock": v["valu_busy_frac_at_held_clock"],
            "source": "profiles/pmc_valu_%s.json" % name}


F64_MFMA_PEAK_TFS = 78.6   # v_mfma_f64_16x16x4f64: 2,048 flop / 64 cycles / SIMD, 1,024 SIMDs, 2.4 GHz


def mfma_framing(D, steps, avg_launch_ms, valu=None):
    """The full-covariance step's f64 matrix-core framing (mh_fullcov_kernel): 16 chains per MFMA
    tile, the block lower-triangular L^-1 y as sum_{kb < D/4} (kb / 4 + 1) v_mfma_f64_16x16x4f64
    per 16 chain-steps (40 at D 64), against the measured f64 MFMA rate (64 cycles per MFMA per
    SIMD: 78.6 TFLOP/s, scripts/probes/mfma_f64_rate.hip).  achieved: the algorithmic D (D + 1)
    flop per step (triangular solve + squared norm); issued: the MFMA tiles' 2,048 flop each.
    f64 VALU work shares the datapath (scripts/probes/mfma_valu_overlap.hip), so the VALU framing
    rides along as the secondary bound."""
    if not avg_launch_ms:
        return None
    n_mfma = sum(kb // 4 + 1 for kb in range(D // 4))
    t = avg_launch_ms * 1e-3
    alg = steps * D * (D + 1) / t / 1e12
    issued = steps / 16.0 * n_mfma * 2048.0 / t / 1e12
    r = {"bound": "mfma", "achieved": alg, "peak": F64_MFMA_PEAK_TFS, "unit": "TFLOP/s", "frac": alg / F64_MFMA_PEAK_TFS,
         "issued": issued, "issued_frac": issued / F64_MFMA_PEAK_TFS, "mfma_per_16_steps": n_mfma,
         "flop_per_step": D * (D + 1), "peak_source": "measured f64 MFMA rate (64 cycles / MFMA / SIMD)",
         "avg_launch_ms": avg_launch_ms}
    if valu:
        r["valu_secondary"] = valu
        # f64 MFMA and f64 VALU share the datapath (scripts/probes/mfma_valu_overlap.hip: MFMA
        # waves keep 64 clocks per MFMA while a concurrent v_fma_f64 stream slows from 4.78 to
        # 12.79 clocks, i.e. keeps 0.374 of its rate).  Floor of a launch, per SIMD: the MFMA clocks
        # plus the VALU clocks that do not fit beside them (4 per wave64 VALU instruction, all
        # counted as f64); the plain sum is the no-overlap ceiling
        n_simd, clk, keep = 1024.0, 2.4e9, 4.78 / 12.79
        mfma_cyc = steps / 16.0 * n_mfma * 64.0 / n_simd
        valu_cyc = 4.0 * valu["insts_per_launch"] / n_simd
        floor = mfma_cyc + max(0.0, valu_cyc - keep * mfma_cyc)
        r["f64_datapath"] = {"mfma_clocks_per_simd": mfma_cyc, "valu_clocks_per_simd": valu_cyc,
                             "frac": floor / (clk * t), "frac_no_overlap": (mfma_cyc + valu_cyc) / (clk * t),
                             "valu_rate_kept_beside_mfma": keep, "clock_ghz": 2.4,
                             "source": "scripts/probes/mfma_valu_overlap.hip (profiles/r05/c5_datapath)"}
    return r


def shell_log_z(D, r, w, half):
    """Analytic log Z of one Gaussian shell in [-half, half]^D (radial quadrature; the shell
    lies well inside the box)."""
    rr = np.linspace(max(r - 12 * w, 0.0), r + 12 * w, 200001)
    lsurf = math.log(2.0) + (D / 2) * math.log(math.pi) - math.lgamma(D / 2)
    f = np.exp(-(rr - r) ** 2 / (2 * w * w) + (D - 1) * np.log(np.maximum(rr, 1e-300)) - (D - 1) * math.log(r))
    integ = np.trapezoid(f, rr)
    return (lsurf + (D - 1) * math.log(r) + math.log(integ) - math.log(math.sqrt(2 * math.pi) * w)
            - D * math.log(2 * half))


def c1(args):
    """bin/gaussian_cauchy.ml defaults: ndim 1, nsamp 10, nmcmc 100,000, single chain, seed 1."""
    import oracle as O
    rng = np.random.default_rng(1)
    nd, nsamp, nmcmc = 1, 10, 100000
    mus = rng.uniform(-1, 1, nd); sigmas = rng.uniform(0.1, 0.2, nd)
    data = rng.normal(mus, sigmas, size=(nsamp, nd))
    lo = np.concatenate([[-1.0] * nd, [0.1] * nd]); hi = np.concatenate([[1.0] * nd, [0.2] * nd])
    pri = T.box(lo, hi, -nd * (math.log(2.0) + math.log(0.1)))
    dx = np.concatenate([sigmas, sigmas]) / (math.sqrt(nsamp) * nd)
    prop = T.uniform_wrapping(lo, hi, dx)
    x0 = np.concatenate([mus, sigmas])[:, None]
    out = {}
    for name, lik in (("gaussian", T.gauss_data(data)), ("cauchy", T.cauchy_data(data))):
        ctx = Context(seed=1)
        ctx.set_model(lik, pri, prop)
        ctx.init(x0)
        ctx.set_timing(True)
        t0 = time.perf_counter()
        ctx.run(nbin=0, nskip=1, n_rec=nmcmc, record_x=False, record_llp=False, record_accept=True,
                accumulate=True)
        ctx.sync()
        dt = time.perf_counter() - t0
        _, _, _, bits = ctx.records(x=False, llp=False, accept=True)
        mean, sd, lz = ctx.stats()
        acc, rej = ctx.counters()
        m = O.Model(2 * nd, lik.kind, lik.params, pri.kind, pri.params, prop.kind, prop.params)
        ll0 = np.array([m.loglik(x0[:, 0])]); lp0 = np.array([m.logprior(x0[:, 0])])
        t1 = time.perf_counter()
        r = O.mh_run(m, 1, x0, ll0, lp0, nbin=0, nskip=1, n_rec=nmcmc, record_x=False,
                     record_llp=False, accumulate=True, nthreads=1)
        dto = time.perf_counter() - t1
        _, _, lzo = O.combine_tiles(2 * nd, O.tile_stats(2 * nd, 1, nmcmc, r))
        out[name] = {"steps_per_s": (nmcmc - 1) / dt, "accept_frac": acc / (acc + rej),
                     "log_z_harmonic_mean": lz, "bitmap_equal_oracle": bool(np.array_equal(bits, r["bits"])),
                     "log_z_equal_oracle": lz == lzo, "oracle_steps_per_s": (nmcmc - 1) / dto,
                     "posterior_mean": mean.tolist()}
        ctx.close()
    return {"config": "C1 bin/gaussian_cauchy.ml (ndim 1, nsamp 10, nmcmc 100000, single chain)",
            "unit": "MH steps/s", "dtype": "f64", "value": out["gaussian"]["steps_per_s"],
            "note": "single chain: latency-bound plumbing case (one lane of one wavefront)",
            "log_bayes_factor_gauss_vs_cauchy": out["gaussian"]["log_z_harmonic_mean"] - out["cauchy"]["log_z_harmonic_mean"],
            "runs": out}


def c3(args):
    """Nested.nested_evidence on the D=16 Gaussian shell (c=0, r=2, w=0.1, prior U[-6,6]^16),
    nlive 131,072, k 4,096, nmcmc 100, mode_hop 0.1, epsrel 0.01."""
    D, r, w, half = 16, 2.0, 0.1, 6.0
    nlive, k, nmcmc = args.nlive, args.k, args.nmcmc
    lik = T.gauss_shell(np.zeros(D), r, w)
    pri = T.box(-half * np.ones(D), half * np.ones(D))
    ctx = Context(seed=args.seed)
    # args.reps timed runs in one context after a warm-up run (the same seed: identical runs),
    # then one run with per-walk HIP events for the roofline
    # value: the run with its inputs and outputs in HBM (log Z, log dZ, weights and ll / lp come
    # back; the n x D dead points stay on the device); the full call that also copies the points
    # to the host (457 MB over PCIe at C3) is reported beside it
    walls, walls_pts = [], []
    # one untimed run first: the first call in a context allocates the live set, keys, draw tables
    # and dead buffers (~50 ms), which no later run pays
    out = nested.nested_evidence(lik, pri, epsrel=0.01, nmcmc=nmcmc, nlive=nlive, mode_hopping_frac=0.1,
                                 k=k, ctx=ctx, points=False)
    out = None
    for _ in range(max(1, args.reps)):
        out = None              # the previous run's arrays are freed outside the timed call (~25 ms)
        t0 = time.perf_counter()
        out = nested.nested_evidence(lik, pri, epsrel=0.01, nmcmc=nmcmc, nlive=nlive,
                                     mode_hopping_frac=0.1, k=k, ctx=ctx, points=False)
        walls.append(time.perf_counter() - t0)
    for _ in range(max(1, args.reps)):
        out = None
        t0 = time.perf_counter()
        out = nested.nested_evidence(lik, pri, epsrel=0.01, nmcmc=nmcmc, nlive=nlive,
                                     mode_hopping_frac=0.1, k=k, ctx=ctx)
        walls_pts.append(time.perf_counter() - t0)
    dt = float(np.median(walls))
    dt_pts = float(np.median(walls_pts))
    ctx.set_timing(True)
    nested.nested_evidence(lik, pri, epsrel=0.01, nmcmc=nmcmc, nlive=nlive, mode_hopping_frac=0.1, k=k, ctx=ctx)
    tw = ctx.kernel_timing("nested_walk")
    log_ev, log_dev = out[0], out[1]
    wts = np.exp(out[3])
    H = float(np.sum(wts * out.ll) - log_ev)
    sigma = math.sqrt(max(H, 0.0) / nlive)
    truth = shell_log_z(D, r, w, half)
    csteps = float(out.n_gen) * k * nmcmc
    line = {"config": "C3 nested D=16 Gaussian shell, nlive %d, k %d, nmcmc %d" % (nlive, k, nmcmc),
            "unit": "constrained MH steps/s", "dtype": "f64", "value": csteps / dt,
            "wall_s": dt, "wall_s_runs": walls, "n_dead": int(out.n_dead), "n_gen": int(out.n_gen),
            "with_points_d2h": {"value": csteps / dt_pts, "wall_s": dt_pts, "wall_s_runs": walls_pts,
                                "note": "the same runs plus the n x D dead points copied to the host"},
            "dead_points_per_s": out.n_dead / dt,
            "log_evidence": {"nested": log_ev, "analytic": truth, "abs_delta": abs(log_ev - truth),
                             "sigma_H": sigma, "within_1sigma": abs(log_ev - truth) <= sigma,
                             "log_dev": log_dev, "H": H,
                             "log_total_error_estimate": nested.log_total_error_estimate(log_ev, log_dev, nlive)},
            "roofline": ic_gather("mcg::nest_walk_kernel<16,SHELL>", k * nmcmc, 16.0 * D, tw, c3_pmc(k, nmcmc)),
            "roofline_hbm": hbm_secondary(roofline("mcg::nest_walk_kernel<16,SHELL>", k * nmcmc,
                                                   8.0 * (D + 2) + 16.0 * D, tw))}
    ctx.close()
    return line


def c2(args):
    """The headline C2 MH workload (bench.py's timed part, for same-box A/B): D=32 diagonal
    Gaussian, 65,536 chains, launches of 1,000 sweeps folded into the moments."""
    D, N, S, K = 32, 65536, 1000, args.launches // 10
    rng = np.random.default_rng(42)
    mu, sg = rng.uniform(-1.0, 1.0, D), rng.uniform(0.5, 2.0, D)
    s = 2.38 / math.sqrt(D) * float(np.median(sg))
    ctx = Context(seed=args.seed)
    ctx.set_model(T.diag_gauss(mu, sg), T.box(-10 * np.ones(D), 10 * np.ones(D)), T.gauss(s))
    ctx.init(np.random.default_rng(1000).normal(mu[:, None], sg[:, None], size=(D, N)))
    ctx.run(nbin=S, nskip=1, n_rec=1, record_x=False, record_llp=False, accumulate=True)
    ctx.sync()
    ctx.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(K):
        ctx.run(nbin=0, nskip=1, n_rec=S, record_x=False, record_llp=False, accumulate=True, append=True)
    ctx.sync()
    dt = time.perf_counter() - t0
    line = {"config": "C2 D=32 diagonal Gaussian, %d chains, %d sweeps" % (N, K * S), "unit": "MH steps/s",
            "dtype": "f64", "value": N * S * K / dt, "lanes": ctx.lanes(),
            "roofline": roofline("mcg::mh_kernel<32,P,DIAG_GAUSS,GAUSS>", N * S, 8.0 * (D + 2),
                                 ctx.kernel_timing("mh"))}
    ctx.close()
    return line


def c4(args):
    """Interpolate_pdf kD-tree independence proposal, D=8 N(0,1) target, M=32,768 exact draws,
    32,768 chains."""
    D, N, M, S, K = 8, args.c4_chains, 32768, 1000, args.launches // 10
    rng = np.random.default_rng(4)
    pts = rng.normal(size=(M, D))
    lo, hi = -10 * np.ones(D), 10 * np.ones(D)
    ctx = Context(seed=args.seed)
    ctx.set_model(T.diag_gauss(np.zeros(D), np.ones(D)), T.box(lo, hi), T.KdInterp(pts, lo, hi))
    ctx.init(rng.normal(size=(D, N)))
    ctx.run(nbin=S, nskip=1, n_rec=1, record_x=False, record_llp=False, accumulate=True)
    ctx.sync()
    ctx.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(K):
        ctx.run(nbin=0, nskip=1, n_rec=S, record_x=False, record_llp=False, accumulate=True, append=True)
    mean, sd, lz = ctx.stats()
    dt = time.perf_counter() - t0
    acc, rej = ctx.counters()
    depth = math.ceil(math.log2(M))
    bps = 8.0 * (D + 2) + 16.0 * D + 2 * depth * 12.0
    line = {"config": "C4 kD interp proposal D=8, M=%d, %d chains, %d sweeps" % (M, N, K * S),
            "unit": "MH steps/s", "dtype": "f64", "value": N * S * K / dt,
            "accept_frac": acc / (acc + rej),
            # the independence proposal from a 32,768-point tree accepts ~0.1 % of its draws: the
            # rate of accepted moves is the figure to compare across proposals
            "accepted_steps_per_s": N * S * K / dt * acc / (acc + rej),
            "posterior_check": {"max_abs_mean_err": float(np.max(np.abs(mean))),
                                "max_rel_sd_err": float(np.max(np.abs(sd - 1)))},
            "log_z_harmonic_mean": lz, "log_z_analytic": -D * math.log(20.0),
            "roofline_hbm": hbm_secondary(roofline("mcg::mh_kernel<8,P,DIAG_GAUSS,KD_INTERP>", N * S, bps,
                                                   ctx.kernel_timing("mh"))),
            "roofline_note": "the 4 MB tree and the boxes are cache-resident and strict-interior draws "
                             "skip the descents, so the step is instruction-issue bound (DESIGN 5.4): "
                             "the primary roofline is VALU issue from the committed PMC pass"}
    line["roofline"] = valu_framing("c4", D, N, S, line["roofline_hbm"]["avg_launch_ms"]) or \
        {"bound": "valu", "frac": None, "note": "no PMC pass committed for this configuration"}
    ctx.close()
    return line


def c5(args):
    """D=64 full-covariance Gaussian, Sigma = Q diag(lambda) Q^T, lambda log-uniform [0.1, 10],
    131,072 chains (one GPU's share of 1,048,576 over 8)."""
    D, N, S, K = 64, args.c5_chains, 500, args.launches // 5
    rng = np.random.default_rng(5)
    Q, _ = np.linalg.qr(rng.normal(size=(D, D)))
    lam = np.exp(rng.uniform(math.log(0.1), math.log(10.0), D))
    cov = (Q * lam) @ Q.T
    cov = 0.5 * (cov + cov.T)
    mu = rng.uniform(-1, 1, D)
    s = 2.38 / math.sqrt(D) * math.sqrt(lam.min())
    ctx = Context(seed=args.seed)
    ctx.set_model(T.fullcov_gauss(mu, cov), T.flat_prior(), T.gauss(s))
    L = np.linalg.cholesky(cov)
    ctx.init(mu[:, None] + L @ rng.normal(size=(D, N)))
    ctx.run(nbin=S, nskip=1, n_rec=1, record_x=False, record_llp=False, accumulate=True)
    ctx.sync()
    ctx.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(K):
        ctx.run(nbin=0, nskip=1, n_rec=S, record_x=False, record_llp=False, accumulate=True, append=True)
    mean, sd, lz = ctx.stats()
    dt = time.perf_counter() - t0
    acc, rej = ctx.counters()
    line = {"config": "C5 D=64 full-covariance Gaussian, %d chains/GPU, %d sweeps" % (N, K * S),
            "unit": "MH steps/s", "dtype": "f64", "value": N * S * K / dt,
            "accept_frac": acc / (acc + rej),
            "posterior_check": {"max_abs_mean_err_over_sd": float(np.max(np.abs(mean - mu) / np.sqrt(np.diag(cov)))),
                                "max_rel_sd_err": float(np.max(np.abs(sd / np.sqrt(np.diag(cov)) - 1)))},
            "roofline_hbm": hbm_secondary(roofline("mcg::mh_fullcov_kernel<64,0>", N * S, 8.0 * (D + 2),
                                                   ctx.kernel_timing("mh"))),
            "flops_per_step": D * (D + 1)}
    ms = line["roofline_hbm"]["avg_launch_ms"]
    line["roofline"] = mfma_framing(D, N * S, ms, valu_framing("c5", D, N, S, ms)) or \
        {"bound": "mfma", "frac": None, "note": "no kernel timing"}
    ctx.close()
    return line


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="*", default=["c1", "c3", "c3k8", "c3n1k", "c4", "c5"])
    ap.add_argument("--out", default=None)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--nlive", type=int, default=131072)
    ap.add_argument("--k", type=int, default=4096)
    ap.add_argument("--nmcmc", type=int, default=100)
    ap.add_argument("--launches", type=int, default=100,
                    help="C4/C5: timed sweeps / 100 (C4: launches of 1,000 sweeps, C5: of 500 -- at or under\n                    the runtime's own launch length min(4096, 2^26/N))")
    ap.add_argument("--reps", type=int, default=5, help="C3: timed nested runs after a warm-up run (median reported)")
    ap.add_argument("--c5-chains", type=int, default=131072)
    ap.add_argument("--c4-chains", type=int, default=32768, help="C4 chains (BASELINE configs[3]: 32,768)")
    args = ap.parse_args()
    def c3k8(a):
        """C3 with 8,192 retirements a generation (two walker waves per draw-table workgroup)."""
        b = argparse.Namespace(**vars(a))
        b.k = 8192
        return c3(b)

    def c3n1k(a):
        """C3 at nested_evidence's own default walk length, nmcmc 1,000 (nested.ml:122)."""
        b = argparse.Namespace(**vars(a))
        b.nmcmc = 1000
        return c3(b)

    fns = {"c1": c1, "c2": c2, "c3": c3, "c3k8": c3k8, "c3n1k": c3n1k, "c4": c4, "c5": c5}
    for c in args.configs:
        line = fns[c](args)
        s = json.dumps(line)
        print(s, flush=True)
        if args.out:
            with open(args.out, "a") as fh:
                fh.write(s + "\n")


if __name__ == "__main__":
    main()
