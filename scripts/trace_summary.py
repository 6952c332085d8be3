#!/usr/bin/env python3
"""Per-launch durations of the headline MH kernel from a rocprofv3 --kernel-trace run of bench.py
(scripts/gpu_profile.sh), with the warmup launch(es) separated from the timed ones.

bench.py runs the burn-in (warmup x sweeps) as one launch of several hundred sweeps before the
timed launches of `sweeps` each; rocprofv3's --stats average mixes the two.  This reports the
mean / median / min of the launches of the timed length, the figure bench.py's HIP-event
`roofline.avg_launch_ms` measures.

  python scripts/trace_summary.py gpurun_out/prof/trace/run_kernel_trace.csv out.json [pattern] [--last K]

--last K: the last K launches of the kernel are the timed ones (bench.py --steps K: its burn-in
--warmup W x 1,000 sweeps runs as W launches of the same length before them, so the length test
cannot separate them); the line's roofline frac is then reproduced from the trace as
K launches x 65,536 chains x 1,000 sweeps x 272 B / their summed duration / 8 TB/s.
"""
import csv
import json
import statistics
import sys


def main():
    args = sys.argv[1:]
    last = None
    if "--last" in args:
        i = args.index("--last")
        last = int(args[i + 1])
        del args[i:i + 2]
    path, out = args[0], args[1]
    pat = args[2] if len(args) > 2 else "mh_kernel<32, 4"
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            for r in csv.DictReader(open(path)) if pat in r["Kernel_Name"]]
    med = statistics.median(durs)
    if last:
        timed, warm = durs[-last:], durs[:-last]
    else:
        timed = [d for d in durs if d < 1.5 * med]    # the burn-in launch runs several x longer
        warm = [d for d in durs if d >= 1.5 * med]
    res = {"kernel_pattern": pat, "launches": len(durs), "timed_launches": len(timed),
           "warmup_launch_ms": warm,
           "timed_mean_ms": statistics.fmean(timed), "timed_median_ms": statistics.median(timed),
           "timed_min_ms": min(timed), "timed_max_ms": max(timed)}
    if last and pat.startswith("mh_kernel<32, 4"):
        res["c2_hbm_frac_from_trace"] = 65536 * 1000 * 272.0 / (res["timed_mean_ms"] * 1e-3) / 8e12
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
