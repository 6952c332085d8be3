#!/usr/bin/env python3
"""Per-launch durations of the headline MH kernel from a rocprofv3 --kernel-trace run of bench.py
(scripts/gpu_profile.sh), with the warmup launch(es) separated from the timed ones.

bench.py runs the burn-in (warmup x sweeps) as one launch of several hundred sweeps before the
timed launches of `sweeps` each; rocprofv3's --stats average mixes the two.  This reports the
mean / median / min of the launches of the timed length, the figure bench.py's HIP-event
`roofline.avg_launch_ms` measures.

  python scripts/trace_summary.py gpurun_out/prof/trace/run_kernel_trace.csv out.json
"""
import csv
import json
import statistics
import sys


def main():
    path, out = sys.argv[1], sys.argv[2]
    pat = sys.argv[3] if len(sys.argv) > 3 else "mh_kernel<32, 4"
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            for r in csv.DictReader(open(path)) if pat in r["Kernel_Name"]]
    med = statistics.median(durs)
    timed = [d for d in durs if d < 1.5 * med]        # the burn-in launch runs several x longer
    res = {"kernel_pattern": pat, "launches": len(durs), "timed_launches": len(timed),
           "warmup_launch_ms": [d for d in durs if d >= 1.5 * med],
           "timed_mean_ms": statistics.fmean(timed), "timed_median_ms": statistics.median(timed),
           "timed_min_ms": min(timed), "timed_max_ms": max(timed)}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
