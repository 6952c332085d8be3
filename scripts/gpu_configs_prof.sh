#!/bin/bash
# Kernel-trace statistics of the non-headline configs (C3, C4, C5 through bench_configs.py):
# per-kernel average durations for DESIGN.md (the C3 host loop runs slower under the tracer, the
# kernel durations do not).
mkdir -p gpurun_out/cfgprof
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/cfgprof/trace -o run --output-format csv -- \
  python3 scripts/bench_configs.py c3 c4 c5 --out gpurun_out/cfgprof/configs.jsonl > gpurun_out/cfgprof/trace.log 2>&1 || exit 1
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/cfgprof/trace/run_kernel_stats.csv")):
    if any(k in r["Name"] for k in ("nest_walk", "merge_fused", "mh_kernel<8", "fullcov")):
        print("%-60s %8s calls %10.2f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1000))
PY
