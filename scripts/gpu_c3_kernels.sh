#!/bin/bash
# nested GPU tests, then the C3 kernels' average times (kernel trace) and the host breakdown
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_nested.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_nested.log 2>&1 || { tail -5 gpurun_out/pytest_nested.log; exit 1; }
tail -1 gpurun_out/pytest_nested.log
rm -rf gpurun_out/c3k
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/c3k -o run --output-format csv -- python3 scripts/probes/c3_once.py > gpurun_out/c3k.log 2>&1 || exit 1
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/c3k/run_kernel_stats.csv")):
    if any(k in r["Name"] for k in ("nest_walk", "rank_count", "merge_new")):
        print("%-40s %.2f us" % (r["Name"][:40], float(r["AverageNs"]) / 1000))
PY
MCG_NESTED_PROFILE=1 timeout -k 10 200 python scripts/probes/c3_profile.py 2>&1 | tail -4
