#!/bin/bash
# C3 fused sort+merge (default) vs the two-launch rank count + merge (MCG_NESTED_MERGE2=1): nested
# GPU tests, then per arm the C3 config line (3 timed runs, median) and a kernel trace of one run.
mkdir -p gpurun_out/c3m
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_nested.py tests/test_golden.py -x -q --timeout 100 --timeout-method thread > gpurun_out/c3m/pytest.log 2>&1 || { tail -30 gpurun_out/c3m/pytest.log; exit 1; }
tail -1 gpurun_out/c3m/pytest.log
for arm in fused merge2 fused merge2; do
  if [ $arm = merge2 ]; then export MCG_NESTED_MERGE2=1; else unset MCG_NESTED_MERGE2; fi
  timeout -k 10 200 python scripts/bench_configs.py c3 --out gpurun_out/c3m/$arm.jsonl > /dev/null 2>&1 || exit 1
  tail -1 gpurun_out/c3m/$arm.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$arm', d['value'], d['wall_s_runs'], d['roofline']['avg_launch_ms'], d['log_evidence']['abs_delta'], d['log_evidence']['sigma_H'])"
done
for arm in fused merge2; do
  if [ $arm = merge2 ]; then export MCG_NESTED_MERGE2=1; else unset MCG_NESTED_MERGE2; fi
  rm -rf gpurun_out/c3m/tr_$arm
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/c3m/tr_$arm -o run --output-format csv -- python3 scripts/probes/c3_once.py > gpurun_out/c3m/tr_$arm.log 2>&1 || exit 1
  python3 - $arm <<'PY'
import csv, sys
arm = sys.argv[1]
for r in csv.DictReader(open("gpurun_out/c3m/tr_%s/run_kernel_stats.csv" % arm)):
    if any(k in r["Name"] for k in ("nest_walk", "rank_count", "merge_new", "merge_fused")):
        print("%-7s %-34s %6d calls %.2f us" % (arm, r["Name"][:34], int(r["Calls"]), float(r["AverageNs"]) / 1000))
PY
done
