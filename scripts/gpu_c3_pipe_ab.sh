#!/bin/bash
# C3 pipelined merges (MCG_NESTED_PIPE=1) vs the serial merge (default): nested GPU tests, then for each
# arm the C3 config line (3 timed runs, median) and a kernel trace of one run.
mkdir -p gpurun_out/c3ab
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_nested.py tests/test_golden.py -x -q --timeout 100 --timeout-method thread > gpurun_out/c3ab/pytest.log 2>&1 || { tail -5 gpurun_out/c3ab/pytest.log; exit 1; }
tail -1 gpurun_out/c3ab/pytest.log
for arm in pipe serial pipe serial; do
  if [ $arm = pipe ]; then export MCG_NESTED_PIPE=1; else unset MCG_NESTED_PIPE; fi
  timeout -k 10 200 python scripts/bench_configs.py c3 --out gpurun_out/c3ab/$arm.jsonl > /dev/null 2>&1 || exit 1
  tail -1 gpurun_out/c3ab/$arm.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$arm', d['value'], d['wall_s_runs'], d['roofline']['avg_launch_ms'])"
done
for arm in pipe serial; do
  if [ $arm = pipe ]; then export MCG_NESTED_PIPE=1; else unset MCG_NESTED_PIPE; fi
  rm -rf gpurun_out/c3ab/tr_$arm
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/c3ab/tr_$arm -o run --output-format csv -- python3 scripts/probes/c3_once.py > gpurun_out/c3ab/tr_$arm.log 2>&1 || exit 1
  python3 - $arm <<'PY'
import csv, sys
arm = sys.argv[1]
for r in csv.DictReader(open("gpurun_out/c3ab/tr_%s/run_kernel_stats.csv" % arm)):
    if any(k in r["Name"] for k in ("nest_walk", "rank_count", "merge_new", "head_merge")):
        print("%-7s %-34s %6d calls %.2f us" % (arm, r["Name"][:34], int(r["Calls"]), float(r["AverageNs"]) / 1000))
PY
done
