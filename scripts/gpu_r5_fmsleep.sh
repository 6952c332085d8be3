#!/bin/bash
# Round 5, C3: the fused walk + merge against the two-launch path, by the merge role's poll
# interval (MCG_NESTED_FM_SLEEP, units of 512 clocks)
mkdir -p gpurun_out/fmsleep
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for v in two 1 p2 two; do
  if [ $v = two ]; then export MCG_NESTED_FM=0; elif [ $v = p2 ]; then export MCG_NESTED_FM=2; else unset MCG_NESTED_FM; export MCG_NESTED_FM_SLEEP=$v; fi
  timeout -k 10 300 python3 scripts/bench_configs.py c3 --reps 2 --out gpurun_out/fmsleep/$v.jsonl > gpurun_out/fmsleep/$v.log 2>&1 || { echo "$v rc=$?"; exit 1; }
  python3 -c "import json;l=json.loads(open('gpurun_out/fmsleep/$v.jsonl').read().splitlines()[-1]);print('$v', '%.4g'%l['value'], l['wall_s_runs'], l['n_gen'], l['log_evidence']['abs_delta'])"
done
for v in 0 2; do
  export MCG_NESTED_FM=$v
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/fmsleep/trace$v -o run --output-format csv -- python3 scripts/probes/nested_breakdown.py > gpurun_out/fmsleep/trace$v.log 2>&1 || exit 1
  head -5 gpurun_out/fmsleep/trace$v/run_kernel_stats.csv | cut -c1-150
done
