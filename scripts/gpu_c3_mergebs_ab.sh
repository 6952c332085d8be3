#!/bin/bash
# fused-merge workgroup size A/B: nested GPU tests at 512 and 1024 survivors per workgroup, then
# the C3 line at 256 / 512 / 1024
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for bs in 1024 512; do
  MCG_NESTED_MERGE_BS=$bs timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nested.py > gpurun_out/nt_$bs.log 2>&1 || { tail -20 gpurun_out/nt_$bs.log; exit 1; }
  echo "bs $bs: $(tail -1 gpurun_out/nt_$bs.log)"
done
for bs in 256 512 1024; do
  MCG_NESTED_MERGE_BS=$bs timeout -k 10 240 python scripts/bench_configs.py c3 --reps 7 > gpurun_out/c3_bs$bs.log 2>&1 || exit 1
  python -c "
import json;d=json.loads(open('gpurun_out/c3_bs$bs.log').read().strip().splitlines()[-1]);print('bs $bs C3 %.4g' % d['value'], [round(x*1e3,1) for x in d['wall_s_runs']])"
done
