#!/bin/bash
# C3 host-loop A/B: nested GPU tests, then the host breakdown and the C3 line at max batch 64 / 128
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nested.py tests/test_golden.py > gpurun_out/nt.log 2>&1 || { tail -20 gpurun_out/nt.log; exit 1; }
tail -1 gpurun_out/nt.log
for mb in 64 128; do
  MCG_NESTED_MAX_BATCH=$mb MCG_NESTED_PROFILE=1 timeout -k 10 120 python scripts/probes/c3_profile.py > gpurun_out/c3p_$mb.log 2>&1 || exit 1
  MCG_NESTED_MAX_BATCH=$mb timeout -k 10 240 python scripts/bench_configs.py c3 --reps 7 > gpurun_out/c3_$mb.log 2>&1 || exit 1
  echo "max batch $mb"; tail -4 gpurun_out/c3p_$mb.log
  python -c "
import json;d=json.loads(open('gpurun_out/c3_$mb.log').read().strip().splitlines()[-1]);print('C3 %.4g' % d['value'], [round(x*1e3,1) for x in d['wall_s_runs']])"
done
