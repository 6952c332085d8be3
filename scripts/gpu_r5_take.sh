#!/bin/bash
# Round 5, C3: nested_evidence's ll / lp / weights handed over without a copy (mcg_nested_take):
# the state and nested GPU tests, then the C3 lines and the wall split
mkdir -p gpurun_out/take
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_state.py tests/test_gpu_nested.py tests/test_gpu_gauss_prior.py tests/test_gpu_gauss_mix.py tests/test_gpu_rccl.py > gpurun_out/take/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/take/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python3 scripts/bench_configs.py c3 c3k8 --reps 3 --out gpurun_out/take/c3.jsonl > gpurun_out/take/c3.$i.log 2>&1 || exit 1
done
python3 -c "
import json
for l in open('gpurun_out/take/c3.jsonl'):
    d=json.loads(l); print(d['config'][40:70], '%.4g'%d['value'], [round(x,4) for x in d['wall_s_runs']])"
MCG_NESTED_PROFILE=1 timeout -k 10 120 python3 scripts/probes/c3_wall.py > gpurun_out/take/wall.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/take/wall.log | tail -4
