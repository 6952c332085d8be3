#!/bin/bash
# (needs the stop-in-estimate build of LABLOG round 5, since reverted: MCG_NESTED_STOP_IN_WALK no longer exists)
# Round 5, C3: the next generation's stop test made by the merge kernel's estimate workgroup
# (the walk then only reads the stop flag) -- nested parity, then a same-box A/B of the C3 line
# against MCG_NESTED_STOP_IN_WALK=1 (the walk makes the test, as before), alternated
mkdir -p gpurun_out/stopest
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_nested.py tests/test_gpu_gauss_prior.py tests/test_gpu_fuzz.py tests/test_gpu_gauss_mix.py tests/test_gpu_fullsize.py -k "nested or Nested" > gpurun_out/stopest/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/stopest/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for v in est walk; do
    if [ $v = walk ]; then export MCG_NESTED_STOP_IN_WALK=1; else unset MCG_NESTED_STOP_IN_WALK; fi
    timeout -k 10 300 python3 scripts/bench_configs.py c3 --reps 3 --out gpurun_out/stopest/$v.jsonl > gpurun_out/stopest/$v$i.log 2>&1 || { echo "$v rc=$?"; exit 1; }
    python3 -c "import json;l=json.loads(open('gpurun_out/stopest/$v.jsonl').read().splitlines()[-1]);print('$v', '%.4g'%l['value'], l['wall_s_runs'], l['n_gen'], l['log_evidence']['abs_delta'])"
  done
done
