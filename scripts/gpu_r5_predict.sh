#!/bin/bash
# Round 5, C3: the last batches sized from the predicted stop (default) against full batches
# (MCG_NESTED_NO_PREDICT=1): the nested tests, a same-box A/B of the C3 lines, and the
# generations launched per run (MCG_NESTED_PROFILE)
mkdir -p gpurun_out/predict
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_nested.py tests/test_gpu_gauss_prior.py tests/test_gpu_gauss_mix.py tests/test_gpu_state.py > gpurun_out/predict/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/predict/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for v in predict full; do
    if [ $v = full ]; then export MCG_NESTED_NO_PREDICT=1; else unset MCG_NESTED_NO_PREDICT; fi
    timeout -k 10 300 python3 scripts/bench_configs.py c3 c3k8 --reps 3 --out gpurun_out/predict/$v.jsonl > gpurun_out/predict/$v$i.log 2>&1 || { echo "$v rc=$?"; exit 1; }
  done
done
unset MCG_NESTED_NO_PREDICT
python3 - <<'PY'
import json
for v in ("predict", "full"):
    for l in open("gpurun_out/predict/%s.jsonl" % v):
        d = json.loads(l)
        print(v, d["config"][40:70], "%.4g" % d["value"], [round(x, 4) for x in d["wall_s_runs"]], d["n_gen"])
PY
MCG_NESTED_PROFILE=1 timeout -k 10 120 python3 scripts/probes/c3_wall.py > gpurun_out/predict/wall.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/predict/wall.log | tail -4
