#!/bin/bash
# Round 5, C3: the retiring kernels write each batch's dead ll / lp straight into mapped pinned
# host memory (default) against two device-to-host copies per batch (MCG_NESTED_STAGE_COPY=1):
# the nested parity tests, then a same-box A/B of the C3 lines, alternated
mkdir -p gpurun_out/stage
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_nested.py tests/test_gpu_gauss_prior.py tests/test_gpu_gauss_mix.py tests/test_gpu_rccl.py > gpurun_out/stage/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/stage/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for v in direct copy; do
    if [ $v = copy ]; then export MCG_NESTED_STAGE_COPY=1; else unset MCG_NESTED_STAGE_COPY; fi
    timeout -k 10 300 python3 scripts/bench_configs.py c3 c3k8 --reps 3 --out gpurun_out/stage/$v.jsonl > gpurun_out/stage/$v$i.log 2>&1 || { echo "$v rc=$?"; exit 1; }
  done
done
python3 - <<'PY'
import json
for v in ("direct", "copy"):
    for l in open("gpurun_out/stage/%s.jsonl" % v):
        d = json.loads(l)
        print(v, d["config"][40:70], "%.4g" % d["value"], [round(x, 4) for x in d["wall_s_runs"]])
PY
