#!/bin/bash
# Round 5: the nested GPU tests (incl. the one-launch walk + merge, MCG_NESTED_FM=1), then the
# C3 line on the default two-launch path
mkdir -p gpurun_out/nested
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_nested.py tests/test_gpu_rccl.py > gpurun_out/nested/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/nested/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/bench_configs.py c3 --reps 3 --out gpurun_out/nested/c3.jsonl > gpurun_out/nested/c3.log 2>&1 || exit 1
python3 -c "import json;l=json.loads(open('gpurun_out/nested/c3.jsonl').read().splitlines()[-1]);print('%.4g'%l['value'], l['wall_s_runs'], l['n_gen'], l['log_evidence']['abs_delta'])"
