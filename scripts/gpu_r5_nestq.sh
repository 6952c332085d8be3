#!/bin/bash
# Round 5: the nested and state GPU tests, then the C3 line (quick check after a host-side change)
mkdir -p gpurun_out/nestq
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_nested.py tests/test_gpu_gauss_prior.py tests/test_gpu_rccl.py tests/test_gpu_state.py > gpurun_out/nestq/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/nestq/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/bench_configs.py c3 --reps 3 --out gpurun_out/nestq/c3.jsonl > gpurun_out/nestq/c3.log 2>&1 || exit 1
python3 -c "import json;l=json.loads(open('gpurun_out/nestq/c3.jsonl').read().splitlines()[-1]);print('%.4g'%l['value'], l['wall_s_runs'])"
