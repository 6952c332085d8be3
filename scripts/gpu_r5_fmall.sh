#!/bin/bash
# Round 5: every nested GPU test with the one-launch walk + merge switched on (MCG_NESTED_FM=1)
mkdir -p gpurun_out/fmall
export PYTHONUNBUFFERED=1 TMPDIR=/tmp MCG_NESTED_FM=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_nested.py tests/test_gpu_gauss_prior.py tests/test_gpu_gauss_mix.py tests/test_gpu_rccl.py tests/test_gpu_state.py > gpurun_out/fmall/pytest.log 2>&1
rc=$?; tail -4 gpurun_out/fmall/pytest.log; exit $rc
