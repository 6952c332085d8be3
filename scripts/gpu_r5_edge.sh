#!/bin/bash
# Round 5: the k > 4,096 nested parity cases (lane-split and merge-variant boundaries)
mkdir -p gpurun_out/edge
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_nested.py -k "large_k" tests/test_gpu_gauss_prior.py > gpurun_out/edge/pytest.log 2>&1
rc=$?; tail -8 gpurun_out/edge/pytest.log; exit $rc
