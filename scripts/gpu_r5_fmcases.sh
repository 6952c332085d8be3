#!/bin/bash
# Round 5: the one-launch walk + merge parity tests (all walker instances)
mkdir -p gpurun_out/fmcases
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_nested.py -k "one_launch" > gpurun_out/fmcases/pytest.log 2>&1
rc=$?; tail -12 gpurun_out/fmcases/pytest.log; exit $rc
