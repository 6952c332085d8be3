#!/bin/bash
# The GPU suite alone (one process, per-test time limit).
mkdir -p gpurun_out/suite
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rf --timeout 150 --timeout-method thread > gpurun_out/suite/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/suite/pytest.log; exit $rc
