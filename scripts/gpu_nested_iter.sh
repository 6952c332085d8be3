#!/bin/bash
# nested iteration: nested GPU parity tests, then the C3 kernel-trace profile
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_nested.py -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1 || exit $?
bash scripts/gpu_prof_nested.sh
