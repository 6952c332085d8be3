#!/bin/bash
# Round 5: the randomised GPU parity sweep (tests/test_gpu_fuzz.py), every case run (no -x)
mkdir -p gpurun_out/fuzz
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v -rf --timeout 150 --timeout-method thread tests/test_gpu_fuzz.py > gpurun_out/fuzz/pytest.log 2>&1
rc=$?; grep -E "FAILED|passed|failed" gpurun_out/fuzz/pytest.log | tail -30; exit $rc
