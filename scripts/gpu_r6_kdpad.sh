#!/bin/bash
OUT=gpurun_out/r6_kdpad; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_any_dim.py tests/test_gpu_fuzz.py tests/test_gpu_mh.py tests/test_gpu_rj.py -x -q -m gpu -rf --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 $OUT/tests.log; exit $rc
