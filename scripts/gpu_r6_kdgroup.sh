#!/bin/bash
OUT=gpurun_out/r6_kdgroup; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_mh.py -k "kd_grouped or kd" > $OUT/t.log 2>&1
rc=$?; tail -12 $OUT/t.log; exit $rc
