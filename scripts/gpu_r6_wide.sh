#!/bin/bash
# Round 6: the lane-split wrap / DE kernels and the D 64 kD store probe
OUT=gpurun_out/r6_wide; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_any_dim.py tests/test_gpu_mh.py -x -q -m gpu -rf --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
MCG_LIBRARY=$PWD/mcmc-ocaml_amd/lib/libmcg_kd64.so timeout -k 10 200 python3 scripts/probes/kd64_store.py > $OUT/kd64.log 2>&1
echo "kd64 rc=$?"; cat $OUT/kd64.log | tail -12
