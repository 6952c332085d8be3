#!/bin/bash
# Same-box A/B of two builds of libmcg.so on bench_configs lines (A B A B), after the given GPU
# tests pass with build B.  usage: gpu_ab_lib.sh <libA> <libB> "<configs>" "<pytest targets>"
mkdir -p gpurun_out/ab
export PYTHONUNBUFFERED=1
A=$1; B=$2; CFG=$3; TESTS=$4
if [ -n "$TESTS" ]; then
  MCG_LIBRARY=$B timeout -k 10 600 python -u -m pytest $TESTS -q -m gpu -rf --timeout 150 --timeout-method thread > gpurun_out/ab/tests_B.log 2>&1
  rc=$?; echo "tests(B) rc=$rc" | tee -a gpurun_out/status.log; [ $rc -eq 0 ] || exit $rc
fi
for rep in 1 2; do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    MCG_LIBRARY=$lib timeout -k 10 600 python scripts/bench_configs.py $CFG --out gpurun_out/ab/${v}${rep}.jsonl > gpurun_out/ab/${v}${rep}.log 2>&1
    rc=$?; echo "$v$rep rc=$rc" | tee -a gpurun_out/status.log; [ $rc -eq 0 ] || exit $rc
  done
done
