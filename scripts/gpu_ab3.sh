#!/bin/bash
# Same-box A/B/C of three builds on bench_configs lines (rounds of A B C), after the given GPU
# tests pass with build B.  usage: gpu_ab3.sh <libA> <libB> <libC> "<configs>" "<pytest targets>"
mkdir -p gpurun_out/ab
export PYTHONUNBUFFERED=1
A=$1; B=$2; C=$3; CFG=$4; TESTS=$5
if [ -n "$TESTS" ]; then
  MCG_LIBRARY=$B timeout -k 10 600 python -u -m pytest $TESTS -q -m gpu -rf --timeout 150 --timeout-method thread > gpurun_out/ab/tests_B.log 2>&1
  rc=$?; echo "tests(B) rc=$rc" | tee -a gpurun_out/status.log; [ $rc -eq 0 ] || exit $rc
fi
for rep in 1 2; do
  for v in A B C; do
    lib=$A; [ $v = B ] && lib=$B; [ $v = C ] && lib=$C
    MCG_LIBRARY=$lib timeout -k 10 600 python scripts/bench_configs.py $CFG --out gpurun_out/ab/${v}${rep}.jsonl > gpurun_out/ab/${v}${rep}.log 2>&1
    rc=$?; echo "$v$rep rc=$rc" | tee -a gpurun_out/status.log; [ $rc -eq 0 ] || exit $rc
  done
done
