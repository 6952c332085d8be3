#!/bin/bash
# Same-box comparison of N builds of libmcg.so on bench_configs lines (rounds of all builds),
# after the given GPU tests pass with each build but the first.
# usage: gpu_abn.sh "<configs>" "<pytest targets>" <lib0> <lib1> ...
mkdir -p gpurun_out/ab
export PYTHONUNBUFFERED=1
CFG=$1; TESTS=$2; shift 2
LIBS=("$@")
if [ -n "$TESTS" ]; then
  for i in "${!LIBS[@]}"; do
    [ $i -eq 0 ] && continue
    MCG_LIBRARY=${LIBS[$i]} timeout -k 10 600 python -u -m pytest $TESTS -q -m gpu -rf --timeout 150 --timeout-method thread > gpurun_out/ab/tests_$i.log 2>&1
    rc=$?; echo "tests($i) rc=$rc" | tee -a gpurun_out/status.log; [ $rc -eq 0 ] || exit $rc
  done
fi
for rep in 1 2; do
  for i in "${!LIBS[@]}"; do
    MCG_LIBRARY=${LIBS[$i]} timeout -k 10 600 python scripts/bench_configs.py $CFG --out gpurun_out/ab/L${i}_${rep}.jsonl > gpurun_out/ab/L${i}_${rep}.log 2>&1
    rc=$?; echo "L$i/$rep rc=$rc" | tee -a gpurun_out/status.log; [ $rc -eq 0 ] || exit $rc
  done
done
