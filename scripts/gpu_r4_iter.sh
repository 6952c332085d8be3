#!/bin/bash
# Iteration session: the given test files, then bench_configs on the given configs.
# usage: gpu_r4_iter.sh "<pytest targets>" "<configs>"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest $1 -q -m gpu -rf --timeout 150 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1
rc=$?; echo "tests rc=$rc" | tee -a gpurun_out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python scripts/bench_configs.py $2 --out gpurun_out/configs.jsonl > gpurun_out/configs.log 2>&1
rc=$?; echo "configs rc=$rc" | tee -a gpurun_out/status.log; exit $rc
