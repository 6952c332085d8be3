#!/bin/bash
# bench.py (C2 headline, with the CPU baseline) and the other configs' lines, each step under its
# own time limit; the first failure ends the script.
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python bench.py "$@" > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc" | tee -a gpurun_out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python scripts/bench_configs.py c1 c3 c4 c5 --out gpurun_out/configs.jsonl > gpurun_out/configs.log 2>&1
rc=$?; echo "configs rc=$rc" | tee -a gpurun_out/status.log; exit $rc
