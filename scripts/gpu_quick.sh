#!/bin/bash
# quick GPU iteration: MH parity tests + bench (no CPU baseline)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests -m gpu -q -x -rf > gpurun_out/pytest_quick.log 2>&1
rc=$?; echo "pytest rc=$rc" | tee gpurun_out/status.log
if [ $rc -ge 2 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/bench_quick.log 2>&1
rc=$?; echo "bench rc=$rc" | tee -a gpurun_out/status.log; exit $rc
