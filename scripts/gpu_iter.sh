#!/bin/bash
# GPU iteration: all parity tests, a short bench (no CPU baseline), then the C3/C5 config lines.
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" | tee gpurun_out/status.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --nested-seeds 0 "$@" > gpurun_out/bench_quick.log 2>&1
rc=$?; echo "bench rc=$rc" | tee -a gpurun_out/status.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python scripts/bench_configs.py c3 c5 --out gpurun_out/configs.jsonl > gpurun_out/configs.log 2>&1
rc=$?; echo "configs rc=$rc" | tee -a gpurun_out/status.log; exit $rc
