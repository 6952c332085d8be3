#!/bin/bash
# Full GPU-box session: parity tests + smoke + bench (with CPU baseline), then the rocprofv3
# kernel-trace / PMC profile of the bench, then one line per non-headline config.
# Every GPU step runs under its own time limit and the first failure ends the script.
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
bash scripts/gpu_check.sh "$@" || exit $?
bash scripts/gpu_profile.sh "$@" || exit $?
timeout -k 10 900 python scripts/bench_configs.py c1 c3 c3k8 c3n1k c4 c5 --out gpurun_out/configs.jsonl > gpurun_out/configs.log 2>&1
rc=$?; echo "configs rc=$rc" | tee -a gpurun_out/status.log; exit $rc
