#!/bin/bash
# Round-4 full GPU session: the GPU suite, smoke, bench (+ CPU baseline), the rocprofv3
# kernel-trace / PMC profile of the bench, one line per other config, and the VALU / detail PMC
# passes of the C4 / C5 config kernels.  Every GPU step runs under its own time limit; the first
# failure ends the script.
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
bash scripts/gpu_full.sh "$@" || exit $?
bash scripts/gpu_pmc_cfg.sh > gpurun_out/pmc_cfg_run.log 2>&1
rc=$?; echo "pmc cfg rc=$rc" | tee -a gpurun_out/status.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_configs_prof.sh > gpurun_out/cfgprof.txt 2>&1
rc=$?; echo "configs trace rc=$rc" | tee -a gpurun_out/status.log; exit $rc
