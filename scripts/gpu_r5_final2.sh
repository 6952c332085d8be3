#!/bin/bash
# Round 5, final session part 2: the nested GPU tests on the k > 4,096 lane default, the C3 lines,
# then the PMC passes of the C4 / C5 config kernels and the kernel-trace statistics of C3-C5.
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_nested.py > gpurun_out/nested_final.log 2>&1
rc=$?; tail -2 gpurun_out/nested_final.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 scripts/bench_configs.py c3 c3k8 c3n1k --out gpurun_out/configs_c3.jsonl > gpurun_out/configs_c3.log 2>&1 || exit 1
bash scripts/gpu_pmc_cfg.sh > gpurun_out/pmc_cfg_run.log 2>&1
rc=$?; echo "pmc cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_configs_prof.sh > gpurun_out/cfgprof.txt 2>&1
rc=$?; echo "configs trace rc=$rc"; cat gpurun_out/cfgprof.txt; exit $rc
