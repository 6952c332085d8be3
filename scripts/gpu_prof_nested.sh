#!/bin/bash
# rocprofv3 kernel-trace stats of the C3 nested-sampling config (one run)
mkdir -p gpurun_out/prof_c3
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3/trace -o run --output-format csv -- python3 scripts/bench_configs.py c3 --out gpurun_out/prof_c3/c3.jsonl > gpurun_out/prof_c3/trace.log 2>&1
rc=$?; echo "c3 prof rc=$rc"; exit $rc
