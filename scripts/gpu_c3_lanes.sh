#!/bin/bash
# kernel-trace stats of C3 with each walker lane split (walk kernel time per generation)
mkdir -p gpurun_out/c3lanes
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for l in narrow wide narrow wide; do
  MCG_NEST_LANES=$l timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/c3lanes/$l -o run --output-format csv -- python3 scripts/probes/c3_once.py >> gpurun_out/c3lanes/log.txt 2>&1 || exit $?
  grep -h "nest_walk\|rank_count\|merge_new" gpurun_out/c3lanes/$l/run_kernel_stats.csv | cut -d, -f1-4 | sed "s/^/$l: /" >> gpurun_out/c3lanes/summary.txt
done
cat gpurun_out/c3lanes/summary.txt; grep wall gpurun_out/c3lanes/log.txt
