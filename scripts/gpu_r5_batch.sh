#!/bin/bash
# Round 5, C3: generations per host batch (MCG_NESTED_MAX_BATCH) with the direct staging, same
# box, and the host-side split of a run (MCG_NESTED_PROFILE) at 64 and 16
mkdir -p gpurun_out/batch
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for i in 1 2; do
  for v in 64 32 16 128; do
    MCG_NESTED_MAX_BATCH=$v timeout -k 10 300 python3 scripts/bench_configs.py c3 --reps 3 --out gpurun_out/batch/b$v.jsonl > gpurun_out/batch/b$v.$i.log 2>&1 || { echo "$v rc=$?"; exit 1; }
  done
done
for v in 64 16; do
  MCG_NESTED_PROFILE=1 MCG_NESTED_MAX_BATCH=$v timeout -k 10 120 python3 scripts/probes/c3_wall.py > gpurun_out/batch/prof$v.log 2>&1 || exit 1
done
