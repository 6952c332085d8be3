#!/bin/bash
# Round 5, C3: the wall split of one nested_evidence call (scripts/probes/c3_wall.py)
mkdir -p gpurun_out/c3wall
export PYTHONUNBUFFERED=1 TMPDIR=/tmp MCG_NESTED_PROFILE=1 MCG_NESTED_FM=0
timeout -k 10 120 python3 scripts/probes/c3_wall.py > gpurun_out/c3wall/wall.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/c3wall/wall.log; exit $rc
