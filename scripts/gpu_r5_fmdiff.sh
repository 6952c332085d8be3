#!/bin/bash
# Round 5: where the fused walk + merge departs from the oracle (scripts/probes/fm_diff.py)
mkdir -p gpurun_out/fmdiff
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 240 python3 -u scripts/probes/fm_diff.py > gpurun_out/fmdiff/diff.log 2>&1
rc=$?; cat gpurun_out/fmdiff/diff.log; exit $rc
