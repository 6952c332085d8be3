#!/bin/bash
# Round 5, C3: how long the per-batch staging copies (dead ll / lp, state) hold the stream:
# kernel + memory-copy trace of scripts/probes/c3_once.py
mkdir -p gpurun_out/copies
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/copies/trace -o run --output-format csv -- python3 scripts/probes/c3_once.py > gpurun_out/copies/trace.log 2>&1 || exit 1
ls gpurun_out/copies/trace
