#!/bin/bash
# Round 5, C3: in-kernel phase stamps (MCG_NEST_TRACE build) of generation 200, fused walk + merge
# against two launches
mkdir -p gpurun_out/fmtrace
export PYTHONUNBUFFERED=1 TMPDIR=/tmp MCG_LIBRARY=$PWD/mcmc-ocaml_amd/lib/libmcg_trace.so MCG_NEST_TRACE=200
for v in 1 0; do
  export MCG_NESTED_FM=$v
  timeout -k 10 120 python3 scripts/probes/c3_once.py > gpurun_out/fmtrace/fm$v.log 2>&1 || { echo "fm$v failed"; tail -5 gpurun_out/fmtrace/fm$v.log; exit 1; }
  grep "trace gen" gpurun_out/fmtrace/fm$v.log | tail -40
done
