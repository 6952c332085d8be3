#!/bin/bash
# phase stamps of C3 generation 200 (MCG_NEST_TRACE build lib/libmcg_trace.so), split on / off
OUT=gpurun_out/r6_stamps; mkdir -p $OUT
for sp in 1 0; do
  MCG_NESTED_SPLIT=$sp MCG_LIBRARY=$PWD/mcmc-ocaml_amd/lib/libmcg_trace.so MCG_NEST_TRACE=200 timeout -k 10 120 python3 scripts/probes/c3_once.py > $OUT/stamps$sp.log 2>&1 || exit 1
  echo "== stamps split=$sp"; grep "trace gen" $OUT/stamps$sp.log | sort -k4,4 -k6,6n
done
