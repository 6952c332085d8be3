#!/bin/bash
# Round 6 (b): changed-area GPU tests, then C3 split vs one-launch merge alternated, then the
# phase stamps of generation 200 with the MCG_NEST_TRACE build (lib/libmcg_trace.so)
set -o pipefail
OUT=gpurun_out/r6_b; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_nested.py tests/test_gpu_rj.py tests/test_mixture.py tests/test_gpu_mh.py -x -q -m gpu -rf --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for sp in 0 1; do
    MCG_NESTED_SPLIT=$sp timeout -k 10 300 python scripts/bench_configs.py c3 --out $OUT/c3_s${sp}_${rep}.jsonl > $OUT/c3_s${sp}_${rep}.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "c3 rc=$rc"; exit $rc; }
    python -c "import json;d=json.loads(open('$OUT/c3_s${sp}_${rep}.jsonl').read().splitlines()[-1]);print('split',$sp,'%.4g'%d['value'],d['log_evidence']['nested'],d['n_gen'])"
  done
done
for sp in 1 0; do
  MCG_NESTED_SPLIT=$sp MCG_LIBRARY=$PWD/mcmc-ocaml_amd/lib/libmcg_trace.so MCG_NEST_TRACE=200 timeout -k 10 120 python3 scripts/probes/c3_once.py > $OUT/stamps$sp.log 2>&1 || exit 1
  echo "== stamps split=$sp"; grep "trace gen" $OUT/stamps$sp.log | tail -16
done
