#!/bin/bash
# (needs lib/libmcg_old.so built from commit 47b1624 and lib/libmcg_trace.so from the counting-form sources, both since removed)
# Round 5, C3: the merge's counting form for small subsets (every survivor against every subset
# key, wave-ballot counts; no binary searches) and 32-bit tie compares -- nested parity, then a
# same-box A/B of the C3 line against lib/libmcg_old.so (the previous commit's merge), alternated,
# then the phase stamps of generation 200 from lib/libmcg_trace.so
mkdir -p gpurun_out/mcount
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_nested.py tests/test_gpu_gauss_prior.py tests/test_gpu_fuzz.py -k "nested" > gpurun_out/mcount/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/mcount/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then export MCG_LIBRARY=$PWD/mcmc-ocaml_amd/lib/libmcg_old.so; else unset MCG_LIBRARY; fi
    timeout -k 10 300 python3 scripts/bench_configs.py c3 --reps 3 --out gpurun_out/mcount/$v.jsonl > gpurun_out/mcount/$v$i.log 2>&1 || { echo "$v rc=$?"; exit 1; }
    python3 -c "import json;l=json.loads(open('gpurun_out/mcount/$v.jsonl').read().splitlines()[-1]);print('$v', '%.4g'%l['value'], l['wall_s_runs'], l['n_gen'], l['log_evidence']['abs_delta'])"
  done
done
unset MCG_LIBRARY
MCG_LIBRARY=$PWD/mcmc-ocaml_amd/lib/libmcg_trace.so MCG_NEST_TRACE=200 timeout -k 10 120 python3 scripts/probes/c3_once.py > gpurun_out/mcount/stamps.log 2>&1 || exit 1
grep "trace gen" gpurun_out/mcount/stamps.log | tail -14
