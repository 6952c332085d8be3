#!/bin/bash
# Round 5, C3: the one-launch walk + merge (MCG_NESTED_FM=1) -- its parity tests, then a same-box
# A/B of the C3 line against the default two launches, alternated, then the phase stamps of
# generation 200 (MCG_NEST_TRACE build in lib/libmcg_trace.so, when present).
mkdir -p gpurun_out/c3fm
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_nested.py -k "one_launch or alternate or batched" > gpurun_out/c3fm/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/c3fm/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in fm two; do
    if [ $v = fm ]; then export MCG_NESTED_FM=1; else unset MCG_NESTED_FM; fi
    timeout -k 10 300 python3 scripts/bench_configs.py c3 --reps 3 --out gpurun_out/c3fm/$v.jsonl > gpurun_out/c3fm/$v$i.log 2>&1 || { echo "$v rc=$?"; exit 1; }
    python3 -c "import json;l=json.loads(open('gpurun_out/c3fm/$v.jsonl').read().splitlines()[-1]);print('$v', '%.4g'%l['value'], l['wall_s_runs'], l['n_gen'], l['log_evidence']['abs_delta'], l['log_evidence']['sigma_H'])"
  done
done
unset MCG_NESTED_FM
if [ -f mcmc-ocaml_amd/lib/libmcg_trace.so ]; then
  for v in 1 0; do
    MCG_NESTED_FM=$v MCG_LIBRARY=$PWD/mcmc-ocaml_amd/lib/libmcg_trace.so MCG_NEST_TRACE=200 timeout -k 10 120 python3 scripts/probes/c3_once.py > gpurun_out/c3fm/stamps$v.log 2>&1 || exit 1
    grep "trace gen" gpurun_out/c3fm/stamps$v.log | tail -12
  done
fi
