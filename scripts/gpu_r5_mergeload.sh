#!/bin/bash
# (needs lib/libmcg_trace.so: the nested objects rebuilt with -DMCG_NEST_TRACE and linked beside the rest, as in LABLOG round 5)
# Round 5, C3: merge workgroups of 512 survivors at k <= 4096 (half the workgroups, so half the
# new-key classification) -- nested parity, then a same-box A/B of the C3 line against
# MCG_MERGE_BS=256, alternated, then the phase stamps of generation 200 for both from
# lib/libmcg_trace.so (MCG_NEST_TRACE build)
mkdir -p gpurun_out/mload
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_nested.py tests/test_gpu_gauss_prior.py tests/test_gpu_fuzz.py -k "nested" > gpurun_out/mload/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/mload/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for v in 512 256; do
    MCG_MERGE_BS=$v timeout -k 10 300 python3 scripts/bench_configs.py c3 --reps 3 --out gpurun_out/mload/bs$v.jsonl > gpurun_out/mload/bs$v-$i.log 2>&1 || { echo "$v rc=$?"; exit 1; }
    python3 -c "import json;l=json.loads(open('gpurun_out/mload/bs$v.jsonl').read().splitlines()[-1]);print('bs$v', '%.4g'%l['value'], l['wall_s_runs'], l['n_gen'], l['log_evidence']['abs_delta'])"
  done
done
for v in 512 256; do
  MCG_MERGE_BS=$v MCG_LIBRARY=$PWD/mcmc-ocaml_amd/lib/libmcg_trace.so MCG_NEST_TRACE=200 timeout -k 10 120 python3 scripts/probes/c3_once.py > gpurun_out/mload/stamps$v.log 2>&1 || exit 1
  echo "bs $v"; grep "trace gen" gpurun_out/mload/stamps$v.log | tail -14
done
