#!/bin/bash
# Round 5, C3: the nested parity tests on the fused walk + merge launch (default), then a same-box
# A/B of the C3 config line: fused (default) vs two launches (MCG_NESTED_FM=0), alternated.
mkdir -p gpurun_out/c3fm
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_nested.py tests/test_gpu_gauss_prior.py tests/test_gpu_gauss_mix.py tests/test_gpu_rccl.py > gpurun_out/c3fm/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/c3fm/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_mh.py tests/test_gpu_any_dim.py -k fullcov > gpurun_out/c3fm/pytest_fc.log 2>&1
rc=$?; tail -3 gpurun_out/c3fm/pytest_fc.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in fm two; do
    if [ $v = two ]; then export MCG_NESTED_FM=0; else unset MCG_NESTED_FM; fi
    timeout -k 10 300 python3 scripts/bench_configs.py c3 --reps 3 --out gpurun_out/c3fm/$v.jsonl > gpurun_out/c3fm/$v$i.log 2>&1 || { echo "$v rc=$?"; exit 1; }
    python3 -c "import json;l=json.loads(open('gpurun_out/c3fm/$v.jsonl').read().splitlines()[-1]);print('$v', '%.4g'%l['value'], l['wall_s_runs'], l['n_gen'], l['log_evidence']['abs_delta'], l['log_evidence']['sigma_H'])"
  done
done
unset MCG_NESTED_FM
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/c3fm/trace -o run --output-format csv -- python3 scripts/probes/nested_breakdown.py > gpurun_out/c3fm/trace.log 2>&1 || exit 1
head -6 gpurun_out/c3fm/trace/run_kernel_stats.csv | cut -c1-180
