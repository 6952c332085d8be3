#!/bin/bash
# (record of a round-5 experiment: needs the tree of commit a349d96, whose C5 variants and
# timing-probe macros were removed afterwards; see profiles/r05/c5_datapath)
# Round 5, C5: the full-covariance parity tests on the default (software-pipelined) kernel, then
# a same-box A/B of the C5 config line: pipelined step vs the round-4 step (MCG_FC_KERNEL=1),
# alternated twice.
mkdir -p gpurun_out/c5ab
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_mh.py tests/test_gpu_c5_shards.py tests/test_gpu_any_dim.py tests/test_gpu_fullsize.py -k "fullcov or c5 or C5" > gpurun_out/c5ab/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/c5ab/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in pipe v1; do
    if [ $v = v1 ]; then export MCG_FC_KERNEL=1; else unset MCG_FC_KERNEL; fi
    timeout -k 10 200 python3 scripts/bench_configs.py c5 --launches 40 --out gpurun_out/c5ab/$v.jsonl > gpurun_out/c5ab/$v$i.log 2>&1 || { echo "$v rc=$?"; exit 1; }
    python3 -c "import json;l=json.loads(open('gpurun_out/c5ab/$v.jsonl').read().splitlines()[-1]);print('$v', l['value'], l['roofline_hbm']['avg_launch_ms'], l['posterior_check'])"
  done
done
unset MCG_FC_KERNEL
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/c5ab/trace -o run --output-format csv -- python3 scripts/bench_configs.py c5 --launches 10 > gpurun_out/c5ab/trace.log 2>&1 || exit 1
grep -h fullcov gpurun_out/c5ab/trace/run_kernel_stats.csv | cut -c1-200
