#!/bin/bash
# Round 5: the RCCL device-exchange tests, the C3 walk kernel's TCC / fabric-read PMC passes, and
# the config lines (C3 at k 4,096 with the Infinity-Cache framing, C4 / C5 with VALU primary).
mkdir -p gpurun_out/c3pmc
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_rccl.py \
  > gpurun_out/c3pmc/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/c3pmc/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_EA0_RDREQ_sum --kernel-include-regex nest_walk \
  -d gpurun_out/c3pmc/p1 -o run --output-format csv -- python3 scripts/probes/nested_breakdown.py > gpurun_out/c3pmc/p1.log 2>&1 || { echo "p1 rc=$?"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex nest_walk \
  -d gpurun_out/c3pmc/p2 -o run --output-format csv -- python3 scripts/probes/nested_breakdown.py > gpurun_out/c3pmc/p2.log 2>&1 || { echo "p2 rc=$?"; exit 1; }
python3 scripts/pmc_c3.py gpurun_out/c3pmc gpurun_out/c3pmc/pmc_c3_walk.json && cp gpurun_out/c3pmc/pmc_c3_walk.json profiles/pmc_c3_walk.json
timeout -k 10 600 python3 scripts/bench_configs.py c3 c4 c5 --out gpurun_out/c3pmc/configs.jsonl > gpurun_out/c3pmc/configs.log 2>&1
rc=$?; echo "configs rc=$rc"; exit $rc
