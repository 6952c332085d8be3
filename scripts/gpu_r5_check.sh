#!/bin/bash
# Round 5, end of session: the whole GPU suite, smoke, and the bench with the driver's flags
mkdir -p gpurun_out/check
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rf --timeout 150 --timeout-method thread > gpurun_out/check/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/check/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/check/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/check/smoke.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/check/bench.log 2>&1 || exit $?
grep '^{"metric"' gpurun_out/check/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'])"
