#!/bin/bash
# The whole GPU suite (one process, per-test time limit), then the smoke check.
OUT=gpurun_out/r6_suite; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -rf --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; grep -E "PASSED|FAILED" $OUT/pytest.log | grep -c PASSED; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; tail -2 $OUT/smoke.log; exit $rc
