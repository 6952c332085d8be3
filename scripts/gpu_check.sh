#!/bin/bash
# One GPU-box session: parity tests, smoke, short bench.  Each GPU step has its own time limit;
# a crash / timeout (exit >= 2 from pytest, or any signal) stops the script.
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -v -s -m gpu -rf --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" | tee -a gpurun_out/status.log
if [ $rc -ge 2 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?
echo "smoke rc=$rc" | tee -a gpurun_out/status.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py "$@" > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc" | tee -a gpurun_out/status.log
exit $rc
