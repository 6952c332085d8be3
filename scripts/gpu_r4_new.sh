#!/bin/bash
# Round 4: the new parity tests first (mixture, padded widths, observer), then the whole GPU suite.
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_gauss_mix.py tests/test_gpu_any_dim.py \
  tests/test_gpu_rccl.py "tests/test_gpu_nested.py::test_nested_observer_sees_every_dead_point" -v -rf --timeout 150 \
  --timeout-method thread > gpurun_out/pytest_new.log 2>&1
rc=$?
echo "new tests rc=$rc" | tee -a gpurun_out/status.log
if [ $rc -ge 2 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -q -m gpu -rf --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "gpu suite rc=$rc" | tee -a gpurun_out/status.log
exit $rc
