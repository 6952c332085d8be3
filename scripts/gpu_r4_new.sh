#!/bin/bash
# The round-4 parity tests (RCCL, mixture), then the whole GPU suite.
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_rccl.py "tests/test_gpu_gauss_mix.py::test_gauss_mix_mh_bit_exact" \
  -v -rf --timeout 150 --timeout-method thread > gpurun_out/pytest_new.log 2>&1
rc=$?
echo "new tests rc=$rc" | tee -a gpurun_out/status.log
if [ $rc -ge 2 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -q -m gpu -rf --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "gpu suite rc=$rc" | tee -a gpurun_out/status.log
exit $rc
