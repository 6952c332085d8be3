#!/bin/bash
# Round 5: the multi-rank bench entry point on one GPU (bench.py --gpus 2 self-launch over gloo,
# the C5 runner's 1-vs-2-rank digest), then the bench under rocprofv3 with the driver's exact flags
# (--steps 20 --warmup 5), so the line's roofline frac can be reproduced from profiles/.
mkdir -p gpurun_out/r5launch
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_bench_launch.py tests/test_gpu_c5_shards.py > gpurun_out/r5launch/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r5launch/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5launch/driver_flags -o run --output-format csv \
  -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5launch/driver_flags.log 2>&1
rc=$?; tail -c 600 gpurun_out/r5launch/driver_flags.log; exit $rc
