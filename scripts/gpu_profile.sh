#!/bin/bash
# rocprofv3 kernel-trace stats of the bench, then separate PMC passes (FETCH_SIZE, WRITE_SIZE, VALU issue)
# of the same MH launches (the PMC passes skip the nested leg, which holds no MH launch).
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
ARGS="--steps 10 --warmup 1 --no-cpu-baseline $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/fetch -o run --output-format csv -- python3 bench.py $ARGS --nested-nlive 0 > gpurun_out/prof/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/write -o run --output-format csv -- python3 bench.py $ARGS --nested-nlive 0 > gpurun_out/prof/write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/prof/valu -o run --output-format csv -- python3 bench.py $ARGS --nested-nlive 0 > gpurun_out/prof/valu.log 2>&1 || exit $?
echo profile-ok
python3 scripts/pmc_traffic.py gpurun_out/prof gpurun_out/prof/pmc_traffic.json
python3 scripts/pmc_valu.py gpurun_out/prof gpurun_out/prof/pmc_valu.json
python3 scripts/trace_summary.py gpurun_out/prof/trace/run_kernel_trace.csv gpurun_out/prof/trace_summary.json
