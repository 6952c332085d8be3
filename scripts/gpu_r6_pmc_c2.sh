#!/bin/bash
# C2 VALU-issue PMC pass on the final library (SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE) ->
# gpurun_out/pmc_c2/pmc_valu.json (the bench line's `roofline.valu` source)
mkdir -p gpurun_out/pmc_c2
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/pmc_c2/valu -o run --output-format csv -- \
  python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --nested-seeds 0 > gpurun_out/pmc_c2/run.log 2>&1 || exit 1
python3 scripts/pmc_valu.py gpurun_out/pmc_c2 gpurun_out/pmc_c2/pmc_valu.json --kernel "mh_kernel<32" --ndim 32 --chains 65536 --sweeps 1000 && cat gpurun_out/pmc_c2/pmc_valu.json
