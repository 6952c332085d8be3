#!/bin/bash
# PMC passes (one counter group per pass, kernel-trace only) over the C3 nested run
mkdir -p gpurun_out/pmc_c3
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY" \
           "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-include-regex "nest_walk" -d gpurun_out/pmc_c3/p$i -o run --output-format csv -- python3 scripts/probes/nested_breakdown.py > gpurun_out/pmc_c3/p$i.log 2>&1 || { echo "pass $i rc=$?"; exit 1; }
done
echo pmc-done
