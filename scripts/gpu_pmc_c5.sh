#!/bin/bash
# PMC passes over the C5 full-covariance run (kernel-trace + one counter group per pass)
mkdir -p gpurun_out/pmc_c5
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc_c5/trace -o run --output-format csv -- python3 scripts/bench_configs.py c5 --launches 5 --out gpurun_out/pmc_c5/c5.jsonl > gpurun_out/pmc_c5/trace.log 2>&1 || exit 1
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY" \
           "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-include-regex "fullcov" -d gpurun_out/pmc_c5/p$i -o run --output-format csv -- python3 scripts/bench_configs.py c5 --launches 5 --out gpurun_out/pmc_c5/c5_p$i.jsonl > gpurun_out/pmc_c5/p$i.log 2>&1 || { echo "pass $i rc=$?"; exit 1; }
done
echo pmc-done
