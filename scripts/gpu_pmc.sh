#!/bin/bash
# PMC passes for the MH kernel (one counter group per pass, kernel-trace only)
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
ARGS="--steps 5 --warmup 1 --no-cpu-baseline --nested-seeds 0 $*"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY" \
           "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_SMEM" \
           "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp -d gpurun_out/pmc/p$i -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc/p$i.log 2>&1 || echo "pass $i rc=$?" >> gpurun_out/pmc/status.txt
done
# keep only the MH kernel rows (the nested leg adds thousands of launches)
for f in gpurun_out/pmc/p*/run_counter_collection.csv; do
  (head -1 "$f"; grep mh_kernel "$f") > "$f.mh" && mv "$f.mh" "$f"
done
echo pmc-done
