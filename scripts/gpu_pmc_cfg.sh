#!/bin/bash
# VALU-issue PMC pass (SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE) of the C4 and C5 config kernels,
# then two detail passes per config (instruction mix, waits, LDS conflicts).  One counter group
# per rocprofv3 run, each under its own time limit.
mkdir -p gpurun_out/pmc_cfg
export TMPDIR=/tmp PYTHONUNBUFFERED=1
declare -A RX=([c4]="mh_kernel<8," [c5]="fullcov")
for c in ${CFGS:-c4 c5}; do
  timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/pmc_cfg/$c/valu -o run --output-format csv -- python3 scripts/bench_configs.py $c --launches 20 > gpurun_out/pmc_cfg/$c.log 2>&1 || exit 1
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY" \
             "SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-include-regex "${RX[$c]}" -d gpurun_out/pmc_cfg/$c/p$i -o run --output-format csv -- python3 scripts/bench_configs.py $c --launches 5 > gpurun_out/pmc_cfg/${c}_p$i.log 2>&1 || { echo "$c pass $i failed"; exit 1; }
  done
done
python3 scripts/pmc_valu.py gpurun_out/pmc_cfg/c4 gpurun_out/pmc_cfg/pmc_valu_c4.json --kernel "mh_kernel<8," --ndim 8 --chains 32768 --sweeps 1000 || true
python3 scripts/pmc_valu.py gpurun_out/pmc_cfg/c5 gpurun_out/pmc_cfg/pmc_valu_c5.json --kernel "mh_fullcov_kernel<64" --ndim 64 --chains 131072 --sweeps 500 || true
python3 scripts/pmc_summary.py gpurun_out/pmc_cfg/c4 > gpurun_out/pmc_cfg/c4_summary.txt 2>&1 || true
python3 scripts/pmc_summary.py gpurun_out/pmc_cfg/c5 fullcov > gpurun_out/pmc_cfg/c5_summary.txt 2>&1 || true
echo pmc-cfg-ok
