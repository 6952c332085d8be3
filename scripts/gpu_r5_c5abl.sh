#!/bin/bash
# (record of a round-5 experiment: needs the tree of commit a349d96, whose C5 variants and
# timing-probe macros were removed afterwards; see profiles/r05/c5_datapath)
# Round 5, C5 ablation (timing probes, wrong values): the round-4 step (MCG_FC_KERNEL=1) as built,
# with a VALU fma in place of each MFMA (NOMFMA), and with a 2-multiply hash in place of each
# Philox call (NOPHILOX); plus the product library's pipelined step for reference.
mkdir -p gpurun_out/c5abl
export PYTHONUNBUFFERED=1 TMPDIR=/tmp MCG_FC_KERNEL=1
L=$PWD/mcmc-ocaml_amd/lib
for i in 1 2; do
for v in base nomfma nophilox; do
  lib=$L/libmcg.so; [ $v != base ] && lib=$L/libmcg_probe_$v.so
  MCG_LIBRARY=$lib timeout -k 10 200 python3 scripts/bench_configs.py c5 --launches 40 --out gpurun_out/c5abl/$v.jsonl > gpurun_out/c5abl/$v$i.log 2>&1 || { echo "$v rc=$?"; exit 1; }
  python3 -c "import json;l=json.loads(open('gpurun_out/c5abl/$v.jsonl').read().splitlines()[-1]);print('$v', l['value'], l['roofline_hbm']['avg_launch_ms'])"
done
done
for v in nomfma nophilox; do
  MCG_LIBRARY=$L/libmcg_probe_$v.so timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_MFMA_F64 SQ_ACTIVE_INST_ANY \
    --kernel-include-regex fullcov -d gpurun_out/c5abl/pmc_$v -o run --output-format csv -- python3 scripts/bench_configs.py c5 --launches 5 > gpurun_out/c5abl/pmc_$v.log 2>&1 || { echo "pmc $v rc=$?"; exit 1; }
done
MCG_LIBRARY=$L/libmcg.so timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_MFMA_F64 SQ_ACTIVE_INST_ANY \
    --kernel-include-regex fullcov -d gpurun_out/c5abl/pmc_base -o run --output-format csv -- python3 scripts/bench_configs.py c5 --launches 5 > gpurun_out/c5abl/pmc_base.log 2>&1 || exit 1
echo done
