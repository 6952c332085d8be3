#!/bin/bash
# Round 5, C5 attribution: the C5 config line with the product library and with two timing-probe
# builds of the normal-table gathers (wrong values, timing only): BCAST (every lane gathers row 0:
# the same LDS instructions without bank conflicts) and NOLDS (no gathers).  Then one PMC pass
# per build (LDS conflict / wait / VALU counters of mh_fullcov_kernel).
mkdir -p gpurun_out/c5probe
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
L=mcmc-ocaml_amd/lib
for v in base bcast nolds; do
  lib=$L/libmcg.so; [ $v != base ] && lib=$L/libmcg_probe_$v.so
  MCG_LIBRARY=$PWD/$lib timeout -k 10 200 python3 scripts/bench_configs.py c5 --launches 40 --out gpurun_out/c5probe/$v.jsonl > gpurun_out/c5probe/$v.log 2>&1 || { echo "$v rc=$?"; exit 1; }
  python3 -c "import json;l=json.loads(open('gpurun_out/c5probe/$v.jsonl').read().splitlines()[-1]);print('$v', l['value'], l['roofline_hbm']['avg_launch_ms'])"
done
for v in base bcast nolds; do
  lib=$L/libmcg.so; [ $v != base ] && lib=$L/libmcg_probe_$v.so
  MCG_LIBRARY=$PWD/$lib timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_LDS \
    --kernel-include-regex fullcov -d gpurun_out/c5probe/pmc_$v -o run --output-format csv -- python3 scripts/bench_configs.py c5 --launches 5 > gpurun_out/c5probe/pmc_$v.log 2>&1 || { echo "pmc $v rc=$?"; exit 1; }
done
echo done
