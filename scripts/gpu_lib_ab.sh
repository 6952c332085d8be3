#!/bin/bash
# Same-box A/B of two builds of libmcg on one bench_configs config, alternating A B A B:
#   bash scripts/gpu_lib_ab.sh <config> <libA> <libB>
# prints value and the dominant kernel's average launch time per run
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cfg=$1; A=$2; B=$3
for i in 1 2; do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    MCG_LIBRARY=$PWD/$lib timeout -k 10 240 python scripts/bench_configs.py $cfg > gpurun_out/ab_${cfg}_$v$i.log 2>&1 || { tail -5 gpurun_out/ab_${cfg}_$v$i.log; exit 1; }
    python -c "
import json;d=json.loads(open('gpurun_out/ab_${cfg}_$v$i.log').read().strip().splitlines()[-1]);print('$v$i %s %.4g kernel %.4f ms' % ('$cfg', d['value'], d['roofline']['avg_launch_ms']))"
  done
done
