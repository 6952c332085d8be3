#!/bin/bash
# C4 latency probe: throughput per chain-step at 32K / 64K / 128K chains and 2 / 4 lanes per chain
OUT=gpurun_out/r6_c4scan; mkdir -p $OUT
for n in 32768 65536 131072; do
  for l in 4 2; do
    MCG_LANES_PER_CHAIN=$l timeout -k 10 120 python3 scripts/bench_configs.py c4 --c4-chains $n --launches 50 --out $OUT/c4_${n}_$l.jsonl > $OUT/c4_${n}_$l.log 2>&1 || exit 1
    python3 -c "import json;d=json.loads(open('$OUT/c4_${n}_$l.jsonl').read().splitlines()[-1]);print($n, $l, '%.4g'%d['value'], d['roofline_hbm']['avg_launch_ms'])"
  done
done
