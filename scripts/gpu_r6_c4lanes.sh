#!/bin/bash
# C4 at its configured 32,768 chains on 4 and 2 lanes a chain (grouped kD step), alternated
OUT=gpurun_out/r6_c4lanes; mkdir -p $OUT
for i in 1 2; do
  for l in 4 2; do
    MCG_LANES_PER_CHAIN=$l timeout -k 10 120 python3 scripts/bench_configs.py c4 --launches 100 --out $OUT/c4_${l}_$i.jsonl > $OUT/c4_${l}_$i.log 2>&1 || exit 1
    python3 -c "import json;d=json.loads(open('$OUT/c4_${l}_$i.jsonl').read().splitlines()[-1]);print($l, '%.4g'%d['value'], d['roofline_hbm']['avg_launch_ms'])"
  done
done
