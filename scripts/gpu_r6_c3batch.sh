#!/bin/bash
# C3 (k 4,096, nmcmc 100) at generation-batch caps 64 (default) / 32 / 16, alternated twice
OUT=gpurun_out/r6_c3batch; mkdir -p $OUT
for i in 1 2; do
  for b in ${BATCHES:-64 32 16}; do
    MCG_NESTED_MAX_BATCH=$b timeout -k 10 200 python3 scripts/bench_configs.py c3 --out $OUT/c3_${b}_$i.jsonl > $OUT/c3_${b}_$i.log 2>&1 || exit 1
    python3 -c "import json;d=json.loads(open('$OUT/c3_${b}_$i.jsonl').read().splitlines()[-1]);print($b, '%.4g'%d['value'])"
  done
done
