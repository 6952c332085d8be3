#!/bin/bash
# C4 A/B on one box: the round-6-start library (lib/libmcg_base.so, built from commit 6ab13ef)
# against the current one, alternated three times
OUT=gpurun_out/r6_c4ab; mkdir -p $OUT
for i in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then export MCG_LIBRARY=$PWD/mcmc-ocaml_amd/lib/libmcg_base.so; else unset MCG_LIBRARY; fi
    timeout -k 10 120 python3 scripts/bench_configs.py c4 --launches 100 --out $OUT/c4_${v}_$i.jsonl > $OUT/c4_${v}_$i.log 2>&1 || exit 1
    python3 -c "import json;d=json.loads(open('$OUT/c4_${v}_$i.jsonl').read().splitlines()[-1]);print('$v', '%.4g'%d['value'], d['roofline_hbm']['avg_launch_ms'])"
  done
done
