#!/bin/bash
# C2 A/B on one box: libmcg_u0.so (step loop not unrolled) against libmcg.so (unrolled by P),
# alternated three times with the driver's bench flags
OUT=gpurun_out/r6_c2ab; mkdir -p $OUT
for i in 1 2 3; do
  for v in u0 u1; do
    if [ $v = u0 ]; then export MCG_LIBRARY=$PWD/mcmc-ocaml_amd/lib/libmcg_u0.so; else unset MCG_LIBRARY; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/b_${v}_$i.log 2>&1 || exit 1
    grep '^{"metric"' $OUT/b_${v}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', '%.4g' % d['value'], d['roofline']['avg_launch_ms'])"
  done
done
