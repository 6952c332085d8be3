#!/bin/bash
# grouped kD records: kD tests, then C4 A/B against the previous library (lib/libmcg_prev.so)
OUT=gpurun_out/r6_c4rec; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_any_dim.py tests/test_gpu_mh.py tests/test_gpu_fuzz.py tests/test_gpu_gauss_prior.py \
  tests/test_gpu_fullsize.py -k "kd or Kd or KD or c4 or any_dim or padded" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2 3; do
  for v in prev new; do
    if [ $v = prev ]; then export MCG_LIBRARY=$PWD/mcmc-ocaml_amd/lib/libmcg_prev.so; else unset MCG_LIBRARY; fi
    timeout -k 10 120 python3 scripts/bench_configs.py c4 --launches 100 --out $OUT/c4_${v}_$i.jsonl > $OUT/c4_${v}_$i.log 2>&1 || exit 1
    python3 -c "import json;d=json.loads(open('$OUT/c4_${v}_$i.jsonl').read().splitlines()[-1]);print('$v', '%.4g'%d['value'], d['roofline_hbm']['avg_launch_ms'])"
  done
done
