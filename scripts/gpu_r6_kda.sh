#!/bin/bash
# kD prefetch depth: the kD bit-exact tests, then C4 at its configured 32,768 chains
OUT=gpurun_out/r6_kda; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_any_dim.py tests/test_gpu_mh.py tests/test_gpu_fuzz.py tests/test_gpu_gauss_prior.py \
  tests/test_gpu_fullsize.py -k "kd or Kd or KD or c4 or any_dim or padded" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
for i in 1 2; do
  timeout -k 10 120 python3 scripts/bench_configs.py c4 --launches 100 --out $OUT/c4_$i.jsonl > $OUT/c4_$i.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('$OUT/c4_$i.jsonl').read().splitlines()[-1]);print('%.4g'%d['value'], d['roofline_hbm']['avg_launch_ms'], d['accept_frac'])"
done
