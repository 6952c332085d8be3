#!/bin/bash
# C2 with the step loop unrolled by P (experiment): C2 parity tests, then the bench twice
OUT=gpurun_out/r6_c2u; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mh.py -k "c2 or staggered or lanes" > $OUT/t.log 2>&1 || { tail -20 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/b$i.log 2>&1 || exit 1
  grep '^{"metric"' $OUT/b$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.4g' % d['value'], d['roofline']['avg_launch_ms'])"
done
