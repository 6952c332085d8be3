#!/bin/bash
# Round 6: the split merge (head kernel + tail in the next walk).  Nested GPU tests, then C3
# with MCG_NESTED_SPLIT=0/1 alternated on one box, then a kernel trace of the split C3 run.
set -o pipefail
OUT=gpurun_out/r6_split; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_nested.py -x -q -m gpu -rf --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for sp in 0 1; do
    MCG_NESTED_SPLIT=$sp timeout -k 10 300 python scripts/bench_configs.py c3 --out $OUT/c3_s${sp}_${rep}.jsonl > $OUT/c3_s${sp}_${rep}.log 2>&1
    rc=$?; echo "c3 split=$sp rep=$rep rc=$rc"; [ $rc -eq 0 ] || exit $rc
    python -c "import json;d=json.loads(open('$OUT/c3_s${sp}_${rep}.jsonl').read().splitlines()[-1]);print('split',$sp,d.get('value'),d['log_evidence']['nested'],d.get('n_gen'))"
  done
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o c3 -- python scripts/bench_configs.py c3 --out $OUT/c3_prof.jsonl > $OUT/prof.log 2>&1
echo "prof rc=$?"
