#!/bin/bash
# Round 6 (c): nested GPU tests, C3 split vs one-launch merge alternated (3 rounds), kernel trace
set -o pipefail
OUT=gpurun_out/r6_f; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_nested.py -x -q -m gpu -rf --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for sp in 0 1; do
    MCG_NESTED_SPLIT=$sp timeout -k 10 300 python scripts/bench_configs.py c3 --out $OUT/c3_s${sp}_${rep}.jsonl > $OUT/c3_s${sp}_${rep}.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "c3 rc=$rc"; exit $rc; }
    python -c "import json;d=json.loads(open('$OUT/c3_s${sp}_${rep}.jsonl').read().splitlines()[-1]);print('split',$sp,'%.4g'%d['value'],d['log_evidence']['nested'],d['n_gen'])"
  done
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o c3 --output-format csv -- python3 scripts/probes/c3_once.py > $OUT/prof.log 2>&1
echo "prof rc=$?"
python3 - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/r6_f/prof/**/*kernel_stats.csv', recursive=True)
for r in csv.DictReader(open(f[0])):
    print('%-60s %8s %10.2f' % (r['Name'][:60], r['Calls'], float(r['AverageNs']) / 1000))
PY
