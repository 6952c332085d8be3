#!/bin/bash
# Round 6, end of session on the final tree: the whole GPU suite, smoke, bench.py with its
# defaults and with the driver's flags, the rocprofv3 kernel trace of the default bench, and the
# BASELINE config lines (C1-C5).  Every GPU step under its own time limit; stop at the first failure.
OUT=gpurun_out/r6_end; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit $?
tail -2 $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench_default.log 2>&1 || exit $?
grep '^{"metric"' $OUT/bench_default.log > $OUT/bench_line_default.json
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || exit $?
grep '^{"metric"' $OUT/bench.log > $OUT/bench_line.json
for f in bench_line_default bench_line; do
  python3 -c "import json; d=json.load(open('$OUT/$f.json')); print('$f', '%.4g' % d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'])"
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py > $OUT/prof.log 2>&1 || exit 1
grep '^{"metric"' $OUT/prof.log > $OUT/bench_line_under_rocprof.json || true
timeout -k 10 900 python3 scripts/bench_configs.py c1 c2 c3 c3k8 c3n1k c4 c5 --out $OUT/configs.jsonl > $OUT/configs.log 2>&1 || exit 1
python3 -c "
import json
for l in open('$OUT/configs.jsonl'):
    d=json.loads(l); c=d['config']; c=c if isinstance(c, str) else c.get('workload')
    print(c[:70], '%.4g' % d['value'], d.get('roofline', {}).get('frac'))"
echo end-ok
