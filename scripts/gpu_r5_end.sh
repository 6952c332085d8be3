#!/bin/bash
# Round 5, end of session on the final tree: the whole GPU suite, smoke, the bench with the
# driver's flags, the C3 config lines, and the kernel trace of C3 (walk / merge averages)
mkdir -p gpurun_out/end
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 150 --timeout-method thread > gpurun_out/end/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/end/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/end/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/end/smoke.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/end/bench.log 2>&1 || exit $?
grep '^{"metric"' gpurun_out/end/bench.log > gpurun_out/end/bench_line.json
python3 -c "import json; d=json.load(open('gpurun_out/end/bench_line.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 400 python3 scripts/bench_configs.py c3 c3k8 c3n1k --out gpurun_out/end/configs_c3.jsonl > gpurun_out/end/configs_c3.log 2>&1 || exit 1
python3 -c "
import json
for l in open('gpurun_out/end/configs_c3.jsonl'):
    d=json.loads(l); print(d['config'] if isinstance(d['config'], str) else d['config'].get('workload'), '%.4g' % d['value'], d['roofline'].get('frac'))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/end/trace -o run --output-format csv -- \
  python3 scripts/bench_configs.py c3 --out gpurun_out/end/trace_configs.jsonl > gpurun_out/end/trace.log 2>&1 || exit 1
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/end/trace/run_kernel_stats.csv")):
    if any(k in r["Name"] for k in ("nest_walk", "merge_fused")):
        print("%-60s %8s calls %10.2f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1000))
PY
