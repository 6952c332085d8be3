#!/bin/bash
# C3 same-box A/B of two libmcg builds: nested GPU tests on B, then per library (A B A B) the
# kernel-trace medians of the walk and merge kernels and the C3 line.
#   bash scripts/gpu_c3_lib_ab.sh <libA> <libB>
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
A=$1; B=$2
MCG_LIBRARY=$PWD/$B timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nested.py > gpurun_out/ab_nt.log 2>&1 || { tail -20 gpurun_out/ab_nt.log; exit 1; }
tail -1 gpurun_out/ab_nt.log
for i in 1 2; do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    rm -rf gpurun_out/ab_tr_$v$i
    MCG_LIBRARY=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/ab_tr_$v$i -o run --output-format csv -- python3 scripts/probes/c3_once.py > gpurun_out/ab_tr_$v$i.log 2>&1 || exit 1
    MCG_LIBRARY=$PWD/$lib timeout -k 10 240 python scripts/bench_configs.py c3 --reps 5 > gpurun_out/ab_c3_$v$i.log 2>&1 || exit 1
    python3 - "$v$i" <<'PY'
import csv, json, statistics as st, sys, glob
tag = sys.argv[1]
f = glob.glob("gpurun_out/ab_tr_%s/**/run_kernel_trace.csv" % tag, recursive=True)[0]
d = {}
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"]
    k = "walk" if "nest_walk" in n else "merge" if "merge_fused" in n else None
    if k: d.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
c3 = json.loads(open("gpurun_out/ab_c3_%s.log" % tag).read().strip().splitlines()[-1])
print(tag, "walk med %.2f us, merge med %.2f us, C3 %.4g" % (st.median(d["walk"]), st.median(d["merge"]), c3["value"]),
      [round(x * 1e3, 1) for x in c3["wall_s_runs"]])
PY
  done
done
