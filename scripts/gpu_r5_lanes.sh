#!/bin/bash
# Round 5, C3: the walker's lane split re-measured on the current walker (draw table, in-walk
# retirement): 4 lanes x 4 dims (default at D 16) against 8 lanes x 2 dims (MCG_NEST_LANES=wide,
# 512 walker waves, two per draw-table workgroup), same box, alternated
mkdir -p gpurun_out/lanes
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for i in 1 2; do
  for v in narrow wide; do
    MCG_NEST_LANES=$v timeout -k 10 300 python3 scripts/bench_configs.py c3 c3k8 --reps 3 --out gpurun_out/lanes/$v.jsonl > gpurun_out/lanes/$v$i.log 2>&1 || { echo "$v rc=$?"; exit 1; }
  done
done
python3 - <<'PY'
import json
for v in ("narrow", "wide"):
    for l in open("gpurun_out/lanes/%s.jsonl" % v):
        d = json.loads(l)
        print(v, d["config"][:40], "%.4g" % d["value"], d["roofline"].get("avg_launch_ms"))
PY
