#!/bin/bash
# A/B of library variants on the C3 config (walk launch time from HIP events, wall over reps):
#   bash scripts/gpu_c3_ab.sh libmcg.so libmcg_x.so ...
mkdir -p gpurun_out/c3ab
export PYTHONUNBUFFERED=1
for round in 1 2; do
  for lib in "$@"; do
    MCG_LIBRARY=$PWD/mcmc-ocaml_amd/lib/$lib timeout -k 10 200 python scripts/bench_configs.py c3 --reps 3 --out gpurun_out/c3ab/$lib.$round.jsonl > gpurun_out/c3ab/$lib.$round.log 2>&1 || exit $?
  done
done
python3 - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/c3ab/*.jsonl")):
    d = json.loads(open(f).read().strip().split("\n")[-1])
    print("%-40s walk %.2f us  wall %.4f s  value %.3g  logZ %.5f" % (f.split("/")[-1], d["roofline"]["avg_launch_ms"] * 1e3, d["wall_s"], d["value"], d["log_evidence"]["nested"]))
PY
