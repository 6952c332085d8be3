#!/bin/bash
# C2 MH throughput against the chain count (tail of the last dispatch round):
#   bash scripts/gpu_chains_sweep.sh [chains ...]
# 65,536 chains at P = 4 are 4,096 waves; at three waves per SIMD one dispatch round holds 3,072
mkdir -p gpurun_out/sweep
export PYTHONUNBUFFERED=1
set -o pipefail
chains=${*:-49152 65536 73728 98304 131072 196608}
for n in $chains; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 3 --chains $n --no-cpu-baseline \
    --nested-seeds 0 --nested-nlive 0 > gpurun_out/sweep/c$n.json 2>&1 || exit $?
done
python3 - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/sweep/c*.json"), key=lambda s: int(s.split("/c")[-1][:-5])):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    print("%-10s %.4g steps/s  launch %.4f ms  frac %.3f" % (f.split("/")[-1], d["value"], d["roofline"]["avg_launch_ms"], d["roofline"]["frac"]))
PY
