#!/bin/bash
# C2 launch time against sweeps per launch and chain count (fixed per-launch cost vs per-sweep cost)
mkdir -p gpurun_out/sweeps
export PYTHONUNBUFFERED=1
for n in ${CHAINS:-49152 65536}; do
  for s in ${SWEEPS:-25 50 100 200 400}; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 2 --chains $n --sweeps $s --no-cpu-baseline \
      --nested-seeds 0 --nested-nlive 0 > gpurun_out/sweeps/c${n}_s$s.json 2>&1 || exit $?
  done
done
python3 - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/sweeps/c*.json")):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    print("%-18s %.4g steps/s  launch %.4f ms  frac %.3f" % (f.split("/")[-1], d["value"], d["roofline"]["avg_launch_ms"], d["roofline"]["frac"]))
PY
