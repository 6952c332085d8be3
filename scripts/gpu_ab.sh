#!/bin/bash
# A/B bench of library variants (interleaved, 2 rounds), after the MH parity tests of each:
#   bash scripts/gpu_ab.sh libmcg.so libmcg_w3.so@MCG_LANES_PER_CHAIN=8 ...
# each spec is a library file under mcmc-ocaml_amd/lib, optionally followed by @VAR=VALUE[@...]
mkdir -p gpurun_out/ab
export PYTHONUNBUFFERED=1
# parity tests of the first library only (the others may predate the current oracle spec)
for spec in "$1"; do
  lib=${spec%%@*}
  MCG_LIBRARY=$PWD/mcmc-ocaml_amd/lib/$lib timeout -k 10 300 python -m pytest tests/test_gpu_mh.py tests/test_golden.py -q -x -m gpu > gpurun_out/ab/pytest_$lib.log 2>&1 || { echo "pytest $lib failed"; tail -5 gpurun_out/ab/pytest_$lib.log; exit 1; }
done
for round in 1 2; do
  for spec in "$@"; do
    lib=${spec%%@*}
    envs=""
    [ "$spec" != "$lib" ] && envs=$(echo "${spec#*@}" | tr '@' ' ')
    name=$(echo "$spec" | tr '@=/' '___')
    env $envs MCG_LIBRARY=$PWD/mcmc-ocaml_amd/lib/$lib timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --nested-seeds 0 --nested-nlive 0 > gpurun_out/ab/$name.$round.json 2>&1 || exit $?
  done
done
python3 - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/ab/*.json")):
    try:
        d = json.loads([l for l in open(f) if l.startswith("{")][-1])
        print("%-50s %.4g steps/s  launch %.4f ms  frac %.3f" % (f.split("/")[-1], d["value"], d["roofline"]["avg_launch_ms"], d["roofline"]["frac"]))
    except Exception as e:
        print(f, "unreadable", e)
PY
