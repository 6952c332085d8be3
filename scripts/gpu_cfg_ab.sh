#!/bin/bash
# A/B of library variants on one bench_configs config: bash scripts/gpu_cfg_ab.sh c5 libA.so libB.so ...
cfg=$1; shift
mkdir -p gpurun_out/cfgab
for round in 1 2; do
  for lib in "$@"; do
    MCG_LIBRARY=$PWD/mcmc-ocaml_amd/lib/$lib timeout -k 10 200 python scripts/bench_configs.py $cfg --out gpurun_out/cfgab/$cfg.$lib.$round.jsonl > gpurun_out/cfgab/$cfg.$lib.$round.log 2>&1 || exit $?
  done
done
python3 - "$cfg" <<'PY'
import glob, json, sys
for f in sorted(glob.glob("gpurun_out/cfgab/%s.*.jsonl" % sys.argv[1])):
    d = json.loads(open(f).read().strip().split("\n")[-1])
    print("%-45s value %.4g  %s" % (f.split("/")[-1], d["value"], {k: d[k] for k in ("accept_frac", "posterior_check") if k in d}))
PY
