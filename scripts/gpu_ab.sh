#!/bin/bash
# A/B bench of library variants (interleaved, 2 rounds):
#   bash scripts/gpu_ab.sh libmcg.so libmcg_w3.so@MCG_LANES_PER_CHAIN=8 ...
# each spec is a library file under mcmc-ocaml_amd/lib, optionally followed by @VAR=VALUE[@...]
mkdir -p gpurun_out/ab
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest tests/test_gpu_mh.py -q -x > gpurun_out/ab/pytest.log 2>&1 || exit $?
for round in 1 2; do
  for spec in "$@"; do
    lib=${spec%%@*}
    envs=""
    [ "$spec" != "$lib" ] && envs=$(echo "${spec#*@}" | tr '@' ' ')
    name=$(echo "$spec" | tr '@=/' '___')
    env $envs MCG_LIBRARY=$PWD/mcmc-ocaml_amd/lib/$lib timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/ab/$name.$round.json 2>&1 || exit $?
  done
done
echo ab-done
