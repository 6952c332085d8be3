#!/bin/bash
# 2-rank rehearsal of the bench's multi-rank flow on one GPU (gloo collectives), per library
mkdir -p gpurun_out
for lib in "$@"; do
  MCG_DEBUG_REPLICAS=1 MCG_LIBRARY=$PWD/mcmc-ocaml_amd/lib/$lib MCG_BENCH_BACKEND=gloo MCG_BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu-baseline --nested-seeds 0 > gpurun_out/reh_$lib.log 2>&1 || exit $?
done
