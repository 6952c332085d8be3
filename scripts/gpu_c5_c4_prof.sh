#!/bin/bash
# C5's sharded form rehearsed on one GPU (scripts/bench_c5.py with 1, 2 and 4 gloo ranks over the
# same 524,288 global chains: the moments digests must agree), the C5 per-GPU weak line, and the
# VALU PMC passes of the C4 / C5 config kernels.
mkdir -p gpurun_out/c5r gpurun_out/pmc_cfg
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for w in 1 2 4; do
  MCG_BENCH_BACKEND=gloo MCG_BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $w \
    --master-addr 127.0.0.1 --master-port $((29600 + w)) scripts/bench_c5.py --gpus $w --total-chains 524288 --steps 4 --warmup 1 \
    --out gpurun_out/c5r/rehearsal.jsonl > gpurun_out/c5r/w$w.log 2>&1 || { tail -20 gpurun_out/c5r/w$w.log; exit 1; }
  tail -1 gpurun_out/c5r/rehearsal.jsonl | cut -c1-200
done
timeout -k 10 300 python scripts/bench_c5.py --steps 10 --warmup 1 --out gpurun_out/c5r/weak1.jsonl > gpurun_out/c5r/weak1.log 2>&1 || exit 1
tail -1 gpurun_out/c5r/weak1.jsonl | cut -c1-300
for c in c4 c5; do
  timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/pmc_cfg/$c/valu -o run --output-format csv -- python3 scripts/bench_configs.py $c --launches 20 > gpurun_out/pmc_cfg/$c.log 2>&1 || exit 1
done
python3 scripts/pmc_valu.py gpurun_out/pmc_cfg/c4 gpurun_out/pmc_cfg/pmc_valu_c4.json --kernel "mh_kernel<8," --ndim 8 --chains 32768 --sweeps 1000
python3 scripts/pmc_valu.py gpurun_out/pmc_cfg/c5 gpurun_out/pmc_cfg/pmc_valu_c5.json --kernel "mh_fullcov_kernel<64" --ndim 64 --chains 131072 --sweeps 500
