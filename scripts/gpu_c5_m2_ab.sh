#!/bin/bash
# C5 A/B: Welford M2 accumulators in LDS (MCG_FC_M2LDS=1), alone and with the normals gathered one
# ahead (MCG_FC_PIPE=1), against the default build; fullcov / C5 GPU tests on the first variant.
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
MCG_LIBRARY=$PWD/mcmc-ocaml_amd/lib/ab/libmcg_m2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_mh.py tests/test_gpu_fullsize.py -v -m gpu -k "fullcov or c5" --timeout 120 --timeout-method thread > gpurun_out/m2_tests.log 2>&1 || { tail -20 gpurun_out/m2_tests.log; exit 1; }
tail -1 gpurun_out/m2_tests.log
bash scripts/gpu_lib_ab.sh c5 mcmc-ocaml_amd/lib/ab/libmcg_base.so mcmc-ocaml_amd/lib/ab/libmcg_m2.so > gpurun_out/ab_m2.txt 2>&1 || exit 1
cat gpurun_out/ab_m2.txt
bash scripts/gpu_lib_ab.sh c5 mcmc-ocaml_amd/lib/ab/libmcg_base.so mcmc-ocaml_amd/lib/ab/libmcg_m2p.so > gpurun_out/ab_m2p.txt 2>&1 || exit 1
cat gpurun_out/ab_m2p.txt
