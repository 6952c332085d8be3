mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
MCG_LIBRARY=$PWD/mcmc-ocaml_amd/lib/ab/libmcg_y16.so timeout -k 10 300 python -u -m pytest tests/test_gpu_mh.py tests/test_gpu_fullsize.py -v -m gpu -k "fullcov or c5" --timeout 120 --timeout-method thread > gpurun_out/y16_tests.log 2>&1 || { tail -20 gpurun_out/y16_tests.log; exit 1; }
tail -1 gpurun_out/y16_tests.log
bash scripts/gpu_lib_ab.sh c5 mcmc-ocaml_amd/lib/ab/libmcg_y0.so mcmc-ocaml_amd/lib/ab/libmcg_y16.so > gpurun_out/ab_y16.txt 2>&1 || exit 1
cat gpurun_out/ab_y16.txt
bash scripts/gpu_lib_ab.sh c5 mcmc-ocaml_amd/lib/ab/libmcg_y0.so mcmc-ocaml_amd/lib/ab/libmcg_y8.so > gpurun_out/ab_y8.txt 2>&1 || exit 1
cat gpurun_out/ab_y8.txt
