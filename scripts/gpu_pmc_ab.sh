#!/bin/bash
# PMC passes (one counter group per pass, kernel-trace only) for each library given:
#   bash scripts/gpu_pmc_ab.sh libmcg.so libmcg_x.so
# writes gpurun_out/pmcab/<lib>/p<i>/run_counter_collection.csv (MH kernel rows only)
mkdir -p gpurun_out/pmcab
export TMPDIR=/tmp
ARGS="--steps 5 --warmup 1 --no-cpu-baseline --nested-seeds 0 --nested-nlive 0"
for lib in "$@"; do
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_BUSY_CYCLES" \
             "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    MCG_LIBRARY=$PWD/mcmc-ocaml_amd/lib/$lib timeout -s KILL 120 rocprofv3 --pmc $grp -d gpurun_out/pmcab/$lib/p$i -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmcab/$lib.p$i.log 2>&1 || { echo "pass $lib $i rc=$?"; exit 1; }
  done
done
for f in gpurun_out/pmcab/*/p*/run_counter_collection.csv; do
  (head -1 "$f"; grep mh_kernel "$f") > "$f.mh" && mv "$f.mh" "$f"
done
for lib in "$@"; do echo "== $lib"; python3 scripts/pmc_summary.py gpurun_out/pmcab/$lib; done > gpurun_out/pmcab/summary.txt 2>&1
echo pmc-done
