#!/usr/bin/env python3
"""VALU issue per launch of the dominant kernel from the rocprofv3 PMC pass of
scripts/gpu_profile.sh (SQ_INSTS_VALU, SQ_WAVES, GRBM_GUI_ACTIVE in one run).

SQ_INSTS_VALU counts wave-level VALU instructions over the whole chip; on gfx950 an fp64 / int32 /
DPP VALU instruction of a wave64 issues in ~4 SIMD cycles (profiles/r02/valu_rates.txt), so the
VALU-issue framing of a launch is  4 x SQ_INSTS_VALU / (1024 SIMDs x cycles).  GRBM_GUI_ACTIVE is
summed over the 8 XCDs (MI355X_MICROARCH.md, DVFS give-back): / 8 = the launch's cycles at the
clock it actually held.

  python scripts/pmc_valu.py gpurun_out/prof profiles/pmc_valu.json [--ndim 32 --chains 65536 --sweeps 1000]
"""
import argparse
import collections
import csv
import json
import os

SIMDS = 1024
CYCLES_PER_VALU = 4.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("out")
    ap.add_argument("--kernel", default="mcg::mh_kernel<")
    ap.add_argument("--ndim", type=int, default=32)
    ap.add_argument("--chains", type=int, default=65536)
    ap.add_argument("--sweeps", type=int, default=1000)
    a = ap.parse_args()
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(os.path.join(a.prof_dir, "valu", "run_counter_collection.csv"))):
        agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    name = next(k for k in agg if a.kernel in k)
    c = agg[name]

    def mean(k):
        v = c[k][1:] or c[k]            # drop the first (burn-in) launch
        return sum(v) / len(v)
    valu, waves, grbm = mean("SQ_INSTS_VALU"), mean("SQ_WAVES"), mean("GRBM_GUI_ACTIVE")
    cycles = grbm / 8.0
    steps = float(a.chains) * a.sweeps
    out = {"kernel": name, "config": {"ndim": a.ndim, "chains_per_gpu": a.chains, "sweeps_per_step": a.sweeps},
           "launches": len(c["SQ_INSTS_VALU"]), "valu_insts_per_launch": valu, "waves_per_launch": waves,
           "valu_insts_per_mh_step_per_wave_lane": valu * 64.0 / steps / (waves * 64.0 / a.chains),
           "valu_insts_per_chain_step": valu * 64.0 / steps,
           "cycles_per_launch": cycles,
           "valu_busy_frac_at_held_clock": CYCLES_PER_VALU * valu / (SIMDS * cycles),
           "note": "4 SIMD cycles per wave64 VALU instruction; GRBM_GUI_ACTIVE / 8 XCDs = cycles"}
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
