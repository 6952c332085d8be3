#!/usr/bin/env python3
"""L2 (TCC) hit / miss and fabric-read counters of the C3 walk kernel (nest_walk_kernel) from the
rocprofv3 PMC passes of scripts/gpu_r5_c3pmc.sh (scripts/probes/nested_breakdown.py: two C3 runs,
nlive 131,072, k 4,096, nmcmc 100), averaged per launch over every walk dispatch.

  pass 1: TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_EA0_RDREQ_sum    pass 2: FETCH_SIZE

The walk's algorithmic random-row bytes are k x nmcmc x 2 rows x 128 B (D 16): the DE partner
rows (nested.ml:53), gathered from the 16.8 MB live set, which fits the 256 MiB Infinity Cache and
no XCD's 4 MiB L2.  TCC_EA0_RDREQ counts the L2's memory-side read requests: misses of the L2 that
go to the Infinity Cache (hits there included, MI355X_MICROARCH.md HBM section) -- x 128 B per
request (FETCH_SIZE = RDREQ x 64 B on gfx950: the guide's 1/2 correction).

  python scripts/pmc_c3.py gpurun_out/c3pmc profiles/pmc_c3_walk.json [--k 4096 --nmcmc 100]
"""
import argparse
import collections
import csv
import glob
import json
import os


def load(d):
    agg = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "nest_walk_kernel" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("out")
    ap.add_argument("--k", type=int, default=4096)
    ap.add_argument("--nmcmc", type=int, default=100)
    ap.add_argument("--D", type=int, default=16)
    a = ap.parse_args()
    c = {}
    for p in ("p1", "p2"):
        c.update(load(os.path.join(a.prof_dir, p)))
    mean = lambda k: sum(c[k]) / len(c[k]) if c.get(k) else None
    hit, miss, req, rd, fetch = (mean(k) for k in ("TCC_HIT_sum", "TCC_MISS_sum", "TCC_REQ_sum",
                                                   "TCC_EA0_RDREQ_sum", "FETCH_SIZE"))
    alg = a.k * a.nmcmc * 2.0 * a.D * 8
    out = {"kernel": "mcg::nest_walk_kernel<16, SHELL, ...>", "config": {"k": a.k, "nmcmc": a.nmcmc},
           "launches": len(c.get("TCC_HIT_sum", [])),
           "tcc_hit_per_launch": hit, "tcc_miss_per_launch": miss, "tcc_req_per_launch": req,
           "tcc_hit_rate": hit / (hit + miss) if hit is not None and (hit + miss) > 0 else None,
           "ea_rdreq_per_launch": rd,
           "l2_miss_read_bytes_per_launch": rd * 128.0 if rd is not None else None,
           "fetch_size_kb_per_launch": fetch,
           "fetch_bytes_per_launch_x2": fetch * 1024 * 2 if fetch is not None else None,
           "algorithmic_row_bytes_per_launch": alg,
           "note": "L2 misses go to the Infinity Cache (16.8 MB live set); EA RDREQ x 128 B = the bytes "
                   "the L2 read from the fabric; FETCH_SIZE (KB) x 2: the gfx950 correction"}
    if rd is not None:
        out["l2_miss_bytes_over_algorithmic"] = rd * 128.0 / alg
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
