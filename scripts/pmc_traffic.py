#!/usr/bin/env python3
"""HBM traffic per launch of the dominant kernel from the rocprofv3 PMC passes of
scripts/gpu_profile.sh (FETCH_SIZE and WRITE_SIZE in separate runs, values in KB).

gfx950 correction (MI355X_MICROARCH.md, HBM/rocprofv3 section): FETCH_SIZE reports half the bytes
of wide coalesced streaming reads -> doubled; WRITE_SIZE is exact for 16-B/lane stores.

  python scripts/pmc_traffic.py gpurun_out/prof profiles/r01/pmc_traffic.json [--ndim 32 --chains 65536 --sweeps 1000]
"""
import argparse
import collections
import csv
import json
import os


def per_kernel(path, counter):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return agg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("out")
    ap.add_argument("--kernel", default="mcg::mh_kernel<")
    ap.add_argument("--ndim", type=int, default=32)
    ap.add_argument("--chains", type=int, default=65536)
    ap.add_argument("--sweeps", type=int, default=1000)
    a = ap.parse_args()
    fetch = per_kernel(os.path.join(a.prof_dir, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(a.prof_dir, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    name = next(k for k in fetch if a.kernel in k)
    # drop the first launch of each pass (cold caches / first-touch), average the rest
    f = fetch[name][1:] or fetch[name]
    w = write[name][1:] or write[name]
    fetch_b = 2.0 * 1024.0 * sum(f) / len(f)
    write_b = 1024.0 * sum(w) / len(w)
    alg = 8.0 * (a.ndim + 2) * a.chains * a.sweeps
    out = {"kernel": name, "config": {"ndim": a.ndim, "chains_per_gpu": a.chains, "sweeps_per_step": a.sweeps},
           "launches": [len(fetch[name]), len(write[name])],
           "fetch_bytes": fetch_b, "write_bytes": write_b, "traffic_bytes": fetch_b + write_b,
           "algorithmic_bytes": alg, "traffic_over_algorithmic": (fetch_b + write_b) / alg,
           "correction": "FETCH_SIZE x2 (gfx950 half-count of wide coalesced reads), KB -> bytes x1024"}
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
