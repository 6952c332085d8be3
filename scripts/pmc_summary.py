#!/usr/bin/env python3
"""Average each PMC counter over the launches of one kernel (rocprofv3 --pmc csv passes)."""
import collections, csv, glob, sys
d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
pat = sys.argv[2] if len(sys.argv) > 2 else "mh_kernel"
vals = collections.defaultdict(list)
for f in sorted(glob.glob(d + "/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in vals.items():
    v = v[1:] or v
    print("%-28s %16.4g" % (k, sum(v) / len(v)))
