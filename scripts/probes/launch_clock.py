#!/usr/bin/env python3
"""Per-dispatch clock of the MH kernel from a rocprofv3 --pmc GRBM_GUI_ACTIVE run: cycles per
XCD (GRBM_GUI_ACTIVE / 8) over the dispatch's duration, in launch order.
  python scripts/probes/launch_clock.py <pmc output dir>"""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True)[0]
rows = []
for r in csv.DictReader(open(f)):
    if "mh_kernel" in r["Kernel_Name"] and r["Counter_Name"] == "GRBM_GUI_ACTIVE":
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        rows.append((s, e, float(r["Counter_Value"])))
rows.sort()
for s, e, c in rows:
    dur = (e - s) / 1e9
    print("dur %.3f ms  cycles/XCD %.3e  clock %.3f GHz" % (dur * 1e3, c / 8, c / 8 / dur / 1e9))
