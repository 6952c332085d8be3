#!/usr/bin/env python3
import glob, json, collections, os
res = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/ab/*.json")):
    name = os.path.basename(f).rsplit(".", 2)[0]
    try:
        d = json.loads(open(f).read().strip().split("\n")[-1])
        res[name].append((d["value"], d["roofline"]["avg_launch_ms"]))
    except Exception as e:
        res[name].append(("ERR", str(e)[:60]))
for k, v in res.items():
    print("%-50s %s" % (k, "  ".join("%.4g/%.4fms" % x if x[0] != "ERR" else str(x) for x in v)))
