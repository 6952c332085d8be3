#!/usr/bin/env python3
"""Per-kernel register and scratch report of libmcg.so's HIP translation units (the compiler's
-Rpass-analysis=kernel-resource-usage remarks), written as a table: kernel, VGPRs, AGPRs,
SGPR / VGPR spills, scratch bytes per lane, LDS.  Usage: scripts/scratch_report.py [out.txt]"""
import concurrent.futures as cf
import glob
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "mcmc-ocaml_amd", "csrc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
         "-I" + os.path.join(ROOT, "include"), "-I" + CSRC, "-c", "-o", "/dev/null",
         "-Rpass-analysis=kernel-resource-usage"]
KEYS = {"VGPRs": "vgpr", "AGPRs": "agpr", "SGPRs Spill": "sgpr_spill", "VGPRs Spill": "vgpr_spill",
        "ScratchSize [bytes/lane]": "scratch", "LDS Size [bytes/block]": "lds"}


def one(src):
    extra = ["-fno-slp-vectorize"] if src.endswith("_gauss.hip") else []
    p = subprocess.run(["/opt/rocm/bin/hipcc"] + FLAGS + extra + [src], capture_output=True, text=True, cwd=CSRC)
    rows, cur = [], None
    for line in p.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"kernel": m.group(1), "tu": os.path.basename(src)}
            rows.append(cur)
            continue
        for k, v in KEYS.items():
            m = re.search(re.escape(k) + r": (\d+)", line)
            if m and cur is not None:
                cur[v] = int(m.group(1))
    return rows


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "scratch_per_instance.txt")
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    rows = []
    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 8)) as ex:
        for r in ex.map(one, srcs):
            rows += r
    kern = [r for r in rows if "kernel" in r["kernel"] or "Kernel" in r["kernel"]]
    kern.sort(key=lambda r: (-r.get("scratch", 0), r["kernel"]))
    with open(out, "w") as fh:
        fh.write("# libmcg.so kernels: compiler resource usage (scripts/scratch_report.py)\n")
        fh.write("# %d kernels, %d with scratch\n" % (len(kern), sum(1 for r in kern if r.get("scratch", 0))))
        fh.write("%-9s %-6s %-6s %-11s %-11s %-6s  %s\n" % ("scratch", "vgpr", "agpr", "sgpr_spill", "vgpr_spill", "lds", "kernel"))
        for r in kern:
            fh.write("%-9d %-6d %-6d %-11d %-11d %-6d  %s\n" % (r.get("scratch", 0), r.get("vgpr", 0), r.get("agpr", 0),
                                                             r.get("sgpr_spill", 0), r.get("vgpr_spill", 0),
                                                             r.get("lds", 0), r["kernel"]))
    print(out, len(kern), "kernels,", sum(1 for r in kern if r.get("scratch", 0)), "with scratch")


if __name__ == "__main__":
    main()
