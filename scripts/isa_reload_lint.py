#!/usr/bin/env python3
"""Static check of the gfx950 ISA of libmcg.so's kernels for the round-6 miscompile pattern
(DESIGN.md §5.9): a 12-byte folded reload (scratch_load_dwordx3) into registers R[b..b+2] of a
value whose fourth dword R[b+3] is then read as part of a 64-bit pair before anything writes it
-- the compiler assumed the spilled tuple's last dword was still in R[b+3] (in the D 64 one-lane
kD kernel it held a kD box bound, so every chain's final x[3] came out wrong).  Compiles every
HIP translation unit to assembly (or scans the given .s files) and prints each suspect reload.
Usage: scripts/isa_reload_lint.py [file.s ...]"""
import concurrent.futures as cf
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "mcmc-ocaml_amd", "csrc")
REG = re.compile(r"\b([av])(?:\[(\d+):(\d+)\]|(\d+)\b)")
RELOAD = re.compile(r"scratch_load_dwordx3\s+([av])\[(\d+):(\d+)\].*12-byte Folded Reload")
WINDOW = 400


def regs(text):
    out = set()
    for m in REG.finditer(text):
        k = m.group(1)
        if m.group(4) is not None:
            out.add((k, int(m.group(4))))
        else:
            out.update((k, r) for r in range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def split_ops(line):
    op, _, rest = line.partition(" ")
    rest = rest.split(";")[0]
    parts = [p.strip() for p in rest.split(",")] if rest.strip() else []
    return op, parts


def scan(path):
    found = []
    fn = None
    lines = open(path).read().split("\n")
    for n, raw in enumerate(lines):
        if raw and not raw.startswith((" ", "\t", ".", ";")) and raw.endswith(":"):
            fn = raw[:-1]
        m = RELOAD.search(raw)
        if not m:
            continue
        k, b = m.group(1), int(m.group(2))
        last = (k, b + 3)
        # the compiler's own pattern restores the fourth dword right beside the 12-byte reload
        # (v_accvgpr_read_b32 R[b+3], aN ; Reload Reuse): a write of R[b+3] among the few
        # instructions before it makes the tuple whole
        prev = [x.strip() for x in lines[max(0, n - 12):n] if x.strip() and not x.strip().startswith(";")][-4:]
        if any(last in regs(split_ops(x)[1][0]) for x in prev if split_ops(x)[1] and "store" not in split_ops(x)[0]):
            continue
        for l in lines[n + 1:n + 1 + WINDOW]:
            s = l.strip()
            if not s or s.startswith((";", ".")) or s.endswith(":"):
                continue
            if s.startswith(("s_endpgm", "s_setpc")):
                break
            op, parts = split_ops(s)
            writes_first = not any(t in op for t in ("store", "ds_write", "s_waitcnt", "s_cbranch", "s_branch"))
            dst = regs(parts[0]) if parts and writes_first else set()
            src = set()
            for p in (parts[1:] if writes_first else parts):
                src |= regs(p)
            if last in src:
                found.append((fn, n + 1, raw.strip(), s))
                break
            if last in dst:
                break
    return found


def compile_asm(src, tmp):
    out = os.path.join(tmp, os.path.basename(src) + ".s")
    extra = ["-fno-slp-vectorize"] if src.endswith("_gauss.hip") else []
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
                    "-fno-fast-math", "-I" + os.path.join(ROOT, "include"), "-I" + CSRC, "-S", "--cuda-device-only",
                    "-o", out, src] + extra, check=True, capture_output=True, cwd=CSRC)
    return out


def main():
    files = sys.argv[1:]
    tmp = None
    if not files:
        tmp = tempfile.mkdtemp()
        srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
        with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 8)) as ex:
            files = list(ex.map(lambda s: compile_asm(s, tmp), srcs))
    total, reloads = 0, 0
    for f in files:
        reloads += sum(1 for l in open(f) if RELOAD.search(l))
        for fn, ln, rl, use in scan(f):
            total += 1
            print("%s:%d %s\n    reload: %s\n    first read of the 4th dword: %s" % (os.path.basename(f), ln, fn, rl, use))
    print("%d 12-byte folded reloads scanned, %d suspect" % (reloads, total))
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main())
