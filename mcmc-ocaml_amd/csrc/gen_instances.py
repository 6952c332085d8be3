#!/usr/bin/env python3
"""Generates the explicit kernel instantiations (mcg_inst_*.hip) and the dispatch registry.

The MH kernel is templated on (D, P, likelihood, proposal) so that chain state lives in VGPRs
with compile-time indexing.  This script decides which combinations are compiled; the
registry (mcg_registry.hip) maps runtime descriptors to launchers.
"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))

LIK = {"FLAT": "MCG_LIK_FLAT", "DIAG": "MCG_LIK_DIAG_GAUSS", "SHELL": "MCG_LIK_GAUSS_SHELL",
       "FULLCOV": "MCG_LIK_FULLCOV_GAUSS", "DATA": "MCG_LIK_GAUSS_DATA", "GMIX": "MCG_LIK_GAUSS_MIX"}
PROP = {"GAUSS": "MCG_PROP_GAUSS", "WRAP": "MCG_PROP_WRAP_UNIFORM", "KD": "MCG_PROP_KD_INTERP",
        "MIX": "MCG_PROP_MIXTURE", "DE": "MCG_PROP_DE"}

SMALL = [1, 2, 3, 4, 5, 6, 7, 8]
MID = [12, 16, 24, 32, 48, 64]
# Widths every padded ndim lands on (mcg_runtime.cpp pad_width): an ndim between two of them runs
# on the next one up with zero-padded dims, so each (likelihood, proposal) pair that pads is
# compiled at all of them.  FULLCOV pads to SMALL + [16, 32, 48, 64].
PAD = SMALL + MID


def combos():
    out = []  # (lik, prop, D, P)
    for lik in ("FLAT", "DIAG", "SHELL"):
        for D in SMALL + MID:
            out.append((lik, "GAUSS", D, 1))
            for P in (2, 4, 8):
                if D >= 8 and D % (4 * P) == 0:
                    out.append((lik, "GAUSS", D, P))
    for D in SMALL + [16, 32, 48, 64]:
        out.append(("FULLCOV", "GAUSS", D, 1))
    for D in (16, 32, 48, 64):
        out.append(("FULLCOV", "GAUSS", D, 4))        # matrix-core path (mcg_fullcov_kernel.h)
    for D in (2, 4, 6, 8):
        out.append(("DATA", "GAUSS", D, 1))
    # Mcmc.uniform_wrapping on every likelihood at every width an ndim pads to (one lane per chain)
    FULL = SMALL + [16, 32, 48, 64]
    for lik in ("FLAT", "DIAG", "SHELL", "GMIX"):
        for D in PAD:
            out.append((lik, "WRAP", D, 1))
    for D in FULL:
        out.append(("FULLCOV", "WRAP", D, 1))
    for D in (2, 4, 6, 8):
        out.append(("DATA", "WRAP", D, 1))
    # the kD interpolated proposal (Interpolate_pdf) at widths 1-8 and 16, unpadded (its tree is
    # built at the caller's ndim); one lane per chain on every likelihood, split over lanes on
    # the separable ones.  (A one-lane kD kernel at D 64 spills ~3.8 KB a lane, and the compiler
    # miscompiles it: its final state store reads x[3]'s high dword from a register it never
    # restored (profiles/r06/kd64_miscompile).  kD stays at D <= 16.)
    for lik in ("FLAT", "DIAG", "SHELL", "GMIX", "FULLCOV"):
        for D in SMALL + [16]:
            out.append((lik, "KD", D, 1))
            if lik in ("GMIX", "FULLCOV"):
                continue
            for P in (2, 4, 8):
                # kD draw split over P lanes per chain: four-dim lane blocks (D % 4P == 0), or
                # two dims per lane (D = 2P, mcg_mh_kernel.h Layout W = 2)
                if (D % (4 * P) == 0 and P < 8) or D == 2 * P:
                    out.append((lik, "KD", D, P))
    # kD at the padding widths (round 6: an ndim without a kernel of its own runs zero-padded):
    # 12 on every kind but full covariance (whose 9-15 pad to 16), 24 / 32 split over lanes on
    # the separable kinds (at most 16 dims a lane)
    for lik in ("FLAT", "DIAG", "SHELL", "GMIX"):
        out.append((lik, "KD", 12, 1))
    for lik in ("FLAT", "DIAG", "SHELL"):
        out.append((lik, "KD", 24, 2))
        out.append((lik, "KD", 32, 2))
        out.append((lik, "KD", 32, 4))
    # the multimodal target of test/nested_test.ml:41-64 (one lane per chain)
    for D in PAD:
        out.append(("GMIX", "GAUSS", D, 1))
    # Mcmc.combine_jump_proposals mixtures (one lane per chain)
    for lik in ("FLAT", "DIAG", "SHELL", "GMIX"):
        for D in PAD:
            out.append((lik, "MIX", D, 1))
    for D in FULL:
        out.append(("FULLCOV", "MIX", D, 1))
    for D in (2, 4, 6, 8):
        out.append(("DATA", "MIX", D, 1))
    # the wrapping-uniform and DE proposals on the lane-split likelihoods at the wide widths, split
    # so a lane holds at most 16 dims (D 24 / 32 on 2 lanes, 48 / 64 on 4): one lane per chain
    # spills 0.2-1.7 KB a lane at D 48 / 64 (round 6)
    for lik in ("FLAT", "DIAG", "SHELL", "GMIX"):
        for prop in ("WRAP", "DE"):
            for D, P in ((24, 2), (32, 2), (48, 4), (64, 4)):
                out.append((lik, prop, D, P))
    # Mcmc.differential_evolution_proposal over a caller-supplied sample array (one lane per chain)
    for lik in ("FLAT", "DIAG", "SHELL", "GMIX"):
        for D in PAD:
            out.append((lik, "DE", D, 1))
    for D in FULL:
        out.append(("FULLCOV", "DE", D, 1))
    for D in (2, 4, 6, 8):
        out.append(("DATA", "DE", D, 1))
    return out


def nested_combos():
    out = []
    for lik in ("FLAT", "DIAG", "SHELL", "GMIX"):
        for D in PAD:
            out.append((lik, D))
    for D in SMALL + [16, 32]:
        out.append(("FULLCOV", D))
    for D in (2, 4, 6, 8):
        out.append(("DATA", D))
    return out


def write_if_changed(path, text):
    if os.path.exists(path) and open(path).read() == text:
        return
    with open(path, "w") as f:
        f.write(text)


def main():
    cs = combos()
    groups = {}
    for c in cs:
        # the matrix-core full-covariance kernels get a translation unit of their own (its
        # rebuilds then skip the slow one-lane FULLCOV instances)
        grp = "MFMA" if (c[0] == "FULLCOV" and c[3] == 4) else c[1]
        groups.setdefault((c[0], grp), []).append(c)
    files = []
    decls = []
    table = []
    for (lik, prop), lst in sorted(groups.items()):
        fn = "mcg_inst_%s_%s.hip" % (lik.lower(), prop.lower())
        files.append(fn)
        lines = ['// generated by gen_instances.py -- do not edit',
                 '#include "mcg_fullcov_kernel.h"' if lik == "FULLCOV" else '#include "mcg_mh_kernel.h"',
                 "namespace mcg {"]
        for (_, cprop, D, P) in lst:
            name = "mh_%s_%s_%d_%d" % (lik.lower(), cprop.lower(), D, P)
            if lik == "FULLCOV" and P == 4:
                lines.append("hipError_t %s(const MhArgs& a, int64_t n, hipStream_t s) "
                             "{ return launch_mh_fullcov<%d>(a, n, s); }" % (name, D))
            else:
                lines.append("hipError_t %s(const MhArgs& a, int64_t n, hipStream_t s) "
                             "{ return launch_mh<%d, %d, %s, %s>(a, n, s); }" % (name, D, P, LIK[lik], PROP[cprop]))
            decls.append("hipError_t %s(const MhArgs&, int64_t, hipStream_t);" % name)
            table.append("  {%d, %d, %s, %s, %s}," % (D, P, LIK[lik], PROP[cprop], name))
        if prop == "GAUSS":
            for (_, _, D, P) in lst:
                if P == 1:
                    name = "ev_%s_%d" % (lik.lower(), D)
                    lines.append("hipError_t %s(const MhArgs& a, hipStream_t s) "
                                 "{ return launch_eval<%d, %s>(a, s); }" % (name, D, LIK[lik]))
        lines.append("}  // namespace mcg")
        write_if_changed(os.path.join(HERE, fn), "\n".join(lines) + "\n")
    evs = []
    for (lik, prop), lst in sorted(groups.items()):
        if prop != "GAUSS":
            continue
        for (_, _, D, P) in lst:
            if P == 1:
                name = "ev_%s_%d" % (lik.lower(), D)
                decls.append("hipError_t %s(const MhArgs&, hipStream_t);" % name)
                evs.append("  {%d, %s, %s}," % (D, LIK[lik], name))
    reg = ['// generated by gen_instances.py -- do not edit', '#include "mcg_device.h"',
           '#include "mcg.h"', "namespace mcg {"] + decls + [
        "struct MhEntry { int D, P, lik, prop; mh_launch_fn fn; };",
        "static const MhEntry kMh[] = {"] + table + ["};",
        "struct EvEntry { int D, lik; eval_launch_fn fn; };",
        "static const EvEntry kEv[] = {"] + evs + ["};",
        "mh_launch_fn find_mh_kernel(int D, int P, int lik, int prop) {",
        "  if (lik == MCG_LIK_CAUCHY_DATA) lik = MCG_LIK_GAUSS_DATA;",
        "  for (const auto& e : kMh) if (e.D == D && e.P == P && e.lik == lik && e.prop == prop) return e.fn;",
        "  return nullptr;", "}",
        "eval_launch_fn find_eval_kernel(int D, int lik) {",
        "  if (lik == MCG_LIK_CAUCHY_DATA) lik = MCG_LIK_GAUSS_DATA;",
        "  for (const auto& e : kEv) if (e.D == D && e.lik == lik) return e.fn;",
        "  return nullptr;", "}",
        "}  // namespace mcg"]
    # nested-sampling walkers / initial draws: one translation unit per likelihood (parallel
    # builds), the lookup tables in mcg_inst_nested.hip
    nl = ['// generated by gen_instances.py -- do not edit', '#include "mcg_nested_kernel.h"',
          "namespace mcg {"]
    wt, it = [], []
    per_lik = {}
    for (lik, D) in nested_combos():
        w = "nw_%s_%d" % (lik.lower(), D)
        i = "ni_%s_%d" % (lik.lower(), D)
        per_lik.setdefault(lik, []).extend([
            "hipError_t %s(const NestArgs& a, hipStream_t s) { return launch_nest_walk<%d, %s>(a, s); }"
            % (w, D, LIK[lik]),
            "hipError_t %s(const NestArgs& a, double* l, long long* t, int* k, hipStream_t s) "
            "{ return launch_nest_init<%d, %s>(a, l, t, k, s); }" % (i, D, LIK[lik])])
        nl.append("hipError_t %s(const NestArgs& a, hipStream_t s);" % w)
        nl.append("hipError_t %s(const NestArgs& a, double* l, long long* t, int* k, hipStream_t s);" % i)
        wt.append("  {%d, %s, %s}," % (D, LIK[lik], w))
        it.append("  {%d, %s, %s}," % (D, LIK[lik], i))
    for lik, lines in sorted(per_lik.items()):
        fn = "mcg_inst_nested_%s.hip" % lik.lower()
        write_if_changed(os.path.join(HERE, fn), "\n".join(
            ['// generated by gen_instances.py -- do not edit', '#include "mcg_nested_kernel.h"',
             "namespace mcg {"] + lines + ["}  // namespace mcg"]) + "\n")
        files.append(fn)
    nl += ["struct NwEntry { int D, lik; nest_walk_fn fn; };", "static const NwEntry kNw[] = {"] + wt + ["};",
           "struct NiEntry { int D, lik; nest_init_fn fn; };", "static const NiEntry kNi[] = {"] + it + ["};",
           "nest_walk_fn find_nest_walk(int D, int lik) {",
           "  if (lik == MCG_LIK_CAUCHY_DATA) lik = MCG_LIK_GAUSS_DATA;",
           "  for (const auto& e : kNw) if (e.D == D && e.lik == lik) return e.fn;",
           "  return nullptr;", "}",
           "nest_init_fn find_nest_init(int D, int lik) {",
           "  if (lik == MCG_LIK_CAUCHY_DATA) lik = MCG_LIK_GAUSS_DATA;",
           "  for (const auto& e : kNi) if (e.D == D && e.lik == lik) return e.fn;",
           "  return nullptr;", "}", "}  // namespace mcg"]
    write_if_changed(os.path.join(HERE, "mcg_inst_nested.hip"), "\n".join(nl) + "\n")
    files.append("mcg_inst_nested.hip")
    write_if_changed(os.path.join(HERE, "mcg_registry.hip"), "\n".join(reg) + "\n")
    write_if_changed(os.path.join(HERE, "instances.mk"), "INST_SRCS = " + " ".join(files) + "\n")
    print("%d kernels in %d files" % (len(cs), len(files)))


if __name__ == "__main__":
    main()
