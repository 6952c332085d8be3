"""The OCaml binding (mcmc-ocaml_amd/ocaml/, shipped as source: no OCaml toolchain here) checked
against the C-ABI it binds: every `foreign` symbol exists in include/mcg.h with the same number
of arguments and compatible types, every ctypes structure lists the C struct's fields in order
with matching types, the likelihood / prior / proposal kind numbers it passes are the header's
enum values, and its run options for mcmc_array equal the Python mirror's (mcmc_amd.mcmc)."""
import pathlib
import re

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
HDR = (ROOT / "include" / "mcg.h").read_text()
ML = (ROOT / "mcmc-ocaml_amd" / "ocaml" / "mcmc_gpu.ml").read_text()
MLI = (ROOT / "mcmc-ocaml_amd" / "ocaml" / "mcmc_gpu.mli").read_text()


def _strip_comments(s):
    return re.sub(r"/\*.*?\*/", " ", s, flags=re.S)


def c_prototypes():
    src = _strip_comments(HDR)
    out = {}
    for m in re.finditer(r"^([A-Za-z_][\w ]*?[\w\*])\s*\b(mcg_\w+)\(([^;]*?)\);", src, re.M):
        ret, name, args = m.group(1).strip(), m.group(2), " ".join(m.group(3).split())
        params = [] if args in ("", "void") else [a.strip() for a in args.split(",")]
        out[name] = (ret, params)
    return out


def c_structs():
    src = _strip_comments(HDR)
    out = {}
    for m in re.finditer(r"typedef struct \{(.*?)\}\s*(\w+);", src, re.S):
        fields = []
        for decl in m.group(1).split(";"):
            decl = " ".join(decl.split())
            if not decl:
                continue
            fm = re.match(r"(.*?)(\w+)$", decl)
            fields.append((fm.group(2), fm.group(1).strip()))
        out[m.group(2)] = fields
    return out


def ml_foreign():
    out = []
    for m in re.finditer(r'fn "(mcg_\w+)" \((.*?)\)\n', ML):
        parts = [p.strip() for p in m.group(2).split("@->")]
        assert parts[-1].startswith("returning "), m.group(0)
        out.append((m.group(1), parts[:-1], parts[-1][len("returning "):].strip()))
    return out


def ml_structs():
    out = {}
    for m in re.finditer(r'let (\w+) : \w+ structure typ = structure "(\w+)"', ML):
        var, cname = m.group(1), m.group(2)
        fields = re.findall(r'let \w+ = field ' + var + r' "(\w+)" (.+)', ML)
        out[cname] = (var, [(n, t.strip()) for n, t in fields])
    return out


SCALAR = {"int32_t": "int32_t", "int": "int", "uint32_t": "uint32_t", "int64_t": "int64_t",
          "uint64_t": "uint64_t", "size_t": "size_t", "double": "double", "void": "void",
          "uint8_t": "uint8_t"}
STRUCT_VARS = {"mcg_opts": "opts", "mcg_run_opts": "run_opts", "mcg_nested_opts": "nested_opts",
               "mcg_nested_result": "nested_result", "mcg_rj_model": "rj_model_s"}


def compatible(ctype, mltype, arg=True):
    """Whether the ctypes type `mltype` may bind the C parameter / field type `ctype`."""
    c = re.sub(r"\bconst\b", "", ctype)
    c = re.sub(r"\s*\*", "*", " ".join(c.split())).strip()
    c = re.sub(r"\s+\w+$", "", c) if arg and not c.endswith("*") and " " in c else c
    c = re.sub(r"(\*)\w+$", r"\1", c)
    if c in ("int", "int32_t") and mltype in ("int", "int32_t"):
        return True
    if c in SCALAR:
        return SCALAR[c] == mltype
    if c == "char*":
        return mltype in ("string", "string_opt")
    if c == "mcg_observer_fn":
        return mltype in ("funptr observer_t", "ptr void")
    if c.endswith("**"):
        return mltype == "ptr (ptr void)"
    base = c[:-1]
    if base in ("mcg_ctx", "void"):
        return mltype == "ptr void"
    if base in STRUCT_VARS:
        return mltype == "ptr " + STRUCT_VARS[base]
    if base in SCALAR:
        return mltype == "ptr " + SCALAR[base]
    return False


def test_every_foreign_symbol_matches_the_header():
    protos = c_prototypes()
    bound = ml_foreign()
    assert len(bound) >= 25
    for name, args, ret in bound:
        assert name in protos, f"{name} is bound in mcmc_gpu.ml but not declared in mcg.h"
        cret, cparams = protos[name]
        assert len(args) == len(cparams), (name, args, cparams)
        for a, p in zip(args, cparams):
            # parameter declarations carry a name: drop it
            ptype = re.sub(r"\s*\b\w+$", "", p) if not p.endswith("*") else p
            ptype = re.sub(r"/\*.*?\*/", "", ptype)
            assert compatible(ptype, a, arg=False), (name, p, a)
        assert compatible(cret, ret, arg=False), (name, cret, ret)


def test_ctypes_structures_match_the_header_structs():
    cs, ms = c_structs(), ml_structs()
    for cname in ("mcg_opts", "mcg_run_opts", "mcg_nested_opts", "mcg_nested_result", "mcg_rj_model"):
        assert cname in ms, cname
        _, mlfields = ms[cname]
        cfields = cs[cname]
        assert [n for n, _ in mlfields] == [n for n, _ in cfields], cname
        for (n, mt), (_, ct) in zip(mlfields, cfields):
            mt = mt.replace("(ptr double)", "ptr double")
            assert compatible(ct, mt, arg=False), (cname, n, ct, mt)


def _enum(name):
    m = re.search(name + r"\s*=\s*(\d+)", HDR)
    return int(m.group(1))


def test_kind_numbers_are_the_header_enums():
    body = ML[ML.index("let set_model"):ML.index("type state")]
    kinds = dict(re.findall(r"\| (\w+) [^\n]*?-> (\d+), ", body))
    assert int(kinds["Flat"]) == _enum("MCG_LIK_FLAT")
    assert int(kinds["Diag_gauss"]) == _enum("MCG_LIK_DIAG_GAUSS")
    assert int(kinds["Fullcov_gauss"]) == _enum("MCG_LIK_FULLCOV_GAUSS")
    assert int(kinds["Gauss_shell"]) == _enum("MCG_LIK_GAUSS_SHELL")
    assert int(kinds["Gauss_data"]) == _enum("MCG_LIK_GAUSS_DATA")
    assert int(kinds["Cauchy_data"]) == _enum("MCG_LIK_CAUCHY_DATA")
    assert int(kinds["Gauss_mix"]) == _enum("MCG_LIK_GAUSS_MIX")
    props = dict(re.findall(r"\| Some \((\w+)[^\n]*?c_set_proposal ctx (\d+)l", body))
    assert int(props["Gauss"]) == _enum("MCG_PROP_GAUSS")
    assert "c_set_proposal ctx 2l" in body and _enum("MCG_PROP_WRAP_UNIFORM") == 2
    assert "c_set_proposal ctx 5l" in body and _enum("MCG_PROP_MIXTURE") == 5
    assert "Open_box _ -> 2l" in body and _enum("MCG_PRIOR_OPEN_BOX") == 2
    assert _enum("MCG_PRIOR_BOX") == 1
    assert "c_set_prior ctx 3l" in body and _enum("MCG_PRIOR_DIAG_GAUSS") == 3


def _ml_run_opts(fun):
    body = ML[ML.index("let " + fun):]
    body = body[:body.index("check ctx (c_run")]
    return {k: v for k, v in re.findall(r"setf o r_(\w+) ([^;]+?)(?:;|\n)", body)}


def test_mcmc_array_run_options_match_the_python_mirror():
    """Mcmc_gpu.mcmc_array and mcmc_amd.mcmc.mcmc_array make the same mcg_run call."""
    import inspect
    from mcmc_amd import mcmc
    o = _ml_run_opts("mcmc_array")
    assert o["rx"].strip() == "1l" and o["rllp"].strip() == "1l" and o["accum"].strip() == "1l"
    assert o["racc"].strip() == "0l" and o["append"].strip() == "0l"
    src = inspect.getsource(mcmc.mcmc_array)
    assert "record_x=True" in src and "record_llp=True" in src
    s = _ml_run_opts("make_core")
    assert s["nbin"].strip() == "1L" and s["nrec"].strip() == "0L" and s["accum"].strip() == "0l"


def test_gauss_mix_packing_matches_targets():
    """Gauss_mix packs (m, then per component mu, sigma) as mcmc_amd.targets.gauss_mix does."""
    import numpy as np
    from mcmc_amd import targets
    body = ML[ML.index("let mix_params"):]
    body = body[:body.index("\n\n")]
    assert "float (Array.length mus)" in body and "Array.append mu" in body
    mus, sg = np.array([[0.25, 0.75], [0.5, 0.5]]), np.array([[0.05, 0.05], [0.1, 0.2]])
    d = targets.gauss_mix(mus, sg)
    assert d.params[0] == 2
    np.testing.assert_array_equal(d.params[1:], np.concatenate([mus[0], sg[0], mus[1], sg[1]]))


def test_sampler_residency_is_tied_to_the_context_token():
    """the OCaml make_mcmc_sampler skips the mcg_init upload only when the argument is
    its last result (physically), still equal to its private snapshot, and the context's state
    token is unchanged since its own step; the compat layer decides accept / reject by the step's
    accept count, not by comparing values."""
    body = ML[ML.index("let make_core"):ML.index("let reset_counters")]
    assert "c_state_token ctx" in body and "Unsigned.UInt64.equal !tok_mine" in body
    assert "x = sx && ll = sll && lp = slp" in body
    # a moved token re-applies the sampler's own model before stepping
    assert "if not ours then set_model ctx lik pri (Some prop)" in body
    assert re.search(r'fn "mcg_state_token" \(ptr void @-> returning uint64_t\)', ML)
    assert "uint64_t mcg_state_token(const mcg_ctx* ctx);" in HDR
    compat = (ROOT / "mcmc-ocaml_amd" / "ocaml" / "mcmc_gpu_compat.ml").read_text()
    c = compat[compat.index("let make_mcmc_sampler"):compat.index("let mcmc_array")]
    # one counter read per step (make_mcmc_step), not two
    assert "Mcmc_gpu.make_mcmc_step ctx" in c and "if nacc = 0 then s" in c
    assert "Mcmc_gpu.get_counters" not in c
    assert "val make_mcmc_step" in MLI
    assert "s.Mcmc.value = v0" in c
