"""CPU tests of the C-ABI boundary: libmcg.so loads, exports every symbol include/mcg.h
declares, and fails loudly (MCG_EDEVICE) without a GPU -- no silent CPU fallback."""
import ctypes as C
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "mcg.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mcg_[a-z0-9_]+)\s*\(", src)) - {"mcg_observer_fn"})


def test_library_exports_every_header_symbol(gpu_lib):
    L = gpu_lib.lib()
    syms = header_symbols()
    assert len(syms) >= 25
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    # and the Python mirror binds exactly those
    assert set(gpu_lib.SIGNATURES) == set(syms)


def test_abi_version_and_arch(gpu_lib):
    L = gpu_lib.lib()
    assert L.mcg_abi_version() == 3
    assert L.mcg_device_arch() == b"gfx950"


def test_fails_loudly_without_device(gpu_lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    L = gpu_lib.lib()
    p = C.c_void_p()
    o = gpu_lib.McgOpts()
    assert L.mcg_ctx_create(C.byref(p), C.byref(o)) == gpu_lib.MCG_EDEVICE
    from mcmc_amd import Context
    with pytest.raises(gpu_lib.McgError):
        Context(seed=1)


def test_combine_tiles_is_host_only(gpu_lib):
    """mcg_combine_tiles is the cross-GPU combine step: pure host code, usable without a device.
    Two tiles with known moments combine to the pooled mean / sample std."""
    import numpy as np
    from mcmc_amd.context import combine_tiles
    D = 2
    a = np.array([3, 1.0, 2.0, 2.0, 8.0, 0.0, 1.0])   # n, mean[2], m2[2], hm_m, hm_s
    b = np.array([2, 4.0, 2.0, 1.0, 2.0, 0.0, 1.0])
    mean, sd, lz = combine_tiles(D, np.stack([a, b]))
    np.testing.assert_allclose(mean, [(3 * 1 + 2 * 4) / 5, 2.0])
    m2 = 2.0 + 1.0 + 9.0 * 3 * 2 / 5
    np.testing.assert_allclose(sd[0], np.sqrt(m2 / 4))
    np.testing.assert_allclose(lz, np.log(5) - np.log(2.0))


def test_oracle_not_imported_by_product():
    """The product package never imports the oracle (it is test infrastructure)."""
    pkg = os.path.join(ROOT, "mcmc-ocaml_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                txt = open(os.path.join(dp, f)).read()
                assert "import oracle" not in txt and "liboracle" not in txt and "oracle.h" not in txt, f
