#!/usr/bin/env python3
"""Wall-time breakdown of one C3 Nested.nested_evidence call: the Python layers around
mcg_nested / mcg_nested_get (run with MCG_NESTED_PROFILE=1 for the C++ side)."""
import os, sys, time, ctypes as C
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "mcmc-ocaml_amd"))
import numpy as np
from mcmc_amd import Context, targets as T
from mcmc_amd import _lib as L

D = 16
lik = T.gauss_shell(np.zeros(D), 2.0, 0.1)
pri = T.box(-6 * np.ones(D), 6 * np.ones(D))
ctx = Context(seed=1)
for rep in range(4):
    t0 = time.perf_counter()
    ctx.set_model(lik, pri, None)
    t1 = time.perf_counter()
    o = L.McgNestedOpts(131072, 100, 4096, 0.01, 0.1, 0)
    r = L.McgNestedResult()
    L.check(L.lib().mcg_nested(ctx.ptr, C.byref(o), C.byref(r), L.OBSERVER(), None), ctx.ptr)
    t2 = time.perf_counter()
    n = r.n_total
    pts = np.zeros((n, D)); ll = np.zeros(n); lp = np.zeros(n); w = np.zeros(n)
    t3 = time.perf_counter()
    L.check(L.lib().mcg_nested_get(ctx.ptr, L.dptr(pts), L.dptr(ll), L.dptr(lp), L.dptr(w)), ctx.ptr)
    t4 = time.perf_counter()
    del pts, ll, lp, w
    t5 = time.perf_counter()
    print("rep %d: set_model %.1f ms, mcg_nested %.1f ms, np.zeros %.1f ms, get %.1f ms, free %.1f ms, total %.1f ms" % (
        rep, 1e3 * (t1 - t0), 1e3 * (t2 - t1), 1e3 * (t3 - t2), 1e3 * (t4 - t3), 1e3 * (t5 - t4), 1e3 * (t5 - t0)), flush=True)
