"""Wall-time breakdown of one C3 nested run: mcg_nested (device generations + host weights),
mcg_nested_get (copies), Python wrapper."""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "mcmc-ocaml_amd"))
from mcmc_amd import Context, _lib as L, targets as T  # noqa: E402

D = 16
lik = T.gauss_shell(np.zeros(D), 2.0, 0.1)
pri = T.box(-6 * np.ones(D), 6 * np.ones(D))
for rep in range(2):
    ctx = Context(seed=1)
    ctx.set_model(lik, pri, None)
    o = L.McgNestedOpts(131072, 100, 4096, 0.01, 0.1, 0)
    r = L.McgNestedResult()
    t0 = time.perf_counter()
    L.check(L.lib().mcg_nested(ctx.ptr, C.byref(o), C.byref(r), L.OBSERVER(), None), ctx.ptr)
    t1 = time.perf_counter()
    n = r.n_total
    pts = np.empty((n, D)); ll = np.empty(n); lp = np.empty(n); w = np.empty(n)
    t2 = time.perf_counter()
    L.check(L.lib().mcg_nested_get(ctx.ptr, L.dptr(pts), L.dptr(ll), L.dptr(lp), L.dptr(w)), ctx.ptr)
    t3 = time.perf_counter()
    print("rep %d: mcg_nested %.3f s, alloc %.3f s, mcg_nested_get %.3f s, n_total %d" % (rep, t1 - t0, t2 - t1, t3 - t2, n))
    ctx.close()
