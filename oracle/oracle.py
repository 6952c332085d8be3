"""ctypes loader for the CPU oracle (liboracle.so) -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, and
only as the checker.  See oracle.h for the parity status (RNG-driven paths are pinned
statistically against the reference's own tests; deterministic pieces by its KATs).
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

_dp = C.POINTER(C.c_double)
_u64p = C.POINTER(C.c_uint64)


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


class OrModel(C.Structure):
    _fields_ = [("ndim", C.c_int32), ("lik_kind", C.c_int32), ("lik_params", _dp),
                ("n_lik_params", C.c_int64), ("prior_kind", C.c_int32), ("prior_params", _dp),
                ("n_prior_params", C.c_int64), ("prop_kind", C.c_int32), ("prop_params", _dp),
                ("n_prop_params", C.c_int64), ("kd", C.c_void_p)]


class OrRunOpts(C.Structure):
    _fields_ = [("nbin", C.c_int64), ("nskip", C.c_int64), ("n_rec", C.c_int64),
                ("record_x", C.c_int32), ("record_llp", C.c_int32),
                ("record_accept", C.c_int32), ("accumulate", C.c_int32)]


class OrAccum(C.Structure):
    _fields_ = [("mean", _dp), ("m2", _dp), ("hm_m", _dp), ("hm_s", _dp)]


class OrNestedOpts(C.Structure):
    _fields_ = [("nlive", C.c_int64), ("nmcmc", C.c_int64), ("k", C.c_int64),
                ("epsrel", C.c_double), ("mode_hop", C.c_double),
                ("ref_stop_quirk", C.c_int32), ("max_iter", C.c_int64)]


class OrNestedResult(C.Structure):
    _fields_ = [("log_ev", C.c_double), ("log_dev", C.c_double), ("n_dead", C.c_int64),
                ("n_total", C.c_int64), ("n_gen", C.c_int64), ("status", C.c_int32)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.or_philox.argtypes = [C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        for name in ("or_log", "or_exp", "or_sqrt"):
            getattr(L, name).argtypes = [C.c_double]
            getattr(L, name).restype = C.c_double
        L.or_u53.argtypes = [C.c_uint32, C.c_uint32]
        L.or_u53.restype = C.c_double
        L.or_randint.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32]
        L.or_randint.restype = C.c_uint32
        L.or_normal.argtypes = [C.c_uint32]
        L.or_normal.restype = C.c_double
        L.or_step_normals.argtypes = [C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint32, C.c_int, _dp]
        L.or_set_literal.argtypes = [C.c_int]
        L.or_get_literal.restype = C.c_int
        L.or_mh_literal_shadow.argtypes = [C.POINTER(OrModel), C.c_uint64, C.c_int64, C.c_uint64, C.c_int64,
                                           _dp, _dp, _dp, C.POINTER(C.c_int64), _dp, _dp]
        L.or_wrap_uniform.argtypes = [C.c_double] * 5
        L.or_wrap_uniform.restype = C.c_double
        L.or_log_sum_logs.argtypes = [C.c_double, C.c_double]
        L.or_log_sum_logs.restype = C.c_double
        for name in ("or_mean", "or_std"):
            getattr(L, name).argtypes = [_dp, C.c_int64]
            getattr(L, name).restype = C.c_double
        for name in ("or_multi_mean", "or_multi_std"):
            getattr(L, name).argtypes = [_dp, C.c_int64, C.c_int, _dp]
        for name in ("or_log_gaussian", "or_log_cauchy", "or_log_lognormal"):
            getattr(L, name).argtypes = [C.c_double, C.c_double, C.c_double]
            getattr(L, name).restype = C.c_double
        L.or_log_multi_gaussian.argtypes = [_dp, _dp, _dp, C.c_int]
        L.or_log_multi_gaussian.restype = C.c_double
        L.or_loglik.argtypes = [C.POINTER(OrModel), _dp]
        L.or_loglik.restype = C.c_double
        L.or_logprior.argtypes = [C.POINTER(OrModel), _dp]
        L.or_logprior.restype = C.c_double
        L.or_mh_run.argtypes = [C.POINTER(OrModel), C.c_uint64, C.c_uint32, C.c_int64, C.c_uint64,
                                _dp, _dp, _dp, _u64p, C.POINTER(OrRunOpts), _dp, _dp, _dp, _u64p,
                                C.POINTER(OrAccum), C.c_int]
        L.or_mh_run.restype = C.c_int
        L.or_tile_stats.argtypes = [C.c_int, C.c_int64, C.c_int64, C.POINTER(OrAccum), _dp]
        L.or_combine_tiles.argtypes = [C.c_int, C.c_int64, _dp, _dp, _dp, _dp]
        L.or_harmonic_mean_naive.argtypes = [_dp, C.c_int64]
        L.or_harmonic_mean_naive.restype = C.c_double
        L.or_nested.argtypes = [C.POINTER(OrModel), C.c_uint64, C.POINTER(OrNestedOpts), _dp, _dp,
                                _dp, _dp, C.c_int64, C.POINTER(OrNestedResult)]
        L.or_nested.restype = C.c_int
        L.or_evidence_weights.argtypes = [C.c_int64, C.c_int64, C.c_int64, _dp, _dp, _dp, _dp]
        L.or_log_total_error_estimate.argtypes = [C.c_double, C.c_double, C.c_int64]
        L.or_log_total_error_estimate.restype = C.c_double
        L.or_weight_binary_search_index.argtypes = [C.c_double, _dp, C.c_int64]
        L.or_weight_binary_search_index.restype = C.c_int64
        L.or_posterior_indices.argtypes = [C.c_uint64, C.c_uint32, _dp, C.c_int64, C.c_int64,
                                           C.POINTER(C.c_int64)]
        L.or_kd_build.argtypes = [_dp, C.c_int64, C.c_int, _dp, _dp]
        L.or_kd_build.restype = C.c_void_p
        L.or_kd_free.argtypes = [C.c_void_p]
        L.or_kd_nnodes.argtypes = [C.c_void_p]
        L.or_kd_nnodes.restype = C.c_int64
        L.or_kd_nleaves.argtypes = [C.c_void_p]
        L.or_kd_nleaves.restype = C.c_int64
        L.or_kd_export.argtypes = [C.c_void_p, C.POINTER(C.c_int32), _dp, C.POINTER(C.c_int32),
                                   C.POINTER(C.c_int32), C.POINTER(C.c_int32), _dp]
        L.or_kd_find_leaf.argtypes = [C.c_void_p, _dp]
        L.or_kd_find_leaf.restype = C.c_int64
        L.or_kd_log_jump_prob.argtypes = [C.c_void_p, _dp]
        L.or_kd_log_jump_prob.restype = C.c_double
        L.or_kd_jump_prob.argtypes = [C.c_void_p, _dp]
        L.or_kd_jump_prob.restype = C.c_double
        _lib = L
    return _lib


def dptr(a):
    return None if a is None else a.ctypes.data_as(_dp)


def u64ptr(a):
    return None if a is None else a.ctypes.data_as(_u64p)


def f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


# ---- scalar helpers ----
def philox(ctr, key):
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    lib().or_philox(c, k, o)
    return list(o)


def normal(w):
    """Spec-v5 standard normal of one 32-bit word (oracle.c or_normal)."""
    return lib().or_normal(w)


def step_normals(seed, chain, step, D, tag=1):
    z = np.zeros(D)
    lib().or_step_normals(seed, chain, step, tag, D, dptr(z))
    return z


class Model:
    """Holds numpy parameter arrays alive for an OrModel (same layouts as include/mcg.h)."""

    def __init__(self, ndim, lik_kind, lik_params=(), prior_kind=0, prior_params=(),
                 prop_kind=1, prop_params=(1.0,), kd=None):
        self.lik_params = f64(lik_params if len(lik_params) else [0.0])
        self.prior_params = f64(prior_params if len(prior_params) else [0.0])
        self.prop_params = f64(prop_params if len(prop_params) else [0.0])
        self.kd = kd
        self.s = OrModel(ndim, lik_kind, dptr(self.lik_params), len(lik_params), prior_kind,
                         dptr(self.prior_params), len(prior_params), prop_kind,
                         dptr(self.prop_params), len(prop_params), kd.ptr if kd else None)
        self.ndim = ndim

    def loglik(self, x):
        x = f64(x)
        return lib().or_loglik(C.byref(self.s), dptr(x))

    def logprior(self, x):
        x = f64(x)
        return lib().or_logprior(C.byref(self.s), dptr(x))


class KdTree:
    def __init__(self, pts, low, high):
        self.pts = f64(pts)
        M, D = self.pts.shape
        self.low, self.high = f64(low), f64(high)
        self.ptr = lib().or_kd_build(dptr(self.pts), M, D, dptr(self.low), dptr(self.high))
        self.D, self.M = D, M

    def __del__(self):
        try:
            lib().or_kd_free(self.ptr)
        except Exception:
            pass

    def export(self):
        nn = lib().or_kd_nnodes(self.ptr)
        nl = lib().or_kd_nleaves(self.ptr)
        dim = np.zeros(nn, np.int32)
        split = np.zeros(nn)
        right = np.zeros(nn, np.int32)
        leaf = np.zeros(nn, np.int32)
        cnt = np.zeros(nl, np.int32)
        box = np.zeros((nl, 2, self.D))
        i32 = lambda a: a.ctypes.data_as(C.POINTER(C.c_int32))
        lib().or_kd_export(self.ptr, i32(dim), dptr(split), i32(right), i32(leaf), i32(cnt), dptr(box))
        return dict(dim=dim, split=split, right=right, leaf=leaf, count=cnt, box=box)

    def find_leaf(self, pt):
        return lib().or_kd_find_leaf(self.ptr, dptr(f64(pt)))

    def jump_prob(self, pt):
        return lib().or_kd_jump_prob(self.ptr, dptr(f64(pt)))

    def log_jump_prob(self, pt):
        return lib().or_kd_log_jump_prob(self.ptr, dptr(f64(pt)))


def mh_run(model, seed, x, ll, lp, nbin=0, nskip=1, n_rec=1, record_x=True, record_llp=True,
           record_accept=True, accumulate=True, step0=0, chain_offset=0, nacc=None, nthreads=1):
    """Batched Mcmc.mcmc_array on the CPU.  x: (D, N) array (modified copy returned)."""
    x = f64(x).copy()
    D, N = x.shape
    ll = f64(ll).copy()
    lp = f64(lp).copy()
    nacc = np.zeros(N, np.uint64) if nacc is None else nacc.copy()
    nsteps = nbin + max(0, n_rec - 1) * nskip
    rec_x = np.zeros((n_rec, D, N)) if record_x else None
    rec_ll = np.zeros((n_rec, N)) if record_llp else None
    rec_lp = np.zeros((n_rec, N)) if record_llp else None
    bits = np.zeros((max(nsteps, 1), (N + 63) // 64), np.uint64) if record_accept else None
    mean = np.zeros((D, N)); m2 = np.zeros((D, N)); hm_m = np.zeros((8, N)); hm_s = np.zeros((8, N))
    acc = OrAccum(dptr(mean), dptr(m2), dptr(hm_m), dptr(hm_s))
    o = OrRunOpts(nbin, nskip, n_rec, int(record_x), int(record_llp), int(record_accept),
                  int(accumulate))
    rc = lib().or_mh_run(C.byref(model.s), seed, chain_offset, N, step0, dptr(x), dptr(ll),
                         dptr(lp), u64ptr(nacc), C.byref(o), dptr(rec_x), dptr(rec_ll),
                         dptr(rec_lp), u64ptr(bits), C.byref(acc), nthreads)
    if rc != 0:
        raise RuntimeError("or_mh_run failed: %d" % rc)
    return dict(x=x, ll=ll, lp=lp, nacc=nacc, rec_x=rec_x, rec_ll=rec_ll, rec_lp=rec_lp,
                bits=bits[:nsteps] if bits is not None else None, mean=mean, m2=m2,
                hm_m=hm_m, hm_s=hm_s, acc=acc, nsteps=nsteps)


def tile_stats(D, N, nrec, res):
    ntiles = (N + 255) // 256
    tiles = np.zeros((ntiles, 2 * D + 3))
    lib().or_tile_stats(D, N, nrec, C.byref(res["acc"]), dptr(tiles))
    return tiles


def combine_tiles(D, tiles):
    tiles = f64(tiles)
    mean = np.zeros(D); sd = np.zeros(D); lz = C.c_double()
    lib().or_combine_tiles(D, tiles.shape[0], dptr(tiles), dptr(mean), dptr(sd), C.byref(lz))
    return mean, sd, lz.value


def nested(model, seed, nlive=1000, nmcmc=1000, k=1, epsrel=0.01, mode_hop=0.1, quirk=True,
           max_iter=0, cap=None):
    D = model.ndim
    cap = cap or nlive * 200
    pts = np.zeros((cap, D)); ll = np.zeros(cap); lp = np.zeros(cap); w = np.zeros(cap)
    o = OrNestedOpts(nlive, nmcmc, k, epsrel, mode_hop, int(quirk), max_iter)
    r = OrNestedResult()
    rc = lib().or_nested(C.byref(model.s), seed, C.byref(o), dptr(pts), dptr(ll), dptr(lp),
                         dptr(w), cap, C.byref(r))
    if rc == -2:
        raise RuntimeError("Failure: constraint violated in draw_new_live_point")
    if rc != 0:
        raise RuntimeError("or_nested failed: %d" % rc)
    n = r.n_total
    return dict(log_ev=r.log_ev, log_dev=r.log_dev, n_dead=r.n_dead, n_total=n, n_gen=r.n_gen,
                pts=pts[:n].copy(), ll=ll[:n].copy(), lp=lp[:n].copy(), log_wts=w[:n].copy())


def evidence_weights(ll, nlive, k=1):
    ll = f64(ll)
    n = len(ll)
    w = np.zeros(n); le = C.c_double(); ld = C.c_double()
    lib().or_evidence_weights(n, nlive, k, dptr(ll), C.byref(le), C.byref(ld), dptr(w))
    return le.value, ld.value, w


def _lse(a, b):
    """Stats.log_sum_logs (stats.ml:240-248)."""
    if a == -np.inf and b == -np.inf:
        return -np.inf
    if b > a:
        a, b = b, a
    return a + np.log1p(np.exp(b - a))


def nested_merge(runs):
    """Restatement of run merging for nested replicas: runs = [(ll, nlive, k)],
    each ll in nested_output order (nested.ml:143).  The live count at each merged point is the
    sum over runs of the count of the run's first point at or above that level (dead point i:
    nlive - i mod k; final live point j: nlive - j), and the trapezoid of
    evidence_error_and_weights (nested.ml:81-120) runs with that per-point count.
    Returns (order, log_ev, log_dev, log_wts in merged order)."""
    lls, counts = [], []
    for ll, nlive, k in runs:
        ll = np.asarray(ll, np.float64)
        ndead = len(ll) - nlive
        i = np.arange(len(ll))
        counts.append(np.where(i < ndead, nlive - i % k, nlive - (i - ndead)))
        lls.append(ll)
    cat = np.concatenate(lls)
    order = np.argsort(cat, kind="stable")
    L = cat[order]
    nps = np.zeros(len(L), np.int64)
    for ll, c in zip(lls, counts):
        i = np.searchsorted(ll, L, side="left")
        ok = i < len(ll)
        nps[ok] += c[i[ok]]
    half = -0.69314718055994530942
    n = len(L)
    w = np.full(n, -np.inf)
    low = high = -np.inf
    log_x = 0.0
    for p in range(n):
        log_dv = log_x + np.log(1.0 / nps[p])
        with np.errstate(divide="ignore"):
            log_x += np.log1p(-1.0 / nps[p])
        q = min(p + 1, n - 1)
        dl, dh = log_dv + L[p], log_dv + L[q]
        low, high = _lse(low, dl), _lse(high, dh)
        w[p] = _lse(w[p], half + dl)
        w[q] = _lse(w[q], half + dh)
    log_ev = half + _lse(low, high)
    log_dev = high + np.log1p(-np.exp(low - high))
    return order, log_ev, log_dev, w - log_ev


class OrRjModel(C.Structure):
    _fields_ = [("ndim", C.c_int32),
                ("lik_kind", C.c_int32), ("lik_params", _dp), ("n_lik", C.c_int64),
                ("prior_kind", C.c_int32), ("prior_params", _dp), ("n_prior", C.c_int64),
                ("jump_kind", C.c_int32), ("jump_params", _dp), ("n_jump", C.c_int64),
                ("into_kind", C.c_int32), ("into_params", _dp), ("n_into", C.c_int64),
                ("kd", C.c_void_p), ("model_prior", C.c_double)]


def rj_run(model_a, model_b, seed, xa, xb, nbin=0, nskip=1, n_rec=1, tags=None, nthreads=8):
    """Restated Mcmc.rjmcmc_array over N chains.  model_x: dicts with ndim, lik (kind, params),
    prior (kind, params), jump (kind, params), into (kind, params), kd (KdTree or None), p."""
    keep = []

    def mk(m):
        arrs = [f64(m[k][1] if len(m[k][1]) else [0.0]) for k in ("lik", "prior", "jump", "into")]
        keep.extend(arrs)
        kd = m.get("kd")
        return OrRjModel(m["ndim"], m["lik"][0], dptr(arrs[0]), len(m["lik"][1]), m["prior"][0],
                         dptr(arrs[1]), len(m["prior"][1]), m["jump"][0], dptr(arrs[2]),
                         len(m["jump"][1]), m["into"][0], dptr(arrs[3]), len(m["into"][1]),
                         kd.ptr if kd is not None else None, m["p"])

    a, b = mk(model_a), mk(model_b)
    xa, xb = f64(xa), f64(xb)
    N = xa.shape[1]
    DM = max(model_a["ndim"], model_b["ndim"])
    draw = tags is None
    tag = np.zeros(N, np.uint8) if draw else np.ascontiguousarray(tags, np.uint8)
    x = np.zeros((DM, N)); ll = np.zeros(N); lp = np.zeros(N)
    nacc = np.zeros(N, np.uint64); nb = np.zeros(N, np.uint64)
    nsteps = nbin + max(0, n_rec - 1) * nskip
    rec_x = np.zeros((n_rec, DM, N)); rec_ll = np.zeros((n_rec, N)); rec_lp = np.zeros((n_rec, N))
    rec_tag = np.zeros((n_rec, N), np.uint8)
    bits = np.zeros((max(nsteps, 1), (N + 63) // 64), np.uint64)
    o = OrRunOpts(nbin, nskip, n_rec, 1, 1, 1, 1)
    u8 = lambda v: v.ctypes.data_as(C.POINTER(C.c_uint8))
    L = lib()
    L.or_rj_run.argtypes = [C.POINTER(OrRjModel), C.POINTER(OrRjModel), C.c_uint64, C.c_int64,
                            C.POINTER(C.c_uint8), C.c_int, _dp, _dp, _dp, _dp, _dp, _u64p, _u64p,
                            C.POINTER(OrRunOpts), _dp, _dp, _dp, C.POINTER(C.c_uint8), _u64p, C.c_int]
    L.or_rj_run.restype = C.c_int
    rc = L.or_rj_run(C.byref(a), C.byref(b), seed, N, u8(tag), int(draw), dptr(xa), dptr(xb), dptr(x),
                     dptr(ll), dptr(lp), u64ptr(nacc), u64ptr(nb), C.byref(o), dptr(rec_x),
                     dptr(rec_ll), dptr(rec_lp), u8(rec_tag), u64ptr(bits), nthreads)
    if rc != 0:
        raise RuntimeError("or_rj_run failed: %d" % rc)
    return dict(x=x, ll=ll, lp=lp, tag=tag, nacc=nacc, nb=nb, rec_x=rec_x, rec_ll=rec_ll,
                rec_lp=rec_lp, rec_tag=rec_tag, bits=bits[:nsteps])
