"""Context: one libmcg sampling context (device buffers, Philox seed, counters)."""
import ctypes as C

import numpy as np

from . import _lib as L
from . import targets as T


class Context:
    def __init__(self, seed=0, device=0, chain_offset=0, lanes_per_chain=0, steps_per_launch=0,
                 flags=0):
        self._p = C.c_void_p()
        o = L.McgOpts(device, flags, seed, chain_offset, lanes_per_chain, steps_per_launch)
        rc = L.lib().mcg_ctx_create(C.byref(self._p), C.byref(o))
        if rc != L.MCG_OK:
            raise L.McgError(rc, "mcg_ctx_create failed (no HIP device or libmcg.so unusable)")
        self.seed = seed
        self.ndim = None
        self.nchains = 0
        self._keep = []

    @property
    def ptr(self):
        return self._p

    def close(self):
        if self._p:
            L.lib().mcg_ctx_destroy(self._p)
            self._p = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc):
        L.check(rc, self._p)

    # ---- model ----
    def set_model(self, log_likelihood, log_prior=None, jump=None):
        lk = log_likelihood
        self._check(L.lib().mcg_set_likelihood(self._p, lk.kind, lk.ndim, L.dptr(lk.params),
                                               len(lk.params)))
        self.ndim = lk.ndim
        self._keep = [lk]
        if log_prior is not None:
            pr = log_prior
            self._check(L.lib().mcg_set_prior(self._p, pr.kind, L.dptr(pr.params), len(pr.params)))
            self._keep.append(pr)
        if jump is not None:
            if isinstance(jump, T.DifferentialEvolution):
                M = jump.samples.shape[0]
                if jump.samples.shape[1] != lk.ndim:
                    raise L.InvalidArgument(L.MCG_EINVAL, "DE samples have %d dims, model has %d"
                                            % (jump.samples.shape[1], lk.ndim))
                self._check(L.lib().mcg_set_de_proposal(self._p, L.dptr(jump.samples), M,
                                                        jump.mode_hopping_frac))
            elif isinstance(jump, T.KdInterp):
                M = jump.pts.shape[0]
                self._check(L.lib().mcg_set_kd_proposal(self._p, L.dptr(jump.pts), M,
                                                        L.dptr(jump.low), L.dptr(jump.high)))
            else:
                kd = getattr(jump, "kd", None)
                if kd is not None:      # a mixture with a kD component: build the tree first
                    self._check(L.lib().mcg_set_kd_proposal(self._p, L.dptr(kd.pts), kd.pts.shape[0],
                                                            L.dptr(kd.low), L.dptr(kd.high)))
                self._check(L.lib().mcg_set_proposal(self._p, jump.kind, L.dptr(jump.params),
                                                     len(jump.params)))
            self._keep.append(jump)

    def init(self, x_soa, ll=None, lp=None):
        x = np.ascontiguousarray(np.asarray(x_soa, dtype=np.float64))
        if x.ndim == 1:
            x = x[:, None]
        D, N = x.shape
        if D != self.ndim:
            raise L.InvalidArgument(L.MCG_EINVAL, "start has %d dims, model has %d" % (D, self.ndim))
        lld = None if ll is None else np.ascontiguousarray(ll, dtype=np.float64)
        lpd = None if lp is None else np.ascontiguousarray(lp, dtype=np.float64)
        self._check(L.lib().mcg_init(self._p, N, L.dptr(x), L.dptr(lld), L.dptr(lpd)))
        self.nchains = N

    def state(self):
        D, N = self.ndim, self.nchains
        x = np.zeros((D, N)); ll = np.zeros(N); lp = np.zeros(N)
        self._check(L.lib().mcg_get_state(self._p, L.dptr(x), L.dptr(ll), L.dptr(lp)))
        return x, ll, lp

    # ---- runs ----
    def run(self, nbin=0, nskip=1, n_rec=1, record_x=True, record_llp=True, record_accept=False,
            accumulate=False, append=False):
        o = L.McgRunOpts(nbin, nskip, n_rec, int(record_x), int(record_llp), int(record_accept),
                         int(accumulate), int(append))
        self._check(L.lib().mcg_run(self._p, C.byref(o)))
        self._last = o

    def records(self, x=True, llp=True, accept=False):
        o = self._last
        D, N, R = self.ndim, self.nchains, o.n_rec
        rx = np.zeros((R, D, N)) if x else None
        rll = np.zeros((R, N)) if llp else None
        rlp = np.zeros((R, N)) if llp else None
        nsteps = L.lib().mcg_last_run_steps(self._p)
        bits = np.zeros((max(nsteps, 1), (N + 63) // 64), np.uint64) if accept else None
        self._check(L.lib().mcg_get_records(self._p, L.dptr(rx), L.dptr(rll), L.dptr(rlp),
                                            L.u64ptr(bits)))
        if bits is not None:
            bits = bits[:nsteps]
        return rx, rll, rlp, bits

    def lanes(self):
        """Lanes per chain of the last MH run (the runtime's auto choice unless set)."""
        return int(L.lib().mcg_last_run_lanes(self._p))

    def counters(self):
        a = np.zeros(1, np.uint64); r = np.zeros(1, np.uint64)
        self._check(L.lib().mcg_get_counters(self._p, L.u64ptr(a), L.u64ptr(r)))
        return int(a[0]), int(r[0])

    def reset_counters(self):
        self._check(L.lib().mcg_reset_counters(self._p))

    def tile_stats(self):
        nt = L.lib().mcg_num_tiles(self._p)
        tiles = np.zeros((nt, 2 * self.ndim + 3))
        self._check(L.lib().mcg_tile_stats(self._p, L.dptr(tiles)))
        return tiles

    def tile_stats_device(self):
        p = C.c_void_p(); nt = C.c_int64()
        self._check(L.lib().mcg_tile_stats_device(self._p, C.byref(p), C.byref(nt)))
        return p.value, nt.value

    def num_tiles(self):
        return int(L.lib().mcg_num_tiles(self._p))

    def tile_stats_into(self, dev_ptr):
        """Tile partials written into a caller-owned device buffer (an int device address of
        num_tiles() x (2D+3) doubles on this context's device), complete on return."""
        self._check(L.lib().mcg_tile_stats_into(self._p, C.c_void_p(int(dev_ptr))))

    def nested_rows_into(self, dev_ptr, row_stride, with_points=True):
        """The last nested run's rows (pts | ll | lp, or ll | lp) written into a caller-owned
        device buffer of n_total rows x row_stride doubles (an int device address on this
        context's device), complete on return (include/mcg.h mcg_nested_rows_into)."""
        self._check(L.lib().mcg_nested_rows_into(self._p, C.c_void_p(int(dev_ptr)), int(row_stride),
                                                 int(bool(with_points))))

    def stats(self):
        D = self.ndim
        mean = np.zeros(D); sd = np.zeros(D); lz = np.zeros(1)
        self._check(L.lib().mcg_stats(self._p, L.dptr(mean), L.dptr(sd), L.dptr(lz)))
        return mean, sd, float(lz[0])

    def set_timing(self, on=True):
        self._check(L.lib().mcg_set_timing(self._p, int(on)))

    def kernel_timing(self, kernel="mh"):
        t = L.McgKernelTiming()
        self._check(L.lib().mcg_get_kernel_timing(self._p, kernel.encode(), C.byref(t)))
        return dict(launches=t.launches, total_ms=t.total_ms, last_ms=t.last_ms)

    def reseed(self, seed):
        """Random.init seed: new Philox key, step counter back to 0 (include/mcg.h mcg_reseed)."""
        self._check(L.lib().mcg_reseed(self._p, seed))
        self.seed = seed

    def rng_step(self):
        """Philox step index of the next MH step."""
        return int(L.lib().mcg_rng_step(self._p))

    def sync(self):
        self._check(L.lib().mcg_sync(self._p))


def combine_tiles(ndim, tiles):
    tiles = np.ascontiguousarray(tiles, dtype=np.float64)
    mean = np.zeros(ndim); sd = np.zeros(ndim); lz = np.zeros(1)
    L.check(L.lib().mcg_combine_tiles(ndim, tiles.shape[0], L.dptr(tiles), L.dptr(mean),
                                      L.dptr(sd), L.dptr(lz)))
    return mean, sd, float(lz[0])
