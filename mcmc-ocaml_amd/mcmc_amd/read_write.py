"""Mirror of the reference's Read_write module (read_write.mli) over libmcg's native text I/O.

Same file formats as read_write.ml:19-101 (OCaml Printf "%g", space separated, one sample per
line), so GPU output feeds the reference's tools (bin/evidence_tool.ml:44,
bin/harmonic_evidence.ml:39) and the reference's files load here.  Samples are the
structure-of-arrays records of mcmc_amd.mcmc.Samples; a file holds one chain's samples in
record order, or several chains one after another (chain-major).
"""
import ctypes as C
import os

import numpy as np

from . import _lib as L
from .mcmc import Samples
from .nested import NestedOutput


def _path(f):
    return os.fsencode(f if isinstance(f, (str, bytes, os.PathLike)) else f.name)


def _check(rc, what):
    if rc != L.MCG_OK:
        raise (L.InvalidArgument if rc == L.MCG_EINVAL else L.Failure)(rc, what)


def write_rows(path, rows, header=None, append=False):
    rows = np.ascontiguousarray(rows, dtype=np.float64)
    if rows.ndim == 1:
        rows = rows[None, :]
    _check(L.lib().mcg_write_rows(_path(path), int(append), None if header is None else header.encode(),
                                  rows.shape[0], rows.shape[1], L.dptr(rows)), "write %s" % path)


def read_rows(path, skip_lines=0, nheader=0):
    n = C.c_int64()
    m = C.c_int32()
    _check(L.lib().mcg_read_rows_shape(_path(path), skip_lines, C.byref(n), C.byref(m)), "read %s" % path)
    rows = np.zeros((n.value, m.value))
    hdr = np.zeros(nheader) if nheader else None
    _check(L.lib().mcg_read_rows(_path(path), skip_lines, n.value, m.value, L.dptr(rows), L.dptr(hdr),
                                 nheader), "read %s" % path)
    return rows, hdr


def _sample_rows(samples, chains):
    x, ll, lp = samples.value, samples.log_likelihood, samples.log_prior   # (n, D, N), (n, N)
    chains = range(x.shape[2]) if chains is None else np.atleast_1d(chains)
    return np.concatenate([np.column_stack([x[:, :, c], ll[:, c], lp[:, c]]) for c in chains])


def write(path, samples, chains=None, append=False):
    """Read_write.write (read_write.ml:26-30): every record of the selected chains (default all,
    chain after chain), one line each: coords, log_likelihood, log_prior."""
    write_rows(path, _sample_rows(samples, chains), append=append)


def write_sample(path, value, log_likelihood, log_prior, append=True):
    """Read_write.write_sample (read_write.ml:19-24): one line."""
    write_rows(path, np.concatenate([np.atleast_1d(value), [log_likelihood, log_prior]]), append=append)


def read(path):
    """Read_write.read (read_write.ml:46-56): one chain of samples, as Samples with N = 1."""
    rows, _ = read_rows(path)
    if rows.shape[1] < 2:
        raise L.Failure(L.MCG_EFAIL, "read %s: fewer than two fields per line" % path)
    return Samples(rows[:, :-2, None].copy(), rows[:, -2:-1].copy(), rows[:, -1:].copy())


def write_nested(path, output):
    """Read_write.write_nested (read_write.ml:58-66): "log_ev log_dev", then coords, ll, lp, log_wt."""
    log_ev, log_dev, pts, wts = output[0], output[1], np.asarray(output[2]), np.asarray(output[3])
    head = "%s %s\n" % (_g(log_ev), _g(log_dev))
    write_rows(path, np.column_stack([pts, output.ll, output.lp, wts]), header=head)


def read_nested(path):
    """Read_write.read_nested (read_write.ml:90-101) -> NestedOutput."""
    rows, hdr = read_rows(path, skip_lines=1, nheader=2)
    D = rows.shape[1] - 3
    return NestedOutput(float(hdr[0]), float(hdr[1]), rows[:, :D].copy(), rows[:, D + 2].copy(),
                        rows[:, D].copy(), rows[:, D + 1].copy(), 0, 0)


def _g(v):
    return "nan" if v != v else "%g" % v
