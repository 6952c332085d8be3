"""Read_write text formats (read_write.ml:19-101) through libmcg's native writer/reader: the
reference's own round-trip tests (test/read_write_test.ml) and exact text against Printf "%g"
(Python's "%g" is C's %g).  Host-only: no GPU needed."""
import math

import numpy as np
import pytest


@pytest.fixture
def RW(gpu_lib):
    from mcmc_amd import read_write
    return read_write


def _samples(n, D, N, seed=0):
    from mcmc_amd.mcmc import Samples
    rng = np.random.default_rng(seed)
    x = rng.normal(size=(n, D, N)) * 10.0 ** rng.integers(-8, 8, size=(n, D, N))
    return Samples(x, rng.normal(size=(n, N)) - 50, np.full((n, N), -math.log(20.0)))


def test_read_write_inverses(RW, tmp_path):
    """test/read_write_test.ml:23-45: write then read gives the samples back within 1e-3."""
    s = _samples(1000, 1, 1)
    f = tmp_path / "mcmc_test.dat"
    RW.write(f, s)
    r = RW.read(f)
    np.testing.assert_allclose(r.value, s.value, rtol=1e-3, atol=1e-3)
    np.testing.assert_allclose(r.log_likelihood, s.log_likelihood, rtol=1e-3, atol=1e-3)
    np.testing.assert_allclose(r.log_prior, s.log_prior, rtol=1e-3, atol=1e-3)


def test_text_is_printf_g(RW, tmp_path):
    """Every field is "%g", fields separated by one space, one sample per line
    (read_write.ml:19-24); chains are written one after another."""
    s = _samples(7, 3, 2, seed=1)
    f = tmp_path / "s.dat"
    RW.write(f, s)
    want = []
    for c in range(2):
        for i in range(7):
            vals = list(s.value[i, :, c]) + [s.log_likelihood[i, c], s.log_prior[i, c]]
            want.append(" ".join("%g" % v for v in vals))
    assert f.read_text() == "\n".join(want) + "\n"


def test_large_parallel_write_matches_sequential_format(RW, tmp_path):
    rng = np.random.default_rng(5)
    rows = rng.standard_cauchy(size=(70000, 4))
    rows[::997, 1] = np.inf
    rows[::991, 2] = -np.inf
    f = tmp_path / "big.dat"
    RW.write_rows(f, rows)
    text = f.read_text().splitlines()
    assert len(text) == rows.shape[0]
    for i in (0, 1, 997, 991 * 3, 69999):
        assert text[i] == " ".join("%g" % v for v in rows[i])
    back, _ = RW.read_rows(f)
    np.testing.assert_allclose(back, rows, rtol=1e-5)


def test_nested_read_write(RW, tmp_path):
    """test/read_write_test.ml:47-78 on a nested output: log_ev, log_dev, samples and log
    weights survive a write_nested / read_nested round trip within 1%."""
    from mcmc_amd.nested import NestedOutput
    rng = np.random.default_rng(2)
    n = 300
    ll = np.sort(rng.normal(size=n))
    w = ll - np.log(np.exp(ll).sum())
    out = NestedOutput(-1.2345678, -4.5, rng.random((n, 1)), w, ll, np.zeros(n), n - 50, 10)
    f = tmp_path / "nested_test.dat"
    RW.write_nested(f, out)
    assert f.read_text().splitlines()[0] == "%g %g" % (-1.2345678, -4.5)
    r = RW.read_nested(f)
    assert abs(r[0] - out[0]) <= 0.01 * abs(out[0]) and abs(r[1] - out[1]) <= 0.01 * abs(out[1])
    np.testing.assert_allclose(r[2], out[2], rtol=1e-3, atol=1e-3)
    np.testing.assert_allclose(r.ll, ll, rtol=1e-3, atol=1e-3)
    np.testing.assert_allclose(r[3], w, rtol=0.01)


def test_reader_accepts_blanks_and_rejects_ragged_rows(RW, tmp_path):
    f = tmp_path / "odd.dat"
    f.write_text("  1 2\t3   \n\n4 5 6\n nan -inf 7\n")
    r, _ = RW.read_rows(f)
    assert r.shape == (3, 3) and math.isnan(r[2, 0]) and r[2, 1] == -np.inf
    g = tmp_path / "ragged.dat"
    g.write_text("1 2 3\n4 5\n")
    from mcmc_amd._lib import Failure
    with pytest.raises(Failure):
        RW.read_rows(g)
    h = tmp_path / "bad.dat"
    h.write_text("1 x 3\n")
    with pytest.raises(Failure):
        RW.read_rows(h)


def test_write_sample_appends(RW, tmp_path):
    f = tmp_path / "one.dat"
    RW.write_sample(f, [0.5, 1e-9], -3.0, 0.0, append=False)
    RW.write_sample(f, [1.5, 2.0], -4.0, 0.0)
    assert f.read_text() == "0.5 1e-09 -3 0\n1.5 2 -4 0\n"
