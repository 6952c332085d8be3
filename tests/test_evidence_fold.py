"""The host evidence fold (EvFold in csrc/mcg_nested.cpp, exported as mcg_evidence_weights): the
fold mcg_nested runs on host threads beside the GPU, here on CPU inputs.  It must give the
oracle's evidence_error_and_weights (nested.ml:81-120, oracle.c or_evidence_weights) bit for bit
over several fold blocks (65,536 iterations each), for k = 1 and k > 1, whatever chunks the dead
points stream in, and with -inf log-likelihoods (the lse shortcut for a -inf side)."""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def nested():
    from mcmc_amd import nested
    return nested


def _run(ntot, nlive, seed, ninf=0):
    rng = np.random.default_rng(seed)
    ll = np.sort(rng.normal(size=ntot) * 3.0)
    ll[:ninf] = -np.inf
    return ll


@pytest.mark.parametrize("ntot,nlive,k,ninf", [
    (300, 50, 1, 0),
    (150_000 + 2048, 2048, 1, 3),          # three fold blocks of dead points, k = 1
    (256_000 + 16_384, 16_384, 512, 0),    # four blocks, k > 1: the C3 shape at a sixteenth
    (70_000, 4096, 2048, 5),               # live points crossing a block edge
])
def test_host_fold_equals_oracle(oracle, nested, ntot, nlive, k, ninf):
    ll = _run(ntot, nlive, 7 + k, ninf)
    le, ld, w = nested.evidence_weights(ll, nlive, k)
    ole, old, ow = oracle.evidence_weights(ll, nlive, k)
    assert le == ole and ld == old
    np.testing.assert_array_equal(w, ow)


@pytest.mark.parametrize("chunk", [1, 4096, 12_345, 65_536, 10**9])
def test_host_fold_does_not_depend_on_streaming(nested, chunk):
    ll = _run(200_000 + 8192, 8192, 3, 2)
    ref = nested.evidence_weights(ll, 8192, 256)
    got = nested.evidence_weights(ll, 8192, 256, chunk=chunk)
    assert got[0] == ref[0] and got[1] == ref[1]
    np.testing.assert_array_equal(got[2], ref[2])


def test_host_fold_rejects_bad_sizes(nested):
    from mcmc_amd._lib import McgError
    ll = np.zeros(10)
    for nlive, k in [(20, 1), (4, 8), (4, 4), (4, 0)]:
        with pytest.raises(McgError):
            nested.evidence_weights(ll, nlive, k)
