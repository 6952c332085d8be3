"""The RCCL leg of the multi-GPU path, run for real on one GPU: a one-rank "nccl"
process group (RCCL over xGMI on ROCm; one rank, so the collectives are local copies through
RCCL's own kernels) carries

  - the end-of-run exchange of the MH statistics: the tile kernel writes this rank's partials into
    a torch device buffer (mcg_tile_stats_into) that is the send buffer of all_gather_into_tensor,
    and the host folds the gathered tiles -- bit-identical to the host path (mcg_tile_stats +
    mcg_combine_tiles);
  - the nested replica exchange (allgather_runs): counts, then the padded (pts | ll | lp) rows --
    from host copies, or from the device (allgather_runs_device: mcg_nested_rows_into writes the
    run's rows into the RCCL send buffer), bit-identical.

The 2-rank versions of both run on gloo in tests/test_distributed.py."""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rccl():
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1)
    assert dist.get_backend() == "nccl"
    yield torch.device("cuda", 0)
    dist.destroy_process_group()


def test_tile_allgather_over_rccl_equals_host_combine(rccl):
    from mcmc_amd import Context, targets as T
    from mcmc_amd.context import combine_tiles
    from mcmc_amd.parallel import allgather_tiles_device, reduce_stats, reduce_stats_device
    D, N = 32, 4096 + 100                     # a partial last tile
    rng = np.random.default_rng(3)
    mu, sg = rng.uniform(-1, 1, D), rng.uniform(0.5, 2, D)
    ctx = Context(seed=5)
    ctx.set_model(T.diag_gauss(mu, sg), T.box(-10 * np.ones(D), 10 * np.ones(D)), T.gauss(0.3))
    ctx.init(rng.normal(mu[:, None], sg[:, None], size=(D, N)))
    ctx.run(nbin=10, nskip=1, n_rec=50, record_x=False, record_llp=False, accumulate=True)
    host_tiles = ctx.tile_stats()
    dev_tiles = allgather_tiles_device(ctx, rccl)
    np.testing.assert_array_equal(dev_tiles, host_tiles)
    a = reduce_stats_device(ctx, rccl)
    b = combine_tiles(D, host_tiles)
    c = reduce_stats(D, host_tiles, device=rccl)   # host tiles through RCCL's list all_gather
    for x, y, z in zip(a, b, c):
        np.testing.assert_array_equal(x, y)
        np.testing.assert_array_equal(x, z)
    assert np.max(np.abs(a[0] - mu)) < 0.5 and math.isfinite(a[2])
    ctx.close()


def test_nested_run_allgather_over_rccl(rccl):
    from mcmc_amd import Context, nested, targets as T
    from mcmc_amd.parallel import allgather_runs
    lik, pri = T.diag_gauss([0.5, 0.5], [0.1, 0.1]), T.box([0, 0], [1, 1], 0.0, open_=True)
    ctx = Context(seed=9)
    out = nested.nested_evidence(lik, pri, nlive=200, nmcmc=20, k=4, ctx=ctx)
    ctx.close()
    runs = allgather_runs(out, 200, 4, device=rccl)
    assert len(runs) == 1
    got, nl, k = runs[0]
    assert (nl, k) == (200, 4) and got.n_dead == out.n_dead and got.n_gen == out.n_gen
    np.testing.assert_array_equal(got[2], out[2])
    np.testing.assert_array_equal(got.ll, out.ll)
    np.testing.assert_array_equal(got.lp, out.lp)
    merged = nested.merge_runs(runs)
    np.testing.assert_array_equal(merged.ll, out.ll)


@pytest.mark.parametrize("points", [True, False])
def test_nested_device_allgather_equals_host_path(rccl, points):
    """The device-resident replica exchange (mcg_nested_rows_into -> all_gather_into_tensor) gives
    the host path's runs bit for bit, and the same merge; D 3 pads to the kernel width 4, so the
    rows are the caller's dims only."""
    from mcmc_amd import Context, nested, targets as T
    from mcmc_amd.parallel import allgather_runs, allgather_runs_device
    D = 3
    lik = T.gauss_shell(np.zeros(D), 1.0, 0.2)
    pri = T.box(-2 * np.ones(D), 2 * np.ones(D))
    with Context(seed=11) as ctx:
        res = nested.run_nested(lik, pri, nlive=300, nmcmc=15, k=8, ctx=ctx)
        host = nested.fetch(ctx, res, D, points=points, k=8)
        dev_runs = allgather_runs_device(ctx, res, 300, 8, rccl, points=points)
    host_runs = allgather_runs(host, 300, 8, device=rccl, points=points)
    assert len(dev_runs) == len(host_runs) == 1
    (d, dn, dk), (h, hn, hk) = dev_runs[0], host_runs[0]
    assert (dn, dk) == (hn, hk) == (300, 8)
    assert d.n_dead == h.n_dead == res.n_dead and d.n_gen == h.n_gen == res.n_gen
    np.testing.assert_array_equal(d.ll, host.ll)
    np.testing.assert_array_equal(d.lp, host.lp)
    if points:
        np.testing.assert_array_equal(d[2], host[2])
    else:
        assert d[2] is None
    a, b = nested.merge_runs(dev_runs), nested.merge_runs(host_runs)
    np.testing.assert_array_equal(a.ll, b.ll)
    np.testing.assert_array_equal(a[3], b[3])
    assert a[0] == b[0]
