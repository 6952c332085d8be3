"""Multi-process (world_size 2, gloo, CPU) test of the sharded-chain reduction path used by
bench.py for N > 1 GPUs: each rank samples its chain shard (global ids via chain_offset; the
oracle stands in for the GPU here), the tile partials are all-gathered with torch.distributed and
combined by libmcg's host combine -- the result must be bit-identical to one rank holding every
chain."""
import math
import sys
import os

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _model():
    import oracle as O
    D = 6
    rng = np.random.default_rng(42)
    mu = rng.uniform(-1, 1, D)
    sg = rng.uniform(0.5, 2, D)
    m = O.Model(D, 1, np.concatenate([mu, sg]), 1,
                np.concatenate([-10 * np.ones(D), 10 * np.ones(D), [-D * math.log(20)]]), 1, [0.9])
    return O, m, mu, sg


def _shard(rank, N):
    O, m, mu, sg = _model()
    x0 = np.random.default_rng(7).normal(mu[:, None], sg[:, None], size=(len(mu), 2 * N))
    x0 = x0[:, rank * N:(rank + 1) * N]
    ll = np.array([m.loglik(x0[:, i]) for i in range(N)])
    lp = np.array([m.logprior(x0[:, i]) for i in range(N)])
    r = O.mh_run(m, 3, x0, ll, lp, nbin=5, nskip=1, n_rec=40, chain_offset=rank * N,
                 record_x=False, record_llp=False)
    return O.tile_stats(len(mu), N, 40, r)


def _worker(rank, world, port, N, q):
    import sys
    for p in (os.path.join(ROOT, "mcmc-ocaml_amd"), os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mcmc_amd.parallel import allgather_tiles, reduce_stats
    tiles = _shard(rank, N)
    allt = allgather_tiles(tiles)
    mean, sd, lz = reduce_stats(6, tiles)
    q.put((rank, allt, mean, sd, lz))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_reduction_matches_single_rank():
    import random
    N = 512
    port = 29500 + random.randint(0, 2000)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, N, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda t: t[0])
    # single "rank" holding both shards: concatenated tiles in global order
    from mcmc_amd.context import combine_tiles
    full = np.concatenate([_shard(0, N), _shard(1, N)])
    ref = combine_tiles(6, full)
    for rank, allt, mean, sd, lz in res:
        np.testing.assert_array_equal(allt, full)
        np.testing.assert_array_equal(mean, ref[0])
        np.testing.assert_array_equal(sd, ref[1])
        assert lz == ref[2]


def test_replica_sizes_keep_k_below_nlive():
    """Per-replica (nlive, k) stay inside mcg_nested's bounds at any rank count (1 <= k < nlive,
    k <= 16384): nlive 32768 with k 2048 on 16 ranks gives 2048 live points and k 2047."""
    from mcmc_amd.parallel import MAX_K, replica_sizes
    assert replica_sizes(32768, 2048, 1) == (32768, 2048)
    assert replica_sizes(32768, 2048, 8) == (4096, 2048)
    assert replica_sizes(32768, 2048, 16) == (2048, 2047)
    assert replica_sizes(2 ** 20, 2 ** 15, 2) == (2 ** 19, MAX_K)
    assert replica_sizes(8, 1, 4) == (2, 1)
    with pytest.raises(ValueError):
        replica_sizes(100, 1, 3)          # not a multiple of the rank count
    with pytest.raises(ValueError):
        replica_sizes(4, 1, 4)            # one live point per replica


def test_c5_start_points_do_not_depend_on_sharding():
    """scripts/bench_c5.py: a chain's start point is a function of its global id, so any split of
    the global chains over ranks starts the same chains at the same points (the premise of the
    rank-count invariance the GPU test checks)."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import bench_c5 as b
    mu, cov, _ = b.c5_target()
    assert np.all(np.linalg.eigvalsh(cov) > 0)
    whole = b.start_points(mu, cov, 0, 4 * 8192 + 512)
    for world in (2, 4, 8):
        n = whole.shape[1] // world
        parts = [b.start_points(mu, cov, r * n, n) for r in range(world)]
        np.testing.assert_array_equal(np.concatenate(parts, axis=1), whole[:, :n * world])
