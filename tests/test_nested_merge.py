"""Nested replicas: independent runs, one per GPU, merged into one run.

CPU tests: libmcg's host merge (mcg_nested_merge) against the oracle's restatement
(oracle.nested_merge), the statistical properties of merged runs on the reference's
nested_test.ml target, and the world-size-2 gloo all-gather path.  The runs themselves are
produced by the oracle here (test data); the GPU test drives the real replicas."""
import math
import os

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIK_DIAG, PRIOR_OPEN, PROP_GAUSS = 1, 2, 1


def _unit_square_gauss(O):
    """test/nested_test.ml:23-28: N((0.5, 0.5), 0.1^2) in the open unit square, Z = 1."""
    return O.Model(2, LIK_DIAG, [0.5, 0.5, 0.1, 0.1], PRIOR_OPEN, [0, 0, 1, 1, 0.0], PROP_GAUSS, [1.0])


def _runs(O, seeds, nlive, k=1, nmcmc=60):
    m = _unit_square_gauss(O)
    return [O.nested(m, s, nlive=nlive, nmcmc=nmcmc, k=k) for s in seeds]


def _merge(runs, nlive, k):
    from mcmc_amd import nested
    outs = [(nested.NestedOutput(r["log_ev"], r["log_dev"], r["pts"], r["log_wts"], r["ll"],
                                 r["lp"], r["n_dead"], r["n_gen"]), nlive, k) for r in runs]
    return nested.merge_runs(outs)


@pytest.mark.parametrize("k", [1, 4])
def test_merge_matches_oracle_restatement(oracle, k):
    runs = _runs(oracle, [3, 4, 5], 48, k=k)
    got = _merge(runs, 48, k)
    order, le, ld, w = oracle.nested_merge([(r["ll"], 48, k) for r in runs])
    cat = np.concatenate([r["ll"] for r in runs])
    np.testing.assert_array_equal(got.ll, cat[order])
    np.testing.assert_allclose(got[0], le, rtol=1e-13)
    np.testing.assert_allclose(got[1], ld, rtol=1e-13)
    np.testing.assert_allclose(got[3], w, rtol=1e-12, atol=1e-12)
    assert np.all(np.diff(got.ll) >= 0)
    assert abs(np.exp(got[3]).sum() - 1.0) < 1e-8


def test_merge_of_one_run_is_the_reference_estimate(oracle):
    """A single run through the merge differs from evidence_error_and_weights (nested.ml:81-120)
    only in how the final live points share the last volume (retired one by one with counts
    n, n-1, .., 1 instead of equal shares): far below the run's own error."""
    r = _runs(oracle, [11], 200, nmcmc=100)[0]
    got = _merge([r], 200, 1)
    err = math.exp(oracle.lib().or_log_total_error_estimate(r["log_ev"], r["log_dev"], 200))
    assert abs(math.exp(got[0]) - math.exp(r["log_ev"])) < 0.05 * err
    np.testing.assert_array_equal(got.ll, r["ll"])


def test_merged_replicas_estimate_unit_evidence(oracle):
    """nested_test.ml:23-39 on merged runs: 4 replicas of 250 live points = one run of 1000.

    The reference's check |Z - 1| < 2 err is a ~1.5-sigma test: log_total_error_estimate
    (nested.ml:148-150) puts err ~ Z / sqrt(nlive), while the spread of Z is Z sqrt(H / nlive)
    with H ~ 1.8 nats here, so a single seed set fails it now and then, as the reference test
    itself would.  The check is therefore made on an ensemble of 12 consecutive seed sets
    (21-24, 25-28, ..., 65-68; no selection): the mean of (Z - 1)/err must be within 3 standard
    errors of 0 (a systematic evidence bias of ~1.4 err would fail it), the spread must stay near
    the sqrt(H)-inflated error scale, and most sets must pass the reference's own 2-err check.
    (Spec v7: mean -0.19, sd 1.58, 10 of 12 sets pass.)"""
    zs = []
    for base in range(21, 21 + 4 * 12, 4):
        got = _merge(_runs(oracle, [base, base + 1, base + 2, base + 3], 250, nmcmc=1000), 250, 1)
        ev = math.exp(got[0])
        err = math.exp(oracle.lib().or_log_total_error_estimate(got[0], got[1], 1000))
        assert err < 0.1
        w = np.exp(got[3])
        assert abs(w.sum() - 1.0) < 1e-8
        assert abs((w * got[2][:, 0]).sum() - 0.5) < 0.1
        # the merged run is one run of 1000 live points: its information gives the error scale
        assert float(np.sum(w * got.ll) - got[0]) > 0
        zs.append((ev - 1.0) / err)
    zs = np.array(zs)
    sd = zs.std(ddof=1)
    assert abs(zs.mean()) < 3 * sd / math.sqrt(len(zs)), zs
    assert 0.5 < sd < 2.5, zs
    assert np.sum(np.abs(zs) < 2) >= 8, zs


def test_merge_rejects_bad_arguments(gpu_lib):
    from mcmc_amd import nested
    bad = nested.NestedOutput(0.0, 0.0, np.zeros((3, 1)), None, np.zeros(3), np.zeros(3), 0, 0)
    with pytest.raises(Exception):
        nested.merge_runs([(bad, 5, 1)])        # fewer points than live points


def _worker(rank, world, port, q):
    import sys
    for p in (os.path.join(ROOT, "mcmc-ocaml_amd"), os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    import torch.distributed as dist
    import oracle as O
    from mcmc_amd import nested
    from mcmc_amd.parallel import allgather_runs, replica_seed
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    r = O.nested(_unit_square_gauss(O), replica_seed(9, rank), nlive=40, nmcmc=40)
    out = nested.NestedOutput(r["log_ev"], r["log_dev"], r["pts"], r["log_wts"], r["ll"], r["lp"],
                              r["n_dead"], r["n_gen"])
    merged = nested.merge_runs(allgather_runs(out, 40, 1))
    light = nested.merge_runs(allgather_runs(out, 40, 1, points=False))   # ll / lp only
    assert light[2] is None and light[0] == merged[0]
    np.testing.assert_array_equal(light[3], merged[3])
    q.put((rank, merged[0], merged[1], merged.ll, merged[2], merged[3]))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_replica_merge():
    """Each rank runs a replica, the runs are all-gathered (torch.distributed, gloo) and merged on
    every rank: both ranks hold the merge of the two runs made in one process."""
    import random
    import oracle as O
    port = 29500 + random.randint(2001, 4000)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(2)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from mcmc_amd.parallel import replica_seed
    runs = [O.nested(_unit_square_gauss(O), replica_seed(9, r), nlive=40, nmcmc=40)
            for r in range(2)]
    ref = _merge(runs, 40, 1)
    for _, le, ld, ll, pts, w in res:
        assert le == ref[0] and ld == ref[1]
        np.testing.assert_array_equal(ll, ref.ll)
        np.testing.assert_array_equal(pts, ref[2])
        np.testing.assert_array_equal(w, ref[3])
