"""Multi-GPU reduction of the MH statistics: one process per GPU (torch.distributed; "nccl" is
RCCL over xGMI on ROCm, "gloo" on CPU for tests).

Chains are sharded in contiguous blocks (rank r owns global chain ids [r*N, (r+1)*N), passed to
the context as chain_offset), so every chain's Philox stream is independent of the GPU count.
The only exchange of a run is this end-of-run all-gather of the fixed-size 256-chain tile
partials (2D+3 doubles per tile); every rank then folds the tiles in global order with
mcg_combine_tiles, which makes the moments and the harmonic-mean evidence bit-identical for any
number of GPUs.
"""
import os
import sys
import warnings

import numpy as np

from . import nested as _nested
from .context import Context, combine_tiles

MAX_K = 16384          # mcg_nested's cap on points retired per generation (include/mcg.h)

GOLDEN64 = 0x9E3779B97F4A7C15


def allgather_tiles(tiles, device=None, group=None):
    """All-gather every rank's tile partials (same tile count per rank), in rank order."""
    import torch
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized():
        return np.asarray(tiles)
    t = torch.from_numpy(np.ascontiguousarray(tiles, dtype=np.float64))
    if device is not None:
        t = t.to(device)
    out = [torch.empty_like(t) for _ in range(dist.get_world_size(group))]
    dist.all_gather(out, t, group=group)
    return torch.cat(out).cpu().numpy()


def reduce_stats(ndim, tiles, device=None, group=None):
    """Global Stats.multi_mean / multi_std and log Z_HM from this rank's tile partials."""
    return combine_tiles(ndim, allgather_tiles(tiles, device, group))


def allgather_tiles_device(ctx, device, group=None):
    """The device path of the end-of-run exchange (RCCL over xGMI): the tile kernel writes this
    rank's partials straight into a torch device buffer (mcg_tile_stats_into), which is the send
    buffer of one all_gather_into_tensor; only the gathered tiles come back to the host for the
    combine.  The collective runs whenever a process group is up -- a one-rank group too, so the
    RCCL leg is exercised on one GPU -- and is skipped only without torch.distributed."""
    import torch
    import torch.distributed as dist
    nt, w = ctx.num_tiles(), 2 * ctx.ndim + 3
    send = torch.empty((nt, w), dtype=torch.float64, device=device)
    # the buffer comes from torch's caching allocator: let torch's own stream finish with the
    # memory before the context's stream writes it
    torch.cuda.synchronize(device)
    ctx.tile_stats_into(send.data_ptr())
    if not dist.is_available() or not dist.is_initialized():
        return send.cpu().numpy()
    recv = torch.empty((dist.get_world_size(group) * nt, w), dtype=torch.float64, device=device)
    dist.all_gather_into_tensor(recv, send, group=group)
    return recv.cpu().numpy()


def reduce_stats_device(ctx, device, group=None):
    """reduce_stats over the device path (allgather_tiles_device): the same bits as the host
    path, every rank folding the gathered tiles in global order."""
    return combine_tiles(ctx.ndim, allgather_tiles_device(ctx, device, group))


def replica_seed(seed, rank):
    """Philox key of nested replica `rank`: rank 0 keeps the caller's seed, so a one-GPU run is
    the single-context run exactly."""
    return (int(seed) + int(rank) * GOLDEN64) % (1 << 64)


def _world(group):
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized():
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


def allgather_runs(output, nlive, k, device=None, group=None, points=True):
    """All-gather every rank's nested run: the point counts first, then the (pts | ll | lp) rows
    padded to the longest run (points=False: ll | lp only, enough for log Z).  Returns
    [(output, nlive, k)] in rank order."""
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized():
        return [(output, nlive, k)]
    import torch
    rank, world = _world(group)
    pts = np.asarray(output[2], np.float64) if points else np.zeros((len(output.ll), 0))
    D = pts.shape[1]
    rows = np.concatenate([pts, output.ll[:, None], output.lp[:, None]], axis=1)
    meta = torch.tensor([rows.shape[0], nlive, k, output.n_gen], dtype=torch.int64, device=device)
    metas = [torch.empty_like(meta) for _ in range(world)]
    dist.all_gather(metas, meta, group=group)
    metas = [m.cpu().numpy() for m in metas]
    cap = int(max(m[0] for m in metas))
    buf = np.zeros((cap, D + 2))
    buf[:rows.shape[0]] = rows
    t = torch.from_numpy(buf).to(device) if device is not None else torch.from_numpy(buf)
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t, group=group)
    runs = []
    for m, o in zip(metas, outs):
        r = o.cpu().numpy()[:int(m[0])]
        run = _nested.NestedOutput(0.0, 0.0, r[:, :D].copy() if points else None, None, r[:, D].copy(),
                                   r[:, D + 1].copy(), int(m[0] - m[1]), int(m[3]))
        runs.append((run, int(m[1]), int(m[2])))
    return runs


def allgather_runs_device(ctx, res, nlive, k, device, group=None, points=True):
    """allgather_runs from the device: the finished run's rows (pts | ll | lp, or ll | lp) are
    written by mcg_nested_rows_into straight into a torch device buffer padded to the longest run,
    which is the send buffer of one all_gather_into_tensor (RCCL over xGMI); only the gathered rows
    come back to the host, for the merge.  res: the run's McgNestedResult (nested.run_nested).
    Returns [(output, nlive, k)] in rank order, equal to allgather_runs of the same runs."""
    import torch
    import torch.distributed as dist
    rank, world = _world(group)
    D = ctx.ndim if points else 0
    w = D + 2
    meta = torch.tensor([res.n_total, nlive, k, res.n_gen, int(bool(res.converged))], dtype=torch.int64,
                        device=device)
    metas = torch.empty((world, meta.numel()), dtype=torch.int64, device=device)
    if dist.is_available() and dist.is_initialized():
        dist.all_gather_into_tensor(metas, meta, group=group)
    else:
        metas[0] = meta
    metas = metas.cpu().numpy()
    cap = int(metas[:, 0].max())
    send = torch.zeros((cap, w), dtype=torch.float64, device=device)
    # the buffer comes from torch's caching allocator: let torch's stream finish with it before
    # the context's stream writes it
    torch.cuda.synchronize(device)
    ctx.nested_rows_into(send.data_ptr(), w, points)
    if dist.is_available() and dist.is_initialized():
        recv = torch.empty((world * cap, w), dtype=torch.float64, device=device)
        dist.all_gather_into_tensor(recv, send, group=group)
    else:
        recv = send
    allr = recv.cpu().numpy().reshape(world, cap, w)
    runs = []
    for m, r in zip(metas, allr):
        r = r[:int(m[0])]
        run = _nested.NestedOutput(0.0, 0.0, r[:, :D].copy() if points else None, None, r[:, D].copy(),
                                   r[:, D + 1].copy(), int(m[0] - m[1]), int(m[3]), bool(m[4]))
        runs.append((run, int(m[1]), int(m[2])))
    return runs


def replica_sizes(nlive, k, world):
    """(live points, points retired per generation) of one of `world` replicas: nlive / world
    live points, k clamped to what mcg_nested accepts (1 <= k < nlive, k <= MAX_K)."""
    if nlive % world:
        raise ValueError("nlive (%d) must be a multiple of the number of ranks (%d)" % (nlive, world))
    nl = nlive // world
    if nl < 2:
        raise ValueError("nlive / ranks = %d: every replica needs at least 2 live points" % nl)
    return nl, max(1, min(k, nl - 1, MAX_K))


def nested_evidence_replicas(log_likelihood, log_prior, epsrel=0.01, nmcmc=1000, nlive=1000,
                             mode_hopping_frac=0.1, k=1, seed=0, device=0, group=None,
                             comm_device=None, points=True):
    """Nested.nested_evidence (nested.ml:122-146) as one replica per GPU: every
    rank runs an independent nested run with nlive / world live points on its own Philox key,
    the runs are all-gathered and merged (mcg_nested_merge) into one run of nlive points.  Every
    rank returns the same merged NestedOutput (points=False: gather ll / lp only; the merged
    output then has no points)."""
    rank, world = _world(group)
    nl, kk = replica_sizes(nlive, k, world)
    if kk != k:
        warnings.warn("nested_evidence_replicas: k = %d retired per generation cannot run on "
                      "%d live points per replica; using k = %d (recorded as .k)" % (k, nl, kk),
                      RuntimeWarning, stacklevel=2)
    # RCCL (comm_device set) with several ranks: the exchange reads the run's rows on the device
    # (allgather_runs_device); otherwise (one rank, or a gloo rehearsal) the host copy is used
    dev_x = world > 1 and comm_device is not None
    with Context(seed=replica_seed(seed, rank), device=device) as ctx:
        if dev_x:
            res = _nested.run_nested(log_likelihood, log_prior, epsrel=epsrel, nmcmc=nmcmc, nlive=nl,
                                     mode_hopping_frac=mode_hopping_frac, k=kk, ctx=ctx)
            runs = allgather_runs_device(ctx, res, nl, kk, comm_device, group, points=points)
            out = runs[rank][0]
            out = _nested.NestedOutput(res.log_ev, res.log_dev, out[2], None, out.ll, out.lp,
                                       res.n_dead, res.n_gen, bool(res.converged))
        else:
            out = _nested.nested_evidence(log_likelihood, log_prior, epsrel=epsrel, nmcmc=nmcmc,
                                          nlive=nl, mode_hopping_frac=mode_hopping_frac, k=kk, ctx=ctx,
                                          points=points)
    if os.environ.get("MCG_DEBUG_REPLICAS"):
        print("replica rank %d: log Z %.6f n_dead %d n_gen %d" % (rank, out[0], out.n_dead, out.n_gen),
              file=sys.stderr, flush=True)
    if world == 1:
        out.k = kk
        return out
    if not dev_x:
        runs = allgather_runs(out, nl, kk, comm_device, group, points=points)
    merged = _nested.merge_runs(runs)
    if os.environ.get("MCG_DEBUG_REPLICAS"):
        for i, (o, a, b) in enumerate(runs):
            print("rank %d sees run %d: n %d nlive %d k %d ll[0] %.4f ll[-1] %.4f sorted %s" % (
                rank, i, len(o.ll), a, b, o.ll[0], o.ll[-1], bool(np.all(np.diff(o.ll) >= 0))),
                file=sys.stderr, flush=True)
        print("rank %d merged log Z %.6f" % (rank, merged[0]), file=sys.stderr, flush=True)
    merged.k = kk
    return merged
