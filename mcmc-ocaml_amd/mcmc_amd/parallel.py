"""Multi-GPU reduction of the MH statistics: one process per GPU (torch.distributed; "nccl" is
RCCL over xGMI on ROCm, "gloo" on CPU for tests).

Chains are sharded in contiguous blocks (rank r owns global chain ids [r*N, (r+1)*N), passed to
the context as chain_offset), so every chain's Philox stream is independent of the GPU count.
The only exchange of a run is this end-of-run all-gather of the fixed-size 256-chain tile
partials (2D+3 doubles per tile); every rank then folds the tiles in global order with
mcg_combine_tiles, which makes the moments and the harmonic-mean evidence bit-identical for any
number of GPUs.
"""
import numpy as np

from .context import combine_tiles


def allgather_tiles(tiles, device=None, group=None):
    """All-gather every rank's tile partials (same tile count per rank), in rank order."""
    import torch
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
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
