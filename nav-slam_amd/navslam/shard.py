"""Multi-GPU plumbing of the benchmark configurations.

One process per GPU. K3: every rank matches its own scan pair (replicas, no
data-path collective). K4: the batch of independent pairs is split into
contiguous blocks over the ranks, and the per-pair match buffers are
all-gathered once (RCCL over xGMI on the GPU box, gloo in the CPU tests).
"""
import torch
import torch.distributed as dist


def pair_seeds(rank):
    """(source, target) seeds of rank r's K3 pair: (1 + 2r, 2 + 2r)."""
    return 1 + 2 * rank, 2 + 2 * rank


def shard_pairs(total, world, rank):
    """Contiguous block [lo, hi) of `total` pairs owned by `rank`; the first
    total % world ranks take one extra pair."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    base, extra = divmod(total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def max_over_ranks(value, device):
    """Max of a float over all ranks (the slowest rank's time)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value, device):
    """Sum of a count over all ranks (matches of the whole job)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def gather_matches(local, out=None):
    """All-gather the per-pair match buffers of every rank, in rank order:
    local [p, ...] -> [world * p, ...]. Every rank must hold the same p (K4
    sizes the shards so; a ragged tail is padded by the caller)."""
    world = dist.get_world_size()
    if out is None:
        out = torch.empty((world * local.shape[0],) + tuple(local.shape[1:]),
                          dtype=local.dtype, device=local.device)
    if dist.get_backend() == "nccl":
        dist.all_gather_into_tensor(out, local)
    else:  # gloo: list form
        parts = list(out.chunk(world, dim=0))
        dist.all_gather(parts, local)
    return out
