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


def match_views(packed, pairs, R, C):
    """The K4 match set of `pairs` pairs as one packed byte buffer of
    pairs * R * C * 12 bytes: nn_idx [pairs][R][C] int32 first, then nn_dist
    [pairs][R][C] float64 (idx + dist, 12 B per match). Returns the
    (idx, dist) views the kernels write into."""
    n = pairs * R * C
    if packed.numel() != 12 * n or packed.dtype != torch.uint8:
        raise ValueError("packed match buffer must be uint8[pairs*R*C*12]")
    idx = packed[: 4 * n].view(torch.int32).view(pairs, R, C)
    dist = packed[4 * n:].view(torch.float64).view(pairs, R, C)
    return idx, dist


def unpack_gathered(gathered, world, pairs, R, C):
    """Rank-ordered (idx [world*pairs][R][C], dist [world*pairs][R][C]) from
    the all-gathered packed buffers."""
    parts = gathered.view(world, -1)
    idx = torch.cat([match_views(parts[w], pairs, R, C)[0] for w in range(world)])
    dist = torch.cat([match_views(parts[w], pairs, R, C)[1] for w in range(world)])
    return idx, dist


def gather_matches(local, out=None):
    """All-gather the per-pair match buffers of every rank, in rank order:
    local [p, ...] -> [world * p, ...]. Every rank must hold the same p (K4
    sizes the shards so: ceil(total / world) slots per rank, the ragged
    tail's unused slots padded by the caller)."""
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
