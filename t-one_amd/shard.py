"""Data-parallel sharding of independent streams across the GPUs of a node.

Streams never interact (eval-mode BatchNorm, per-stream masks and state), so a batch
of B streams is split into contiguous per-rank blocks with no collective on the data path.  The
only exchange is the host-decoding hand-off: every rank's logprobs [B_r, 10, 35] are all-gathered
(RCCL over xGMI with the "nccl" backend; gloo in the CPU tests) so that the decoding rank holds the
whole batch in stream order.  Shards of unequal size are padded to the largest shard for the
collective and trimmed afterwards.
"""

from __future__ import annotations


def shard_bounds(n_streams: int, world: int, rank: int) -> tuple[int, int]:
    """[start, end) of rank's contiguous block; the first n % world ranks get one extra stream."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} for world {world}")
    base, extra = divmod(n_streams, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def shard_sizes(n_streams: int, world: int) -> list[int]:
    return [e - s for s, e in (shard_bounds(n_streams, world, r) for r in range(world))]


def gather_logprobs(local, n_streams: int, group=None):
    """All-gather every rank's logprobs (B_r, T, V) into (n_streams, T, V) in global stream order."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    sizes = shard_sizes(n_streams, world)
    cap = max(sizes)
    if local.shape[0] != sizes[dist.get_rank(group)]:
        raise ValueError(f"local shard has {local.shape[0]} streams, expected {sizes[dist.get_rank(group)]}")
    if local.shape[0] < cap:
        pad = torch.zeros((cap - local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        local = torch.cat([local, pad])
    out = torch.empty((world * cap,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, local.contiguous(), group=group)
    if all(s == cap for s in sizes):
        return out
    return torch.cat([out[r * cap: r * cap + s] for r, s in enumerate(sizes)])
