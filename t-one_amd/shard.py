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


def broadcast_weights(weights, src: int = 0, group=None, device=None):
    """Checkpoint replica on every rank from ONE load on ``src`` (weights are
    broadcast once).  ``weights`` is the state dict on ``src`` (ignored elsewhere); all ranks get an
    OrderedDict of fp32 numpy arrays in the ``PARAM_SHAPES`` catalogue order.  The whole checkpoint
    travels as one flat fp32 tensor (287 MB, one collective): on ``device`` (RCCL over xGMI with the
    "nccl" backend) or on the host (gloo)."""
    from collections import OrderedDict

    import numpy as np
    import torch
    import torch.distributed as dist

    from .weights import N_PARAMS, PARAM_SHAPES

    rank = dist.get_rank(group)
    if rank == src:
        missing = [k for k in PARAM_SHAPES if k not in weights]
        if missing:
            raise KeyError(f"checkpoint lacks {len(missing)} tensors, e.g. {missing[0]}")
        flat = np.concatenate([np.asarray(weights[k], np.float32).reshape(-1) for k in PARAM_SHAPES])
        buf = torch.from_numpy(flat)
        if device is not None:
            buf = buf.to(device)
    else:
        buf = torch.empty(N_PARAMS, dtype=torch.float32, device=device)
    dist.broadcast(buf, src=src if group is None else dist.get_global_rank(group, src), group=group)
    host = buf.cpu().numpy()
    out, o = OrderedDict(), 0
    for k, shp in PARAM_SHAPES.items():
        n = int(np.prod(shp))
        out[k] = host[o: o + n].reshape(shp)
        o += n
    return out


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
