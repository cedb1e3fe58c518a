"""Data-parallel sharding of a metric batch over the ranks of one node.

Every utterance is independent: rank r scores its own contiguous shard of the
batch with no exchange during compute, then ONE all-gather of the per-utterance score
vectors (RCCL over xGMI with the "nccl" backend on MI355X; gloo on CPU) gives every rank the
full result.  The message is [B, k] float32 (k = 1 for PESQ, 2 for STOI/ESTOI): latency-bound.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_bounds(batch: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous, balanced [start, stop) of `rank` (shards differ by at most one)."""
    base, extra = divmod(batch, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def gather_scores(local: torch.Tensor, batch: int, group=None) -> torch.Tensor:
    """All-gather per-rank score rows [n_r, k] into [batch, k] (rank order)."""
    world = dist.get_world_size(group)
    k = local.shape[1]
    cap = -(-batch // world)  # ceil: shards are padded to equal length for the collective
    buf = torch.zeros(cap, k, dtype=local.dtype, device=local.device)
    buf[:local.shape[0]] = local
    out = torch.empty(world * cap, k, dtype=local.dtype, device=local.device)
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, buf, group=group)
    else:
        dist.all_gather(list(out.chunk(world)), buf, group=group)
    rows = [out[r * cap:r * cap + (shard_bounds(batch, world, r)[1] - shard_bounds(batch, world, r)[0])]
            for r in range(world)]
    return torch.cat(rows, 0)


def sharded_scores(metric, clean: torch.Tensor, noisy: torch.Tensor, group=None, **kw) -> torch.Tensor:
    """Score the full batch [B, L] data-parallel: this rank computes its shard with
    ``metric.scores`` and the results are all-gathered -> [B, k] on every rank."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    B = clean.shape[0]
    lo, hi = shard_bounds(B, world, rank)
    res = metric.scores(clean[lo:hi], noisy[lo:hi], **kw)
    cols = res if isinstance(res, tuple) else (res,)
    local = torch.stack([c.to(torch.float32) for c in cols], dim=1)
    return gather_scores(local, B, group)
