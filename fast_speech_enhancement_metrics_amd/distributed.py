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


def lpt_shards(lengths, world: int) -> list[list[int]]:
    """Longest-processing-time assignment of ragged utterances to ranks:
    utterances in decreasing length, each to the rank with the least total samples so far
    (ties -> lowest rank).  Deterministic, so every rank computes the same plan locally."""
    import heapq
    order = sorted(range(len(lengths)), key=lambda i: (-int(lengths[i]), i))
    heap = [(0, r) for r in range(world)]
    shards: list[list[int]] = [[] for _ in range(world)]
    for i in order:
        load, r = heapq.heappop(heap)
        shards[r].append(i)
        heapq.heappush(heap, (load + int(lengths[i]), r))
    return [sorted(s) for s in shards]


def sharded_scores_ragged(metric, clean, noisy, group=None, device=None) -> torch.Tensor:
    """Score a ragged batch (lists of 1-D utterances) data-parallel with LPT balancing by total
    length: this rank scores its utterances as one padded batch with per-row lengths
    (``metric.scores(..., lengths=...)``), then the [n_r, k] score rows are all-gathered and put
    back in the caller's order -> [B, k] on every rank."""
    from .batching import pad_batch
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    lengths = [int(x.numel()) for x in noisy]
    plan = lpt_shards(lengths, world)
    mine = plan[rank]
    c, n, lens = pad_batch([clean[i] for i in mine], [noisy[i] for i in mine]) if mine else (None, None, None)
    if device is not None and c is not None:
        c, n = c.to(device), n.to(device)
    if mine:
        # STOI.scores takes the input rate (its resampler is fused); PESQ / PESQ_STOI take 16 kHz rows
        kw = {"sample_rate": metric.sample_rate} if hasattr(metric, "N") else {}
        res = metric.scores(c, n, lengths=lens, **kw)
        cols = res if isinstance(res, tuple) else (res,)
        local = torch.stack([x.to(torch.float32) for x in cols], dim=1)
    else:
        k = 3 if metric.__class__.__name__ == "PESQ_STOI" else (2 if hasattr(metric, "N") else 1)
        local = torch.zeros(0, k, dtype=torch.float32, device=device or "cpu")
    cap = max(len(s) for s in plan)
    k = local.shape[1]
    buf = torch.full((cap, k), float("nan"), dtype=torch.float32, device=local.device)
    buf[:local.shape[0]] = local
    out = torch.empty(world * cap, k, dtype=torch.float32, device=local.device)
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, buf, group=group)
    else:
        dist.all_gather(list(out.chunk(world)), buf, group=group)
    full = torch.empty(len(lengths), k, dtype=torch.float32, device=local.device)
    for r, idx in enumerate(plan):
        if idx:
            full[torch.tensor(idx, device=local.device)] = out[r * cap:r * cap + len(idx)]
    return full
