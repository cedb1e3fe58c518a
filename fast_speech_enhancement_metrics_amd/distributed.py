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


def score_columns(metric) -> int:
    """Columns of ``metric.scores``: 3 (PESQ_STOI: mos, stoi, estoi), 2 (STOI: stoi, estoi), 1 (PESQ)."""
    from .joint import PESQ_STOI
    from .STOI import STOI
    return 3 if isinstance(metric, PESQ_STOI) else (2 if isinstance(metric, STOI) else 1)


def collective_device(group, fallback) -> torch.device:
    """Where the all-gather's tensors must live: the current HIP device for RCCL ("nccl"),
    else the caller's device (gloo: CPU)."""
    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device(fallback) if fallback is not None else torch.device("cpu")


def _local_scores(metric, clean, noisy, lengths, device) -> torch.Tensor:
    """[n, k] float32 scores of this rank's rows (rows at metric.sample_rate), n may be 0."""
    k = score_columns(metric)
    if noisy is None or noisy.shape[0] == 0:
        return torch.zeros(0, k, dtype=torch.float32, device=device)
    res = metric.scores(clean, noisy, lengths=lengths, sample_rate=metric.sample_rate)
    cols = res if isinstance(res, tuple) else (res,)
    return torch.stack([c.to(torch.float32) for c in cols], dim=1).to(device)


def sharded_scores(metric, clean: torch.Tensor, noisy: torch.Tensor, group=None, lengths=None) -> torch.Tensor:
    """Score the full batch [B, L] data-parallel: this rank computes its shard with
    ``metric.scores`` and the results are all-gathered -> [B, k] on every rank.

    Rows are at the metric's configured rate (``metric.sample_rate``; PESQ resamples them to
    16 kHz, STOI to 10 kHz, as the reference's BaseMetric does); ``lengths`` optionally gives
    per-row lengths.  A rank whose shard is empty (B < world size) contributes no rows."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    B = clean.shape[0]
    lo, hi = shard_bounds(B, world, rank)
    lens = None if lengths is None else torch.as_tensor(lengths).reshape(-1)[lo:hi]
    dev = collective_device(group, noisy.device)
    local = _local_scores(metric, clean[lo:hi], noisy[lo:hi], lens, dev)
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
    """Score a ragged batch (lists of 1-D utterances at ``metric.sample_rate``) data-parallel with
    LPT balancing by total length: this rank scores its utterances as one padded batch with
    per-row lengths (``metric.scores(..., lengths=...)``), then the [n_r, k] score rows are
    all-gathered and put back in the caller's order -> [B, k] on every rank.  ``device``: where
    this rank computes (default: where the utterances are)."""
    from .batching import pad_batch
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    lengths = [int(x.numel()) for x in noisy]
    plan = lpt_shards(lengths, world)
    mine = plan[rank]
    coll = collective_device(group, device if device is not None else (noisy[0].device if noisy else None))
    if mine:
        c, n, lens = pad_batch([clean[i] for i in mine], [noisy[i] for i in mine])
        if device is not None:
            c, n = c.to(device), n.to(device)
        local = _local_scores(metric, c, n, lens, coll)
    else:  # empty shard: no rows, but the collective still runs on the right device
        local = _local_scores(metric, None, None, None, coll)
    cap = max(len(s) for s in plan)
    k = local.shape[1]
    buf = torch.full((cap, k), float("nan"), dtype=torch.float32, device=coll)
    buf[:local.shape[0]] = local
    out = torch.empty(world * cap, k, dtype=torch.float32, device=coll)
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, buf, group=group)
    else:
        dist.all_gather(list(out.chunk(world)), buf, group=group)
    full = torch.empty(len(lengths), k, dtype=torch.float32, device=coll)
    for r, idx in enumerate(plan):
        if idx:
            full[torch.tensor(idx, device=coll)] = out[r * cap:r * cap + len(idx)]
    return full


def scatter_batch(clean, noisy, src: int = 0, group=None, lengths=None, device=None):
    """Inputs on one device: rank ``src`` holds the whole [B, L] batch (other ranks
    pass None); every rank receives its contiguous shard (``shard_bounds``) by point-to-point
    sends from ``src`` -- over xGMI with RCCL, one link per destination GPU, all in flight at
    once -- into ``device`` (default: the collective's device).  Returns (clean_shard,
    noisy_shard, lengths_shard or None, B).  The copy is the only data movement: ``src`` sends
    views of its rows, no padded staging copy."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    gsrc = dist.get_global_rank(group, src) if group is not None else src
    dev = collective_device(group, device if device is not None else (noisy.device if noisy is not None else None))
    # shape, dtype code and whether lengths come along: one small broadcast.  A bad call is
    # reported through the broadcast (code -1) so that every rank raises -- raising on `src`
    # alone would leave the other ranks blocked in the broadcast.
    dtypes = [torch.float32, torch.float16, torch.bfloat16, torch.float64]
    meta = torch.zeros(4, dtype=torch.int64, device=dev)
    if rank == src:
        ok = (clean is not None and noisy is not None and clean.shape == noisy.shape and clean.dim() == 2)
        if ok and (clean.dtype != noisy.dtype or noisy.dtype not in dtypes):
            # one wire dtype for both signals: mixed or other dtypes (int16 codes, ...) go as the
            # float32 the metrics compute in
            clean, noisy = clean.to(torch.float32), noisy.to(torch.float32)
        if ok:
            meta[0], meta[1] = clean.shape[0], clean.shape[1]
            meta[2] = dtypes.index(noisy.dtype)
            meta[3] = 0 if lengths is None else 1
        else:
            meta[2] = -1
    dist.broadcast(meta, gsrc, group=group)
    B, L, code, has_len = (int(v) for v in meta.tolist())
    if code < 0:
        raise ValueError("scatter_batch: clean / noisy on the source rank must be [B, L] of one shape")
    dtype = dtypes[code]
    lens_all = torch.empty(B, dtype=torch.int64, device=dev)
    if has_len:
        if rank == src:
            lens_all.copy_(torch.as_tensor(lengths).reshape(-1).to(torch.int64))
        dist.broadcast(lens_all, gsrc, group=group)
    lo, hi = shard_bounds(B, world, rank)
    ops = []
    if rank == src:
        c_src, n_src = clean.to(dev), noisy.to(dev)
        for r in range(world):
            if r == src:
                continue
            a, b = shard_bounds(B, world, r)
            if b > a:
                peer = dist.get_global_rank(group, r) if group is not None else r
                ops.append(dist.P2POp(dist.isend, c_src[a:b].contiguous(), peer, group=group))
                ops.append(dist.P2POp(dist.isend, n_src[a:b].contiguous(), peer, group=group))
        c_loc, n_loc = c_src[lo:hi], n_src[lo:hi]
    else:
        c_loc = torch.empty(hi - lo, L, dtype=dtype, device=dev)
        n_loc = torch.empty(hi - lo, L, dtype=dtype, device=dev)
        if hi > lo:
            ops.append(dist.P2POp(dist.irecv, c_loc, gsrc, group=group))
            ops.append(dist.P2POp(dist.irecv, n_loc, gsrc, group=group))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    lens_loc = lens_all[lo:hi] if has_len else None
    return c_loc, n_loc, lens_loc, B


def sharded_scores_from(metric, clean, noisy, src: int = 0, group=None, lengths=None, device=None) -> torch.Tensor:
    """``sharded_scores`` for a batch that lives on rank ``src`` only: scatter the shards
    (``scatter_batch``), score them, all-gather the scores -> [B, k] on every rank."""
    c, n, lens, B = scatter_batch(clean, noisy, src=src, group=group, lengths=lengths, device=device)
    local = _local_scores(metric, c, n, lens, collective_device(group, c.device))
    return gather_scores(local, B, group)
