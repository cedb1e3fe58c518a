"""Variable-length batches.

The reference requires equal shapes (``fast_se_metrics/base.py:26-27``) and has no notion of
per-utterance length.  Here a batch may be ragged: a list of 1-D utterances, or a padded
[B, L] tensor plus ``lengths``.  Each utterance's result is DEFINED as the reference's result
for that unpadded utterance called alone, so it is pinned by the same oracle; utterances the
reference rejects when called alone (too short) score NaN instead of failing the batch.
"""
from __future__ import annotations

import math
from typing import Sequence

import torch


def pad_batch(clean: Sequence[torch.Tensor] | None, noisy: Sequence[torch.Tensor]):
    """Lists of 1-D utterances -> (clean [B, Lcap] | None, noisy [B, Lcap], lengths int32 [B]).

    Rows are zero-padded to a common capacity rounded up to a multiple of 4 (the engine reads
    rows in 16-byte pieces, include/fsem.h).  Pairs must have equal lengths (base.py:26-27).
    """
    noisy = [torch.as_tensor(x).reshape(-1) for x in noisy]
    if clean is not None:
        clean = [torch.as_tensor(x).reshape(-1) for x in clean]
        if len(clean) != len(noisy) or any(c.shape != n.shape for c, n in zip(clean, noisy)):
            raise Exception("`clean_speech` and `denoised_speech` should have the same shape.")
    if not noisy:
        raise ValueError("empty batch")
    lengths = torch.tensor([x.numel() for x in noisy], dtype=torch.int32)
    cap = max(4, int(math.ceil(int(lengths.max()) / 4)) * 4)

    def stack(xs):
        out = torch.zeros(len(xs), cap, dtype=torch.float32, device=xs[0].device)
        for i, x in enumerate(xs):
            out[i, :x.numel()] = x.to(torch.float32)
        return out

    return (stack(clean) if clean is not None else None), stack(noisy), lengths


def as_lengths(lengths, batch: int, capacity: int) -> torch.Tensor:
    """Validate per-row lengths -> int32 CPU tensor [batch] with 0 <= length <= capacity."""
    t = torch.as_tensor(lengths).reshape(-1).to("cpu", torch.int64)
    if t.numel() != batch:
        raise ValueError(f"lengths has {t.numel()} entries for a batch of {batch}")
    if bool((t < 0).any()) or bool((t > capacity).any()):
        raise ValueError(f"lengths must lie in [0, {capacity}]")
    return t.to(torch.int32)


def resampled_lengths(lengths: torch.Tensor, orig_freq: int, new_freq: int) -> torch.Tensor:
    """Per-row length after torchaudio Resample(orig, new): ceil(n * new / orig) (reduced rates)."""
    g = math.gcd(int(orig_freq), int(new_freq))
    o, n = int(orig_freq) // g, int(new_freq) // g
    return ((lengths.to(torch.int64) * n + o - 1) // o).to(torch.int32)
