"""Opt-in time alignment of (clean, degraded) pairs before PESQ.

The reference's PESQ has no time alignment (``fast_se_metrics/PESQ.py:19-22``: "1. no time
alignment"), so the drop-in classes leave it off; ``PESQ(..., time_align=True)`` (or this
module directly) estimates each row's delay after ITU-T P.862 section 10 and scores the
degraded row shifted back by it:

* crude delay: 4 ms voice-activity log envelopes (P.862 ``apply_VAD``), the lag of their
  largest plain cross-correlation within +-``max_delay`` samples (P.862 ``crude_align``);
* fine delay: within +-383 samples of it, the lag of the largest cross-correlation of the two
  signals' first differences over the whole row (P.862 refines per utterance with a histogram
  of per-frame correlation peaks; this build does not split rows into utterances);
* ``delay > 0``: the degraded row lags, ``deg[n] ~ ref[n - delay]``; the aligned row is
  ``deg[n + delay]`` inside the row, zero elsewhere.

GPU rows run ``fsem_time_align_f32`` (``csrc/align.hip``); CPU rows the float64 FFT form in
``_cpu.py``.  Parity against P.862 implementations is unpinned (none is importable here); the
tests pin both paths to ``oracle/align_oracle.py`` and to known synthetic delays.
"""
from __future__ import annotations

import torch

from . import _cpu, _native
from .base import as_rows, device_lengths

DEFAULT_MAX_DELAY = 16000  # samples at 16 kHz (1 s)


def time_align(clean: torch.Tensor, noisy: torch.Tensor, lengths=None,
               max_delay: int = DEFAULT_MAX_DELAY) -> tuple[torch.Tensor, torch.Tensor]:
    """(aligned noisy [B, L] float32, delays [B] int32) of 16 kHz rows, on the rows' device.

    ``lengths`` (optional [B] ints): row b holds lengths[b] samples; the aligned row is zero
    past them.  ``max_delay``: the crude search range in samples (rounded up to 4 ms frames).
    """
    c = as_rows(clean)
    n = as_rows(noisy)
    if c.shape != n.shape:
        raise Exception("`clean_speech` and `denoised_speech` should have the same shape.")
    if max_delay < 0:
        raise ValueError("max_delay must be >= 0")
    max_delay = min(int(max_delay), 2**31 - 1)  # the C-ABI's int32
    B, L = c.shape
    if not c.is_cuda:
        lens = None if lengths is None else device_lengths(lengths, B, L, "cpu")
        return _cpu.time_align(c, n, lens, int(max_delay))
    lib = _native.load()
    lens = device_lengths(lengths, B, L, c.device) if lengths is not None else None
    c = c.float()
    n = n.float()
    if (c.stride(0) % 4 or n.stride(0) != c.stride(0) or L % 4 or c.data_ptr() % 16 or n.data_ptr() % 16
            or not (c.is_contiguous() and n.is_contiguous())):
        pad = (-L) % 4  # 16-byte aligned rows read in 16-byte pieces, one stride (include/fsem.h)
        c = torch.nn.functional.pad(c, (0, pad)).contiguous()
        n = torch.nn.functional.pad(n, (0, pad)).contiguous()
    out = torch.empty(B, L + (-L) % 4, dtype=torch.float32, device=c.device)[:, :L]  # float4 row stores
    delays = torch.empty(B, dtype=torch.int32, device=c.device)
    ws = _native.workspace(lib.fsem_time_align_workspace_bytes(B, L), c.device)
    _native.check(lib.fsem_time_align_f32(c.data_ptr(), n.data_ptr(), B, L, c.stride(0),
                                          lens.data_ptr() if lens is not None else None, int(max_delay),
                                          delays.data_ptr(), out.data_ptr(), out.stride(0), ws.data_ptr(),
                                          ws.numel(), _native.stream_handle(c.device)), "time alignment")
    return out, delays
