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

``mode="utterance"`` (``time_align_segments``) follows P.862's per-utterance structure instead
(sections 10.3-10.5): the reference's utterances (speech runs of 16 ms or more joined across gaps under 200 ms,
at least 200 ms long, at most 16 per row) own the row's regions (boundaries in the middle of the
gaps); each gets its own crude delay (its envelope +-300 ms, within 300 ms of the row's crude
delay) and fine delay (as above, over its region), and a region splits once where a delay
change within it raises the summed correlation peak by 20 %.  The degraded row is realigned
segment by segment; ``delays`` is then each row's longest segment's delay.

``mode="p862"`` completes P.862's per-utterance stages (sections 10.5-10.6) on the same pieces:
each 320 ms piece of an utterance's region votes for its correlation peak's lag (weight
peak^0.125, pieces under 5 % of the utterance's largest peak do not vote), a range of pieces takes
the first maximum of its triangle-smoothed vote histogram as delay and that maximum's share of
the votes as confidence, and a range splits where both halves are more confident and disagree by
1 ms or more -- recursively, two levels (up to 4 segments per utterance).

GPU rows run ``fsem_time_align_f32`` / ``fsem_time_align_utt_f32`` / ``fsem_time_align_p862_f32``
(``csrc/align.hip``); CPU rows
the float64 FFT form in ``_cpu.py``.  Parity against P.862 implementations is unpinned (none is importable here); the
tests pin both paths to ``oracle/align_oracle.py`` and to known synthetic delays.
"""
from __future__ import annotations

import torch

from . import _cpu, _native
from .base import as_rows, device_lengths, same_device

DEFAULT_MAX_DELAY = 16000  # samples at 16 kHz (1 s)


MODES = ("row", "utterance", "p862")


def _prepare(clean, noisy, max_delay):
    c = as_rows(clean)
    n = as_rows(noisy)
    if c.shape != n.shape:
        raise Exception("`clean_speech` and `denoised_speech` should have the same shape.")
    same_device(c, n)
    if max_delay < 0:
        raise ValueError("max_delay must be >= 0")
    return c, n, min(int(max_delay), 2**31 - 1)  # the C-ABI's int32


def _device_rows(c, n):
    """float32 rows as the C-ABI reads them: 16-byte aligned, one stride, L % 4 == 0."""
    L = c.shape[1]
    c = c.float()
    n = n.float()
    if (c.stride(0) % 4 or n.stride(0) != c.stride(0) or L % 4 or c.data_ptr() % 16 or n.data_ptr() % 16
            or not (c.is_contiguous() and n.is_contiguous())):
        pad = (-L) % 4
        c = torch.nn.functional.pad(c, (0, pad)).contiguous()
        n = torch.nn.functional.pad(n, (0, pad)).contiguous()
    return c, n


def time_align(clean: torch.Tensor, noisy: torch.Tensor, lengths=None,
               max_delay: int = DEFAULT_MAX_DELAY, mode: str = "row") -> tuple[torch.Tensor, torch.Tensor]:
    """(aligned noisy [B, L] float32, delays [B] int32) of 16 kHz rows, on the rows' device.

    ``lengths`` (optional [B] ints): row b holds lengths[b] samples; the aligned row is zero
    past them.  ``max_delay``: the crude search range in samples (rounded up to 4 ms frames).
    ``mode``: "row" (one delay per row), "utterance" or "p862" (per-utterance delays, see
    ``time_align_segments``; ``delays`` = each row's longest segment's delay).
    """
    if mode not in MODES:
        raise ValueError(f"mode must be one of {MODES}")
    if mode in ("utterance", "p862"):
        out, delays, *_ = time_align_segments(clean, noisy, lengths, max_delay, mode=mode)
        return out, delays
    c, n, max_delay = _prepare(clean, noisy, max_delay)
    B, L = c.shape
    if not c.is_cuda:
        lens = None if lengths is None else device_lengths(lengths, B, L, "cpu")
        return _cpu.time_align(c, n, lens, max_delay)
    lib = _native.load()
    lens = device_lengths(lengths, B, L, c.device) if lengths is not None else None
    c, n = _device_rows(c, n)
    out = torch.empty(B, L + (-L) % 4, dtype=torch.float32, device=c.device)[:, :L]  # float4 row stores
    delays = torch.empty(B, dtype=torch.int32, device=c.device)
    ws = _native.workspace(lib.fsem_time_align_workspace_bytes(B, L), c.device)
    _native.check(lib.fsem_time_align_f32(c.data_ptr(), n.data_ptr(), B, L, c.stride(0),
                                          lens.data_ptr() if lens is not None else None, max_delay,
                                          delays.data_ptr(), out.data_ptr(), out.stride(0), ws.data_ptr(),
                                          ws.numel(), _native.stream_handle(c.device)), "time alignment")
    return out, delays


def time_align_segments(clean: torch.Tensor, noisy: torch.Tensor, lengths=None,
                        max_delay: int = DEFAULT_MAX_DELAY, mode: str = "utterance"):
    """Per-utterance alignment (P.862 sections 10.3-10.5, or with ``mode="p862"`` 10.3-10.6, see the
    module docstring) of 16 kHz rows.

    Returns (aligned [B, L] float32, delays [B], n_seg [B], seg_start [B, 33], seg_delay [B, 32])
    on the rows' device (int32 but ``aligned``): segment k of row b covers samples
    [seg_start[b, k], seg_start[b, k + 1]) for k < n_seg[b] and is shifted by seg_delay[b, k];
    ``delays`` is each row's longest segment's delay.
    """
    if mode not in ("utterance", "p862"):
        raise ValueError('mode must be "utterance" or "p862"')
    c, n, max_delay = _prepare(clean, noisy, max_delay)
    B, L = c.shape
    if not c.is_cuda:
        lens = None if lengths is None else device_lengths(lengths, B, L, "cpu")
        return _cpu.time_align_utterances(c, n, lens, max_delay, mode=mode)
    lib = _native.load()
    lens = device_lengths(lengths, B, L, c.device) if lengths is not None else None
    c, n = _device_rows(c, n)
    S = _native.ALIGN_MAX_SEGMENTS
    out = torch.empty(B, L + (-L) % 4, dtype=torch.float32, device=c.device)[:, :L]
    i32 = dict(dtype=torch.int32, device=c.device)
    delays, nseg = torch.empty(B, **i32), torch.empty(B, **i32)
    starts, sdel = torch.zeros(B, S + 1, **i32), torch.zeros(B, S, **i32)
    wsb, entry = ((lib.fsem_time_align_p862_workspace_bytes, lib.fsem_time_align_p862_f32) if mode == "p862"
                  else (lib.fsem_time_align_utt_workspace_bytes, lib.fsem_time_align_utt_f32))
    ws = _native.workspace(wsb(B, L), c.device)
    _native.check(entry(c.data_ptr(), n.data_ptr(), B, L, c.stride(0), lens.data_ptr() if lens is not None else None,
                        max_delay, delays.data_ptr(), nseg.data_ptr(), starts.data_ptr(), sdel.data_ptr(),
                        out.data_ptr(), out.stride(0), ws.data_ptr(), ws.numel(), _native.stream_handle(c.device)),
                  "time alignment")
    return out, delays, nseg, starts, sdel


def realign_bad_intervals(clean: torch.Tensor, noisy: torch.Tensor, aligned: torch.Tensor, frames: torch.Tensor,
                          n_seg: torch.Tensor, seg_start: torch.Tensor, seg_delay: torch.Tensor, lengths=None):
    """P.862's realignment of bad intervals (section 10.7; ``fsem_pesq_bad_intervals_f32``) of
    16 kHz rows on the GPU, after ``time_align_segments(..., mode="p862")`` and the aligned rows'
    per-frame disturbances (``PESQ.frame_disturbances``, [B, 2, F]).

    Returns (n_bad [B], bad [B, 16, 3], second [B, L]) on the rows' device: row b's intervals
    bad[b, i] = (first frame, end frame, delay) for i < n_bad[b] -- runs of frames whose symmetric
    disturbance exceeds 30, joined across gaps under 4 frames, from 5 frames long -- each with the
    delay of the first-difference correlation's first maximum over its samples [256 f0,
    256 f1 + 256) within +-383 of its segment's delay; ``second`` is ``aligned`` with those
    samples taken at the interval's delay instead.
    """
    c, n, _ = _prepare(clean, noisy, 0)
    if not c.is_cuda:
        raise RuntimeError("realign_bad_intervals: GPU rows only (the CPU path is _cpu.pesq_p862)")
    B, L = c.shape
    lib = _native.load()
    F = lib.fsem_pesq_frames(L)
    S = _native.ALIGN_MAX_SEGMENTS
    # the kernels index these by row, frame and segment: shapes checked before any launch, every
    # operand moved to the rows' device
    want = {"aligned": (aligned, (B, L)), "frames": (frames, (B, 2, F)), "n_seg": (n_seg, (B,)),
            "seg_start": (seg_start, (B, S + 1)), "seg_delay": (seg_delay, (B, S))}
    for name, (t, shape) in want.items():
        if tuple(t.shape) != shape:
            raise ValueError(f"{name} must have shape {list(shape)}, got {list(t.shape)}")
    lens = device_lengths(lengths, B, L, c.device) if lengths is not None else None
    c, n = _device_rows(c, n)
    frames = frames.to(device=c.device, dtype=torch.float32).contiguous()
    a = aligned.to(device=c.device, dtype=torch.float32)
    if a.stride(1) != 1 or a.stride(0) % 4 or a.stride(0) < L or a.data_ptr() % 16:
        a = torch.nn.functional.pad(a.contiguous(), (0, (-L) % 4))[:, :L]
    second = torch.empty(B, a.stride(0), dtype=torch.float32, device=c.device)[:, :L]
    i32 = dict(dtype=torch.int32, device=c.device)
    n_bad = torch.empty(B, **i32)
    bad = torch.zeros(B, _native.PESQ_MAX_BAD, 3, **i32)
    segs = [t.to(**i32).contiguous() for t in (n_seg, seg_start, seg_delay)]
    if B and (int(segs[0].min()) < 0 or int(segs[0].max()) > S):
        raise ValueError(f"n_seg must lie in [0, {S}]")
    ws = _native.workspace(lib.fsem_pesq_bad_intervals_workspace_bytes(B, L), c.device)
    _native.check(lib.fsem_pesq_bad_intervals_f32(c.data_ptr(), n.data_ptr(), a.data_ptr(), B, L, c.stride(0),
                                                  lens.data_ptr() if lens is not None else None, frames.data_ptr(),
                                                  segs[0].data_ptr(), segs[1].data_ptr(), segs[2].data_ptr(),
                                                  n_bad.data_ptr(), bad.data_ptr(), second.data_ptr(), a.stride(0),
                                                  ws.data_ptr(), ws.numel(), _native.stream_handle(c.device)),
                  "bad-interval realignment")
    return n_bad, bad, second
