"""PESQ-wb + STOI/ESTOI from one pass over the inputs.

The reference computes the two metrics with two calls, each reading both signals:
``PESQ(16000)(clean, noisy)`` (PESQ.py:232-245) and ``STOI(16000)(clean, noisy)``
(base.py:19-20 resampling to 10 kHz, STOI.py:153-205).  ``PESQ_STOI`` returns the same
numbers -- on the GPU bitwise those of the two separate engine calls -- while the engine reads
each input once: the PESQ front end's LDS tiles also feed the fused 16 -> 10 kHz resampler
(``fsem_pesq_stoi_f32``).  At other input rates the two metrics keep the reference's own
resampling paths (PESQ: sr -> 16 kHz, STOI: sr -> 10 kHz directly, base.py:19-20) and are
computed by the PESQ and STOI engines separately.
"""
from __future__ import annotations

import warnings

import torch

from . import _native
from .PESQ import PESQ
from .STOI import STOI
from .base import BaseMetric, as_rows, check_row_rate, device_lengths, noisy_shape, same_device


_KEYS = ("PESQ", "STOI", "ESTOI")


class PESQ_STOI(BaseMetric):
    higher_is_better = True
    EXPECTED_SAMPLING_RATE = 16000

    def __init__(self, sample_rate: int = 16000, use_gpu: bool = False, *, devices=None):
        super().__init__(sample_rate, use_gpu, devices=devices)
        self._pesq = PESQ(sample_rate, use_gpu, devices=devices)
        self._stoi = STOI(sample_rate, use_gpu, devices=devices)
        self._ws_bytes: dict = {}

    def __call__(self, clean_speech, denoised_speech, lengths=None) -> list[dict[str, float]]:
        if lengths is None and self._fast_ok(clean_speech, denoised_speech):
            return self._fast_call(clean_speech, denoised_speech)
        if self.sample_rate == self.EXPECTED_SAMPLING_RATE:
            return super().__call__(clean_speech, denoised_speech, lengths)
        # STOI must resample sr -> 10 kHz itself (not via 16 kHz) to match the reference
        p = self._pesq(clean_speech, denoised_speech, lengths)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", RuntimeWarning)
            try:
                s = self._stoi(clean_speech, denoised_speech, lengths)
            except TypeError:  # no utterance has a STOI segment (STOI.py:162-165)
                s = [{"STOI": float("nan"), "ESTOI": float("nan")}] * len(p)
        return [{**a, **b} for a, b in zip(p, s)]

    def scores(self, clean_speech: torch.Tensor, denoised_speech: torch.Tensor, lengths=None,
               sample_rate: int | None = None):
        """(mos[B], stoi[B], estoi[B]) on the metric's device (no host sync on GPU).

        Rows at ``sample_rate`` (None: 16 kHz, which requires a 16 kHz metric).  16 kHz rows take the
        fused single-read engine; other rates keep the reference's own resampling paths (PESQ:
        sr -> 16 kHz, STOI: sr -> 10 kHz directly) through the two engines.
        """
        sr = check_row_rate(self, sample_rate)
        if sr != self.EXPECTED_SAMPLING_RATE:
            mos = self._pesq.scores(clean_speech, denoised_speech, lengths, sample_rate=sr)
            s, e = self._stoi.scores(clean_speech, denoised_speech, sr, lengths=lengths)
            return mos, s, e
        if self.fans_out():
            if noisy_shape(clean_speech) != noisy_shape(denoised_speech):
                raise Exception("`clean_speech` and `denoised_speech` should have the same shape.")
            return self.fan_out(self._rows_scores, clean_speech, denoised_speech, lengths, 3, balance=lengths)
        return self._rows_scores(clean_speech, denoised_speech, lengths)

    def _rows_scores(self, clean_speech, denoised_speech, lengths):
        """(mos, stoi, estoi) [B] of 16 kHz rows on their own device (one fused engine call)."""
        clean = as_rows(clean_speech)
        noisy = as_rows(denoised_speech)
        if noisy.shape != clean.shape:
            raise Exception("`clean_speech` and `denoised_speech` should have the same shape.")
        same_device(clean, noisy)
        B, L = clean.shape
        if not clean.is_cuda:
            mos = self._pesq.scores(clean, noisy, lengths, sample_rate=16000)
            s, e = self._stoi.scores(clean, noisy, 16000, lengths=lengths)
            return mos, s, e
        lib = _native.load()
        lens = device_lengths(lengths, B, L, clean.device) if lengths is not None else None
        if clean.stride(0) != noisy.stride(0) or L % 4:
            pad = (-L) % 4  # rows readable up to ceil4(L) floats (include/fsem.h)
            clean = torch.nn.functional.pad(clean, (0, pad)).contiguous()
            noisy = torch.nn.functional.pad(noisy, (0, pad)).contiguous()
        out = torch.empty(3, B, dtype=torch.float32, device=clean.device)
        ws = _native.workspace(lib.fsem_pesq_stoi_workspace_bytes(B, L), clean.device)
        rc = lib.fsem_pesq_stoi_f32(clean.data_ptr(), noisy.data_ptr(), B, L, clean.stride(0),
                                    lens.data_ptr() if lens is not None else None, out[0].data_ptr(),
                                    out[1].data_ptr(), out[2].data_ptr(), ws.data_ptr(), ws.numel(),
                                    _native.stream_handle(clean.device))
        if rc == _native.FSEM_ESHORT:
            # the reference's PESQ raises first for short inputs (its unfold, PESQ.py:169)
            raise RuntimeError("input too short for PESQ (20 frames) or STOI (one 10 kHz frame)")
        _native.check(rc, "PESQ_STOI")
        return out[0], out[1], out[2]

    def compute_metric(self, clean_speech: torch.Tensor | None, denoised_speech: torch.Tensor,
                       lengths=None) -> list[dict[str, float]]:
        assert clean_speech is not None
        return self._listed(clean_speech, denoised_speech, lengths)[0]

    # ---- the drop-in call's fast path (the common case: one 16 kHz float32 [B, L] pair of device
    # tensors on the current device, no lengths, one device).  The GPU idles between two calls
    # while the host finishes one and starts the next: the scores' copy, the list's fill, the
    # caller dropping the previous list (4096 dicts + 12288 floats: ~0.1-0.2 ms of deallocation),
    # and the next call's Python path up to its first launch.  Here the launch comes first, the
    # dicts are built and the PREVIOUS call's list is released while the GPU computes, and the
    # returned list is also held by the metric (through the fill handle) until its next call --
    # so the caller's drop of the list is cheap and the expensive deallocation overlaps the next
    # call's kernels.
    # Same scores, same dicts, same warnings and exceptions as the generic path.

    def _fast_ok(self, clean, noisy) -> bool:
        if self.device != "cuda" or self._fanout is not None or self.sample_rate != 16000:
            return False
        if not (isinstance(clean, torch.Tensor) and isinstance(noisy, torch.Tensor)):
            return False
        if clean.dim() != 2 or clean.shape != noisy.shape or clean.dtype != torch.float32 \
                or noisy.dtype != torch.float32 or not (clean.is_cuda and noisy.is_cuda):
            return False
        B, L = noisy.shape
        if B < 1 or L % 4 or clean.stride(1) != 1 or noisy.stride(1) != 1 or clean.stride(0) != noisy.stride(0) \
                or noisy.stride(0) < L or clean.requires_grad or noisy.requires_grad:
            return False
        dev = noisy.device.index
        return clean.device.index == dev and dev == torch.cuda.current_device()

    def _fast_call(self, clean: torch.Tensor, noisy: torch.Tensor, device_scores: bool = False):
        """The list of dicts; with ``device_scores`` also the [B, 3] float32 scores on the device
        (for ``call_with_scores``: the scores then land in a device buffer and reach the host by
        one copy)."""
        lib = _native.load()
        B, L = noisy.shape
        dev = noisy.device
        stream = torch.cuda.current_stream(dev)
        wsb = self._ws_bytes.get((B, L))
        if wsb is None:
            wsb = self._ws_bytes[(B, L)] = lib.fsem_pesq_stoi_workspace_bytes(B, L)
        # the scores go straight into the thread's pinned host buffer when the device maps it
        # (no device->host copy behind the kernels: ~20 us of the step's idle tail)
        slot = _native.mapped_host_slot(self, 3 * B, dev) if self.host_scores and not device_scores else None
        if slot is not None:
            o = slot[0].data_ptr()
            outs = (o, o + 4 * B, o + 8 * B)
        else:
            out = torch.empty(3, B, dtype=torch.float32, device=dev)
            outs = (out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr())
        ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
        rc = lib.fsem_pesq_stoi_f32(clean.data_ptr(), noisy.data_ptr(), B, L, clean.stride(0), None, *outs,
                                    ws.data_ptr(), wsb, stream.cuda_stream)
        if rc == _native.FSEM_ESHORT:
            raise RuntimeError("input too short for PESQ (20 frames) or STOI (one 10 kHz frame)")
        _native.check(rc, "PESQ_STOI")
        if slot is not None:
            res, _ = _native.list_from_host(self, slot, 3, B, _KEYS, dev)
        else:
            res, _ = _native.list_from_device(self, out, _KEYS)
        if res[0]["STOI"] != res[0]["STOI"] and all(d["STOI"] != d["STOI"] for d in res):  # STOI.py:162-165
            warnings.warn("Not enough non-silent frames. Please check your sound files", RuntimeWarning, stacklevel=3)
        return (res, out.t()) if device_scores else res

    # Rows per chunk when the drop-in call splits a GPU batch into consecutive engine calls
    # (below); 0: one call.  The chunks existed to overlap building chunk k's dicts with chunk
    # k+1's kernels (round 3, profiles/r3_c/dropin.json: 2 x 2048 rows 8.29 ms per call against
    # 8.39 ms for one).  Since the dicts are built before the scores exist and only filled
    # afterwards (score_list_alloc / score_list_fill), one call is the faster plan at 4096 x 10 s:
    # 7.363 ms against 7.428 ms for 2 x 2048 (tools/ab_dropin_chunks.py,
    # profiles/r4_zz/ab_dropin_fill.txt) -- one kernel tail instead of two.
    pipeline_rows = 0
    # the fast path's scores written by the kernels into mapped pinned host memory (False: a
    # device buffer and one copy, as the generic path)
    host_scores = True

    def _listed(self, clean_speech, denoised_speech, lengths):
        """(list of dicts, [B, 3] float32 scores on the metric's device) of 16 kHz rows.

        On the GPU a large batch is scored in consecutive chunks, all enqueued at once, each
        followed by an asynchronous copy of its scores into pinned host memory.  The result's dicts
        are built while the GPU computes (score_list_alloc, ~100 ns per utterance) and each chunk's
        scores are written into them when its copy lands (score_list_fill, ~10 ns per
        utterance), so little host work trails the GPU.  Scores are those of
        one call over the whole batch (rows are independent; the PESQ back end's summation order
        depends only on the batch's size class, pesq.hip back_waves)."""
        with torch.inference_mode():
            rows = torch.atleast_2d(denoised_speech)
            B = rows.shape[0]
            bounds = self.chunk_bounds(B, rows.is_cuda)
            K = len(bounds)
            if K <= 1:
                out = torch.stack([t.float() for t in self.scores(clean_speech, denoised_speech, lengths,
                                                                  sample_rate=16000)])
                if out.is_cuda:  # the dicts are built while the GPU computes, then filled
                    res, _ = _native.list_from_device(self, out, _KEYS)
                else:
                    res = _native.score_list(out, _KEYS)
            else:
                clean = torch.atleast_2d(clean_speech)
                lens = None if lengths is None else device_lengths(lengths, B, rows.shape[-1], rows.device)
                pinned = self._pinned(3 * B)
                stream = torch.cuda.current_stream(rows.device)
                parts, done = [], []
                for lo, hi in bounds:
                    part = torch.stack([t.float() for t in self.scores(
                        clean[lo:hi], rows[lo:hi], None if lens is None else lens[lo:hi], sample_rate=16000)])
                    # a contiguous pinned slice per chunk: the copy stays asynchronous
                    pinned[3 * lo:3 * hi].view(3, hi - lo).copy_(part, non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(stream)
                    parts.append(part)
                    done.append(ev)
                out = torch.cat(parts, dim=1)
                res, h = _native.score_list_alloc(B, _KEYS)  # while the GPU computes
                for (lo, hi), ev in zip(bounds, done):
                    ev.synchronize()
                    _native.score_list_fill(h, lo, pinned[3 * lo:3 * hi].view(3, hi - lo).numpy(), _KEYS)
        if all(d["STOI"] != d["STOI"] for d in res):  # as STOI (STOI.py:162-165)
            warnings.warn("Not enough non-silent frames. Please check your sound files", RuntimeWarning, stacklevel=4)
        return res, out.t()

    def chunk_bounds(self, batch: int, on_gpu: bool = True) -> list[tuple[int, int]]:
        """Row ranges of the engine calls the drop-in call makes for `batch` rows: one range, or
        batch // pipeline_rows consecutive ones on the GPU (bench.py times the dominant kernel and
        the scores path at this per-call size, so every launch in the bench has one size)."""
        # a multi-device call scores its shards concurrently already: one range
        K = batch // self.pipeline_rows if (on_gpu and self.pipeline_rows > 0 and self._fanout is None) else 1
        K = max(K, 1)
        return [(k * batch // K, (k + 1) * batch // K) for k in range(K)]

    def _pinned(self, n: int) -> torch.Tensor:
        """A pinned host float32 buffer of at least n elements, kept across calls.  A call waits for
        its copies before returning, so the next call may reuse it."""
        buf = getattr(self, "_pinned_buf", None)
        if buf is None or buf.numel() < n:
            buf = torch.empty(n, dtype=torch.float32, pin_memory=True)
            self._pinned_buf = buf
        return buf[:n]

    def call_with_scores(self, clean_speech, denoised_speech, lengths=None):
        """The drop-in call's list of dicts together with the same scores as a [B, 3] float32 tensor
        (PESQ, STOI, ESTOI) on the metric's device -- for callers that also hand the scores on
        (e.g. an all-gather across ranks) without rebuilding them from the dicts."""
        if self.sample_rate != self.EXPECTED_SAMPLING_RATE:
            res = self(clean_speech, denoised_speech, lengths)
            t = torch.tensor([[d["PESQ"], d["STOI"], d["ESTOI"]] for d in res], dtype=torch.float32)
            return res, t.to(self.device)
        if lengths is None and self._fast_ok(clean_speech, denoised_speech):
            return self._fast_call(clean_speech, denoised_speech, device_scores=True)
        clean_speech, denoised_speech, lengths = self.split_ragged(clean_speech, denoised_speech, lengths)
        clean_speech, denoised_speech = self.prepare_inputs(clean_speech, denoised_speech, lengths)
        assert clean_speech is not None
        return self._listed(clean_speech, denoised_speech, lengths)
