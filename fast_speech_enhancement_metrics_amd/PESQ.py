"""PESQ-wb metric -- drop-in for the reference's ``fast_se_metrics.PESQ`` (PESQ.py:13-245).

P.862-like wideband model without time alignment and with IIR level alignment
(reference PESQ.py:17-23).  ``use_gpu=True``: the whole per-utterance pipeline runs in
libfsem's gfx950 kernels (``fsem_pesq_wb_f32``) with one device->host copy of the scores;
``use_gpu=False``: the package's CPU implementation.
"""
from __future__ import annotations

import torch

from . import _cpu, _native
from .base import BaseMetric, as_rows, check_row_rate, device_lengths, noisy_shape, resample_rows


class PESQ(BaseMetric):
    higher_is_better = True
    EXPECTED_SAMPLING_RATE = 16000

    def __init__(self, sample_rate: int = 16000, use_gpu: bool = False):
        super().__init__(sample_rate, use_gpu)

    @staticmethod
    def equalize_ranges(clean_speech: torch.Tensor, noisy_speech: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
        """Both rows divided by their joint peak |x| (PESQ.py:115-121).  The engine skips this step:
        it cancels under the level alignment (amplitude range)."""
        m = torch.maximum(clean_speech.abs().amax(dim=1, keepdim=True), noisy_speech.abs().amax(dim=1, keepdim=True))
        return clean_speech / m, noisy_speech / m

    # ------------------------------------------------------------------ reference attributes
    # The reference's filter coefficients (PESQ.py:79-90), float32 on the metric's device, built
    # on first access (the engine carries its own copies in constant memory).
    @property
    def power_filter(self) -> torch.Tensor:
        """[2, 11] (b; a) of the order-5 Butterworth band-pass 325-3250 Hz at 16 kHz (PESQ.py:80-81)."""
        if getattr(self, "_power_filter", None) is None:
            import numpy as np
            from scipy.signal import butter
            out = np.asarray(butter(5, [325, 3250], fs=16000, btype="band"))
            self._power_filter = torch.as_tensor(out, device=self.device, dtype=torch.float32)
        return self._power_filter

    @property
    def pre_filter(self) -> torch.Tensor:
        """[2, 3] (b; a) of the pre-emphasis IIR (PESQ.py:84-88)."""
        if getattr(self, "_pre_filter", None) is None:
            self._pre_filter = torch.tensor([[2.740826, -5.4816519, 2.740826], [1.0, -1.9444777, 0.94597794]],
                                            device=self.device, dtype=torch.float32)
        return self._pre_filter

    @property
    def taper_weights(self) -> torch.Tensor:
        """[15] edge taper (k + 1) / 16 of the first / last 15 samples (PESQ.py:90)."""
        if getattr(self, "_taper_weights", None) is None:
            self._taper_weights = torch.linspace(0, 15, 16, device=self.device)[1:] / 16.0
        return self._taper_weights

    # ------------------------------------------------------------------ device paths
    def scores(self, clean_speech: torch.Tensor, denoised_speech: torch.Tensor, lengths=None,
               sample_rate: int | None = None) -> torch.Tensor:
        """Per-utterance MOS as a tensor on the metric's device (no host sync on GPU).

        Rows at ``sample_rate``; None means rows already at 16 kHz, which requires a 16 kHz metric
        (a ``PESQ(8000)`` must be told its rows' rate, or it would score them as 16 kHz).  Other
        rates are resampled to 16 kHz first, each row as the row alone (BaseMetric.prepare_audio,
        base.py:19-20).  ``lengths`` (optional, [B] ints at that rate): row b holds lengths[b]
        samples and scores as the reference would on that unpadded row alone; rows under 20
        frames give NaN.
        """
        sr = check_row_rate(self, sample_rate)
        if noisy_shape(clean_speech) != noisy_shape(denoised_speech):
            raise Exception("`clean_speech` and `denoised_speech` should have the same shape.")
        if sr != self.EXPECTED_SAMPLING_RATE:
            clean_speech, denoised_speech, lengths = resample_rows(clean_speech, denoised_speech, lengths, sr,
                                                                   self.EXPECTED_SAMPLING_RATE)
        clean = as_rows(clean_speech)
        noisy = as_rows(denoised_speech)
        B, L = clean.shape
        if noisy.shape != clean.shape:
            raise Exception("`clean_speech` and `denoised_speech` should have the same shape.")
        lib = _native.load() if clean.is_cuda else None
        if lib is None:
            if lengths is None:
                return _cpu.pesq(clean, noisy)
            return _cpu.per_row(_cpu.pesq, clean, noisy, device_lengths(lengths, B, L, "cpu"))
        F = lib.fsem_pesq_frames(L)
        lens = device_lengths(lengths, B, L, clean.device) if lengths is not None else None
        if F < 20 and lens is None:
            # the reference's unfold(1, size=20, step=10) fails here (PESQ.py:169)
            raise RuntimeError(f"maximum size for tensor at dimension 1 is {max(F, 0)} but size is 20")
        if clean.stride(0) != noisy.stride(0) or L % 4:
            # rows must be readable up to ceil4(L) floats (include/fsem.h): pad odd lengths
            pad = (-L) % 4
            clean = torch.nn.functional.pad(clean, (0, pad)).contiguous()
            noisy = torch.nn.functional.pad(noisy, (0, pad)).contiguous()
        mos = torch.empty(B, dtype=torch.float32, device=clean.device)
        ws = _native.workspace(lib.fsem_pesq_workspace_bytes(B, L), clean.device)
        _native.check(lib.fsem_pesq_wb_f32(clean.data_ptr(), noisy.data_ptr(), B, L, clean.stride(0),
                                           lens.data_ptr() if lens is not None else None,
                                           mos.data_ptr(), ws.data_ptr(), ws.numel(),
                                           _native.stream_handle(clean.device)), "PESQ")
        return mos

    def compute_metric(self, clean_speech: torch.Tensor | None, denoised_speech: torch.Tensor,
                       lengths=None) -> list[dict[str, float]]:
        assert clean_speech is not None
        with torch.inference_mode():
            mos = self.scores(clean_speech, denoised_speech, lengths, sample_rate=self.EXPECTED_SAMPLING_RATE)
            return [{"PESQ": m} for m in mos.tolist()]
