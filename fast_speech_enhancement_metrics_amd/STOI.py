"""STOI / ESTOI metric -- drop-in for the reference's ``fast_se_metrics.STOI`` (STOI.py:7-205).

Runs at 10 kHz internally (STOI.py:9).  ``use_gpu=True``: libfsem's gfx950 kernels
(``fsem_stoi_f32``) with the 16 -> 10 kHz resampler fused into them (the reference
resamples in BaseMetric.prepare_audio, base.py:19-20; same arithmetic), one device->host
copy of the scores.  ``use_gpu=False``: the package's CPU implementation.
"""
from __future__ import annotations

import warnings

import torch

from . import _cpu, _native
from .base import BaseMetric, as_rows, check_row_rate, device_lengths, zero_tail
from .batching import resampled_lengths


class STOI(BaseMetric):
    higher_is_better = True
    EXPECTED_SAMPLING_RATE = 10000

    def __init__(self, sample_rate: int = 10000, use_gpu: bool = False):
        super().__init__(sample_rate, use_gpu)
        self.sampling_frequency = self.EXPECTED_SAMPLING_RATE
        self.win_length = 256
        self.hop_length = self.win_length // 2
        self.n_fft = 512
        self.num_octave_bands = 15
        self.min_frequency = 150
        self.N = 30
        self.beta = -15.0
        self.dynamic_range = 40

    @staticmethod
    def normalize(x: torch.Tensor, dim: int = 0) -> torch.Tensor:
        """In place, as STOI.py:113-119: centre along ``dim`` and divide by the L2 norm.  Without the
        reference's ``1e-12 * randn`` term (deterministic, as the engine): a zero-variance slice
        becomes 0 instead of a random unit vector."""
        x -= x.mean(dim=dim, keepdim=True)
        n = torch.linalg.vector_norm(x, ord=2, dim=dim, keepdim=True)
        x.copy_(torch.where(n > 0, x / torch.where(n > 0, n, torch.ones_like(n)), torch.zeros_like(x)))
        return x

    # ------------------------------------------------------------------ reference attributes
    def get_octave_band_matrix(self) -> torch.Tensor:
        """[15, 257] float32 1/3-octave band matrix (STOI.py:26-47): band i covers the FFT bins
        from the one nearest 150 * 2^((2i - 1) / 6) Hz up to (excluding) the one nearest
        150 * 2^((2i + 1) / 6) Hz."""
        return _cpu._OBM.to(torch.float32).clone()

    @property
    def octave_band_matrix(self) -> torch.Tensor:
        """STOI.py:19, on the metric's device (built on first access)."""
        if getattr(self, "_octave_band_matrix", None) is None:
            self._octave_band_matrix = self.get_octave_band_matrix().to(self.device)
        return self._octave_band_matrix

    @property
    def window(self) -> torch.Tensor:
        """[256] float32 analysis window hann(257)[1:] (STOI.py:24), on the metric's device."""
        if getattr(self, "_window", None) is None:
            self._window = torch.hann_window(self.win_length + 1, dtype=torch.float32, device=self.device)[1:]
        return self._window

    def scores(self, clean_speech: torch.Tensor, denoised_speech: torch.Tensor, sample_rate: int | None = None,
               lengths=None):
        """(stoi[B], estoi[B]) tensors on the metric's device; NaN where no segment exists.

        Rows at ``sample_rate``; None means rows already at 10 kHz, which requires a 10 kHz metric
        (``STOI(16000).scores`` must be told its rows' rate).  ``lengths`` (optional, [B] ints at that rate):
        row b holds lengths[b] samples and scores as the reference would on the unpadded row.
        """
        sr = check_row_rate(self, sample_rate)
        clean = as_rows(clean_speech)
        noisy = as_rows(denoised_speech)
        if noisy.shape != clean.shape:
            raise Exception("`clean_speech` and `denoised_speech` should have the same shape.")
        B, L = clean.shape
        if not clean.is_cuda:
            if lengths is not None:
                lens = device_lengths(lengths, B, L, "cpu")
                if sr != self.EXPECTED_SAMPLING_RATE:
                    clean, noisy = self._resample_cpu(zero_tail(clean, lens), sr), self._resample_cpu(zero_tail(noisy, lens), sr)
                    lens = resampled_lengths(lens, sr, self.EXPECTED_SAMPLING_RATE)
                return _cpu.per_row(_cpu.stoi, clean, noisy, lens)
            if sr != self.EXPECTED_SAMPLING_RATE:
                clean, noisy = self._resample_cpu(clean, sr), self._resample_cpu(noisy, sr)
            return _cpu.stoi(clean, noisy)
        lib = _native.load()
        lens = device_lengths(lengths, B, L, clean.device) if lengths is not None else None
        if clean.stride(0) != noisy.stride(0) or L % 4:
            # rows must be readable up to ceil4(L) floats (include/fsem.h): pad odd lengths
            pad = (-L) % 4
            clean = torch.nn.functional.pad(clean, (0, pad)).contiguous()
            noisy = torch.nn.functional.pad(noisy, (0, pad)).contiguous()
        s = torch.empty(B, dtype=torch.float32, device=clean.device)
        e = torch.empty(B, dtype=torch.float32, device=clean.device)
        nbytes = lib.fsem_stoi_workspace_bytes(B, L, sr)
        if nbytes == 0:
            raise NotImplementedError(f"unsupported sample rate {sr}: its resampling filter to 10 kHz would be longer "
                                      "than 8192 taps (include/fsem.h, FSEM_ERATE)")
        ws = _native.workspace(nbytes, clean.device)
        rc = lib.fsem_stoi_f32(clean.data_ptr(), noisy.data_ptr(), B, L, clean.stride(0),
                               lens.data_ptr() if lens is not None else None, sr, s.data_ptr(),
                               e.data_ptr(), ws.data_ptr(), ws.numel(), _native.stream_handle(clean.device))
        if rc == _native.FSEM_ESHORT:
            raise RuntimeError("STOI input shorter than one 256-sample frame at 10 kHz")
        _native.check(rc, "STOI")
        return s, e

    def _finish(self, stois: torch.Tensor, estois: torch.Tensor) -> list[dict[str, float]]:
        s, e = torch.stack([stois.float(), estois.float()]).tolist()
        if all(x != x for x in s):  # no utterance has a 30-frame segment (STOI.py:162-165)
            warnings.warn("Not enough non-silent frames. Please check your sound files", RuntimeWarning, stacklevel=3)
            raise TypeError("iteration over a 0-d tensor")
        return [{"STOI": a, "ESTOI": b} for a, b in zip(s, e)]

    def _resample_cpu(self, x: torch.Tensor, sr: int) -> torch.Tensor:
        if sr == self.sample_rate:
            return self.resampler(x)
        from .resample import Resample
        return Resample(sr, self.EXPECTED_SAMPLING_RATE)(x)

    def compute_metric(self, clean_speech: torch.Tensor | None, denoised_speech: torch.Tensor,
                       lengths=None) -> list[dict[str, float]]:
        assert clean_speech is not None
        with torch.no_grad():
            return self._finish(*self.scores(clean_speech, denoised_speech, self.EXPECTED_SAMPLING_RATE,
                                             lengths=lengths))

    def __call__(self, clean_speech, denoised_speech, lengths=None) -> list[dict[str, float]]:
        if self.device == "cuda" and clean_speech is not None:
            # GPU: resampling is fused into the STOI kernels -- skip BaseMetric's resampler
            clean_speech, denoised_speech, lengths = self.split_ragged(clean_speech, denoised_speech, lengths)
            if clean_speech.shape != denoised_speech.shape:
                raise Exception("`clean_speech` and `denoised_speech` should have the same shape.")
            clean = torch.atleast_2d(clean_speech).to(self.device)
            noisy = torch.atleast_2d(denoised_speech).to(self.device)
            with torch.no_grad():
                return self._finish(*self.scores(clean, noisy, self.sample_rate, lengths=lengths))
        return super().__call__(clean_speech, denoised_speech, lengths)
