"""BaseMetric -- the reference's drop-in boundary (fast_se_metrics/base.py:6-43), unchanged API.

``metric = PESQ(sample_rate, use_gpu)`` then ``metric(clean, denoised) -> list[dict]``.
``use_gpu=True`` runs the gfx950 HIP engine (libfsem); it raises at construction if the
engine is missing -- there is no silent fallback.  ``use_gpu=False`` runs the package's
own CPU implementation (``_cpu.py``), the reference's CPU mode.
"""
from __future__ import annotations

from abc import ABC, abstractmethod

import torch

from . import _native
from .resample import Resample


class BaseMetric(ABC):
    higher_is_better: bool
    EXPECTED_SAMPLING_RATE: int

    def __init__(self, sample_rate: int = 16000, use_gpu: bool = False):
        self.sample_rate = sample_rate
        self.device = "cuda" if use_gpu else "cpu"
        self.resampler = Resample(sample_rate, self.EXPECTED_SAMPLING_RATE)
        self.resampler.to(self.device)
        if use_gpu:
            if not torch.cuda.is_available():
                raise RuntimeError("use_gpu=True but no HIP device is visible")
            _native.load()

    def prepare_audio(self, audio: torch.Tensor) -> torch.Tensor:
        audio = torch.atleast_2d(audio)
        audio = audio.to(self.device)
        if self.sample_rate != self.EXPECTED_SAMPLING_RATE:
            audio = self.resampler(audio)
        return audio

    def prepare_inputs(self, clean_speech: torch.Tensor | None, denoised_speech: torch.Tensor):
        if clean_speech is not None and clean_speech.shape != denoised_speech.shape:
            raise Exception("`clean_speech` and `denoised_speech` should have the same shape.")
        if clean_speech is not None:
            clean_speech = self.prepare_audio(clean_speech)
        denoised_speech = self.prepare_audio(denoised_speech)
        return clean_speech, denoised_speech

    @abstractmethod
    def compute_metric(self, clean_speech: torch.Tensor | None, denoised_speech: torch.Tensor) -> list[dict[str, float]]:
        raise NotImplementedError

    def __call__(self, clean_speech: torch.Tensor | None, denoised_speech: torch.Tensor) -> list[dict[str, float]]:
        clean_speech, denoised_speech = self.prepare_inputs(clean_speech, denoised_speech)
        return self.compute_metric(clean_speech, denoised_speech)


def as_rows(x: torch.Tensor) -> torch.Tensor:
    """float32 [B, L] with unit stride along time (row stride = x.stride(0))."""
    x = torch.atleast_2d(x)
    if x.dtype != torch.float32:
        x = x.to(torch.float32)
    if x.dim() != 2 or x.stride(-1) != 1 or x.stride(0) < x.shape[1]:
        x = x.reshape(-1, x.shape[-1]).contiguous()
    return x
