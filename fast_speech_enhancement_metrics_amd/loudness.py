"""Zwicker loudness of the PESQ model -- host-side mirror of the reference's
``fast_se_metrics.utils.loudness`` (loudness.py:26-67), importable as that module path.

The engine evaluates the same formulas inside ``pesq_back`` (csrc/pesq.hip); this class serves
the stage API (``PESQ.loudness``, ``PESQ.equalize_bark_bands``):

* ``threshs`` [1, 1, nbark]: hearing threshold per band; ``exp`` [nbark]: the Zwicker exponent
  0.23 * clamp(6 / (centre_bark + 2), 1, 2)^0.15;
* ``audible_frame_power(bands, factor)`` [batch, frame, 1]: per-frame sum of the bands above
  ``factor`` x threshold;
* ``mean_audible_band_power(bands, silent)`` [batch, nbark]: per-band mean over ALL frames of the
  power above 100 x threshold in the non-silent frames;
* ``loudness(p)``: Sl * (2T)^e ((0.5 + 0.5 p / T)^e - 1), 0 where p <= T.
"""
from __future__ import annotations

import torch

from . import _tables as T
from .bark import centre_of_band_bark_16k, interp

# the reference's module-level names (loudness.py:9-23)
abs_thresh_power_16k = list(T.ABS_THRESH_POWER)
zwicker_power = T.ZWICKER_POWER
Sl_16k = T.SL_16K


class Loudness:
    def __init__(self, nbark: int = 49, device: str = "cpu"):
        self.threshs = interp(T.ABS_THRESH_POWER, nbark).reshape(1, 1, -1).to(device)
        base = (6.0 / (torch.tensor(centre_of_band_bark_16k) + 2.0)).clamp(1.0, 2.0)
        self.exp = (base ** 0.15 * T.ZWICKER_POWER).to(device)

    def audible_frame_power(self, bark_bands: torch.Tensor, hearing_threshold_factor: float = 1.0) -> torch.Tensor:
        audible = bark_bands > self.threshs * hearing_threshold_factor
        return (bark_bands * audible).sum(dim=2, keepdim=True)

    def mean_audible_band_power(self, bark_bands: torch.Tensor, frame_is_silent: torch.Tensor) -> torch.Tensor:
        audible = (bark_bands > self.threshs * 100.0) & ~frame_is_silent
        return (bark_bands * audible).mean(dim=1)

    def loudness(self, power_density: torch.Tensor) -> torch.Tensor:
        t = self.threshs
        v = (2.0 * t) ** self.exp * ((0.5 + 0.5 * power_density / t) ** self.exp - 1.0)
        return torch.where(power_density <= t, torch.zeros((), dtype=v.dtype, device=v.device), v) * T.SL_16K
