"""Bark filterbank of the PESQ model -- host-side mirror of the reference's
``fast_se_metrics.utils.bark`` (bark.py:79-204), importable as that module path.

The engine carries these constants in constant memory (``csrc/fsem_tables.inc``, generated from
``_tables.py``); this module exposes them as the reference's Python objects for callers that use
the stage API (``PESQ.get_bark_bands`` / ``PESQ.filter_bank`` ...):

* ``interp(values, n)``: linear resampling of a 49-entry table onto ``n`` points spaced 49 / n
  apart (bark.py:79-97; the identity at 49; like scipy's ``interp1d`` it raises ``ValueError``
  for points beyond the last entry);
* ``BarkFilterBank(nfreqs, nbarks, device)``: the 0/1 matrix ``fbank`` [nbarks, nfreqs] (P.862's
  contiguous bin counts for the default 256 x 49, else bins around each band centre),
  ``forward`` = band sums of the power bins (the last bin dropped) times the power-density
  correction, ``weighted_norm`` = the band-width weighted p-norm over bands 1.. (bark.py:169-204).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import _tables as T

# the reference's module-level table names (bark.py:9-76)
nr_of_hz_bands_per_bark_band_16k = list(T.BINS_PER_BAND)
centre_of_band_bark_16k = list(T.CENTRE_BARK)
centre_of_band_hz_16k = list(T.CENTRE_HZ)
width_of_band_bark_16k = list(T.WIDTH_BARK)
width_of_band_hz_16k = list(T.WIDTH_HZ)
pow_dens_correction_factor_16k = list(T.POW_DENS_CORRECTION)
Sp_16k = T.SP_16K


def interp(values, nelms_new: int) -> torch.Tensor:
    """float64 [nelms_new]: ``values`` (a table over 0 .. n-1) sampled at k * 49 / nelms_new."""
    v = np.asarray(values, dtype=np.float64)
    x = np.arange(nelms_new, dtype=np.float64) * (49.0 / nelms_new)
    if x.size and (x[-1] > v.size - 1 or x[0] < 0):
        raise ValueError("A value in x_new is above the interpolation range.")
    return torch.from_numpy(np.interp(x, np.arange(v.size, dtype=np.float64), v))


class BarkFilterBank(torch.nn.Module):
    def __init__(self, nfreqs: int = 256, nbarks: int = 49, device: str = "cpu"):
        super().__init__()
        self.pow_dens_correction = (interp(T.POW_DENS_CORRECTION, nbarks) * T.SP_16K).to(device)
        self.width_hz = interp(T.WIDTH_HZ, nbarks).to(device)
        self.width_bark = interp(T.WIDTH_BARK, nbarks).to(device)
        self.centre = interp(T.CENTRE_HZ, nbarks).to(device)
        self.fbank = self._matrix(nfreqs, nbarks).to(device)
        self.total_width = self.width_bark[1:].sum()

    def _matrix(self, nfreqs: int, nbarks: int) -> torch.Tensor:
        m = torch.zeros(nbarks, nfreqs)
        if (nfreqs, nbarks) == (256, 49):
            # P.862's bin counts per band, laid end to end
            edges = np.concatenate([[0], np.cumsum(T.BINS_PER_BAND)])
            for k in range(nbarks):
                m[k, int(edges[k]):int(edges[k + 1])] = 1.0
            return m
        # generic: bins covering each band's [centre - width/2, centre + width/2), no overlap
        hz_per_bin = 8000.0 / nfreqs
        lo_floor = 0
        for k in range(nbarks):
            half = float(self.width_hz[k]) / hz_per_bin / 2
            c = float(self.centre[k]) / hz_per_bin
            a, b = max(lo_floor, int(math.floor(c - half))), min(nfreqs, int(math.ceil(c + half)))
            m[k, a:b] = 1.0
            lo_floor = b
        return m

    def weighted_norm(self, tensor: torch.Tensor, p: float = 2) -> torch.Tensor:
        """[batch, frame, band] -> [batch, frame]: total_width * || w_k x_k / total_width^(1/p) ||_p
        over bands 1.. (band 0 excluded)."""
        scaled = (self.width_bark * tensor / self.total_width ** (1.0 / p))[..., 1:]
        return self.total_width * torch.linalg.vector_norm(scaled, ord=p, dim=2)

    def forward(self, tensor: torch.Tensor) -> torch.Tensor:
        """[batch, frame, nfreqs + 1] power bins -> [batch, frame, nbarks] Bark powers (float64 as
        the reference: the correction table is float64)."""
        bands = torch.matmul(tensor[..., :-1], self.fbank.to(tensor.dtype).t())
        return bands * self.pow_dens_correction
