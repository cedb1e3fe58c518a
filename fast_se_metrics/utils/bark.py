"""Drop-in module path ``fast_se_metrics.utils.bark`` (reference fast_se_metrics/utils/bark.py):
the P.862 tables, ``interp`` and ``BarkFilterBank``."""
from fast_speech_enhancement_metrics_amd.bark import (  # noqa: F401
    BarkFilterBank, Sp_16k, centre_of_band_bark_16k, centre_of_band_hz_16k, interp, nr_of_hz_bands_per_bark_band_16k,
    pow_dens_correction_factor_16k, width_of_band_bark_16k, width_of_band_hz_16k)
