"""Drop-in module path ``fast_se_metrics.utils.loudness`` (reference
fast_se_metrics/utils/loudness.py): the hearing thresholds and ``Loudness``."""
from fast_speech_enhancement_metrics_amd.loudness import Loudness, Sl_16k, abs_thresh_power_16k, zwicker_power  # noqa: F401
