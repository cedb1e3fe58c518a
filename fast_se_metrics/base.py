"""Drop-in module path of the reference's ``fast_se_metrics/base.py``."""
from fast_speech_enhancement_metrics_amd.base import BaseMetric  # noqa: F401
