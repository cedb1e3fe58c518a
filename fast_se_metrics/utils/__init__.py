"""Drop-in package path ``fast_se_metrics.utils`` (reference fast_se_metrics/utils/)."""
