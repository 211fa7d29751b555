"""``feature.variancethresholdselector`` stages."""
from flink_ml_amd.models import VarianceThresholdSelector, VarianceThresholdSelectorModel  # noqa: F401

__all__ = ['VarianceThresholdSelector', 'VarianceThresholdSelectorModel']
