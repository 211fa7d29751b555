"""``feature.univariatefeatureselector`` stages."""
from flink_ml_amd.models import UnivariateFeatureSelector, UnivariateFeatureSelectorModel  # noqa: F401

__all__ = ['UnivariateFeatureSelector', 'UnivariateFeatureSelectorModel']
