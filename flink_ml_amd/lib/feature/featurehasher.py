"""``feature.featurehasher`` stages."""
from flink_ml_amd.models import FeatureHasher  # noqa: F401

__all__ = ['FeatureHasher']
