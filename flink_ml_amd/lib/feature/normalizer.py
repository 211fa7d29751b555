"""``feature.normalizer`` stages."""
from flink_ml_amd.models import Normalizer  # noqa: F401

__all__ = ['Normalizer']
