"""``feature.binarizer`` stages."""
from flink_ml_amd.models import Binarizer  # noqa: F401

__all__ = ['Binarizer']
