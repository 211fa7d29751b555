"""``feature.vectorslicer`` stages."""
from flink_ml_amd.models import VectorSlicer  # noqa: F401

__all__ = ['VectorSlicer']
