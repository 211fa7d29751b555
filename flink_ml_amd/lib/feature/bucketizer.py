"""``feature.bucketizer`` stages."""
from flink_ml_amd.models import Bucketizer  # noqa: F401

__all__ = ['Bucketizer']
