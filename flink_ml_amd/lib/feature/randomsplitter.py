"""``feature.randomsplitter`` stages."""
from flink_ml_amd.models import RandomSplitter  # noqa: F401

__all__ = ['RandomSplitter']
