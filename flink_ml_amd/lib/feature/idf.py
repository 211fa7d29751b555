"""``feature.idf`` stages."""
from flink_ml_amd.models import IDF, IDFModel  # noqa: F401

__all__ = ['IDF', 'IDFModel']
