"""``feature.vectorindexer`` stages."""
from flink_ml_amd.models import VectorIndexer, VectorIndexerModel  # noqa: F401

__all__ = ['VectorIndexer', 'VectorIndexerModel']
