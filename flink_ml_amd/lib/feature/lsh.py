"""``feature.lsh`` stages."""
from flink_ml_amd.models import MinHashLSH, MinHashLSHModel  # noqa: F401

__all__ = ['MinHashLSH', 'MinHashLSHModel']
