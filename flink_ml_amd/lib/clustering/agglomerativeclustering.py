"""``clustering.agglomerativeclustering`` stages."""
from flink_ml_amd.models import AgglomerativeClustering  # noqa: F401

__all__ = ['AgglomerativeClustering']
