"""``classification.knn`` stages."""
from flink_ml_amd.models import KNN, KNNModel  # noqa: F401

__all__ = ['KNN', 'KNNModel']
