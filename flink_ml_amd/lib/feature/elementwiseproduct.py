"""``feature.elementwiseproduct`` stages."""
from flink_ml_amd.models import ElementwiseProduct  # noqa: F401

__all__ = ['ElementwiseProduct']
