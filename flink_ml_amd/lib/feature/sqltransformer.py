"""``feature.sqltransformer`` stages."""
from flink_ml_amd.models import SQLTransformer  # noqa: F401

__all__ = ['SQLTransformer']
