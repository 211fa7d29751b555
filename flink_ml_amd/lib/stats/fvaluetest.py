"""``stats.fvaluetest`` stages."""
from flink_ml_amd.models import FValueTest  # noqa: F401

__all__ = ['FValueTest']
