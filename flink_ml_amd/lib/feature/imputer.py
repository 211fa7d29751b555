"""``feature.imputer`` stages."""
from flink_ml_amd.models import Imputer, ImputerModel  # noqa: F401

__all__ = ['Imputer', 'ImputerModel']
