"""``feature.maxabsscaler`` stages."""
from flink_ml_amd.models import MaxAbsScaler, MaxAbsScalerModel  # noqa: F401

__all__ = ['MaxAbsScaler', 'MaxAbsScalerModel']
