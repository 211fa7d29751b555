"""``feature.standardscaler`` stages."""
from flink_ml_amd.models import StandardScaler, StandardScalerModel  # noqa: F401

__all__ = ['StandardScaler', 'StandardScalerModel']
