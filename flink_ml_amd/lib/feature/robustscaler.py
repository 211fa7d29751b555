"""``feature.robustscaler`` stages."""
from flink_ml_amd.models import RobustScaler, RobustScalerModel  # noqa: F401

__all__ = ['RobustScaler', 'RobustScalerModel']
