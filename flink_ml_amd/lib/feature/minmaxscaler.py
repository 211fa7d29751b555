"""``feature.minmaxscaler`` stages."""
from flink_ml_amd.models import MinMaxScaler, MinMaxScalerModel  # noqa: F401

__all__ = ['MinMaxScaler', 'MinMaxScalerModel']
