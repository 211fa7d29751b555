"""``feature.onehotencoder`` stages."""
from flink_ml_amd.models import OneHotEncoder, OneHotEncoderModel  # noqa: F401

__all__ = ['OneHotEncoder', 'OneHotEncoderModel']
