"""``feature.dct`` stages."""
from flink_ml_amd.models import DCT  # noqa: F401

__all__ = ['DCT']
