"""``feature.hashingtf`` stages."""
from flink_ml_amd.models import HashingTF  # noqa: F401

__all__ = ['HashingTF']
