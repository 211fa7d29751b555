"""``feature.interaction`` stages."""
from flink_ml_amd.models import Interaction  # noqa: F401

__all__ = ['Interaction']
