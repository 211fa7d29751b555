"""``stats.chisqtest`` stages."""
from flink_ml_amd.models import ChiSqTest  # noqa: F401

__all__ = ['ChiSqTest']
