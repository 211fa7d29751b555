"""``stats.anovatest`` stages."""
from flink_ml_amd.models import ANOVATest  # noqa: F401

__all__ = ['ANOVATest']
